"""CLI of the w4 GEMM static checker (fault_tolerant_llm_training_amd/_w4check.py; the build runs
the same check on the linked object's assembly).

    python scripts/w4_asm_check.py [--src FILE.hip] [--asm FILE.s] [--keep OUT.s]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._w4check import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
