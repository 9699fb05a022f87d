"""Training entry point — same CLI as the reference's ``train.py`` (reference train.py:131-134).

    python train.py --sequence-length 2048 --batch-size 1 --learning-rate 5e-5 \
        --lr-warmup-steps 100 --training-steps 1000 [--checkpoint-id JOBID] ...

One process per GPU: launch with ``srun`` (see ``train.sh``) or
``torchrun --nproc-per-node N train.py ...`` for data parallelism.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from fault_tolerant_llm_training_amd.trainer import main  # noqa: E402

if __name__ == "__main__":
    main()
