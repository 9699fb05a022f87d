"""Every ops module imports on its own in a fresh interpreter (attention and functional import each
other: the order must not matter)."""
import subprocess
import sys

import pytest


@pytest.mark.parametrize("mod", ["ops.attention", "ops.functional", "ops.routing", "models.llama", "trainer"])
def test_module_imports_first(mod):
    r = subprocess.run([sys.executable, "-c", f"import fault_tolerant_llm_training_amd.{mod}"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
