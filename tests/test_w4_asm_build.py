"""The w4 static check (fault_tolerant_llm_training_amd/_w4check.py) on the REAL compiled kernels
(hipcc cross-compiles gfx950 here, no GPU): every instantiated w4 kernel of the three layout
translation units is free of the unsafe compiler placements, and a deliberately reintroduced
undeclared SCC clobber in the LDS-DMA asm (the round-4 NJ = 4 bug) is caught -- so the build
(_build.build, which runs the same check on the linked objects' kept assembly) refuses it."""
import concurrent.futures as cf
import os
import shutil
import subprocess

import pytest

from fault_tolerant_llm_training_amd import _build, _w4check

pytestmark = pytest.mark.slow

KDIR = _build.CSRC / "kernels"


def _compile_s(src, out, include_first=None):
    cmd = [_build._hipcc(), *_build._common_flags("_kernels"), f"--offload-arch={_build.ARCH}", "-x", "hip",
           "--cuda-device-only", "-S", str(src), "-o", str(out)]
    if include_first:
        cmd[1:1] = ["-I", str(include_first)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return str(out)


def _fresh_kept_asm(stem):
    """The build's kept assembly of a TU if it is newer than the source and every header it includes."""
    src = KDIR / f"{stem}.hip"
    asm = _build._asm_of(src, _build.BUILD / f"_kernels_{stem}.o")
    if not asm.exists():
        return None
    t = asm.stat().st_mtime
    deps = [src, *_build._includes(src, [KDIR])]
    return str(asm) if all(d.stat().st_mtime <= t for d in deps) else None


def test_compiled_w4_kernels_have_no_unsafe_placement(tmp_path):
    asms = {}
    todo = []
    for stem in _build.W4_CHECKED:
        a = _fresh_kept_asm(stem)
        if a:
            asms[stem] = a
        else:
            todo.append(stem)
    with cf.ThreadPoolExecutor(max_workers=3) as ex:
        futs = {s: ex.submit(_compile_s, KDIR / f"{s}.hip", tmp_path / f"{s}.s") for s in todo}
        for s, f in futs.items():
            asms[s] = f.result()
    total = 0
    for stem, asm in asms.items():
        n, bad = _w4check.check_asm(asm)
        assert n > 0, stem
        assert not bad, _w4check.report(n, bad)
        total += n
    assert total >= 64  # 2 dtypes x 4 tile widths x the epilogues of the three layouts


def test_reintroduced_scc_clobber_fails_the_check(tmp_path):
    hdr = (KDIR / "gemm_w4.h").read_text()
    assert hdr.count(': "memory", "scc");') == 1  # the LDS-DMA asm declares its SCC write
    (tmp_path / "gemm_w4.h").write_text(hdr.replace(': "memory", "scc");', ': "memory");'))
    # the dX translation unit: since round 6 the forward one keeps its K-loop condition out of SCC
    # (the dead-tail descriptor selects read SCC right after their compare), so the undeclared
    # clobber has nothing to corrupt there; the dX / dW loops still branch on SCC
    shutil.copy(KDIR / "gemm_w4_dx.hip", tmp_path / "gemm_w4_dx.hip")
    asm = _compile_s(tmp_path / "gemm_w4_dx.hip", tmp_path / "dx.s", include_first=tmp_path)
    n, bad = _w4check.check_asm(asm)
    assert n > 0 and bad, "the SCC clobber was not detected"
    assert any("between" in e for _, errs in bad for e in errs)
    with pytest.raises(RuntimeError, match="w4 static check failed"):
        _build.check_w4_asm(asm)
