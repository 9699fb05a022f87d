"""Investigation build of the kernel library with the w4 GEMM's full timing probe (-DFT_W4_PROBE:
entry / end of prologue / drain / end of epilogue staging / exit stamps per workgroup) into
probe/_kernels_probe.so, linked with the regular build's other objects. Load it with
FT_KERNELS_SO=probe/_kernels_probe.so (scripts/w4_timeline.py --full). Not statically checked: the
stamps change the K loops' register allocation, so its times are for the phase split, not for
the absolute rate.

    python scripts/w4_probe_build.py
"""
import concurrent.futures as cf
import os
import sys
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd import _build as B  # noqa: E402


def main():
    B.build(verbose=False)  # the regular objects (and _kernels.so) first
    out = Path(B.ROOT) / "probe"
    out.mkdir(exist_ok=True)
    flags = B._common_flags("_kernels") + ["-DFT_W4_PROBE=1"]
    srcs = sorted((B.CSRC / "kernels").glob("*.hip"))
    objs, work = [], []
    for s in srcs:
        if s.stem in B.W4_CHECKED or s.stem == "gemm_w4":
            o = B.BUILD / f"probe_{s.stem}.o"
            work.append((s, o))
        else:
            o = B.BUILD / f"_kernels_{s.stem}.o"
        objs.append(o)
    saved = B.W4_CHECKED
    B.W4_CHECKED = ()  # no static check / kept assembly for the probe objects
    try:
        with cf.ThreadPoolExecutor(4) as ex:
            for f in [ex.submit(B._compile, s, o, flags, True) for s, o in work]:
                print(f"[probe] compiled {f.result().name}", flush=True)
    finally:
        B.W4_CHECKED = saved
    B._link(objs, out / "_kernels_probe.so", True)
    print(f"[probe] linked {out / '_kernels_probe.so'}", flush=True)


if __name__ == "__main__":
    main()
