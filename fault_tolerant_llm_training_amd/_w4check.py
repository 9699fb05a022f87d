"""Static check of the w4 GEMM kernels' compiled gfx950 code (csrc/kernels/gemm_w4.hip).

Run by :func:`fault_tolerant_llm_training_amd._build.build` on the assembly the compiler keeps
(``-save-temps``) for the very object that is linked into ``_kernels.so``: the link is refused
when any kernel has an unsafe placement. Standalone: ``python -m
fault_tolerant_llm_training_amd._w4check [--src FILE.hip] [--asm FILE.s] [--keep OUT.s]``.

The kernels issue their LDS reads, LDS-DMA loads and MFMAs as inline asm, which the compiler
treats as instantaneous register producers. Three compiler placements are therefore unsafe and
have each produced wrong results once; this script compiles the file to device assembly (no GPU
needed) and fails if any kernel contains one:

  1. scratch use inside the K loop (any spill there), or an accumulator (AGPR) spill before the
     drain: until then the asm MFMAs may still be writing the accumulators the compiler would
     spill. Outside those, a spill is correct (an address spilled in the prologue; accumulators
     spilled after the drain hold their final values): the split-K epilogue of the widest dX
     tile spills a few registers there;
  2. inside the K loop: any compiler-generated accumulator access (v_accvgpr_*) or VGPR write
     (a copy of a value whose asm producer has not landed yet);
  3. between the K-loop exit and the drain (``s_waitcnt vmcnt(0) lgkmcnt(0)`` + MFMA pad): a
     compiler-generated write of a register that an asm LDS read in the loop targets (it races
     the in-flight dead reads), or any accumulator access (a read right behind the MFMAs still
     writing it).
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile


def compile_asm(src, out):
    """Device assembly of ``src`` (the build's flags, gfx950) into ``out``."""
    from . import _build

    cmd = [_build._hipcc(), *_build._common_flags("_kernels"), f"--offload-arch={_build.ARCH}",
           "-x", "hip", "--cuda-device-only", "-S", str(src), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr[-4000:])


def kernels(lines):
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*gemm_w4_kernel\S*:", l)]
    for a in starts:
        b = next(i for i in range(a, len(lines)) if lines[i].startswith(".Lfunc_end"))
        yield lines[a].split(":")[0], a, b


def instrs(lines, a, b):
    """(index, text, from_asm) of every instruction / label in lines[a:b]."""
    inasm = False
    for i in range(a, b):
        s = lines[i].strip()
        if s.startswith(";;#ASMSTART"):
            inasm = True
            continue
        if s.startswith(";;#ASMEND"):
            inasm = False
            continue
        if not s or s.startswith(";") or (s.startswith(".") and not s.endswith(":") and "LBB" not in s):
            continue
        yield i, s.split(";")[0].strip(), inasm


def dst_regs(text):
    """VGPR / AGPR numbers (v: n, a: 1000 + n) an instruction writes; empty for stores etc."""
    op, _, rest = text.partition(" ")
    if op.startswith(("s_", "buffer_store", "global_store", "ds_write")) or op.endswith(":"):
        return set()
    dst = rest.split(",")[0].strip()
    m = re.match(r"^([va])(?:(\d+)|\[(\d+):(\d+)\])$", dst)
    if not m:
        return set()
    lo = int(m.group(2) or m.group(3))
    hi = int(m.group(2) or m.group(4))
    base = 1000 if m.group(1) == "a" else 0
    return set(range(base + lo, base + hi + 1))


def check(name, lines, a, b, scratch):
    errs = []
    ins = list(instrs(lines, a, b))
    # the K loop: the backward conditional branch whose body holds the asm MFMAs
    labels = {t[:-1]: k for k, (_, t, _) in enumerate(ins) if t.endswith(":")}
    loop = None
    for k, (_, t, _) in enumerate(ins):
        m = re.match(r"s_cbranch_\w+ (\.LBB\S+)", t)
        if m and m.group(1) in labels and labels[m.group(1)] < k:
            body = ins[labels[m.group(1)]:k]
            if sum(1 for _, x, asm in body if asm and x.startswith("v_mfma")) >= 32:
                loop = (labels[m.group(1)], k)
                break
    if loop is None:
        return errs + ["K loop not found"]
    targets = set()
    for _, t, asm in ins[loop[0]:loop[1]]:
        if asm and t.startswith("ds_read"):
            targets |= dst_regs(t)
        if not asm and (t.startswith("v_accvgpr") or dst_regs(t)):
            errs.append(f"in loop: {t}")
    drained = False
    drain_at = len(ins)
    for k, (_, t, asm) in enumerate(ins[loop[1] + 1:], start=loop[1] + 1):
        if asm and t.startswith("s_waitcnt vmcnt(0) lgkmcnt(0)"):
            drained = True
            drain_at = k
            break
        if not asm and (t.startswith("v_accvgpr") or dst_regs(t) & targets):
            errs.append(f"before drain: {t}")
    if not drained:
        errs.append("no drain after the K loop")
    is_scr = lambda t: t.startswith("scratch_")  # noqa: E731
    in_loop = [t for _, t, _ in ins[loop[0]:loop[1]] if is_scr(t)]
    acc_early = [t for _, t, _ in ins[:drain_at] if is_scr(t) and re.search(r"\ba\[?\d", t)]
    if in_loop:
        errs.append(f"scratch in the K loop: {in_loop[0]}")
    if acc_early:
        errs.append(f"accumulator spilled before the drain: {acc_early[0]}")
    # 4. an asm that writes SCC (s_add_u32 m0 of the LDS-DMA) between a compiler compare and the
    # branch that reads it (an undeclared SCC clobber: the loop exits on the carry)
    scc = None
    for _, t, asm in ins:
        if not asm and t.startswith(("s_cmp", "s_bitcmp")):
            scc = t
        elif asm and scc and t.startswith(("s_add_", "s_sub_", "s_and_", "s_or_", "s_cmp")):
            errs.append(f"asm {t!r} between {scc!r} and its branch")
            scc = None
        elif t.startswith(("s_cbranch_scc", "s_cselect")) or t.endswith(":"):
            scc = None
    return errs


def check_asm(path):
    """(kernels checked, [(kernel, [errors])] of the unsafe ones) for the assembly file ``path``."""
    lines = open(path).read().split("\n")
    scratch, cur = {}, None
    for l in lines:
        m = re.match(r"^\s*\.name:\s+(\S*gemm_w4_kernel\S*)", l)
        if m:
            cur = m.group(1)
        m = re.match(r"^\s*\.private_segment_fixed_size:\s+(\d+)", l)
        if m and cur:
            scratch[cur] = int(m.group(1))
    n, bad = 0, []
    for name, a, b in kernels(lines):
        n += 1
        errs = check(name, lines, a, b, scratch)
        if errs:
            bad.append((name, errs))
    return n, bad


def report(n, bad) -> str:
    out = [f"{name}\n    " + "\n    ".join(errs[:6]) for name, errs in bad]
    out.append(f"{n} w4 kernels checked, {len(bad)} with unsafe placements")
    return "\n".join(out)


def main(argv=None):
    from . import _build

    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=str(_build.CSRC / "kernels" / "gemm_w4.hip"), help="kernel source to compile")
    ap.add_argument("--keep", default=None, help="write the assembly here")
    ap.add_argument("--asm", default=None, help="check this assembly instead of compiling")
    args = ap.parse_args(argv)
    out = args.asm or args.keep or os.path.join(tempfile.mkdtemp(), "gemm_w4.s")
    if not args.asm:
        compile_asm(args.src, out)
    n, bad = check_asm(out)
    print(report(n, bad))
    return 1 if bad or not n else 0


if __name__ == "__main__":
    sys.exit(main())
