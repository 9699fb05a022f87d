"""Static check of the w4 GEMM kernels' compiled gfx950 code (csrc/kernels/gemm_w4.hip).

The kernels issue their LDS reads, LDS-DMA loads and MFMAs as inline asm, which the compiler
treats as instantaneous register producers. Three compiler placements are therefore unsafe and
have each produced wrong results once; this script compiles the file to device assembly (no GPU
needed) and fails if any kernel contains one:

  1. scratch use (accumulator spills);
  2. inside the K loop: any compiler-generated accumulator access (v_accvgpr_*) or VGPR write
     (a copy of a value whose asm producer has not landed yet);
  3. between the K-loop exit and the drain (``s_waitcnt vmcnt(0) lgkmcnt(0)`` + MFMA pad): a
     compiler-generated write of a register that an asm LDS read in the loop targets (it races
     the in-flight dead reads), or any accumulator access (a read right behind the MFMAs still
     writing it).

    python scripts/w4_asm_check.py [--keep OUT.s]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd import _build  # noqa: E402

SRC = _build.CSRC / "kernels" / "gemm_w4.hip"


def compile_asm(out):
    cmd = [_build._hipcc(), *_build._common_flags("_kernels"), f"--offload-arch={_build.ARCH}",
           "-x", "hip", "--cuda-device-only", "-S", str(SRC), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-4000:])


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
    if scratch.get(name, 0):
        errs.append(f"scratch {scratch[name]} B")
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
    for _, t, asm in ins[loop[1] + 1:]:
        if asm and t.startswith("s_waitcnt vmcnt(0) lgkmcnt(0)"):
            drained = True
            break
        if not asm and (t.startswith("v_accvgpr") or dst_regs(t) & targets):
            errs.append(f"before drain: {t}")
    if not drained:
        errs.append("no drain after the K loop")
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keep", default=None, help="write the assembly here")
    ap.add_argument("--asm", default=None, help="check this assembly instead of compiling")
    args = ap.parse_args()
    out = args.asm or args.keep or os.path.join(tempfile.mkdtemp(), "gemm_w4.s")
    if not args.asm:
        compile_asm(out)
    lines = open(out).read().split("\n")
    scratch, cur = {}, None
    for l in lines:
        m = re.match(r"^\s*\.name:\s+(\S*gemm_w4_kernel\S*)", l)
        if m:
            cur = m.group(1)
        m = re.match(r"^\s*\.private_segment_fixed_size:\s+(\d+)", l)
        if m and cur:
            scratch[cur] = int(m.group(1))
    n = bad = 0
    for name, a, b in kernels(lines):
        n += 1
        errs = check(name, lines, a, b, scratch)
        if errs:
            bad += 1
            print(name, *errs[:6], sep="\n    ")
    print(f"{n} w4 kernels checked, {bad} with unsafe placements")
    sys.exit(1 if bad or not n else 0)


if __name__ == "__main__":
    main()
