"""scripts/w4_asm_check.py's rules on hand-made gfx950 assembly (no compiler, no GPU): each unsafe
compiler placement it exists to catch in the w4 GEMM is detected, and a clean loop passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fault_tolerant_llm_training_amd import _w4check as chk  # noqa: E402


def _asm(body_loop, after_loop, cmp_then_asm=False):
    """A fake kernel: 32 asm MFMAs + LDS reads in a loop, then the post-loop code."""
    a = lambda t: [";;#ASMSTART", "\t" + t, ";;#ASMEND"]
    lines = ["_ZN12_GLOBAL__N_114gemm_w4_kernelI5EBF16Li8ELi0ELb0ELb0EEEvNS_6W4ArgsE:", ".LBB0_1:"]
    lines += a("ds_read_b128 v[2:5], v63 offset:0")
    for _ in range(32):
        lines += a("v_mfma_f32_16x16x32_bf16 a[0:3], v[2:5], v[6:9], a[0:3]")
    lines += body_loop
    if cmp_then_asm:
        lines += ["\ts_cmp_lt_i32 s9, s6"] + a("s_add_u32 m0, s7, 0x1000") + a("buffer_load_dwordx4 v51, s[0:3], s28 offen lds")
    else:
        lines += a("s_add_u32 m0, s7, 0x1000") + a("buffer_load_dwordx4 v51, s[0:3], s28 offen lds") + ["\ts_cmp_lt_i32 s9, s6"]
    lines += ["\ts_cbranch_scc1 .LBB0_1"]
    lines += after_loop
    lines += a("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 7")
    lines += ["\tv_accvgpr_read_b32 v4, a0", "\ts_endpgm", ".Lfunc_end0:"]
    return lines


def _errs(lines):
    (name, a, b), = list(chk.kernels(lines))
    return chk.check(name, lines, a, b, {})


def test_clean_loop_passes():
    assert _errs(_asm([], ["\tv_and_b32_e32 v120, 15, v0"])) == []


def test_scc_clobber_between_compare_and_branch():
    e = _errs(_asm([], [], cmp_then_asm=True))
    assert any("s_add_u32 m0" in x and "s_cmp_lt_i32" in x for x in e), e


def test_register_reuse_racing_the_dead_reads():
    e = _errs(_asm([], ["\tv_and_b32_e32 v2, 15, v0"]))  # v2 is an in-flight ds_read target
    assert any("before drain" in x and "v2" in x for x in e), e


def test_accumulator_copy_inside_the_loop():
    e = _errs(_asm(["\tv_accvgpr_mov_b32 a5, a1"], []))
    assert any("in loop" in x for x in e), e


def test_accumulator_read_before_the_drain():
    e = _errs(_asm([], ["\tv_accvgpr_read_b32 v130, a3"]))
    assert any("before drain" in x for x in e), e


def test_scratch_in_the_loop_is_unsafe():
    lines = _asm(["\tscratch_store_dword off, v7, off"], [])
    (name, a, b), = list(chk.kernels(lines))
    e = chk.check(name, lines, a, b, {name: 4})
    assert any("scratch in the K loop" in x for x in e), e


def test_accumulator_spill_before_the_drain_is_unsafe():
    lines = _asm([], ["\tscratch_store_dwordx4 off, a[4:7], off"])
    (name, a, b), = list(chk.kernels(lines))
    e = chk.check(name, lines, a, b, {name: 16})
    assert any("accumulator spilled before the drain" in x for x in e), e


def test_scratch_after_the_drain_is_allowed():
    lines = _asm([], [])
    i = next(k for k, l in enumerate(lines) if "v_accvgpr_read_b32 v4, a0" in l)
    lines.insert(i, "\tscratch_store_dwordx4 off, a[0:3], off")
    (name, a, b), = list(chk.kernels(lines))
    assert chk.check(name, lines, a, b, {name: 16}) == []
