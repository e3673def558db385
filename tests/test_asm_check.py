"""CPU check of the built gfx950 code objects: no instruction may touch the destination registers of
an inline-asm transposed LDS read (common.h ds_read_tr16_asm, uncounted by the compiler) before a
`s_waitcnt lgkmcnt` retires it (tools/check_asm.py).  Plus a synthetic disassembly on which the
checker must fire, so a silent parser failure cannot pass."""
import glob
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_asm  # noqa: E402

HDR = "0000000000001000 <kern>:\n"


def _ins(addr, text):
    return f"\t{text:<58s}// {addr:012X}: 00000000\n"


def test_checker_flags_early_use():
    dis = HDR + _ins(0x1000, "ds_read_b64_tr_b16 v[10:11], v2") + _ins(0x1008, "v_mov_b32_e32 v20, v10") + \
        _ins(0x100C, "s_waitcnt lgkmcnt(0)") + _ins(0x1010, "s_endpgm")
    k, v = check_asm.check_text(dis)
    assert k == {"kern"} and len(v) == 1 and "v[10]" in v[0][1]


def test_checker_accepts_waited_use_and_counted_waits():
    dis = HDR + _ins(0x1000, "ds_read_b64_tr_b16 v[10:11], v2") + _ins(0x1008, "ds_read_b128 v[12:15], v3") + \
        _ins(0x1010, "s_waitcnt lgkmcnt(1)") + _ins(0x1014, "v_mov_b32_e32 v20, v10") + \
        _ins(0x1018, "s_waitcnt lgkmcnt(0)") + _ins(0x101C, "v_mov_b32_e32 v21, v12") + _ins(0x1020, "s_endpgm")
    k, v = check_asm.check_text(dis)
    assert k == {"kern"} and v == []


def test_checker_follows_back_edges():
    # loop: the read at the bottom is outstanding when the back edge reaches the use at the top
    dis = HDR + _ins(0x1000, "v_mov_b32_e32 v20, v10") + _ins(0x1004, "ds_read_b64_tr_b16 v[10:11], v2") + \
        _ins(0x100C, "s_cbranch_scc1 65532") + _ins(0x1010, "s_waitcnt lgkmcnt(0)") + _ins(0x1014, "s_endpgm")
    _, v = check_asm.check_text(dis)
    assert len(v) == 1 and "v_mov" in v[0][1]


def test_checker_flags_fma_in_colsum_epilogue():
    dis = "0000000000001000 <_ZN3vit2g213gemm_kernel_sILi9ELb0EEEvNS_10GemmParamsE>:\n" + \
        _ins(0x1000, "v_pk_fma_f32 v[4:5], v[0:1], v[2:3], v[4:5]") + _ins(0x1008, "s_endpgm") + \
        "0000000000002000 <_ZN3vit2g213gemm_kernel_sILi8ELb0EEEvNS_10GemmParamsE>:\n" + \
        _ins(0x2000, "v_fma_f32 v4, v0, v2, v4") + _ins(0x2008, "s_endpgm")
    v = check_asm.colsum_fma_violations(dis)
    assert v == [("_ZN3vit2g213gemm_kernel_sILi9ELb0EEEvNS_10GemmParamsE", 1)]


def test_built_code_objects_have_no_early_asm_read_use():
    objs = sorted(glob.glob(os.path.join(ROOT, "vit.rs_amd", "build", "*.o")))
    if not objs or not os.path.exists(os.path.join(check_asm.LLVM, "llvm-objdump")):
        pytest.skip("no build objects / ROCm LLVM tools here")
    assert check_asm.main(objs) == 0
