"""The shipped library's DPP / permlane reads keep their wait states after VALU writes (tools/isa_hazards.py).

The rollout kernels issue DPP reduce-scatters from inline asm that LLVM's hazard recognizer cannot see into;
their first DPP reads registers written by the preceding asm block.  This pins the ordering on the built code
object, and the synthetic listings show that the checker catches each rule.
"""
import os
import shutil

import pytest

import tools.isa_hazards as ih

_HDR = "0000000000001000 <k>:\n"


def _fn(lines):
    text = _HDR + "".join("\t%s // %012X: 00000000\n" % (ln, 0x1000 + 4 * i) for i, ln in enumerate(lines))
    return ih.functions(text)["k"]


def test_checker_flags_a_dpp_read_right_after_its_valu_write():
    bad = ih.hazards("k", _fn(["v_add_f32_e32 v4, v1, v2",
                               "v_add_f32_dpp v0, v4, v0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf"]))
    assert len(bad) == 1 and bad[0][3] == 0


def test_checker_counts_snop_and_packed_writes():
    ok = _fn(["v_pk_fma_f32 v[4:5], v[0:1], v[2:3], v[4:5]", "s_nop 1",
              "v_add_f32_dpp v0, v5, v0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf"])
    assert ih.hazards("k", ok) == []
    one = _fn(["v_pk_fma_f32 v[4:5], v[0:1], v[2:3], v[4:5]", "s_nop 0",
               "v_add_f32_dpp v0, v5, v0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf"])
    assert len(ih.hazards("k", one)) == 1
    # src1 of a DPP instruction is an ordinary operand
    assert ih.hazards("k", _fn(["v_add_f32_e32 v4, v1, v2",
                                "v_add_f32_dpp v0, v7, v4 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf"])) == []


def test_checker_follows_back_edges_and_permlane_and_exec():
    loop = _fn(["s_nop 4",
                "v_add_f32_dpp v0, v4, v0 row_half_mirror row_mask:0xf bank_mask:0xf",  # loop head
                "v_mov_b32_e32 v9, v0",
                "v_add_f32_e32 v4, v1, v2",
                "s_cbranch_scc1 65532 // <k+0x4>"])
    # llvm-objdump prints the target after the encoding; rebuild the line in that form
    loop[-1].target = 0x1004
    bad = ih.hazards("k", loop)
    assert len(bad) == 1 and bad[0][2] == 0x100C  # the back edge's write, 1 wait state (the branch)
    perm = _fn(["v_mov_b32_e32 v1, v0", "v_permlane16_swap_b32_e32 v0, v1"])
    assert len(ih.hazards("k", perm)) == 1
    ex = _fn(["v_cmpx_gt_f32_e32 vcc, v1, v2", "s_nop 2",
              "v_mov_b32_dpp v0, v7 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"])
    assert len(ih.hazards("k", ex)) == 1


@pytest.mark.skipif(not os.path.exists(ih.DEFAULT_SO) or not shutil.which(os.path.join(ih.LLVM, "llvm-objdump")),
                    reason="libfdr.so or llvm-objdump missing")
def test_shipped_library_has_no_dpp_hazards():
    bad, n = ih.check()
    assert n > 1000, "no DPP reads found: disassembly parse broke"
    assert not bad, {k: v[:3] for k, v in bad.items()}
