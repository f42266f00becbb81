"""The built library carries no 16-B store whose data VGPRs a VALU instruction overwrites within the
two wait states gfx950 requires, on the fall-through or a branch path (the
store-data hazard behind round 4's bf16 quad-epilogue and k_conv3m co-run nondeterminism; see
conv_common.hpp store_b128_guarded).  Static: disassembles the gfx950 code objects, no GPU."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import store_hazard_check as shc  # noqa: E402

LIB = os.path.join(ROOT, "vae-diffusion-toy-crystals_amd", "toycrystals_amd", "libtcx.so")


def test_scanner_flags_the_pattern(tmp_path):
    """the shape hipcc emitted for k_conv3lb's quad epilogue (store ends a branch, the join block's
    first instruction rewrites the store's first data dword) is flagged; a padded one is not"""
    bad = tmp_path / "bad.s"
    bad.write_text("_ZN3tcx1kEv:\n"
                   "\tbuffer_store_dwordx4 v[66:69], v92, s[12:15], s20 offen\n"
                   ".LBB4_107:\n"
                   "\tv_cndmask_b32_e64 v66, 0, 1, s[10:11]\n")
    good = tmp_path / "good.s"
    good.write_text("_ZN3tcx1kEv:\n"
                    "\tbuffer_store_dwordx4 v[66:69], v92, s[12:15], s20 offen\n"
                    "\ts_nop 1\n"
                    ".LBB4_107:\n"
                    "\tv_cndmask_b32_e64 v66, 0, 1, s[10:11]\n")
    assert shc.scan(str(bad)) == 1
    assert shc.scan(str(good)) == 0


def test_scanner_counts_wait_states_and_follows_branches(tmp_path):
    """gfx950 needs TWO wait states between the store and a VALU write of its data (store_b128_guarded
    pads with s_nop 1): an unrelated instruction in between is one, s_nop 0 is one, s_nop 1 is two;
    the write may also sit at the target of a branch that follows the store (hipcc -S labels and
    llvm-objdump <func+0xoff> targets)."""
    def scan(body):
        f = tmp_path / "t.s"
        f.write_text("_ZN3tcx1kEv:\n" + body)
        return shc.scan(str(f))
    st = "\tbuffer_store_dwordx4 v[66:69], v92, s[12:15], s20 offen\n"
    assert scan(st + "\tv_mov_b32_e32 v1, v2\n\tv_cndmask_b32_e64 v67, 0, 1, s[10:11]\n") == 1  # distance 2
    assert scan(st + "\ts_nop 0\n\tv_mov_b32_e32 v68, 0\n") == 1
    assert scan(st + "\ts_nop 1\n\tv_mov_b32_e32 v68, 0\n") == 0
    assert scan(st + "\tv_mov_b32_e32 v1, v2\n\tv_mov_b32_e32 v3, v2\n\tv_mov_b32_e32 v66, 0\n") == 0
    # branch straight after the store: the write at the target is one wait state away
    assert scan(st + "\ts_branch .LBB0_9\n\tv_mov_b32_e32 v1, 0\n.LBB0_9:\n\tv_mov_b32_e32 v69, 0\n") == 1
    assert scan(st + "\ts_cbranch_scc1 .LBB0_9\n\ts_nop 3\n.LBB0_9:\n\tv_mov_b32_e32 v66, 0\n") == 1
    assert scan(st + "\ts_cbranch_scc1 .LBB0_9\n\tv_mov_b32_e32 v66, 0\n.LBB0_9:\n\ts_endpgm\n") == 1
    # llvm-objdump form: the target as <function+offset>
    obj = ("0000000000001000 <_ZN3tcx1kEv>:\n"
           "\tbuffer_store_dwordx4 v[66:69], v92, s[12:15], s20 offen // 000000001000: E07C1000 80056681\n"
           "\ts_branch 1 // 000000001008: BF820001 <_ZN3tcx1kEv+0x10>\n"
           "\ts_nop 7 // 00000000100C: BF800007\n"
           "\tv_mov_b32_e32 v66, 0 // 000000001010: 7E840280\n")
    f = tmp_path / "o.s"
    f.write_text(obj)
    assert shc.scan(str(f)) == 1


@pytest.mark.skipif(not os.path.exists(LIB), reason="libtcx.so not built (run __graft_entry__.build())")
def test_library_has_no_store_data_hazard(tmp_path):
    files = shc.lib_listings(LIB, str(tmp_path))
    assert len(files) >= 20  # one code object per HIP translation unit
    assert sum(shc.scan(p) for p in files) == 0
