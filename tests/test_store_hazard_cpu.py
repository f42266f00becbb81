"""The built library carries no 16-B store whose data VGPRs the next instruction overwrites (the
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


@pytest.mark.skipif(not os.path.exists(LIB), reason="libtcx.so not built (run __graft_entry__.build())")
def test_library_has_no_store_data_hazard(tmp_path):
    files = shc.lib_listings(LIB, str(tmp_path))
    assert len(files) >= 20  # one code object per HIP translation unit
    assert sum(shc.scan(p) for p in files) == 0
