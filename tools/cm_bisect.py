"""Whole-forward A/B of TCX_SKIP_CM settings (one child process per setting): max |difference| of the
eps output against TCX_SKIP_CM=0 at 64^2 and 32^2 (f16x3, B = 64)."""
import os
import sys
import tempfile
import pathlib

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_passes import _forward  # noqa: E402

tmp = pathlib.Path(tempfile.mkdtemp())
for H in (64, 32):
    ref = _forward(tmp, f"r{H}", {"TCX_SKIP_CM": "0"}, "f16x3", 64, H)
    ref2 = _forward(tmp, f"r2{H}", {"TCX_SKIP_CM": "0"}, "f16x3", 64, H)
    print(f"H {H}: SKIP_CM 0 vs 0 (two processes): max {float(np.abs(ref - ref2).max()):.3e}", flush=True)
    for m in ("1", "2", "3"):
        a = _forward(tmp, f"m{m}{H}", {"TCX_SKIP_CM": m}, "f16x3", 64, H)
        print(f"H {H}: SKIP_CM {m} vs 0: max {float(np.abs(a - ref).max()):.3e}", flush=True)
