"""k_conv3m (h2 sources, PRO 0) at 64^2 and 32^2 rows, Bt = 256, Cout = 96, single source, Cin = 96 .. 384:
time against Cin, to separate the per-workgroup fixed cost (pipeline fill, epilogue) from the per-chunk
cost (a linear fit t = a + b Cin per row width).  Uses tools/convbench.py's bench()."""
import os
import sys

os.environ["LAYER"] = "none"  # convbench's module-level loop runs nothing
os.environ.setdefault("H2", "1")
os.environ.setdefault("PRO", "0")
os.environ.setdefault("GN", "1")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import convbench as cb  # noqa: E402
import numpy as np  # noqa: E402

for _ in range(3):  # clocks up before the measured sweep (the first layer measured ~15 % slow cold)
    cb.bench("warm", 64, 384, 0, 96, 3, 1, 1, 0, reps=20)
for H in (64, 32):
    cins, ts = [], []
    for cin in (96, 192, 288, 384):
        us, fl = cb.bench(f"cin{cin}", H, cin, 0, 96, 3, 1, 1, 0, reps=20)
        cins.append(cin)
        ts.append(us)
    b, a = np.polyfit(cins, ts, 1)
    print(f"H {H}: t = {a:.1f} us + {b:.3f} us per input channel (fixed share at Cin 96: {a / ts[0]:.2f})", flush=True)
