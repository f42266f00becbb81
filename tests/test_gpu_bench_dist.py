"""GPU: `bench.py --gpus 2` end to end on the box's one GPU (ranks over gloo).

The driver's scaling run calls `bench.py --gpus N` (or torchrun with WORLD_SIZE = N).  Here the
bench launches its two ranks itself (`_spawn_ranks`: torch.distributed.run as a child process),
`TCX_DIST_BACKEND=gloo` lets both share the one MI355X (RCCL refuses two ranks per device), and the
whole N > 1 branch executes: process-group init, the barriers, the max-over-ranks elapsed time, the
per-rank conditioning slice and Philox element offset.  The 2-rank images must equal a 1-rank run of
the global batch (2 x 128 = 256) with the same seed bit for bit: sampling shards over images with
one noise stream for the whole batch (/root/reference/src/toycrystals/models/sde_score_model.py:508-569,
one `torch.randn` per step for the batch at :537,558).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(tmp_path, tag, *args, world_env=None):
    out = str(tmp_path / f"{tag}.npy")
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["TCX_DIST_BACKEND"] = "gloo"
    env.setdefault("OMP_NUM_THREADS", "4")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0", "--n-steps", "3",
           "--no-cpu-baseline", "--fp32-passes", "0", "--save-images", out] + [str(a) for a in args]
    r = subprocess.run(cmd, cwd=str(tmp_path), capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, f"bench {args} failed:\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0]), np.load(out)


def test_bench_two_ranks_equal_one_rank_of_global_batch(tmp_path):
    line2, img2 = _bench(tmp_path, "w2", "--gpus", "2")
    assert line2["n_gpus"] == 2 and line2["config"]["global_batch"] == 256, line2
    assert line2["config"]["batch_per_gpu"] == 128 and line2["scaling"] == "weak"
    assert line2["value"] > 0 and line2["config"]["parallelism"].startswith("dp2")
    assert "cpu_baseline" not in line2
    line1, img1 = _bench(tmp_path, "w1", "--gpus", "1", "--batch", "256")
    assert line1["n_gpus"] == 1 and line1["config"]["global_batch"] == 256
    assert img2.shape == img1.shape == (256, 1, 64, 64)
    assert np.isfinite(img2).all()
    diff = int((img2 != img1).sum())
    print(f"2-rank vs 1-rank images: {diff} differing pixels of {img1.size}; "
          f"2-rank {line2['value']:.3f} img/s (2 ranks on one GPU), 1-rank {line1['value']:.3f}")
    assert diff == 0

