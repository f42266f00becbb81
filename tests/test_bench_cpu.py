"""CPU: the launcher logic of bench.py that runs before any GPU call."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_refuses_gpus_not_equal_world(tmp_path):
    """Under a launcher (WORLD_SIZE set) a --gpus that disagrees with the world is an error, not a
    silently mislabelled line."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       cwd=str(tmp_path), capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stdout + r.stderr), r.stderr[-2000:]
