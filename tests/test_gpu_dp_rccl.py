"""GPU: the RCCL data path of batch-DP training, executed on the one-GPU box.

The world-2 tests (test_gpu_dp_scripts.py) share one GPU between two ranks, which RCCL refuses, so
they run gloo with host-staged collectives.  Here the real scripts run under
`torchrun --nproc-per-node 1` with backend nccl (RCCL) and TCX_DP_FORCE=1, which builds the process
group at world 1 and keeps every collective of the N-GPU path: `init_process_group(device_id=...)`
(eager communicator on the rank's device), the bucketed gradient all-reduce launched asynchronously
from post-accumulate-grad hooks on device buckets and waited with `Work.wait` (score net), the
ZeRO-1 reduce-scatter / sharded fused Adam / all-gather (prior), the latent-cache broadcast and the
generator-state broadcast.  At world 1 every collective is an identity, so the checkpoint must equal
the non-DP run's BIT FOR BIT: any ordering bug between RCCL's stream and the libtcx kernels on the
compute stream (a gradient read before backward wrote it, a parameter used before the all-gather
landed) shows up as a difference.

Reference step bodies: /root/reference/scripts/train_sde_score_model.py:217-243,
/root/reference/scripts/train_diffusion_prior.py:248-277.
"""
import os
import shutil
import subprocess
import sys

import pytest
import torch

from test_gpu_dp_scripts import SCRIPTS, _free_port, dataset  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu


def run(cwd, dp, script, *args):
    path = os.path.join(SCRIPTS, script)
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "TCX_DIST_BACKEND", "TCX_DP_FORCE"):
        env.pop(k, None)
    if dp:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), path]
        env.update(TCX_DP_FORCE="1", TCX_DIST_BACKEND="nccl", NCCL_DEBUG="INFO", OMP_NUM_THREADS="4")
    else:
        cmd = [sys.executable, path]
    cmd += [str(a) for a in args]
    os.makedirs(cwd, exist_ok=True)
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True, timeout=400, env=env)
    assert r.returncode == 0, f"{script} (dp={dp}) failed:\n{r.stdout[-4000:]}\n{r.stderr[-4000:]}"
    return r.stdout + r.stderr


def assert_bitwise(a, b, label):
    assert set(a) == set(b), label
    for k in sorted(a):
        x, y = a[k], b[k]
        if isinstance(x, dict):
            assert_bitwise(x, y, f"{label}.{k}")
        elif torch.is_tensor(x):
            assert x.shape == y.shape and x.dtype == y.dtype, (label, k)
            assert torch.equal(x, y), f"{label}.{k}: max |diff| {float((x.double() - y.double()).abs().max()):.3e}"
        else:
            assert x == y, (label, k, x, y)


def test_score_and_prior_scripts_on_rccl_equal_non_dp(tmp_path, dataset):  # noqa: F811
    score_args = ["--data-path", dataset, "--base-ch", 32, "--batch-size", 32, "--epochs", 2, "--sample-every", 1,
                  "--sample-steps", 2, "--ema-decay", 0.9, "--seed", 3]
    out = {}
    for dp in (False, True):
        out[dp] = run(tmp_path, dp, "train_sde_score_model.py", *score_args, "--out-dir", tmp_path / f"s{int(dp)}")
    assert "NCCL INFO" in out[True], "RCCL did not initialise (no NCCL INFO lines)"
    c0 = torch.load(tmp_path / "s0" / "checkpoints" / "sde_score_model_last.pt", map_location="cpu", weights_only=True)
    c1 = torch.load(tmp_path / "s1" / "checkpoints" / "sde_score_model_last.pt", map_location="cpu", weights_only=True)
    assert_bitwise(c0["model"], c1["model"], "score model")
    assert_bitwise(c0["ema"], c1["ema"], "score ema")
    assert_bitwise(c0["opt"]["state"], c1["opt"]["state"], "score adam")
    assert c0["loss_hist"] == c1["loss_hist"]

    vae_args = ["--data-path", dataset, "--epochs", 1, "--batch-size", 32, "--seed", 5]
    vout = {}
    for dp in (False, True):
        vout[dp] = run(tmp_path / f"vae{int(dp)}", dp, "train_vae.py", *vae_args)
    v0 = torch.load(tmp_path / "vae0" / "checkpoints" / "vae_last.pt", map_location="cpu", weights_only=True)
    v1 = torch.load(tmp_path / "vae1" / "checkpoints" / "vae_last.pt", map_location="cpu", weights_only=True)
    assert_bitwise(v0, v1, "vae")

    prior_args = ["--data-path", dataset, "--epochs", 2, "--batch-size", 32, "--width", 256, "--T", 50,
                  "--ddim-steps", 3, "--latent-cache", "lat.pt", "--seed", 7]
    pk = {}
    for dp in (False, True):
        d = tmp_path / f"prior{int(dp)}"
        os.makedirs(d / "checkpoints", exist_ok=True)
        shutil.copy(tmp_path / "vae0" / "checkpoints" / "vae_last.pt", d / "checkpoints" / "vae_last.pt")
        o = run(d, dp, "train_diffusion_prior.py", *prior_args)
        if dp:
            assert "NCCL INFO" in o
        pk[dp] = torch.load(d / "checkpoints" / "diffusion_prior_last.pt", map_location="cpu", weights_only=True)
    assert_bitwise(pk[False], pk[True], "prior (ZeRO-1 on RCCL vs non-DP)")
    print("score / vae / prior on RCCL at world 1 (TCX_DP_FORCE=1): bit-identical to the non-DP runs")


def test_zero_adam_world1_equals_fused_adam():
    """ZeroAdam without a process group (one flat shard per bucket) against optim.Adam per tensor: the same
    element-wise update, so bit-identical parameters over several steps; the packed-weight cache key changes
    after each step (the version bump)."""
    sys.path.insert(0, os.path.join(os.path.dirname(SCRIPTS)))
    from toycrystals_amd.dist import ZeroAdam
    from toycrystals_amd.optim import Adam
    torch.manual_seed(0)
    mk = lambda: torch.nn.Sequential(torch.nn.Linear(37, 300), torch.nn.SiLU(), torch.nn.Linear(300, 11)).cuda()
    m0, m1 = mk(), mk()
    m1.load_state_dict(m0.state_dict())
    o0 = Adam(m0.parameters(), lr=1e-2, weight_decay=0.01)
    o1 = ZeroAdam(list(m1.parameters()), lr=1e-2, weight_decay=0.01, bucket_mb=0.01)  # several buckets
    assert len(o1.buckets) > 1
    x = torch.randn(64, 37, device="cuda")
    for _ in range(4):
        v_before = [p._version for p in m1.parameters()]
        o0.zero_grad(set_to_none=True)
        m0(x).square().mean().backward()
        o0.step()
        o1.zero_grad()
        m1(x).square().mean().backward()
        o1.step()
        assert all(p._version > v for p, v in zip(m1.parameters(), v_before))
    for a, b in zip(m0.parameters(), m1.parameters()):
        assert torch.equal(a, b)
