"""GPU, world size 2 on ONE GPU: the real batch-DP training scripts under torchrun.

`TCX_DIST_BACKEND=gloo` lets two ranks share the box's single MI355X (RCCL refuses two ranks per
device), so the code of SURVEY.md §8(e) rows e1-e3 executes end to end: `_common.init_dp`, the
per-rank shard of every global batch (`DeviceBatches`), `--global-draws 1` slicing, the bucketed
all-reduce with gradient-as-bucket-view (`dist.BucketedGradAllReduce`), the latent-cache broadcast,
`allreduce_scalar_mean`, and the lead-only writes and sample grids (whose draws are rolled back so
the ranks' generators stay in step).  Each world-2 run is compared with a world-1 run of the same
global batch and seed: every checkpoint tensor after the Adam steps, and the logged losses.

The reference step bodies an N-rank run must equal: /root/reference/scripts/train_sde_score_model.py:212-243,
/root/reference/scripts/train_vae.py:292-321, /root/reference/scripts/train_diffusion_prior.py:240-277.

Gate: a world-2 gradient is the mean of two half-batch means (the same sum in a different order), so
it differs from the world-1 gradient by fp32 rounding only (~1e-7 relative, tests/test_gpu_dp.py).
Adam turns gradient differences into parameter differences of at most lr per step where a gradient
component is at rounding-noise level (its update is ~sign(g) * lr); the gate is therefore
max |p2 - p1| <= 1e-5 * max(|p1|max, 1) per tensor (lr 1e-4 * 6 steps would allow 6e-4 if such a
component flipped), and the mean difference must be far below it.
"""
import os
import re
import shutil
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPTS = os.path.join(ROOT, "vae-diffusion-toy-crystals_amd", "scripts")
REL_GATE = 1e-5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run(cwd, world, script, *args):
    path = os.path.join(SCRIPTS, script)
    env = dict(os.environ)
    if world == 1:
        cmd = [sys.executable, path]
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            env.pop(k, None)
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(world),
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), path]
        env["TCX_DIST_BACKEND"] = "gloo"
        env["OMP_NUM_THREADS"] = "4"
    cmd += [str(a) for a in args]
    os.makedirs(cwd, exist_ok=True)
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True, timeout=400, env=env)
    assert r.returncode == 0, f"{script} (world {world}) failed:\n{r.stdout[-4000:]}\n{r.stderr[-4000:]}"
    return r.stdout


def compare_tensors(a: dict, b: dict, label: str):
    assert set(a) == set(b), label
    worst = (0.0, "")
    for k in sorted(a):
        x, y = a[k], b[k]
        if isinstance(x, dict):
            compare_tensors(x, y, f"{label}.{k}")
            continue
        if not torch.is_tensor(x):
            assert x == y, (label, k, x, y)
            continue
        assert x.shape == y.shape and x.dtype == y.dtype, (label, k)
        if not x.is_floating_point():
            assert torch.equal(x, y), (label, k)
            continue
        d = (x.double() - y.double()).abs()
        scale = max(float(x.double().abs().max()), 1.0)
        rel = float(d.max()) / scale
        worst = max(worst, (rel, k))
        assert rel <= REL_GATE, f"{label}.{k}: max|diff| {float(d.max()):.3e} = {rel:.3e} of scale {scale:.3e}"
        assert float(d.mean()) <= REL_GATE * scale / 10, (label, k, float(d.mean()))
    print(f"{label}: worst tensor {worst[1]} at {worst[0]:.3e} of its scale")


def losses(stdout, key):
    return [float(v) for v in re.findall(rf"{key}=([0-9.eE+-]+)", stdout)]


@pytest.fixture(scope="module")
def dataset(tmp_path_factory):
    d = tmp_path_factory.mktemp("dpdata")
    g = torch.Generator().manual_seed(0)
    N = 96
    x = (torch.rand(N, 1, 64, 64, generator=g) * 255).to(torch.uint8)
    y_cat = torch.arange(N) % 4
    y_cont = torch.zeros(N, 4)
    y_cont[:, 1] = torch.rand(N, generator=g) * 1.047
    path = d / "toy.pt"
    torch.save({"x_u8": x, "y_cat": y_cat, "y_cont": y_cont}, path)
    return str(path)


def test_score_script_world2_equals_world1(tmp_path, dataset):
    """train_sde_score_model.py, base 32, global batch 32, 2 epochs x 3 steps, EMA, a sample grid
    after epoch 1 on rank 0 only (the lockstep case): checkpoint (model, EMA, Adam moments) and
    loss_hist of world 2 equal world 1."""
    args = ["--data-path", dataset, "--base-ch", 32, "--batch-size", 32, "--epochs", 2, "--sample-every", 1,
            "--sample-steps", 2, "--ema-decay", 0.9, "--seed", 3]
    out = {}
    for world in (1, 2):
        od = tmp_path / f"w{world}"
        out[world] = run(tmp_path, world, "train_sde_score_model.py", *args, "--out-dir", od)
    c1 = torch.load(tmp_path / "w1" / "checkpoints" / "sde_score_model_last.pt", map_location="cpu", weights_only=True)
    c2 = torch.load(tmp_path / "w2" / "checkpoints" / "sde_score_model_last.pt", map_location="cpu", weights_only=True)
    assert c1["epoch_next"] == c2["epoch_next"] == 2
    compare_tensors(c1["model"], c2["model"], "model")
    compare_tensors(c1["ema"], c2["ema"], "ema")
    for i in c1["opt"]["state"]:
        compare_tensors(c1["opt"]["state"][i], c2["opt"]["state"][i], f"adam[{i}]")
    l1, l2 = c1["loss_hist"], c2["loss_hist"]
    print("loss_hist world1", l1, "world2", l2)
    assert len(l1) == len(l2) == 2 and all(abs(a - b) <= 1e-5 * abs(a) for a, b in zip(l1, l2))
    # rank 0 alone logs and writes: one line per epoch, one checkpoint, one grid per epoch
    assert out[2].count("epoch 001/2: loss=") == 1 and out[2].count("epoch 002/2: loss=") == 1
    assert len(open(tmp_path / "w2" / "metrics.jsonl").read().splitlines()) == 2
    assert sorted(p.name for p in (tmp_path / "w2" / "results").iterdir()) == [
        "sde_loss.png", "sde_samples_epoch_001.png", "sde_samples_epoch_002.png"]


def test_vae_and_prior_scripts_world2_equal_world1(tmp_path, dataset):
    """train_vae.py (CondVAE, cond-drop 0.1: the reparameterise and keep-mask draws are global-batch
    draws sliced per rank) and train_diffusion_prior.py (width 256; latent cache built on rank 0 and
    broadcast; DDIM sample grid each epoch on rank 0 only) at world 2 equal world 1."""
    vae_args = ["--data-path", dataset, "--epochs", 2, "--batch-size", 32, "--cond-drop", 0.1, "--seed", 5]
    out = {}
    for world in (1, 2):
        out[world] = run(tmp_path / f"vae{world}", world, "train_vae.py", *vae_args)
    v1 = torch.load(tmp_path / "vae1" / "checkpoints" / "vae_last.pt", map_location="cpu", weights_only=True)
    v2 = torch.load(tmp_path / "vae2" / "checkpoints" / "vae_last.pt", map_location="cpu", weights_only=True)
    compare_tensors(v1, v2, "vae")
    for key in ("loss", "recon", "kl"):
        a, b = losses(out[1], key), losses(out[2], key)
        print(key, a, b)
        assert len(a) == len(b) == 2 and all(abs(x - y) <= 1e-4 * max(abs(x), 1e-3) for x, y in zip(a, b)), key
    assert out[2].count("epoch 02/2 loss=") == 1

    # the prior at world 1, at world 2 and 3 with ZeRO-1 (the default: reduce-scatter, sharded fused Adam,
    # all-gather; 3 ranks make shards that cut tensors at odd offsets) and at world 2 with the bucketed
    # all-reduce (--zero 0).  Global batch 48 (divisible by 2 and 3), 2 steps per epoch.
    prior_args = ["--data-path", dataset, "--epochs", 2, "--batch-size", 48, "--width", 256, "--T", 50,
                  "--ddim-steps", 3, "--latent-cache", "lat.pt", "--seed", 7]
    runs = {"w1": (1, []), "w2": (2, []), "w3": (3, []), "w2ar": (2, ["--zero", 0])}
    ck, outp = {}, {}
    for name, (world, extra) in runs.items():
        d = tmp_path / f"prior_{name}"
        os.makedirs(d / "checkpoints", exist_ok=True)
        shutil.copy(tmp_path / "vae1" / "checkpoints" / "vae_last.pt", d / "checkpoints" / "vae_last.pt")
        outp[name] = run(d, world, "train_diffusion_prior.py", *prior_args, *extra)
        ck[name] = torch.load(d / "checkpoints" / "diffusion_prior_last.pt", map_location="cpu", weights_only=True)
    for name in ("w2", "w3", "w2ar"):
        compare_tensors(ck["w1"], ck[name], f"prior {name}")
        a, b = losses(outp["w1"], "diffusion_loss"), losses(outp[name], "diffusion_loss")
        print("diffusion_loss", name, a, b)
        assert len(a) == len(b) == 2 and all(abs(x - y) <= 1e-5 * abs(x) for x, y in zip(a, b))
        assert outp[name].count("epoch 02/2 diffusion_loss=") == 1
    # ZeRO-1 at world 2 vs the all-reduce form at world 2: the same two-term sums, the same element-wise Adam
    zd = max(float((ck["w2"][k].double() - ck["w2ar"][k].double()).abs().max()) for k in ck["w2"])
    print(f"prior world 2: ZeRO-1 vs bucketed all-reduce max |diff| {zd:.3e}")
    assert zd == 0.0
    l1 = torch.load(tmp_path / "prior_w1" / "lat.pt", map_location="cpu", weights_only=True)
    for name in ("w2", "w3"):
        assert torch.equal(l1["z0"], torch.load(tmp_path / f"prior_{name}" / "lat.pt", map_location="cpu",
                                                weights_only=True)["z0"])
