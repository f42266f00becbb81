"""GPU: the four CLI mirrors end to end on a tiny synthetic disk dataset (the reference's
build_dataset.py format): checkpoint layout and keys, metrics.jsonl, --resume, sampling from a
checkpoint, VAE -> latent cache -> prior chain.  Each script runs as a child process in turn."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPTS = os.path.join(ROOT, "vae-diffusion-toy-crystals_amd", "scripts")


def run(cwd, script, *args):
    cmd = [sys.executable, os.path.join(SCRIPTS, script)] + [str(a) for a in args]
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, f"{script} failed:\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    return r.stdout


@pytest.fixture(scope="module")
def dataset(tmp_path_factory):
    d = tmp_path_factory.mktemp("data")
    g = torch.Generator().manual_seed(0)
    N = 96
    x = (torch.rand(N, 1, 64, 64, generator=g) * 255).to(torch.uint8)
    y_cat = torch.arange(N) % 4
    y_cont = torch.zeros(N, 4)
    y_cont[:, 1] = torch.rand(N, generator=g) * 1.047
    path = d / "toy.pt"
    torch.save({"x_u8": x, "y_cat": y_cat, "y_cont": y_cont}, path)
    return str(path)


def test_score_train_resume_and_sample(tmp_path, dataset):
    out = tmp_path / "run"
    common = ["--data-path", dataset, "--out-dir", out, "--base-ch", 16, "--batch-size", 32, "--sample-steps", 2,
              "--ema-decay", 0.9]
    run(tmp_path, "train_sde_score_model.py", *common, "--epochs", 1)
    ck = out / "checkpoints" / "sde_score_model_last.pt"
    obj = torch.load(ck, map_location="cpu", weights_only=True)
    assert set(obj) == {"epoch_next", "model", "opt", "loss_hist", "config", "ema"}
    assert obj["epoch_next"] == 1 and len(obj["loss_hist"]) == 1
    assert set(obj["opt"]["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}
    assert (out / "results" / "sde_samples_epoch_001.png").exists()
    run(tmp_path, "train_sde_score_model.py", *common, "--epochs", 2, "--resume")
    obj = torch.load(ck, map_location="cpu", weights_only=True)
    assert obj["epoch_next"] == 2 and len(obj["loss_hist"]) == 2
    lines = [json.loads(s) for s in open(out / "metrics.jsonl")]
    assert [r["epoch"] for r in lines] == [1, 2]
    assert all(0.0 < r["loss"] < 10.0 for r in lines)
    msg = run(tmp_path, "sample_sde_score_model.py", "--out-dir", out, "--steps", 3, "--cfg", 1.5, "--sampler", "sde",
              "--use-ema", 1)
    assert "Saved samples" in msg
    assert any(p.name.startswith("samples_ckpt-sde_score_model_last_steps3_cfg1.50") for p in (out / "results").iterdir())


def test_vae_then_prior(tmp_path, dataset):
    run(tmp_path, "train_vae.py", "--data-path", dataset, "--epochs", 2, "--batch-size", 32, "--cond-drop", 0.1)
    sd = torch.load(tmp_path / "checkpoints" / "vae_last.pt", map_location="cpu", weights_only=True)
    assert "enc_fc.weight" in sd and sd["enc_fc.weight"].shape == (256, 4096 + 8)
    for f in ("vae_recon.png", "vae_samples_prior.png", "vae_samples_mop.png", "vae_loss.png"):
        assert (tmp_path / "results" / f).exists(), f
    run(tmp_path, "train_diffusion_prior.py", "--data-path", dataset, "--epochs", 2, "--batch-size", 32, "--width", 64,
        "--T", 50, "--ddim-steps", 3, "--latent-cache", tmp_path / "lat.pt")
    lat = torch.load(tmp_path / "lat.pt", map_location="cpu", weights_only=True)
    assert set(lat) == {"z0", "y_cat", "y_cont", "z_mean", "z_std"} and lat["z0"].shape == (96, 32)
    psd = torch.load(tmp_path / "checkpoints" / "diffusion_prior_last.pt", map_location="cpu", weights_only=True)
    assert psd["blocks.7.fc1.weight"].shape == (256, 64)
    assert (tmp_path / "results" / "diffusion_samples.png").exists()
    run(tmp_path, "train_diffusion_prior.py", "--data-path", dataset, "--width", 64, "--T", 50, "--ddim-steps", 3,
        "--latent-cache", tmp_path / "lat.pt", "--sample-only")


def test_build_dataset_and_preview(tmp_path):
    """build_dataset.py writes the reference's file ({x_u8 [N,1,S,S] uint8, y_cat [N] int64,
    y_cont [N,4] f32}) from the GPU renderer; preview_data.py saves the 6 x 6 PNG grid."""
    out = tmp_path / "data" / "toy.pt"
    run(tmp_path, "build_dataset.py", "--out", out, "--n-samples", 50, "--render-batch", 16)
    d = torch.load(out, weights_only=True)
    assert set(d) == {"x_u8", "y_cat", "y_cont"}
    assert d["x_u8"].shape == (50, 1, 64, 64) and d["x_u8"].dtype == torch.uint8
    assert d["y_cat"].shape == (50,) and d["y_cat"].dtype == torch.int64
    assert d["y_cont"].shape == (50, 4) and d["y_cont"].dtype == torch.float32
    assert int(d["x_u8"].max()) == 255  # every image is max-normalised
    run(tmp_path, "preview_data.py")
    png = tmp_path / "results" / "preview_toycrystals.png"
    assert png.exists() and png.stat().st_size > 10_000
