"""GPU: the drop-in modules and samplers (HIP path through the C ABI) vs the reference goldens
and the numpy oracle.

Tolerances (north star: <= 1e-4 max-abs vs the CPU reference, fp32):
  * one U-Net forward / CFG evaluation: 2e-5 x max(1, |eps|max)  (observed ~1e-6 relative)
  * short sampler trajectories with injected noise: 1e-4 x max(1, |x0|max)
  * samplers: 1e-4 max-abs on the clamped [0,1] image (the metric's output) AND 1e-4 relative
    (to max(1, |x0_hat|max)) on the unclamped x0_hat of every golden; the 300-step reverse SDE
    runs on a genuinely trained base_ch-96 model (98.5 % of its golden pixels unsaturated).
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def cu(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def unet(base, sd=None):
    from toycrystals_amd.models.sde_score_model import CondUNetTiny
    torch.manual_seed(0)
    m = CondUNetTiny(4, 4, base)
    if sd is not None:
        m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return m.cuda().eval()


@pytest.fixture(params=["f16x3", "fp32"])
def prec(request):
    """Run the score-U-Net evaluator with each conv precision (the split f16x3 path applies at
    base_ch % 32 == 0; other nets fall back to fp32 inside either setting)."""
    from toycrystals_amd import _lib
    old = _lib.conv_precision()
    _lib.set_conv_precision(request.param)
    yield request.param
    _lib.set_conv_precision(old)


def rel_err(a, ref):
    return float(np.abs(a - ref).max()) / max(1.0, float(np.abs(ref).max()))


@pytest.mark.parametrize("name,base,stored", [("unet16_b3", 16, True), ("unet96_b2", 96, False),
                                              ("unet32_b2_h32", 32, False), ("unet96_b2_h256", 96, False)])
@pytest.mark.parametrize("grad", [False, True], ids=["fused", "autograd"])
def test_unet_forward_vs_reference(golden, name, base, stored, grad, prec):
    """The fused evaluator (no grad) and the autograd training chain (grad) against the reference."""
    g = golden(name)
    sd = {k[2:]: v for k, v in g.items() if k.startswith("w/")} if stored else None
    m = unet(base, sd)
    with torch.set_grad_enabled(grad):
        eps = m(cu(g["x_t"]), cu(g["t"]), cu(g["y_cat"]), cu(g["y_cont"]))
        assert eps.requires_grad == grad
        eps = eps.detach().cpu().numpy()
    assert eps.shape == g["eps"].shape
    assert rel_err(eps, g["eps"]) < 2e-5


def test_predict_eps_cfg_vs_reference(golden):
    from toycrystals_amd.models.sde_score_model import predict_eps_cfg
    g = golden("cfg16_b3")
    m = unet(16)
    args = (cu(g["x_t"]), cu(g["t"]), cu(g["y_cat"]), cu(g["y_cont"]))
    e = predict_eps_cfg(m, *args, guidance_scale=1.5).cpu().numpy()
    assert rel_err(e, g["eps"]) < 2e-5
    e0 = predict_eps_cfg(m, *args, guidance_scale=0.0).cpu().numpy()
    assert rel_err(e0, g["eps0"]) < 2e-5


def test_batch_independence_and_oracle_at_full_size(prec):
    """B=128 (the metric's batch) with CFG doubling to 256: every sample equals the same sample
    evaluated alone, and a random subset matches the fp64 oracle."""
    from oracle.score_model import ScoreUNet, predict_eps_cfg as o_cfg
    from toycrystals_amd.models.sde_score_model import predict_eps_cfg
    m = unet(96)
    B = 128
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(B, 1, 64, 64, generator=gen)
    t = torch.full((B,), 0.42)
    y_cat = torch.arange(B) % 4
    y_cont = torch.zeros(B, 4)
    y_cont[:, 1] = torch.linspace(0, math.pi / 3, B)
    e = predict_eps_cfg(m, x.cuda(), t.cuda(), y_cat.cuda(), y_cont.cuda(), 1.5).cpu()
    idx = [0, 77, 127]
    e_small = predict_eps_cfg(m, x[idx].cuda(), t[idx].cuda(), y_cat[idx].cuda(), y_cont[idx].cuda(), 1.5).cpu()
    assert torch.allclose(e[idx], e_small, atol=1e-5, rtol=0)
    o = ScoreUNet({k: v.cpu().numpy() for k, v in m.state_dict().items()}, dt=np.float64)
    ref = o_cfg(o, x[idx].double().numpy(), t[idx].numpy(), y_cat[idx].numpy(), y_cont[idx].numpy(), 1.5)
    assert rel_err(e[idx].numpy(), ref) < 2e-5


def test_256px_pass_chunking_is_batch_independent():
    """256x256 (config 5) with CFG: B=48 doubles to 96 rows, above the 84-image cap that keeps every
    activation under 2 GiB (32-bit buffer offsets), so the evaluator runs two passes (42 + 6
    images).  Every sample must equal the same sample evaluated alone."""
    from toycrystals_amd.models.sde_score_model import predict_eps_cfg
    m = unet(96)
    B = 48
    gen = torch.Generator().manual_seed(9)
    x = torch.randn(B, 1, 256, 256, generator=gen)
    t = torch.rand(B, generator=gen) * 0.9 + 0.05
    y_cat = torch.arange(B) % 5
    y_cont = torch.rand(B, 4, generator=gen)
    e = predict_eps_cfg(m, x.cuda(), t.cuda(), y_cat.cuda(), y_cont.cuda(), 1.5).cpu()
    assert torch.isfinite(e).all()
    for idx in ([0], [41, 42], [47]):
        e1 = predict_eps_cfg(m, x[idx].cuda(), t[idx].cuda(), y_cat[idx].cuda(), y_cont[idx].cuda(), 1.5).cpu()
        assert torch.allclose(e[idx], e1, atol=1e-5, rtol=0)


def check_sampler_outputs(what, out, x0_hat, g, x0_gate=1e-4):
    """The reference's two outputs of a sampler call: the clamped [0,1] image (the metric's output,
    1e-4 max-abs) and the unclamped projection x0_hat (sde_score_model.py:500,566), gated relative
    to max(1, |x0_hat|max).  The clamp saturates most pixels of an untrained net's image, so the
    x0_hat gate is the one that sees every pixel; the image must also equal the reference's own
    map of OUR x0_hat (clamp((x0_hat + 1)/2, 0, 1), :568-569) to rounding."""
    img_err = float(np.abs(out - g["out"]).max())
    x0_err = rel_err(x0_hat, g["x0_unclamped"])
    unsat = float(np.mean((g["out"] > 0.0) & (g["out"] < 1.0)))
    print(f"{what}: image max-abs {img_err:.3e}, x0_hat rel {x0_err:.3e} "
          f"(|x0|max {np.abs(g['x0_unclamped']).max():.3g}, unsaturated {100 * unsat:.1f} %)")
    assert img_err < 1e-4
    assert x0_err < x0_gate
    assert np.abs(np.clip((x0_hat + 1.0) * 0.5, 0.0, 1.0) - out).max() < 1e-6


def run_sde(m, g, noise, shape, **kw):
    from toycrystals_amd.models.sde_score_model import VPSDE, sample_reverse_sde_euler_maruyama
    args = (m, VPSDE(float(g["beta_min"]), float(g["beta_max"])), cu(g["y_cat"]), cu(g["y_cont"]), shape)
    kw = dict(n_steps=int(g["steps"]), guidance_scale=float(g["cfg"]), t_end=float(g["t_end"]), noise=noise, **kw)
    out = sample_reverse_sde_euler_maruyama(*args, **kw).cpu().numpy()
    x0 = sample_reverse_sde_euler_maruyama(*args, return_x0_hat=True, **kw).cpu().numpy()
    return out, x0


def run_ode(m, g, x_init, **kw):
    from toycrystals_amd.models.sde_score_model import VPSDE, sample_probability_flow_ode
    args = (m, VPSDE(float(g["beta_min"]), float(g["beta_max"])), cu(g["y_cat"]), cu(g["y_cont"]), tuple(x_init.shape))
    kw = dict(n_steps=int(g["steps"]), guidance_scale=float(g["cfg"]), t_end=float(g["t_end"]), **kw)
    out = sample_probability_flow_ode(*args, x_init=x_init.clone(), **kw).cpu().numpy()
    x0 = sample_probability_flow_ode(*args, x_init=x_init.clone(), return_x0_hat=True, **kw).cpu().numpy()
    return out, x0


@pytest.mark.parametrize("name", ["sde16_3step", "sde96_2step_b2"])
def test_sde_sampler_vs_reference(golden, name, prec):
    g = golden(name)
    m = unet(int(g["base_ch"]))
    out, x0 = run_sde(m, g, cu(g["noise"]), tuple(g["noise"].shape[1:]))
    check_sampler_outputs(name, out, x0, g)


def test_ode_sampler_vs_reference(golden):
    g = golden("ode16_2step")
    m = unet(16)
    out, x0 = run_ode(m, g, cu(g["noise"][0]))
    check_sampler_outputs("ode16_2step", out, x0, g)


def test_trained_ode20_vs_reference(golden, prec):
    g = golden("ode32_trained_20")
    m = unet(32, golden("trained32_state"))
    torch.manual_seed(int(g["noise_seed"]))
    x = torch.randn((int(g["B"]), 1, 64, 64))
    out, x0 = run_ode(m, g, x.cuda())
    check_sampler_outputs("ode32_trained_20", out, x0, g)


@pytest.mark.parametrize("lanes", [1, 4])
def test_trained_sde300_vs_reference(golden, prec, monkeypatch, lanes):
    """The metric's sampler (300-step reverse SDE, CFG 1.5, t_end 0.005, base_ch 96) end to end on
    a genuinely trained model — tests/golden/trained96_ema.npz, the EMA weights of the README recipe
    (40 epochs, profiles/r02_a_recipe40_metrics.jsonl) — against the REFERENCE's CPU run of the same
    weights and draws (tests/golden/make_goldens.py trained96).  98.5 % of the golden image's
    pixels are unsaturated, so the clamped image and x0_hat both see the whole trajectory.

    Noise floor: the fp32 reference itself differs from the fp64 trajectory of the same draws by
    3.0e-5 relative on x0_hat (tests/golden/sde96_trained_300_fp64.npz, make_fp64_floor.py); this
    path is gated at 1e-4 against BOTH.  A single step-table scalar perturbed by 1e-5 moves x0_hat
    by at most ~2e-5 (printed), below that floor: no gate can see it.  Discrimination: alpha(t_end)
    scaled by 1 + 2e-4 (a ~2e-4 change of x0_hat, ~7x the floor) must fail the gate.

    `lanes` = 4 is bench.py's timed configuration (tcx_set_sample_lanes(4): the batch as four
    concurrent per-stream chains, two images each here): the same gates, and the outputs must equal
    the one-lane run bit for bit."""
    import toycrystals_amd.models.sde_score_model as S
    from toycrystals_amd._lib import lib
    from toycrystals_amd.models.sde_score_model import host_noise
    g = golden("sde96_trained_300")
    f64 = golden("sde96_trained_300_fp64")["x0_fp64"]
    m = unet(96, golden("trained96_ema"))
    B, steps = int(g["B"]), int(g["steps"])
    torch.manual_seed(int(g["noise_seed"]))
    noise = host_noise((B, 1, 64, 64), steps + 1).cuda()
    prev = lib().tcx_set_sample_lanes(lanes)
    try:
        out, x0 = run_sde(m, g, noise, (B, 1, 64, 64))
    finally:
        lib().tcx_set_sample_lanes(prev)
    check_sampler_outputs(f"sde96_trained_300 ({prec}, {lanes} lanes)", out, x0, g)
    e64 = rel_err(x0, f64)
    print(f"  x0_hat rel err vs the fp64 trajectory {e64:.3e} (fp32 reference vs fp64: "
          f"{rel_err(g['x0_unclamped'], f64):.3e})")
    assert e64 < 1e-4
    if lanes != 1:
        prev = lib().tcx_set_sample_lanes(1)
        try:
            out1, x01 = run_sde(m, g, noise, (B, 1, 64, 64))
        finally:
            lib().tcx_set_sample_lanes(prev)
        assert np.array_equal(out, out1) and np.array_equal(x0, x01)
        return
    base = S.step_table

    def perturbed_run(row, col, f):
        def tab_fn(sde, n, t_end):
            tab = base(sde, n, t_end).clone()
            tab[row, col] *= 1.0 + f
            return tab

        monkeypatch.setattr(S, "step_table", tab_fn)
        try:
            return run_sde(m, g, noise, (B, 1, 64, 64))[1]
        finally:
            monkeypatch.setattr(S, "step_table", base)

    for row, col, what in ((steps, 7, "alpha(t_end), final projection"), (steps, 4, "sigma(t_end)"),
                           (steps - 1, 3, "beta, last EM step"), (steps // 2, 3, "beta, step 150"),
                           (0, 4, "sigma(1), first step")):
        x0p = perturbed_run(row, col, 1e-5)
        print(f"  {what} x (1 + 1e-5): x0_hat rel err vs reference {rel_err(x0p, g['x0_unclamped']):.3e}, "
              f"vs unperturbed {rel_err(x0p, x0):.3e}")
    x0p = perturbed_run(steps, 7, 2e-4)
    perr = rel_err(x0p, g["x0_unclamped"])
    print(f"  alpha(t_end) x (1 + 2e-4): x0_hat rel err vs reference {perr:.3e} (must exceed the 1e-4 gate)")
    assert perr > 1e-4


def test_trained_ode50_vs_reference(golden, prec):
    """PF-ODE Heun, 50 steps, CFG 1.5 on the trained fixture (80 % unsaturated pixels)."""
    g = golden("ode96_trained_50")
    m = unet(96, golden("trained96_ema"))
    torch.manual_seed(int(g["noise_seed"]))
    x = torch.randn((int(g["B"]), 1, 64, 64))
    out, x0 = run_ode(m, g, x.cuda())
    check_sampler_outputs(f"ode96_trained_50 ({prec})", out, x0, g)


def test_sde_256px_vs_reference(golden, prec):
    """Config 5's sampler at 256x256 (base_ch 96, CFG 1.5): 2 reverse-SDE steps + the final
    projection against the reference, noise regenerated from its seed (tests/golden/make_goldens.py
    unet256).  Gate as for the short samplers: 1e-4 on the output and relative on x0_hat."""
    from toycrystals_amd.models.sde_score_model import VPSDE, host_noise, sample_reverse_sde_euler_maruyama
    g = golden("sde96_2step_h256")
    m = unet(96)
    B = int(g["B"])
    shape = (B, 1, 256, 256)
    torch.manual_seed(int(g["noise_seed"]))
    noise = host_noise(shape, int(g["steps"]) + 1)
    out, x0 = run_sde(m, g, noise.cuda(), shape)
    assert out.shape == g["out"].shape
    assert 0.0 < float(g["out"].mean()) < 1.0
    check_sampler_outputs("sde96_2step_h256", out, x0, g)


def test_in_kernel_noise_is_seeded_and_standard():
    from toycrystals_amd.models.sde_score_model import VPSDE, sample_reverse_sde_euler_maruyama
    m = unet(16)
    y_cat = torch.arange(8).cuda() % 4
    y_cont = torch.zeros(8, 4).cuda()
    kw = dict(img_shape=(8, 1, 64, 64), n_steps=3, guidance_scale=1.5, t_end=0.005)
    a = sample_reverse_sde_euler_maruyama(m, VPSDE(0.1, 30.0), y_cat, y_cont, seed=11, **kw)
    b = sample_reverse_sde_euler_maruyama(m, VPSDE(0.1, 30.0), y_cat, y_cont, seed=11, **kw)
    c = sample_reverse_sde_euler_maruyama(m, VPSDE(0.1, 30.0), y_cat, y_cont, seed=12, **kw)
    assert torch.equal(a, b) and not torch.equal(a, c)
    assert float(a.min()) >= 0.0 and float(a.max()) <= 1.0


@pytest.mark.parametrize("host_noise", [False, True], ids=["philox", "host-noise"])
def test_sampling_lanes_match_one_lane(golden, prec, host_noise):
    """tcx_set_sample_lanes(L): the batch split into L concurrent per-stream sampling chains gives
    bit-identical images (absolute Philox counters / noise slices; uneven split at L = 3, 4)."""
    from toycrystals_amd._lib import lib
    from toycrystals_amd.models.sde_score_model import VPSDE, sample_reverse_sde_euler_maruyama
    m = unet(32, golden("trained32_state"))
    B, steps = 10, 6
    y_cat = (torch.arange(B) % 5).cuda()
    y_cont = torch.rand(B, 4, generator=torch.Generator().manual_seed(3)).cuda()
    noise = torch.randn(steps + 1, B, 1, 64, 64, generator=torch.Generator().manual_seed(4)) if host_noise else None
    kw = dict(img_shape=(B, 1, 64, 64), n_steps=steps, guidance_scale=1.5, t_end=0.005, seed=21, noise=noise)
    outs = []
    try:
        for lanes in (1, 2, 3, 4):  # lane 0 runs on the caller's stream
            lib().tcx_set_sample_lanes(lanes)  # the workspace query grows with the lanes
            outs.append(sample_reverse_sde_euler_maruyama(m, VPSDE(0.1, 30.0), y_cat, y_cont, **kw))
    finally:
        lib().tcx_set_sample_lanes(0)
    assert 0.0 < float(outs[0].mean()) < 1.0
    assert all(torch.equal(outs[0], o) for o in outs[1:])


def test_ode_lanes_match_one_lane(golden):
    """The PF-ODE Heun sampler under tcx_set_sample_lanes: bit-identical to one lane."""
    from toycrystals_amd._lib import lib
    from toycrystals_amd.models.sde_score_model import VPSDE, sample_probability_flow_ode
    m = unet(32, golden("trained32_state"))
    B = 7
    y_cat = (torch.arange(B) % 5).cuda()
    y_cont = torch.rand(B, 4, generator=torch.Generator().manual_seed(5)).cuda()
    x0 = torch.randn(B, 1, 64, 64, generator=torch.Generator().manual_seed(6)).cuda()
    outs = []
    try:
        for lanes in (1, 3):
            lib().tcx_set_sample_lanes(lanes)
            outs.append(sample_probability_flow_ode(m, VPSDE(0.1, 30.0), y_cat, y_cont, (B, 1, 64, 64), n_steps=4,
                                                    guidance_scale=1.5, t_end=0.005, x_init=x0.clone()))
    finally:
        lib().tcx_set_sample_lanes(0)
    assert torch.equal(outs[0], outs[1])


def test_cpu_tensors_are_rejected():
    from toycrystals_amd._lib import TcxError
    from toycrystals_amd.models.sde_score_model import CondUNetTiny
    m = CondUNetTiny(4, 4, 16)
    with pytest.raises(TcxError):
        m(torch.zeros(1, 1, 64, 64), torch.zeros(1), torch.zeros(1, dtype=torch.int64), torch.zeros(1, 4))


def test_t_end_validation():
    from toycrystals_amd.models.sde_score_model import VPSDE, sample_reverse_sde_euler_maruyama
    m = unet(16)
    with pytest.raises(ValueError):
        sample_reverse_sde_euler_maruyama(m, VPSDE(), torch.zeros(2, dtype=torch.int64).cuda(),
                                          torch.zeros(2, 4).cuda(), (2, 1, 64, 64), t_end=1.5)


@pytest.mark.parametrize("grad", [False, True], ids=["fused", "autograd"])
@pytest.mark.parametrize("name,cond", [("condvae_b4", True), ("vae_b4", False)])
def test_vae_vs_reference(golden, name, cond, grad):
    """Both forward paths: the fused no-grad evaluator and the autograd training chain."""
    from toycrystals_amd.models.vae import CondVAE, VAE
    g = golden(name)
    torch.manual_seed(0)
    m = (CondVAE(z_dim=32, n_types=4, y_cont_dim=4, cond_drop=0.0) if cond else VAE(z_dim=32)).cuda().eval()
    x = cu(g["x"])
    with torch.set_grad_enabled(grad):
        if cond:
            mu, lv = m.encode(x, cu(g["y_cat"]), cu(g["y_cont"]))
        else:
            mu, lv = m.encode(x)
        assert mu.requires_grad == grad
        assert rel_err(mu.detach().cpu().numpy(), g["mu"]) < 2e-5
        assert rel_err(lv.detach().cpu().numpy(), g["logvar"]) < 2e-5
        z = m.reparameterise(mu, lv, cu(g["rep_eps"]))
        x_hat = m.decode(z, cu(g["y_cat"]), cu(g["y_cont"])) if cond else m.decode(z)
        assert np.abs(x_hat.detach().cpu().numpy() - g["x_hat"]).max() < 2e-5
        recon = torch.mean((x_hat.detach() - x) ** 2).item()
    assert abs(recon - float(g["recon"])) < 1e-6


@pytest.mark.parametrize("name,width,stored", [("prior_w64_b2", 64, True), ("prior_w1024_b8", 1024, False)])
def test_prior_vs_reference(golden, name, width, stored):
    from toycrystals_amd.models.diffusion_prior import DiffusionPriorFiLM, DiffusionSchedule
    g = golden(name)
    torch.manual_seed(0)
    m = DiffusionPriorFiLM(32, 4, 4, t_emb_dim=64, width=width, n_blocks=int(g["n_blocks"]), y_cat_emb_dim=64)
    if stored:
        m.load_state_dict({k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("w/")})
    m = m.cuda().eval()
    eps = m(cu(g["z_t"]), cu(g["t"]), cu(g["y_cat"]), cu(g["y_cont"]))
    assert eps.requires_grad  # autograd training chain
    e_train = rel_err(eps.detach().cpu().numpy(), g["eps"])
    with torch.no_grad():  # fused evaluator (skinny-M fp32 MFMA linears at B = 5)
        eps = m(cu(g["z_t"]), cu(g["t"]), cu(g["y_cat"]), cu(g["y_cont"])).cpu().numpy()
    e_eval = rel_err(eps, g["eps"])
    sch = DiffusionSchedule.linear(1000, 1e-4, 0.05, torch.device("cuda"))
    z0 = sch.ddim_sample(m, cu(g["y_cat"]), cu(g["y_cont"]), n_steps=int(g["ddim_steps"]),
                         z_init=cu(g["ddim_z_init"])).cpu().numpy()
    e_ddim = rel_err(z0, g["ddim_z0"])
    print(f"{name}: forward (autograd) {e_train:.2e}, forward (fused) {e_eval:.2e}, DDIM-{int(g['ddim_steps'])} "
          f"{e_ddim:.2e} relative")
    # the U-Net's gate: the frequency table is the reference's own torch.linspace (diffusion_prior.py:30-35
    # of the package), so the t = 999 sinusoid matches to rounding
    assert e_train < 2e-5 and e_eval < 2e-5 and e_ddim < 2e-5
