"""GPU: the skinny-M linears (csrc/skinny.hip) and the native prior forward / DDIM (csrc/prior.hip).

Checks, all through the C ABI:
  * tcx_linear_ws at M <= 64 (split-K partials + fixed-order reduce) vs a float64 torch product on
    ragged shapes (M, N not multiples of 16, K tails, two sources, residual, every activation):
    5e-6 x max|y| (fp32 accumulation over K <= 4096);
  * tcx_prior_forward at B = 36 (skinny path, LayerNorm+FiLM fused into the reduce) and B = 100
    (tiled fallback) vs the float64 numpy oracle (oracle/vae_prior.py): 2e-5 relative;
  * tcx_prior_ddim_sample (hoisted y branch, batched t branch, FiLM split at [t_feat | y_feat],
    DDIM update fused into out_proj) vs the step-by-step loop of the reference's ddim_sample
    (diffusion_prior.py:226-250) run over the native forward: 2e-5 relative, and vs the float64
    oracle's DDIM (observed error and the fp32 oracle's own error printed).
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel_err(a, ref):
    return float(np.abs(a - ref).max()) / max(1.0, float(np.abs(ref).max()))


def _pack(w, npad, kpad):
    from toycrystals_amd._lib import check, lib, stream_ptr
    n, k = w.shape
    wpk = torch.empty((npad, kpad), device="cuda", dtype=torch.float32)
    check(lib().tcx_pack_conv_weight(w.data_ptr(), wpk.data_ptr(), n, k, 1, npad, kpad, stream_ptr()), "pack")
    return wpk


@pytest.mark.parametrize("M,N,K1,K2,act,resid", [
    (1, 1024, 1024, 0, 0, False), (5, 33, 48, 0, 3, False), (17, 100, 96, 32, 1, True), (36, 4096, 1024, 0, 3, False),
    (36, 1024, 4096, 0, 0, True), (50, 16384, 1024, 0, 0, False), (64, 64, 16, 0, 2, False),
    (36, 32, 1024, 0, 0, False), (36, 1024, 32, 0, 0, False), (36, 1024, 64, 64, 3, False)])
def test_skinny_linear_vs_float64(M, N, K1, K2, act, resid):
    from toycrystals_amd._lib import check, lib, stream_ptr
    L = lib()
    g = torch.Generator().manual_seed(M * 7 + N + K1)
    K = K1 + K2
    w = (torch.randn(N, K, generator=g) / K ** 0.5).cuda()
    b = torch.randn(N, generator=g).cuda()
    x1 = torch.randn(M, K1, generator=g).cuda()
    x2 = torch.randn(M, K2, generator=g).cuda() if K2 else None
    r = torch.randn(M, N, generator=g).cuda() if resid else None
    npad, kpad = (N + 31) // 32 * 32, (K + 31) // 32 * 32
    wpk = _pack(w, npad, kpad)
    nb = int(L.tcx_linear_workspace(M, N, K1, K2))
    assert nb > 0
    ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
    y = torch.empty(M, N, device="cuda")
    check(L.tcx_linear_ws(x1.data_ptr(), K1, x2.data_ptr() if K2 else None, K2, wpk.data_ptr(), b.data_ptr(),
                          r.data_ptr() if resid else None, y.data_ptr(), M, N, npad, kpad, act, ws.data_ptr(), nb,
                          stream_ptr()), "tcx_linear_ws")
    x = torch.cat([x1, x2], 1) if K2 else x1
    ref = x.double() @ w.double().T + b.double()
    if resid:
        ref = ref + r.double()
    ref = [ref, torch.relu(ref), torch.sigmoid(ref), torch.nn.functional.silu(ref)][act]
    err = float((y.double() - ref).abs().max()) / max(1.0, float(ref.abs().max()))
    print(f"M={M} N={N} K={K1}+{K2} act={act}: {err:.2e}")
    assert err < 5e-6


def _prior(width=1024, n_blocks=8):
    from toycrystals_amd.models.diffusion_prior import DiffusionPriorFiLM
    torch.manual_seed(0)
    return DiffusionPriorFiLM(32, 4, 4, t_emb_dim=64, width=width, n_blocks=n_blocks, y_cat_emb_dim=64)


def _inputs(B, seed):
    g = torch.Generator().manual_seed(seed)
    z = torch.randn(B, 32, generator=g)
    t = torch.randint(0, 1000, (B,), generator=g)
    y_cat = torch.arange(B) % 4
    y_cont = torch.rand(B, 4, generator=g)
    return z, t, y_cat, y_cont


@pytest.mark.parametrize("B", [36, 100])
def test_prior_forward_native_vs_oracle(B):
    from oracle.vae_prior import PriorFiLM
    m = _prior()
    o64 = PriorFiLM({k: v.numpy() for k, v in m.state_dict().items()}, dt=np.float64)
    z, t, y_cat, y_cont = _inputs(B, 11)
    ref = o64(z.numpy(), t.numpy(), y_cat.numpy(), y_cont.numpy())
    m = m.cuda().eval()
    with torch.no_grad():
        eps = m(z.cuda(), t.cuda(), y_cat.cuda(), y_cont.cuda()).cpu().numpy()
    e = rel_err(eps, ref)
    print(f"prior forward B={B} ({'skinny' if B <= 64 else 'tiled'}) vs float64 oracle: {e:.2e}")
    assert e < 2e-5


def test_prior_ddim_native_vs_stepwise_and_oracle():
    from oracle.vae_prior import PriorFiLM, Schedule
    from toycrystals_amd._lib import check, lib, stream_ptr
    from toycrystals_amd.models.diffusion_prior import DiffusionSchedule
    m = _prior()
    sd = {k: v.numpy() for k, v in m.state_dict().items()}
    B, n_steps = 36, 50
    _, _, y_cat, y_cont = _inputs(B, 5)
    z_init = torch.randn(B, 32, generator=torch.Generator().manual_seed(9))
    m = m.cuda().eval()
    sch = DiffusionSchedule.linear(1000, 1e-4, 0.05, torch.device("cuda"))
    z_native = sch.ddim_sample(m, y_cat.cuda(), y_cont.cuda(), n_steps=n_steps, z_init=z_init.cuda()).cpu().numpy()
    # the reference's loop (diffusion_prior.py:226-250) over the native forward
    ts = torch.unique_consecutive(torch.round(torch.linspace(999, 0, steps=n_steps)).to(torch.int64)).tolist()
    abar = sch.alpha_bars.float().cpu()
    z = z_init.cuda().contiguous().clone()
    with torch.no_grad():
        for i, tv in enumerate(ts):
            eps = m(z, torch.full((B,), tv, device="cuda", dtype=torch.int64), y_cat.cuda(), y_cont.cuda())
            last = i == len(ts) - 1
            check(lib().tcx_ddim_step(z.data_ptr(), eps.contiguous().data_ptr(), z.numel(), float(abar[tv]),
                                      float(abar[ts[i + 1]]) if not last else 1.0, int(last), stream_ptr()), "ddim")
    z_step = z.cpu().numpy()
    e_step = rel_err(z_native, z_step)
    s64 = Schedule(1000, 1e-4, 0.05, dt=np.float64)
    ref64 = s64.ddim_sample(PriorFiLM(sd, dt=np.float64), y_cat.numpy(), y_cont.numpy(), z_init.numpy(), n_steps)
    ref32 = Schedule(1000, 1e-4, 0.05).ddim_sample(PriorFiLM(sd), y_cat.numpy(), y_cont.numpy(), z_init.numpy(),
                                                    n_steps)
    e64, floor = rel_err(z_native, ref64), rel_err(ref32, ref64)
    print(f"DDIM-{n_steps} B={B}: native vs stepwise {e_step:.2e}; vs float64 oracle {e64:.2e} "
          f"(fp32 oracle vs float64: {floor:.2e}; stepwise vs float64 {rel_err(z_step, ref64):.2e})")
    assert e_step < 2e-5
    assert e64 < max(2e-5, 3 * floor)


def test_prior_workspace_and_errors():
    from toycrystals_amd._lib import TcxError, TcxPrior, check, lib
    L = lib()
    m = _prior(64, 2).cuda().eval()
    pk = m._tcx(torch.device("cuda"))
    assert L.tcx_prior_workspace(ctypes.byref(pk.net), 36, 50) > L.tcx_prior_workspace(ctypes.byref(pk.net), 36, 0)
    bad = TcxPrior.from_buffer_copy(pk.net)
    bad.width = 65
    out = torch.empty(4, 32, device="cuda")
    with pytest.raises(TcxError, match="widths"):
        check(L.tcx_prior_forward(ctypes.byref(bad), out.data_ptr(), out.data_ptr(), out.data_ptr(), out.data_ptr(), 4,
                                  out.data_ptr(), None, out.data_ptr(), 1 << 20, None), "tcx_prior_forward")


@pytest.mark.parametrize("B", [3, 80])
def test_prior_ddim_native_vs_stepwise_small(B):
    """B = 80 takes the tiled fallback (column windows of the packed FiLM weight, separate LayerNorm
    and DDIM kernels); B = 3 the skinny path at one row tile."""
    from toycrystals_amd._lib import check, lib, stream_ptr
    from toycrystals_amd.models.diffusion_prior import DiffusionSchedule
    m = _prior(256, 3).cuda().eval()
    _, _, y_cat, y_cont = _inputs(B, 21)
    z_init = torch.randn(B, 32, generator=torch.Generator().manual_seed(4)).cuda()
    sch = DiffusionSchedule.linear(1000, 1e-4, 0.05, torch.device("cuda"))
    z_native = sch.ddim_sample(m, y_cat.cuda(), y_cont.cuda(), n_steps=6, z_init=z_init).cpu().numpy()
    ts = torch.unique_consecutive(torch.round(torch.linspace(999, 0, steps=6)).to(torch.int64)).tolist()
    abar = sch.alpha_bars.float().cpu()
    z = z_init.clone()
    with torch.no_grad():
        for i, tv in enumerate(ts):
            eps = m(z, torch.full((B,), tv, device="cuda", dtype=torch.int64), y_cat.cuda(), y_cont.cuda())
            last = i == len(ts) - 1
            check(lib().tcx_ddim_step(z.data_ptr(), eps.contiguous().data_ptr(), z.numel(), float(abar[tv]),
                                      float(abar[ts[i + 1]]) if not last else 1.0, int(last), stream_ptr()), "ddim")
    e = rel_err(z_native, z.cpu().numpy())
    print(f"DDIM-6 B={B}: native vs stepwise {e:.2e}")
    assert e < 2e-5


def test_prior_f16x3_vs_fp32_and_overflow_fallback(monkeypatch):
    """The f16x3 trunk (fc1 / fc2 / out_proj on split-f16 MFMA) against the fp32 trunk and the float64
    oracle; an activation beyond the f16 range raises the overflow word and the call re-runs in fp32
    (bitwise the fp32 result)."""
    from oracle.vae_prior import PriorFiLM
    import toycrystals_amd.models.diffusion_prior as dp
    m = _prior()
    z, t, y_cat, y_cont = _inputs(36, 13)
    ref = PriorFiLM({k: v.numpy() for k, v in m.state_dict().items()}, dt=np.float64)(
        z.numpy(), t.numpy(), y_cat.numpy(), y_cont.numpy())
    m = m.cuda().eval()
    args = (z.cuda(), t.cuda(), y_cat.cuda(), y_cont.cuda())

    def fwd(prec):
        monkeypatch.setattr(dp, "PRIOR_PRECISION", prec)
        with torch.no_grad():
            return m(*args).cpu().numpy()
    e_h2, e_32 = fwd("f16x3"), fwd("fp32")
    d, e1, e2 = rel_err(e_h2, e_32), rel_err(e_h2, ref), rel_err(e_32, ref)
    print(f"prior B=36: f16x3 vs fp32 {d:.2e}; vs float64 oracle f16x3 {e1:.2e}, fp32 {e2:.2e}")
    assert d < 2e-5 and e1 < 2e-5 and e2 < 2e-5
    with torch.no_grad():
        m.blocks[0].fc1.weight.mul_(1e6)  # fc1 pre-activations ~1e6: a = silu(.) leaves the f16 range
    big_h2, big_32 = fwd("f16x3"), fwd("fp32")
    assert np.isfinite(big_32).all()
    assert np.array_equal(big_h2, big_32)
