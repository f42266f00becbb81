"""GPU: the f16x3 GEMM of the training Linears (csrc/gemm_x3.hip: tcx_h2_rows, tcx_h2_cols,
tcx_absmax_multi, tcx_gemm_x3) through the C ABI, against a float64 torch reference of the same
product, for the three GEMMs of an nn.Linear (forward x W^T, dgrad dy W, wgrad dy^T x) at the
DiffusionPriorFiLM(w=1024) training shapes (diffusion_prior.py:39-55), ragged edges, split-K, the fused
epilogue and operands spanning 2^+-20.

Tolerance: each output is compared with its own bound sum_k |a_mk| |b_kn| (fp64).  The f16x3 split
keeps ~22 bits of every scaled operand (the dropped lo*lo term and the split residuals are < 2^-21
relative) and the accumulation is fp32, so |C - ref| <= 4e-6 * bound; the fp32 MFMA GEMM it replaces
sits at ~1e-6 of the same bound (tests/test_gpu_ops.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = 4e-6


def L():
    from toycrystals_amd._lib import lib
    return lib()


def chk(rc):
    from toycrystals_amd._lib import check
    check(rc)


def st():
    return torch.cuda.current_stream().cuda_stream


def words(*ts):
    from toycrystals_amd.functional import absmax_words
    return absmax_words(ts)


def rows(x):
    from toycrystals_amd.functional import h2_rows
    return h2_rows(x)


def cols(x):
    from toycrystals_amd.functional import h2_cols
    return h2_cols(x)


def run(M, N, K, A, inva, B, sbk, sbn, invb, amax_b, bias=None, resid=None, act=0):
    lib = L()
    C = torch.full((M, N), float("nan"), device="cuda")
    nb = int(lib.tcx_gemm_x3_workspace(M, N, K))
    ws = torch.empty(max(nb, 16), dtype=torch.uint8, device="cuda")
    p = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    chk(lib.tcx_gemm_x3(M, N, K, 1.0, p(A), p(inva), p(B), sbk, sbn, p(invb), p(amax_b), 0.0, p(C), N, p(bias),
                        p(resid), N, act, p(ws), nb, st()))
    torch.cuda.synchronize()
    return C, nb


def fwd(x, w, **kw):
    """y = x W^T: A = h2 rows of x, B = W fp32 (k contiguous)"""
    M, K = x.shape
    N = w.shape[0]
    hx, ix = rows(x)
    aw = words(w)
    return run(M, N, K, hx, ix, w, 1, K, None, aw, **kw)


def dgrad(dy, w):
    """dx = dy W: A = h2 rows of dy, B(k', n) = W[n][k'] (fp32, rows k' contiguous)"""
    M, N = dy.shape
    K = w.shape[1]
    hd, idy = rows(dy)
    aw = words(w)
    return run(M, K, N, hd, idy, w, K, 1, None, aw)


def wgrad(dy, x):
    """dW = dy^T x: A = h2 rows of dy^T, B = h2 rows of x^T"""
    M, N = dy.shape
    K = x.shape[1]
    hd, idt = cols(dy)
    hx, ixt = cols(x)
    return run(N, K, M, hd, idt, hx, 0, 0, ixt, None)


def check_close(C, ref, bound):
    err = ((C.double() - ref).abs() / (bound + 1e-300)).max().item()
    assert err <= TOL, f"max |C - ref| / bound = {err:.3e} > {TOL}"
    return err


CASES = [  # name, M (batch rows), K (in), N (out)
    ("fc1", 256, 1024, 4096),
    ("fc2", 256, 4096, 1024),
    ("cond", 256, 2048, 2048),
    ("batch32", 32, 1024, 4096),
    ("ragged", 40, 136, 48),
]


@pytest.mark.parametrize("name,M,K,N", CASES, ids=[c[0] for c in CASES])
def test_gemm_x3_linear_gemms(name, M, K, N):
    g = torch.Generator(device="cuda").manual_seed(sum(map(ord, name)))
    x = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) * 0.03
    dy = torch.randn(M, N, device="cuda", generator=g) * 1e-3
    x64, w64, d64 = x.double(), w.double(), dy.double()
    y, nb = fwd(x, w)
    e1 = check_close(y, x64 @ w64.t(), x64.abs() @ w64.abs().t())
    dx, _ = dgrad(dy, w)
    e2 = check_close(dx, d64 @ w64, d64.abs() @ w64.abs())
    dw, _ = wgrad(dy, x)
    e3 = check_close(dw, d64.t() @ x64, d64.abs().t() @ x64.abs())
    print(f"{name}: err/bound fwd {e1:.2e} dgrad {e2:.2e} wgrad {e3:.2e} (fwd split-K scratch {nb} B)")
    y2, _ = fwd(x, w)
    assert torch.equal(y, y2), "not deterministic"


def test_gemm_x3_epilogue():
    """bias, residual and SiLU fused (the fc2 forward's residual; split-K and direct epilogues)"""
    g = torch.Generator(device="cuda").manual_seed(5)
    for M, K, N in ((256, 4096, 1024), (64, 96, 256)):
        x = torch.randn(M, K, device="cuda", generator=g)
        w = torch.randn(N, K, device="cuda", generator=g) * 0.03
        bias = torch.randn(N, device="cuda", generator=g)
        resid = torch.randn(M, N, device="cuda", generator=g)
        y, _ = fwd(x, w, bias=bias, resid=resid, act=3)
        x64, w64 = x.double(), w.double()
        pre = x64 @ w64.t() + bias.double() + resid.double()
        ref = pre * torch.sigmoid(pre)
        bound = x64.abs() @ w64.abs().t() + 1e-6 * pre.abs()
        err = ((y.double() - ref).abs() / bound).max().item()
        assert err <= 2 * TOL, f"epilogue M={M}: {err:.3e}"


def test_gemm_x3_row_scales():
    """rows of x spanning 2^-20 .. 2^20 (each row carries its own scale, so every row keeps the tight
    gate), an all-zero operand (scale 1, y = bias) and the multi-tensor max word"""
    g = torch.Generator(device="cuda").manual_seed(9)
    M, K, N = 128, 512, 256
    x = torch.randn(M, K, device="cuda", generator=g) * torch.pow(2.0, torch.linspace(-20, 20, M, device="cuda"))[:, None]
    w = torch.randn(N, K, device="cuda", generator=g)
    y, _ = fwd(x, w)
    x64, w64 = x.double(), w.double()
    check_close(y, x64 @ w64.t(), x64.abs() @ w64.abs().t())
    dy = torch.randn(M, N, device="cuda", generator=g) * torch.pow(2.0, torch.linspace(-20, 20, N, device="cuda"))
    dw, _ = wgrad(dy, x)
    d64 = dy.double()
    check_close(dw, d64.t() @ x64, d64.abs().t() @ x64.abs())
    bias = torch.randn(N, device="cuda", generator=g)
    y0, _ = fwd(torch.zeros(M, K, device="cuda"), w, bias=bias)
    assert torch.equal(y0, bias.expand(M, N))
    ts = [torch.randn(1000 + 4 * i, device="cuda", generator=g) for i in range(5)]
    got = words(*ts).cpu().view(torch.float32)
    want = torch.stack([t.abs().max().cpu() for t in ts])
    assert torch.equal(got, want)


def test_h2_records_roundtrip():
    """tcx_h2_rows / tcx_h2_cols: (hi + lo) * inv reproduces x to 2^-21 of the row (column) max, and
    every inv is an exact power of two"""
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(64, 136, device="cuda", generator=g) * 7.0
    for f, ref in ((rows, x), (cols, x.t().contiguous())):
        rec, inv = f(x)
        R, K = ref.shape
        h = rec.view(torch.float16).view(R, K // 8, 2, 8).float()
        val = (h[:, :, 0, :] + h[:, :, 1, :]).reshape(R, K) * inv[:, None]
        rowmax = ref.abs().max(dim=1, keepdim=True).values
        assert ((val - ref).abs() <= rowmax * 2.0 ** -21).all()
        assert torch.equal(torch.log2(inv), torch.round(torch.log2(inv)))


def test_linear_fn_x3_vs_fp32():
    """functional.LinearFn with the weight's max word (f16x3 forward, dgrad, wgrad) against the fp32-MFMA
    LinearFn on the same inputs: outputs and all three gradients within 4e-6 of their bounds"""
    from toycrystals_amd import functional as TF
    g = torch.Generator(device="cuda").manual_seed(11)
    M, K, N = 256, 1024, 512
    x = torch.randn(M, K, device="cuda", generator=g).requires_grad_()
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.03).requires_grad_()
    b = torch.randn(N, device="cuda", generator=g).requires_grad_()
    r = torch.randn(M, N, device="cuda", generator=g)
    gy = torch.randn(M, N, device="cuda", generator=g) * 1e-3
    outs = []
    for aw in (None, words(w)):
        y = TF.LinearFn.apply(x, w, b, r, aw)
        dx, dw, db = torch.autograd.grad(y, (x, w, b), gy)
        outs.append((y, dx, dw, db))
    (y0, dx0, dw0, db0), (y1, dx1, dw1, db1) = outs
    x64, w64, g64 = x.detach().double(), w.detach().double(), gy.double()
    for a, c, bound in ((y1, y0, x64.abs() @ w64.abs().t() + 1.0), (dx1, dx0, g64.abs() @ w64.abs()),
                        (dw1, dw0, g64.abs().t() @ x64.abs())):
        assert ((a.double() - c.double()).abs() / bound).max().item() <= 2 * TOL
    assert torch.equal(db1, db0)
