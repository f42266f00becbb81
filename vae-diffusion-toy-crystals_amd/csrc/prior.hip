// Native DiffusionPriorFiLM forward and DDIM sampler (diffusion_prior.py:57-127, 203-252).
//
// The prior is a stack of nn.Linear over a few dozen latents, so its cost is streaming 412 MB of
// fp32 weights per forward and the launches between them.  The forward runs entirely here (one C
// call, no Python between launches) on the skinny kernels of skinny.hip:
//   in_proj   partials + [reduce + bias -> h, LayerNorm_0 + FiLM_0 -> hn]
//   block j   fc1: one launch, epilogue bias + SiLU -> a
//             fc2: partials + [reduce + bias + h -> h', LayerNorm_{j+1} (+FiLM) -> hn]
//   out_proj  one launch, epilogue bias -> eps (DDIM: + the z update)
// With an overflow word (ovf != NULL) and h2 packs on fc1 / fc2 / out_proj, those three run as
// f16x3 products (hi*hi + hi*lo + lo*hi, fp32 accumulate, ~2^-21 relative per product) with hn and a
// kept in h2 storage; a value leaving the f16 range raises *ovf and the caller re-runs in fp32.
// The DDIM hoists what does not change across its steps (the reference recomputes it per step):
//   * the y branch (embedding, y_cont_mlp, y_fuse) and the y half of every FiLM projection,
//     G_y = y_feat Wc[:, W:2W]^T + b_c, once per call;
//   * the t branch for ALL n_steps timesteps as one n-row batch and the t half of every FiLM
//     projection, G_t = t_feat Wc[:, :W]^T, in one GEMM that streams Wc once (not once per step).
// FiLM then takes gamma|beta = G_y[row] + G_t[step] (the same K = 2W dot product split at the
// [t_feat | y_feat] boundary, summed in fp32).  Batches above 64 rows fall back to the tiled GEMMs
// (tcx_linear_ws) with separate LayerNorm / DDIM kernels.
#include "skinny.hpp"

#include <algorithm>

namespace tcx {
namespace {

struct Arena {
    char* base;
    size_t used = 0;
    bool dry;
    void* take(size_t bytes) {
        const size_t off = align_up(used, 256);
        used = off + bytes;
        return dry ? nullptr : base + off;
    }
    float* f(size_t n) { return static_cast<float*>(take(n * sizeof(float))); }
};

struct I64Chunk {
    long long v[64];
};

__global__ void k_fill_i64(int64_t* __restrict__ dst, int n, I64Chunk c) {
    const int i = threadIdx.x;
    if (i < n) dst[i] = c.v[i];
}

size_t lin_need(int M, int N, int K1, int K2) {
    if (M <= 0) return 0;
    if (skinny_ok(M, N, K1, K2)) return skinny_part_floats(skinny_plan(K1, K2), M, N) * sizeof(float);
    return tcx_linear_workspace(M, N, K1, K2);
}

bool sk_fits(const tcx_linear_w& L, int M, int K) {
    return skinny_ok(M, L.n, K, 0) && L.npad >= 16 * cdiv(L.n, 16);
}

struct Ctx {
    hipStream_t st;
    float* part;
    size_t part_bytes;
};

// y = act(x1 W[:, koff : koff+K1]^T (+ x2 W[:, koff+K1 : koff+K1+K2]^T) (+ b) (+ resid))
int lin(const Ctx& c, const tcx_linear_w& L, int koff, const float* x1, int K1, const float* x2, int K2, bool bias,
        const float* resid, float* y, int M, int act) {
    return tcx_linear_ws(x1, K1, x2, K2, L.w + koff, bias ? L.b : nullptr, resid, y, M, L.n, L.npad, L.kpad, act,
                         c.part, c.part_bytes, c.st);
}

// h_out = x W^T + b (+ resid); hn = LayerNorm(h_out) (+ FiLM from gy (+ gt)), or hn in h2 storage
// (hn_h2, skinny path only) for an f16x3 consumer
int lin_ln(const Ctx& c, const tcx_linear_w& L, const float* x, int K, const float* resid, float* h_out, int M,
           const float* lw, const float* lb, const float* gy, int ld_gy, const float* gt, float eps, float* hn,
           void* hn_h2 = nullptr, unsigned* ovf = nullptr) {
    if (sk_fits(L, M, K) && skinny_ln_ok(L.n)) {
        const SkPlan p = skinny_plan(K, 0);
        TCX_TRY(skinny_partials(x, K, K, nullptr, 0, 0, L.w, L.kpad, M, L.n, p, c.part, c.st));
        SkEpi e;
        e.b = L.b; e.resid = resid; e.y = h_out;
        SkLn ln;
        ln.lw = lw; ln.lb = lb; ln.gy = gy; ln.ld_gy = ld_gy; ln.gt = gt; ln.eps = eps;
        if (hn_h2) ln.yn_h2 = hn_h2, ln.ovf = ovf;
        else ln.yn = hn;
        return skinny_reduce_ln(c.part, p.s1, M, L.n, e, ln, c.st);
    }
    TCX_REQUIRE(!hn_h2, "prior: the h2 LayerNorm output needs the skinny path");
    TCX_TRY(lin(c, L, 0, x, K, nullptr, 0, true, resid, h_out, M, 0));
    return launch_layernorm_film(h_out, hn, M, L.n, lw, lb, gy, ld_gy, gt, eps, c.st);
}

// eps = x W^T + b, then the DDIM eta=0 update of z with it (k_ddim_step's arithmetic)
int lin_ddim(const Ctx& c, const tcx_linear_w& L, const float* x, int K, float* z, float* eps_tmp, int M, float abar_t,
             float abar_prev, int last) {
    if (sk_fits(L, M, K)) {
        SkEpi e;
        e.b = L.b; e.z = z; e.abar_t = abar_t; e.abar_prev = abar_prev; e.last = last;
        return skinny_linear(x, K, K, nullptr, 0, 0, L.w, L.kpad, M, L.n, c.part, e, c.st);
    }
    TCX_TRY(lin(c, L, 0, x, K, nullptr, 0, true, nullptr, eps_tmp, M, 0));
    return tcx_ddim_step(z, eps_tmp, (size_t)M * L.n, abar_t, abar_prev, last, c.st);
}

int check_net(const tcx_prior* P) {
    TCX_REQUIRE(P && P->fc1 && P->fc2 && P->norm_w && P->norm_b && P->temb_freqs && P->y_cat_emb && P->out_norm_w &&
                    P->out_norm_b,
                "tcx_prior: null pointer");
    const int W = P->width, E = P->y_cat_emb_dim;
    TCX_REQUIRE(W > 0 && E > 0 && P->n_blocks >= 1 && P->z_dim > 0 && P->t_emb_dim > 0 && P->y_cont_dim > 0,
                "tcx_prior: bad sizes");
    auto ok = [](const tcx_linear_w& L, int n, int k) {
        return L.w && L.b && L.n == n && L.k == k && L.npad >= n && L.kpad >= k && L.kpad % 4 == 0;
    };
    TCX_REQUIRE(ok(P->t_mlp0, W, P->t_emb_dim) && ok(P->t_mlp2, W, W) && ok(P->y_cont0, E, P->y_cont_dim) &&
                    ok(P->y_cont2, E, E) && ok(P->y_fuse0, W, 2 * E) && ok(P->y_fuse2, W, W) &&
                    ok(P->in_proj, W, P->z_dim) && ok(P->cond_all, 2 * W * P->n_blocks, 2 * W) &&
                    ok(P->out_proj, P->z_dim, W),
                "tcx_prior: linear shapes do not match the widths");
    for (int j = 0; j < P->n_blocks; ++j) {
        TCX_REQUIRE(ok(P->fc1[j], P->fc1[0].n, W) && ok(P->fc2[j], W, P->fc1[0].n) && P->norm_w[j] && P->norm_b[j],
                    "tcx_prior: block %d shapes", j);
    }
    return TCX_OK;
}

// buffers of one call; with A.dry only the sizes are accumulated
struct Bufs {
    int64_t* ts;
    float *te, *t1, *tf, *yc1, *yc, *ycat, *yf1, *yf, *gy, *gt, *h0, *h1, *hn, *a, *eps, *part;
    void *hn_h2, *a_h2;  // f16x3 trunk: the fc1 / fc2 / out_proj operands in h2 storage
    size_t part_bytes;
};

Bufs layout(const tcx_prior& P, int B, int n, Arena& A) {
    const int W = P.width, E = P.y_cat_emb_dim, G = 2 * W * P.n_blocks, F = P.fc1[0].n, T = P.t_emb_dim;
    const int Mt = n > 0 ? n : B;  // rows of the t branch
    Bufs b{};
    b.ts = n > 0 ? static_cast<int64_t*>(A.take((size_t)n * sizeof(int64_t))) : nullptr;
    b.te = A.f((size_t)Mt * T);
    b.t1 = A.f((size_t)Mt * W);
    b.tf = A.f((size_t)Mt * W);
    b.yc1 = A.f((size_t)B * E);
    b.yc = A.f((size_t)B * E);
    b.ycat = A.f((size_t)B * E);
    b.yf1 = A.f((size_t)B * W);
    b.yf = A.f((size_t)B * W);
    b.gy = A.f((size_t)B * G);
    b.gt = n > 0 ? A.f((size_t)n * G) : nullptr;
    b.h0 = A.f((size_t)B * W);
    b.h1 = A.f((size_t)B * W);
    b.hn = A.f((size_t)B * W);
    b.a = A.f((size_t)B * F);
    b.eps = A.f((size_t)B * P.z_dim);
    b.hn_h2 = A.take((size_t)B * W * 4);
    b.a_h2 = A.take((size_t)B * F * 4);
    size_t need = 0;
    auto upd = [&](size_t v) { need = std::max(need, v); };
    upd(lin_need(Mt, W, T, 0));
    upd(lin_need(Mt, W, W, 0));
    upd(lin_need(B, E, P.y_cont_dim, 0));
    upd(lin_need(B, E, E, 0));
    upd(lin_need(B, W, E, E));
    upd(lin_need(B, W, W, 0));
    if (n > 0) {
        upd(lin_need(B, G, W, 0));
        upd(lin_need(n, G, W, 0));
    } else {
        upd(lin_need(B, G, W, W));
    }
    upd(lin_need(B, W, P.z_dim, 0));
    upd(lin_need(B, F, W, 0));
    upd(lin_need(B, W, F, 0));
    upd(lin_need(B, P.z_dim, W, 0));
    if (skinny_h2_ok(B, W, F)) upd(skinny_h2_part_floats(B, W, F) * sizeof(float));
    if (skinny_h2_ok(B, F, W)) upd(skinny_h2_part_floats(B, F, W) * sizeof(float));
    if (skinny_h2_ok(B, P.z_dim, W)) upd(skinny_h2_part_floats(B, P.z_dim, W) * sizeof(float));
    b.part_bytes = std::max<size_t>(need, 256);
    b.part = static_cast<float*>(A.take(b.part_bytes));
    return b;
}

// the y branch (diffusion_prior.py:113-118): y_feat = y_fuse([y_cat_emb(y_cat) | y_cont_mlp(y_cont)])
int y_branch(const Ctx& c, const tcx_prior& P, const int64_t* y_cat, const float* y_cont, int B, const Bufs& b) {
    const int E = P.y_cat_emb_dim, W = P.width;
    TCX_TRY(lin(c, P.y_cont0, 0, y_cont, P.y_cont_dim, nullptr, 0, true, nullptr, b.yc1, B, 3));
    TCX_TRY(lin(c, P.y_cont2, 0, b.yc1, E, nullptr, 0, true, nullptr, b.yc, B, 0));
    TCX_TRY(tcx_embedding_fwd(y_cat, P.y_cat_emb, B, E, b.ycat, c.st));
    TCX_TRY(lin(c, P.y_fuse0, 0, b.ycat, E, b.yc, E, true, nullptr, b.yf1, B, 3));
    return lin(c, P.y_fuse2, 0, b.yf1, W, nullptr, 0, true, nullptr, b.yf, B, 0);
}

// the t branch (:108-112): t_feat = t_mlp(timestep_embedding(t)) for M rows of t
int t_branch(const Ctx& c, const tcx_prior& P, const int64_t* t, int M, const Bufs& b) {
    TCX_TRY(tcx_prior_temb(t, P.temb_freqs, M, P.t_emb_dim, b.te, c.st));
    TCX_TRY(lin(c, P.t_mlp0, 0, b.te, P.t_emb_dim, nullptr, 0, true, nullptr, b.t1, M, 3));
    return lin(c, P.t_mlp2, 0, b.t1, P.width, nullptr, 0, true, nullptr, b.tf, M, 0);
}

// the f16x3 trunk applies: every fc1 / fc2 / out_proj carries an h2 pack, B <= 64, widths % 32
bool use_h2(const tcx_prior& P, int B, const unsigned* ovf) {
    if (!ovf) return false;
    const int W = P.width, F = P.fc1[0].n;
    if (!(skinny_h2_ok(B, F, W) && skinny_h2_ok(B, W, F) && skinny_h2_ok(B, P.z_dim, W) && skinny_ln_ok(W) &&
          F % 8 == 0 && sk_fits(P.in_proj, B, P.z_dim) && P.out_proj.wh && P.out_proj.winv))
        return false;
    for (int j = 0; j < P.n_blocks; ++j)
        if (!(P.fc1[j].wh && P.fc1[j].winv && P.fc2[j].wh && P.fc2[j].winv)) return false;
    return true;
}

// h = in_proj(z); blocks; hn = out_norm(h) (:119-126).  FiLM rows: gy (+ gt) at block offsets 2W j.
// h2: fc1 / fc2 on f16x3 MFMA with hn and a in h2 storage (the residual stream h stays fp32).
int trunk(const Ctx& c, const tcx_prior& P, const float* z, int B, const float* gy, int ld_gy, const float* gt,
          const Bufs& b, unsigned* ovf_h2) {
    const int W = P.width, F = P.fc1[0].n;
    const bool h2 = ovf_h2 != nullptr;
    float* h = b.h0;
    float* h_next = b.h1;
    TCX_TRY(lin_ln(c, P.in_proj, z, P.z_dim, nullptr, h, B, P.norm_w[0], P.norm_b[0], gy, ld_gy, gt, P.ln_eps, b.hn,
                   h2 ? b.hn_h2 : nullptr, ovf_h2));
    for (int j = 0; j < P.n_blocks; ++j) {
        const bool last = j + 1 == P.n_blocks;
        const float* lw = last ? P.out_norm_w : P.norm_w[j + 1];
        const float* lb = last ? P.out_norm_b : P.norm_b[j + 1];
        const float* g1 = last ? nullptr : gy + 2 * W * (j + 1);
        const float* g2 = last || !gt ? nullptr : gt + 2 * W * (j + 1);
        if (h2) {
            SkEpi e1;
            e1.b = P.fc1[j].b; e1.act = 3; e1.y_h2 = b.a_h2; e1.ovf = ovf_h2;
            TCX_TRY(skinny_h2_linear(b.hn_h2, W, P.fc1[j].wh, P.fc1[j].winv, B, F, b.part, e1, c.st));
            TCX_TRY(skinny_h2_partials(b.a_h2, F, P.fc2[j].wh, P.fc2[j].winv, B, W, b.part, c.st));
            SkEpi e2;
            e2.b = P.fc2[j].b; e2.resid = h; e2.y = h_next;
            SkLn ln;
            ln.lw = lw; ln.lb = lb; ln.gy = g1; ln.ld_gy = ld_gy; ln.gt = g2; ln.eps = P.ln_eps;
            ln.yn_h2 = b.hn_h2; ln.ovf = ovf_h2;
            TCX_TRY(skinny_reduce_ln(b.part, skinny_h2_chunks(W, F), B, W, e2, ln, c.st));
        } else {
            TCX_TRY(lin(c, P.fc1[j], 0, b.hn, W, nullptr, 0, true, nullptr, b.a, B, 3));
            TCX_TRY(lin_ln(c, P.fc2[j], b.a, F, h, h_next, B, lw, lb, g1, ld_gy, g2, P.ln_eps, b.hn));
        }
        std::swap(h, h_next);
    }
    return TCX_OK;
}

}  // namespace
}  // namespace tcx

using namespace tcx;

extern "C" size_t tcx_prior_workspace(const tcx_prior* net, int B, int n_steps) {
    if (!net || !net->fc1 || B <= 0 || n_steps < 0) return 0;
    Arena A{nullptr, 0, true};
    layout(*net, B, n_steps, A);
    return A.used + 256;
}

extern "C" int tcx_prior_forward(const tcx_prior* net, const float* z_t, const int64_t* t, const int64_t* y_cat,
                                 const float* y_cont, int B, float* eps_out, unsigned* ovf, void* ws,
                                 size_t ws_bytes, void* stream) {
    TCX_TRY(check_net(net));
    TCX_REQUIRE(z_t && t && y_cat && y_cont && eps_out && B >= 0, "tcx_prior_forward: bad args");
    if (B == 0) return TCX_OK;
    const size_t need = tcx_prior_workspace(net, B, 0);
    TCX_REQUIRE(ws && ws_bytes >= need, "tcx_prior_forward: workspace %zu < %zu bytes", ws_bytes, need);
    const tcx_prior& P = *net;
    Arena A{static_cast<char*>(ws), 0, false};
    const Bufs b = layout(P, B, 0, A);
    const Ctx c{(hipStream_t)stream, b.part, b.part_bytes};
    const int W = P.width, G = 2 * W * P.n_blocks;
    TCX_TRY(t_branch(c, P, t, B, b));
    TCX_TRY(y_branch(c, P, y_cat, y_cont, B, b));
    TCX_TRY(lin(c, P.cond_all, 0, b.tf, W, b.yf, W, true, nullptr, b.gy, B, 0));  // [gamma|beta] of all blocks
    unsigned* h2 = use_h2(P, B, ovf) ? ovf : nullptr;
    TCX_TRY(trunk(c, P, z_t, B, b.gy, G, nullptr, b, h2));
    if (h2) {
        SkEpi e;
        e.b = P.out_proj.b; e.y = eps_out;
        return skinny_h2_linear(b.hn_h2, W, P.out_proj.wh, P.out_proj.winv, B, P.z_dim, b.part, e, c.st);
    }
    return lin(c, P.out_proj, 0, b.hn, W, nullptr, 0, true, nullptr, eps_out, B, 0);
}

extern "C" int tcx_prior_ddim_sample(const tcx_prior* net, const int64_t* y_cat, const float* y_cont, int B,
                                     const int64_t* ts, const float* abar_t, const float* abar_prev, int n_steps,
                                     float* z, unsigned* ovf, void* ws, size_t ws_bytes, void* stream) {
    TCX_TRY(check_net(net));
    TCX_REQUIRE(y_cat && y_cont && z && ts && abar_t && abar_prev && B >= 0 && n_steps >= 1,
                "tcx_prior_ddim_sample: bad args");
    if (B == 0) return TCX_OK;
    const size_t need = tcx_prior_workspace(net, B, n_steps);
    TCX_REQUIRE(ws && ws_bytes >= need, "tcx_prior_ddim_sample: workspace %zu < %zu bytes", ws_bytes, need);
    const tcx_prior& P = *net;
    hipStream_t st = (hipStream_t)stream;
    Arena A{static_cast<char*>(ws), 0, false};
    const Bufs b = layout(P, B, n_steps, A);
    const Ctx c{st, b.part, b.part_bytes};
    const int W = P.width, G = 2 * W * P.n_blocks;
    for (int i0 = 0; i0 < n_steps; i0 += 64) {
        I64Chunk ch{};
        const int cnt = std::min(64, n_steps - i0);
        for (int i = 0; i < cnt; ++i) ch.v[i] = ts[i0 + i];
        hipLaunchKernelGGL(k_fill_i64, dim3(1), dim3(64), 0, st, b.ts + i0, cnt, ch);
        TCX_TRY(check_launch("tcx_prior_ddim_sample(ts)"));
    }
    // loop invariants: G_y = y_feat Wc[:, W:]^T + b_c (B rows), G_t = t_feat Wc[:, :W]^T (n_steps rows)
    TCX_TRY(y_branch(c, P, y_cat, y_cont, B, b));
    TCX_TRY(lin(c, P.cond_all, W, b.yf, W, nullptr, 0, true, nullptr, b.gy, B, 0));
    TCX_TRY(t_branch(c, P, b.ts, n_steps, b));
    TCX_TRY(lin(c, P.cond_all, 0, b.tf, W, nullptr, 0, false, nullptr, b.gt, n_steps, 0));
    unsigned* h2 = use_h2(P, B, ovf) ? ovf : nullptr;
    for (int i = 0; i < n_steps; ++i) {
        TCX_TRY(trunk(c, P, z, B, b.gy, G, b.gt + (size_t)i * G, b, h2));
        const int last = i == n_steps - 1;
        const float a_prev = last ? 1.0f : abar_prev[i];
        if (h2) {
            SkEpi e;
            e.b = P.out_proj.b; e.z = z; e.abar_t = abar_t[i]; e.abar_prev = a_prev; e.last = last;
            TCX_TRY(skinny_h2_linear(b.hn_h2, W, P.out_proj.wh, P.out_proj.winv, B, P.z_dim, b.part, e, c.st));
        } else {
            TCX_TRY(lin_ddim(c, P.out_proj, b.hn, W, z, b.eps, B, abar_t[i], a_prev, last));
        }
    }
    return TCX_OK;
}
