"""Skinny-M linear microbenchmark: tcx_linear_ws at the prior's DDIM shapes, HIP-event timed
(profiling helper; TCX_NO_SKINNY=1 for the split-K GEMM)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "vae-diffusion-toy-crystals_amd"))
from toycrystals_amd._lib import check, lib, stream_ptr  # noqa: E402


def bench(M, N, K, act=0, iters=200):
    L = lib()
    w = torch.randn(N, K, device="cuda") / K ** 0.5
    npad, kpad = (N + 31) // 32 * 32, (K + 31) // 32 * 32
    wpk = torch.empty(npad, kpad, device="cuda")
    check(L.tcx_pack_conv_weight(w.data_ptr(), wpk.data_ptr(), N, K, 1, npad, kpad, stream_ptr()), "pack")
    b = torch.randn(N, device="cuda")
    x = torch.randn(M, K, device="cuda")
    y = torch.empty(M, N, device="cuda")
    nb = int(L.tcx_linear_workspace(M, N, K, 0))
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device="cuda")
    # rotate over SK_COPIES weight copies: 1 = L2-resident (2 MB per XCD), 8 = ~135 MB (MALL-sized),
    # 24 = ~400 MB (streams from HBM)
    nc = int(os.environ.get("SK_COPIES", "8"))
    wps = [wpk] + [wpk.clone() for _ in range(nc - 1)]

    def run(i):
        check(L.tcx_linear_ws(x.data_ptr(), K, None, 0, wps[i % nc].data_ptr(), b.data_ptr(), None, y.data_ptr(), M, N,
                              npad, kpad, act, ws.data_ptr(), nb, stream_ptr()), "linear")
    for i in range(20):
        run(i)
    torch.cuda.synchronize()
    # captured into a graph: the replay is GPU-bound (ctypes launches from Python are ~5-10 us each)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for i in range(iters):
                run(i)
    torch.cuda.synchronize()
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    g.replay()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (2 * iters)
    return {"M": M, "N": N, "K": K, "us": round(us, 2), "TBps": round(N * K * 4 / us / 1e6, 2)}


def bench_trivial(n, iters=200):
    """per-launch time of a trivial kernel (tcx_ddim_step on n floats), graph-replayed"""
    L = lib()
    z = torch.randn(max(n, 1), device="cuda")
    e = torch.randn(max(n, 1), device="cuda")

    def run():
        check(L.tcx_ddim_step(z.data_ptr(), e.data_ptr(), n, 0.5, 0.6, 0, stream_ptr()), "ddim")
    run()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                run()
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    g.replay()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return {"trivial_kernel_n": n, "us": round(e0.elapsed_time(e1) * 1e3 / (2 * iters), 2)}


if __name__ == "__main__":
    if os.environ.get("SK_TRIVIAL"):
        for n in (1, 1152, 1 << 20):
            print(json.dumps(bench_trivial(n)), flush=True)
        sys.exit(0)
    for M, N, K in [(36, 4096, 1024), (36, 1024, 4096), (36, 32, 1024)]:
        print(json.dumps({"copies": os.environ.get("SK_COPIES", "8"), **bench(M, N, K)}), flush=True)
