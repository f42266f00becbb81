#!/usr/bin/env python3
"""DDIM-50 of the w1024 x 8 prior on the 36-sample grid: the native one-call sampler
(tcx_prior_ddim_sample, 27 launches per step) timed as issued from the host vs the same call
captured once into a HIP graph and replayed; prints both and the max difference of the outputs."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vae-diffusion-toy-crystals_amd"))
import torch  # noqa: E402

from toycrystals_amd import functional as TF  # noqa: E402
from toycrystals_amd._lib import check, lib, ptr, stream_ptr  # noqa: E402
from toycrystals_amd.models.diffusion_prior import DiffusionPriorFiLM, DiffusionSchedule  # noqa: E402


def main():
    torch.manual_seed(0)
    dev = torch.device("cuda")
    n = 36
    m = DiffusionPriorFiLM(32, 4, 4, t_emb_dim=64, width=1024, n_blocks=8, y_cat_emb_dim=64).to(dev).eval()
    sched = DiffusionSchedule.linear(1000, 1e-4, 0.05, dev)
    y_cat = (torch.arange(n, device=dev) % 4).to(torch.int64)
    y_cont = torch.rand(n, 4, device=dev)
    z0 = torch.randn(n, 32, device=dev)
    with torch.no_grad():
        for _ in range(3):
            ref = sched.ddim_sample(m, y_cat, y_cont, n_steps=50, z_init=z0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        K = 20
        for _ in range(K):
            sched.ddim_sample(m, y_cat, y_cont, n_steps=50, z_init=z0)
        torch.cuda.synchronize()
        t_native = (time.perf_counter() - t0) / K

        # the same native call, captured
        T = int(sched.betas.shape[0])
        ts = torch.unique_consecutive(torch.round(torch.linspace(T - 1, 0, steps=50)).to(torch.int64)).tolist()
        nn_ = len(ts)
        abar = sched.alpha_bars.detach().float().cpu()
        a_t = [float(abar[ts[i]]) for i in range(nn_)]
        a_p = [float(abar[ts[i + 1]]) if i + 1 < nn_ else 1.0 for i in range(nn_)]
        pk = m._tcx(dev)
        L = lib()
        nb = int(L.tcx_prior_workspace(ctypes.byref(pk.net), n, nn_))
        ws = torch.empty(nb // 4 + 64, dtype=torch.float32, device=dev)
        z = torch.empty_like(z0)
        ovf = torch.zeros(1, dtype=torch.int32, device=dev)
        tsa = (ctypes.c_longlong * nn_)(*ts)
        ata = (ctypes.c_float * nn_)(*a_t)
        apa = (ctypes.c_float * nn_)(*a_p)

        def call():
            z.copy_(z0)
            check(L.tcx_prior_ddim_sample(ctypes.byref(pk.net), ptr(y_cat), ptr(y_cont), n, tsa, ata, apa, nn_, ptr(z),
                                          ptr(ovf), ptr(ws), nb, stream_ptr(dev)), "ddim")

        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                call()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            call()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            g.replay()
        torch.cuda.synchronize()
        t_graph = (time.perf_counter() - t0) / K
        diff = float((z - ref).abs().max())
    print(json.dumps({"ddim50_native_ms": round(t_native * 1e3, 3), "ddim50_graph_ms": round(t_graph * 1e3, 3),
                      "max_abs_diff": diff, "ovf": int(ovf.item())}), flush=True)


if __name__ == "__main__":
    main()
