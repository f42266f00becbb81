#!/usr/bin/env python3
"""Headline benchmark: denoised images/sec of the 300-step reverse-SDE sampler with CFG 1.5
(BASELINE.json `metric`, config 2: CondUNetTiny(base_ch=96), batch 128 per GPU, 64x64, t_end
0.005, VPSDE(0.1, 30)) on the MI355X path of this repo.

One "step" = one complete sampling pass over one batch: 300 fused CFG-doubled U-Net
evaluations (Bt = 256) + the final x0 projection, producing 128 denoised images (reference:
sample_reverse_sde_euler_maruyama, /root/reference/src/toycrystals/models/sde_score_model.py:507-569).
Inputs are synthetic (y_cat = i % 4, theta = linspace(0, pi/3, B), the save_sde_samples pattern
:317-321), weights random-init from torch.manual_seed(0), noise from in-kernel Philox; everything
is resident in HBM before the timed region.

Multi-GPU: one process per GPU.  `--gpus N` without WORLD_SIZE starts the N ranks itself under
torch.distributed.run (a child process, before any GPU call); under a launcher WORLD_SIZE is the
world.  Rank r samples images [r*B, (r+1)*B) of ONE global batch of N*B (its conditioning slice and
Philox element offset), so the N-GPU images are the 1-GPU images of batch N*B bit for bit (weak
scaling, no data-path collective); the only collectives are the timing barriers and the
max-over-ranks reduction of the elapsed time (and the image gather of --save-images, after timing).

Also reports, on one JSON line:
  roofline     — the split-path conv kernels (k_conv3lg / k_conv3g / k_conv4s2g / k_lin1x1), timed with
                 HIP events around every conv launch on its own stream in a SEPARATE one-lane pass of the
                 same K sampling passes after the timed region (`one_lane`; with 4 lanes' kernels co-running
                 a per-launch event no longer times one kernel): achieved algorithmic (fp32-equivalent)
                 TFLOP/s vs the peak of the MFMA it runs on — f16x3 split path (default): the 2.5 PFLOP/s
                 dense f16 MFMA peak / 3 MFMA products per fp32 multiply-add = 833.3; fp32 path
                 (--precision fp32): the 157.3 TFLOP/s fp32 MFMA peak (MI355X_MICROARCH.md).
  fp32_path    — the same sampler with the fp32-MFMA convs (one lane), value + roofline, beside the f16x3 line.
  cpu_baseline — the reference's CPU arithmetic (oracle/score_model_torch.py: torch CPU ops) on the same
                 inputs at B=128, timed at 2 and 4 sampler steps on this host's cores (rank 0, N=1 only), the
                 per-forward cost fitted and extrapolated to the 602-forward run.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "vae-diffusion-toy-crystals_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

GFLOP_PER_IMG_FWD = 7.142544384  # CondUNetTiny(96) forward at 64x64 (reference's 17-ch first conv)
FWD_PER_IMG = 602                # 300 steps x 2 CFG evaluations + 2 for the final projection
FP32_PEAK_TFLOPS = 157.3         # MI355X fp32 MFMA (= vector) peak, MI355X_MICROARCH.md
F16_PEAK_TFLOPS = 2500.0         # MI355X dense f16/bf16 MFMA peak (no sparsity), MI355X_MICROARCH.md
SPLIT_PRODUCTS = 3               # f16x3: hi*hi + hi*lo + lo*hi MFMAs per fp32 multiply-add
# HBM bytes per conv launch (the launches the roofline times), measured by rocprofv3 PMC passes on
# this sampler in the roofline's own configuration (one lane: Bt = 256 rows per launch, as the timed
# one-lane pass; tools/gpu/r06finb.sh -> tools/pmc_traffic.py, profiles/r06_fin_pmc_traffic.txt):
# FETCH_SIZE x 2 (gfx950 reports half of 16-B/lane reads) + WRITE_SIZE, averaged over the conv
# launches of two sampler steps.  A counter pass cannot run inside this process, so the measured
# value is carried here with its source; it applies to the f16x3 path it was taken on.
# keyed by (conv precision, image size): the 64x64 headline (f16x3) and config 5 (256x256 bf16)
TRAFFIC_BYTES_PER_CONV_LAUNCH = {("f16x3", 64): 499.2e6, ("bf16", 256): 997.5e6}
TRAFFIC_SOURCE = {
    ("f16x3", 64): ("rocprofv3 --pmc FETCH_SIZE (x2) + WRITE_SIZE in separate passes over bench.py --lanes 1 "
                    "(Bt = 256 per launch, the one-lane pass the roofline times), averaged over the 135 split-path "
                    "conv launches (k_conv3m 16/32/64 h2-source and GN+SiLU-prologue forms, k_conv4s2g, k_lin1x1) "
                    "of two sampler steps, profiles/r06_fin_pmc_traffic.txt"),
    ("bf16", 256): ("rocprofv3 --pmc FETCH_SIZE (x2) + WRITE_SIZE in separate passes over bench.py --img-size 256 "
                    "--batch 64 --precision bf16 --lanes 1 (64 images per launch: the evaluation runs in two passes "
                    "under the 2 GiB cap), averaged over the 270 conv launches (k_conv3lb, k_conv4s2g, k_lin1x1) of "
                    "two sampler steps, profiles/r06_v_cfg5_pmc_traffic.txt"),
}


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:  # pragma: no cover
        pass
    return "unknown"


def cpu_baseline(state_dict, B: int, steps_a: int, steps_b: int, cfg: float, t_end: float) -> dict:
    """the reference's CPU arithmetic (oracle/score_model_torch.py: torch CPU ops,
    the ATen kernels the reference's modules call) on the same synthetic inputs, B images, timed
    at `steps_a` and `steps_b` reverse-SDE steps (+ the final projection); the per-forward cost is
    fitted from the difference and extrapolated to the 602 forwards of the 300-step run."""
    from oracle.score_model_torch import TorchScoreUNet, sample_reverse_sde
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    o = TorchScoreUNet({k: v.detach().cpu() for k, v in state_dict.items()})
    y_cat = torch.arange(B) % 4
    y_cont = torch.zeros(B, 4)
    y_cont[:, 1] = torch.linspace(0, math.pi / 3, B)

    def run(n):
        gen = torch.Generator().manual_seed(1234)
        t0 = time.perf_counter()
        out = sample_reverse_sde(o, 0.1, 30.0, y_cat, y_cont, (B, 1, 64, 64), n, cfg, t_end, generator=gen)
        assert bool(torch.isfinite(out).all())
        return time.perf_counter() - t0

    o(torch.zeros(2, 1, 64, 64), torch.full((2,), 0.5), y_cat[:2], y_cont[:2])  # warm the CPU kernels (untimed)
    ta, tb = run(steps_a), run(steps_b)
    torch.set_num_threads(prev)
    fa, fb = 2 * steps_a + 2, 2 * steps_b + 2  # U-Net calls of batch B (CFG: 2 per step, 2 for the projection)
    per_fwd = (tb - ta) / (fb - fa)
    fixed = max(0.0, ta - per_fwd * fa)
    sec_per_pass = fixed + per_fwd * FWD_PER_IMG  # the 300-step run = 602 U-Net calls of batch B
    return {"value": round(B / sec_per_pass, 5), "unit": "images/s", "cores": threads, "kind": "port",
            "cpu": _cpu_model(),
            "sample": f"torch-CPU restatement of the reference arithmetic (oracle/score_model_torch.py), "
                      f"B={B}, reverse SDE {steps_a} and {steps_b} steps + projection with CFG {cfg} "
                      f"({fa} and {fb} U-Net calls of B={B}) in {ta:.1f}s / {tb:.1f}s; fit {per_fwd:.2f}s per call, "
                      f"extrapolated to the {FWD_PER_IMG} calls of the 300-step run; torch threads {threads}"}


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` started without a launcher: run the N ranks under torch.distributed.run as
    a CHILD process (never exec: nothing here has touched the GPU yet, and the ranks initialise it
    themselves) with this script's own arguments; rank 0's JSON line goes to the inherited stdout."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this host driver
    env.setdefault("OMP_NUM_THREADS", "1")  # torchrun would otherwise warn and set it itself
    return subprocess.run(cmd, env=env).returncode


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node (one rank each).  Without WORLD_SIZE in the environment, N > 1 "
                         "launches `torch.distributed.run --nproc-per-node N` on this script as a child "
                         "process (before any GPU call) and relays its JSON line and exit code; under "
                         "torchrun it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=3, help="timed sampling passes (each = 300 sampler steps)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=128, help="images per GPU")
    ap.add_argument("--n-steps", type=int, default=300)
    ap.add_argument("--cfg", type=float, default=1.5)
    ap.add_argument("--t-end", type=float, default=0.005)
    ap.add_argument("--base-ch", type=int, default=96)
    ap.add_argument("--img-size", type=int, default=64,
                    help="64 (the metric's config 2); 256 with --batch 64 = config 5's per-GPU share (512 over 8)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=128)
    ap.add_argument("--lanes", "--lanes-alt", dest="lanes", type=int, default=4,
                    help="concurrent sampling lanes of the timed region (tcx_set_sample_lanes, 1-4; images are "
                         "bit-identical for every value); the roofline pass after it always runs one lane")
    ap.add_argument("--precision", choices=["f16x3", "fp32", "bf16"], default="f16x3",
                    help="conv arithmetic: f16x3 split MFMA (fp32-grade, default) or fp32 MFMA")
    ap.add_argument("--fp32-passes", type=int, default=1,
                    help="with the f16x3 headline: timed one-lane passes of the fp32-MFMA path reported beside it "
                         "(`fp32_path`; 0 skips)")
    ap.add_argument("--cpu-steps-a", type=int, default=2)
    ap.add_argument("--cpu-steps-b", type=int, default=4)
    ap.add_argument("--save-images", default="",
                    help="write the last timed pass's denoised images of ALL ranks (gathered in rank order) to "
                         "this .npy file from rank 0 (tests: an N-rank run equals the 1-rank run of N x batch)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        return _spawn_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world} (launch one rank per GPU)")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    from toycrystals_amd.dist import all_reduce_, dist_backend, local_device
    device = local_device(local_rank)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(device)
        backend = dist_backend()  # nccl (RCCL); TCX_DIST_BACKEND=gloo only to rehearse ranks sharing a GPU
        dist.init_process_group(backend, **({"device_id": device} if backend == "nccl" else {}))

    from toycrystals_amd._lib import lib, set_conv_precision
    set_conv_precision(args.precision)
    from toycrystals_amd.models.sde_score_model import CondUNetTiny, VPSDE, sample_reverse_sde_euler_maruyama

    torch.manual_seed(0)
    model = CondUNetTiny(n_types=4, y_cont_dim=4, base_ch=args.base_ch).to(device).eval()
    sde = VPSDE(beta_min=0.1, beta_max=30.0)
    B = args.batch
    # rank r holds images [r*B, (r+1)*B) of ONE global batch of world*B (its conditioning slice and,
    # in run(), its Philox element offset), so the gathered images equal a 1-GPU run of world*B
    G = world * B
    y_cat = (torch.arange(G) % 4)[rank * B:(rank + 1) * B].to(device)
    y_cont = torch.zeros(G, 4)
    y_cont[:, 1] = torch.linspace(0.0, math.pi / 3.0, G)
    y_cont = y_cont[rank * B:(rank + 1) * B].to(device)
    S = args.img_size
    shape = (B, 1, S, S)

    def run(i: int) -> torch.Tensor:
        # rank r samples images [r*B, (r+1)*B) of ONE global batch: one seed per pass, the shard's
        # Philox element offset (dist.sample_sharded semantics), so N GPUs = the 1-GPU images of N*B
        return sample_reverse_sde_euler_maruyama(model, sde, y_cat, y_cont, shape, n_steps=args.n_steps,
                                                 guidance_scale=args.cfg, t_end=args.t_end,
                                                 seed=1_000_003 + i, elem_offset=rank * B * S * S)

    _last_out = [None]

    def timed(fn) -> float:
        """K passes bracketed by a barrier + synchronize on both sides; max over ranks."""
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for i in range(args.steps):
            _last_out[0] = fn(i)
        torch.cuda.synchronize(device)
        el = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
            t = torch.tensor([el], device=device, dtype=torch.float64)
            all_reduce_(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    L = lib()
    # The timed region runs the sampler with args.lanes concurrent sampling lanes (tcx_set_sample_lanes:
    # the batch split into per-stream chains, images bit-identical to one lane) so one lane's
    # HBM-bound passes overlap another's MFMA-bound convs.
    prev_lanes = L.tcx_set_sample_lanes(max(1, args.lanes))
    for i in range(args.warmup):
        run(-1 - i)
    torch.cuda.synchronize(device)
    elapsed = timed(lambda i: run(i))
    timed_out = _last_out[0]
    L.tcx_set_sample_lanes(prev_lanes)
    # the precision the evaluator actually ran (bf16 falls back to f16x3 where the split attention does
    # not apply, a split run to fp32 after a range overflow): a line labelled with another is invalid
    from toycrystals_amd._lib import used_conv_precision
    if used_conv_precision() != args.precision:
        raise SystemExit(f"bench: requested {args.precision} but the sampler ran in {used_conv_precision()}")

    # Roofline pass: the same K passes on ONE stream with the conv launches bracketed by HIP events
    # (with kernels of several streams co-running, a per-launch event duration no longer times a
    # kernel alone).  Not part of `value`.
    L.tcx_set_sample_lanes(1)
    run(-100)
    torch.cuda.synchronize(device)
    L.tcx_prof_enable(1)
    el1 = timed(lambda i: run(100 + i))
    ms, n, fl = ctypes.c_double(), ctypes.c_longlong(), ctypes.c_double()
    L.tcx_prof_read(ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl))
    L.tcx_prof_enable(0)
    L.tcx_set_sample_lanes(prev_lanes)
    out = _last_out[0]
    assert out is not None and bool(torch.isfinite(out).all()) and float(out.min()) >= 0.0 and float(out.max()) <= 1.0

    # The fp32-MFMA path beside the f16x3 headline (same sampler, one lane, conv launches timed by
    # HIP events as above): what the f16x3 split path buys at equal (fp32-grade) parity gates.
    fp32_path = None
    if args.precision == "f16x3" and args.fp32_passes > 0:
        set_conv_precision("fp32")
        L.tcx_set_sample_lanes(1)
        run(-200)
        torch.cuda.synchronize(device)
        steps_saved = args.steps
        args.steps = args.fp32_passes
        L.tcx_prof_enable(1)
        el32 = timed(lambda i: run(200 + i))
        ms32, n32, fl32 = ctypes.c_double(), ctypes.c_longlong(), ctypes.c_double()
        L.tcx_prof_read(ctypes.byref(ms32), ctypes.byref(n32), ctypes.byref(fl32))
        L.tcx_prof_enable(0)
        L.tcx_set_sample_lanes(prev_lanes)
        set_conv_precision(args.precision)
        ach32 = (fl32.value / max(1, n32.value)) / ((ms32.value / max(1, n32.value)) * 1e-3) / 1e12 if n32.value else 0.0
        fp32_path = {"value": round(world * B * args.fp32_passes / el32, 4), "unit": "images/s", "lanes": 1,
                     "passes": args.fp32_passes, "ms_per_step": round(el32 / args.fp32_passes * 1e3, 3),
                     "roofline": {"bound": "mfma", "kernel": "k_conv (fp32-MFMA implicit GEMM, v_mfma_f32_32x32x2_f32)",
                                  "achieved": round(ach32, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                                  "frac": round(ach32 / FP32_PEAK_TFLOPS, 4),
                                  "avg_launch_ms": round(ms32.value / max(1, n32.value), 5)}}
        args.steps = steps_saved

    if args.precision == "f16x3":
        kname = ("split-path convs: k_conv3m (3x3 at 16/32/64-px rows, v_mfma_f32_16x16x32_f16; h2 sources or the "
                 "GroupNorm+SiLU prologue form), k_conv4s2g (4x4/s2, LDS-DMA), k_lin1x1 (1x1) — f16x3, 3 f16 "
                 "MFMAs per fp32 MAC; all conv launches of the pass")
        peak = F16_PEAK_TFLOPS / SPLIT_PRODUCTS
        peak_basis = "2500 TFLOP/s dense f16 MFMA / 3 products per fp32 MAC; achieved in fp32-equivalent FLOPs"
    elif args.precision == "bf16":
        kname = ("bf16 single-product convs (config 5): k_conv3lb (LDS-DMA 3x3 at 64/128/256-px rows, "
                 "v_mfma_f32_32x32x16_bf16; TCX_CONV3MB=1 adds k_conv3mb's 16x16x32 tap pairs at Cin >= 192), "
                 "k_conv4s2g (chunk-major skip planes), k_lin1x1 — one bf16 MFMA per MAC; all conv launches of the pass")
        peak = F16_PEAK_TFLOPS
        peak_basis = "2500 TFLOP/s dense bf16 MFMA"
    else:
        kname = "k_conv (fp32-MFMA implicit-GEMM conv, v_mfma_f32_32x32x2_f32)"
        peak = FP32_PEAK_TFLOPS
        peak_basis = "157.3 TFLOP/s fp32 MFMA"
    images = world * B * args.steps
    value = images / elapsed
    conv_avg_ms = ms.value / max(1, n.value)
    conv_avg_flop = fl.value / max(1, n.value)
    achieved = conv_avg_flop / (conv_avg_ms * 1e-3) / 1e12 if n.value else 0.0
    traffic = TRAFFIC_BYTES_PER_CONV_LAUNCH.get((args.precision, S))
    result = {
        "metric": "denoised images/sec (300-step reverse-SDE, CFG=1.5) at 1/2/4/8 MI355X",
        "value": round(value, 4),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": {"fp32": "fp32", "bf16": "bf16 (single-product MFMA, fp32 accumulation)"}.get(
            args.precision, "fp32 (f16x3 split MFMA, fp32-grade)"),
        "data": "synthetic (y_cat=i%4, theta=linspace(0,pi/3,B); random-init weights seed 0; Philox noise)",
        "config": {"workload": f"reverse-SDE {args.n_steps} steps, CFG {args.cfg}, t_end {args.t_end}, "
                               f"CondUNetTiny(base_ch={args.base_ch}) {S}x{S}, batch {B}/GPU",
                   "batch_per_gpu": B, "global_batch": world * B, "n_steps": args.n_steps, "cfg": args.cfg,
                   "image": [1, S, S], "conv_precision": args.precision, "sample_lanes": max(1, args.lanes),
                   "parallelism": "replicas" if world == 1 else f"dp{world} (independent shards)"},
        "path_tflops": round(value / world * FWD_PER_IMG * GFLOP_PER_IMG_FWD / 1e3, 3) if S == 64 else None,
        "roofline": {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 3), "peak": round(peak, 1),
                     "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                     "traffic": traffic,
                     "traffic_unit": "HBM bytes per conv launch",
                     "traffic_source": TRAFFIC_SOURCE[(args.precision, S)] if traffic is not None else
                     "not measured for this configuration (PMC passes exist for the 64x64 f16x3 headline and the "
                     "256x256 bf16 config 5 only)",
                     "peak_basis": peak_basis,
                     "measured_on": "one-lane roofline pass (same K sampling passes on one stream, HIP events per conv launch)",
                     "avg_launch_ms": round(conv_avg_ms, 5), "avg_launch_gflop": round(conv_avg_flop / 1e9, 4),
                     "launches": n.value,
                     "conv_share_of_step": round(ms.value / 1e3 / el1, 4)},
        "one_lane": {"value": round(images / el1, 4), "unit": "images/s", "ms_per_step": round(el1 / args.steps * 1e3, 3),
                     "lanes_speedup": round(el1 / elapsed, 4)},
    }
    if fp32_path is not None:
        result["fp32_path"] = fp32_path
    if args.save_images:
        imgs = timed_out
        if world > 1:
            from toycrystals_amd.dist import all_gather_
            bufs = [torch.empty_like(imgs) for _ in range(world)]
            all_gather_(bufs, imgs.contiguous())
            imgs = torch.cat(bufs, 0)
        if rank == 0:
            import numpy as np
            np.save(args.save_images, imgs.cpu().numpy())
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(model.state_dict(), args.cpu_batch, args.cpu_steps_a, args.cpu_steps_b,
                                              args.cfg, args.t_end)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
