"""Shared plumbing of the CLI mirrors: package path, device choice, optional torchrun batch-DP."""
from __future__ import annotations

import os
import sys

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG_ROOT not in sys.path:
    sys.path.insert(0, _PKG_ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from toycrystals_amd.dist import all_reduce_, broadcast_, dist_backend, dp_forced, local_device  # noqa: E402


def pick_device(name: str) -> torch.device:
    """The reference falls back to CPU without CUDA; this build has no CPU path, so it refuses."""
    if name == "cpu":
        raise SystemExit("this MI355X build has no CPU path: use --device cuda (the MI355X under PyTorch-ROCm)")
    if not torch.cuda.is_available():
        raise SystemExit("no GPU visible: this build runs on the MI355X only")
    return torch.device(name)


def init_dp():
    """One process per GPU under torchrun (backend nccl = RCCL over xGMI; TCX_DIST_BACKEND=gloo lets
    ranks share one GPU, toycrystals_amd.dist); (rank, world, device).  Under RCCL the group is bound
    to this rank's device (device_id: the communicator is created eagerly on it, not on whatever
    device is current at the first collective).  TCX_DP_FORCE=1 builds the group at world 1 too, so
    a one-GPU run executes the collectives of the N-GPU path."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 and not (dp_forced() and "RANK" in os.environ):
        return 0, 1, None
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", rank))
    device = local_device(local)
    torch.cuda.set_device(device)
    backend = dist_backend()
    if backend == "nccl":
        dist.init_process_group(backend, rank=rank, world_size=world, device_id=device)
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    return rank, world, device


def lead_only_rng(device):
    """Context for work only rank 0 does between training steps (sample grids): its torch CPU and
    device generator draws are rolled back afterwards, so every rank's generators stay in lockstep
    (the shuffle permutation and the --global-draws noise of the next steps are the same on all
    ranks, and equal the one-GPU run's)."""
    return torch.random.fork_rng(devices=[device])


def sync_rng_from_lead(world: int, device) -> None:
    """Every rank adopts rank 0's torch CPU and device generator states (identity at world 1).
    For work rank 0 does ALONE whose draws the one-GPU run also makes (the latent-cache build with
    --z-target sample): the one-GPU run's generators have advanced by those draws, so the ranks
    must continue from rank 0's advanced state, not roll it back."""
    if not dist.is_initialized():  # (world 1 under TCX_DP_FORCE=1 still runs the collective)
        return
    st = [None]
    if dist.get_rank() == 0:
        st = [(torch.get_rng_state(), torch.cuda.get_rng_state(device))]
    dist.broadcast_object_list(st, src=0)
    torch.set_rng_state(st[0][0])
    torch.cuda.set_rng_state(st[0][1], device)


def shutdown_dp(world: int) -> None:
    if dist.is_initialized():  # world > 1, or world 1 under TCX_DP_FORCE=1
        dist.barrier()
        dist.destroy_process_group()


def allreduce_scalar_mean(v: float, world: int, device) -> float:
    if not dist.is_initialized():
        return v
    t = torch.tensor([v], dtype=torch.float64, device=device)
    all_reduce_(t)
    return float(t.item()) / world


def broadcast_from_lead(tensors, world: int, device):
    """Rank 0's list of CPU tensors on every rank (shapes and dtypes travel first); identity without
    a process group.  Rank 0 keeps its own tensors (so its arithmetic is the one-GPU run's); the
    other ranks receive CPU copies."""
    if not dist.is_initialized():
        return tensors
    meta = [None]
    if dist.get_rank() == 0:
        meta = [[(tuple(t.shape), t.dtype) for t in tensors]]
    dist.broadcast_object_list(meta, src=0)
    out = []
    for i, (shape, dtype) in enumerate(meta[0]):
        buf = tensors[i].to(device).contiguous() if dist.get_rank() == 0 else torch.empty(shape, dtype=dtype, device=device)
        broadcast_(buf, src=0)
        out.append(tensors[i].cpu() if dist.get_rank() == 0 else buf.cpu())
    return out
