"""Disk dataset of the reference (toycrystals/disk_data.py:8-31) and a device-side batch pipeline.

`ToyCrystalsDiskDataset` is the drop-in: the same file format (a torch.save dict with
x_u8 [N,1,H,W] uint8, y_cat [N] int64, y_cont [N,4] float32, written by the reference's
scripts/build_dataset.py), the same item semantics (x = x_u8 / 255 as float32).  The file is
loaded with torch.load(weights_only=True): tensors only, nothing executed.

`DeviceBatches` replaces `DataLoader(ds, batch_size, shuffle, drop_last)` on the training path:
the uint8 images stay resident in HBM (50k 64x64 images = 205 MB) and each batch is one
tcx_u8_gather launch (shuffled index gather + /255) instead of per-item host work.  Shuffling
uses torch.randperm on the CPU generator, so `torch.manual_seed` governs the order.  With
`rank/world` it yields this rank's equal slice of every global batch (batch-DP training).
"""
from __future__ import annotations

from pathlib import Path
from typing import Iterator, Optional, Tuple

import torch

from ._lib import check, lib, ptr, stream_ptr


class ToyCrystalsDiskDataset(torch.utils.data.Dataset):
    def __init__(self, path) -> None:
        obj = torch.load(Path(path), map_location="cpu", weights_only=True)
        self.x_u8: torch.Tensor = obj["x_u8"]
        self.y_cat: torch.Tensor = obj["y_cat"]
        self.y_cont: torch.Tensor = obj["y_cont"]

    def __len__(self) -> int:
        return int(self.x_u8.shape[0])

    def __getitem__(self, idx: int):
        x = self.x_u8[idx].to(torch.float32) / 255.0
        return x, self.y_cat[idx], self.y_cont[idx]


class DeviceBatches:
    """Iterate (x [B,1,H,W] f32, y_cat [B], y_cont [B,D]) batches of a dataset held on `device`."""

    def __init__(self, ds: ToyCrystalsDiskDataset, batch_size: int, device, shuffle: bool = True,
                 drop_last: bool = True, rank: int = 0, world: int = 1,
                 generator: Optional[torch.Generator] = None,
                 fixed_order: Optional[torch.Tensor] = None) -> None:
        if batch_size % world != 0:
            raise ValueError(f"global batch {batch_size} must be divisible by world size {world}")
        self.device = torch.device(device)
        # float images (toycrystals_amd.data.RenderedSet, the in-memory renderer) or uint8 (disk)
        xf = getattr(ds, "x_f32", None)
        self.x_f32 = xf.to(self.device).contiguous() if xf is not None else None
        self.x_u8 = ds.x_u8.to(self.device).contiguous() if xf is None else None
        xs = self.x_f32 if xf is not None else self.x_u8
        self.y_cat = ds.y_cat.to(self.device, torch.int64).contiguous()
        self.y_cont = ds.y_cont.to(self.device, torch.float32).contiguous()
        self.N = int(xs.shape[0])
        self.shape = tuple(xs.shape[1:])
        self.npix = int(xs[0].numel())
        self.batch_size, self.shuffle, self.drop_last = int(batch_size), shuffle, drop_last
        self.rank, self.world = rank, world
        self.generator = generator
        # a recorded item order (replay of a reference run's DataLoader permutation): used for
        # every epoch instead of a fresh shuffle
        self.fixed_order = None if fixed_order is None else torch.as_tensor(fixed_order, dtype=torch.int64)
        if self.fixed_order is not None and self.fixed_order.numel() < len(self) * self.batch_size:
            raise ValueError(f"fixed_order holds {self.fixed_order.numel()} items, an epoch needs "
                             f"{len(self) * self.batch_size}")

    def __len__(self) -> int:
        if self.drop_last:
            return self.N // self.batch_size
        return (self.N + self.batch_size - 1) // self.batch_size

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
        if self.fixed_order is not None:
            order = self.fixed_order
        else:
            order = torch.randperm(self.N, generator=self.generator) if self.shuffle else torch.arange(self.N)
        order = order.to(self.device)
        L = lib()
        st = stream_ptr(self.device)
        for i in range(len(self)):
            g = order[i * self.batch_size:(i + 1) * self.batch_size]
            per = g.shape[0] // self.world
            idx = g[self.rank * per:(self.rank + 1) * per].contiguous() if self.world > 1 else g.contiguous()
            B = idx.shape[0]
            if self.x_f32 is not None:
                x = self.x_f32.index_select(0, idx)
            else:
                x = torch.empty((B,) + self.shape, device=self.device, dtype=torch.float32)
                check(L.tcx_u8_gather(ptr(self.x_u8), ptr(idx), B, self.npix, ptr(x), st), "tcx_u8_gather")
            yield x, self.y_cat.index_select(0, idx), self.y_cont.index_select(0, idx)
