#!/usr/bin/env python3
"""Export the weights of a score-model checkpoint (train_sde_score_model.py layout:
{"model", "ema", ...}) to a pickle-free .npz: `export_ckpt.py CKPT OUT.npz [model|ema]`."""
import sys

import numpy as np
import torch

ckpt, out = sys.argv[1], sys.argv[2]
key = sys.argv[3] if len(sys.argv) > 3 else "ema"
obj = torch.load(ckpt, map_location="cpu", weights_only=True)
sd = obj[key] if key in obj else obj["model"]
np.savez_compressed(out, **{k: v.detach().cpu().float().numpy() for k, v in sd.items()})
print(f"exported {key} ({len(sd)} tensors, epoch_next={obj.get('epoch_next')}) -> {out}")
