#!/usr/bin/env python3
"""Determinism / batch-invariance diagnostic of the full encoder (fp32 and bf16)."""
import os
import sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "conformer-nemo_amd"), os.path.join(ROOT, "tests", "golden")]
from recipe import make_inputs, make_state_dict  # noqa: E402
from conformer_amd import NativeEncoder, make_cfg  # noqa: E402

cfg = dict(d_model=512, n_heads=8, n_layers=int(os.environ.get("LAYERS", "17")))
sd = make_state_dict(cfg, 7)
for compute in ("fp32", "bf16"):
    enc = NativeEncoder(make_cfg(80, cfg["n_layers"], 512, n_heads=8), compute=compute)
    enc.set_weights({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    x, lens = make_inputs(32, 1000, seed=11)
    xd, ld = torch.from_numpy(x).cuda(), torch.from_numpy(lens).cuda()
    ys = [enc.forward(xd, ld)[0].cpu().numpy() for _ in range(3)]
    enc.set_microbatches(1)
    y1 = enc.forward(xd, ld)[0].cpu().numpy()
    yb1 = enc.forward(xd[30:31], ld[30:31])[0].cpu().numpy()
    d = lambda a, b: float(np.abs(a - b).max())
    print(compute, "rerun", d(ys[0], ys[1]), d(ys[0], ys[2]), "mb1-vs-mb2", d(ys[0], y1), "B1-vs-B32", d(yb1[0], ys[0][30]),
          flush=True)
