#!/usr/bin/env python3
"""conv.2 weight / bias gradient of one bf16 training step at the train_large shape (d_model 512, 512 conv
channels, B x T from tests/golden/train_large.npz), saved to an npz (run once per CFM_TN_CONV setting):
    python tools/tn_conv_check.py OUT.npz            -> saves the gradients
    python tools/tn_conv_check.py --cmp A.npz B.npz  -> relL2 / max-abs between the two runs"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conformer-nemo_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def run(out):
    import torch
    from nemo.collections.asr.modules import ConformerEncoder
    from recipe import make_inputs, make_state_dict
    z = np.load(os.path.join(ROOT, "tests", "golden", "train_large.npz"))
    cfg = json.loads(str(z["cfg_json"]))
    enc = ConformerEncoder(**cfg, dropout=0.0, dropout_emb=0.0, dropout_att=0.0)
    sd = make_state_dict(cfg, int(z["seed"]))
    ref = enc.state_dict()
    enc.load_state_dict({k: torch.from_numpy(np.asarray(v)).reshape(ref[k].shape) for k, v in sd.items()})
    enc.set_compute_mode("bf16")
    enc = enc.cuda().train()
    B, T = int(z["B"]), int(z["T"])
    x, ln = make_inputs(B, T, 80, int(z["seed"]) + 100, [int(v) for v in z["lengths"]])
    y, _ = enc(audio_signal=torch.from_numpy(x).cuda(), length=torch.from_numpy(ln).cuda())
    R = np.random.default_rng(int(z["seed"]) + 200).standard_normal(tuple(y.shape)).astype(np.float32)
    (y * torch.from_numpy(R).cuda()).sum().backward()
    torch.cuda.synchronize()
    p = dict(enc.named_parameters())
    np.savez(out, w=p["pre_encode.conv.2.weight"].grad.cpu().numpy(), b=p["pre_encode.conv.2.bias"].grad.cpu().numpy(),
             w0=p["pre_encode.conv.0.weight"].grad.cpu().numpy())


def cmp(a, b):
    za, zb = np.load(a), np.load(b)
    for k in za.files:
        x, y = za[k].astype(np.float64), zb[k].astype(np.float64)
        print(f"{k}: relL2 {np.linalg.norm(x - y) / max(np.linalg.norm(y), 1e-30):.3e} max|d| {np.abs(x - y).max():.3e} "
              f"|ref| {np.linalg.norm(y):.3e}")


if __name__ == "__main__":
    if sys.argv[1] == "--cmp":
        cmp(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1])
