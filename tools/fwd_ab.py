#!/usr/bin/env python3
"""Time the Large-17 bf16 encoder forward (B=32, T=1000) in THIS process's environment
(CFM_TILES, CFM_MICROBATCH, ... are read once per process):
    python tools/fwd_ab.py LABEL [iters]         -> one line: LABEL ms/forward (median of 5 bursts)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "conformer-nemo_amd"))
import torch  # noqa: E402

from conformer_amd import NativeEncoder, make_cfg  # noqa: E402


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else "run"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    B, T = int(os.environ.get("AB_B", 32)), int(os.environ.get("AB_T", 1000))
    torch.manual_seed(0)
    enc = NativeEncoder(make_cfg(80, 17, 512, n_heads=8), device=0, compute="bf16")
    shapes = enc.param_names()
    w = {}
    for k, n in shapes.items():
        if "running_var" in k:
            w[k] = torch.rand(n) + 0.5
        elif k.endswith("num_batches_tracked"):
            continue
        else:
            w[k] = torch.randn(n) * (0.02 if n > 4096 else 0.1)
    enc.set_weights(w)
    x = torch.randn(B, 80, T, device="cuda")
    ln = torch.full((B,), T, dtype=torch.int32, device="cuda")
    for _ in range(3):
        enc.forward(x, ln)
    torch.cuda.synchronize()
    res = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            enc.forward(x, ln)
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / iters)
    res.sort()
    print(f"{label:40s} {res[2]:.3f} ms  (min {res[0]:.3f})", flush=True)


if __name__ == "__main__":
    main()
