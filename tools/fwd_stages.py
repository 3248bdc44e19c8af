#!/usr/bin/env python3
"""Per-stage device time of the Large-17 bf16 encoder forward (B=32, T=1000) in THIS process's
environment (cfm_encoder_forward_timed, mean of 3 forwards).  With CFM_GEMM_PROBE set the GEMM stages
run without main-loop loads (1), without epilogue (2) or with one K-step (4): timing only.
    python tools/fwd_stages.py LABEL      -> one line per stage: LABEL stage ms launches"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "conformer-nemo_amd"))
import torch  # noqa: E402

from conformer_amd import NativeEncoder, make_cfg  # noqa: E402


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else "run"
    B, T = int(os.environ.get("AB_B", 32)), int(os.environ.get("AB_T", 1000))
    d, L, H = int(os.environ.get("AB_D", 512)), int(os.environ.get("AB_L", 17)), int(os.environ.get("AB_H", 8))
    torch.manual_seed(0)
    enc = NativeEncoder(make_cfg(80, L, d, n_heads=H), device=0, compute="bf16")
    w = {}
    for k, n in enc.param_names().items():
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
    agg = {}
    for _ in range(3):
        for k, (ms, n) in enc.forward_timed(x, ln).items():
            a = agg.setdefault(k, [0.0, n])
            a[0] += ms / 3
    tot = 0.0
    for k, (ms, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        if n:
            print(f"{label:14s} {k:22s} {ms:8.4f} ms  {n:3d}", flush=True)
            tot += ms
    print(f"{label:14s} {'sum':22s} {tot:8.4f} ms", flush=True)


if __name__ == "__main__":
    main()
