"""Config-4 joint (B=16, T'=400, U+1=101, H=640, V+1=1025) timed alone with stream events: the fused logits
kernel (CFM_JOINT_FUSED=1) with timing probes (CFM_JOINT_PROBE: 1 no logits stores, 2 no MFMAs, 4 no hidden
formation) and the hidden kernel + GEMM path (CFM_JOINT_FUSED=0). Device time per call, median of 5 x 10."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "conformer-nemo_amd"))
from conformer_amd.joint import NativeJoint  # noqa: E402

B, T, U, H1, H2, H, C = 16, 400, 101, 512, 640, 640, 1025
torch.manual_seed(0)
j = NativeJoint(H1, H2, H, C, activation="relu", compute="bf16")
j.set_weights(torch.randn(H, H1, device="cuda") / H1 ** 0.5, torch.zeros(H, device="cuda"),
              torch.randn(H, H2, device="cuda") / H2 ** 0.5, torch.zeros(H, device="cuda"),
              torch.randn(C, H, device="cuda") / H ** 0.5, torch.zeros(C, device="cuda"))
enc = torch.randn(B, H1, T, device="cuda")
dec = torch.randn(B, H2, U, device="cuda")
out = torch.empty(B, T, U, C, device="cuda")
split = os.environ.get("CFM_JOINT_SPLIT", "1")
cases = [("fused", "1", "0", split), ("split0", "1", "0", "0"), ("unfused", "0", "0", split)] + \
    [(f"probe{p}", "1", str(p), split) for p in (1, 2, 4, 6, 3, 7)] + [("fused", "1", "0", split), ("split0", "1", "0", "0")]
for name, fused, probe, sp in cases:
    os.environ["CFM_JOINT_FUSED"], os.environ["CFM_JOINT_PROBE"], os.environ["CFM_JOINT_SPLIT"] = fused, probe, sp
    j.forward(enc, dec, out=out)
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            j.forward(enc, dec, out=out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 10)
    ts.sort()
    print(f"{name:8s} joint {ts[2]:.4f} ms  (min {ts[0]:.4f})", flush=True)
