#!/usr/bin/env python3
"""Micro-batch bitwise check of the bf16 Large-17 forward (B=32, T=1000) in THIS process's environment:
max |y(mb) - y(1)| for mb in 3, 8, and part 0 of mb=3 (utterances 0-10) run alone as B=11."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "conformer-nemo_amd"))
import torch  # noqa: E402

from conformer_amd import NativeEncoder, make_cfg  # noqa: E402


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else "run"
    torch.manual_seed(0)
    enc = NativeEncoder(make_cfg(80, 17, 512, n_heads=8), device=0, compute="bf16")
    w = {}
    for k, n in enc.param_names().items():
        if "running_var" in k:
            w[k] = torch.rand(n) + 0.5
        elif k.endswith("num_batches_tracked"):
            continue
        else:
            w[k] = torch.randn(n) * (0.02 if n > 4096 else 0.1)
    enc.set_weights(w)
    x = torch.randn(32, 80, 1000, device="cuda")
    ln = torch.full((32,), 1000, dtype=torch.int32, device="cuda")
    if os.environ.get("MB_POISON_WS"):   # NaN-fill the workspace: a read of a byte no kernel wrote shows
        enc.set_microbatches(3)
        enc._workspace(enc.workspace_size(32, 1000)).fill_(255)
        enc.set_microbatches(1)
        enc._workspace(enc.workspace_size(32, 1000)).fill_(255)
    y1, _ = enc.forward(x, ln)
    if os.environ.get("MB_JUNK2"):   # beside small-LDS elementwise kernels that can share CUs with the forward's blocks
        side = torch.cuda.Stream()
        j = torch.randn(64 << 20, device="cuda")
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            for _ in range(200):
                j.mul_(1.0001).add_(1e-6)
        y1b, _ = enc.forward(x, ln)
        torch.cuda.synchronize()
        print(label, f"junk2 {(y1 - y1b).abs().max().item():.3e}", flush=True)
        return
    if os.environ.get("MB_JUNK"):   # run the single-stream forward again beside unrelated work on another stream
        side = torch.cuda.Stream()
        a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            for _ in range(40):
                a = (a @ a).clamp_(-1, 1)
        y1b, _ = enc.forward(x, ln)
        torch.cuda.synchronize()
    else:
        y1b, _ = enc.forward(x, ln)
    out = [f"det {(y1 - y1b).abs().max().item():.3e} finite {bool(torch.isfinite(y1).all())} sum {y1.double().sum().item():.10e}"]
    if os.environ.get("MB_ONLY_SINGLE"):
        print(label, " ".join(out), flush=True)
        return
    for mb in (3, 8):
        enc.set_microbatches(mb)
        if os.environ.get("MB_POISON_WS"):
            enc._workspace(enc.workspace_size(32, 1000)).fill_(255)
        ym, _ = enc.forward(x, ln)
        if os.environ.get("MB_POISON_WS"):
            enc._workspace(enc.workspace_size(32, 1000)).fill_(255)
        ym2, _ = enc.forward(x, ln)
        torch.cuda.synchronize()
        out.append(f"mb{mb} {(ym - y1).abs().max().item():.3e} (rerun {(ym2 - ym).abs().max().item():.3e}, finite {bool(torch.isfinite(ym).all())})")
        if mb == 3:
            per = (ym - y1).abs().flatten(1).max(1).values.cpu().tolist()
            out.append("per-utt " + ",".join(f"{v:.0e}" for v in per))
    enc.set_microbatches(1)
    y11, _ = enc.forward(x[:11].contiguous(), ln[:11].contiguous())
    out.append(f"B11 {(y11 - y1[:11]).abs().max().item():.3e}")
    y1s, _ = enc.forward(x[30:31].contiguous(), ln[30:31].contiguous())
    out.append(f"B1 {(y1s - y1[30:31]).abs().max().item():.3e}")
    print(label, " ".join(out), flush=True)


if __name__ == "__main__":
    main()
