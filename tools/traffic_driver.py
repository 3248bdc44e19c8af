#!/usr/bin/env python3
"""Run the north-star encoder forward (Large-17, B=32, T=1000, bf16, single stream: micro-batch
split off) for rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/profile_round.sh).
tools/traffic_summary.py maps the last forward's dispatches to stages (tools/stage_trace.py rules).
    python tools/traffic_driver.py [forwards]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conformer-nemo_amd"))
import torch  # noqa: E402
from nemo.collections.asr.modules import ConformerEncoder  # noqa: E402


def main(forwards):
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    enc = ConformerEncoder(feat_in=80, n_layers=17, d_model=512, n_heads=8).to(dev).eval()
    enc.set_compute_mode("bf16")
    x = torch.randn(32, 80, 1000, device=dev)
    lengths = torch.full((32,), 1000, dtype=torch.int64, device=dev)
    with torch.inference_mode():
        enc(audio_signal=x, length=lengths)                 # weight upload + workspace
        enc._native_for(dev).set_microbatches(1)
        for _ in range(forwards):
            y, _ = enc(audio_signal=x, length=lengths)
    torch.cuda.synchronize()
    assert torch.isfinite(y).all().item()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 2)
