#!/usr/bin/env python3
"""Host-side phase timing of the config-3 training step (where does the host block on the GPU?):
    python tools/train_host_timing.py [steps]
Prints per phase the host wall time; a phase whose host time is close to its GPU work is blocking."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conformer-nemo_amd"))


def main():
    from nemo.collections.asr.losses import CTCLoss
    from nemo.collections.asr.modules import ConformerEncoder, ConvASRDecoder
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    B, T, V, U = 32, 1000, 256, 60
    enc = ConformerEncoder(feat_in=80, n_layers=17, d_model=512, n_heads=8, dropout=0.1, dropout_emb=0.0,
                           dropout_att=0.1).to(dev).train()
    dec = ConvASRDecoder(feat_in=512, num_classes=V).to(dev).train()
    loss_fn = CTCLoss(num_classes=V, zero_infinity=True, reduction="mean_batch")
    params = [p for m in (enc, dec) for p in m.parameters()]
    opt = torch.optim.AdamW(params, lr=1e-4, betas=(0.9, 0.98), weight_decay=1e-3, fused=True)
    g = torch.Generator(device=dev).manual_seed(1000)
    x = torch.randn(B, 80, T, device=dev, generator=g)
    lengths = torch.full((B,), T, dtype=torch.int64, device=dev)
    targets = torch.randint(0, V, (B, U), device=dev, generator=g)
    tlen = torch.full((B,), U, dtype=torch.int64, device=dev)
    names = ["zero_grad", "enc_fwd", "dec_fwd", "loss", "backward", "opt_step"]
    for s in range(steps):
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        opt.zero_grad(set_to_none=True)
        t.append(time.perf_counter())
        y, yl = enc(audio_signal=x, length=lengths)
        t.append(time.perf_counter())
        lp = dec(encoder_output=y)
        t.append(time.perf_counter())
        loss = loss_fn(log_probs=lp, targets=targets, input_lengths=yl, target_lengths=tlen)
        t.append(time.perf_counter())
        loss.backward()
        t.append(time.perf_counter())
        opt.step()
        t.append(time.perf_counter())
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        ph = " ".join(f"{n} {1e3 * (t[i + 1] - t[i]):7.2f}" for i, n in enumerate(names))
        print(f"step {s}: host {ph} | drain {1e3 * (t[-1] - t[-2]):7.2f} | total {1e3 * (t[-1] - t[0]):7.2f} ms",
              flush=True)


if __name__ == "__main__":
    main()
