#!/usr/bin/env python3
"""Check that bench.py's CPU baseline (oracle/conformer_torch_cpu.py) runs at the reference's speed:
time the REFERENCE ConformerEncoder (imported by path, tests/golden/gen_goldens.py's loader — only
where /root/reference exists) and the restatement on the same host cores, same weights and input
(cfg2: Large-17, B=32, T=1000, fp32, eval, torch.no_grad), 1 warm-up + min of 3 each, and check
they agree numerically.  SURVEY §8d asks for the two to be within +-10 %.
    python tools/cpu_baseline_check.py [threads] [B]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import conformer_torch_cpu as TC  # noqa: E402
from gen_goldens import load_reference, ref_encoder  # noqa: E402
from recipe import make_inputs  # noqa: E402


def tmin(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else (os.cpu_count() or 8)
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    T = 1000
    torch.set_num_threads(threads)
    cfg = dict(d_model=512, n_heads=8, n_layers=17)
    R = load_reference()
    enc, sd = ref_encoder(R, cfg, seed=1)
    sdt = {k: torch.from_numpy(np.asarray(v)).reshape(enc.state_dict()[k].shape) for k, v in sd.items()}
    x, ln = make_inputs(B, T, 80, 0, [T] * B)
    xt, lt = torch.from_numpy(x), torch.from_numpy(ln)
    with torch.no_grad():
        y_ref, _ = enc(audio_signal=xt, length=lt)
        y_tc, _ = TC.encoder_forward(xt, lt, sdt, cfg)
        err = float((y_tc - y_ref).norm() / y_ref.norm())
        t_ref = tmin(lambda: enc(audio_signal=xt, length=lt))
        t_tc = tmin(lambda: TC.encoder_forward(xt, lt, sdt, cfg))
    cpu = "unknown"
    with open("/proc/cpuinfo") as f:
        cpu = next((ln_.split(":", 1)[1].strip() for ln_ in f if ln_.startswith("model name")), cpu)
    print(f"host: {cpu}, {threads} threads, torch {torch.__version__}")
    print(f"workload: Large-17 encoder forward, B={B}, T={T}, fp32 eval; 1 warm-up + min of 3")
    print(f"reference ConformerEncoder : {t_ref:.3f} s  = {B * T / t_ref:.0f} frames/s")
    print(f"conformer_torch_cpu        : {t_tc:.3f} s  = {B * T / t_tc:.0f} frames/s  "
          f"({100.0 * (t_tc / t_ref - 1):+.1f} % time vs reference)")
    print(f"relL2(restatement, reference) = {err:.2e}")


if __name__ == "__main__":
    main()
