"""Host-side profile of the config-4 RNN-T training step (bench.py --mode rnnt_train): where the Python /
launch time goes, and how far the host runs ahead of the GPU.  Replaces bench.timed_loop with a loop that
records, per step phase, the host time to enqueue it (no syncs added) and, with stream events, the GPU
time at which the phase's work starts and ends.

    python tools/rnnt_host_profile.py [--steps 3]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

PHASES = []


def patched(step, warmup, steps, barrier):
    for _ in range(warmup):
        r = step()
    barrier()
    torch.cuda.synchronize()
    for s in range(steps):
        PHASES.clear()
        t0 = time.perf_counter()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        r = step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"step {s}: host enqueue {1e3 * (t1 - t0):7.2f} ms, wall {1e3 * (t2 - t0):7.2f} ms")
        prev_t, prev_e = t0, e0
        for name, t, e in PHASES:
            print(f"   {name:14s} host {1e3 * (t - prev_t):7.2f} ms   gpu {prev_e.elapsed_time(e):7.2f} ms   "
                  f"(gpu done at {e0.elapsed_time(e):7.2f}, host at {1e3 * (t - t0):7.2f})")
            prev_t, prev_e = t, e
    barrier()
    return 1.0, r


def mark(name):
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    PHASES.append((name, time.perf_counter(), e))


orig_backward = torch.Tensor.backward


def backward(self, *a, **k):
    orig_backward(self, *a, **k)
    mark("backward")


torch.Tensor.backward = backward
orig_step = torch.optim.AdamW.step


def opt_step(self, *a, **k):
    r = orig_step(self, *a, **k)
    mark("opt_step")
    return r


torch.optim.AdamW.step = opt_step
bench.timed_loop = patched
# module hooks: wrap the module classes' __call__ targets after construction via forward hooks
from torch.nn.modules.module import register_module_forward_hook  # noqa: E402

TOP = {"ConformerEncoder": "encoder", "RNNTDecoder": "prediction_net", "RNNTJoint": "joint", "RNNTLoss": "loss"}


def hook(mod, inp, out):
    n = TOP.get(type(mod).__name__)
    if n:
        mark(n)


register_module_forward_hook(hook)
if __name__ == "__main__":
    steps = sys.argv[sys.argv.index("--steps") + 1] if "--steps" in sys.argv else "3"
    sys.argv = ["bench.py", "--mode", "rnnt_train", "--steps", steps, "--warmup", "2"]
    bench.main()
