#!/usr/bin/env python3
"""Where does the bf16 compute mode's error come from?  CPU emulation on the reference-pinned torch
restatement (oracle/conformer_torch_cpu.py): the operands of chosen op classes are rounded to bf16
(fp32 accumulation, fp32 residual stream - what the HIP bf16 path does), and the output is compared
with the fp32 forward on the enc_large17 golden input (Large-17, B=2, T=1000):

    python tools/bf16_error_study.py [variant ...]

Op classes: sub (subsampling convs + Linear), ffn (linear1/linear2), qkv, out (linear_out), pos
(linear_pos), pw (pointwise convs), dw (depthwise conv), score (q.k and q.p), pv (probs.v)."""
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as TF

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import conformer_torch_cpu as ct  # noqa: E402
from recipe import make_state_dict  # noqa: E402

ALL = ("sub", "ffn", "qkv", "out", "pos", "pw", "dw", "score", "pv")


ROUND = os.environ.get("ROUND", "both")   # both | act | wt : which GEMM operand is rounded


LOWP = torch.float16 if os.environ.get("LOWP") == "fp16" else torch.bfloat16


def rb(t):
    return t.to(LOWP).to(torch.float32)


def rx(t):
    return rb(t) if ROUND in ("both", "act") else t


def rw(t):
    return rb(t) if ROUND in ("both", "wt") else t


def make_F(active, names):
    def cls_of(w):
        n = names.get(id(w), "")
        if n.startswith("pre_encode"):
            return "sub"
        if "feed_forward" in n:
            return "ffn"
        if any(k in n for k in ("linear_q", "linear_k", "linear_v")):
            return "qkv"
        if "linear_out" in n:
            return "out"
        if "linear_pos" in n:
            return "pos"
        if "pointwise" in n:
            return "pw"
        if "depthwise" in n:
            return "dw"
        return "other"

    def linear(x, w, b=None):
        if cls_of(w) in active:
            x, w = rx(x), rw(w)
        return TF.linear(x, w, b)

    def conv1d(x, w, b=None, **kw):
        if cls_of(w) in active:
            x, w = rx(x), rw(w)
        return TF.conv1d(x, w, b, **kw)

    def conv2d(x, w, b=None, **kw):
        if cls_of(w) in active:
            x, w = rx(x), rw(w)
        return TF.conv2d(x, w, b, **kw)

    ns = types.SimpleNamespace(**{k: getattr(TF, k) for k in dir(TF) if not k.startswith("_")})
    ns.linear, ns.conv1d, ns.conv2d = linear, conv1d, conv2d
    return ns


def run(active, sd, x, ln, cfg):
    names = {id(v): k for k, v in sd.items()}
    ct.F = make_F(active, names)
    mm = torch.matmul
    state = {"i": 0}

    def matmul(a, b):
        # mhsa issues q.k^T, q.p^T (scores) then probs.v: the 3rd of every 3 is P.V
        state["i"] += 1
        kind = "pv" if state["i"] % 3 == 0 else "score"
        if kind in active:
            a, b = rb(a), rb(b)
        return mm(a, b)

    ct.torch = types.SimpleNamespace(**{k: getattr(torch, k) for k in dir(torch) if not k.startswith("__")})
    ct.torch.matmul = matmul
    try:
        y, _ = ct.encoder_forward(x, ln, sd, cfg)
    finally:
        ct.F, ct.torch = TF, torch
    return y.numpy()


def main():
    torch.set_num_threads(8)
    z = np.load(os.path.join(ROOT, "tests", "golden", "enc_large17.npz"))
    cfg = json.loads(str(z["cfg_json"]))
    sd = {k: torch.from_numpy(np.asarray(v, dtype=np.float32)) for k, v in make_state_dict(cfg, int(z["seed"])).items()}
    x, ln = torch.from_numpy(z["x"]), torch.from_numpy(z["lengths"])
    ref = run(set(), sd, x, ln, cfg)
    print(f"fp32 vs golden relL2 {np.linalg.norm(ref - z['y']) / np.linalg.norm(z['y']):.2e}", flush=True)
    variants = sys.argv[1:] or ["all"] + [f"all-{c}" for c in ALL] + list(ALL)
    for v in variants:
        if v == "all":
            active = set(ALL)
        elif v.startswith("all-"):
            active = set(ALL) - set(v[4:].split("+"))
        else:
            active = set(v.split("+"))
        y = run(active, sd, x, ln, cfg)
        e = np.linalg.norm(y - ref) / np.linalg.norm(ref)
        print(f"{v:16s} relL2 {e:.3e}", flush=True)


if __name__ == "__main__":
    main()
