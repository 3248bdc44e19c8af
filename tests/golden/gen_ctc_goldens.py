"""Generate the CTC head / CTC loss golden fixtures by running the REFERENCE (only where
/root/reference exists):

    python tests/golden/gen_ctc_goldens.py        # writes tests/golden/ctc_*.npz

The loss is the reference's own CTCLoss class (nemo/collections/asr/losses/ctc.py), loaded by file
path under typing-only shims (typecheck no-op, Serialization/Typing empty bases, neural-type
dummies — none touches arithmetic), called exactly as EncDecCTCModel does (zero_infinity=True,
reduction 'mean_batch', ctc_models.py:190-194, 608-610).  The ConvASRDecoder module itself
cannot be imported here (conv_asr.py needs omegaconf and the Jasper stack), so its forward
expression conv_asr.py:444 — log_softmax(Conv1d(k=1)(x).transpose(1, 2), -1) — is evaluated with
the same torch ops.  Gradients come from torch autograd through both.  Only arrays are written.
"""
import importlib.util
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def load_reference_ctc():
    for n in ["nemo", "nemo.collections", "nemo.collections.asr", "nemo.collections.asr.losses", "nemo.core"]:
        m = types.ModuleType(n)
        m.__path__ = []
        sys.modules[n] = m

    class typecheck:
        def __init__(self, *a, **k):
            pass

        def __call__(self, f):
            return f

    classes = types.ModuleType("nemo.core.classes")
    classes.Serialization = type("Serialization", (), {})
    classes.Typing = type("Typing", (), {})
    classes.typecheck = typecheck
    sys.modules["nemo.core.classes"] = classes
    nt = types.ModuleType("nemo.core.neural_types")
    for k in ["LabelsType", "LengthsType", "LogprobsType", "LossType", "NeuralType"]:
        setattr(nt, k, lambda *a, **kw: None)
    sys.modules["nemo.core.neural_types"] = nt
    spec = importlib.util.spec_from_file_location("nemo.collections.asr.losses.ctc",
                                                  f"{REF}/nemo/collections/asr/losses/ctc.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.CTCLoss


def make_case(seed, B, T, D, V, U, in_len, tgt_len, repeat=False):
    g = np.random.default_rng(seed)
    C = V + 1
    enc = g.standard_normal((B, D, T)).astype(np.float32)
    bound = 1.0 / np.sqrt(D)
    w = g.uniform(-bound, bound, (C, D, 1)).astype(np.float32)
    b = g.uniform(-bound, bound, (C,)).astype(np.float32)
    tg = g.integers(0, V, (B, U)).astype(np.int32)
    if repeat:          # consecutive repeats need a blank between them
        tg[:, 1] = tg[:, 0]
        tg[:, 2] = tg[:, 0]
    return dict(enc=enc, w=w, b=b, targets=tg, in_len=np.asarray(in_len, np.int32),
                tgt_len=np.asarray(tgt_len, np.int32), blank=np.int32(V))


def run(CTCLoss, c):
    enc = torch.tensor(c["enc"], dtype=torch.float64, requires_grad=True)
    w = torch.tensor(c["w"], dtype=torch.float64, requires_grad=True)
    b = torch.tensor(c["b"], dtype=torch.float64, requires_grad=True)
    logits = torch.nn.functional.conv1d(enc, w, b)                     # Conv1d(k=1), conv_asr.py:438-439
    lp = torch.nn.functional.log_softmax(logits.transpose(1, 2), dim=-1)   # conv_asr.py:444
    lp.retain_grad()
    loss_fn = CTCLoss(num_classes=int(c["blank"]), zero_infinity=True, reduction="mean_batch")
    loss = loss_fn(log_probs=lp, targets=torch.tensor(c["targets"]), input_lengths=torch.tensor(c["in_len"]),
                   target_lengths=torch.tensor(c["tgt_len"]))
    loss.backward()
    per = CTCLoss(num_classes=int(c["blank"]), zero_infinity=True, reduction="none")(
        log_probs=lp.detach(), targets=torch.tensor(c["targets"]), input_lengths=torch.tensor(c["in_len"]),
        target_lengths=torch.tensor(c["tgt_len"]))
    out = dict(c)
    out.update(log_probs=lp.detach().numpy(), greedy=lp.detach().numpy().argmax(-1).astype(np.int32),
               loss=np.float64(loss.item()), nll=per.numpy(), grad_lp=lp.grad.numpy(),
               grad_enc=enc.grad.numpy(), grad_w=w.grad.numpy()[:, :, 0], grad_b=b.grad.numpy())
    return out


def main():
    CTCLoss = load_reference_ctc()
    cases = {
        # small: ragged input/target lengths, repeated labels, an empty target, an infeasible one
        "ctc_small": make_case(1, B=5, T=20, D=16, V=5, U=6, in_len=[20, 17, 12, 20, 3],
                               tgt_len=[6, 4, 6, 0, 5], repeat=True),
        # BASELINE cfg 3 geometry at reduced width: T'=250, V=256 (+blank), U=60
        "ctc_cfg3": make_case(2, B=4, T=250, D=64, V=256, U=60, in_len=[250, 230, 200, 126],
                              tgt_len=[60, 55, 40, 60]),
    }
    for name, c in cases.items():
        out = run(CTCLoss, c)
        # float64 runs, float32 storage (losses kept in float64)
        out = {k: (v.astype(np.float32) if isinstance(v, np.ndarray) and v.dtype == np.float64 and k != "nll" else v)
               for k, v in out.items()}
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        print(name, "loss", float(out["loss"]), "nll", out["nll"])


if __name__ == "__main__":
    main()
