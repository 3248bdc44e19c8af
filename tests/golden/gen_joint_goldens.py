"""Golden fixtures for the RNN-T joint (include/cfm_joint.h), from the REFERENCE RNNTJoint
(nemo/collections/asr/modules/rnnt.py:613-1038), eval mode, float32 on CPU.  Only where
/root/reference exists:

    python tests/golden/gen_joint_goldens.py   # writes tests/golden/joint_*.npz

The reference module is loaded with the same typing-only shims as gen_goldens.py plus three more
that carry no arithmetic: `nemo.utils.logging` (a no-op logger), `nemo.core.NeuralModule`
(torch.nn.Module) and extra neural-type names.  Weights are seeded, the joint's parameters and
inputs are stored (they are small), and both logits (log_softmax=False) and log-probs
(log_softmax=True) are recorded.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_goldens import REF, load_reference  # noqa: E402


def load_joint():
    load_reference()    # package stubs + typing shims

    class _Log:
        def __getattr__(self, _n):
            return lambda *a, **k: None

    utils = types.ModuleType("nemo.utils")
    utils.logging = _Log()
    sys.modules["nemo.utils"] = utils
    core = sys.modules["nemo.core"]
    core.NeuralModule = torch.nn.Module
    sys.modules["nemo.core.classes"].typecheck = sys.modules["nemo.core.classes.common"].typecheck
    nt = sys.modules["nemo.core.neural_types"]
    for name in ["EmbeddedTextType", "LogprobsType", "LossType", "ElementType", "LabelsType", "LengthsType",
                 "AcousticEncodedRepresentation", "NeuralType"]:
        setattr(nt, name, lambda *a, **kw: None)
    for n, p in [("nemo.collections.common", "nemo/collections/common"),
                 ("nemo.collections.common.parts", "nemo/collections/common/parts")]:
        m = types.ModuleType(n)
        m.__path__ = [f"{REF}/{p}"]
        sys.modules[n] = m
    import importlib.util
    spec = importlib.util.spec_from_file_location("nemo.collections.asr.modules.rnnt",
                                                  f"{REF}/nemo/collections/asr/modules/rnnt.py")
    mod = importlib.util.module_from_spec(spec)
    sys.modules["nemo.collections.asr.modules.rnnt"] = mod
    spec.loader.exec_module(mod)
    return mod


CASES = {
    # name: (jointnet, num_classes, B, T, U, seed)
    "joint_relu": (dict(encoder_hidden=32, pred_hidden=24, joint_hidden=40, activation="relu", dropout=0.1), 32, 2, 7,
                   5, 1),
    "joint_tanh": (dict(encoder_hidden=64, pred_hidden=48, joint_hidden=64, activation="tanh"), 29, 3, 11, 4, 2),
    "joint_sigmoid_h30": (dict(encoder_hidden=16, pred_hidden=20, joint_hidden=30, activation="sigmoid"), 16, 1, 9,
                          6, 3),
}


def main():
    rnnt = load_joint()
    for name, (jn, V, B, T, U, seed) in CASES.items():
        torch.manual_seed(seed)
        joint = rnnt.RNNTJoint(jointnet=dict(jn), num_classes=V).eval()
        with torch.no_grad():
            for p in joint.parameters():
                p.uniform_(-0.4, 0.4)
        g = np.random.default_rng(seed)
        enc = torch.tensor(g.standard_normal((B, jn["encoder_hidden"], T)), dtype=torch.float32)
        dec = torch.tensor(g.standard_normal((B, jn["pred_hidden"], U)), dtype=torch.float32)
        out = {"jointnet": np.array(repr(sorted(jn.items()))), "num_classes": np.int64(V), "enc": enc.numpy(),
               "dec": dec.numpy()}
        with torch.no_grad():
            joint.log_softmax = False
            out["logits"] = joint(encoder_outputs=enc, decoder_outputs=dec).numpy()
            joint.log_softmax = True
            out["logprobs"] = joint(encoder_outputs=enc, decoder_outputs=dec).numpy()
        for k, v in joint.state_dict().items():
            out["p__" + k] = v.numpy()
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        print(name, out["logits"].shape)


if __name__ == "__main__":
    main()
