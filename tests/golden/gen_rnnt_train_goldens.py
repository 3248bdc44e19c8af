"""Golden fixtures for RNN-T training (VERDICT r02 'What's missing' #1): gradients of the REFERENCE
RNNTDecoder (prediction net: embedding + LSTM, rnnt.py:50-283) and RNNTJoint (rnnt.py:613-1038) under
torch autograd, CPU float32.  Only where /root/reference exists:

    python tests/golden/gen_rnnt_train_goldens.py     # writes tests/golden/rnnt_train_*.npz

Loaded with gen_joint_goldens.load_joint's typing-only shims.  The modules run in eval mode (dropout off:
the reference's dropout masks come from torch's RNG and cannot be matched) with gradients enabled; the
joint's log_softmax is False (logits, the GPU training configuration).  The upstream gradient of the
logits is a fixed random tensor G (the loss is sum(logits * G)), so the fixture pins the joint and
prediction-net backward independently of the RNN-T loss (pinned separately by rnnt_loss_*.npz).
Stored: inputs, weights (w::<module>.<key>), G, logits, and every gradient (g::<module>.<key>, g::enc).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_joint_goldens import load_joint  # noqa: E402

CASES = {
    # name: (V, pred_hidden, layers, enc_hidden, joint_hidden, activation, B, T, U, seed)
    "rnnt_train_small": (30, 32, 1, 24, 40, "relu", 3, 7, 5, 1),
    "rnnt_train_2layer_tanh": (17, 16, 2, 32, 24, "tanh", 2, 9, 4, 2),
}


def main():
    rnnt = load_joint()
    for name, (V, Hp, L, H1, J, act, B, T, U, seed) in CASES.items():
        torch.manual_seed(seed)
        dec = rnnt.RNNTDecoder(prednet=dict(pred_hidden=Hp, pred_rnn_layers=L, dropout=0.0), vocab_size=V).eval()
        joint = rnnt.RNNTJoint(jointnet=dict(encoder_hidden=H1, pred_hidden=Hp, joint_hidden=J, activation=act),
                               num_classes=V, log_softmax=False).eval()
        g = torch.Generator().manual_seed(100 + seed)
        with torch.no_grad():   # non-trivial weights (the embedding's padding row stays zero)
            for m in (dec, joint):
                for k, p in m.named_parameters():
                    p.copy_(torch.randn(p.shape, generator=g) * 0.3)
            dec.prediction["embed"].weight[V].zero_()
        enc = (torch.randn(B, H1, T, generator=g)).requires_grad_(True)
        y = torch.randint(0, V, (B, U), generator=g)
        yl = torch.full((B,), U, dtype=torch.int64)
        gout, _, _ = dec(targets=y, target_length=yl)
        out = joint(encoder_outputs=enc, decoder_outputs=gout)
        G = torch.randn(out.shape, generator=g)
        (out * G).sum().backward()
        arrs = {"enc": enc.detach().numpy(), "y": y.numpy(), "G": G.numpy(), "logits": out.detach().numpy(),
                "g::enc": enc.grad.numpy(),
                "meta": np.array([V, Hp, L, H1, J, B, T, U]), "act": np.array(act)}
        for mname, m in (("dec", dec), ("joint", joint)):
            for k, p in m.named_parameters():
                arrs[f"w::{mname}.{k}"] = p.detach().numpy()
                arrs[f"g::{mname}.{k}"] = p.grad.numpy()
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrs)
        print("wrote", name, out.shape)


if __name__ == "__main__":
    main()
