"""Golden fixture for RNN-T training at the config-4 hidden size: gradients of the
REFERENCE RNNTDecoder (LSTM, pred_hidden 640, rnnt.py:50-283) and RNNTJoint (joint_hidden 640,
rnnt.py:613-1038) under torch autograd, CPU float32, U = 24 labels.  Only where /root/reference exists:

    python tests/golden/gen_rnnt_train_h640_golden.py     # writes tests/golden/rnnt_train_h640.npz

Set-up as gen_rnnt_train_goldens.py (eval mode, log_softmax False, loss = sum(logits * G)), except that the
640-wide weights are NOT stored: they come from a recipe the test replays - torch.Generator seeded with
`wseed`, one torch.randn(shape) per parameter in named_parameters order (decoder, then joint), scaled by
1/sqrt(fan_in) (0.1 for vectors), the embedding's padding row zeroed.  Stored: the inputs, G, the logits,
d(enc), every gradient of up to 65,536 elements in full (g::<module>.<key>), and for the larger ones the
gradient at a fixed sample of 16,384 flat indices (gi:: / gs::) plus its full L2 norm (gn::).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_joint_goldens import load_joint  # noqa: E402

# V, pred_hidden, layers, enc_hidden, joint_hidden, activation, B, T, U, seed
CASE = (40, 640, 1, 64, 640, "tanh", 2, 6, 24, 7)
FULL_MAX = 65536
SAMPLE = 16384


def recipe_weights(modules, wseed, V):
    """The weights the test replays: one randn per parameter in order, 1/sqrt(fan_in) scale."""
    g = torch.Generator().manual_seed(wseed)
    with torch.no_grad():
        for m in modules:
            for _, p in m.named_parameters():
                scale = 1.0 / float(np.sqrt(p.shape[-1])) if p.dim() > 1 else 0.1
                p.copy_(torch.randn(p.shape, generator=g) * scale)
        modules[0].prediction["embed"].weight[V].zero_()


def main():
    rnnt = load_joint()
    V, Hp, L, H1, J, act, B, T, U, seed = CASE
    torch.manual_seed(seed)
    dec = rnnt.RNNTDecoder(prednet=dict(pred_hidden=Hp, pred_rnn_layers=L, dropout=0.0), vocab_size=V).eval()
    joint = rnnt.RNNTJoint(jointnet=dict(encoder_hidden=H1, pred_hidden=Hp, joint_hidden=J, activation=act),
                           num_classes=V, log_softmax=False).eval()
    wseed = 500 + seed
    recipe_weights([dec, joint], wseed, V)
    g = torch.Generator().manual_seed(900 + seed)
    enc = torch.randn(B, H1, T, generator=g).requires_grad_(True)
    y = torch.randint(0, V, (B, U), generator=g)
    yl = torch.full((B,), U, dtype=torch.int64)
    gout, _, _ = dec(targets=y, target_length=yl)
    out = joint(encoder_outputs=enc, decoder_outputs=gout)
    G = torch.randn(out.shape, generator=g)
    (out * G).sum().backward()
    arrs = {"enc": enc.detach().numpy(), "y": y.numpy(), "G": G.numpy(), "logits": out.detach().numpy(),
            "g::enc": enc.grad.numpy(), "meta": np.array([V, Hp, L, H1, J, B, T, U]), "act": np.array(act),
            "wseed": np.array(wseed),
            "porder": np.array([f"{mn}.{k}" for mn, m in (("dec", dec), ("joint", joint)) for k, _ in m.named_parameters()])}
    rs = np.random.default_rng(seed)
    for mname, m in (("dec", dec), ("joint", joint)):
        for k, p in m.named_parameters():
            gr = p.grad.numpy().reshape(-1)
            if gr.size <= FULL_MAX:
                arrs[f"g::{mname}.{k}"] = p.grad.numpy()
            else:
                idx = np.sort(rs.choice(gr.size, SAMPLE, replace=False)).astype(np.int64)
                arrs[f"gi::{mname}.{k}"] = idx
                arrs[f"gs::{mname}.{k}"] = gr[idx]
                arrs[f"gn::{mname}.{k}"] = np.array(np.linalg.norm(gr.astype(np.float64)))
    np.savez_compressed(os.path.join(HERE, "rnnt_train_h640.npz"), **arrs)
    print("wrote rnnt_train_h640", out.shape, {k: v.shape for k, v in arrs.items() if k.startswith(("g", "gs"))})


if __name__ == "__main__":
    main()
