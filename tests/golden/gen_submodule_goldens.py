"""Golden fixtures for the standalone submodules (ConformerLayer, ConformerFeedForward, ConformerConvolution,
RelPositionMultiHeadAttention, MultiHeadAttention, ConvSubsampling) from the REFERENCE modules (only where /root/reference
exists; loaded as gen_goldens.load_reference does):

    python tests/golden/gen_submodule_goldens.py      # writes tests/golden/sub_*.npz

Each fixture holds the module's seeded weights ("w::<state_dict key>"), its inputs and the reference
module's eval-mode output.  Masks are the encoder's (conformer_encoder.py:257-270) for the stored lengths.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_goldens import load_reference  # noqa: E402


def masks(lengths, T, ctx):
    rng = torch.arange(T)
    pad = rng.unsqueeze(0) < lengths.unsqueeze(-1)
    att = pad.unsqueeze(1).repeat([1, T, 1])
    att = torch.logical_and(att, att.transpose(1, 2))
    if ctx[0] >= 0:
        att = att.triu(diagonal=-ctx[0])
    if ctx[1] >= 0:
        att = att.tril(diagonal=ctx[1])
    return ~att, ~pad


def randomize(module, seed):
    g = torch.Generator().manual_seed(seed)
    sd = module.state_dict()
    out = {}
    for k, v in sd.items():
        if not torch.is_floating_point(v):
            out[k] = v
        elif k.endswith("running_var"):
            out[k] = torch.rand(v.shape, generator=g) + 0.5
        elif k.endswith("running_mean"):
            out[k] = torch.randn(v.shape, generator=g) * 0.3
        elif k.endswith(".weight") and v.dim() == 1:           # norm scales
            out[k] = 1.0 + 0.2 * torch.randn(v.shape, generator=g)
        else:
            fan = v[0].numel() if v.dim() > 1 else v.numel()
            out[k] = torch.randn(v.shape, generator=g) / max(fan, 1) ** 0.5
    module.load_state_dict(out)
    return {f"w::{k}": v.numpy() for k, v in out.items() if torch.is_floating_point(v)}


def save(name, **arrs):
    np.savez_compressed(os.path.join(HERE, f"sub_{name}.npz"), **arrs)
    print("wrote", name, {k: v.shape for k, v in arrs.items() if not k.startswith("w::")})


def main():
    R = load_reference()
    torch.manual_seed(0)
    B, T, d, H, dff = 2, 37, 64, 4, 256
    lengths = torch.tensor([37, 20])
    g = torch.Generator().manual_seed(123)
    x = torch.randn(B, T, d, generator=g)
    pe = R.mha.RelPositionalEncoding(d_model=d, dropout_rate=0.0, max_len=5000, xscale=None)
    pe.extend_pe(T, torch.device("cpu"))
    _, pos_emb = pe(x)
    with torch.no_grad():
        for case, ctx, norm, seed in (("layer", (-1, -1), "batch_norm", 1), ("layer_ctx_ln", (8, 4), "layer_norm", 2)):
            pu = torch.nn.Parameter(torch.randn(H, d // H, generator=g) * 0.1)
            pv = torch.nn.Parameter(torch.randn(H, d // H, generator=g) * 0.1)
            layer = R.cm.ConformerLayer(d_model=d, d_ff=dff, self_attention_model="rel_pos", n_heads=H,
                                        conv_kernel_size=31, conv_norm_type=norm, dropout=0.1, dropout_att=0.1,
                                        pos_bias_u=pu, pos_bias_v=pv).eval()
            w = randomize(layer, seed)
            att, pad = masks(lengths, T, ctx)
            y = layer(x=x, att_mask=att, pos_emb=pos_emb, pad_mask=pad)
            save(case, x=x.numpy(), lengths=lengths.numpy(), ctx=np.array(ctx), pos_emb=pos_emb.numpy(),
                 att_mask=att.numpy(), pad_mask=pad.numpy(), y=y.numpy(), norm=np.array(norm), **w)
        ff = R.cm.ConformerFeedForward(d_model=d, d_ff=dff, dropout=0.1).eval()
        w = randomize(ff, 3)
        save("ffn", x=x.numpy(), y=ff(x).numpy(), **w)
        for case, norm, use_pad, seed in (("conv_bn", "batch_norm", True, 4), ("conv_ln_nopad", "layer_norm", False, 5)):
            conv = R.cm.ConformerConvolution(d_model=d, kernel_size=31, norm_type=norm).eval()
            w = randomize(conv, seed)
            _, pad = masks(lengths, T, (-1, -1))
            y = conv(x, pad if use_pad else None)
            save(case, x=x.numpy(), lengths=lengths.numpy(), pad_mask=pad.numpy(), use_pad=np.array(use_pad),
                 norm=np.array(norm), y=y.numpy(), **w)
        rel = R.mha.RelPositionMultiHeadAttention(n_head=H, n_feat=d, dropout_rate=0.1, pos_bias_u=None,
                                                  pos_bias_v=None).eval()
        w = randomize(rel, 6)
        att, _ = masks(lengths, T, (10, 3))
        y = rel(query=x, key=x, value=x, mask=att, pos_emb=pos_emb)
        save("relattn", x=x.numpy(), pos_emb=pos_emb.numpy(), att_mask=att.numpy(), y=y.numpy(), **w)
        mha = R.mha.MultiHeadAttention(n_head=H, n_feat=d, dropout_rate=0.1).eval()
        w = randomize(mha, 7)
        att, _ = masks(lengths, T, (-1, -1))
        x2 = torch.randn(B, T, d, generator=g)
        y = mha(query=x, key=x2, value=x2, mask=att)
        save("mha", x=x.numpy(), x2=x2.numpy(), att_mask=att.numpy(), y=y.numpy(), **w)
        # ConvSubsampling ('striding', factor 4): x (B, T, feat_in) with ragged lengths (subsampling.py:163-176)
        for case, (Bs, Ts, F, C, dd, seed) in (("subsampling", (3, 101, 80, 64, 96, 8)),
                                                 ("subsampling_c176", (2, 64, 40, 176, 176, 9))):
            sub = R.sub.ConvSubsampling(subsampling="striding", subsampling_factor=4, feat_in=F, feat_out=dd,
                                        conv_channels=C, activation=torch.nn.ReLU()).eval()
            w = randomize(sub, seed)
            xs = torch.randn(Bs, Ts, F, generator=g)
            ls = torch.tensor([Ts - 29 * i for i in range(Bs)])
            ys, ylen = sub(xs, ls)
            save(case, x=xs.numpy(), lengths=ls.numpy(), y=ys.numpy(), y_len=ylen.numpy(), **w)


if __name__ == "__main__":
    main()
