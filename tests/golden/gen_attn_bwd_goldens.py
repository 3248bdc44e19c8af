"""Golden fixture for the relative-position attention backward (cfm_op_rel_attention_backward,
include/cfm_train.h), from the REFERENCE's own RelPositionMultiHeadAttention
(multi_head_attention.py:124-210) under torch autograd in float64, dropout off, with the attention
mask built as ConformerEncoder.forward builds it (conformer_encoder.py:260-267: pad mask on both
axes, optional att_context_size band) — only where /root/reference exists:

    python tests/golden/gen_attn_bwd_goldens.py   # writes tests/golden/bwd_attn.npz

q, k, v, p (the linear_q/k/v/pos outputs) and the context (linear_out input) are recorded with
hooks, together with their gradients; only arrays are written.  Two cases: full context ("full")
and a limited window att_context_size = [6, 2] ("ctx").
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_goldens import load_reference  # noqa: E402


def att_mask(lens, T, left, right):
    """conformer_encoder.py:260-267."""
    pad = torch.arange(T)[None, :] < torch.tensor(lens)[:, None]          # valid frames
    m = pad.unsqueeze(1).repeat([1, T, 1])
    m = torch.logical_and(m, m.transpose(1, 2))
    if left >= 0:
        m = m.triu(diagonal=-left)
    if right >= 0:
        m = m.tril(diagonal=right)
    return ~m


def run_case(ref, seed, B, T, d, H, lens, left, right):
    torch.manual_seed(seed)
    att = ref.mha.RelPositionMultiHeadAttention(n_head=H, n_feat=d, dropout_rate=0.0, pos_bias_u=None,
                                                pos_bias_v=None).double().train()
    with torch.no_grad():
        for p in att.parameters():
            p.uniform_(-0.25, 0.25)
    g = np.random.default_rng(seed)
    x = torch.tensor(g.standard_normal((B, T, d)), dtype=torch.float64, requires_grad=True)
    pos = torch.tensor(g.standard_normal((1, 2 * T - 1, d)), dtype=torch.float64)
    rec = {}

    def keep(name):
        def hook(_m, _inp, out):
            out.retain_grad()
            rec[name] = out
        return hook

    def keep_in(name):
        def hook(_m, inp):
            inp[0].retain_grad()
            rec[name] = inp[0]
        return hook

    for n in ("q", "k", "v", "pos"):
        getattr(att, "linear_" + n).register_forward_hook(keep(n))
    att.linear_out.register_forward_pre_hook(keep_in("ctx"))
    out = att(x, x, x, att_mask(lens, T, left, right), pos)
    dout = torch.tensor(g.standard_normal((B, T, d)), dtype=torch.float64)
    out.backward(dout)
    f = lambda t: t.detach().reshape(-1, d).numpy().astype(np.float32)
    gr = lambda t: t.grad.reshape(-1, d).numpy().astype(np.float32)
    return dict(B=np.int32(B), T=np.int32(T), H=np.int32(H), lens=np.asarray(lens, np.int32),
                ctx_left=np.int32(left), ctx_right=np.int32(right),
                x=f(x), pos_emb=f(pos), dout=f(dout), q=f(rec["q"]), k=f(rec["k"]), v=f(rec["v"]), p=f(rec["pos"]),
                ctx=f(rec["ctx"]), out=f(out),
                u=att.pos_bias_u.detach().numpy().reshape(-1).astype(np.float32),
                vb=att.pos_bias_v.detach().numpy().reshape(-1).astype(np.float32),
                w_q=att.linear_q.weight.detach().numpy().astype(np.float32),
                w_k=att.linear_k.weight.detach().numpy().astype(np.float32),
                w_v=att.linear_v.weight.detach().numpy().astype(np.float32),
                w_pos=att.linear_pos.weight.detach().numpy().astype(np.float32),
                w_out=att.linear_out.weight.detach().numpy().astype(np.float32),
                d_ctx=gr(rec["ctx"]), d_q=gr(rec["q"]), d_k=gr(rec["k"]), d_v=gr(rec["v"]), d_p=gr(rec["pos"]),
                d_u=att.pos_bias_u.grad.numpy().reshape(-1).astype(np.float32),
                d_vb=att.pos_bias_v.grad.numpy().reshape(-1).astype(np.float32),
                d_x=gr(x), d_w_pos=att.linear_pos.weight.grad.numpy().astype(np.float32),
                d_w_q=att.linear_q.weight.grad.numpy().astype(np.float32),
                d_b_q=att.linear_q.bias.grad.numpy().astype(np.float32))


def main():
    ref = load_reference()
    cases = {"full": run_case(ref, 11, B=3, T=45, d=128, H=4, lens=[45, 30, 17], left=-1, right=-1),
             "ctx": run_case(ref, 12, B=2, T=37, d=64, H=2, lens=[37, 20], left=6, right=2)}
    flat = {f"{c}.{k}": v for c, kv in cases.items() for k, v in kv.items()}
    np.savez_compressed(os.path.join(HERE, "bwd_attn.npz"), **flat)
    print("bwd_attn written")


if __name__ == "__main__":
    main()
