"""Golden fixtures for the backward building blocks (include/cfm_train.h), from the REFERENCE's
own modules under torch autograd (only where /root/reference exists):

    python tests/golden/gen_bwd_goldens.py       # writes tests/golden/bwd_ffn.npz

The macaron FFN sub-block of ConformerLayer.forward (conformer_modules.py:98-101):
    out = x + 0.5 * feed_forward1(norm_feed_forward1(x))
with the reference ConformerLayer's own LayerNorm and ConformerFeedForward (loaded as in
gen_goldens.py), float64, dropout inactive (eval), an upstream gradient dout of the same shape.
Only arrays are written.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_goldens import load_reference  # noqa: E402


def main():
    ref = load_reference()
    torch.manual_seed(0)
    d, B, T = 64, 2, 37
    layer = ref.cm.ConformerLayer(d_model=d, d_ff=4 * d, n_heads=4, conv_kernel_size=31, dropout=0.0).double().eval()
    with torch.no_grad():
        for p in layer.parameters():
            p.uniform_(-0.3, 0.3)
        layer.norm_feed_forward1.weight.uniform_(0.5, 1.5)
    g = np.random.default_rng(3)
    x = torch.tensor(g.standard_normal((B, T, d)), requires_grad=True)
    dout = torch.tensor(g.standard_normal((B, T, d)))
    hn = layer.norm_feed_forward1(x)
    hn.retain_grad()
    z = layer.feed_forward1.linear1(hn)
    z.retain_grad()
    u = layer.feed_forward1.activation(z)
    u.retain_grad()
    y = layer.feed_forward1.linear2(layer.feed_forward1.dropout(u))
    out = x + y * layer.fc_factor
    out.backward(dout)
    ln, l1, l2 = layer.norm_feed_forward1, layer.feed_forward1.linear1, layer.feed_forward1.linear2
    arr = lambda t: (t.detach().numpy().reshape(B * T, -1) if t.dim() == 3 else t.detach().numpy()).astype(np.float32)
    np.savez_compressed(
        os.path.join(HERE, "bwd_ffn.npz"),
        x=arr(x), dout=arr(dout), hn=arr(hn), z=arr(z), u=arr(u), out=arr(out),
        ln_w=arr(ln.weight), ln_b=arr(ln.bias), w1=arr(l1.weight), b1=arr(l1.bias), w2=arr(l2.weight),
        b2=arr(l2.bias), fc_factor=np.float64(layer.fc_factor),
        d_x=arr(x.grad), d_hn=arr(hn.grad), d_z=arr(z.grad), d_u=arr(u.grad),
        d_ln_w=arr(ln.weight.grad), d_ln_b=arr(ln.bias.grad), d_w1=arr(l1.weight.grad), d_b1=arr(l1.bias.grad),
        d_w2=arr(l2.weight.grad), d_b2=arr(l2.bias.grad))
    print("bwd_ffn written: |dx|", float(x.grad.norm()))


if __name__ == "__main__":
    main()
