"""Golden fixture for the convolution-module backward ops (include/cfm_train.h), from the
REFERENCE's own ConformerConvolution (conformer_modules.py:124-180) in TRAINING mode (BatchNorm1d
batch statistics, running-stat update) under torch autograd, float32 (the module casts the GLU
output with .float(), conformer_modules.py:166, so it only runs in fp32), with a pad mask
(only where /root/reference exists):

    python tests/golden/gen_conv_bwd_goldens.py   # writes tests/golden/bwd_conv.npz

Intermediates are recorded with forward hooks on the reference submodules; only arrays are written.
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
    d, B, T = 64, 3, 45
    conv = ref.cm.ConformerConvolution(d_model=d, kernel_size=31).float().train()
    with torch.no_grad():
        for p in conv.parameters():
            p.uniform_(-0.3, 0.3)
        conv.batch_norm.weight.uniform_(0.5, 1.5)
        conv.batch_norm.running_mean.uniform_(-0.2, 0.2)
        conv.batch_norm.running_var.uniform_(0.5, 1.5)
    rm0, rv0 = conv.batch_norm.running_mean.clone(), conv.batch_norm.running_var.clone()
    g = np.random.default_rng(4)
    lens = np.array([45, 30, 17], np.int32)
    x = torch.tensor(g.standard_normal((B, T, d)), dtype=torch.float32, requires_grad=True)
    pad_mask = torch.arange(T)[None, :] >= torch.tensor(lens)[:, None]
    rec = {}

    def keep(name):
        def hook(_m, _inp, out):
            out.retain_grad()
            rec[name] = out
        return hook

    conv.pointwise_conv1.register_forward_hook(keep("pre"))       # (B, 2d, T)
    conv.depthwise_conv.register_forward_hook(keep("h"))          # (B, d, T) pre-BN
    conv.batch_norm.register_forward_hook(keep("bn"))             # (B, d, T)
    conv.pointwise_conv2.register_forward_hook(keep("y2"))
    out = conv(x, pad_mask)
    dout = torch.tensor(g.standard_normal((B, T, d)), dtype=torch.float32)
    out.backward(dout)
    cl = lambda t: t.detach().transpose(1, 2).reshape(B * T, -1).numpy().astype(np.float32)   # (B,C,T) -> rows
    pre = rec["pre"]
    glu = torch.nn.functional.glu(pre.detach(), dim=1).masked_fill(pad_mask.unsqueeze(1), 0.0)
    bnm = conv.batch_norm
    np.savez_compressed(
        os.path.join(HERE, "bwd_conv.npz"),
        x=x.detach().reshape(B * T, d).numpy().astype(np.float32), lens=lens, B=np.int32(B), T=np.int32(T),
        dout=dout.reshape(B * T, d).numpy().astype(np.float32),
        pre=cl(pre), glu=cl(glu), h=cl(rec["h"]), bn=cl(rec["bn"]), out=out.detach().reshape(B * T, d).numpy(),
        pw1_w=conv.pointwise_conv1.weight.detach().numpy()[:, :, 0].astype(np.float32),
        pw1_b=conv.pointwise_conv1.bias.detach().numpy().astype(np.float32),
        dw_w=conv.depthwise_conv.weight.detach().numpy().astype(np.float32),
        dw_b=conv.depthwise_conv.bias.detach().numpy().astype(np.float32),
        bn_w=bnm.weight.detach().numpy().astype(np.float32), bn_b=bnm.bias.detach().numpy().astype(np.float32),
        bn_rm0=rm0.numpy().astype(np.float32), bn_rv0=rv0.numpy().astype(np.float32),
        bn_rm1=bnm.running_mean.numpy().astype(np.float32), bn_rv1=bnm.running_var.numpy().astype(np.float32),
        bn_momentum=np.float32(bnm.momentum),
        pw2_w=conv.pointwise_conv2.weight.detach().numpy()[:, :, 0].astype(np.float32),
        pw2_b=conv.pointwise_conv2.bias.detach().numpy().astype(np.float32),
        d_x=x.grad.reshape(B * T, d).numpy().astype(np.float32), d_pre=cl(pre.grad), d_h=cl(rec["h"].grad),
        d_bn=cl(rec["bn"].grad),
        d_pw1_w=conv.pointwise_conv1.weight.grad.numpy()[:, :, 0].astype(np.float32),
        d_pw1_b=conv.pointwise_conv1.bias.grad.numpy().astype(np.float32),
        d_dw_w=conv.depthwise_conv.weight.grad.numpy().astype(np.float32),
        d_dw_b=conv.depthwise_conv.bias.grad.numpy().astype(np.float32),
        d_bn_w=bnm.weight.grad.numpy().astype(np.float32), d_bn_b=bnm.bias.grad.numpy().astype(np.float32),
        d_pw2_w=conv.pointwise_conv2.weight.grad.numpy()[:, :, 0].astype(np.float32),
        d_pw2_b=conv.pointwise_conv2.bias.grad.numpy().astype(np.float32))
    print("bwd_conv written")


if __name__ == "__main__":
    main()
