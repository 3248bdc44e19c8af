"""ConvSubsampling parameter container + calc_length (reference subsampling.py:44-176, 272-282).

Only the 'striding' mode (2 x Conv2d(3, stride 2, pad 1) + ReLU, then Linear(C * F/4 -> d)) is
on the north-star path and implemented natively (the 2nd conv runs as an implicit-GEMM MFMA
kernel, csrc/gemm.hip).  The module holds the parameters with the reference's names; inside
ConformerEncoder its arithmetic runs in the encoder's native forward, and called on its own (eval) it
runs the same front-end kernels on a zero-layer handle.
"""
from __future__ import annotations

import math

import torch
from torch import nn


def calc_length(lengths, padding: int, kernel_size: int, stride: int, ceil_mode: bool, repeat_num: int = 1):
    """Output length of `repeat_num` strided convs; float32 arithmetic, floor/ceil, int32 result
    (reference subsampling.py:272-282)."""
    add_pad = float(padding * 2 - kernel_size)
    out = lengths.to(dtype=torch.float32)
    for _ in range(repeat_num):
        out = (out + add_pad) / float(stride) + 1.0
        out = torch.ceil(out) if ceil_mode else torch.floor(out)
    return out.to(dtype=torch.int32)


class ConvSubsampling(nn.Module):
    def __init__(self, subsampling, subsampling_factor, feat_in, feat_out, conv_channels, activation=None):
        super().__init__()
        if subsampling != "striding":
            raise NotImplementedError(f"subsampling='{subsampling}' has no native implementation (only 'striding')")
        if subsampling_factor % 2 != 0:
            raise ValueError("Sampling factor should be a multiply of 2!")
        self._subsampling = subsampling
        self._sampling_num = int(math.log(subsampling_factor, 2))
        if self._sampling_num != 2:
            raise NotImplementedError("the native path implements subsampling_factor=4")
        self._padding, self._stride, self._kernel_size, self._ceil_mode = 1, 2, 3, False
        self.feat_out = feat_out
        act = activation if activation is not None else nn.ReLU()
        layers, cin = [], 1
        for _ in range(self._sampling_num):
            layers += [nn.Conv2d(cin, conv_channels, kernel_size=3, stride=2, padding=1), act]
            cin = conv_channels
        self.conv = nn.Sequential(*layers)
        f = feat_in
        for _ in range(self._sampling_num):
            f = (f + 2 * self._padding - self._kernel_size) // self._stride + 1
        self.out = nn.Linear(conv_channels * f, feat_out)

    def forward(self, x, lengths):
        """subsampling.py:163-176: x (B, T, feat_in) -> ((B, T', feat_out), lengths (B,) int32), on the
        encoder's front-end kernels (eval; a zero-layer native handle, see submodule_ops.SubsamplingRunner)."""
        from conformer_amd import submodule_ops as ops
        ops.check_inference(self, x)
        if not isinstance(self.conv[1], nn.ReLU):
            raise NotImplementedError("the native subsampling fuses ReLU; other activations are not implemented")
        if x.dim() != 3:
            raise ValueError("ConvSubsampling expects x of shape (B, T, feat_in)")
        lengths = torch.as_tensor(lengths, device=x.device)
        return ops.SUBSAMPLING.forward(self, x, lengths, ops.compute_mode(self))
