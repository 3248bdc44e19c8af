"""Swish activation (reference activations.py:20): x * sigmoid(x) == nn.SiLU."""
from torch import nn


class Swish(nn.SiLU):
    """Swish == SiLU; fused into the native GEMM / conv epilogues."""
