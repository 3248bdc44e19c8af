#!/usr/bin/env python3
"""Epilogue cost probe: one GEMM shape timed with different epilogues (cfm_bench_gemm)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "conformer-nemo_amd"))
import torch  # noqa: E402,F401
from conformer_amd import _lib  # noqa: E402

lib = _lib.load()
for (M, N, K, tile) in [(8000, 2048, 512, 11), (8000, 512, 512, 5), (8000, 512, 2048, 5)]:
    row = []
    for epi, name in [(0, "store"), (2, "swish"), (3, "resid"), (5, "glu")]:
        ms = ctypes.c_float(0)
        st = lib.cfm_bench_gemm(1, tile, epi, M, N, K, 30, ctypes.byref(ms))
        row.append(f"{name} {ms.value * 1000:6.1f}us" if st == 0 else f"{name} err")
    print(f"{M}x{N}x{K} tile{tile}: " + "  ".join(row), flush=True)
