#!/usr/bin/env python3
"""QKV GEMM epilogue cost: 8000 x 1536 x 512 on the 64x128 tile with the EPI_QKV epilogue vs a plain store."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "conformer-nemo_amd"))
import torch  # noqa: E402,F401
from conformer_amd import _lib  # noqa: E402

lib = _lib.load()
for rep in range(2):
    row = []
    for epi, name in [(0, "store"), (6, "qkv"), (0 | 32, "store-noepi")]:
        ms = ctypes.c_float(0)
        st = lib.cfm_bench_gemm(1, 5, epi, 8000, 1536, 512, 30, ctypes.byref(ms))
        row.append(f"{name} {ms.value * 1000:6.1f}us" if st == 0 else f"{name} err")
    print("  ".join(row), flush=True)
