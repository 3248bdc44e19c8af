#!/usr/bin/env python3
"""GEMM microbenchmark over the encoder's shapes (and 4096^3 as a reference point) for each tile
configuration: prints TFLOP/s and the achieved fraction of the 2.5 PF bf16 dense peak."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "conformer-nemo_amd"))
import torch  # noqa: E402,F401
from conformer_amd import _lib  # noqa: E402

SHAPES = [  # name, M, N, K, epilogue (0 store, 2 swish, 3 resid, 5 glu, 6 qkv)
    ("ref4096", 4096, 4096, 4096, 0),
    ("ffn_up", 8000, 2048, 512, 2),
    ("ffn_down", 8000, 512, 2048, 3),
    ("qkv", 8000, 1536, 512, 6),
    ("out/pw2", 8000, 512, 512, 3),
    ("pw1_glu", 8000, 512, 512, 5),
    ("conv2", 160000, 512, 4608, 0),
    ("sub_out", 8000, 512, 10240, 3),
]


def main():
    lib = _lib.load()
    tiles = [int(t) for t in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["-1", "0", "1", "2", "3"])]
    dt = int(os.environ.get("DT", "1"))
    print(f"{'shape':10s} " + " ".join(f"{'tile' + str(t):>16s}" for t in tiles))
    for name, M, N, K, epi in SHAPES:
        row = []
        for t in tiles:
            ms = ctypes.c_float(0)
            iters = 5 if M * N * K > 1e11 else 20
            st = lib.cfm_bench_gemm(dt, t, epi, M, N, K, iters, ctypes.byref(ms))
            if st != 0:
                row.append(f"{'err':>16s}")
                continue
            tf = 2.0 * M * N * K / (ms.value * 1e-3) / 1e12
            row.append(f"{ms.value * 1000:8.1f}us {tf:5.0f}T")
        print(f"{name:10s} " + " ".join(row), flush=True)


if __name__ == "__main__":
    main()
