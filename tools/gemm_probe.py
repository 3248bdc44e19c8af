#!/usr/bin/env python3
"""Split a GEMM's time into its load and MFMA parts: full kernel, loads only (no MFMA), MFMA only
(no main-loop loads) for the given tiles and shapes.
    python tools/gemm_probe.py TILES SHAPES     e.g. 11,5 ref4096,ffn_up"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "conformer-nemo_amd"))
import torch  # noqa: E402,F401
from conformer_amd import _lib  # noqa: E402
from op_driver import GEMM_SHAPES  # noqa: E402

lib = _lib.load()
tiles = [int(t) for t in sys.argv[1].split(",")]
for name in sys.argv[2].split(","):
    M, N, K, epi = GEMM_SHAPES[name]
    for t in tiles:
        row = []
        for probe, label in ((0, "full"), (1, "no-loads"), (2, "no-epi"), (3, "mfma-only"), (4, "1-kstep"), (6, "skeleton")):
            ms = ctypes.c_float(0)
            _lib.check(lib.cfm_bench_gemm(1, t, epi + 16 * probe, M, N, K, 10, ctypes.byref(ms)), name)
            row.append(f"{label} {ms.value * 1e3:8.1f}us")
        print(f"{name:9s} tile{t:<3d} " + "  ".join(row), flush=True)
