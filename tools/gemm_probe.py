#!/usr/bin/env python3
"""Split a GEMM's time into its parts with the kernel's probe bits (csrc/gemm.hip GemmParams.probe):
1 no main-loop loads, 2 no epilogue, 4 one K-step, 8 plain residual stores (EPI_RESID_LN),
16 no LayerNorm tail.
    python tools/gemm_probe.py TILES SHAPES          e.g. 11,5 ref4096,ffn_up
    PROBES=0,8,16,24 python tools/gemm_probe.py 5 out_ln"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "conformer-nemo_amd"))
import torch  # noqa: E402,F401
from conformer_amd import _lib  # noqa: E402
from op_driver import GEMM_SHAPES  # noqa: E402

PROBES = [(0, "full"), (1, "no-loads"), (2, "no-epi"), (3, "mfma-only"), (4, "1-kstep"), (6, "skeleton")]


def main():
    lib = _lib.load()
    tiles = [int(t) for t in sys.argv[1].split(",")]
    probes = PROBES
    if os.environ.get("PROBES"):
        probes = [(int(x), "p" + x) for x in os.environ["PROBES"].split(",")]
    for name in sys.argv[2].split(","):
        M, N, K, epi = GEMM_SHAPES[name]
        for t in tiles:
            row = []
            for probe, label in probes:
                ms = ctypes.c_float(0)
                _lib.check(lib.cfm_bench_gemm(1, t, epi + 16 * probe, M, N, K, 10, ctypes.byref(ms)), name)
                row.append(f"{label} {ms.value * 1e3:8.1f}us")
            print(f"{name:9s} tile{t:<3d} " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
