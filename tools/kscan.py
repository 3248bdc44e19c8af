import ctypes, os, sys
sys.path.insert(0, "conformer-nemo_amd")
import torch
from conformer_amd import _lib
lib = _lib.load()
for epi in (0, 2, 3):
    for (M, N) in [(8000, 2048), (8000, 512)]:
        row = []
        for K in (256, 512, 1024, 2048, 4096, 8192):
            ms = ctypes.c_float(0)
            _lib.check(lib.cfm_bench_gemm(1, 1 if N == 2048 else 0, epi, M, N, K, 10, ctypes.byref(ms)), "b")
            row.append(f"K{K}:{ms.value*1000:7.1f}us {2*M*N*K/ms.value/1e9:5.0f}T")
        print(f"epi{epi} M{M} N{N}: " + "  ".join(row), flush=True)
