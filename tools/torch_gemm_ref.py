#!/usr/bin/env python3
"""Reference point only (not used by the product): torch.matmul (hipBLASLt) bf16 time on the encoder's
GEMM shapes, C[M,N] = A[M,K] @ W[N,K]^T, no epilogue."""
import torch

SHAPES = [("ref4096", 4096, 4096, 4096), ("ffn_up", 8000, 2048, 512), ("ffn_down", 8000, 512, 2048),
          ("qkv", 8000, 1536, 512), ("out/pw2", 8000, 512, 512), ("pw1_glu", 8000, 1024, 512),
          ("conv2", 160000, 512, 4608), ("sub_out", 8000, 512, 10240)]
for name, M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ w.t()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 5 if M * N * K > 1e11 else 20
    e0.record()
    for _ in range(it):
        c = a @ w.t()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    print(f"{name:10s} {ms * 1e3:8.1f} us  {2 * M * N * K / ms / 1e9:6.0f} TF/s", flush=True)
