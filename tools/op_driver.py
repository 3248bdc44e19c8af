#!/usr/bin/env python3
"""Run one encoder kernel repeatedly at the north-star shape (for rocprofv3 PMC passes).
   python tools/op_driver.py attn|gemm [iters]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "conformer-nemo_amd"))
import torch  # noqa: E402
from conformer_amd import _lib  # noqa: E402


def attn(iters):
    lib = _lib.load()
    B, T, H, dk = 32, 250, 8, 64
    g = torch.Generator().manual_seed(0)
    q, k, v = (torch.randn(B * T, H * dk, generator=g).to(torch.bfloat16).cuda() for _ in range(3))
    p = torch.randn(2 * T - 1, H * dk, generator=g).to(torch.bfloat16).cuda()
    u = torch.zeros(H, dk).cuda()
    lens = torch.full((B,), T, dtype=torch.int32).cuda()
    out = torch.empty(B * T, H * dk, dtype=torch.bfloat16, device="cuda")
    ws = torch.empty(lib.cfm_op_rel_attention_ws_size(1, B, T, H, dk), dtype=torch.uint8, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(iters):
        _lib.check(lib.cfm_op_rel_attention(1, q.data_ptr(), k.data_ptr(), v.data_ptr(), p.data_ptr(), u.data_ptr(),
                                            u.data_ptr(), lens.data_ptr(), B, T, H, dk, -1, -1, out.data_ptr(),
                                            ws.data_ptr(), st), "attn")
    torch.cuda.synchronize()


GEMM_SHAPES = {"ffn_up": (8000, 2048, 512, 2), "ffn_down": (8000, 512, 2048, 3), "qkv": (8000, 1536, 512, 6), "qkvs": (8000, 1536, 512, 0), "qkvs4k": (4000, 1536, 512, 0),
               "ffn_up4k": (4000, 2048, 512, 2), "ffn_down4k": (4000, 512, 2048, 3), "out4k": (4000, 512, 512, 3),
               "out": (8000, 512, 512, 3), "ffd_split2": (16000, 512, 1024, 4), "ffd_split4": (32000, 512, 512, 4),
               "ffd": (8000, 512, 2048, 4), "ref4096": (4096, 4096, 4096, 0), "conv2": (160000, 512, 4608, 0),
               "ref4096s": (4096, 4096, 4096, 2), "conv2s": (160000, 512, 4608, 2)}


def gemm(iters):
    """gemm [iters] [tile] [shape,shape...] — env-free tile choice for PMC passes."""
    lib = _lib.load()
    ms = ctypes.c_float(0)
    tile = int(sys.argv[3]) if len(sys.argv) > 3 else -1
    names = sys.argv[4].split(",") if len(sys.argv) > 4 else ["ffn_up", "ffn_down"]
    for name in names:
        M, N, K, epi = GEMM_SHAPES[name]
        _lib.check(lib.cfm_bench_gemm(1, tile, epi, M, N, K, iters, ctypes.byref(ms)), name)
        print(f"{name} tile {tile}: {ms.value * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    {"attn": attn, "gemm": gemm}[sys.argv[1]](int(sys.argv[2]) if len(sys.argv) > 2 else 10)
