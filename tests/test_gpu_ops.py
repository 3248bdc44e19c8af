"""Per-kernel GPU parity through the kernel-level C-ABI entry points (include/cfm_encoder.h):
LayerNorm, the MFMA GEMM (+ activations) and the fused relative-position attention core.
References: the oracle's functions (numpy, float64) on the same inputs."""
import ctypes

import numpy as np
import pytest
import torch

import conformer_oracle as O
from conftest import max_rel, rel_l2

pytestmark = pytest.mark.gpu

DT = {"fp32": (0, torch.float32), "bf16": (1, torch.bfloat16)}
TOL = {"fp32": 2e-5, "bf16": 1.5e-2}


def lib():
    from conformer_amd import _lib
    return _lib.load()


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def chk(st):
    from conformer_amd import _lib
    _lib.check(st, "op")


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
@pytest.mark.parametrize("rows,d", [(1, 64), (37, 176), (300, 512), (64, 1024), (5, 40)])
def test_layernorm(compute, rows, d):
    mode, tdt = DT[compute]
    g = torch.Generator().manual_seed(rows * 7 + d)
    x = (torch.randn(rows, d, generator=g) * 3 + 1).cuda()
    w = (torch.rand(d, generator=g) + 0.5).cuda()
    b = torch.randn(d, generator=g).cuda()
    yf = torch.empty(rows, d, device="cuda")
    yt = torch.empty(rows, d, device="cuda", dtype=tdt)
    chk(lib().cfm_op_layernorm(mode, x.data_ptr(), rows, d, w.data_ptr(), b.data_ptr(), yf.data_ptr(), yt.data_ptr(),
                               stream()))
    ref = O.layer_norm(x.cpu().double().numpy(), w.cpu().double().numpy(), b.cpu().double().numpy())
    assert rel_l2(yf.cpu().numpy(), ref) < 1e-6
    assert rel_l2(yt.float().cpu().numpy(), ref) < (1e-6 if compute == "fp32" else 5e-3)


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
@pytest.mark.parametrize("M,K,N,act", [(1, 64, 1, 0), (100, 80, 50, 1), (257, 512, 300, 2), (8000, 512, 2048, 2),
                                       (333, 2048, 512, 0), (130, 3520, 176, 0)])
def test_linear(compute, M, K, N, act):
    mode, tdt = DT[compute]
    g = torch.Generator().manual_seed(M + K + N)
    x = torch.randn(M, K, generator=g).to(tdt).cuda()
    w = (torch.randn(N, K, generator=g) / K ** 0.5).cuda()
    b = torch.randn(N, generator=g).cuda()
    y = torch.full((M, N), float("nan"), device="cuda", dtype=tdt)
    need = ctypes.c_size_t(0)
    chk(lib().cfm_op_linear(mode, x.data_ptr(), M, K, w.data_ptr(), b.data_ptr(), N, act, y.data_ptr(), None,
                            ctypes.byref(need), stream()))
    ws = torch.empty(need.value, dtype=torch.uint8, device="cuda")
    chk(lib().cfm_op_linear(mode, x.data_ptr(), M, K, w.data_ptr(), b.data_ptr(), N, act, y.data_ptr(), ws.data_ptr(),
                            ctypes.byref(need), stream()))
    torch.cuda.synchronize()
    wq = w.to(tdt).double().cpu().numpy()
    ref = x.double().cpu().numpy() @ wq.T + b.double().cpu().numpy()
    if act == 1:
        ref = np.maximum(ref, 0)
    elif act == 2:
        ref = O.swish(ref)
    out = y.float().cpu().numpy()
    assert np.isfinite(out).all()
    assert rel_l2(out, ref) < TOL[compute]


def attention_core_ref(q, k, v, p, u, vb, lens, ctx):
    """(q+u)k^T + rel_shift((q+v)p^T) / sqrt(dk), masked softmax, P.V — the arithmetic of
    multi_head_attention.py:183-210 / 94-115 after the projections (float64)."""
    B, T, H, dk = q.shape
    qh = q.transpose(0, 2, 1, 3)
    kh = k.transpose(0, 2, 1, 3)
    vh = v.transpose(0, 2, 1, 3)
    ph = p.reshape(1, 2 * T - 1, H, dk).transpose(0, 2, 1, 3)
    ac = (qh + u[None, :, None, :]) @ kh.transpose(0, 1, 3, 2)
    bd = (qh + vb[None, :, None, :]) @ ph.transpose(0, 1, 3, 2)
    bd = O.rel_shift(bd)[..., :T]
    s = (ac + bd) / np.sqrt(dk)
    _, att = O.make_masks(T, lens, ctx)
    m = att[:, None]
    s = np.where(m, -10000.0, s)
    e = np.exp(s - s.max(-1, keepdims=True))
    a = np.where(m, 0.0, e / e.sum(-1, keepdims=True))
    return (a @ vh).transpose(0, 2, 1, 3).reshape(B, T, H * dk)


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
@pytest.mark.parametrize("B,T,H,dk,ctx", [(2, 16, 4, 16, (-1, -1)), (3, 50, 4, 44, (-1, -1)), (2, 77, 8, 22, (-1, -1)),
                                          (2, 250, 8, 64, (-1, -1)), (1, 100, 8, 128, (-1, -1)),
                                          (2, 40, 4, 10, (-1, -1)), (2, 64, 4, 16, (4, 2)), (2, 70, 2, 32, (-1, 0))])
def test_rel_attention(compute, B, T, H, dk, ctx):
    mode, tdt = DT[compute]
    g = torch.Generator().manual_seed(B * 1000 + T + dk)
    d = H * dk
    q = torch.randn(B * T, d, generator=g).to(tdt)
    k = torch.randn(B * T, d, generator=g).to(tdt)
    v = torch.randn(B * T, d, generator=g).to(tdt)
    p = torch.randn(2 * T - 1, d, generator=g).to(tdt)
    u = torch.randn(H, dk, generator=g) * 0.3
    vb = torch.randn(H, dk, generator=g) * 0.3
    lens = torch.tensor([T] + [max(1, T * (i + 2) // (i + 4)) for i in range(B - 1)], dtype=torch.int32)
    out = torch.full((B * T, d), float("nan"), dtype=tdt, device="cuda")
    L = lib()
    ws = torch.empty(L.cfm_op_rel_attention_ws_size(mode, B, T, H, dk), dtype=torch.uint8, device="cuda")
    qc, kc, vc, pc, uc, vbc, lc = (t.cuda() for t in (q, k, v, p, u, vb, lens))
    chk(L.cfm_op_rel_attention(mode, qc.data_ptr(), kc.data_ptr(), vc.data_ptr(), pc.data_ptr(), uc.data_ptr(),
                               vbc.data_ptr(), lc.data_ptr(), B, T, H, dk, ctx[0], ctx[1], out.data_ptr(),
                               ws.data_ptr(), stream()))
    torch.cuda.synchronize()
    f = lambda t: t.double().numpy()
    ref = attention_core_ref(f(q).reshape(B, T, H, dk), f(k).reshape(B, T, H, dk), f(v).reshape(B, T, H, dk), f(p),
                             f(u), f(vb), lens.numpy(), ctx)
    got = out.float().cpu().numpy().reshape(B, T, d)
    assert np.isfinite(got).all()
    # padded query rows are exactly zero (multi_head_attention.py:107)
    for b in range(B):
        assert (got[b, int(lens[b]):] == 0).all()
    tol = 1e-5 if compute == "fp32" else 2e-2
    assert rel_l2(got, ref) < tol, rel_l2(got, ref)
