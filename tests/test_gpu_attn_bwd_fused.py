"""The bf16 attention backward's fused score producer (attn_bwd.hip, attn_bwd_scores_kernel) at shapes
the golden fixtures do not reach: T' up to 512 (1-8 waves per block), head dims 16-128 (1-8 MFMA
k-slabs, including the odd count 3), padded utterances and a context window.

Reference: the same op in fp32 parity mode (materialised fp32 score images, fp32 MFMA) on the
bf16-rounded operands, itself pinned to the reference module's autograd by test_gpu_train_ops.py.
Gate: rel-L2 <= 2e-2 per gradient (bf16 GEMM operands), as the other bf16 backward tests.
"""
import ctypes

import numpy as np
import pytest
import torch

from conftest import rel_l2

pytestmark = pytest.mark.gpu

CASES = {   # B, T', H, dk, ctx_left, ctx_right
    "t250_dk64": (2, 250, 4, 64, -1, -1),
    "t300_dk48_window": (2, 300, 2, 48, 40, 7),
    "t511_dk128": (1, 511, 2, 128, -1, -1),
    "t64_dk16": (3, 64, 4, 16, -1, -1),
    "t33_dk32": (2, 33, 2, 32, 3, 3),
}


def _run(lib, dt, q, k, v, p, u, vb, lens, B, T, H, dk, cl, cr, dctx):
    from conformer_amd import _lib
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    d = H * dk
    M = B * T
    dq, dkey, dv = (torch.empty(M, d, device="cuda") for _ in range(3))
    dp = torch.empty(2 * T - 1, d, device="cuda")
    du, dvb = torch.empty(d, device="cuda"), torch.empty(d, device="cuda")
    n = lib.cfm_op_rel_attention_backward_ws_size(dt, B, T, H, dk)
    ws = torch.empty(n, dtype=torch.uint8, device="cuda")
    _lib.check(lib.cfm_op_rel_attention_backward(dt, q.data_ptr(), k.data_ptr(), v.data_ptr(), p.data_ptr(),
                                                 u.data_ptr(), vb.data_ptr(), lens.data_ptr(), B, T, H, dk, cl, cr,
                                                 dctx.data_ptr(), dq.data_ptr(), dkey.data_ptr(), dv.data_ptr(),
                                                 dp.data_ptr(), du.data_ptr(), dvb.data_ptr(), ws.data_ptr(), n, st),
               "rel_attention_backward")
    return dict(dq=dq, dk=dkey, dv=dv, dp=dp, du=du, dvb=dvb)


@pytest.mark.parametrize("case", sorted(CASES))
def test_fused_attention_backward_matches_fp32(case):
    from conformer_amd import _lib
    lib = _lib.load()
    B, T, H, dk, cl, cr = CASES[case]
    d = H * dk
    M = B * T
    g = torch.Generator().manual_seed(7)
    # bf16-representable operands so both modes see the same values
    q, k, v = (torch.randn(M, d, generator=g).bfloat16().float().cuda() for _ in range(3))
    p = torch.randn(2 * T - 1, d, generator=g).bfloat16().float().cuda()
    u, vb = (0.1 * torch.randn(d, generator=g)).cuda(), (0.1 * torch.randn(d, generator=g)).cuda()
    dctx = torch.randn(M, d, generator=g).cuda()
    lens = torch.tensor([T - (5 * b) % max(1, T // 3) for b in range(B)], dtype=torch.int32).cuda()
    ref = _run(lib, 0, q, k, v, p, u, vb, lens, B, T, H, dk, cl, cr, dctx)
    got = _run(lib, 1, q.bfloat16(), k.bfloat16(), v.bfloat16(), p.bfloat16(), u, vb, lens, B, T, H, dk, cl, cr, dctx)
    torch.cuda.synchronize()
    for name in ref:
        a, b = got[name].cpu().numpy(), ref[name].cpu().numpy()
        assert np.isfinite(a).all(), name
        e = rel_l2(a, b)
        assert e <= 2e-2, f"{case} {name}: relL2 {e:.3e}"
    # padded query rows and keys carry no gradient
    for b, L in enumerate(lens.tolist()):
        if L < T:
            assert float(got["dq"][b * T + L:(b + 1) * T].abs().max()) == 0.0
            assert float(got["dk"][b * T + L:(b + 1) * T].abs().max()) == 0.0
            assert float(got["dv"][b * T + L:(b + 1) * T].abs().max()) == 0.0


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
def test_attention_backward_t250_matches_reference(compute):
    """The attention backward at the BASELINE shape (T'=250, dk=64, 8 heads, padded second utterance)
    against the REFERENCE RelPositionMultiHeadAttention's float64 autograd (tests/golden/bwd_attn_t250.npz:
    identity projections, so its gradients are those of the attention core w.r.t. q, k, v, p).
    bf16 runs the fused score producer on bf16-rounded operands.  Gates: fp32 1e-3, bf16 2e-2."""
    import os
    from conftest import GOLDEN, summary_err
    from gen_large_goldens import attn_inputs
    from conformer_amd import _lib
    z = np.load(os.path.join(GOLDEN, "bwd_attn_t250.npz"))
    B, T, H = int(z["B"]), int(z["T"]), int(z["H"])
    d = 512
    dk = d // H
    q, k, v, p, dctx, u, vb = (torch.from_numpy(a) for a in attn_inputs(int(z["seed"]), B, T, d))
    lens = torch.from_numpy(z["lens"]).cuda()
    dt = 0 if compute == "fp32" else 1
    cast = (lambda t: t.cuda()) if compute == "fp32" else (lambda t: t.bfloat16().cuda())
    got = _run(_lib.load(), dt, cast(q), cast(k), cast(v), cast(p), u.cuda(), vb.cuda(), lens, B, T, H, dk, -1, -1,
               dctx.cuda())
    torch.cuda.synchronize()
    gate = 1e-3 if compute == "fp32" else 2e-2
    for name in ("dq", "dk", "dv", "dp"):
        es, en, ep = summary_err(name, got[name].cpu().numpy(), z, "ref__")
        assert es <= gate and en <= gate and ep <= 3 * gate, (name, es, en, ep)
    for name, key in (("du", "ref__du"), ("dvb", "ref__dvb")):
        assert rel_l2(got[name].cpu().numpy(), z[key]) <= gate, name
