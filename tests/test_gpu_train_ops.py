"""GPU parity of the backward building blocks (include/cfm_train.h) against the reference modules
under torch autograd, composed from the native ops:
  * bwd_ffn.npz  (gen_bwd_goldens.py): macaron FFN sub-block x + 0.5 * FFN(LayerNorm(x));
  * bwd_conv.npz (gen_conv_bwd_goldens.py): ConformerConvolution in training mode;
  * bwd_attn.npz (gen_attn_bwd_goldens.py): RelPositionMultiHeadAttention, full and windowed context.

Gates: fp32 GEMM operands rel-L2 <= 1e-4 per gradient; bf16 operands rel-L2 <= 2e-2.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, rel_l2

pytestmark = pytest.mark.gpu
GATE = {"fp32": 1e-4, "bf16": 2e-2}
DT = {"fp32": 0, "bf16": 1}


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()


def _st():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def linear_backward(lib, dt, x, w, dy):
    from conformer_amd import _lib
    M, K = x.shape
    N = w.shape[0]
    dx, dw, db = torch.empty_like(x), torch.empty_like(w), torch.empty(N, device="cuda")
    n = lib.cfm_op_linear_backward_ws_size(dt, M, K, N)
    ws = torch.empty(n, dtype=torch.uint8, device="cuda")
    _lib.check(lib.cfm_op_linear_backward(dt, x.data_ptr(), M, K, w.data_ptr(), N, dy.data_ptr(), dx.data_ptr(),
                                          dw.data_ptr(), db.data_ptr(), ws.data_ptr(), n, _st()), "linear_backward")
    return dx, dw, db


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
def test_ffn_block_backward(compute):
    from conformer_amd import _lib
    lib = _lib.load()
    z = np.load(os.path.join(GOLDEN, "bwd_ffn.npz"))
    dt = DT[compute]
    fc = float(z["fc_factor"])
    dy_ffn = _t(z["dout"] * fc)
    # linear2: y = u W2^T + b2
    du, dw2, db2 = linear_backward(lib, dt, _t(z["u"]), _t(z["w2"]), dy_ffn)
    # Swish
    dzv = torch.empty_like(du)
    zz = _t(z["z"])
    _lib.check(lib.cfm_op_swish_backward(zz.data_ptr(), du.data_ptr(), dzv.data_ptr(), du.numel(), _st()),
               "swish_backward")
    # linear1
    dhn, dw1, db1 = linear_backward(lib, dt, _t(z["hn"]), _t(z["w1"]), dzv)
    # LayerNorm, accumulated onto the residual-stream gradient dout
    x = _t(z["x"])
    M, d = x.shape
    dx = _t(z["dout"])
    dlnw, dlnb = torch.empty(d, device="cuda"), torch.empty(d, device="cuda")
    n = lib.cfm_op_layernorm_backward_ws_size(M, d)
    ws = torch.empty(n, dtype=torch.uint8, device="cuda")
    ln_w = _t(z["ln_w"])    # keep every tensor whose pointer is passed alive across the call
    _lib.check(lib.cfm_op_layernorm_backward(x.data_ptr(), M, d, ln_w.data_ptr(), dhn.data_ptr(),
                                             dx.data_ptr(), 1, dlnw.data_ptr(), dlnb.data_ptr(), ws.data_ptr(), n,
                                             _st()), "layernorm_backward")
    torch.cuda.synchronize()
    g = GATE[compute]
    for name, got in [("d_u", du), ("d_w2", dw2), ("d_b2", db2), ("d_z", dzv), ("d_hn", dhn), ("d_w1", dw1),
                      ("d_b1", db1), ("d_x", dx), ("d_ln_w", dlnw), ("d_ln_b", dlnb)]:
        e = rel_l2(got.cpu().numpy(), z[name])
        assert e <= g, f"{name}: relL2 {e:.3e} > {g}"


def test_linear_backward_deterministic_ragged():
    """M not a multiple of any tile, K/N odd multiples of 4: bitwise-repeatable gradients."""
    from conformer_amd import _lib
    lib = _lib.load()
    g = np.random.default_rng(1)
    x, w, dy = _t(g.standard_normal((1001, 52))), _t(g.standard_normal((300, 52))), _t(g.standard_normal((1001, 300)))
    a = [t.cpu().numpy() for t in linear_backward(lib, 0, x, w, dy)]
    b = [t.cpu().numpy() for t in linear_backward(lib, 0, x, w, dy)]
    for u, v in zip(a, b):
        np.testing.assert_array_equal(u, v)
    xd, wd, dyd = (t.double().cpu() for t in (x, w, dy))
    assert rel_l2(a[0], (dyd @ wd).numpy()) <= 1e-5
    assert rel_l2(a[1], (dyd.T @ xd).numpy()) <= 1e-5
    assert rel_l2(a[2], dyd.sum(0).numpy()) <= 1e-5


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
def test_conv_module_backward(compute):
    """ConformerConvolution in training mode (tests/golden/bwd_conv.npz): BatchNorm batch statistics
    and running-stat update, then the whole backward chain pw2 -> Swish -> BN -> depthwise -> GLU+mask
    -> pw1 from the native ops."""
    from conformer_amd import _lib
    lib = _lib.load()
    z = np.load(os.path.join(GOLDEN, "bwd_conv.npz"))
    dt = DT[compute]
    g = GATE[compute]
    B, T = int(z["B"]), int(z["T"])
    M, d = z["x"].shape
    # BatchNorm forward (train) on the depthwise output
    h = _t(z["h"])
    y, xhat = torch.empty_like(h), torch.empty_like(h)
    mean, rstd = torch.empty(d, device="cuda"), torch.empty(d, device="cuda")
    rm, rv = _t(z["bn_rm0"]), _t(z["bn_rv0"])
    n = lib.cfm_op_batchnorm_train_ws_size(M, d)
    ws = torch.empty(n, dtype=torch.uint8, device="cuda")
    bn_w, bn_b = _t(z["bn_w"]), _t(z["bn_b"])
    _lib.check(lib.cfm_op_batchnorm_train_forward(h.data_ptr(), M, d, bn_w.data_ptr(),
                                                  bn_b.data_ptr(), float(z["bn_momentum"]), rm.data_ptr(),
                                                  rv.data_ptr(), y.data_ptr(), xhat.data_ptr(), mean.data_ptr(),
                                                  rstd.data_ptr(), ws.data_ptr(), n, _st()), "bn_forward")
    torch.cuda.synchronize()
    assert rel_l2(y.cpu().numpy(), z["bn"]) <= 1e-5
    assert rel_l2(rm.cpu().numpy(), z["bn_rm1"]) <= 1e-5 and rel_l2(rv.cpu().numpy(), z["bn_rv1"]) <= 1e-5
    # backward chain
    bn = z["bn"].astype(np.float64)
    s = (bn / (1.0 + np.exp(-bn))).astype(np.float32)
    ds, dw2, db2 = linear_backward(lib, dt, _t(s), _t(z["pw2_w"]), _t(z["dout"]))
    dbn = torch.empty_like(ds)
    bn_t = _t(z["bn"])
    _lib.check(lib.cfm_op_swish_backward(bn_t.data_ptr(), ds.data_ptr(), dbn.data_ptr(), dbn.numel(), _st()),
               "swish_backward")
    dh, dgam, dbet = torch.empty_like(dbn), torch.empty(d, device="cuda"), torch.empty(d, device="cuda")
    _lib.check(lib.cfm_op_batchnorm_train_backward(dbn.data_ptr(), xhat.data_ptr(), M, d, bn_w.data_ptr(),
                                                   rstd.data_ptr(), dh.data_ptr(), dgam.data_ptr(), dbet.data_ptr(),
                                                   ws.data_ptr(), n, _st()), "bn_backward")
    dglu, ddw, ddb = torch.empty_like(dh), torch.empty(d, 1, 31, device="cuda"), torch.empty(d, device="cuda")
    n2 = lib.cfm_op_dwconv_backward_ws_size(B, T, d, 31)
    ws2 = torch.empty(n2, dtype=torch.uint8, device="cuda")
    glu_t, dw_w = _t(z["glu"]), _t(z["dw_w"])
    _lib.check(lib.cfm_op_dwconv_backward(glu_t.data_ptr(), dw_w.data_ptr(), dh.data_ptr(), B, T, d,
                                          31, dglu.data_ptr(), ddw.data_ptr(), ddb.data_ptr(), ws2.data_ptr(), n2,
                                          _st()), "dwconv_backward")
    dpre = torch.empty(M, 2 * d, device="cuda")
    lens = torch.from_numpy(z["lens"]).cuda()
    pre_t = _t(z["pre"])
    _lib.check(lib.cfm_op_glu_backward(pre_t.data_ptr(), dglu.data_ptr(), lens.data_ptr(), B, T, d,
                                       dpre.data_ptr(), _st()), "glu_backward")
    dx, dw1, db1 = linear_backward(lib, dt, _t(z["x"]), _t(z["pw1_w"]), dpre)
    torch.cuda.synchronize()
    for name, got, gate in [("d_pw2_w", dw2, g), ("d_pw2_b", db2, 1e-4), ("d_bn", dbn, g), ("d_h", dh, g),
                            ("d_bn_w", dgam, g), ("d_bn_b", dbet, g), ("d_dw_w", ddw, g),
                            ("d_pre", dpre, g), ("d_x", dx, g), ("d_pw1_w", dw1, g), ("d_pw1_b", db1, g)]:
        e = rel_l2(got.cpu().numpy(), z[name])
        assert e <= gate, f"{name}: relL2 {e:.3e} > {gate}"
    # d_dw_b = sum_t d_h, and train-mode BatchNorm makes every column of d_h sum to zero: the golden is
    # rounding noise (~1e-6), so relL2 on it is meaningless.  Check it is the column sum of our d_h
    # (fp32 accumulation bound), and that both sides are at noise level against |d_h|.
    dh64 = dh.double().cpu().numpy()
    scale = np.sqrt(M) * np.sqrt((dh64 ** 2).mean(0)).max()
    np.testing.assert_allclose(ddb.cpu().numpy(), dh64.sum(0), rtol=0, atol=1e-5 * scale)
    assert np.abs(z["d_dw_b"]).max() <= 1e-4 * scale and np.abs(ddb.cpu().numpy()).max() <= 1e-4 * scale


@pytest.mark.parametrize("case", ["full", "ctx"])
@pytest.mark.parametrize("compute", ["fp32", "bf16"])
def test_rel_attention_backward(compute, case):
    """RelPositionMultiHeadAttention backward (tests/golden/bwd_attn.npz, the reference module under
    float64 autograd with the encoder's pad / context-window mask): the native attention backward,
    then the projections' backward (linear_q/k/v into d_x, linear_pos weight) from linear_backward."""
    from conformer_amd import _lib
    lib = _lib.load()
    z = {k.split(".", 1)[1]: v for k, v in np.load(os.path.join(GOLDEN, "bwd_attn.npz")).items()
         if k.startswith(case + ".")}
    dt = DT[compute]
    g = GATE[compute]
    B, T, H = int(z["B"]), int(z["T"]), int(z["H"])
    M, d = z["q"].shape
    dk = d // H
    ct = torch.float32 if compute == "fp32" else torch.bfloat16
    q, k, v, p = (_t(z[n]).to(ct).contiguous() for n in ("q", "k", "v", "p"))
    u, vb, dctx = _t(z["u"]), _t(z["vb"]), _t(z["d_ctx"])
    lens = torch.from_numpy(z["lens"]).cuda()
    cl, cr = int(z["ctx_left"]), int(z["ctx_right"])
    # forward context first (same operands, checks the window mask)
    ctx = torch.empty(M, d, dtype=ct, device="cuda")
    wsf = torch.empty(lib.cfm_op_rel_attention_ws_size(dt, B, T, H, dk), dtype=torch.uint8, device="cuda")
    _lib.check(lib.cfm_op_rel_attention(dt, q.data_ptr(), k.data_ptr(), v.data_ptr(), p.data_ptr(), u.data_ptr(),
                                        vb.data_ptr(), lens.data_ptr(), B, T, H, dk, cl, cr, ctx.data_ptr(),
                                        wsf.data_ptr(), _st()), "rel_attention")
    dq, dkey, dv = (torch.empty(M, d, device="cuda") for _ in range(3))
    dp = torch.empty(2 * T - 1, d, device="cuda")
    du, dvb = torch.empty(d, device="cuda"), torch.empty(d, device="cuda")
    n = lib.cfm_op_rel_attention_backward_ws_size(dt, B, T, H, dk)
    ws = torch.empty(n, dtype=torch.uint8, device="cuda")
    _lib.check(lib.cfm_op_rel_attention_backward(dt, q.data_ptr(), k.data_ptr(), v.data_ptr(), p.data_ptr(),
                                                 u.data_ptr(), vb.data_ptr(), lens.data_ptr(), B, T, H, dk, cl, cr,
                                                 dctx.data_ptr(), dq.data_ptr(), dkey.data_ptr(), dv.data_ptr(),
                                                 dp.data_ptr(), du.data_ptr(), dvb.data_ptr(), ws.data_ptr(), n,
                                                 _st()), "rel_attention_backward")
    # projections: d_x = dq W_q + dk W_k + dv W_v ; d W_pos = dp^T pos_emb
    x = _t(z["x"])
    dxq, dwq, dbq = linear_backward(lib, dt, x, _t(z["w_q"]), dq)
    dxk, _, _ = linear_backward(lib, dt, x, _t(z["w_k"]), dkey)
    dxv, _, _ = linear_backward(lib, dt, x, _t(z["w_v"]), dv)
    _, dwpos, _ = linear_backward(lib, dt, _t(z["pos_emb"]), _t(z["w_pos"]), dp)
    torch.cuda.synchronize()
    fwd_gate = 1e-5 if compute == "fp32" else 2e-2
    assert rel_l2(ctx.float().cpu().numpy(), z["ctx"]) <= fwd_gate
    for name, got in [("d_q", dq), ("d_k", dkey), ("d_v", dv), ("d_p", dp), ("d_u", du), ("d_vb", dvb),
                      ("d_w_q", dwq), ("d_b_q", dbq), ("d_x", dxq + dxk + dxv), ("d_w_pos", dwpos)]:
        e = rel_l2(got.cpu().numpy(), z[name])
        assert e <= g, f"{name}: relL2 {e:.3e} > {g}"
    # padded query rows / keys carry no gradient
    for b, L in enumerate(z["lens"]):
        assert float(dq[b * T + L:(b + 1) * T].abs().max() if L < T else 0) == 0.0
        assert float(dkey[b * T + L:(b + 1) * T].abs().max() if L < T else 0) == 0.0
