"""GPU parity of the backward building blocks (include/cfm_train.h) against the reference under
torch autograd (tests/golden/bwd_ffn.npz, from tests/golden/gen_bwd_goldens.py): the macaron FFN
sub-block x + 0.5 * FFN(LayerNorm(x)) of ConformerLayer, backward composed from the native ops.

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
    _lib.check(lib.cfm_op_swish_backward(_t(z["z"]).data_ptr(), du.data_ptr(), dzv.data_ptr(), du.numel(), _st()),
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
    _lib.check(lib.cfm_op_layernorm_backward(x.data_ptr(), M, d, _t(z["ln_w"]).data_ptr(), dhn.data_ptr(),
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
