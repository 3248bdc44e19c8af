"""GPU parity of the native RNN-T joint (include/cfm_joint.h) through the drop-in
`nemo.collections.asr.modules.RNNTJoint` against the reference's outputs (tests/golden/joint_*.npz).
Gates: fp32 compute rel-L2 <= 1e-5, bf16 operands rel-L2 <= 2e-2 (logits and log-probs)."""
import ast
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, rel_l2

pytestmark = pytest.mark.gpu
FILES = sorted(glob.glob(os.path.join(GOLDEN, "joint_*.npz")))
GATE = {"fp32": 1e-5, "bf16": 2e-2}


def _joint(z, compute):
    from nemo.collections.asr.modules import RNNTJoint
    jn = dict(ast.literal_eval(str(z["jointnet"])))
    j = RNNTJoint(jointnet=jn, num_classes=int(z["num_classes"]))
    j.load_state_dict({k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("p__")})
    j.set_compute_mode(compute)
    return j.cuda().eval()


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
def test_joint_matches_reference(path, compute):
    z = np.load(path)
    j = _joint(z, compute)
    enc = torch.from_numpy(z["enc"]).cuda()
    dec = torch.from_numpy(z["dec"]).cuda()
    with torch.no_grad():
        j.log_softmax = None            # on a GPU: logits (rnnt.py:998-1002)
        lo = j(encoder_outputs=enc, decoder_outputs=dec)
        j.log_softmax = True
        lp = j(encoder_outputs=enc, decoder_outputs=dec)
        j.log_softmax = False
        lo2 = j.joint(enc.transpose(1, 2), dec.transpose(1, 2))
    torch.cuda.synchronize()
    assert tuple(lo.shape) == z["logits"].shape
    assert rel_l2(lo.cpu().numpy(), z["logits"]) <= GATE[compute]
    assert rel_l2(lp.cpu().numpy(), z["logprobs"]) <= GATE[compute]
    assert rel_l2(lo2.cpu().numpy(), z["logits"]) <= GATE[compute]


def test_joint_large_shape_properties():
    """cfg-4-like shape (odd class count, B*T*U rows not a tile multiple): finite, log-probs normalised,
    and every (b, t, u) row independent of its neighbours (one utterance re-run alone is identical)."""
    from nemo.collections.asr.modules import RNNTJoint
    torch.manual_seed(0)
    j = RNNTJoint(jointnet=dict(encoder_hidden=512, pred_hidden=640, joint_hidden=640, activation="relu"),
                  num_classes=1024, log_softmax=True).cuda().eval()
    enc = torch.randn(3, 512, 37, device="cuda")
    dec = torch.randn(3, 640, 13, device="cuda")
    with torch.no_grad():
        lp = j(encoder_outputs=enc, decoder_outputs=dec)
        one = j(encoder_outputs=enc[1:2].contiguous(), decoder_outputs=dec[1:2].contiguous())
    assert lp.shape == (3, 37, 13, 1025) and torch.isfinite(lp).all()
    s = torch.logsumexp(lp.double(), -1)
    assert torch.allclose(s, torch.zeros_like(s), atol=1e-4)
    assert torch.equal(lp[1:2], one)


def test_joint_tail_columns_match_torch():
    """V + 1 = 1025 classes: the logits GEMM covers 1024 columns and the hidden kernel the last one
    (csrc/joint.hip, tail columns).  Against a torch fp32 restatement of RNNTJoint.joint (rnnt.py:951-1008)
    on the module's own weights: whole logits and the tail column alone within the bf16 gate."""
    from nemo.collections.asr.modules import RNNTJoint
    torch.manual_seed(1)
    j = RNNTJoint(jointnet=dict(encoder_hidden=64, pred_hidden=48, joint_hidden=64, activation="relu"),
                  num_classes=1024).cuda().eval()
    j.set_compute_mode("bf16")
    enc = torch.randn(2, 64, 19, device="cuda")
    dec = torch.randn(2, 48, 7, device="cuda")
    with torch.no_grad():
        j.log_softmax = None
        lo = j(encoder_outputs=enc, decoder_outputs=dec)
        out = j.joint_net[-1]
        f = enc.transpose(1, 2) @ j.enc.weight.t() + j.enc.bias
        g = dec.transpose(1, 2) @ j.pred.weight.t() + j.pred.bias
        hid = torch.relu(f[:, :, None, :] + g[:, None, :, :])
        ref = hid @ out.weight.t() + out.bias
    assert lo.shape == ref.shape == (2, 19, 7, 1025)
    assert rel_l2(lo.cpu().numpy(), ref.cpu().numpy()) <= GATE["bf16"]
    assert rel_l2(lo[..., 1024:].cpu().numpy(), ref[..., 1024:].cpu().numpy()) <= GATE["bf16"]
    assert rel_l2(lo[..., 1000:1024].cpu().numpy(), ref[..., 1000:1024].cpu().numpy()) <= GATE["bf16"]


def _native_pair(act, dims, seed):
    from conformer_amd.joint import NativeJoint
    H1, H2, H, C = dims
    g = torch.Generator().manual_seed(seed)
    w = [torch.randn(H, H1, generator=g) / H1 ** 0.5, torch.randn(H, generator=g) * 0.1,
         torch.randn(H, H2, generator=g) / H2 ** 0.5, torch.randn(H, generator=g) * 0.1,
         torch.randn(C, H, generator=g) / H ** 0.5, torch.randn(C, generator=g) * 0.1]
    j = NativeJoint(H1, H2, H, C, activation=act, compute="bf16")
    j.set_weights(*[t.cuda() for t in w])
    return j


@pytest.mark.parametrize("act", ["relu", "tanh", "sigmoid"])
@pytest.mark.parametrize("shape", [(2, 37, 13, 512, 640, 640, 1025), (1, 20, 101, 512, 640, 640, 1040),
                                   (3, 9, 5, 64, 48, 128, 512), (2, 16, 16, 512, 640, 640, 300)],
                         ids=["cfg4like", "u101_tail16", "small_no_tail", "unfused_c300"])
def test_joint_fused_logits_match_hidden_gemm_path(act, shape, monkeypatch):
    """The logits kernel that forms act(f' + g') in registers (csrc/joint.hip, joint_logits_kernel) against
    the hidden kernel + logits GEMM (CFM_JOINT_FUSED=0) on the same weights: the same bf16 hidden values
    and W, only the fp32 accumulation order differs (rel-L2 <= 1e-5). With joint_net's dropout (training)
    both settings run the hidden kernel + GEMM; the check there is that the masks are reproducible."""
    B, T, U, H1, H2, H, C = shape
    j = _native_pair(act, (H1, H2, H, C), 3)
    torch.manual_seed(4)
    enc = torch.randn(B, H1, T, device="cuda")
    dec = torch.randn(B, H2, U, device="cuda")
    outs = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("CFM_JOINT_FUSED", fused)
        outs[fused] = (j.forward(enc, dec), j.forward(enc, dec, log_softmax=True),
                       j.forward_train(enc, dec, 0.25, 1234))
    torch.cuda.synchronize()
    for a, b in zip(outs["1"], outs["0"]):
        assert a.shape == (B, T, U, C) and torch.isfinite(a).all()
        assert rel_l2(a.cpu().numpy(), b.cpu().numpy()) <= 1e-5
    # dropout zeroed some hidden units: the training logits differ from the eval ones
    assert not torch.equal(outs["1"][0], outs["1"][2])


def test_joint_fused_logits_full_lattice():
    """Config-4 lattice (T' = 400, U + 1 = 101, V + 1 = 1025, 4 utterances = 161600 rows x 1025): fused
    against the hidden kernel + GEMM path, rel-L2 over the whole tensor and per utterance."""
    j = _native_pair("relu", (512, 640, 640, 1025), 5)
    torch.manual_seed(6)
    enc = torch.randn(4, 512, 400, device="cuda")
    dec = torch.randn(4, 640, 101, device="cuda")
    os.environ["CFM_JOINT_FUSED"] = "1"
    try:
        a = j.forward(enc, dec).clone()
        os.environ["CFM_JOINT_FUSED"] = "0"
        b = j.forward(enc, dec)
    finally:
        os.environ.pop("CFM_JOINT_FUSED", None)
    torch.cuda.synchronize()
    for u in range(4):
        d = (a[u].double() - b[u].double()).norm() / b[u].double().norm()
        assert float(d) <= 1e-5
    assert float((a[..., 1024] - b[..., 1024]).abs().max()) <= 1e-3


@pytest.mark.parametrize("act", ["relu", "tanh"])
@pytest.mark.parametrize("dims", [(2, 37, 13, 64, 48, 128, 300), (1, 40, 101, 512, 640, 640, 1025)],
                         ids=["ragged_t", "cfg4_u101"])
def test_joint_act_backward_one_pass_matches_two_pass(act, dims, monkeypatch):
    """joint_act_bwd_tu_kernel (one pass over dh: df per frame, dp as 16-frame tile partials + an ordered tile
    sum) against the two reduction kernels (CFM_JOINT_ACT_FUSED=0), same dropout masks: every gradient of
    cfm_rnnt_joint_backward. df and everything derived from it (d_enc, dW_enc, db_enc) and the output layer's
    gradients within rel-L2 1e-6; dp's fp32 sum over the frames runs in another order (tile partials), and with
    random dlogits it cancels heavily, so d_dec, dW_pred, db_pred within 1e-4."""
    B, T, U, H1, H2, H, C = dims
    j = _native_pair(act, (H1, H2, H, C), 7)
    g = torch.Generator().manual_seed(8)
    w_enc, w_pred, w_out = (torch.randn(H, H1, generator=g).cuda() / H1 ** 0.5,
                            torch.randn(H, H2, generator=g).cuda() / H2 ** 0.5, torch.randn(C, H, generator=g).cuda() / H ** 0.5)
    j.set_weights(w_enc, None, w_pred, None, w_out, None)
    torch.manual_seed(9)
    enc = torch.randn(B, H1, T, device="cuda")
    dec = torch.randn(B, H2, U, device="cuda")
    dl = torch.randn(B, T, U, C, device="cuda") * 1e-3
    res = {}
    for v in ("1", "0"):
        monkeypatch.setenv("CFM_JOINT_ACT_FUSED", v)
        res[v] = j.backward(enc, dec, dl, 0.2, 4321, w_enc, w_pred, w_out, (True,) * 8)
    torch.cuda.synchronize()
    for k, (a, b) in enumerate(zip(res["1"], res["0"])):
        assert torch.isfinite(a).all()
        assert rel_l2(a.cpu().numpy(), b.cpu().numpy()) <= (1e-4 if k in (1, 4, 5) else 1e-6), k
