"""GPU parity of the CTC head and CTC loss (include/cfm_ctc.h) against the reference
(tests/golden/ctc_*.npz from tests/golden/gen_ctc_goldens.py) and the oracle.

Gates: fp32 compute mode rel-L2 <= 1e-4 on log-probs and head gradients (fp32 arithmetic vs the
float64 reference), losses rtol 1e-4; bf16 compute mode (head GEMMs on bf16 operands) rel-L2
<= 2e-2; greedy predictions exact in fp32 mode.  The CTC loss kernel is fp32 in both modes; its
gradient gate is rel-L2 <= 1e-3 (the north-star fp32 tolerance): the posterior exponent
lcab + nll - lp sums log-space terms of magnitude ~1e3 at T' = 250, whose fp32 spacing is ~1e-4.
"""
import glob
import os

import numpy as np
import pytest
import torch

import ctc_oracle as CO
from conftest import GOLDEN, rel_l2

pytestmark = pytest.mark.gpu
CASES = sorted(glob.glob(os.path.join(GOLDEN, "ctc_*.npz")))
GATE = {"fp32": 1e-4, "bf16": 2e-2}


def _t(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return t if dtype is None else t.to(dtype)


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(p)[:-4] for p in CASES])
def test_head_forward_backward(path, compute):
    from conformer_amd.ctc import NativeCtcHead
    z = np.load(path)
    C, D = z["w"].shape[0], z["w"].shape[1]
    head = NativeCtcHead(D, C, compute=compute)
    head.set_weights(_t(z["w"]), _t(z["b"]))
    lp, greedy = head.forward(_t(z["enc"]))
    torch.cuda.synchronize()
    lp = lp.cpu().numpy()
    assert rel_l2(lp, z["log_probs"]) <= GATE[compute]
    if compute == "fp32":
        np.testing.assert_array_equal(greedy.cpu().numpy(), z["greedy"])
    genc, gw, gb = head.backward(_t(z["enc"]), _t(z["log_probs"]), _t(z["grad_lp"]))
    torch.cuda.synchronize()
    assert rel_l2(genc.cpu().numpy(), z["grad_enc"]) <= GATE[compute]
    assert rel_l2(gw.cpu().numpy(), z["grad_w"]) <= GATE[compute]
    assert rel_l2(gb.cpu().numpy(), z["grad_b"]) <= GATE["fp32"]     # column sums are fp32 in both modes


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(p)[:-4] for p in CASES])
def test_ctc_loss_matches_reference(path):
    from conformer_amd.ctc import ctc_loss
    z = np.load(path)
    B = z["log_probs"].shape[0]
    nll, grad = ctc_loss(_t(z["log_probs"]), _t(z["targets"]), _t(z["in_len"]), _t(z["tgt_len"]), int(z["blank"]),
                         True, grad_scale=1.0 / B)
    torch.cuda.synchronize()
    np.testing.assert_allclose(nll.cpu().numpy(), z["nll"], rtol=1e-4, atol=1e-3)
    assert rel_l2(grad.cpu().numpy(), z["grad_lp"]) <= 1e-3
    # deterministic
    nll2, grad2 = ctc_loss(_t(z["log_probs"]), _t(z["targets"]), _t(z["in_len"]), _t(z["tgt_len"]),
                           int(z["blank"]), True, grad_scale=1.0 / B)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(grad.cpu().numpy(), grad2.cpu().numpy())


def test_ctc_loss_long_targets_vs_oracle():
    """2U+1 up to 1023 extended states (SPL 16) and T' = 400 (cfg 4 length) against the oracle."""
    from conformer_amd.ctc import ctc_loss
    g = np.random.default_rng(5)
    B, T, C, U = 2, 400, 40, 300
    lp = CO.log_softmax(g.standard_normal((B, T, C)))
    tg = g.integers(0, C - 1, (B, U)).astype(np.int32)
    il, tl = np.array([400, 380], np.int32), np.array([300, 150], np.int32)
    nll, grad = ctc_loss(_t(lp.astype(np.float32)), _t(tg), _t(il), _t(tl), C - 1, True)
    rn, rg = CO.ctc_loss(lp.astype(np.float32), tg, il, tl, C - 1)
    torch.cuda.synchronize()
    np.testing.assert_allclose(nll.cpu().numpy(), rn, rtol=1e-4)
    assert rel_l2(grad.cpu().numpy(), rg) <= 1e-3


def test_dropin_decoder_and_loss_modules():
    """The nemo-path plugins: ConvASRDecoder + CTCLoss(mean_batch, zero_infinity) with autograd."""
    from nemo.collections.asr.losses import CTCLoss
    from nemo.collections.asr.modules import ConvASRDecoder
    z = np.load(os.path.join(GOLDEN, "ctc_small.npz"))
    C, D = z["w"].shape[0], z["w"].shape[1]
    dec = ConvASRDecoder(feat_in=D, num_classes=C - 1).cuda()
    assert dec.num_classes_with_blank == C
    dec.load_state_dict({"decoder_layers.0.weight": torch.from_numpy(z["w"]),
                         "decoder_layers.0.bias": torch.from_numpy(z["b"])})
    dec.set_compute_mode("fp32")
    enc = _t(z["enc"]).requires_grad_(True)
    with pytest.raises(TypeError):
        dec(enc)
    lp = dec(encoder_output=enc)
    loss_fn = CTCLoss(num_classes=C - 1, zero_infinity=True, reduction="mean_batch")
    loss = loss_fn(log_probs=lp, targets=_t(z["targets"]), input_lengths=_t(z["in_len"]),
                   target_lengths=_t(z["tgt_len"]))
    loss.backward()
    assert abs(loss.item() - float(z["loss"])) <= 1e-4 * abs(float(z["loss"]))
    assert rel_l2(enc.grad.cpu().numpy(), z["grad_enc"]) <= 1e-4
    assert rel_l2(dec.decoder_layers[0].weight.grad.cpu().numpy()[:, :, 0], z["grad_w"]) <= 1e-4
    assert rel_l2(dec.decoder_layers[0].bias.grad.cpu().numpy(), z["grad_b"]) <= 1e-4


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(p)[:-4] for p in CASES])
def test_ctc_loss_concatenated_targets(path):
    """torch's 1-D target form (utterances' labels concatenated, length sum(target_lengths)) gives
    the same losses and gradients as the padded (B, U) form (no silent reshape)."""
    from conformer_amd.ctc import ctc_loss
    z = np.load(path)
    tg, tl = z["targets"], z["tgt_len"]
    flat = np.concatenate([tg[b, :tl[b]] for b in range(tg.shape[0])]).astype(tg.dtype)
    args = (_t(z["in_len"]), _t(tl), int(z["blank"]), True)
    nll, grad = ctc_loss(_t(z["log_probs"]), _t(tg), *args)
    nll1, grad1 = ctc_loss(_t(z["log_probs"]), _t(flat), *args)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(nll.cpu().numpy(), nll1.cpu().numpy())
    np.testing.assert_array_equal(grad.cpu().numpy(), grad1.cpu().numpy())
    with pytest.raises(ValueError):
        ctc_loss(_t(z["log_probs"]), _t(flat[:-1]), *args)
