"""BASELINE configurations 3, 4 and 5 at their stated workloads, on the GPU:

* cfg 4 — Conformer-Transducer-Large encoder (17 layers) at B=16, T=1600 with the reference's output
  for one T=1600 utterance embedded (tests/golden/full_large17_t1600.npz), then the RNN-T joint at
  U+1=101, V+1=1025 with log-softmax: rows normalised, one utterance against a torch fp32 restatement
  of RNNTJoint.joint (rnnt.py:951-1008) on the same device.
* cfg 5 — Conformer-XL (d 1024, 24 layers) at B=64 400-frame buffers with the reference's outputs for
  two buffers embedded (tests/golden/full_xl24_t400.npz).
* cfg 3 — the Conformer-CTC-Large training step at B=32, T=1000 (17 layers, yaml regularisation
  dropout 0.1 / dropout_att 0.1, CTC head V=256 + CTC loss): finite, and bitwise-reproducible loss,
  output and parameter gradients for a fixed seed.
Gates: fp32 relL2 <= 1e-3 (north star), bf16 <= 2e-2; batch independence bitwise.
"""
import functools
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, rel_l2, summary_err
from recipe import make_inputs, make_state_dict

pytestmark = pytest.mark.gpu
GATE = {"fp32": 1e-3, "bf16": 2e-2}


@functools.lru_cache(maxsize=2)
def _weights(cfg_json, seed):
    cfg = json.loads(cfg_json)
    return {k: torch.from_numpy(np.asarray(v)) for k, v in make_state_dict(cfg, seed).items()}


def _native(z, compute):
    from conformer_amd import NativeEncoder, make_cfg
    cfg = json.loads(str(z["cfg_json"]))
    enc = NativeEncoder(make_cfg(80, cfg["n_layers"], cfg["d_model"], n_heads=cfg["n_heads"]), compute=compute)
    enc.set_weights(_weights(str(z["cfg_json"]), int(z["seed"])))
    return enc


def _embedded_batch(z, B, slots, seed):
    T = int(z["T"])
    x, ln = make_inputs(B, T, 80, seed, [T] * B)
    xg, lg = make_inputs(int(z["B"]), T, 80, int(z["in_seed"]), [int(v) for v in z["lengths"]])
    for i, s in enumerate(slots):
        x[s], ln[s] = xg[i], lg[i]
    return torch.from_numpy(x).cuda(), torch.from_numpy(ln).to(torch.int32).cuda()


def _check_golden(y, slots, z, compute):
    for i, s in enumerate(slots):
        es, en, ep = summary_err(f"y{i}", y[s].cpu().numpy(), z, "out__")
        g = GATE[compute]
        assert es <= g and en <= g and ep <= 3 * g, (s, compute, es, en, ep)


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
def test_cfg4_encoder_b16_t1600(compute):
    z = np.load(os.path.join(GOLDEN, "full_large17_t1600.npz"))
    enc = _native(z, compute)
    slots = [9]
    x, ln = _embedded_batch(z, 16, slots, seed=77)
    y, yl = enc.forward(x, ln)
    torch.cuda.synchronize()
    assert y.shape == (16, 512, 400) and torch.isfinite(y).all()
    assert int(yl[9]) == int(z["y_len"][0])
    _check_golden(y, slots, z, compute)
    y1, _ = enc.forward(x[9:10].contiguous(), ln[9:10].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(y1[0], y[9])                          # batch independence, bitwise


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
def test_cfg4_joint_u100_v1024(compute):
    """RNNTJoint at the cfg-4 workload (B=16, T'=400, U+1=101, V+1=1025, log-softmax)."""
    from nemo.collections.asr.modules import RNNTJoint
    torch.manual_seed(4)
    j = RNNTJoint(jointnet=dict(encoder_hidden=512, pred_hidden=640, joint_hidden=640, activation="relu"),
                  num_classes=1024, log_softmax=True).cuda().eval()
    j.set_compute_mode(compute)
    g = torch.Generator(device="cuda").manual_seed(5)
    enc = torch.randn(16, 512, 400, device="cuda", generator=g)
    dec = torch.randn(16, 640, 101, device="cuda", generator=g)
    with torch.no_grad():
        lp = j(encoder_outputs=enc, decoder_outputs=dec)
        torch.cuda.synchronize()
        assert lp.shape == (16, 400, 101, 1025) and torch.isfinite(lp).all()
        s = torch.logsumexp(lp[::3].double(), -1)            # every 3rd utterance: rows normalised
        assert float(s.abs().max()) <= 1e-4
        # torch fp32 restatement of RNNTJoint.joint for utterance 7 (rnnt.py:951-1008)
        f = torch.nn.functional.linear(enc[7].t(), j.enc.weight, j.enc.bias)          # (T, H)
        gg = torch.nn.functional.linear(dec[7].t(), j.pred.weight, j.pred.bias)        # (U, H)
        h = torch.relu(f[:, None, :] + gg[None, :, :])
        out = j.joint_net[-1]
        ref = torch.log_softmax(torch.nn.functional.linear(h, out.weight, out.bias), dim=-1)
        e = rel_l2(lp[7].cpu().numpy(), ref.cpu().numpy())
    assert e <= (1e-5 if compute == "fp32" else 2e-2), e
    del lp


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
def test_cfg5_xl24_b64_buffers(compute):
    z = np.load(os.path.join(GOLDEN, "full_xl24_t400.npz"))
    enc = _native(z, compute)
    slots = [3, 60]
    x, ln = _embedded_batch(z, 64, slots, seed=78)
    y, yl = enc.forward(x, ln)
    torch.cuda.synchronize()
    assert y.shape == (64, 1024, 100) and torch.isfinite(y).all()
    np.testing.assert_array_equal(yl[slots].cpu().numpy(), z["y_len"])
    _check_golden(y, slots, z, compute)
    y1, _ = enc.forward(x[60:61].contiguous(), ln[60:61].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(y1[0], y[60])


def test_cfg3_training_step_b32_t1000_deterministic():
    """The bench's config-3 step (bf16, yaml regularisation) at full size: finite; the same seed gives
    bitwise-identical loss, output and every parameter gradient."""
    from nemo.collections.asr.losses import CTCLoss
    from nemo.collections.asr.modules import ConformerEncoder, ConvASRDecoder
    B, T, V, U = 32, 1000, 256, 60
    torch.manual_seed(0)
    enc = ConformerEncoder(feat_in=80, n_layers=17, d_model=512, n_heads=8, dropout=0.1, dropout_emb=0.0,
                           dropout_att=0.1).cuda().train()
    dec = ConvASRDecoder(feat_in=512, num_classes=V).cuda().train()
    loss_fn = CTCLoss(num_classes=V, zero_infinity=True, reduction="mean_batch")
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(B, 80, T, device="cuda", generator=g)
    lengths = torch.full((B,), T, dtype=torch.int64, device="cuda")
    lengths[1::4] = 731
    targets = torch.randint(0, V, (B, U), device="cuda", generator=g)
    tlen = torch.full((B,), U, dtype=torch.int64, device="cuda")
    params = [p for m in (enc, dec) for p in m.parameters()]
    runs = []
    for _ in range(2):
        for p in params:
            p.grad = None
        torch.manual_seed(1234)                               # -> the step's dropout seed
        y, yl = enc(audio_signal=x, length=lengths)
        loss = loss_fn(log_probs=dec(encoder_output=y), targets=targets, input_lengths=yl, target_lengths=tlen)
        loss.backward()
        torch.cuda.synchronize()
        runs.append((float(loss.detach()), y.detach().clone(), [p.grad.clone() for p in params]))
    assert np.isfinite(runs[0][0])
    assert runs[0][0] == runs[1][0]
    assert torch.equal(runs[0][1], runs[1][1])
    for a, b in zip(runs[0][2], runs[1][2]):
        assert torch.isfinite(a).all()
        assert torch.equal(a, b)


def test_cfg4_rnnt_training_step_b16_t1600_deterministic():
    """The Conformer-Transducer-Large training step at the cfg-4 workload: 17-layer
    encoder at B=16, T=1600 (T'=400) in training mode (dropout 0.1), the prediction net (pred_hidden 640,
    dropout 0.2) on U=100 labels, the joint (joint_hidden 640, relu, dropout 0.2) to raw logits
    (B, 400, 101, 1025) and the native RNN-T loss; loss.backward() runs the loss gradient, the joint
    backward, the prediction-net BPTT and the encoder backward.  Finite, and the same seed gives a
    bitwise-identical loss and every parameter gradient (conformer_transducer_bpe.yaml shapes)."""
    from nemo.collections.asr.losses import RNNTLoss
    from nemo.collections.asr.modules import ConformerEncoder, RNNTDecoder, RNNTJoint
    B, T, V, U = 16, 1600, 1024, 100
    torch.manual_seed(0)
    enc = ConformerEncoder(feat_in=80, n_layers=17, d_model=512, n_heads=8, subsampling_factor=4, dropout=0.1,
                           dropout_emb=0.0, dropout_att=0.1).cuda().train()
    dec = RNNTDecoder(prednet=dict(pred_hidden=640, pred_rnn_layers=1, dropout=0.2), vocab_size=V).cuda().train()
    joint = RNNTJoint(jointnet=dict(encoder_hidden=512, pred_hidden=640, joint_hidden=640, activation="relu",
                                    dropout=0.2), num_classes=V, log_softmax=False).cuda().train()
    loss_fn = RNNTLoss(num_classes=V, reduction="mean_batch")
    g = torch.Generator(device="cuda").manual_seed(12)
    x = torch.randn(B, 80, T, device="cuda", generator=g)
    lengths = torch.full((B,), T, dtype=torch.int64, device="cuda")
    lengths[1::4] = 1203
    y = torch.randint(0, V, (B, U), device="cuda", generator=g)
    ylen = torch.full((B,), U, dtype=torch.int64, device="cuda")
    ylen[2::4] = 71
    params = [p for m in (enc, dec, joint) for p in m.parameters()]
    runs = []
    for _ in range(2):
        for p in params:
            p.grad = None
        torch.manual_seed(4321)                               # -> every dropout seed of the step
        e, el = enc(audio_signal=x, length=lengths)
        d, _, _ = dec(targets=y, target_length=ylen)
        logits = joint(encoder_outputs=e, decoder_outputs=d)
        assert logits.shape == (B, 400, U + 1, V + 1)
        loss = loss_fn(log_probs=logits, targets=y, input_lengths=el, target_lengths=ylen)
        loss.backward()
        torch.cuda.synchronize()
        runs.append((float(loss.detach()), [p.grad.clone() for p in params]))
        del logits, e, d, loss
    assert np.isfinite(runs[0][0]) and runs[0][0] > 0
    assert runs[0][0] == runs[1][0]
    for p, a, b in zip(params, runs[0][1], runs[1][1]):
        assert torch.isfinite(a).all()
        assert torch.equal(a, b)
    assert all(float(a.abs().sum()) > 0 for a in runs[0][1][-8:])     # the decoder and joint receive gradient
