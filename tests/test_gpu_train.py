"""GPU parity of the whole-encoder training step (include/cfm_train.h) against the REFERENCE
ConformerEncoder in training mode under torch autograd (tests/golden/train_*.npz, written by
gen_train_goldens.py): encoder output, every parameter gradient (loss = sum(y * R)) and the
BatchNorm running statistics after one step, through the drop-in module in `.train()` mode.

Gates: fp32 compute mode rel-L2 <= 1e-3 on the output and on every gradient (the north-star fp32
tolerance); bf16 operands rel-L2 <= 2e-2 on the output and <= 6e-2 per gradient (bf16 GEMM
operands through two layers of backward).  Gradients are compared relative to
max(|ref|, 1e-2 x the step's largest gradient norm).
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, rel_l2

pytestmark = pytest.mark.gpu
CASES = ["train_tiny", "train_tiny_dk10", "train_tiny_ctx", "train_tiny_nopad", "train_tiny_abspos"]
GATE_Y = {"fp32": 1e-3, "bf16": 2e-2}
GATE_G = {"fp32": 1e-3, "bf16": 6e-2}


def _encoder(z, compute, dropout=0.0):
    from nemo.collections.asr.modules import ConformerEncoder
    from recipe import make_state_dict
    cfg = json.loads(str(z["cfg_json"]))
    enc = ConformerEncoder(**cfg, dropout=dropout, dropout_emb=0.0, dropout_att=0.0)
    sd = make_state_dict(cfg, int(z["seed"]))
    ref = enc.state_dict()
    enc.load_state_dict({k: torch.from_numpy(np.asarray(v)).reshape(ref[k].shape) for k, v in sd.items()})
    enc.set_compute_mode(compute)
    if "use_pad_mask" in z.files and not bool(z["use_pad_mask"]):   # train_tiny_nopad: enable_pad_mask(False)
        enc.enable_pad_mask(False)
    return enc.cuda().train()


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
@pytest.mark.parametrize("case", CASES)
def test_train_step_matches_reference(case, compute):
    z = np.load(os.path.join(GOLDEN, case + ".npz"))
    enc = _encoder(z, compute)
    x = torch.from_numpy(z["x"]).cuda()
    ln = torch.from_numpy(z["lengths"]).cuda()
    y, ylen = enc(audio_signal=x, length=ln)
    (y * torch.from_numpy(z["dy"]).cuda()).sum().backward()
    torch.cuda.synchronize()
    assert (ylen.cpu().numpy() == z["ylen"]).all()
    e = rel_l2(y.detach().cpu().numpy(), z["y"])
    assert e <= GATE_Y[compute], f"output relL2 {e:.3e}"
    params = dict(enc.named_parameters())
    worst = (0.0, "")
    # some gradients are analytically ~0 (depthwise-conv bias: train-mode BatchNorm removes any
    # per-channel shift), so the relative error is taken against a floor of 1e-2 x the largest
    # gradient norm of the step
    floor = 1e-2 * max(float(np.linalg.norm(z[k])) for k in z.files if k.startswith("grad__"))
    for k in z.files:
        if not k.startswith("grad__"):
            continue
        name = k[len("grad__"):]
        g = params[name].grad
        assert g is not None, f"no gradient for {name}"
        err = float(np.linalg.norm(g.cpu().numpy().astype(np.float64) - z[k]) / max(np.linalg.norm(z[k]), floor))
        worst = max(worst, (err, name))
        assert err <= GATE_G[compute], f"{name}: grad relL2 {err:.3e} > {GATE_G[compute]}"
    bufs = dict(enc.named_buffers())
    for k in z.files:
        if k.startswith("buf__"):
            err = rel_l2(bufs[k[len("buf__"):]].cpu().numpy(), z[k])
            assert err <= GATE_G[compute], f"{k}: relL2 {err:.3e}"
    print(f"{case}/{compute}: y relL2 {e:.2e}, worst grad {worst[1]} {worst[0]:.2e}")


def test_train_step_deterministic_and_dropout():
    """Same seed -> bitwise-identical gradients; dropout > 0 changes the output, keeps it finite,
    and its masks are regenerated consistently in the backward (directional derivative check)."""
    z = np.load(os.path.join(GOLDEN, "train_tiny.npz"))
    x = torch.from_numpy(z["x"]).cuda()
    ln = torch.from_numpy(z["lengths"]).cuda()
    dy = torch.from_numpy(z["dy"]).cuda()
    runs = []
    for _ in range(2):
        torch.manual_seed(123)
        enc = _encoder(z, "fp32", dropout=0.1)
        y, _ = enc(audio_signal=x, length=ln)
        (y * dy).sum().backward()
        runs.append((y.detach().clone(), [p.grad.clone() for p in enc.parameters()]))
    assert torch.equal(runs[0][0], runs[1][0])
    for a, b in zip(runs[0][1], runs[1][1]):
        assert torch.equal(a, b)
    assert torch.isfinite(runs[0][0]).all()
    assert rel_l2(runs[0][0].cpu().numpy(), z["y"]) > 1e-3      # dropout did something
    # directional derivative along one weight, same dropout masks (same seed): (L(w+h v) - L(w-h v)) / 2h
    torch.manual_seed(123)
    enc = _encoder(z, "fp32", dropout=0.1)
    w = enc.layers[0].feed_forward1.linear1.weight
    v = torch.randn_like(w)
    g_dir = float((runs[0][1][[n for n, _ in enc.named_parameters()].index("layers.0.feed_forward1.linear1.weight")]
                   * v).sum())
    h = 1e-3
    vals = []
    for s in (1.0, -1.0):
        torch.manual_seed(123)
        e2 = _encoder(z, "fp32", dropout=0.1)
        with torch.no_grad():
            e2.layers[0].feed_forward1.linear1.weight.add_(s * h * v)
        y2, _ = e2(audio_signal=x, length=ln)
        vals.append(float((y2.double() * dy.double()).sum()))
    fd = (vals[0] - vals[1]) / (2 * h)
    assert abs(fd - g_dir) <= 2e-2 * max(abs(g_dir), 1.0), (fd, g_dir)


def test_train_then_eval_uses_updated_running_stats():
    z = np.load(os.path.join(GOLDEN, "train_tiny.npz"))
    enc = _encoder(z, "fp32")
    x = torch.from_numpy(z["x"]).cuda()
    ln = torch.from_numpy(z["lengths"]).cuda()
    with torch.no_grad():
        y0, _ = enc.eval()(audio_signal=x, length=ln)
        enc.train()
        enc(audio_signal=x, length=ln)
        y1, _ = enc.eval()(audio_signal=x, length=ln)
    assert int(enc.layers[0].conv.batch_norm.num_batches_tracked) == 1
    assert not torch.equal(y0, y1)   # eval repacked the in-place-updated running statistics


def _enc_drop(z, compute, dropout_att, dropout_emb, dropout=0.0):
    from nemo.collections.asr.modules import ConformerEncoder
    from recipe import make_state_dict
    cfg = json.loads(str(z["cfg_json"]))
    enc = ConformerEncoder(**cfg, dropout=dropout, dropout_emb=dropout_emb, dropout_att=dropout_att)
    sd = make_state_dict(cfg, int(z["seed"]))
    ref = enc.state_dict()
    enc.load_state_dict({k: torch.from_numpy(np.asarray(v)).reshape(ref[k].shape) for k, v in sd.items()})
    enc.set_compute_mode(compute)
    return enc.cuda().train()


def _step(z, compute, seed, dropout_att, dropout_emb, perturb=None):
    torch.manual_seed(seed)
    enc = _enc_drop(z, compute, dropout_att, dropout_emb)
    if perturb is not None:
        name, v, h = perturb
        with torch.no_grad():
            dict(enc.named_parameters())[name].add_(h * v)
    x = torch.from_numpy(z["x"]).cuda()
    ln = torch.from_numpy(z["lengths"]).cuda()
    y, _ = enc(audio_signal=x, length=ln)
    loss = (y.double() * torch.from_numpy(z["dy"]).cuda().double()).sum()
    loss.backward()
    return enc, y.detach(), float(loss)


@pytest.mark.parametrize("case", ["train_tiny", "train_tiny_ctx"])
def test_attention_and_embedding_dropout(case):
    """dropout_att (attention probabilities, multi_head_attention.py:111) and dropout_emb (positional
    window, :316), as conformer_ctc_bpe.yaml:130-132 trains: the masks are a function of the step's
    seed only (bitwise-reproducible), they change the output, the native backward regenerates them
    (finite-difference directional derivatives along weights whose gradient flows through the dropped
    probabilities (linear_q, linear_v) and the dropped positional window (linear_pos)), and the bf16
    fused attention backward applies the same masks as the fp32 materialised one."""
    z = np.load(os.path.join(GOLDEN, case + ".npz"))
    enc, y0, _ = _step(z, "fp32", 7, 0.1, 0.1)
    _, y1, _ = _step(z, "fp32", 7, 0.1, 0.1)
    assert torch.equal(y0, y1)
    _, y_nodrop, _ = _step(z, "fp32", 7, 0.0, 0.0)
    assert rel_l2(y0.cpu().numpy(), y_nodrop.cpu().numpy()) > 1e-3
    grads = {n: p.grad.clone() for n, p in enc.named_parameters()}
    g = torch.Generator(device="cuda").manual_seed(3)
    for name in ("layers.0.self_attn.linear_q.weight", "layers.0.self_attn.linear_v.weight",
                 "layers.0.self_attn.linear_pos.weight", "layers.1.self_attn.linear_k.weight"):
        if name not in grads:
            continue
        v = torch.randn(grads[name].shape, device="cuda", generator=g)
        gd = float((grads[name].double() * v.double()).sum())
        h = 1e-3
        lp = _step(z, "fp32", 7, 0.1, 0.1, (name, v, h))[2]
        lm = _step(z, "fp32", 7, 0.1, 0.1, (name, v, -h))[2]
        fd = (lp - lm) / (2 * h)
        assert abs(fd - gd) <= 2e-2 * max(abs(gd), 1.0), (name, fd, gd)
    # bf16 (fused attention backward) against fp32 (materialised), same seed -> same masks
    # (linear_k.bias has an analytically zero gradient: relative to a floor of 1e-2 x the largest norm)
    enc16, _, _ = _step(z, "bf16", 7, 0.1, 0.1)
    floor = 1e-2 * max(float(g_.norm()) for g_ in grads.values())
    for n, p in enc16.named_parameters():
        if "self_attn" in n:
            ref = grads[n].double()
            e = float((p.grad.double() - ref).norm()) / max(float(ref.norm()), floor)
            assert e <= GATE_G["bf16"], (n, e)


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
def test_train_step_large_matches_reference(compute):
    """the training step at the Large shape (d_model 512, 8 heads, dk 64, 512 conv
    channels, T=1000 -> T'=250, ragged lengths; 2 layers) against the REFERENCE encoder's autograd
    (tests/golden/train_large.npz, summarised: norm + 4096 seeded samples + 2 projections per tensor).
    This exercises the shapes the toy goldens never reach: the 160k-row conv2 implicit GEMM and its
    weight gradient, the fused bf16 attention backward at T'=250 / dk=64, split-K weight gradients.
    Gates: fp32 1e-3 (sampled relL2 and norm) / 3e-3 (projections); bf16 2e-2 on the output, 6e-2
    on gradients (projections 1.5x)."""
    from conftest import summary_err
    from recipe import make_inputs
    z = np.load(os.path.join(GOLDEN, "train_large.npz"))
    cfg = json.loads(str(z["cfg_json"]))
    B, T = int(z["B"]), int(z["T"])
    seed = int(z["seed"])
    enc = _encoder(z, compute)
    x, ln = make_inputs(B, T, 80, seed + 100, [int(v) for v in z["lengths"]])
    y, ylen = enc(audio_signal=torch.from_numpy(x).cuda(), length=torch.from_numpy(ln).cuda())
    R = np.random.default_rng(seed + 200).standard_normal(tuple(y.shape)).astype(np.float32)
    assert abs(float(np.abs(R).sum()) - float(z["dy_checksum"])) <= 1e-6 * float(z["dy_checksum"])
    (y * torch.from_numpy(R).cuda()).sum().backward()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ylen.cpu().numpy(), z["ylen"])
    gy = GATE_Y[compute]
    es, en, ep = summary_err("y", y.detach().cpu().numpy(), z, "out__")
    assert es <= gy and en <= gy and ep <= 3 * gy, ("y", es, en, ep)
    gg = GATE_G[compute]
    worst = (0.0, "")
    # relative to max(|ref|, 1e-2 x the step's largest gradient norm), as test_train_step_matches_reference
    floor = 1e-2 * max(float(z[k]) for k in z.files if k.startswith("grad__") and k.endswith("__norm"))
    for name, p in enc.named_parameters():
        es, en, ep = summary_err(name, p.grad.cpu().numpy(), z, "grad__", floor)
        worst = max(worst, (max(es, en), name))
        assert es <= gg and en <= gg and ep <= (3 if compute == "fp32" else 1.5) * gg, (name, es, en, ep)
    bufs = dict(enc.named_buffers())
    for k in z.files:
        if k.startswith("buf__"):
            assert rel_l2(bufs[k[len("buf__"):]].cpu().numpy(), z[k]) <= gg, k
    print(f"train_large/{compute}: worst gradient {worst[1]} {worst[0]:.2e}")
