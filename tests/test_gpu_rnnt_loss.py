"""GPU parity of the native RNN-T loss (include/cfm_rnnt_loss.h) through the drop-in
`nemo.collections.asr.losses.RNNTLoss` against the reference's own numpy RNN-T loss
(tests/golden/rnnt_loss_*.npz) and the float64 oracle of the GPU-kernel formulas.
Gates (fp32 kernels, as the reference's numba kernels): costs rel <= 1e-4, gradients
abs <= 5e-5 * max|grad| (the reference keeps its lattices in float32 too)."""
import glob
import os

import numpy as np
import pytest
import torch

import rnnt_loss_oracle as RO
from conftest import GOLDEN

pytestmark = pytest.mark.gpu
FILES = sorted(glob.glob(os.path.join(GOLDEN, "rnnt_loss_*.npz")))


def _inputs(z):
    acts = torch.from_numpy(z["acts"]).cuda().requires_grad_(True)
    return (acts, torch.from_numpy(z["labels"]).cuda(), torch.from_numpy(z["act_lens"]).cuda(),
            torch.from_numpy(z["label_lens"]).cuda())


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
def test_loss_matches_reference(path):
    from nemo.collections.asr.losses.rnnt import RNNTLoss
    z = np.load(path)
    V1 = z["acts"].shape[-1]
    blank = int(z["blank"])
    kw = {"fastemit_lambda": float(z["fastemit_lambda"]), "clamp": float(z["clamp"])}
    # the reference RNNTLoss fixes blank = num_classes; blank-0 cases use RNNTLossNumba directly
    acts, labels, al, ll = _inputs(z)
    if blank == V1 - 1:
        loss = RNNTLoss(num_classes=V1 - 1, reduction=None, loss_kwargs=kw)
        costs = loss(log_probs=acts, targets=labels, input_lengths=al, target_lengths=ll)
    else:
        from nemo.collections.asr.losses.rnnt import RNNTLossNumba
        costs = RNNTLossNumba(blank=blank, reduction="none", **kw)(acts, labels, al, ll)
    costs.sum().backward()
    np.testing.assert_allclose(costs.detach().cpu().numpy(), z["costs"], rtol=1e-4)
    g = acts.grad.cpu().numpy()
    np.testing.assert_allclose(g, z["grads"], rtol=0, atol=5e-5 * max(1.0, np.abs(z["grads"]).max()))


def test_mean_batch_and_reductions():
    from nemo.collections.asr.losses.rnnt import RNNTLoss
    z = np.load(os.path.join(GOLDEN, "rnnt_loss_blank_last.npz"))
    V = z["acts"].shape[-1] - 1
    acts, labels, al, ll = _inputs(z)
    m = RNNTLoss(num_classes=V)(log_probs=acts, targets=labels, input_lengths=al, target_lengths=ll)
    assert abs(float(m) - z["costs"].mean()) <= 1e-4 * abs(z["costs"].mean())
    m.backward()
    np.testing.assert_allclose(acts.grad.cpu().numpy(), z["grads"] / acts.shape[0], rtol=0, atol=5e-5)
    for red, want in (("sum", z["costs"].sum()), ("mean", z["costs"].sum() / acts.shape[0])):
        v = RNNTLoss(num_classes=V, reduction=red)(log_probs=acts.detach(), targets=labels, input_lengths=al,
                                                   target_lengths=ll)
        assert abs(float(v) - want) <= 1e-4 * abs(want)


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
def test_deferred_gradient_is_bitwise_the_reference_order(path, monkeypatch):
    """The backward-time gradient (cfm_rnnt_loss_grad: pre-scale and per-utterance scale applied in the kernel)
    against the reference order (gradient written in the forward, divided / multiplied in place after it):
    bitwise equal for every reduction, with a non-uniform incoming gradient."""
    from nemo.collections.asr.losses.rnnt import RNNTLoss, RNNTLossNumba
    z = np.load(path)
    blank = int(z["blank"])
    kw = {"fastemit_lambda": float(z["fastemit_lambda"]), "clamp": float(z["clamp"])}
    B = z["acts"].shape[0]
    gen = torch.Generator().manual_seed(5)
    gout = (torch.rand(B, generator=gen) + 0.5).cuda()

    def grad(defer, red):
        monkeypatch.setenv("CFM_RNNT_DEFER_GRAD", "1" if defer else "0")
        acts, labels, al, ll = _inputs(z)
        if red == "mean_batch":
            if blank != acts.shape[-1] - 1:
                return None
            out = RNNTLoss(num_classes=acts.shape[-1] - 1, loss_kwargs=kw)(log_probs=acts, targets=labels,
                                                                          input_lengths=al, target_lengths=ll)
            out.backward()
        else:
            out = RNNTLossNumba(blank=blank, reduction=red, **kw)(acts, labels, al, ll)
            out.backward(gout if red == "none" else gout[:1])
        return acts.grad
    for red in ("none", "sum", "mean", "mean_batch"):
        a, b = grad(True, red), grad(False, red)
        if a is None:
            continue
        assert torch.equal(a, b), red


def test_deferred_gradient_retained_graph_and_inplace_guard(monkeypatch):
    """the deferred gradient keeps its state with the autograd node, so a retained graph gives
    the same gradient on a second backward (accumulated twice, as the reference order does); acts are
    saved through autograd, so changing them in place between forward and backward raises."""
    from nemo.collections.asr.losses.rnnt import RNNTLossNumba
    z = np.load(FILES[0])
    blank = int(z["blank"])
    kw = {"fastemit_lambda": float(z["fastemit_lambda"]), "clamp": float(z["clamp"])}
    grads = {}
    for defer in ("1", "0"):
        monkeypatch.setenv("CFM_RNNT_DEFER_GRAD", defer)
        acts, labels, al, ll = _inputs(z)
        out = RNNTLossNumba(blank=blank, reduction="sum", **kw)(acts, labels, al, ll)
        out.backward(retain_graph=True)
        g1 = acts.grad.clone()
        out.backward()
        assert torch.isfinite(acts.grad).all()
        grads[defer] = (g1, acts.grad.clone())
    assert torch.equal(grads["1"][0], grads["0"][0])
    assert torch.equal(grads["1"][1], 2 * grads["1"][0])
    monkeypatch.setenv("CFM_RNNT_DEFER_GRAD", "1")
    acts, labels, al, ll = _inputs(z)
    out = RNNTLossNumba(blank=blank, reduction="sum", **kw)(acts, labels, al, ll)
    with torch.no_grad():
        acts.mul_(2.0)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        out.backward()


def test_cfg4_shape_against_oracle_and_no_grad():
    """BASELINE config-4-like lattice (V+1=1025, U+1=21, T=40, ragged) vs the oracle; forward-only
    (no grads) returns the same costs."""
    from conformer_amd.rnnt_loss import rnnt_loss
    g = np.random.default_rng(9)
    B, T, U, V1 = 3, 40, 21, 1025
    acts = (g.standard_normal((B, T, U, V1)) * 3).astype(np.float32)
    al = np.array([40, 33, 17], dtype=np.int32)
    ll = np.array([20, 12, 20], dtype=np.int32)
    labels = g.integers(0, V1 - 1, (B, U - 1)).astype(np.int32)
    c, gr = rnnt_loss(torch.from_numpy(acts).cuda(), torch.from_numpy(labels).cuda(), torch.from_numpy(al).cuda(),
                      torch.from_numpy(ll).cuda(), V1 - 1)
    c0, _ = rnnt_loss(torch.from_numpy(acts).cuda(), torch.from_numpy(labels).cuda(), torch.from_numpy(al).cuda(),
                      torch.from_numpy(ll).cuda(), V1 - 1, want_grads=False)
    rc, rg = RO.rnnt_loss(acts, labels, al, ll, V1 - 1)
    np.testing.assert_allclose(c.cpu().numpy(), rc, rtol=1e-4)
    assert torch.equal(c, c0)
    # fp32 lattices against a float64 oracle: log-likelihoods of ~-300 carry ~2e-5 relative rounding
    # into every exp(alpha + beta + logp - ll) term (measured max |err| 8.9e-5)
    np.testing.assert_allclose(gr.cpu().numpy(), rg, rtol=0, atol=2e-4 * max(1.0, np.abs(rg).max()))
    # gradient rows of a valid lattice node sum to ~0 over the vocabulary (softmax Jacobian)
    s = gr.double().sum(-1)
    assert s.abs().max().item() < 1e-4
