"""Model shells on the GPU (ctc_models.py:552-630, rnnt_models.py:620-800 semantics) over the native
drop-ins: forward from spectrograms and from raw audio, the CTC training step end to end (loss,
backward through the native encoder / decoder / CTC kernels, optimizer step), the RNN-T
validation step through the fused joint + native RNN-T loss + greedy-decoding WER."""
import numpy as np
import pytest
import torch

from conftest import rel_l2
from model_configs import CTC_BPE_SMALL, RNNT_BPE_SMALL, make_bpe_tokenizer

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tok_dir(tmp_path_factory):
    return make_bpe_tokenizer(str(tmp_path_factory.mktemp("tok")))


def _batch(B=4, T=240, U=12, V=40, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, 80, T, generator=g).cuda()
    xl = torch.tensor([T - 17 * i for i in range(B)], dtype=torch.int64).cuda()
    y = torch.randint(0, V, (B, U), generator=g).cuda()
    yl = torch.tensor([U - 2 * i for i in range(B)], dtype=torch.int64).cuda()
    return x, xl, y, yl


def _ctc(tok_dir):
    from nemo.collections.asr.models import EncDecCTCModelBPE
    from nemo.core.config import load_config
    torch.manual_seed(0)
    return EncDecCTCModelBPE(load_config(CTC_BPE_SMALL, {"model.tokenizer.dir": tok_dir}).model).cuda()


def test_ctc_forward_is_the_module_composition(tok_dir):
    m = _ctc(tok_dir).eval()
    x, xl, _, _ = _batch(V=m.tokenizer.vocab_size)
    with torch.no_grad():
        lp, el, pred = m.forward(processed_signal=x, processed_signal_length=xl)
        enc, el2 = m.encoder(audio_signal=x, length=xl)
        lp2 = m.decoder(encoder_output=enc)
    assert lp.shape == (4, 60, m.decoder.num_classes_with_blank)
    assert torch.equal(el, el2) and torch.equal(lp, lp2) and torch.equal(pred, lp.argmax(-1))
    # log-softmax rows
    assert float((lp.exp().sum(-1) - 1).abs().max()) < 1e-3
    with pytest.raises(TypeError):
        m.forward(x, xl)                                       # keyword-only (typecheck)
    with pytest.raises(ValueError):
        m.forward(processed_signal=x)                          # lengths missing -> neither input complete


def test_ctc_raw_audio_goes_through_the_preprocessor(tok_dir):
    m = _ctc(tok_dir).eval()
    g = torch.Generator().manual_seed(3)
    wav = (0.1 * torch.randn(2, 32000, generator=g)).cuda()
    wl = torch.tensor([32000, 25000]).cuda()
    with torch.no_grad():
        lp, el, _ = m.forward(input_signal=wav, input_signal_length=wl)
        spec, sl = m.preprocessor(input_signal=wav, length=wl)
        lp2, el2, _ = m.forward(processed_signal=spec, processed_signal_length=sl)
    assert torch.equal(lp, lp2) and torch.equal(el, el2)


def test_ctc_training_step_trains(tok_dir):
    m = _ctc(tok_dir)
    x, xl, y, yl = _batch(V=m.tokenizer.vocab_size)
    opt, _ = m.setup_optimization({"name": "adamw", "lr": 1e-3, "betas": [0.9, 0.98], "weight_decay": 0.0})
    # eval-mode step: the loss is the CTC loss of the forward outputs (same arithmetic, no dropout)
    m.eval()
    with torch.no_grad():
        lp, el, _ = m.forward(processed_signal=x, processed_signal_length=xl)
        want = m.loss(log_probs=lp, targets=y, input_lengths=el, target_lengths=yl)
        got = m.validation_step((x, xl, y, yl), 0, processed_signal=True)["val_loss"]
    assert torch.isfinite(got) and float(abs(got - want)) <= 1e-5 * float(abs(want))
    m.train()
    before = {k: v.detach().clone() for k, v in m.named_parameters()}
    losses = []
    for i in range(4):
        opt.zero_grad(set_to_none=True)
        out = m.training_step((x, xl, y, yl), i, processed_signal=True)
        out["loss"].backward()
        enc_g = [p.grad for n, p in m.named_parameters() if n.startswith("encoder.layers.0.")]
        assert all(g is not None and torch.isfinite(g).all() for g in enc_g)
        assert float(m.decoder.decoder_layers[0].weight.grad.abs().sum()) > 0
        opt.step()
        losses.append(float(out["loss"]))
        assert "training_batch_wer" in out["log"]
    assert all(np.isfinite(losses))
    changed = sum(not torch.equal(before[k], v) for k, v in m.named_parameters())
    assert changed == len(before)
    print("CTC training losses", losses)


def test_rnnt_fused_validation_step_matches_unfused(tok_dir):
    from nemo.collections.asr.models import EncDecRNNTBPEModel
    from nemo.core.config import load_config
    torch.manual_seed(0)
    m = EncDecRNNTBPEModel(load_config(RNNT_BPE_SMALL, {"model.tokenizer.dir": tok_dir}).model).cuda().eval()
    m.joint.set_compute_mode("fp32")
    x, xl, y, yl = _batch(V=m.tokenizer.vocab_size)
    y, yl = y.int(), yl.int()
    out = m.validation_step((x, xl, y, yl), 0, processed_signal=True)
    assert m.joint.fuse_loss_wer and m.joint.fused_batch_size == 2
    with torch.no_grad():
        enc, el = m.forward(processed_signal=x, processed_signal_length=xl)
        dec, tl, _ = m.decoder(targets=y, target_length=yl)
        m.joint.set_fuse_loss_wer(False)
        joint = m.joint(encoder_outputs=enc, decoder_outputs=dec)
        m.joint.set_fuse_loss_wer(True, m.loss, m.wer)
        want = m.loss(log_probs=joint, targets=y, input_lengths=el, target_lengths=tl)
    assert torch.isfinite(out["val_loss"])
    assert rel_l2(float(out["val_loss"]), float(want)) <= 1e-5, (float(out["val_loss"]), float(want))
    assert int(out["val_wer_denom"]) > 0 and out["val_wer"] is not None
    hyps = m.transcribe_processed(x, xl)
    assert len(hyps) == 4 and all(isinstance(h, str) for h in hyps)
    m.eval()
    with torch.no_grad():
        tr = m.training_step((x, xl, y, yl), 0, processed_signal=True)
    assert torch.isfinite(tr["loss"])
