"""Model shells and unchanged-yaml loading (BASELINE north_star: "keeps the EncDecCTCModel /
EncDecRNNTModel plugin surface so conformer_ctc_bpe.yaml / conformer_transducer_bpe.yaml configs load
unchanged").  CPU only: construction, config semantics, parameters, scheduler, WER, .nemo round trip.
The forward / training step on the GPU: tests/test_gpu_models.py."""
import math
import os

import pytest
import torch

from model_configs import CTC_BPE_SMALL, REF_CONFIGS, RNNT_BPE_SMALL, make_bpe_tokenizer


@pytest.fixture(scope="module")
def tok_dir(tmp_path_factory):
    return make_bpe_tokenizer(str(tmp_path_factory.mktemp("tok")))


def _ref(name):
    p = os.path.join(REF_CONFIGS, name)
    if not os.path.exists(p):
        pytest.skip("reference configs not present (only in the build container)")
    return p


def test_config_semantics():
    from nemo.core.config import MissingMandatoryValue, load_config
    c = load_config(CTC_BPE_SMALL)
    m = c.model
    assert m.preprocessor.sample_rate == 16000                 # YAML alias *sample_rate
    assert m.train_ds.sample_rate == 16000                     # ${model.sample_rate}
    assert m.encoder.feat_in == 80                             # ${model.preprocessor.features}
    assert m.optim.sched.d_model == 128 and c.exp_manager.name == "Conformer-CTC-BPE-test"
    with pytest.raises(MissingMandatoryValue):
        _ = m.tokenizer.dir                                    # `???` until overridden
    assert m.tokenizer.is_missing("dir") and "dir" in m.tokenizer
    c2 = load_config(CTC_BPE_SMALL, {"model.tokenizer.dir": "/x", "model.encoder.d_model": 256})
    assert c2.model.tokenizer.dir == "/x" and c2.model.optim.sched.d_model == 256   # overrides before ${}
    assert c2.to_dict()["model"]["encoder"]["feat_in"] == 80


@pytest.mark.parametrize("name", ["conformer_ctc_bpe.yaml", "conformer_transducer_bpe.yaml", "conformer_ctc_char.yaml",
                                  "conformer_transducer_char.yaml"])
def test_reference_yamls_load_unchanged(name, tok_dir):
    """The reference's own yaml files, read as they are; only `???` fields a model reads are set."""
    from nemo.collections.asr import models
    from nemo.core.config import load_config
    path = _ref(name)
    bpe = "bpe" in name
    over = {"model.tokenizer.dir": tok_dir} if bpe else {}
    cfg = load_config(path, over)
    klass = {("ctc", True): models.EncDecCTCModelBPE, ("ctc", False): models.EncDecCTCModel,
             ("transducer", True): models.EncDecRNNTBPEModel, ("transducer", False): models.EncDecRNNTModel}[
        ("ctc" if "ctc" in name else "transducer", bpe)]
    m = klass(cfg.model)
    enc = cfg.model.encoder
    assert m.encoder.d_model == enc.d_model and len(m.encoder.layers) == enc.n_layers
    sd = m.state_dict()
    tops = {k.split(".", 1)[0] for k in sd}
    if "ctc" in name:
        assert tops == {"encoder", "decoder"} | ({"preprocessor"} if any(k.startswith("preprocessor") for k in sd)
                                                 else set())
        assert m.decoder.num_classes_with_blank == len(m.decoder.vocabulary) + 1
        assert m.loss._blank == m.decoder.num_classes_with_blank - 1
    else:
        assert {"encoder", "decoder", "joint"} <= tops
        assert m.joint.num_classes_with_blank == len(m.cfg.labels) + 1
        assert m.joint.fuse_loss_wer == cfg.model.joint.fuse_loss_wer
        if m.joint.fuse_loss_wer:
            assert m.joint.loss is m.loss and m.joint.wer is m.wer
    # Large encoders: the reference's 686-key state_dict layout for 17 layers (+40 per layer)
    n_enc = sum(1 for k in sd if k.startswith("encoder."))
    assert n_enc == 686 + 40 * (enc.n_layers - 17)


def test_bpe_model_requires_tokenizer_dir():
    from nemo.collections.asr.models import EncDecCTCModelBPE
    from nemo.core.config import MissingMandatoryValue, load_config
    with pytest.raises(MissingMandatoryValue):
        EncDecCTCModelBPE(load_config(CTC_BPE_SMALL).model)


def test_small_models_build_and_optimizer(tok_dir):
    from nemo.collections.asr.models import EncDecCTCModelBPE, EncDecRNNTBPEModel
    from nemo.core.config import load_config
    m = EncDecCTCModelBPE(load_config(CTC_BPE_SMALL, {"model.tokenizer.dir": tok_dir}).model)
    assert m.decoder.num_classes_with_blank == m.tokenizer.vocab_size + 1
    opt, sch = m.setup_optimization(max_steps=50)
    assert isinstance(opt, torch.optim.AdamW) and opt.defaults["betas"] == (0.9, 0.98)
    # NoamAnnealing (lr_scheduler.py:444-491): base * d^-0.5 * min(s^-0.5, s * w^-1.5), floor after warm-up
    lrs = []
    for _ in range(30):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        sch.step()
    for s, lr in enumerate(lrs):
        step = max(1, s)
        want = 2.0 * 128 ** -0.5 * min(step ** -0.5, step * 10 ** -1.5)
        if step > 10:
            want = max(want, 1e-6)
        assert math.isclose(lr, want, rel_tol=1e-6), (s, lr, want)
    r = EncDecRNNTBPEModel(load_config(RNNT_BPE_SMALL, {"model.tokenizer.dir": tok_dir}).model)
    assert r.joint.num_classes_with_blank == r.tokenizer.vocab_size + 1 and r.joint.fuse_loss_wer


def test_save_restore_roundtrip(tok_dir, tmp_path):
    from nemo.collections.asr.models import EncDecCTCModelBPE
    from nemo.core.config import load_config
    m = EncDecCTCModelBPE(load_config(CTC_BPE_SMALL, {"model.tokenizer.dir": tok_dir}).model)
    path = str(tmp_path / "m.nemo")
    m.save_to(path)
    r = EncDecCTCModelBPE.restore_from(path)
    a, b = m.state_dict(), r.state_dict()
    assert a.keys() == b.keys() and all(torch.equal(a[k], b[k]) for k in a)


def test_nemo_carries_tokenizer(tok_dir, tmp_path):
    """The tokenizer files are .nemo artifacts (reference mixins.py:85-151, save_restore_connector.py:304-396):
    a saved model restores after its tokenizer directory is gone, with the same vocabulary."""
    import shutil
    from nemo.collections.asr.models import EncDecCTCModelBPE
    from nemo.core.config import load_config
    tdir = str(tmp_path / "tok")
    shutil.copytree(tok_dir, tdir)
    m = EncDecCTCModelBPE(load_config(CTC_BPE_SMALL, {"model.tokenizer.dir": tdir}).model)
    path = str(tmp_path / "m.nemo")
    m.save_to(path)
    shutil.rmtree(tdir)
    r = EncDecCTCModelBPE.restore_from(path)
    assert r.tokenizer.get_vocab() == m.tokenizer.get_vocab()
    assert str(r.cfg.tokenizer.model_path).startswith("nemo:")              # the archive member
    assert os.path.isfile(r.artifacts["tokenizer.model_path"])                 # ... extracted for the model
    a, b = m.state_dict(), r.state_dict()
    assert all(torch.equal(a[k], b[k]) for k in a)
    # a restored model saves again with its artifacts (round trip of a round trip)
    path2 = str(tmp_path / "m2.nemo")
    r.save_to(path2)
    assert EncDecCTCModelBPE.restore_from(path2).tokenizer.get_vocab() == m.tokenizer.get_vocab()


def test_nemo_artifact_paths_stay_inside_the_archive(tok_dir, tmp_path):
    """`nemo:` paths name plain archive members only: '../x' or a directory part is refused."""
    import yaml
    from nemo.collections.asr.models import EncDecCTCModelBPE
    from nemo.core.config import load_config
    from nemo.core.connectors import SaveRestoreConnector
    m = EncDecCTCModelBPE(load_config(CTC_BPE_SMALL, {"model.tokenizer.dir": tok_dir}).model)
    cfg = m.cfg.to_dict()
    cfg["tokenizer"]["model_path"] = "nemo:../../etc/passwd"
    path = str(tmp_path / "bad.nemo")
    SaveRestoreConnector._make_nemo_file_from_members(path, {
        "model_config.yaml": yaml.safe_dump(cfg).encode(), "model_weights.ckpt": _state_bytes(m)})
    with pytest.raises(FileNotFoundError, match="plain archive member"):
        EncDecCTCModelBPE.restore_from(path)


def test_restore_refuses_foreign_targets(tok_dir, tmp_path):
    """A .nemo config is untrusted: a `_target_` outside this package's drop-in modules is refused
    before anything is instantiated (nothing in the file runs)."""
    import yaml
    from nemo.collections.asr.models import EncDecCTCModelBPE
    from nemo.core.config import load_config
    from nemo.core.connectors import SaveRestoreConnector
    m = EncDecCTCModelBPE(load_config(CTC_BPE_SMALL, {"model.tokenizer.dir": tok_dir}).model)
    marker = tmp_path / "pwned"
    cfg = m.cfg.to_dict()
    cfg["encoder"] = {"_target_": "subprocess.getoutput", "cmd": f"touch {marker}"}
    path = str(tmp_path / "evil.nemo")
    SaveRestoreConnector._make_nemo_file_from_members(path, {
        "model_config.yaml": yaml.safe_dump(cfg).encode(), "model_weights.ckpt": _state_bytes(m)})
    with pytest.raises(ValueError, match="refusing"):
        EncDecCTCModelBPE.restore_from(path)
    assert not marker.exists()


def _state_bytes(m):
    import io
    buf = io.BytesIO()
    torch.save(m.state_dict(), buf)
    return buf.getvalue()


def test_wer_metrics():
    from nemo.collections.asr.metrics.wer import WER, word_error_rate
    assert word_error_rate(["a b c", "x"], ["a c c", "x y"]) == pytest.approx(2 / 5)
    assert word_error_rate(["abc"], ["abd"], use_cer=True) == pytest.approx(1 / 3)
    w = WER(vocabulary=list("ab "), batch_dim_index=0)          # blank = 3
    pred = torch.tensor([[0, 0, 3, 0, 2, 1, 1, 3]])             # a a _ a ' ' b b _ -> "aa b"
    assert w.ctc_decoder_predictions_tensor(pred) == ["aa b"]
    w.update(pred, torch.tensor([[0, 0, 2, 1]]), torch.tensor([4]))
    wer, num, den = w.compute()
    assert float(wer) == 0.0 and float(den) == 2
