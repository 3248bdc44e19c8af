""".nemo checkpoint import/export (nemo/core/connectors/save_restore_connector.py), on
CPU: archive format, safe loading, interpolation, and module restoration with the reference's
attribute names and state_dict keys."""
import io
import os
import tarfile

import pytest
import torch
import yaml

# The `model:` skeleton of conformer_ctc_bpe.yaml (configs/conformer_ctc_bpe.yaml:76-125), shrunk,
# with its `${model.preprocessor.features}` interpolation left unresolved as in a hand-written config.
CFG = {"model": {
    "sample_rate": 16000,
    "preprocessor": {"_target_": "nemo.collections.asr.modules.AudioToMelSpectrogramPreprocessor",
                     "sample_rate": 16000, "normalize": "per_feature", "window_size": 0.025, "window_stride": 0.01,
                     "window": "hann", "features": 80, "n_fft": 512, "log": True, "frame_splicing": 1,
                     "dither": 0.00001, "pad_to": 0, "pad_value": 0.0},
    "spec_augment": {"_target_": "nemo.collections.asr.modules.SpectrogramAugmentation",
                     "freq_masks": 2, "time_masks": 10, "freq_width": 27, "time_width": 0.05},
    "encoder": {"_target_": "nemo.collections.asr.modules.ConformerEncoder",
                "feat_in": "${model.preprocessor.features}", "feat_out": -1, "n_layers": 2, "d_model": 64,
                "subsampling": "striding", "subsampling_factor": 4, "subsampling_conv_channels": -1,
                "ff_expansion_factor": 4, "self_attention_model": "rel_pos", "n_heads": 4,
                "att_context_size": [-1, -1], "xscaling": True, "untie_biases": True, "pos_emb_max_len": 5000,
                "conv_kernel_size": 31, "conv_norm_type": "batch_norm", "dropout": 0.1, "dropout_emb": 0.0,
                "dropout_att": 0.1},
    "decoder": {"_target_": "nemo.collections.asr.modules.ConvASRDecoder", "feat_in": None, "num_classes": -1,
                "vocabulary": ["a", "b", "c", "d", "e"]},
}}


def _model_state(seed=0):
    """A state_dict laid out as EncDecCTCModel's (attribute-prefixed), with random values."""
    from nemo.core.connectors.save_restore_connector import resolve_interpolations
    from nemo.core.classes.common import Serialization
    m = resolve_interpolations(CFG)["model"]
    enc = Serialization.from_config_dict(m["encoder"])
    dec_cfg = dict(m["decoder"], feat_in=enc._feat_out, num_classes=len(m["decoder"]["vocabulary"]))
    dec = Serialization.from_config_dict(dec_cfg)
    pre = Serialization.from_config_dict(m["preprocessor"])
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for prefix, mod in (("preprocessor", pre), ("encoder", enc), ("decoder", dec)):
        for k, v in mod.state_dict().items():
            sd[f"{prefix}.{k}"] = torch.randn(v.shape, generator=g).to(v.dtype) if v.is_floating_point() else v
    return sd


@pytest.mark.parametrize("gz", [False, True])
def test_roundtrip_and_restore_modules(tmp_path, gz):
    from nemo.collections.asr.modules import ConformerEncoder, ConvASRDecoder, SpectrogramAugmentation
    from nemo.core.connectors import SaveRestoreConnector, restore_modules
    sd = _model_state()
    path = str(tmp_path / "m.nemo")
    SaveRestoreConnector().save_to(CFG, sd, path)
    if gz:   # pre-1.7 checkpoints are gzip-compressed tars
        raw = open(path, "rb").read()
        with tarfile.open(fileobj=io.BytesIO(raw), mode="r:") as src, tarfile.open(path, "w:gz") as dst:
            for mem in src.getmembers():
                dst.addfile(mem, src.extractfile(mem))
    with tarfile.open(path, "r:*") as t:
        assert sorted(t.getnames()) == ["./model_config.yaml", "./model_weights.ckpt"]
    conf, mods = restore_modules(path)
    assert conf["encoder"]["feat_in"] == 80                      # interpolation resolved, model: unwrapped
    assert isinstance(mods["encoder"], ConformerEncoder) and isinstance(mods["decoder"], ConvASRDecoder)
    assert isinstance(mods["spec_augmentation"], SpectrogramAugmentation)
    assert mods["decoder"].num_classes_with_blank == 6             # ctc_models.py:178-184 fix-up
    for attr in ("preprocessor", "encoder", "decoder"):
        for k, v in mods[attr].state_dict().items():
            assert torch.equal(v, sd[f"{attr}.{k}"]), (attr, k)


def test_extract_state_dict_split_by_module(tmp_path):
    from nemo.core.connectors import SaveRestoreConnector
    sd = _model_state(1)
    path = str(tmp_path / "m.nemo")
    conn = SaveRestoreConnector()
    conn.save_to(CFG, sd, path)
    out = conn.extract_state_dict_from(path, str(tmp_path / "ck"), split_by_module=True)
    assert set(out) == set(sd)
    assert sorted(os.listdir(tmp_path / "ck")) == ["decoder.ckpt", "encoder.ckpt", "preprocessor.ckpt"]
    enc = torch.load(str(tmp_path / "ck" / "encoder.ckpt"), weights_only=True)
    assert all(torch.equal(v, sd["encoder." + k]) for k, v in enc.items())
    assert conn.load_config_and_state_dict(path, return_config=True)["decoder"]["vocabulary"] == list("abcde")


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned",))


def test_pickled_code_in_a_checkpoint_is_refused(tmp_path):
    """Weights are read with torch.load(weights_only=True): an object that would execute code on
    unpickling is rejected instead of run."""
    from nemo.core.connectors import SaveRestoreConnector
    buf = io.BytesIO()
    torch.save({"encoder.x": _Evil()}, buf)
    path = str(tmp_path / "bad.nemo")
    SaveRestoreConnector._make_nemo_file_from_members(
        path, {"model_config.yaml": yaml.safe_dump(CFG).encode(), "model_weights.ckpt": buf.getvalue()})
    with pytest.raises(Exception):
        SaveRestoreConnector().load_config_and_state_dict(path)


def test_unknown_targets_are_skipped_and_missing_file_raises(tmp_path):
    from nemo.core.connectors import SaveRestoreConnector, restore_modules
    cfg = {"model": dict(CFG["model"], decoder={"_target_": "nemo.collections.asr.modules.RNNTDecoderX",
                                                "prednet": {}})}
    sd = {k: v for k, v in _model_state().items() if not k.startswith("decoder.")}
    path = str(tmp_path / "r.nemo")
    SaveRestoreConnector().save_to(cfg, sd, path)
    _, mods = restore_modules(path)
    assert "decoder" not in mods and "encoder" in mods
    with pytest.raises(FileNotFoundError):
        SaveRestoreConnector().load_config_and_state_dict(str(tmp_path / "nope.nemo"))


@pytest.mark.gpu
def test_restored_encoder_reproduces_reference_outputs(tmp_path):
    """A `.nemo` holding reference-seeded encoder weights (tests/golden/enc_tiny.npz recipe) restores
    into the drop-in ConformerEncoder, whose fp32 forward reproduces the REFERENCE's outputs."""
    import json

    import numpy as np

    from conftest import GOLDEN, rel_l2
    from nemo.core.connectors import SaveRestoreConnector, restore_modules
    import inspect

    from nemo.collections.asr.modules import ConformerEncoder
    z = np.load(os.path.join(GOLDEN, "enc_tiny.npz"))
    cfg = json.loads(str(z["cfg_json"]))
    sd = {"encoder." + k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w/")}
    params = inspect.signature(ConformerEncoder.__init__).parameters
    enc_cfg = {"_target_": "nemo.collections.asr.modules.ConformerEncoder", "feat_in": 80,
               **{k: v for k, v in cfg.items() if k in params}}
    path = str(tmp_path / "enc.nemo")
    SaveRestoreConnector().save_to({"model": {"encoder": enc_cfg}}, sd, path)
    _, mods = restore_modules(path, map_location="cuda")
    enc = mods["encoder"].eval()
    enc.set_compute_mode("fp32")
    y, yl = enc(audio_signal=torch.from_numpy(z["x"]).cuda(), length=torch.from_numpy(z["lengths"]).cuda())
    assert rel_l2(y.cpu().numpy(), z["y"]) < 1e-3
    np.testing.assert_array_equal(yl.cpu().numpy(), z["y_len"])


@pytest.mark.parametrize("strict", [False, True])
def test_restore_refuses_foreign_targets(tmp_path, strict):
    """A .nemo config is untrusted input: a `_target_` outside this package's drop-in modules is
    never resolved or called (subprocess.getoutput as an encoder target)."""
    from nemo.core.connectors import SaveRestoreConnector, restore_modules
    marker = tmp_path / "pwned_marker"
    cfg = {"model": {"encoder": {"_target_": "subprocess.getoutput", "cmd": f"touch {marker}"}}}
    path = str(tmp_path / "evil.nemo")
    SaveRestoreConnector().save_to(cfg, {}, path)
    if strict:
        with pytest.raises(ValueError, match="refusing"):
            restore_modules(path, strict=True)
    else:
        _, mods = restore_modules(path, strict=False)
        assert "encoder" not in mods
    assert not marker.exists()
