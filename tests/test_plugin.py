"""Host-side plugin surface (no GPU): the yaml `_target_` path, constructor kwargs, state_dict layout,
keyword-only forward and neural types of the drop-in ConformerEncoder."""
import numpy as np
import pytest
import torch

from recipe import encoder_param_shapes

# The `encoder:` block of conformer_ctc_bpe.yaml (Large: d_model 512, n_heads 8, 17 layers here),
# with feat_in resolved from ${model.preprocessor.features}.
ENCODER_CFG = {
    "_target_": "nemo.collections.asr.modules.ConformerEncoder",
    "feat_in": 80, "feat_out": -1, "n_layers": 17, "d_model": 512,
    "subsampling": "striding", "subsampling_factor": 4, "subsampling_conv_channels": -1,
    "ff_expansion_factor": 4, "self_attention_model": "rel_pos", "n_heads": 8,
    "att_context_size": [-1, -1], "xscaling": True, "untie_biases": True, "pos_emb_max_len": 5000,
    "conv_kernel_size": 31, "conv_norm_type": "batch_norm",
    "dropout": 0.1, "dropout_emb": 0.0, "dropout_att": 0.1,
}


def test_from_config_dict_builds_the_dropin():
    from nemo.collections.asr.modules import ConformerEncoder
    from nemo.core.classes.common import Serialization
    enc = Serialization.from_config_dict(dict(ENCODER_CFG))
    assert isinstance(enc, ConformerEncoder)
    assert enc.d_model == 512 and enc._feat_out == 512


def test_state_dict_layout_matches_reference():
    from nemo.collections.asr.modules import ConformerEncoder
    enc = ConformerEncoder(feat_in=80, n_layers=17, d_model=512, n_heads=8)
    sd = enc.state_dict()
    want = dict(encoder_param_shapes(dict(d_model=512, n_heads=8, n_layers=17)))
    assert len(sd) == 686
    assert set(sd) == set(want)
    for k, shp in want.items():
        assert tuple(sd[k].shape) == tuple(shp), k


def test_forward_is_keyword_only_and_cpu_is_refused():
    """No CPU fallback: eval and train forwards on CPU tensors raise (the product path is HIP only)."""
    from nemo.collections.asr.modules import ConformerEncoder
    enc = ConformerEncoder(feat_in=80, n_layers=1, d_model=64, n_heads=4)
    x = torch.zeros(1, 80, 16)
    ln = torch.tensor([16])
    with pytest.raises(TypeError):
        enc(x, ln)
    for mode in (enc.eval, enc.train):
        mode()
        with pytest.raises(RuntimeError):
            enc(audio_signal=x, length=ln)


def test_neural_types_and_input_example():
    from nemo.collections.asr.modules import ConformerEncoder
    enc = ConformerEncoder(feat_in=80, n_layers=1, d_model=64, n_heads=4)
    assert set(enc.input_types) == {"audio_signal", "length"}
    assert set(enc.output_types) == {"outputs", "encoded_lengths"}
    x, ln = enc.input_example()
    assert x.shape[1] == 80 and ln.shape[0] == x.shape[0]


def test_abs_pos_module_tree():
    """self_attention_model='abs_pos' (conformer_encoder.py:184-189): PositionalEncoding, MultiHeadAttention
    layers and the reference's state_dict keys (no linear_pos / pos_bias), also with untie_biases=False."""
    from nemo.collections.asr.modules import ConformerEncoder
    from nemo.collections.asr.parts.submodules.multi_head_attention import (MultiHeadAttention,
                                                                            RelPositionMultiHeadAttention)
    from recipe import encoder_param_shapes
    cfg = dict(feat_in=80, n_layers=2, d_model=64, n_heads=4, self_attention_model="abs_pos")
    for untie in (True, False):
        enc = ConformerEncoder(**cfg, untie_biases=untie)
        assert type(enc.layers[0].self_attn) is MultiHeadAttention
        assert not isinstance(enc.layers[0].self_attn, RelPositionMultiHeadAttention)
        shapes = dict(encoder_param_shapes(cfg))
        sd = enc.state_dict()
        assert set(sd) == set(shapes)
        assert all(tuple(sd[k].shape) == tuple(v) for k, v in shapes.items())
        assert enc._dropout_emb == 0.0


@pytest.mark.parametrize("bad", [{"subsampling": "vggnet"}, {"self_attention_model": "bogus_pos"},
                                 {"subsampling_factor": 8}])
def test_unsupported_configs_raise(bad):
    from nemo.collections.asr.modules import ConformerEncoder
    kw = dict(feat_in=80, n_layers=1, d_model=64, n_heads=4)
    kw.update(bad)
    with pytest.raises((ValueError, NotImplementedError)):
        ConformerEncoder(**kw)
