"""GPU tests of the cache-aware chunked streaming encoder (include/cfm_cache_stream.h).

Parity unpinned (the reference has no such model): each chunk the native step emits is compared
with the same frames of a full-sequence forward of the causal encoder the header defines
(oracle/cache_aware_oracle.py, itself checked against its own chunked restatement on the CPU in
tests/test_cache_stream_oracle.py).  Gates: fp32 compute relL2 <= 1e-3 per chunk (the encoder's
north-star gate); bf16 compute relL2 <= 2e-2 (the encoder's bf16 gate)."""
import numpy as np
import pytest
import torch

import cache_aware_oracle as CA
from conftest import rel_l2
from recipe import make_state_dict

pytestmark = pytest.mark.gpu


def _native(cfg, sd, compute):
    from conformer_amd import NativeEncoder, make_cfg
    enc = NativeEncoder(make_cfg(cfg["feat_in"], cfg["n_layers"], cfg["d_model"], n_heads=cfg["n_heads"],
                                 conv_kernel_size=cfg.get("conv_kernel_size", 31),
                                 conv_norm_type=cfg.get("conv_norm_type", "batch_norm"),
                                 feat_out=cfg.get("feat_out", -1)),
                        compute=compute)
    enc.set_weights({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return enc


def _run(cfg, B, chunk, left, steps, compute, seed=11):
    from conformer_amd.cache_stream import NativeCacheStream
    sd = make_state_dict(cfg, seed)
    x = np.random.default_rng(seed).standard_normal((B, cfg["feat_in"], 4 * chunk * steps)).astype(np.float32)
    ref = CA.causal_forward(x, sd, cfg, left)
    cs = NativeCacheStream(_native(cfg, sd, compute), B, chunk, left)
    xd = torch.from_numpy(x).cuda()
    outs = []
    for s in range(steps):
        outs.append(cs.step(xd[:, :, 4 * chunk * s:4 * chunk * (s + 1)]).cpu().numpy())
        assert cs.position == chunk * (s + 1)
    return ref, outs, cs, xd


TINY = dict(feat_in=16, n_layers=2, d_model=32, n_heads=4, conv_kernel_size=7)
SMALL = dict(feat_in=80, n_layers=2, d_model=64, n_heads=4, conv_kernel_size=31)


@pytest.mark.parametrize("cfg,B,chunk,left,steps", [
    (TINY, 2, 2, 5, 6),            # rings wrap (left + chunk = 7 < 12 frames)
    (TINY, 3, 1, 3, 8),            # one frame per step
    (SMALL, 2, 4, 16, 7),          # K-1 = 30 > chunk: GLU ring spans several chunks
    (SMALL, 2, 8, 4, 3),           # chunk > left context
    (dict(SMALL, conv_norm_type="layer_norm"), 2, 4, 8, 4),
    (dict(TINY, feat_out=24), 2, 2, 4, 3),
])
def test_chunks_match_full_causal_forward_fp32(cfg, B, chunk, left, steps):
    ref, outs, _, _ = _run(cfg, B, chunk, left, steps, "fp32")
    for s, y in enumerate(outs):
        r = ref[:, :, chunk * s:chunk * (s + 1)]
        assert y.shape == r.shape
        assert rel_l2(y, r) <= 1e-3, (s, rel_l2(y, r))


def test_large_width_fp32_and_bf16():
    cfg = dict(feat_in=80, n_layers=2, d_model=512, n_heads=8, conv_kernel_size=31)
    for compute, tol in (("fp32", 1e-3), ("bf16", 2e-2)):
        ref, outs, _, _ = _run(cfg, 4, 16, 48, 5, compute)
        got = np.concatenate(outs, axis=2)
        assert rel_l2(got, ref) <= tol, (compute, rel_l2(got, ref))


def test_reset_replays_bitwise():
    ref, outs, cs, xd = _run(SMALL, 2, 4, 8, 3, "bf16")
    cs.reset()
    assert cs.position == 0
    again = [cs.step(xd[:, :, 16 * s:16 * (s + 1)]).cpu().numpy() for s in range(3)]
    for a, b in zip(outs, again):
        np.testing.assert_array_equal(a, b)


def test_dropin_streamer():
    from nemo.collections.asr.modules import ConformerEncoder
    cfg = dict(SMALL)
    sd = make_state_dict(cfg, 4)
    enc = ConformerEncoder(feat_in=80, n_layers=2, d_model=64, n_heads=4, conv_kernel_size=31)
    ref_sd = enc.state_dict()
    enc.load_state_dict({k: torch.from_numpy(np.asarray(v)).reshape(ref_sd[k].shape) for k, v in sd.items()})
    enc.set_compute_mode("fp32")
    enc = enc.cuda().eval()
    st = enc.cache_aware_streamer(batch_size=2, chunk_size=4, left_context=12)
    x = np.random.default_rng(2).standard_normal((2, 80, 64)).astype(np.float32)
    ref = CA.causal_forward(x, sd, cfg, 12)
    xd = torch.from_numpy(x).cuda()
    ys = []
    for s in range(4):
        y, yl = st.step(xd[:, :, 16 * s:16 * (s + 1)])
        assert yl.tolist() == [4, 4]
        ys.append(y.cpu().numpy())
    assert rel_l2(np.concatenate(ys, axis=2), ref) <= 1e-3
    with torch.no_grad():
        enc.layers[0].feed_forward1.linear1.bias.add_(0.1)
    with pytest.raises(RuntimeError):
        st.step(xd[:, :, :16])
    st.reset()
    assert st.position == 0


def test_rejects_bad_arguments():
    from conformer_amd import _lib
    from conformer_amd.cache_stream import NativeCacheStream
    sd = make_state_dict(TINY, 1)
    enc = _native(TINY, sd, "fp32")
    with pytest.raises(_lib.CfmError):
        NativeCacheStream(enc, 2, 4, 0)
    cs = NativeCacheStream(enc, 2, 4, 8)
    with pytest.raises(ValueError):
        cs.step(torch.zeros(2, 16, 15, device="cuda"))


def test_block_and_wave_attention_kernels_agree_bitwise():
    """The LDS block kernel (window in LDS) and the per-wave kernel (window read from the ring) sum
    in the same order; the per-wave one is what runs when the window does not fit LDS."""
    import subprocess
    import sys
    code = ("import sys, numpy as np; sys.path[:0] = {p!r}; import test_gpu_cache_stream as t; "
            "ref, outs, _, _ = t._run(t.SMALL, 2, 4, 12, 5, 'bf16'); "
            "np.save({f!r}, np.concatenate(outs, axis=2))")
    import os
    import tempfile
    here = os.path.dirname(os.path.abspath(__file__))
    paths = sys.path[:]
    res = []
    for force in ("0", "1"):
        f = os.path.join(tempfile.mkdtemp(), "y.npy")
        env = dict(os.environ, CFM_CS_ATTN_WAVE=force)
        subprocess.run([sys.executable, "-c", code.format(p=[here] + paths, f=f)], check=True, env=env, timeout=300)
        res.append(np.load(f))
    np.testing.assert_array_equal(res[0], res[1])
