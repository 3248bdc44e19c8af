"""GPU parity of the buffered-streaming front end (include/cfm_stream.h) through the drop-in
`streaming_utils.FeatureFrameBufferer` / `BatchedFeatureFrameBufferer` against the reference's own
buffers (tests/golden/stream_*.npz), and a streaming step (buffer -> native encoder) against the
oracle encoder run on the reference's buffers.
Gates: normalised buffers max|err| <= 2e-5 (the kernel reduces in fp64, the reference in float32
pairwise sums: differences are rounding of mean / std); encoder fp32 gate as test_gpu_encoder."""
import json
import os
from types import SimpleNamespace

import numpy as np
import pytest
import torch

import conformer_oracle as O
from conftest import GOLDEN, rel_l2
from recipe import make_state_dict

pytestmark = pytest.mark.gpu
TOL = 2e-5


def _model(n_feat):
    return SimpleNamespace(_cfg=SimpleNamespace(sample_rate=16000, preprocessor=SimpleNamespace(
        window_stride=0.01, features=n_feat)), device=torch.device("cuda", 0))


def test_single_stream_bufferer_matches_reference():
    from nemo.collections.asr.parts.utils.streaming_utils import FeatureFrameBufferer
    z = np.load(os.path.join(GOLDEN, "stream_single.npz"))
    fb = FeatureFrameBufferer(_model(z["frames"].shape[1]), frame_len=1.6, batch_size=int(z["batch_size"]),
                              total_buffer=4.0)
    fb.set_frame_reader(iter(list(z["frames"])))
    got, sizes = [], []
    while True:
        b = fb.get_buffers_batch()
        if len(b) == 0:
            break
        sizes.append(len(b))
        got += [t.cpu().numpy() for t in b]
    assert sizes == list(z["per_batch"])
    np.testing.assert_allclose(np.stack(got), z["buffers"], rtol=0, atol=TOL)


def test_batched_bufferer_matches_reference():
    from nemo.collections.asr.parts.utils.streaming_utils import BatchedFeatureFrameBufferer
    z = np.load(os.path.join(GOLDEN, "stream_batched.npz"))
    B = z["frames"].shape[1]
    bb = BatchedFeatureFrameBufferer(_model(z["frames"].shape[2]), frame_len=0.3, batch_size=B, total_buffer=0.8)
    for i in range(B):
        bb.set_frame_reader(iter(list(z["frames"][: int(z["n_chunks"][i]), i])), i)
    s = 0
    while True:
        b = bb.get_buffers_batch()
        if len(b) == 0:
            break
        got = np.stack([x[0].cpu().numpy() for x in b])
        np.testing.assert_allclose(got, z["steps"][s], rtol=0, atol=TOL)
        assert [not e for e in bb.signal_end] == list(z["active"][s].astype(bool))
        s += 1
    assert s == z["steps"].shape[0]
    assert bb.signal_end_index == [int(np.argmin(z["active"][:, i])) for i in range(B)]


def test_multi_chunk_step_equals_sequential_steps():
    """k chunks in one call == k single-chunk calls (bitwise), and the buffer advances identically."""
    from conformer_amd.stream import NativeFrameBuffer
    g = torch.Generator().manual_seed(3)
    S, F, n, T, k = 5, 80, 160, 400, 4
    fr = (torch.randn(S, F, k * n, generator=g) * 4 - 5).cuda()
    a = NativeFrameBuffer(S, F, n, T, 1e-5)
    b = NativeFrameBuffer(S, F, n, T, 1e-5)
    out_k = a.step(fr).view(S, k, F, T)
    for i in range(k):
        o = b.step(fr[:, :, i * n:(i + 1) * n].contiguous())
        assert torch.equal(o, out_k[:, i])
    assert torch.equal(a.buffer, b.buffer)


def test_streaming_step_through_native_encoder():
    """One cfg-5-style step at a tiny model: batched buffers -> encoder (fp32) vs the oracle encoder
    on the reference's buffers (full-length utterances, as FrameBatchASR feeds them)."""
    from conformer_amd import NativeEncoder, make_cfg
    from nemo.collections.asr.parts.utils.streaming_utils import BatchedFeatureFrameBufferer
    z = np.load(os.path.join(GOLDEN, "stream_single.npz"))
    frames = z["frames"]                                    # (11, 80, 160): 4 streams x 2 steps below
    cfg = dict(feat_in=80, n_layers=2, d_model=64, n_heads=4)
    sd = make_state_dict(cfg, 7)
    enc = NativeEncoder(make_cfg(80, 2, 64, n_heads=4), compute="fp32")
    enc.set_weights({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    import stream_oracle as SO
    ob = SO.BatchedFeatureFrameBuffererOracle(4, 80, 160, 400)
    bb = BatchedFeatureFrameBufferer(_model(80), frame_len=1.6, batch_size=4, total_buffer=4.0)
    for step in range(2):
        fr = torch.from_numpy(frames[step * 4:(step + 1) * 4]).cuda()
        buf = bb.step(fr)
        ref_buf = ob.step(list(frames[step * 4:(step + 1) * 4]))
        assert np.abs(buf.cpu().numpy() - ref_buf).max() <= TOL
        y, yl = enc.forward(buf, torch.full((4,), 400, dtype=torch.int32, device="cuda"))
        yr, ylr = O.encoder_forward(ref_buf, np.full(4, 400), sd, cfg)
        np.testing.assert_array_equal(yl.cpu().numpy(), ylr)
        assert rel_l2(y.cpu().numpy(), yr) <= 1e-3


def test_rejects_bad_shapes():
    from conformer_amd import _lib
    from conformer_amd.stream import NativeFrameBuffer
    nb = NativeFrameBuffer(2, 8, 10, 30, 1e-8)
    with pytest.raises(ValueError):
        nb.step(torch.zeros(2, 8, 15, device="cuda"))
    with pytest.raises(_lib.CfmError):
        nb.step(torch.zeros(2, 8, 20, device="cuda"), active=torch.ones(2, dtype=torch.uint8))
