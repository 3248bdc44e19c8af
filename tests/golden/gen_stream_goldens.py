"""Golden fixtures for the buffered-streaming front end (include/cfm_stream.h), from the REFERENCE
FeatureFrameBufferer / BatchedFeatureFrameBufferer (nemo/collections/asr/parts/utils/streaming_utils.py
:455-818).  Only where /root/reference exists:

    python tests/golden/gen_stream_goldens.py   # writes tests/golden/stream_*.npz

streaming_utils.py is loaded from the reference tree with stubs for names the bufferers never
touch: `soundfile` (audio file reading), `omegaconf.OmegaConf` (config copy in FrameBatchASR),
`EncDecCTCModelBPE` (FrameBatchASR's preprocessor factory), `nemo.core.classes.IterableDataset`
(torch's IterableDataset) and two neural-type names.  The bufferers only read three config values
(sample_rate, preprocessor.window_stride, preprocessor.features), given by a SimpleNamespace.
Frames are seeded synthetic log-mel chunks; the per-chunk frame width is the reference's
n_frame_len and the last chunk of a stream is zero-padded as AudioFeatureIterator does (370-373).
"""
import importlib.util
import os
import sys
import types
from types import SimpleNamespace

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_goldens import REF, load_reference  # noqa: E402


def load_streaming():
    load_reference()
    stubs = {
        "soundfile": {},
        "omegaconf": {"OmegaConf": type("OmegaConf", (), {})},
        "nemo.collections.asr.models": {},
        "nemo.collections.asr.models.ctc_bpe_models": {"EncDecCTCModelBPE": type("EncDecCTCModelBPE", (), {})},
    }
    for name, attrs in stubs.items():
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
    sys.modules["nemo.core.classes"].IterableDataset = torch.utils.data.IterableDataset
    nt = sys.modules["nemo.core.neural_types"]
    for n in ["LengthsType", "NeuralType", "MelSpectrogramType"]:
        setattr(nt, n, lambda *a, **kw: None)
    name = "nemo.collections.asr.parts.utils.streaming_utils"
    spec = importlib.util.spec_from_file_location(name, f"{REF}/nemo/collections/asr/parts/utils/streaming_utils.py")
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def fake_model(n_feat, window_stride=0.01):
    return SimpleNamespace(_cfg=SimpleNamespace(sample_rate=16000, preprocessor=SimpleNamespace(
        window_stride=window_stride, features=n_feat)))


def chunks(g, n_feat, n_frame, total_frames):
    """Feature chunks of one stream as AudioFeatureIterator yields them (last one zero-padded)."""
    feats = (g.standard_normal((n_feat, total_frames)) * 3.0 - 6.0).astype(np.float32)
    out, start = [], 0
    while True:
        last = start + n_frame
        if last <= total_frames:
            out.append(feats[:, start:last].copy())
            start = last
        else:
            fr = np.zeros((n_feat, n_frame), dtype=np.float32)
            fr[:, : total_frames - start] = feats[:, start:total_frames]
            out.append(fr)
            return out


def main():
    su = load_streaming()
    # (1) single-stream FeatureFrameBufferer: frame_len 1.6 s, buffer 4.0 s, batch_size 4 (cfg 5 shapes)
    g = np.random.default_rng(5)
    n_feat = 80
    fb = su.FeatureFrameBufferer(fake_model(n_feat), frame_len=1.6, batch_size=4, total_buffer=4.0)
    frames = chunks(g, n_feat, fb.n_frame_len, 1750)
    fb.set_frame_reader(iter(frames))
    outs = []
    while True:
        b = fb.get_buffers_batch()
        if len(b) == 0:
            break
        outs.append(np.stack(b))
    np.savez_compressed(os.path.join(HERE, "stream_single.npz"), frames=np.stack(frames), n_frame=fb.n_frame_len,
                        total_len=fb.feature_buffer_len, batch_size=4,
                        buffers=np.concatenate(outs), per_batch=np.array([len(o) for o in outs]))
    # (2) BatchedFeatureFrameBufferer: 3 streams of different lengths (ended streams yield None)
    g = np.random.default_rng(6)
    n_feat, B = 16, 3
    bb = su.BatchedFeatureFrameBufferer(fake_model(n_feat), frame_len=0.3, batch_size=B, total_buffer=0.8)
    lens = [95, 41, 150]
    streams = [chunks(g, n_feat, bb.n_frame_len, L) for L in lens]
    for i in range(B):
        bb.set_frame_reader(iter(streams[i]), i)
    steps, acts = [], []
    while True:
        before = list(bb.signal_end)
        b = bb.get_buffers_batch()
        if len(b) == 0:
            break
        steps.append(np.stack([x[0] for x in b]))
        acts.append([not e for e in bb.signal_end])
    nmax = max(len(s) for s in streams)
    fr = np.zeros((nmax, B, n_feat, bb.n_frame_len), dtype=np.float32)
    for i, s in enumerate(streams):
        fr[: len(s), i] = np.stack(s)
    np.savez_compressed(os.path.join(HERE, "stream_batched.npz"), frames=fr,
                        n_chunks=np.array([len(s) for s in streams]), n_frame=bb.n_frame_len,
                        total_len=bb.feature_buffer_len, steps=np.stack(steps), active=np.array(acts, dtype=np.uint8))
    print("stream goldens:", len(outs), "single batches,", len(steps), "batched steps,",
          "n_frame", fb.n_frame_len, bb.n_frame_len, "total", fb.feature_buffer_len, bb.feature_buffer_len)


if __name__ == "__main__":
    main()
