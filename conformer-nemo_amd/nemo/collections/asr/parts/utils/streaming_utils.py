"""Drop-in buffered-streaming front end: `nemo.collections.asr.parts.utils.streaming_utils`
(reference streaming_utils.py:345-818), SURVEY §8 row a-ext5.

The reference keeps each stream's 4 s feature buffer in host numpy, shifts a 1.6 s chunk in, and
normalises the buffer per feature on the host before every encoder call.  Here the buffers live
on the GPU (`conformer_amd.stream.NativeFrameBuffer`, C-ABI include/cfm_stream.h) and one kernel
does shift + statistics + normalisation, writing the encoder's (B, F, T) input directly.

Same class names, constructor arguments and public flow as the reference:
  * `FeatureFrameBufferer.get_buffers_batch()` -> list of normalised (F, Tbuf) buffers, one per
    chunk of the single stream (eps 1e-5, streaming_utils.py:548-566);
  * `BatchedFeatureFrameBufferer.get_buffers_batch()` -> per stream a one-element list holding its
    normalised buffer, zeros once the stream has ended (eps 1e-8, 751-818), with `signal_end`,
    `signal_end_index` and `buffer_number` kept as the reference does.
Buffers are returned as CUDA tensors (views of one batch tensor; `torch.as_tensor` in the
reference's AudioBuffersDataLayer accepts them unchanged).  `BatchedFeatureFrameBufferer.step()`
is the device-resident hot path: (B, F, n_frame) chunks already on the GPU -> (B, F, Tbuf).
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from conformer_amd.stream import ZERO_LEVEL_SPEC_DB_VAL, NativeFrameBuffer

__all__ = ["AudioFeatureIterator", "AudioBuffersDataLayer", "speech_collate_fn", "FeatureFrameBufferer",
           "BatchedFeatureFrameBufferer"]


def _cfg_get(cfg, key):
    return cfg[key] if isinstance(cfg, dict) else getattr(cfg, key)


class AudioFeatureIterator(torch.utils.data.IterableDataset):
    """Feature chunks of one utterance (streaming_utils.py:345-375): the preprocessor runs once over
    the whole signal, then n_frame-wide chunks are yielded, the last one zero-padded."""

    def __init__(self, samples, frame_len, preprocessor, device):
        self._samples = samples
        self._frame_len = frame_len
        self._start = 0
        self.output = True
        self.count = 0
        timestep_duration = _cfg_get(preprocessor._cfg, "window_stride")
        self._feature_frame_len = frame_len / timestep_duration
        audio_signal = torch.as_tensor(samples).unsqueeze(0).to(device)
        audio_signal_len = torch.tensor([samples.shape[0]], device=device)
        self._features, self._features_len = preprocessor(input_signal=audio_signal, length=audio_signal_len)
        self._features = self._features.squeeze()

    def __iter__(self):
        return self

    def __next__(self):
        if not self.output:
            raise StopIteration
        last = int(self._start + self._feature_frame_len)
        flen = int(self._features_len[0])
        if last <= flen:
            frame = self._features[:, self._start: last]
            self._start = last
        else:
            frame = torch.zeros((self._features.shape[0], int(self._feature_frame_len)), dtype=torch.float32,
                                device=self._features.device)
            frame[:, 0: flen - self._start] = self._features[:, self._start: flen]
            self.output = False
        self.count += 1
        return frame


def speech_collate_fn(batch):
    """Pad 1-d signals to the longest and stack (streaming_utils.py:378-408)."""
    _, audio_lengths = zip(*batch)
    has_audio = audio_lengths[0] is not None
    if not has_audio:
        return None, None
    max_audio_len = max(audio_lengths).item()
    audio_signal = []
    for sig, sig_len in batch:
        sig_len = sig_len.item()
        if sig_len < max_audio_len:
            sig = torch.nn.functional.pad(sig, (0, max_audio_len - sig_len))
        audio_signal.append(sig)
    return torch.stack(audio_signal), torch.stack(audio_lengths)


class AudioBuffersDataLayer(torch.utils.data.IterableDataset):
    """Iterates a list of buffers as (signal, length) pairs (streaming_utils.py:411-440)."""

    def __iter__(self):
        return self

    def __next__(self):
        if self._buf_count == len(self.signal):
            raise StopIteration
        self._buf_count += 1
        return (torch.as_tensor(self.signal[self._buf_count - 1], dtype=torch.float32),
                torch.as_tensor(self.signal_shape[1], dtype=torch.int64))

    def set_signal(self, signals):
        self.signal = signals
        self.signal_shape = self.signal[0].shape
        self._buf_count = 0

    def __len__(self):
        return 1


def _to_device_frame(frame, device) -> torch.Tensor:
    return torch.as_tensor(np.asarray(frame) if not torch.is_tensor(frame) else frame,
                           dtype=torch.float32).to(device, non_blocking=True)


class FeatureFrameBufferer:
    """One stream; each call to get_buffers_batch() consumes up to batch_size consecutive chunks
    (streaming_utils.py:455-566)."""

    _EPS = 1e-5  # normalize_frame_buffers CONSTANT, streaming_utils.py:549

    def __init__(self, asr_model, frame_len=1.6, batch_size=4, total_buffer=4.0):
        self.ZERO_LEVEL_SPEC_DB_VAL = ZERO_LEVEL_SPEC_DB_VAL
        self.asr_model = asr_model
        self.sr = asr_model._cfg.sample_rate
        self.frame_len = frame_len
        timestep_duration = asr_model._cfg.preprocessor.window_stride
        self.n_frame_len = int(frame_len / timestep_duration)
        total_buffer_len = int(total_buffer / timestep_duration)
        self.n_feat = asr_model._cfg.preprocessor.features
        self.batch_size = batch_size
        self.signal_end = False
        self.frame_reader = None
        self.feature_buffer_len = total_buffer_len
        self.device = getattr(asr_model, "device", None)
        self._native = self._make_native(1)
        self.frame_buffers = []
        self.reset()

    def _make_native(self, streams):
        dev = self.device if self.device is not None and torch.device(self.device).type == "cuda" else None
        return NativeFrameBuffer(streams, self.n_feat, self.n_frame_len, self.feature_buffer_len, self._EPS, dev)

    def reset(self):
        self._native.reset()
        self.prev_char = ""
        self.unmerged = []
        self.frame_buffers = []
        self.buffered_len = 0

    @property
    def buffer(self) -> torch.Tensor:
        """The (raw, un-normalised) feature buffer, (n_feat, total_buffer_len) on the GPU."""
        return self._native.buffer[0]

    def set_frame_reader(self, frame_reader):
        self.frame_reader = frame_reader
        self.signal_end = False

    def get_batch_frames(self):
        if self.signal_end:
            return []
        batch_frames = []
        for frame in self.frame_reader:
            batch_frames.append(frame)
            if len(batch_frames) == self.batch_size:
                return batch_frames
        self.signal_end = True
        return batch_frames

    def get_buffers_batch(self) -> List[torch.Tensor]:
        batch_frames = self.get_batch_frames()
        if len(batch_frames) == 0:
            return []
        dev = self._native.device
        frames = torch.cat([_to_device_frame(f, dev) for f in batch_frames], dim=1).unsqueeze(0)
        out = self._native.step(frames)
        self.buffered_len += frames.shape[2]
        self.frame_buffers = list(out.unbind(0))
        return self.frame_buffers


class BatchedFeatureFrameBufferer(FeatureFrameBufferer):
    """B independent streams advanced in lock step (streaming_utils.py:686-818)."""

    _EPS = 1e-8  # streaming_utils.py:804

    def __init__(self, asr_model, frame_len=1.6, batch_size=4, total_buffer=4.0):
        super().__init__(asr_model, frame_len=frame_len, batch_size=batch_size, total_buffer=total_buffer)
        self._native = self._make_native(batch_size)
        self.reset()
        del self.buffered_len

    def reset(self):
        super().reset()
        self.all_frame_reader = [None for _ in range(self.batch_size)]
        self.signal_end = [False for _ in range(self.batch_size)]
        self.signal_end_index = [None for _ in range(self.batch_size)]
        self.buffer_number = 0

    @property
    def buffer(self) -> torch.Tensor:
        return self._native.buffer

    def set_frame_reader(self, frame_reader, idx):
        self.all_frame_reader[idx] = frame_reader
        self.signal_end[idx] = False
        self.signal_end_index[idx] = None

    def get_batch_frames(self):
        if all(self.signal_end):
            return []
        batch_frames = []
        for idx, frame_reader in enumerate(self.all_frame_reader):
            try:
                batch_frames.append(next(frame_reader))
            except StopIteration:
                batch_frames.append(None)
                self.signal_end[idx] = True
                if self.signal_end_index[idx] is None:
                    self.signal_end_index[idx] = self.buffer_number
        self.buffer_number += 1
        return batch_frames

    def step(self, frames: torch.Tensor, active: Optional[torch.Tensor] = None,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Device hot path: frames (B, F, n_frame) -> normalised buffers (B, F, Tbuf)."""
        return self._native.step(frames, active, out)

    def get_buffers_batch(self):
        batch_frames = self.get_batch_frames()
        if len(batch_frames) == 0:
            return []
        dev = self._native.device
        frames = torch.zeros((self.batch_size, self.n_feat, self.n_frame_len), dtype=torch.float32, device=dev)
        active = torch.zeros(self.batch_size, dtype=torch.uint8)
        for idx, f in enumerate(batch_frames):
            if f is not None:
                frames[idx] = _to_device_frame(f, dev)
                active[idx] = 1
        out = self.step(frames, active)
        self.frame_buffers = [[b] for b in out.unbind(0)]
        return self.frame_buffers
