"""CPU oracle (TEST INFRASTRUCTURE ONLY) for the buffered-streaming front end, SURVEY §8 row a-ext5.

numpy float32 restatement of the reference's per-step buffer work:
  * FeatureFrameBufferer        (nemo/collections/asr/parts/utils/streaming_utils.py:455-566)
  * BatchedFeatureFrameBufferer (streaming_utils.py:686-818)
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product path (include/cfm_stream.h) never calls it.  Pinned to the reference itself by
tests/golden/stream_*.npz (tests/golden/gen_stream_goldens.py, run on the reference classes).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np

ZERO_LEVEL_SPEC_DB_VAL = -16.635  # streaming_utils.py:469


def buffer_lengths(frame_len: float = 1.6, total_buffer: float = 4.0, window_stride: float = 0.01):
    """n_frame_len and total_buffer_len as the reference derives them (streaming_utils.py:473-476)."""
    return int(frame_len / window_stride), int(total_buffer / window_stride)


class FeatureFrameBuffererOracle:
    """One audio stream, consecutive chunks -> one normalised buffer per chunk (eps 1e-5)."""

    def __init__(self, n_feat: int, n_frame_len: int, total_buffer_len: int):
        self.n_feat, self.n_frame_len, self.total_len = n_feat, n_frame_len, total_buffer_len
        self.reset()

    def reset(self):  # streaming_utils.py:494-507
        self.buffer = np.ones([self.n_feat, self.total_len], dtype=np.float32) * ZERO_LEVEL_SPEC_DB_VAL
        self.feature_buffer = np.ones([self.n_feat, self.total_len], dtype=np.float32) * ZERO_LEVEL_SPEC_DB_VAL

    def buffers(self, frames: Sequence[np.ndarray]) -> List[np.ndarray]:
        out = []
        for frame in frames:  # get_frame_buffers, streaming_utils.py:520-528
            self.buffer[:, : -self.n_frame_len] = self.buffer[:, self.n_frame_len:]
            self.buffer[:, -self.n_frame_len:] = frame
            out.append(np.copy(self.buffer))
        consts = []
        for frame in frames:  # _update_feature_buffer + get_norm_consts_per_frame, 534-546
            w = frame.shape[1]
            self.feature_buffer[:, :-w] = self.feature_buffer[:, w:]
            self.feature_buffer[:, -w:] = frame
            consts.append((np.mean(self.feature_buffer, axis=1).reshape(self.n_feat, 1),
                           np.std(self.feature_buffer, axis=1).reshape(self.n_feat, 1)))
        return [(b - m) / (s + 1e-5) for b, (m, s) in zip(out, consts)]  # normalize_frame_buffers, 548-551


class BatchedFeatureFrameBuffererOracle:
    """B independent streams, one chunk each per step; `None` = that stream has ended (eps 1e-8)."""

    def __init__(self, batch_size: int, n_feat: int, n_frame_len: int, total_buffer_len: int):
        self.B, self.n_feat, self.n_frame_len, self.total_len = batch_size, n_feat, n_frame_len, total_buffer_len
        self.reset()

    def reset(self):  # streaming_utils.py:717-730
        shape = [self.B, self.n_feat, self.total_len]
        self.buffer = np.ones(shape, dtype=np.float32) * ZERO_LEVEL_SPEC_DB_VAL
        self.feature_buffer = np.ones(shape, dtype=np.float32) * ZERO_LEVEL_SPEC_DB_VAL

    def step(self, frames: Sequence[Optional[np.ndarray]]) -> np.ndarray:
        bufs = []
        for idx in range(self.B):  # get_frame_buffers, streaming_utils.py:757-781
            if frames[idx] is not None:
                self.buffer[idx, :, : -self.n_frame_len] = self.buffer[idx, :, self.n_frame_len:]
                self.buffer[idx, :, -self.n_frame_len:] = frames[idx]
            else:
                self.buffer[idx, :, :] *= 0.0
            bufs.append(np.copy(self.buffer[idx]))
        for idx, frame in enumerate(frames):  # _update_feature_buffer, 787-795
            if frame is not None:
                w = frame.shape[1]
                self.feature_buffer[idx, :, :-w] = self.feature_buffer[idx, :, w:]
                self.feature_buffer[idx, :, -w:] = frame
            else:
                self.feature_buffer[idx, :, :] *= 0.0
        mean = np.mean(self.feature_buffer, axis=2, keepdims=True)  # 797-801
        std = np.std(self.feature_buffer, axis=2, keepdims=True)
        return np.stack([(bufs[i] - mean[i]) / (std[i] + 1e-8) for i in range(self.B)])  # 803-806
