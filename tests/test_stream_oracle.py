"""CPU: the streaming-buffer oracle (oracle/stream_oracle.py) reproduces the reference bufferers'
own outputs (tests/golden/stream_*.npz, made by gen_stream_goldens.py on the reference classes)."""
import os

import numpy as np

import stream_oracle as SO
from conftest import GOLDEN


def test_buffer_lengths_match_reference():
    z = np.load(os.path.join(GOLDEN, "stream_single.npz"))
    assert SO.buffer_lengths(1.6, 4.0) == (int(z["n_frame"]), int(z["total_len"])) == (160, 400)
    zb = np.load(os.path.join(GOLDEN, "stream_batched.npz"))
    assert SO.buffer_lengths(0.3, 0.8) == (int(zb["n_frame"]), int(zb["total_len"]))


def test_single_stream_oracle_matches_reference():
    z = np.load(os.path.join(GOLDEN, "stream_single.npz"))
    o = SO.FeatureFrameBuffererOracle(z["frames"].shape[1], int(z["n_frame"]), int(z["total_len"]))
    got, i = [], 0
    for nb in z["per_batch"]:
        got += o.buffers(list(z["frames"][i:i + nb]))
        i += nb
    np.testing.assert_array_equal(np.stack(got), z["buffers"])


def test_batched_oracle_matches_reference():
    z = np.load(os.path.join(GOLDEN, "stream_batched.npz"))
    B = z["frames"].shape[1]
    o = SO.BatchedFeatureFrameBuffererOracle(B, z["frames"].shape[2], int(z["n_frame"]), int(z["total_len"]))
    for s in range(z["steps"].shape[0]):
        fr = [z["frames"][s, i] if z["active"][s, i] else None for i in range(B)]
        np.testing.assert_array_equal(o.step(fr), z["steps"][s])
    # ended streams emit exact zeros
    assert (z["steps"][-1] == 0).all() and not z["active"][-1].any()
