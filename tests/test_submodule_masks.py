"""Host logic of the standalone submodules (conformer_amd.submodule_ops.masks_to_lengths): the encoder's masks
(conformer_encoder.py:257-270) are turned back into lengths and a context window, and anything else is
refused.  CPU only."""
import numpy as np
import pytest
import torch

from conformer_amd import submodule_ops as ops


@pytest.mark.parametrize("ctx", [(-1, -1), (8, 4), (0, 0), (3, -1), (-1, 2)])
def test_masks_round_trip(ctx):
    lengths = torch.tensor([37, 20, 1], dtype=torch.int32)
    T = 37
    att = ops.canonical_att_mask(lengths, T, *ctx)
    pad = torch.arange(T).unsqueeze(0) >= lengths.unsqueeze(-1)
    got, c = ops.masks_to_lengths(att, pad, 3, T, torch.device("cpu"))
    assert got.tolist() == lengths.tolist()
    assert c == ctx
    got2, c2 = ops.masks_to_lengths(att, None, 3, T, torch.device("cpu"))   # lengths from att_mask alone
    assert got2.tolist() == lengths.tolist() and c2 == ctx


def test_canonical_mask_shape():
    lengths = torch.tensor([5, 3], dtype=torch.int32)
    att = ops.canonical_att_mask(lengths, 5, -1, -1)
    assert att[1, 0, 3] and not att[1, 0, 2] and att[1, 4, 0]


def test_golden_masks_are_canonical(golden_dir):
    """The fixtures' masks (built as the reference encoder builds them) are recognised."""
    import os
    for case in ("layer", "layer_ctx_ln"):
        z = np.load(os.path.join(golden_dir, f"sub_{case}.npz"))
        att, pad = torch.from_numpy(z["att_mask"]), torch.from_numpy(z["pad_mask"])
        lengths, ctx = ops.masks_to_lengths(att, pad, att.shape[0], att.shape[1], torch.device("cpu"))
        assert lengths.tolist() == z["lengths"].tolist() and ctx == tuple(int(c) for c in z["ctx"])


def test_arbitrary_masks_refused():
    lengths = torch.tensor([6, 6], dtype=torch.int32)
    att = ops.canonical_att_mask(lengths, 6, -1, -1).clone()
    att[0, 2, 4] = True
    with pytest.raises(NotImplementedError):
        ops.masks_to_lengths(att, None, 2, 6, torch.device("cpu"))
    pad = torch.tensor([[False, True, False, False, False, False], [False] * 6])
    with pytest.raises(NotImplementedError):
        ops.masks_to_lengths(None, pad, 2, 6, torch.device("cpu"))
