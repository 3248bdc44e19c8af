"""The bench's CPU baseline (oracle/conformer_torch_cpu.py, a torch-CPU restatement of the reference
encoder) against the reference-generated goldens: it must compute what the reference computes, so
that timing it is timing the reference's arithmetic.  Gate relL2 <= 1e-5 (fp32 BLAS
summation order differs from the reference's own CPU run by ~1e-7..1e-6)."""
import glob
import json
import os

import numpy as np
import pytest
import torch

import conformer_torch_cpu as TC
from conftest import GOLDEN, rel_l2
from recipe import make_state_dict

FAST = [p for p in sorted(glob.glob(os.path.join(GOLDEN, "enc_*.npz")))
        if "large17" not in os.path.basename(p) and "xl_h8" not in os.path.basename(p)]


@pytest.mark.parametrize("path", FAST, ids=[os.path.basename(p)[4:-4] for p in FAST])
def test_torch_cpu_restatement_matches_reference(path):
    z = np.load(path)
    cfg = json.loads(str(z["cfg_json"]))
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in make_state_dict(cfg, int(z["seed"])).items()}
    torch.set_num_threads(4)
    y, yl = TC.encoder_forward(torch.from_numpy(z["x"]), torch.from_numpy(z["lengths"]), sd, cfg)
    np.testing.assert_array_equal(yl.numpy(), z["y_len"])
    assert rel_l2(y.numpy(), z["y"]) <= 1e-5
