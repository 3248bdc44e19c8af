"""The numpy joint restatement (oracle/joint_oracle.py) against the reference's own RNNTJoint outputs
(tests/golden/joint_*.npz, written by gen_joint_goldens.py)."""
import ast
import glob
import os

import numpy as np
import pytest

import joint_oracle as J
from conftest import GOLDEN, rel_l2

FILES = sorted(glob.glob(os.path.join(GOLDEN, "joint_*.npz")))


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
def test_joint_oracle_matches_reference(path):
    z = np.load(path)
    jn = dict(ast.literal_eval(str(z["jointnet"])))
    for lsm, key in ((False, "logits"), (True, "logprobs")):
        got = J.joint_forward(z["enc"], z["dec"], *J.joint_params(z), activation=jn["activation"], log_softmax=lsm)
        assert got.shape == z[key].shape
        assert rel_l2(got, z[key]) < 2e-6, key


def test_joint_flops_cfg4():
    # BASELINE config 4 synthetic joint: B=16, T'=400, U+1=101, V+1=1025, H=640: the joint GEMM is
    # ~848 GFLOP (SURVEY a-ext4), plus 5.5 GFLOP of enc/pred projections
    assert abs(J.joint_flops(16, 400, 101, 512, 640, 640, 1025) / 1e9 - 853.6) < 0.5
