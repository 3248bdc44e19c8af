"""CPU restatement (numpy) of the RNN-T joint network — TEST INFRASTRUCTURE ONLY (imported by tests/
and bench.py's cpu_baseline leg, never by the product path).

Follows RNNTJoint.joint (reference nemo/collections/asr/modules/rnnt.py:951-1008) with the module
tree of _joint_net_modules (rnnt.py:1010-1038) in eval mode (dropout = identity):
    f = enc(f) -> (B, T, 1, H);  g = pred(g) -> (B, 1, U, H);  res = joint_net(f + g)
    joint_net = [activation, (Dropout), Linear(H, V + 1)];  log_softmax over the last axis when asked.
Pinned by tests/test_joint_oracle.py against tests/golden/joint_*.npz (written by the reference).
"""
import numpy as np


def _act(x, name):
    if name == "relu":
        return np.maximum(x, 0.0)
    if name == "sigmoid":
        return 1.0 / (1.0 + np.exp(-x))
    if name == "tanh":
        return np.tanh(x)
    raise ValueError(name)


def joint_forward(enc_bdt, dec_bdu, w_enc, b_enc, w_pred, b_pred, w_out, b_out, activation="relu", log_softmax=False):
    """enc (B, H1, T), dec (B, H2, U) -> (B, T, U, V + 1) in float64 (rnnt.py:793-815 transposes first)."""
    f = np.transpose(np.asarray(enc_bdt, np.float64), (0, 2, 1)) @ np.asarray(w_enc, np.float64).T + b_enc
    g = np.transpose(np.asarray(dec_bdu, np.float64), (0, 2, 1)) @ np.asarray(w_pred, np.float64).T + b_pred
    h = _act(f[:, :, None, :] + g[:, None, :, :], activation)
    res = h @ np.asarray(w_out, np.float64).T + b_out
    if log_softmax:
        m = res.max(-1, keepdims=True)
        res = res - (m + np.log(np.exp(res - m).sum(-1, keepdims=True)))
    return res


def joint_params(z):
    """(w_enc, b_enc, w_pred, b_pred, w_out, b_out) from a golden fixture's p__* arrays."""
    last = max(int(k.split(".")[1]) for k in z.files if k.startswith("p__joint_net."))
    return (z["p__enc.weight"], z["p__enc.bias"], z["p__pred.weight"], z["p__pred.bias"],
            z[f"p__joint_net.{last}.weight"], z[f"p__joint_net.{last}.bias"])


def joint_flops(B, T, U, H1, H2, H, C):
    """Algorithmic FLOPs of one joint forward: the two projections + the (B*T*U, C, H) GEMM."""
    return 2 * B * T * H1 * H + 2 * B * U * H2 * H + 2 * B * T * U * H * C
