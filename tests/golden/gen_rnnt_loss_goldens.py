"""Golden fixtures for the RNN-T loss (include/cfm_rnnt_loss.h), from the REFERENCE numpy RNN-T loss
(nemo/collections/asr/parts/numba/rnnt_loss/rnnt_numpy.py, which imports only numpy and torch, so it
is loaded unmodified).  Only where /root/reference exists:

    python tests/golden/gen_rnnt_loss_goldens.py   # writes tests/golden/rnnt_loss_*.npz

Per case: raw joint logits acts (B, T, U+1, V+1), int32 labels / lengths (ragged), per-utterance
costs from rnnt_numpy.transduce_batch on log_softmax(acts) (the CPU path of rnnt_pytorch.py:157-167
and rnnt_numpy.py:326-351), and d(sum of costs)/d(acts) by autograd through rnnt_numpy.RNNTLoss
(clamp applied by its LogSoftmaxGradModification).  The GPU numba kernels the reference runs on a
GPU (gpu_rnnt_kernel.py) compute the same quantities with the softmax folded in; numba is absent here.
"""
import importlib.util
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def load_rnnt_numpy():
    path = f"{REF}/nemo/collections/asr/parts/numba/rnnt_loss/rnnt_numpy.py"
    spec = importlib.util.spec_from_file_location("rnnt_numpy_ref", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


CASES = {
    # name: (B, T, U(labels max), V+1, blank, fastemit_lambda, clamp, seed)
    "rnnt_loss_blank_last": (3, 9, 5, 12, 11, 0.0, -1.0, 1),
    "rnnt_loss_blank0_fastemit": (2, 7, 4, 9, 0, 0.01, -1.0, 2),
    "rnnt_loss_clamp": (2, 6, 3, 33, 32, 0.0, 0.05, 3),
    "rnnt_loss_wide": (2, 13, 11, 129, 128, 0.0, -1.0, 4),
}


def main():
    rn = load_rnnt_numpy()
    for name, (B, T, U, V1, blank, lam, clamp, seed) in CASES.items():
        g = np.random.default_rng(seed)
        acts = (g.standard_normal((B, T, U + 1, V1)) * 2.0).astype(np.float32)
        act_lens = np.array([T] + list(g.integers(max(1, T // 2), T + 1, B - 1)), dtype=np.int32)
        label_lens = np.array([U] + list(g.integers(1, U + 1, B - 1)), dtype=np.int32)
        nonblank = [v for v in range(V1) if v != blank]
        labels = np.array(g.choice(nonblank, (B, U)), dtype=np.int32)
        for b in range(B):
            labels[b, label_lens[b]:] = 0
        lp = torch.log_softmax(torch.from_numpy(acts).double(), -1).float().numpy()
        costs, _ = rn.transduce_batch(lp, labels, act_lens, label_lens, blank, lam)
        a = torch.from_numpy(acts).clone().requires_grad_(True)
        loss = rn.RNNTLoss(blank=blank, fastemit_lambda=lam, clamp=clamp)
        tot = loss(a, torch.from_numpy(labels), torch.from_numpy(act_lens), torch.from_numpy(label_lens))
        tot.sum().backward()
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), acts=acts, labels=labels, act_lens=act_lens,
                            label_lens=label_lens, blank=np.int64(blank), fastemit_lambda=np.float64(lam),
                            clamp=np.float64(clamp), costs=np.array(costs, dtype=np.float64),
                            total=np.float64(tot.item()), grads=a.grad.numpy())
        print(name, np.round(costs, 4), float(tot))


if __name__ == "__main__":
    main()
