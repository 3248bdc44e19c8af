"""RCCL through the C-ABI (include/cfm_comm.h): a communicator, the in-place sum+scale all-reduce,
and gradient buckets whose cfm_grad_buckets_ready_cb the native backward calls itself.  One GPU ->
world 1 (the collective is the identity, the plumbing and ordering are what is checked; the
two-rank arithmetic is covered over gloo in tests/test_dist.py / test_gpu_dp.py)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def test_native_comm_allreduce_scale():
    from conformer_amd.comm import NativeComm
    uid = NativeComm.unique_id()
    assert len(uid) == 128
    c = NativeComm(0, 1, uid, 0)
    x = torch.arange(1003, dtype=torch.float32, device="cuda")
    c.allreduce(x, 0.5)
    torch.cuda.synchronize()
    assert torch.equal(x, torch.arange(1003, dtype=torch.float32, device="cuda") * 0.5)
    fn, user = c.allreduce_cb
    assert fn.value and user.value
    c.close()


def test_native_grad_buckets_in_the_backward():
    from conformer_amd.comm import NativeComm, NativeGradBuckets
    from nemo.collections.asr.modules import ConformerEncoder
    from recipe import make_state_dict
    z = np.load(os.path.join(GOLDEN, "train_tiny_ctx.npz"))
    cfg = json.loads(str(z["cfg_json"]))
    enc = ConformerEncoder(**cfg, dropout=0.0, dropout_emb=0.0, dropout_att=0.0)
    sd = make_state_dict(cfg, int(z["seed"]))
    ref = enc.state_dict()
    enc.load_state_dict({k: torch.from_numpy(np.asarray(v)).reshape(ref[k].shape) for k, v in sd.items()})
    enc.set_compute_mode("fp32")
    enc = enc.cuda().train()
    x, ln, dy = (torch.from_numpy(z[k]).cuda() for k in ("x", "lengths", "dy"))
    buf0 = {n: b.clone() for n, b in enc.named_buffers()}
    y, _ = enc(audio_signal=x, length=ln)
    (y * dy).sum().backward()
    plain = {n: p.grad.clone() for n, p in enc.named_parameters()}
    for p in enc.parameters():
        p.grad = None
    with torch.no_grad():
        for n, b in enc.named_buffers():
            b.copy_(buf0[n])

    seen = []

    class Counting(NativeGradBuckets):
        def finish(self):
            seen.append(self.issued_count())   # ranges the native backward reported
            super().finish()

    comm = NativeComm(0, 1, NativeComm.unique_id(), 0)
    names = enc.native_param_names()
    sdv = enc.state_dict(keep_vars=True)
    gb = Counting(comm, [sdv.get(k) for k in names], [], average=True)
    enc.set_grad_buckets(gb)
    y, _ = enc(audio_signal=x, length=ln)
    (y * dy).sum().backward()
    torch.cuda.synchronize()
    assert seen == [cfg["n_layers"] + 1]
    for n, p in enc.named_parameters():
        assert torch.equal(p.grad, plain[n]), n
        assert gb.flat.data_ptr() <= p.grad.data_ptr() < gb.flat.data_ptr() + 4 * gb.numel
    enc.set_grad_buckets(None)
    del gb
    comm.close()
