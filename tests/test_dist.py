"""N>1 orchestration of bench.py on CPU (world_size 2, gloo): the forward is replicas-only,
so the only cross-rank step is the MAX of elapsed time, and `value` counts every rank's utterances."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import bench
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        t = bench.max_over_ranks(0.5 + rank, torch.device("cpu"), True)
        # every rank sees the slowest rank's time
        q.put((rank, t, bench.job_throughput(t, world, 32, 1000, 10)))
    finally:
        dist.destroy_process_group()


def test_max_over_ranks_and_job_throughput_gloo_ws2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=5) for _ in range(world))
    for rank, t, v in res:
        assert t == pytest.approx(1.5)
        assert v == pytest.approx(2 * 32 * 1000 * 10 / 1.5)


def test_single_rank_is_identity():
    import bench
    assert bench.max_over_ranks(0.25, torch.device("cpu"), False) == 0.25
    assert bench.job_throughput(2.0, 1, 32, 1000, 4) == 32 * 1000 * 4 / 2.0


# ---- training-step data parallelism (conformer_amd.dist, conformer_amd.train) on CPU tensors ----

def _dp_worker(rank, world, port, q):
    import ctypes

    sys.path.insert(0, os.path.join(ROOT, "conformer-nemo_amd"))
    from conformer_amd import dist as cdist
    from conformer_amd.train import EncoderTrainer
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        # one flat all-reduce averages every .grad (shared parameters counted once)
        ps = [torch.nn.Parameter(torch.zeros(3, 2)), torch.nn.Parameter(torch.zeros(5))]
        ps[0].grad = torch.full((3, 2), float(rank + 1))
        ps[1].grad = torch.arange(5, dtype=torch.float32) * (rank + 1)
        bucket = cdist.allreduce_gradients(ps + [ps[0]])
        assert bucket is not None and bucket.numel() >= 11
        # SyncBatchNorm statistics callback: sums a float view of the (here CPU) workspace in place
        tr = EncoderTrainer.__new__(EncoderTrainer)
        tr._group, tr.world = None, world
        tr._ws = torch.zeros(64, dtype=torch.uint8)
        view = tr._ws[16:32].view(torch.float32)
        view.copy_(torch.tensor([1.0, 2.0, 3.0, 4.0]) * (rank + 1))
        cb = tr._make_callback()
        rc = cb(None, ctypes.c_void_p(tr._ws.data_ptr() + 16), 4, None)
        rc_bad = cb(None, ctypes.c_void_p(tr._ws.data_ptr() + 60), 4, None)   # outside the workspace
        q.put((rank, ps[0].grad.tolist(), ps[1].grad.tolist(), rc, rc_bad, view.tolist(),
               cdist.shard_batch(torch.arange(8), rank, world).tolist()))
    finally:
        dist.destroy_process_group()


def test_gradient_allreduce_and_syncbn_callback_gloo_ws2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=5) for _ in range(world))
    for rank, g0, g1, rc, rc_bad, view, shard in res:
        assert g0 == [[1.5, 1.5]] * 3                          # (1 + 2) / 2
        assert g1 == [1.5 * i for i in range(5)]
        assert rc == 0 and rc_bad != 0
        assert view == [3.0, 6.0, 9.0, 12.0]                   # summed, not averaged
        assert shard == list(range(4 * rank, 4 * rank + 4))


def _bucket_worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "conformer-nemo_amd"))
    from conformer_amd import dist as cdist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(11 + rank)
        P = [torch.nn.Parameter(torch.zeros(s)) for s in ((4, 3), (7,), (2, 2), (5,))]
        P[2].requires_grad_(False)                               # frozen: not bucketed
        head = torch.nn.Parameter(torch.zeros(6))
        table = [P[0], torch.zeros(3), None, P[1], P[2], P[3]]   # a buffer row, an empty row
        gb = cdist.GradBuckets(table, [head], average=True)
        want = [True, False, False, True, False, True]
        vals = {i: torch.randn(table[i].shape, generator=g) for i in (0, 3, 5)}
        outs = gb.native_outputs(table, want)                    # what cfm_train_backward writes into
        for i, v in vals.items():
            outs[i].copy_(v.reshape(-1))
        hv = torch.randn(6, generator=g)
        head.grad += hv                                         # autograd accumulation into the view
        gb.on_ready(3, 3)                                       # last "layer" first, as the backward does
        gb.on_ready(0, 3)
        gb.finish()
        bucketed = {i: table[i].grad.clone() for i in (0, 3, 5)}
        bucketed["head"] = head.grad.clone()
        views_ok = all(table[i].grad.data_ptr() >= gb.flat.data_ptr() for i in (0, 3, 5))
        # reference: plain .grad tensors, one flat post-backward all-reduce
        Q = [torch.nn.Parameter(torch.zeros(t.shape)) for t in (P[0], P[1], P[3], head)]
        for qp, v in zip(Q, (vals[0], vals[3], vals[5], hv)):
            qp.grad = v.clone()
        cdist.allreduce_gradients(Q)
        same = all(torch.equal(bucketed[k], qp.grad) for k, qp in zip((0, 3, 5, "head"), Q))
        q.put((rank, same, views_ok, gb.issued, P[2].grad is None))
    finally:
        dist.destroy_process_group()


def test_bucketed_overlapped_allreduce_equals_flat_gloo_ws2():
    """conformer_amd.dist.GradBuckets: grads are views of one flat buffer, buckets are all-reduced
    as grad_ready reports them (last layer first) and the rest at finish(); the averaged gradients
    are bitwise those of the flat post-backward all-reduce."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    for rank, same, views_ok, issued, frozen_none in sorted(q.get(timeout=5) for _ in range(world)):
        assert same and views_ok and frozen_none
        # P1 | P3 (rows 3..5) = flat[12:24], P0 (rows 0..2) = flat[0:12], then the head at finish
        assert issued == [(12, 24), (0, 12), (24, 30)]


def _accum_worker(rank, world, port, q, average=True, order="interleaved"):
    """Two micro-batches per optimizer step through GradBuckets (accumulation): the first
    native backward writes into the views with overlapped per-layer all-reduces, the second writes into
    the scratch and is added in; the result must equal the flat all-reduce of the summed plain grads.
    order "interleaved": fwd1 bwd1 fwd2 bwd2; "pipelined": fwd1 fwd2 bwd1 bwd2 (the second
    forward runs before the first backward's finish).  Either way a train-mode forward after the last
    backward (no backward of its own) must leave the reduced gradients unchanged."""
    sys.path.insert(0, os.path.join(ROOT, "conformer-nemo_amd"))
    from conformer_amd import dist as cdist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(5 + rank)
        P = [torch.nn.Parameter(torch.zeros(s)) for s in ((4, 3), (7,), (5,))]
        head = torch.nn.Parameter(torch.zeros(6))
        gb = cdist.GradBuckets(P, [head], average=average)
        want = [True, True, True]
        micro = [({i: torch.randn(P[i].shape, generator=g) for i in range(3)}, torch.randn(6, generator=g))
                 for _ in range(2)]
        for p in P + [head]:
            p.grad = None                                      # zero_grad(set_to_none=True)
        overlaps = []

        def backward(vals, hv):
            (head * hv).sum().backward()                       # the head's autograd accumulation into its view
            outs = gb.native_outputs(P, want)                  # what cfm_train_backward writes into
            for i, v in vals.items():
                outs[i].copy_(v.reshape(-1))                   # overwrite semantics, as the kernels
            if gb.overlap:
                gb.on_ready(0, 3)
            gb.after_backward()
            gb.finish()

        if order == "interleaved":
            for vals, hv in micro:                             # two forward/backward pairs, one step
                gb.attach()                                    # what the train forward does
                overlaps.append(gb.overlap)
                backward(vals, hv)
        else:
            for _ in micro:
                gb.attach()
                overlaps.append(gb.overlap)
            for vals, hv in micro:
                backward(vals, hv)
        got = [p.grad.clone() for p in P + [head]]
        gb.attach()                                            # a train-mode forward with no backward
        after_fwd = [p.grad.clone() for p in P + [head]]
        Q = [torch.nn.Parameter(torch.zeros(t.shape)) for t in P + [head]]
        for j, qp in enumerate(Q):
            qp.grad = sum((micro[k][0][j] if j < 3 else micro[k][1]) for k in range(2)).clone()
        cdist.allreduce_gradients(Q, average=average)
        close = all(torch.allclose(a, qp.grad, rtol=1e-6, atol=1e-6) for a, qp in zip(got, Q))
        close = close and all(torch.equal(a, b) for a, b in zip(got, after_fwd))
        # a new step (grads set to None) starts from zero again
        for p in P + [head]:
            p.grad = None
        gb.attach()
        fresh_zero = bool((gb.flat == 0).all()) and gb.overlap
        # zero_grad(set_to_none=False) keeps the views: begin_step() marks the new step explicitly
        gb.finish()
        gb.flat.fill_(3.0)
        gb.begin_step()
        gb.attach()
        fresh_zero = fresh_zero and bool((gb.flat == 0).all()) and gb.overlap
        q.put((rank, overlaps, close, fresh_zero))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("order", ["interleaved", "pipelined"])
@pytest.mark.parametrize("average", [True, False])
def test_gradient_accumulation_through_buckets_gloo_ws2(average, order):
    """with average=False the reduced part of the first backward must not come back
    world times after the second backward's all-reduce; ADVICE r04: nor in the pipelined order, and a
    forward after the last backward must not rescale the reduced gradients."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_accum_worker, args=(r, world, port, q, average, order)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    for rank, overlaps, close, fresh_zero in sorted(q.get(timeout=5) for _ in range(world)):
        assert overlaps == [True, False]
        assert close and fresh_zero
