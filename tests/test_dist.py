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
