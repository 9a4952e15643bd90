"""The N>1 bench path on CPU: world_size-2 gloo ranks, max-over-ranks timing and the whole-job
throughput formula of bench.py (one process per GPU on the box; gloo here)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    elapsed = bench.max_over_ranks(1.0 + rank, world, torch.device("cpu"))
    dist.barrier()
    q.put((rank, elapsed))
    dist.destroy_process_group()


def test_max_over_ranks_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == {0: 2.0, 1: 2.0}


def test_job_throughput_weak_scaling():
    # 10 M reads x 120 positions per rank, 4 ranks, 5 steps in 2 s
    assert bench.job_throughput(1.2e9, 4, 5, 2.0) == pytest.approx(1.2e10)
    assert bench.max_over_ranks(3.5, 1, None) == 3.5
