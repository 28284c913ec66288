"""Multi-process (gloo, world_size 2, CPU) tests of the N>1 path: square
sharding, DAH gathering and max-over-ranks timing, with the oracle as the
per-square compute (no GPU)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from celestia_da import replay, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dah(i):
    k = 2 ** (i % 4)
    _, _, _, dah = oracle.extend_and_dah(synth.random_blob_square(k, 3000 + i), k, want_eds=False)
    return dah


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dahs = replay.replay(n, _dah, rank, world, dist)
    # bench.py's max-over-ranks timing reduction
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put((dahs, float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    for n in (0, 1, 7, 8, 8192):
        for world in (1, 2, 3, 8):
            idx = [i for r in range(world) for i in replay.shard_range(n, r, world)]
            assert idx == list(range(n))
            sizes = [len(replay.shard_range(n, r, world)) for r in range(world)]
            assert max(sizes) - min(sizes) <= 1


def test_replay_two_ranks_gloo():
    n, world = 10, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    dahs, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == 2.0
    assert dahs == [_dah(i) for i in range(n)]
