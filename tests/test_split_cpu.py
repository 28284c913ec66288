"""CPU (gloo, world_size 2 and 4) tests of the collectives the oversized-square
split uses (celestia_da.split: all_to_all_blocks, all_gather_flat,
max_status) -- the exact functions the GPU path calls, here on host tensors.
Checks the block layout: after the all-to-all, rank h's receive buffer holds
rows 0..k-1 of its column slab."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from celestia_da import split


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _square(k):
    # cell (r, c) of the [Q0|Q1] rows holds a tag identifying (r, c): 4 bytes
    w = 2 * k
    a = np.zeros((k, w, 8), np.uint8)
    for r in range(k):
        for c in range(w):
            a[r, c, :4] = np.frombuffer(np.uint32(r * w + c).tobytes(), np.uint8)
    return a


def _worker(rank, world, port, k, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w, rows, W = 2 * k, k // world, 2 * k // world
    full = _square(k)
    mine = full[rank * rows:(rank + 1) * rows]            # rows R_g of [Q0|Q1]
    # pack send blocks exactly as dagpu_split_rows_device does
    send = np.concatenate([mine[:, h * W:(h + 1) * W].reshape(-1) for h in range(world)])
    recv = torch.empty(k * W * 8, dtype=torch.uint8)
    split.all_to_all_blocks(dist, recv, torch.from_numpy(send.copy()))
    slab = recv.numpy().reshape(k, W, 8)
    ok_slab = bool((slab == full[:, rank * W:(rank + 1) * W]).all())
    sub = torch.full((w * 3,), rank, dtype=torch.uint8)
    got = torch.empty(world * w * 3, dtype=torch.uint8)
    split.all_gather_flat(dist, got, sub)
    ok_gather = bool((got.view(world, -1) == torch.arange(world, dtype=torch.uint8)[:, None]).all())
    st = split.max_status(dist, torch.tensor([1 if rank == world - 1 else 0], dtype=torch.int32))
    q.put((rank, ok_slab, ok_gather, st))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,k", [(2, 8), (4, 16), (2, 2)])
def test_split_collectives_gloo(world, k):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_slab, ok_gather, st in res:
        assert ok_slab, f"rank {rank}: slab layout after all-to-all"
        assert ok_gather, f"rank {rank}: all-gather order"
        assert st == 1
