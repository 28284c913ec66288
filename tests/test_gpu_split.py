"""GPU parity of the oversized-square split (celestia_da.split; split.cpp):
row/column roots and DAH bit-exact with the oracle's single-square result,
for P = 1..8 parts in one process (all-to-all as device copies) and for two
processes sharing the GPU through torch.distributed (gloo, host-staged)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import oracle  # noqa: E402
from celestia_da import da, split, synth  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = da.Context(0)
    yield c
    c.close()


_ORACLE = {}


def _want(k, seed):
    key = (k, seed)
    if key not in _ORACLE:
        ods = synth.random_blob_square(k, seed)
        _, rr, cr, dah = oracle.extend_and_dah(ods, k, nthreads=16, want_eds=False)
        _ORACLE[key] = (ods, rr.tobytes(), cr.tobytes(), dah)
    return _ORACLE[key]


@pytest.mark.parametrize("k,parts", [(2, 1), (2, 2), (8, 1), (8, 2), (8, 8), (32, 4), (128, 8),
                                     (256, 1), (256, 2), (256, 8), (512, 8), (1024, 8)])
def test_split_local_matches_oracle(ctx, k, parts):
    ods, rr, cr, dah = _want(k, 7100 + k)
    d = torch.from_numpy(np.ascontiguousarray(ods).reshape(-1)).cuda()
    got_rr, got_cr, got_dah = split.extend_split_local(d, k, parts, ctx)
    assert got_rr == rr
    assert got_cr == cr
    assert got_dah == dah


@pytest.mark.parametrize("k,parts", [(16, 1), (256, 1), (256, 4), (512, 2)])
def test_split_on_a_side_stream(ctx, k, parts):
    """advisor r05: the split's library steps only queue work on the caller's
    stream, so the torch-side steps between them run in that stream's order
    too.  A side stream held back by a GPU sleep, the ODS written on it first:
    a read on any other stream would see the old bytes or race the kernels."""
    ods, rr, cr, dah = _want(k, 7300 + k)
    side = torch.cuda.Stream()
    d = torch.zeros(ods.size, dtype=torch.uint8, device="cuda")
    host = torch.from_numpy(np.ascontiguousarray(ods).reshape(-1)).pin_memory()
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        torch.cuda._sleep(int(5e7))
        d.copy_(host, non_blocking=True)
    assert split.extend_split_local(d, k, parts, ctx, stream=side) == (rr, cr, dah)
    part = split.SplitPart(k, 1, 0, ctx, d.device)
    with torch.cuda.stream(side):
        d.zero_()
        torch.cuda._sleep(int(5e7))
        d.copy_(host, non_blocking=True)
    got_rr, got_cr, got_dah = split.extend_split_distributed(None, part, d, stream=side)
    side.synchronize()
    assert (got_rr.cpu().numpy().tobytes(), got_cr.cpu().numpy().tobytes(), got_dah.cpu().numpy().tobytes()) == \
        (rr, cr, dah)


@pytest.mark.parametrize("square", ["0", "1"])
@pytest.mark.parametrize("k", [1, 2, 16, 128, 512])
def test_split_one_part_paths(ctx, monkeypatch, k, square):
    """One part below k = 1024: the square pipeline's roots kernels (default) and
    the forest path (DAGPU_SPLIT_SQUARE=0) give the oracle's roots and DAH."""
    monkeypatch.setenv("DAGPU_SPLIT_SQUARE", square)
    ods, rr, cr, dah = _want(k, 7100 + k)
    d = torch.from_numpy(np.ascontiguousarray(ods).reshape(-1)).cuda()
    assert split.extend_split_local(d, k, 1, ctx) == (rr, cr, dah)


@pytest.mark.parametrize("mode", ["0", "1", "2"])
@pytest.mark.parametrize("k,parts", [(2, 2), (64, 1), (512, 1), (512, 4)])
def test_split_overlap_modes(ctx, monkeypatch, k, parts, mode):
    """DAGPU_SPLIT_OVERLAP (column encode on a side stream beside the leaves of
    rows 0..k-1; 0 = one stream) gives the oracle's roots and DAH; (2, 2) has
    single-leaf top trees (uniform roots addressed by shape, nothing uploaded)."""
    monkeypatch.setenv("DAGPU_SPLIT_OVERLAP", mode)
    ods, rr, cr, dah = _want(k, 7100 + k)
    d = torch.from_numpy(np.ascontiguousarray(ods).reshape(-1)).cuda()
    for _ in range(2):  # the second run reuses the side stream and pooled events
        got_rr, got_cr, got_dah = split.extend_split_local(d, k, parts, ctx)
        assert (got_rr, got_cr, got_dah) == (rr, cr, dah)


@pytest.mark.parametrize("k", [8, 512])
def test_split_distributed_one_part(ctx, k):
    """extend_split_distributed without a process group (bench.py's configs[4]
    line at one GPU): no gathers, the part's own records feed the finish, and
    the returned column roots are the caller's copy (the next square rewrites
    the part's buffers)."""
    ods, rr, cr, dah = _want(k, 7100 + k)
    d = torch.from_numpy(np.ascontiguousarray(ods).reshape(-1)).cuda()
    part = split.SplitPart(k, 1, 0, ctx, d.device)
    got = split.extend_split_distributed(None, part, d)
    torch.cuda.synchronize()
    first = tuple(t.cpu().numpy().tobytes() for t in got)
    assert first == (rr, cr, dah)
    other = torch.from_numpy(np.ascontiguousarray(_want(k, 8100 + k)[0]).reshape(-1)).cuda()
    split.extend_split_distributed(None, part, other)
    torch.cuda.synchronize()
    assert tuple(t.cpu().numpy().tobytes() for t in got) == first


def test_split_push_order(ctx):
    k = 16
    ods = np.ascontiguousarray(synth.random_blob_square(k, 5)).reshape(k, k, 512).copy()
    # swap two cells inside one row whose namespaces differ
    r = 3
    a, b = ods[r, 2].copy(), ods[r, 9].copy()
    assert a[:29].tobytes() != b[:29].tobytes()
    ods[r, 2], ods[r, 9] = b, a
    d = torch.from_numpy(ods.reshape(-1)).cuda()
    with pytest.raises(da.ErrInvalidPushOrder):
        split.extend_split_local(d, k, 4, ctx)


@pytest.mark.parametrize("parts,square", [(1, "1"), (1, "0"), (2, "1"), (4, "1")])
def test_split_column_push_order(ctx, monkeypatch, parts, square):
    """Every row sorted on its own but two rows swapped: only COLUMN trees see
    the violation.  The split must raise like the single-GPU DAH and the oracle
    (the column forest's push-order flag goes to the step's one status word;
    before round 5 it went to a per-tree slot past it and was lost)."""
    monkeypatch.setenv("DAGPU_SPLIT_SQUARE", square)
    k = 16
    ods = np.ascontiguousarray(synth.random_blob_square(k, 12)).reshape(k, k, 512).copy()
    ods[[2, 9]] = ods[[9, 2]]
    ns = ods[:, :, :29]
    assert all(ns[r, c].tobytes() <= ns[r, c + 1].tobytes() for r in range(k) for c in range(k - 1))
    assert any(ns[2, c].tobytes() > ns[3, c].tobytes() for c in range(k))
    with pytest.raises(oracle.OracleError):
        oracle.extend_and_dah(ods.reshape(-1), k)
    eds = da.extend_shares(ods.reshape(k * k, 512), ctx)
    with pytest.raises(da.ErrInvalidPushOrder):
        da.new_data_availability_header(eds)
    d = torch.from_numpy(ods.reshape(-1)).cuda()
    with pytest.raises(da.ErrInvalidPushOrder):
        split.extend_split_local(d, k, parts, ctx)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dist_worker(rank, world, port, k, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = da.Context(0)
    ods = synth.random_blob_square(k, 7100 + k)
    rows = k // world
    flat = np.ascontiguousarray(ods).reshape(-1)
    mine = torch.from_numpy(flat[rank * rows * k * 512:(rank + 1) * rows * k * 512].copy()).cuda()
    part = split.SplitPart(k, world, rank, c, mine.device)
    rr, cr, dah = split.extend_split_distributed(dist, part, mine)
    torch.cuda.synchronize()
    q.put((rank, rr.cpu().numpy().tobytes(), cr.cpu().numpy().tobytes(), dah.cpu().numpy().tobytes()))
    c.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("k,world", [(16, 2), (256, 2), (256, 4), (512, 8)])
def test_split_processes(k, world):
    """One square over `world` processes through torch.distributed (gloo,
    host-staged, all ranks on this one GPU): the RCCL code path of the 8-GPU
    stress square (bench.py --gpus 8 split_stress) with every rank's roots and
    DAH equal to the oracle's single-square result (configs[4]: k = 512, P = 8)."""
    import torch.multiprocessing as mp
    _, rr, cr, dah = _want(k, 7100 + k)
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_dist_worker, args=(r, world, port, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, got_rr, got_cr, got_dah in res:
        assert got_rr == rr and got_cr == cr and got_dah == dah, f"rank {rank}"
