"""GPU tests of the configs[2] and configs[4] workloads at full size and of the
bench's cross-rank checks:

* the seeded 4096-square mixed batch (k = 2^u, u in 0..7, every square
  distinct) through the device-resident path, per k group: every DAH equals
  the host API's, two sampled squares per k bit-exact against the oracle;
* the block-replay rehearsal: bench.py under torch.distributed.run with 2
  ranks sharing GPU 0 (DAGPU_BENCH_SHARED_GPU=1, gloo collectives) replays
  distinct squares host-streamed and device-resident, and the sampled DAHs it
  reports match the oracle;
* the same path with ONE rank keeping its RCCL ("nccl") process group, so the
  replay's and the split square's collectives run through RCCL on this box;
* a deliberately wrong DAH (DAGPU_BENCH_CORRUPT) after the gather, inside a
  rank's own results, or in the split square makes bench.py exit non-zero;
* two host threads issuing device-resident calls on ONE context, one of them
  failing on purpose: both results intact, the failing thread reads its own
  error message (include/dagpu.h threading contract).
"""
import json
import os
import socket
import subprocess
import sys
import threading

import numpy as np
import pytest
import torch

import oracle
from celestia_da import _abi, da, synth
from celestia_da.device import DeviceSquares

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = da.Context(0)
    yield c
    c.close()


def test_mixed_batch_full_size(ctx):
    """configs[2]: 4096 distinct squares, the bench's own input (bench.mixed_batch)."""
    import bench

    ks, groups, hosts = bench.mixed_batch(ctx)
    assert len(ks) == 4096 and set(ks) == {1, 2, 4, 8, 16, 32, 64, 128}
    for ds in groups.values():
        ds.extend()
    torch.cuda.synchronize()
    for k, ds in groups.items():
        st = ds.status.cpu().numpy()
        dah = ds.dah.cpu().numpy()
        assert (st == 0).all(), k
        assert len({d.tobytes() for d in dah}) == ds.n, k  # distinct squares
        _, _, _, hdah, hst = da.extend_batch(hosts[k].reshape(-1), [k] * ds.n, ctx)
        assert (hst == 0).all() and (hdah == dah).all(), k
        for i in (0, ds.n - 1):
            _, orr, ocr, odah = oracle.extend_and_dah(hosts[k][i].reshape(k * k, 512), k, nthreads=16,
                                                      want_eds=False)
            assert dah[i].tobytes() == odah, (k, i)
            assert (ds.row_roots[i].cpu().numpy() == orr).all() and (ds.col_roots[i].cpu().numpy() == ocr).all()
    del groups
    torch.cuda.empty_cache()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_bench(args, corrupt=None, timeout=110, nccl=False):
    """bench.py under torch.distributed.run: 2 ranks sharing GPU 0 over gloo,
    or (nccl=True) ONE rank that keeps its RCCL process group, so the N > 1
    code path runs its collectives through RCCL on a one-GPU box."""
    if nccl:
        env = dict(os.environ, DAGPU_BENCH_FORCE_DIST="1", MASTER_ADDR="127.0.0.1")
        env.pop("DAGPU_BENCH_SHARED_GPU", None)
        nproc = "1"
    else:
        env = dict(os.environ, DAGPU_BENCH_SHARED_GPU="1", MASTER_ADDR="127.0.0.1")
        nproc = "2"
    if corrupt:
        env["DAGPU_BENCH_CORRUPT"] = corrupt
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", nproc,
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", nproc] + args
    return subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)


_REPLAY = ["--steps", "2", "--warmup", "1", "--batch", "8", "--replay-blocks", "40", "--no-cpu",
           "--no-split"]


def test_replay_rehearsal_two_ranks(tmp_path):
    dump = str(tmp_path / "replay.json")
    out = _run_bench(_REPLAY + ["--replay-dump", dump])
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    rep = line["block_replay"]
    assert rep["bit_exact"] is True and rep["distinct_squares"] == 40 and rep["per_rank"] == 20
    assert rep["host_streamed"]["squares_per_s"] > 0 and rep["device_resident"]["squares_per_s"] > 0
    # each rank's NUMA placement (celestia_da/numa.py), gathered from every rank
    assert len(rep["numa"]) == 2 and all(r["affinity"] and "numa_node" in r for r in rep["numa"]), rep["numa"]
    d = json.load(open(dump))
    k, seed = d["k"], d["seed"]
    assert sorted(int(b) for b in d["sampled_dah"]) == [0, 19, 20, 39]
    for b, hexdah in d["sampled_dah"].items():
        sq = synth.blob_squares(k, seed, int(b), 1)[0].reshape(k * k, 512)
        _, _, _, odah = oracle.extend_and_dah(sq, k, nthreads=16, want_eds=False)
        assert odah.hex() == hexdah, b


@pytest.mark.parametrize("corrupt", ["replay-gather", "replay-compute"])
def test_replay_corruption_is_fatal(corrupt):
    out = _run_bench(_REPLAY, corrupt=corrupt)
    assert out.returncode != 0
    assert "FATAL: block replay DAH check failed" in out.stderr
    assert not [x for x in out.stdout.splitlines() if x.startswith("{")]


def test_split_corruption_is_fatal():
    out = _run_bench(["--mode", "split", "--split-k", "16", "--steps", "1", "--warmup", "1"],
                     corrupt="split")
    assert out.returncode != 0
    assert "FATAL: split square k=16" in out.stderr


def test_rccl_path_one_rank(tmp_path):
    """The N > 1 bench path with its RCCL process group kept at one rank: the
    replay's all-gathers and max-reduces and the split square's all-to-all and
    all-gathers run through RCCL (torch backend "nccl"); outputs bit-exact."""
    dump = str(tmp_path / "replay.json")
    out = _run_bench(["--steps", "2", "--warmup", "1", "--batch", "8", "--replay-blocks", "24", "--no-cpu",
                      "--split-k", "16", "256", "--split-steps", "1", "--replay-dump", dump], nccl=True)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["block_replay"]["bit_exact"] is True
    for k in ("16", "256"):
        sp = line["split_stress"][k]
        assert sp["dah_matches_single_gpu"] is True and "nccl" in sp["collective"], sp
    d = json.load(open(dump))
    for b, hexdah in d["sampled_dah"].items():
        sq = synth.blob_squares(d["k"], d["seed"], int(b), 1)[0].reshape(d["k"] ** 2, 512)
        _, _, _, odah = oracle.extend_and_dah(sq, d["k"], nthreads=16, want_eds=False)
        assert odah.hex() == hexdah, b


def test_rccl_replay_corruption_is_fatal():
    out = _run_bench(_REPLAY, corrupt="replay-gather", nccl=True)
    assert out.returncode != 0
    assert "FATAL: block replay DAH check failed" in out.stderr


def test_two_threads_one_context(ctx):
    """Device-resident calls from two host threads on one context, each on its
    own stream; thread B fails on purpose (k = 3, then twice the widest
    supported k) on every
    iteration while thread A extends squares."""
    L = ctx._L
    too_wide = 2 * L.dagpu_max_square_width()  # rejected before anything is enqueued
    k, n = 32, 6
    ods = synth.blob_squares(k, 31337, 0, n)
    _, _, _, want, _ = da.extend_batch(ods.reshape(-1), [k] * n, ctx)
    ds = DeviceSquares(k, n, ctx=ctx)
    ds.ods.copy_(torch.from_numpy(ods))
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    errors = []
    iters = 200
    results = {}

    def worker_a():
        try:
            for _ in range(iters // 10):
                ds.extend(sa)
            sa.synchronize()
            results["a"] = ds.dah.cpu().numpy().copy()
        except Exception as e:  # pragma: no cover - reported below
            errors.append(("a", repr(e)))

    def worker_b():
        try:
            for i in range(iters):
                bad_k = 3 if i % 2 == 0 else too_wide
                rc = L.dagpu_extend_batch_device(ctx.handle, bad_k, 1, _abi.addr(ds.ods), _abi.addr(ds.eds),
                                                 _abi.addr(ds.row_roots), _abi.addr(ds.col_roots),
                                                 _abi.addr(ds.dah), _abi.addr(ds.status),
                                                 _abi.addr(ds.workspace), int(sb.cuda_stream))
                msg = L.dagpu_last_error(ctx.handle).decode()
                if bad_k == 3:
                    ok = rc == _abi.ERR_ARG and msg == "square width must be a power of two"
                else:
                    ok = rc == _abi.ERR_UNSUPPORTED and msg.startswith("square width k > ")
                if not ok:
                    errors.append(("b", i, rc, msg))
                    return
        except Exception as e:  # pragma: no cover
            errors.append(("b", repr(e)))

    ta, tb = threading.Thread(target=worker_a), threading.Thread(target=worker_b)
    ta.start()
    tb.start()
    ta.join(timeout=100)
    tb.join(timeout=100)
    assert not errors, errors
    assert (results["a"] == want).all()
    assert (ds.status.cpu().numpy() == 0).all()


def test_device_batch_in_place_matches(ctx):
    """ODS resident in Q0 of the EDS buffer (d_ods = NULL) gives the same EDS,
    roots and DAHs as a separate ODS buffer, over repeated steps."""
    k, n = 128, 6
    ods = synth.blob_squares(k, 4242, 0, n)
    a = DeviceSquares(k, n, ctx=ctx)
    b = DeviceSquares(k, n, ctx=ctx, in_place=True)
    a.load_ods(ods)
    b.load_ods(ods)
    for _ in range(2):
        a.extend()
        b.extend()
    torch.cuda.synchronize()
    assert torch.equal(a.eds, b.eds) and torch.equal(a.dah, b.dah)
    assert torch.equal(a.row_roots, b.row_roots) and torch.equal(a.col_roots, b.col_roots)
    _, _, _, hdah, _ = da.extend_batch(ods.reshape(-1), [k] * n, ctx)
    assert (b.dah.cpu().numpy() == hdah).all()


@pytest.mark.parametrize("n,slices,in_place", [
    (64, None, True),     # the headline shape: 4 slices of 16, ODS in Q0
    (67, None, True),     # uneven slices
    (70, "2", False),
    (65, "8", True),
    (64, "3", False),     # slice count that does not divide n
    (64, "1", True),      # pipeline off
    (65, "5", True),
])
def test_pipelined_device_batch(ctx, monkeypatch, n, slices, in_place):
    """The RS/NMT slice pipeline of dagpu_extend_batch_device at k = 128 under
    several slice counts (DAGPU_PIPE_SLICES, read per call), with the ODS in
    place or separate, over two steps: every DAH and root equals the host API's
    (unsliced chain), and two squares equal the oracle's."""
    k = 128
    if slices is None:
        monkeypatch.delenv("DAGPU_PIPE_SLICES", raising=False)
    else:
        monkeypatch.setenv("DAGPU_PIPE_SLICES", slices)
    ods = synth.blob_squares(k, 6400 + n, 0, n, threads=16)
    ds = DeviceSquares(k, n, ctx=ctx, in_place=in_place)
    ds.load_ods(ods)
    for _ in range(2):
        ds.extend()
    torch.cuda.synchronize()
    assert (ds.status.cpu().numpy() == 0).all()
    _, hrr, hcr, hdah, hst = da.extend_batch(ods.reshape(-1), [k] * n, ctx)
    assert (hst == 0).all()
    dah = ds.dah.cpu().numpy()
    rr, cr = ds.row_roots.cpu().numpy(), ds.col_roots.cpu().numpy()
    assert (dah == hdah).all()
    for i in range(n):
        assert (rr[i] == hrr[i]).all() and (cr[i] == hcr[i]).all(), i
    for i in (0, n - 1):
        _, orr, ocr, odah = oracle.extend_and_dah(ods[i].reshape(k * k, 512), k, nthreads=16, want_eds=False)
        assert dah[i].tobytes() == odah and (rr[i] == orr).all() and (cr[i] == ocr).all(), i
    del ds
    torch.cuda.empty_cache()


def test_two_threads_pipelined(ctx):
    """Two host threads, each with its own stream and buffers, issuing the
    sliced k = 128 device pipeline concurrently on ONE context: every result
    equals the host API's (each caller stream gets its own RS side stream)."""
    k, n = 128, 64
    out, errors = {}, []
    sets = {}
    for name, seed in (("a", 900), ("b", 901)):
        ods = synth.blob_squares(k, seed, 0, n, threads=16)
        ds = DeviceSquares(k, n, ctx=ctx, in_place=True)
        ds.load_ods(ods)
        _, _, _, want, _ = da.extend_batch(ods.reshape(-1), [k] * n, ctx)
        sets[name] = (ds, want, torch.cuda.Stream())
    torch.cuda.synchronize()

    def worker(name):
        ds, _, st = sets[name]
        try:
            for _ in range(3):
                ds.extend(st)
            st.synchronize()
            out[name] = ds.dah.cpu().numpy().copy()
        except Exception as e:  # pragma: no cover
            errors.append((name, repr(e)))

    ts = [threading.Thread(target=worker, args=(x,)) for x in sets]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not errors, errors
    for name, (ds, want, _) in sets.items():
        assert (out[name] == want).all(), name
        assert (ds.status.cpu().numpy() == 0).all()
    del sets
    torch.cuda.empty_cache()


def test_headline_check_fatal():
    """bench.py's headline bit-exact check fires on a corrupted DAH."""
    env = dict(os.environ, DAGPU_BENCH_CORRUPT="headline")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                          "--batch", "64", "--no-cpu", "--no-replay", "--no-e2e", "--no-configs"],
                         env=env, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode != 0
    assert "FATAL: headline bit-exact check (1 DAHs" in out.stderr, out.stderr[-2000:]
