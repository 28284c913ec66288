"""Started Repairs (dagpu_repair_start / dagpu_repair_join): the call returns
at once and a library worker thread makes the crossword's host decisions on a
stream of its own; the join makes a stream wait for the repair.  Outputs
(status, every EDS byte, the presence map) must equal dagpu_repair_batch_device's
for the same inputs; slices started back to back run side by side; handles
are checked; a context closed with repairs in flight stays correct."""
import numpy as np
import pytest
import torch

from celestia_da import _abi, da, synth
from celestia_da.device import DeviceSquares

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = da.Context(0)
    yield c
    c.close()


def _setup(ctx, k, n, seed, kind="subgrid"):
    w = 2 * k
    ds = DeviceSquares(k, n, ctx=ctx)
    ds.load_ods(synth.blob_squares(k, seed, 0, n))
    ds.extend()
    torch.cuda.synchronize()
    rng = np.random.default_rng(seed)
    pres = np.zeros((n, w, w), np.uint8)
    for i in range(n):
        if kind == "subgrid":
            pres[i][np.ix_(rng.choice(w, k, replace=False), rng.choice(w, k, replace=False))] = 1
        else:  # random density: some squares unrepairable
            pres[i] = rng.random((w, w)) < float(rng.choice([0.3, 0.6, 0.8]))
    pres_t = torch.from_numpy(pres.reshape(n, -1)).cuda()
    ref = ds.eds.clone()
    damaged = (ds.eds.view(n, w * w, 512) * pres_t.view(n, w * w, 1)).view(n, -1).clone()
    return ds, pres_t, ref, damaged


def _inputs(ds, pres_t, damaged):
    ds.eds.copy_(damaged)
    present = pres_t.clone()
    status = torch.full((ds.n,), 99, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    return present, status


@pytest.mark.parametrize("k,n,kind", [(16, 24, "random"), (128, 16, "subgrid")])
def test_started_equals_batch_call(ctx, k, n, kind):
    ds, pres_t, ref, damaged = _setup(ctx, k, n, 900 + k, kind)
    present, status = _inputs(ds, pres_t, damaged)
    ds.repair(present, status, ds.repair_workspace())
    torch.cuda.synchronize()
    eds1, p1, st1 = ds.eds.clone(), present.clone(), status.clone()
    present, status = _inputs(ds, pres_t, damaged)
    s = torch.cuda.Stream()
    h = ds.repair_start(present, status, ds.repair_workspace(), stream=s)
    ds.repair_join(h, stream=s)
    with torch.cuda.stream(s):
        snapshot = ds.eds.clone()  # queued behind the repair on the joined stream
    s.synchronize()
    assert torch.equal(status, st1) and torch.equal(present, p1)
    assert torch.equal(ds.eds, eds1) and torch.equal(snapshot, eds1)
    if kind == "subgrid":
        assert (st1.cpu().numpy() == 0).all() and torch.equal(eds1, ref)
    else:
        assert set(st1.cpu().numpy().tolist()) <= {0, _abi.ERR_UNREPAIRABLE}


def test_start_returns_at_once_and_slices_run_side_by_side(ctx):
    # Structural, not wall-clock: the caller's stream is held by a GPU sleep
    # queued before the starts, so no repair kernel can have run when the three
    # starts return; the sleep's completion event must still be pending then
    # (a start that waited for its repair could only return after it).
    k, n = 128, 64
    ds, pres_t, ref, damaged = _setup(ctx, k, n, 4242)
    present, status = _inputs(ds, pres_t, damaged)
    cut = [0, 16, 40, 64]  # uneven slices
    wss = [ds.repair_workspace(cut[j + 1] - cut[j]) for j in range(3)]
    s = torch.cuda.current_stream()
    torch.cuda._sleep(int(2e8))
    held = torch.cuda.Event()
    held.record(s)
    hs = [ds.repair_start(present, status, wss[j], first=cut[j], count=cut[j + 1] - cut[j]) for j in range(3)]
    assert not held.query(), "a start waited for device work queued before it"
    for h in hs:
        ds.repair_join(h)
    torch.cuda.synchronize()
    assert torch.equal(ds.eds, ref) and (status.cpu().numpy() == 0).all() and bool(present.all())


def test_worker_failure_reaches_the_joining_thread(ctx, monkeypatch):
    # the worker's message is re-raised on the caller's thread at the join,
    # and the slot is free again afterwards
    k, n = 8, 2
    ds, pres_t, ref, damaged = _setup(ctx, k, n, 32)
    present, status = _inputs(ds, pres_t, damaged)
    monkeypatch.setenv("DAGPU_TEST_WORKER_FAIL", "1")
    h = ds.repair_start(present, status, ds.repair_workspace())
    with pytest.raises(da.DAError, match="injected worker failure"):
        ds.repair_join(h)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == _abi.ERR_DEVICE).all()
    monkeypatch.delenv("DAGPU_TEST_WORKER_FAIL")
    present, status = _inputs(ds, pres_t, damaged)
    h = ds.repair_start(present, status, ds.repair_workspace())
    ds.repair_join(h)
    torch.cuda.synchronize()
    assert torch.equal(ds.eds, ref) and (status.cpu().numpy() == 0).all()


def test_joins_from_threads_run_side_by_side(ctx):
    # two host threads each start and join their own repair on one context;
    # a join holds the slot table only to claim its slot (advisor r04)
    import threading

    k, n = 128, 16
    ds, pres_t, ref, damaged = _setup(ctx, k, n, 515)
    present, status = _inputs(ds, pres_t, damaged)
    errs = []

    def run(j):
        try:
            h = ds.repair_start(present, status, ds.repair_workspace(8), first=8 * j, count=8)
            ds.repair_join(h)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=run, args=(j,)) for j in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    torch.cuda.synchronize()
    assert not errs, errs
    assert torch.equal(ds.eds, ref) and (status.cpu().numpy() == 0).all()


def test_handles_are_checked(ctx):
    k, n = 8, 2
    ds, pres_t, ref, damaged = _setup(ctx, k, n, 31)
    present, status = _inputs(ds, pres_t, damaged)
    h = ds.repair_start(present, status, ds.repair_workspace())
    ds.repair_join(h)
    with pytest.raises(da.DAError, match="already joined"):
        ds.repair_join(h)  # a handle joins once
    with pytest.raises(da.DAError, match="unknown"):
        ds.repair_join(h + (1 << 20))
    torch.cuda.synchronize()
    assert torch.equal(ds.eds, ref)


def test_many_started_repairs(ctx):
    # 40 repairs started on one square each (40 worker threads at once), joined
    # in a mixed order; then 40 more, reusing the slots
    k, n = 8, 40
    ds, pres_t, ref, damaged = _setup(ctx, k, n, 77)
    for _ in range(2):
        present, status = _inputs(ds, pres_t, damaged)
        wss = [ds.repair_workspace(1) for _ in range(n)]
        hs = [ds.repair_start(present, status, wss[i], first=i, count=1) for i in range(n)]
        for h in hs[1::2] + hs[0::2][::-1]:
            ds.repair_join(h)
        torch.cuda.synchronize()
        assert torch.equal(ds.eds, ref) and (status.cpu().numpy() == 0).all() and bool(present.all())


def test_close_with_repairs_started():
    c = da.Context(0)
    k, n = 128, 32
    ds, pres_t, ref, damaged = _setup(c, k, n, 99)
    present, status = _inputs(ds, pres_t, damaged)
    ds.repair_start(present, status, ds.repair_workspace())
    c.close()  # joins the worker and drains its stream
    torch.cuda.synchronize()
    assert torch.equal(ds.eds, ref) and (status.cpu().numpy() == 0).all()


def test_started_repair_holds_its_tensors(ctx):
    """A started repair's tensors stay allocated until its join, even when the
    caller passes temporaries (the workspace below): the DeviceSquares wrapper
    holds them.  Before round 5 the temporary went back to the caching
    allocator at once, and a same-size allocation right after the start (here
    filled with junk while the repair runs) could be handed the repair's own
    workspace."""
    k, n = 128, 8
    ds, pres_t, ref, damaged = _setup(ctx, k, n, 616)
    present, status = _inputs(ds, pres_t, damaged)
    h = ds.repair_start(present, status, ds.repair_workspace())
    junk = torch.empty((ctx._L.dagpu_repair_workspace_size(k, n),), dtype=torch.uint8, device="cuda")
    junk.fill_(0xA5)
    ds.repair_join(h)
    torch.cuda.synchronize()
    assert torch.equal(ds.eds, ref) and (status.cpu().numpy() == 0).all()
    assert h not in ds._held
