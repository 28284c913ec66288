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


_WORKER_FAIL_SCRIPT = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from celestia_da import _abi, da, synth
from celestia_da.device import DeviceSquares
import os
ctx = da.Context(0)
k, n, w = 8, 2, 16
ds = DeviceSquares(k, n, ctx=ctx)
ds.load_ods(synth.blob_squares(k, 32, 0, n))
ds.extend()
torch.cuda.synchronize()
ref = ds.eds.clone()
pres = np.zeros((n, w, w), np.uint8)
pres[:, :k, :k] = 1
pres_t = torch.from_numpy(pres.reshape(n, -1)).cuda()
damaged = (ds.eds.view(n, w * w, 512) * pres_t.view(n, w * w, 1)).view(n, -1).clone()
def inputs():
    ds.eds.copy_(damaged)
    st = torch.full((n,), 99, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    return pres_t.clone(), st
present, status = inputs()
os.environ["DAGPU_TEST_WORKER_FAIL"] = "1"
h = ds.repair_start(present, status, ds.repair_workspace())
del os.environ["DAGPU_TEST_WORKER_FAIL"]  # the start call took it already
try:
    ds.repair_join(h)
    print("JOIN_OK")
except da.DAError as e:
    print("JOIN_ERR", e)
torch.cuda.synchronize()
print("STATUS", status.cpu().numpy().tolist())
present, status = inputs()
h = ds.repair_start(present, status, ds.repair_workspace())
ds.repair_join(h)
torch.cuda.synchronize()
print("AFTER", bool(torch.equal(ds.eds, ref)), status.cpu().numpy().tolist())
ctx.close()
"""


@pytest.mark.parametrize("lib", ["libdagpu_test.so", "libdagpu.so"])
def test_worker_failure_reaches_the_joining_thread(lib):
    """The test build (DAGPU_TEST_HOOKS, libdagpu_test.so) injects a worker
    failure: its message is re-raised on the caller's thread at the join, the
    statuses say ERR_DEVICE, and the slot serves the next repair.  The product
    library carries no such hook: the same environment repairs normally."""
    import os
    import subprocess
    import sys

    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "celestia-app_amd")
    env = dict(os.environ, DAGPU_LIB=os.path.join(pkg, lib))
    r = subprocess.run([sys.executable, "-c", _WORKER_FAIL_SCRIPT, pkg], env=env, capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    out = r.stdout
    if lib == "libdagpu_test.so":
        assert "JOIN_ERR" in out and "injected worker failure" in out, out
        assert f"STATUS {[_abi.ERR_DEVICE] * 2}" in out, out
    else:
        assert "JOIN_OK" in out and "STATUS [0, 0]" in out, out
    assert "AFTER True [0, 0]" in out, out


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


def test_join_on_another_stream_keeps_tensors_until_it(ctx):
    """A repair started on the default stream and joined on a side stream: the
    wrapper releases its held tensors with record_stream(join stream), so the
    caching allocator does not hand the workspace to a same-size allocation on
    the default stream (filled with junk at once, while the repair still runs on
    the library's stream) before the joined stream has passed the repair."""
    k, n = 128, 16
    ds, pres_t, ref, damaged = _setup(ctx, k, n, 617)
    for _ in range(2):
        present, status = _inputs(ds, pres_t, damaged)
        side = torch.cuda.Stream()
        h = ds.repair_start(present, status, ds.repair_workspace())  # temporary workspace
        ds.repair_join(h, stream=side)
        junk = torch.empty((ctx._L.dagpu_repair_workspace_size(k, n),), dtype=torch.uint8, device="cuda")
        junk.fill_(0x5A)
        side.synchronize()
        torch.cuda.synchronize()
        assert torch.equal(ds.eds, ref) and (status.cpu().numpy() == 0).all()
        del junk


_KEY_COLLIDE_SCRIPT = r"""
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np, torch
from celestia_da import da, synth
from celestia_da.device import DeviceSquares
ctx = da.Context(0)
rng = np.random.default_rng(77)
for k, n in ((8, 3), (128, 4), (256, 2), (512, 1), (1024, 1)):
    w = 2 * k
    ds = DeviceSquares(k, n, ctx=ctx)
    ds.load_ods(synth.blob_squares(k, 40 + k, 0, n))
    ds.extend()
    torch.cuda.synchronize()
    ref = ds.eds.clone()
    # every row and column its own erasure pattern (70 % of the cells given):
    # a candidate head accepted without the flag check would decode with
    # another vector's locators
    pres = (rng.random((n, w, w)) < 0.7).astype(np.uint8)
    pres_t = torch.from_numpy(pres.reshape(n, -1)).cuda()
    ds.eds.copy_((ds.eds.view(n, w * w, 512) * pres_t.view(n, w * w, 1)).view(n, -1))
    status = torch.full((n,), 99, dtype=torch.int32, device="cuda")
    ds.repair(pres_t.clone(), status, ds.repair_workspace())
    torch.cuda.synchronize()
    print("K", k, bool(torch.equal(ds.eds, ref)), status.cpu().numpy().tolist())
    del ds
    torch.cuda.empty_cache()
ctx.close()
"""


@pytest.mark.parametrize("lib", ["libdagpu_test.so", "libdagpu.so"])
def test_locator_key_collisions_fall_back_to_own_heads(lib):
    """Every locator key equal (the test build's DAGPU_TEST_KEY_COLLIDE): each
    vector's candidate head is its square's first vector, and the flag-by-flag
    check inside the locator kernels (GF(2^8), GF(2^16) fold, k = 1024) must
    send every vector with another erasure pattern to its own locators -- the
    Repairs of squares whose every axis has its own pattern stay bit-exact.
    The product library ignores the variable."""
    import os
    import subprocess
    import sys

    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "celestia-app_amd")
    env = dict(os.environ, DAGPU_LIB=os.path.join(pkg, lib), DAGPU_TEST_KEY_COLLIDE="1")
    r = subprocess.run([sys.executable, "-c", _KEY_COLLIDE_SCRIPT, pkg], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    for k, n in ((8, 3), (128, 4), (256, 2), (512, 1), (1024, 1)):
        assert f"K {k} True {[0] * n}" in r.stdout, r.stdout
