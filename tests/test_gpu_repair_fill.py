"""Repair fill route and deferral (dagpu.cpp repair_device, repair.hip
repair_plan_kernel): with DAGPU_REPAIR_FILL on (the default) a decodable axis
whose data half is complete is re-encoded instead of decoded, one whose parity
half is complete is rebuilt by the reverse transform (EncodeArgs.reverse), and
decodes of axes i >= k wait when every axis i < k is being rebuilt.  All must leave
exactly what the plain decoder schedule leaves -- status, every EDS byte and
the presence map -- for consistent squares, corrupted given shares (also in
the parity half of a filled axis or the data half of a reverse-filled one,
which sends it back to the decoder),
unrepairable patterns and a committed square that is not a codeword square
(the deferred-axis check and the re-run without deferral).  Statuses are also
checked against the oracle's rsmt2d restatement."""
import numpy as np
import pytest
import torch

import oracle
from celestia_da import _abi, da, synth
from celestia_da.device import DeviceSquares

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = da.Context(0)
    yield c
    c.close()


def _pattern(kind, k, rng):
    w = 2 * k
    p = np.zeros((w, w), bool)
    if kind == "subgrid":  # the maximal erasure pattern (configs[3])
        p[np.ix_(rng.choice(w, k, replace=False), rng.choice(w, k, replace=False))] = True
    elif kind == "subgrid_top":  # kept rows are the data rows
        p[np.ix_(np.arange(k), rng.choice(w, k, replace=False))] = True
    elif kind == "q0":  # the original data only: every axis is filled
        p[:k, :k] = True
    elif kind == "q3":  # parity of parity only (bench --mode repair): reverse row and column fills
        p[k:, k:] = True
    elif kind == "subgrid_right":  # kept columns are the parity columns
        p[np.ix_(rng.choice(w, k, replace=False), np.arange(k, w))] = True
    elif kind == "right_half":  # every row reverse-fillable, some data shards given (compared)
        p[:, k:] = True
        p[:, :k] = rng.random((w, k)) < 0.3
    elif kind == "left_half":  # every row decodable by its data half, some parity given
        p[:, :k] = True
        p[:, k:] = rng.random((w, k)) < 0.3
    elif kind == "rows_plus":  # data rows over-determined, parity rows exactly k: deferral + check
        for r in range(w):
            p[r, rng.choice(w, k + max(1, min(5, k // 2)) if r < k else k, replace=False)] = True
    elif kind == "unrepairable":
        p[np.ix_(rng.choice(w, k, replace=False), rng.choice(w, k, replace=False))] = True
        r, c = np.argwhere(p)[0]
        p[r, :] = False
        p[:, c] = False
    else:  # random density
        p = rng.random((w, w)) < float(kind)
    return p


def _corrupt(eds, p, how, rng, k):
    """Flip one byte of a given share: any, or one in the parity half of a row
    whose data half is complete (the fill route compares it)."""
    if how is None:
        return
    cells = np.argwhere(p)
    if how == "parity_half":
        cells = [(r, c) for r, c in cells if c >= k and p[r, :k].all()] or list(cells)
    elif how == "data_half":  # a given data share of a row whose parity half is complete
        cells = [(r, c) for r, c in cells if c < k and p[r, k:].all()] or list(cells)
    r, c = cells[rng.integers(len(cells))]
    eds[r, c, rng.integers(512)] ^= 1 << int(rng.integers(8))


def _run(ctx, k, eds_dmg, pres, rr, cr, monkeypatch, fill):
    monkeypatch.setenv("DAGPU_REPAIR_FILL", "1" if fill else "0")
    n = len(eds_dmg)
    w = 2 * k
    ds = DeviceSquares(k, n, ctx=ctx)
    ds.eds.copy_(torch.from_numpy(eds_dmg.reshape(n, -1)))
    ds.row_roots.copy_(torch.from_numpy(rr))
    ds.col_roots.copy_(torch.from_numpy(cr))
    present = torch.from_numpy(pres.reshape(n, -1).astype(np.uint8)).cuda()
    status = torch.full((n,), -99, dtype=torch.int32, device="cuda")
    ds.repair(present, status, ds.repair_workspace())
    torch.cuda.synchronize()
    out = (status.cpu().numpy(), ds.eds.cpu().numpy().reshape(n, w, w, 512), present.cpu().numpy().reshape(n, w, w))
    del ds
    torch.cuda.empty_cache()
    return out


def _case(ctx, monkeypatch, k, specs, seed, oracle_check=True, bad_encoding=()):
    rng = np.random.default_rng(seed)
    n = len(specs)
    w = 2 * k
    ods = synth.blob_squares(k, seed, 0, n, threads=16)
    eds_l, rr_l, cr_l, dmg_l, pres_l = [], [], [], [], []
    for i, (kind, corrupt) in enumerate(specs):
        eds, rr, cr, _ = oracle.extend_and_dah(ods[i].reshape(k * k, 512), k, nthreads=16)
        p = _pattern(kind, k, rng)
        if i in bad_encoding:
            # commit to a square that is not a codeword square: garbage in the
            # cells of Q3 that are missing, roots computed over it
            q3 = np.zeros((w, w), bool)
            q3[k:, k:] = True
            eds = eds.copy()
            eds[q3 & ~p] = rng.integers(0, 256, (int((q3 & ~p).sum()), 512), dtype=np.uint8)
            rr, cr = oracle.compute_roots(eds, k, nthreads=16)
        dmg = eds * p[:, :, None]
        _corrupt(dmg, p, corrupt, rng, k)
        eds_l.append(eds); rr_l.append(rr); cr_l.append(cr); dmg_l.append(dmg); pres_l.append(p)
    dmg = np.stack(dmg_l)
    pres = np.stack(pres_l)
    rr, cr = np.stack(rr_l), np.stack(cr_l)
    st1, e1, p1 = _run(ctx, k, dmg, pres, rr, cr, monkeypatch, True)
    st0, e0, p0 = _run(ctx, k, dmg, pres, rr, cr, monkeypatch, False)
    for i, spec in enumerate(specs):
        assert st1[i] == st0[i], (i, spec, st1[i], st0[i])
        assert (p1[i] == p0[i]).all(), (i, spec)
        assert (e1[i] == e0[i]).all(), (i, spec)
        if st1[i] == 0:
            assert (e1[i] == eds_l[i]).all() and p1[i].all(), (i, spec)
        if oracle_check:
            orc, _ = oracle.repair(dmg_l[i], pres_l[i], k, rr_l[i], cr_l[i])
            assert st1[i] == orc, (i, spec, st1[i], orc)
    return st1


@pytest.mark.parametrize("k", [4, 16, 64])
def test_fill_equals_decoder_small(ctx, monkeypatch, k):
    specs = [("subgrid", None), ("subgrid_top", None), ("q0", None), ("left_half", None),
             ("rows_plus", None), ("0.5", None), ("0.65", None), ("0.8", None),
             ("subgrid", "any"), ("left_half", "parity_half"), ("rows_plus", "any"),
             ("unrepairable", None), ("unrepairable", "any"), ("q0", "any"),
             ("q3", None), ("subgrid_right", None), ("right_half", None), ("q3", "any"),
             ("right_half", "data_half")]
    st = _case(ctx, monkeypatch, k, specs, 300 + k)
    assert st[0] == 0 and st[2] == 0 and st[9] == _abi.ERR_BYZANTINE
    assert (st[14:17] == 0).all() and st[18] == _abi.ERR_BYZANTINE


def test_fill_equals_decoder_k128(ctx, monkeypatch):
    """The bit-sliced k = 128 fill (forward and reverse pair lists) and decoder."""
    specs = [("subgrid", None), ("subgrid", None), ("subgrid_top", None), ("q0", None),
             ("left_half", None), ("rows_plus", None), ("0.6", None), ("subgrid", "any"),
             ("left_half", "parity_half"), ("rows_plus", "any"), ("unrepairable", None),
             ("q3", None), ("subgrid_right", None), ("right_half", None), ("right_half", "data_half"),
             ("q3", "any")]
    st = _case(ctx, monkeypatch, 128, specs, 1280, oracle_check=False)
    assert (st[:7] == 0).all() and st[8] == _abi.ERR_BYZANTINE
    assert (st[11:14] == 0).all() and st[14] == _abi.ERR_BYZANTINE


@pytest.mark.parametrize("k", [16, 128])
def test_fill_bad_encoding(ctx, monkeypatch, k):
    """Committed squares that are not codeword squares (garbage in the missing
    Q3 cells, roots over it): the same outcome with and without the shortcut,
    including the deferred-axis check and the re-run without deferral."""
    specs = [("subgrid", None), ("rows_plus", None), ("rows_plus", "any"), ("left_half", None),
             ("subgrid_top", None), ("0.6", None), ("right_half", None), ("subgrid_right", None)]
    _case(ctx, monkeypatch, k, specs, 4400 + k, oracle_check=(k <= 16), bad_encoding=range(len(specs)))


def test_fill_equals_decoder_gf16(ctx, monkeypatch):
    """GF(2^16) (k = 256): the register-resident fill encoder (both directions) and decoder."""
    specs = [("subgrid", None), ("left_half", "parity_half"), ("rows_plus", None), ("q3", None),
             ("right_half", "data_half")]
    st = _case(ctx, monkeypatch, 256, specs, 2560, oracle_check=False)
    assert st[0] == 0 and st[1] == _abi.ERR_BYZANTINE and st[2] == 0
    assert st[3] == 0 and st[4] == _abi.ERR_BYZANTINE


def test_fill_equals_decoder_gf16_k512(ctx, monkeypatch):
    """k = 512 (the M = 512 register-resident encoder, reverse direction): the
    EDS comes from the library's own extend (the oracle is too slow at this
    size; the GF(2^16) encode is checked against it in tests/test_gpu_gf16.py),
    then the maximal Q3-only pattern and a right half with a corrupted given
    data share are repaired with and without the shortcut."""
    k, n = 512, 2
    w = 2 * k
    rng = np.random.default_rng(5120)
    ds = DeviceSquares(k, n, ctx=ctx, in_place=True)
    ds.load_ods(synth.blob_squares(k, 5120, 0, n, threads=16))
    ds.extend()
    torch.cuda.synchronize()
    eds = ds.eds.cpu().numpy().reshape(n, w, w, 512)
    rr, cr = ds.row_roots.cpu().numpy(), ds.col_roots.cpu().numpy()
    del ds
    torch.cuda.empty_cache()
    pres = np.stack([_pattern("q3", k, rng), _pattern("right_half", k, rng)])
    dmg = eds * pres[..., None]
    _corrupt(dmg[1], pres[1], "data_half", rng, k)
    st1, e1, p1 = _run(ctx, k, dmg, pres, rr, cr, monkeypatch, True)
    st0, e0, p0 = _run(ctx, k, dmg, pres, rr, cr, monkeypatch, False)
    assert list(st1) == list(st0) == [0, _abi.ERR_BYZANTINE]
    assert (e1 == e0).all() and (p1 == p0).all()
    assert (e1[0] == eds[0]).all() and p1[0].all()


@pytest.mark.parametrize("k", [8, 32])
def test_fill_random_sweep(ctx, monkeypatch, k):
    """54 squares, each a random pattern kind and density, half of them with
    one corrupted given share: the shortcut equals the plain schedule byte for
    byte, and every status equals the oracle's."""
    rng = np.random.default_rng(9000 + k)
    kinds = ["subgrid", "subgrid_top", "q0", "left_half", "rows_plus", "unrepairable",
             "q3", "subgrid_right", "right_half"]
    specs = []
    for i in range(54):
        kind = kinds[i % len(kinds)] if i < 27 else f"{rng.uniform(0.35, 0.9):.2f}"
        corrupt = ("any", "parity_half", None, "data_half")[i % 4]
        specs.append((kind, corrupt))
    _case(ctx, monkeypatch, k, specs, 9100 + k)


def test_two_threads_repair_one_context(ctx):
    """Two host threads repairing their own k = 64 batches on their own streams
    through ONE context (each call takes its own page-locked mailbox for the
    round counters): both batches come back bit-exact."""
    import threading

    k, n = 64, 16
    w = 2 * k
    sets, out, errors = {}, {}, []
    for name, seed in (("a", 1700), ("b", 1701)):
        rng = np.random.default_rng(seed)
        ds = DeviceSquares(k, n, ctx=ctx, in_place=True)
        ds.load_ods(synth.blob_squares(k, seed, 0, n, threads=16))
        ds.extend()
        torch.cuda.synchronize()
        ref = ds.eds.clone()
        pres = np.stack([_pattern("subgrid", k, rng) for _ in range(n)]).reshape(n, -1).astype(np.uint8)
        present = torch.from_numpy(pres).cuda()
        ds.eds.copy_((ds.eds.view(n, w * w, 512) * present.view(n, w * w, 1)).view(n, -1))
        status = torch.full((n,), -99, dtype=torch.int32, device="cuda")
        sets[name] = (ds, ref, present, status, ds.repair_workspace(), torch.cuda.Stream())
    torch.cuda.synchronize()

    def worker(name):
        ds, _, present, status, ws, st = sets[name]
        try:
            ds.repair(present, status, ws, stream=st)
            st.synchronize()
            out[name] = status.cpu().numpy().copy()
        except Exception as e:  # pragma: no cover
            errors.append((name, repr(e)))

    ts = [threading.Thread(target=worker, args=(x,)) for x in sets]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not errors, errors
    for name, (ds, ref, present, _, _, _) in sets.items():
        assert (out[name] == 0).all(), name
        assert torch.equal(ds.eds, ref) and bool((present == 1).all()), name
    del sets
    torch.cuda.empty_cache()


@pytest.mark.parametrize("k", [8, 16])
def test_fill_classification_mixed_halves(ctx, k):
    """The plan's classification itself (dagpu_repair_stats), not just the
    bytes: even rows keep k/2 data + k/2 parity shards (decoder), odd rows
    their parity half (reverse fill).  At k = 8 the row counter's 16-flag loads
    would straddle index k and count parity flags as data, sending the mixed
    rows to the forward fill; the counts must be the same at both
    k.  Round 1 (rows): k reverse fills, k/2 decodes of rows < k, k/2 deferred
    decodes of rows >= k; round 2 (columns): the k columns that are not already
    complete are re-encoded from their complete data half."""
    w = 2 * k
    eds, rr, cr, _ = oracle.extend_and_dah(synth.random_blob_square(k, 808 + k), k)
    p = np.zeros((w, w), bool)
    h = k // 2
    for r in range(w):
        if r % 2 == 0:
            p[r, :h] = True
            p[r, k:k + h] = True
        else:
            p[r, k:] = True
    fixed, pres = da.repair(eds * p[:, :, None], p, rr, cr, ctx)
    assert pres.all() and (fixed == eds).all()
    assert ctx.repair_stats() == {"rounds": 2, "fills": k, "reverse_fills": k, "decodes": h, "deferred": h}
