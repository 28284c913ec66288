"""GPU Repair error reports against the oracle's sequential rsmt2d restatement
(oracle/da_oracle.c orc_repair_ex): status code, ErrByzantineData axis and
index, the rebuilt axis whose shares rsmt2d attaches, and the presence map
rsmt2d leaves behind, for random erasures with corrupted shares (own-root and
orthogonal-root failures, byzantine-and-unrepairable squares), the pre-repair
check's ordering, k = 128 (bit-sliced GF(2^8) decoder), k = 256 (GF(2^16)) and
the device batch API (dagpu_repair_batch_device_ex).  Bit-exact comparisons."""
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


def _damage(k, rng, frac, ncorrupt, subgrid, seed):
    w = 2 * k
    ods = synth.random_blob_square(k, seed)
    eds, rr, cr, _ = oracle.extend_and_dah(ods, k, nthreads=8)
    pres = rng.random((w, w)) < frac
    if subgrid:
        pres[np.ix_(rng.choice(w, k, replace=False), rng.choice(w, k, replace=False))] = True
    bad = eds * pres[:, :, None]
    cells = np.argwhere(pres)
    for _ in range(min(ncorrupt, len(cells))):
        r, c = cells[rng.integers(len(cells))]
        bad[r, c, int(rng.integers(29, 512))] ^= int(rng.integers(1, 256))
    return eds, bad, pres, rr, cr


def _gpu_repair(ctx, bad, pres, rr, cr):
    try:
        fixed, p = da.repair(bad, pres, rr, cr, ctx)
        return 0, fixed, p, [-1] * 4, ""
    except da.DAError as e:
        return e.code, e.eds, e.present, e.byz, str(e)


def _check_one(ctx, k, eds, bad, pres, rr, cr, what):
    orc, ofixed, opres, obyz = oracle.repair_ex(bad, pres, k, rr, cr)
    rc, fixed, p, byz, msg = _gpu_repair(ctx, bad, pres, rr, cr)
    assert rc == orc, (what, rc, orc, msg)
    if rc == 0:
        assert (fixed == eds).all() and p.all(), what
        return "ok"
    if rc == _abi.ERR_UNREPAIRABLE:
        assert byz == [-1] * 4 and msg == "failed to solve data square", what
        return "unrepairable"
    assert byz == obyz, (what, byz, obyz)
    axis = ("row", "col")[byz[0]]
    if rc == _abi.ERR_BAD_ROOTS:
        assert msg.startswith(f"bad root input: {axis} {byz[1]} expected ["), (what, msg)
        # rsmt2d returns before the crossword: presence is the input's
        assert (p == pres).all() and (opres.astype(bool) == pres).all(), what
        return "bad-roots"
    assert msg == f"byzantine {axis}: {byz[1]}", (what, msg)
    # the square as rsmt2d leaves it: cells of the attempts before the failing one
    assert (p == opres.astype(bool)).all(), what
    if byz[0] != byz[2] or byz[1] != byz[3]:
        kind = "ortho"
    elif (pres == opres.astype(bool)).all() and (pres[byz[1]] if byz[0] == 0 else pres[:, byz[1]]).all():
        kind = "pre-parity"
    else:
        kind = "own"
    # every present cell holds the bytes the oracle holds (committed or original)
    assert (fixed[p] == ofixed[p]).all(), what
    return kind


@pytest.mark.parametrize("k", [2, 4, 8, 16])
def test_random_damage_matches_oracle(ctx, k):
    rng = np.random.default_rng(7000 + k)
    seen = set()
    for t in range({2: 40, 4: 40, 8: 30, 16: 16}[k]):
        frac = float(rng.choice([0.2, 0.4, 0.55, 0.7, 0.9]))
        eds, bad, pres, rr, cr = _damage(k, rng, frac, int(rng.integers(0, 3)), t % 2 == 1, 100 * k + t)
        seen.add(_check_one(ctx, k, eds, bad, pres, rr, cr, (k, t, frac)))
    assert {"ok", "own"} <= seen, seen


def test_orthogonal_failure_is_reported_as_the_orthogonal_axis(ctx):
    """Search seeded cases until one fails on a newly completed orthogonal
    axis (own root fine, the completed column's root not), then check it."""
    k = 4
    rng = np.random.default_rng(4242)
    for t in range(400):
        eds, bad, pres, rr, cr = _damage(k, rng, float(rng.choice([0.5, 0.6, 0.7])), 1, False, 9000 + t)
        orc, _, _, obyz = oracle.repair_ex(bad, pres, k, rr, cr)
        if orc == _abi.ERR_BYZANTINE and (obyz[0], obyz[1]) != (obyz[2], obyz[3]):
            assert _check_one(ctx, k, eds, bad, pres, rr, cr, t) == "ortho"
            return
    pytest.fail("no orthogonal-root failure in 400 seeded cases")


def test_byzantine_and_unrepairable_square(ctx):
    """A corrupted share in a decodable row of a square that cannot be
    completed: rsmt2d reaches the corrupted row before it stalls."""
    k = 8
    w = 2 * k
    eds, rr, cr, _ = oracle.extend_and_dah(synth.random_blob_square(k, 31), k)
    pres = np.zeros((w, w), bool)
    pres[3, :k + 2] = True            # row 3 decodable
    pres[:k - 1, 10] = True           # column 10 one short: nothing completes the square
    bad = eds * pres[:, :, None]
    bad[3, 1, 100] ^= 0x20
    assert _check_one(ctx, k, eds, bad, pres, rr, cr, "byz+unrep") == "own"
    clean = eds * pres[:, :, None]
    assert _check_one(ctx, k, eds, clean, pres, rr, cr, "unrep") == "unrepairable"


def test_precheck_order(ctx):
    """prerepairSanityCheck: the first of (row root, col root, row parity,
    col parity) over i ascending, whatever the kinds further on."""
    k = 4
    w = 2 * k
    eds, rr, cr, _ = oracle.extend_and_dah(synth.random_blob_square(k, 5), k)
    pres = np.ones((w, w), bool)
    pres[w - 1, w - 1] = False
    # (a) column 1's root wrong, row 3 parity-inconsistent (roots commit to it)
    inc = eds.copy()
    inc[3, w - 2, 60] ^= 1            # parity cell of row 3 (and of column w-2)
    irr, icr = oracle.compute_roots(inc, k)
    wrong_c = icr.copy()
    wrong_c[1, 80] ^= 1
    assert _check_one(ctx, k, inc, inc, pres, irr, wrong_c, "a") == "bad-roots"
    # (b) row 5's root wrong, column 2 parity-inconsistent: column 2 comes first
    inc2 = eds.copy()
    inc2[w - 3, 2, 60] ^= 1           # parity row w-3, column 2 (a Q2 cell)
    irr2, icr2 = oracle.compute_roots(inc2, k)
    wrong_r = irr2.copy()
    wrong_r[5, 80] ^= 1
    rc, _, p, byz, _ = _gpu_repair(ctx, inc2, pres, wrong_r, icr2)
    orc, _, opres, obyz = oracle.repair_ex(inc2, pres, k, wrong_r, icr2)
    assert rc == orc == _abi.ERR_BYZANTINE and byz == obyz == [1, 2, 1, 2]
    # a pre-repair failure leaves the square as given (rsmt2d never reaches
    # solveCrossword): the missing cell stays missing
    assert (p == pres).all() and (opres.astype(bool) == pres).all()
    # (c) the same with a decodable gap pattern: many missing cells, presence untouched
    pres3 = np.ones((w, w), bool)
    pres3[6, [0, 1, 3]] = False       # gaps off row 5 and column 2 (both still complete)
    pres3[:2, 7] = False
    rc, _, p, byz, _ = _gpu_repair(ctx, inc2 * pres3[:, :, None], pres3, irr2, icr2)
    orc, _, opres, obyz = oracle.repair_ex(inc2 * pres3[:, :, None], pres3, k, irr2, icr2)
    assert rc == orc == _abi.ERR_BYZANTINE and byz == obyz == [1, 2, 1, 2]
    assert (p == pres3).all() and (opres.astype(bool) == pres3).all()


def test_k128_byzantine_matches_oracle(ctx):
    """Bit-sliced k = 128 decoder under the maximal erasure pattern with one
    corrupted share."""
    k = 128
    rng = np.random.default_rng(128)
    eds, bad, pres, rr, cr = _damage(k, rng, 0.0, 1, True, 12800)
    assert _check_one(ctx, k, eds, bad, pres, rr, cr, "k128") in ("own", "ortho")


def test_k256_gf16_byzantine_matches_oracle(ctx):
    """GF(2^16) decoder (parity unpinned: no reference vector above k = 128)."""
    k = 256
    w = 2 * k
    eds, rr, cr, _ = oracle.extend_and_dah(synth.random_blob_square(k, 256), k, nthreads=16)
    rng = np.random.default_rng(256)
    pres = np.zeros((w, w), bool)
    pres[np.ix_(rng.choice(w, k, replace=False), rng.choice(w, k, replace=False))] = True
    bad = eds * pres[:, :, None]
    r, c = np.argwhere(pres)[17]
    bad[r, c, 400] ^= 0x81
    assert _check_one(ctx, k, eds, bad, pres, rr, cr, "k256") in ("own", "ortho")


def test_device_batch_ex_matches_oracle(ctx):
    """dagpu_repair_batch_device_ex on 24 k = 16 squares with mixed outcomes:
    per square status, byz and presence equal the oracle's; repaired squares
    equal the extended ones."""
    k, n = 16, 24
    w = 2 * k
    rng = np.random.default_rng(1616)
    ds = DeviceSquares(k, n, ctx=ctx)
    host = synth.blob_squares(k, 1616, 0, n)
    ds.load_ods(host)
    ds.extend()
    torch.cuda.synchronize()
    full = ds.eds.cpu().numpy().reshape(n, w, w, 512)
    rr, cr = ds.row_roots.cpu().numpy(), ds.col_roots.cpu().numpy()
    bads, press = [], []
    for i in range(n):
        pres = rng.random((w, w)) < float(rng.choice([0.3, 0.5, 0.7]))
        if i % 3 == 0:
            pres[np.ix_(rng.choice(w, k, replace=False), rng.choice(w, k, replace=False))] = True
        bad = full[i] * pres[:, :, None]
        cells = np.argwhere(pres)
        for _ in range(int(rng.integers(0, 3))):
            r, c = cells[rng.integers(len(cells))]
            bad[r, c, int(rng.integers(29, 512))] ^= 0x44
        bads.append(bad)
        press.append(pres)
    ds.eds.copy_(torch.from_numpy(np.stack(bads).reshape(n, -1)))
    present = torch.from_numpy(np.stack(press).reshape(n, -1).astype(np.uint8)).cuda()
    status = torch.full((n,), -99, dtype=torch.int32, device="cuda")
    byz = torch.full((n, 4), -99, dtype=torch.int32, device="cuda")
    ds.repair(present, status, ds.repair_workspace(), byz=byz)
    torch.cuda.synchronize()
    st, bz = status.cpu().numpy(), byz.cpu().numpy()
    got_eds = ds.eds.cpu().numpy().reshape(n, w, w, 512)
    got_p = present.cpu().numpy().reshape(n, w, w).astype(bool)
    kinds = set()
    for i in range(n):
        orc, ofixed, opres, obyz = oracle.repair_ex(bads[i], press[i], k, rr[i], cr[i])
        assert st[i] == orc, (i, st[i], orc)
        assert list(bz[i]) == obyz, (i, list(bz[i]), obyz)
        if orc == 0:
            assert (got_eds[i] == full[i]).all() and got_p[i].all(), i
        elif orc == _abi.ERR_BYZANTINE:
            assert (got_p[i] == opres.astype(bool)).all(), i
            assert (got_eds[i][got_p[i]] == ofixed[got_p[i]]).all(), i
        kinds.add(int(orc))
    assert 0 in kinds and _abi.ERR_BYZANTINE in kinds, kinds
