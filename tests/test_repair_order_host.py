"""CPU check of the reasoning behind the GPU Repair's error reporting
(celestia-app_amd/csrc/dagpu.cpp plan_crossword / exact_repair, repair.hip
finalize_repair_kernel), against the oracle's sequential rsmt2d restatement
(oracle/da_oracle.c orc_repair_ex, rsmt2d v0.11.0 solveCrossword order).

The GPU does not run rsmt2d's one-axis-at-a-time loop.  It claims:
  1. the status of the batched crossword (rounds of "every decodable row" or
     "every decodable column", roots verified once at the end) equals the
     sequential loop's status;
  2. the failing axis rsmt2d reports is found by replaying the sequential
     schedule on presence bitmaps, running its attempts level by level (an
     attempt waits only for earlier attempts that filled a cell it reads), and
     judging every attempt from ONE root pass at the end;
  3. the pre-repair check's first failure is the minimum of
     4*i + {row root, col root, row parity, col parity}.
This file restates those three procedures in Python over the oracle's
decode/roots and compares them with orc_repair_ex on random squares with
random erasures and corrupted shares: status, axis, index, rebuilt axis/index
and the presence map rsmt2d leaves behind must all agree.
"""
import numpy as np
import pytest

import oracle
from celestia_da import synth

ROW, COL = 0, 1


def _axis_cells(w, ax, i):
    return [(i, j) if ax == ROW else (j, i) for j in range(w)]


def _axis_root(eds, k, ax, i):
    """Wrapper-tree root of one EDS axis (None when the nmt push order breaks)."""
    out = np.zeros(90, np.uint8)
    rc = oracle.lib().orc_axis_root(k, oracle._p(np.ascontiguousarray(eds)), ax, i, oracle._p(out))
    return None if rc else out.tobytes()


def _roots(eds, k):
    """All 2*2k axis roots of an EDS (None for an axis whose push order breaks)."""
    w = 2 * k
    return {(ax, i): _axis_root(eds, k, ax, i) for ax in (ROW, COL) for i in range(w)}


def _decode_axis(eds, pres, ax, i, k):
    cells = _axis_cells(2 * k, ax, i)
    vec = np.stack([eds[r, c] for r, c in cells])
    p = np.array([pres[r, c] for r, c in cells], np.uint8)
    vec = vec * p[:, None]
    out = oracle.decode(vec, p)
    for j, (r, c) in enumerate(cells):
        if not pres[r, c]:
            eds[r, c] = out[j]
            pres[r, c] = True


def precheck(eds, pres, k, rr, cr):
    """(status, byz) of prerepairSanityCheck in launch order, or None."""
    w = 2 * k
    want = {(ROW, i): bytes(rr[i]) for i in range(w)}
    want.update({(COL, i): bytes(cr[i]) for i in range(w)})
    for i in range(w):
        complete = [pres[i].all(), pres[:, i].all()]
        for ax in (ROW, COL):
            if complete[ax]:
                if _axis_root(eds, k, ax, i) != want[(ax, i)]:
                    return -8, [ax, i, ax, i]
        for ax in (ROW, COL):
            if complete[ax]:
                vec = eds[i] if ax == ROW else eds[:, i]
                if not np.array_equal(oracle.encode(vec[:k]), vec[k:]):
                    return -7, [ax, i, ax, i]
    return None


def batched_status(eds, pres, k, rr, cr):
    """Claim 1: the GPU's round-batched crossword and its end-of-run verify."""
    w = 2 * k
    e, p = eds.copy(), pres.copy()
    before = {(ax, i): bool(p[i].all() if ax == ROW else p[:, i].all()) for ax in (ROW, COL) for i in range(w)}
    for _ in range(4 * w + 4):
        dec = {ax: [i for i in range(w) if k <= (p[i] if ax == ROW else p[:, i]).sum() < w] for ax in (ROW, COL)}
        if not dec[ROW] and not dec[COL]:
            break
        ax = ROW if len(dec[ROW]) >= len(dec[COL]) else COL
        snap = p.copy()
        for i in dec[ax]:
            pp = snap.copy()
            _decode_axis(e, pp, ax, i, k)
            for r, c in _axis_cells(w, ax, i):
                p[r, c] = True
    roots = _roots(e, k)
    want = {(ROW, i): bytes(rr[i]) for i in range(w)}
    want.update({(COL, i): bytes(cr[i]) for i in range(w)})
    byz = incomplete = False
    for (ax, i), got in roots.items():
        if not (p[i].all() if ax == ROW else p[:, i].all()):
            incomplete = True
        elif got != want[(ax, i)] and not before[(ax, i)]:
            byz = True
    pre = precheck(eds, pres, k, rr, cr)
    if pre:
        return pre[0]
    return -7 if byz else (-6 if incomplete else 0)


def plan(pres, k):
    """plan_crossword: attempts in rsmt2d order with orthogonal completions and levels."""
    w = 2 * k
    p = pres.copy()
    miss = [(~p).sum(axis=1).astype(int), (~p).sum(axis=0).astype(int)]
    lvl = [np.full(w, -1), np.full(w, -1)]
    att = []
    while (~p).any():
        progress = False
        for i in range(w):
            for ax in (ROW, COL):
                if miss[ax][i] == 0 or w - miss[ax][i] < k:
                    continue
                L = lvl[ax][i]
                ortho = []
                for j, (r, c) in enumerate(_axis_cells(w, ax, i)):
                    if not p[r, c] and miss[1 - ax][j] == 1:
                        ortho.append(j)
                        L = max(L, lvl[1 - ax][j])
                L += 1
                for j, (r, c) in enumerate(_axis_cells(w, ax, i)):
                    if not p[r, c]:
                        p[r, c] = True
                        miss[ax][i] -= 1
                        miss[1 - ax][j] -= 1
                        lvl[1 - ax][j] = max(lvl[1 - ax][j], L)
                lvl[ax][i] = max(lvl[ax][i], L)
                att.append((ax, i, int(L), ortho))
                progress = True
        if not progress:
            break
    return att, not (~p).any()


def exact(eds, pres, k, rr, cr):
    """Claim 2: level-ordered execution + one root pass -> (byz, presence left)."""
    w = 2 * k
    att, _ = plan(pres, k)
    e, p = eds.copy(), pres.copy()
    for L in range(max([a[2] for a in att], default=-1) + 1):
        for ax in (ROW, COL):
            snap = p.copy()
            for (a, i, l, _) in att:
                if a == ax and l == L:
                    pp = snap.copy()
                    _decode_axis(e, pp, a, i, k)
                    for r, c in _axis_cells(w, a, i):
                        p[r, c] = True
    roots = _roots(e, k)
    want = {(ROW, i): bytes(rr[i]) for i in range(w)}
    want.update({(COL, i): bytes(cr[i]) for i in range(w)})
    for j, (ax, i, _, ortho) in enumerate(att):
        fail = None
        if roots[(ax, i)] != want[(ax, i)]:
            fail = [ax, i, ax, i]
        else:
            for o in ortho:
                if roots[(1 - ax, o)] != want[(1 - ax, o)]:
                    fail = [1 - ax, o, ax, i]
                    break
        if fail:
            left = pres.copy()
            for (a2, i2, _, _) in att[:j]:
                for r, c in _axis_cells(w, a2, i2):
                    left[r, c] = True
            return fail, left
    return None, None


def _case(k, rng, frac, ncorrupt, shape):
    w = 2 * k
    ods = synth.random_blob_square(k, int(rng.integers(1 << 30)))
    eds, rr, cr, _ = oracle.extend_and_dah(ods, k)
    if shape == "subgrid":
        pres = np.zeros((w, w), bool)
        pres[np.ix_(rng.choice(w, k, replace=False), rng.choice(w, k, replace=False))] = True
        extra = rng.random((w, w)) < frac
        pres |= extra
    else:
        pres = rng.random((w, w)) < frac
    bad = eds * pres[:, :, None]
    cells = np.argwhere(pres)
    for t in range(min(ncorrupt, len(cells))):
        r, c = cells[rng.integers(len(cells))]
        bad[r, c, int(rng.integers(29, 512))] ^= int(rng.integers(1, 256))
    return bad, pres, rr, cr


@pytest.mark.parametrize("k", [2, 4, 8])
def test_gpu_repair_procedures_match_sequential_oracle(k):
    rng = np.random.default_rng(1000 + k)
    seen = set()
    n = {2: 60, 4: 40, 8: 16}[k]
    for t in range(n):
        shape = "subgrid" if t % 2 else "random"
        frac = float(rng.choice([0.1, 0.3, 0.5, 0.7, 0.9]))
        bad, pres, rr, cr = _case(k, rng, frac, int(rng.integers(0, 3)), shape)
        want_rc, _, want_left, want_byz = oracle.repair_ex(bad, pres, k, rr, cr)
        got_rc = batched_status(bad, pres, k, rr, cr)
        assert got_rc == want_rc, (t, got_rc, want_rc)
        pre = precheck(bad, pres, k, rr, cr)
        if pre:
            assert [want_rc, want_byz] == [pre[0], pre[1]], t
            seen.add("pre-root" if pre[0] == -8 else "pre-parity")
        elif want_rc == -7:
            byz, left = exact(bad, pres, k, rr, cr)
            assert byz == want_byz, (t, byz, want_byz)
            assert (left == want_left.astype(bool)).all(), t
            seen.add("ortho" if byz[0] != byz[2] else "own")
        else:
            seen.add({0: "ok", -6: "unrepairable"}[want_rc])
    print(k, sorted(seen))
    assert {"ok", "own"} <= seen, seen
