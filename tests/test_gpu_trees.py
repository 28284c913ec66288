"""GPU parity of the generic forest engine (nmt_forest.hip) through the C ABI:
batched nmt roots, the rsmt2d.Tree drop-in (wrapper trees), merkle
HashFromByteSlices and blob share commitments, against the oracle
(oracle/pyref.py restatement of nmt v0.20.0 / crypto/merkle / pkg/inclusion)
and the reference's golden commitment (pkg/inclusion/commitment_test.go:76-82)."""
import hashlib
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import oracle  # noqa: E402
import pyref  # noqa: E402
from celestia_da import da, synth, trees  # noqa: E402

pytestmark = pytest.mark.gpu

NS1 = trees.namespace_v0(b"\x01" * 10)


@pytest.fixture(scope="module")
def ctx():
    c = da.Context(0)
    yield c
    c.close()


def _sorted_pushes(rng, n, length, parity_tail=0):
    ns = sorted(bytes(rng.integers(0, 256, 29, dtype=np.uint8)) for _ in range(n - parity_tail))
    ns += [b"\xff" * 29] * parity_tail
    return [x + bytes(rng.integers(0, 256, length - 29, dtype=np.uint8)) for x in ns]


@pytest.mark.parametrize("length", [29, 30, 64, 541, 1000])
def test_nmt_roots_ragged(ctx, length):
    rng = np.random.default_rng(length)
    sizes = [0, 1, 2, 3, 4, 5, 7, 8, 9, 16, 31, 33, 64, 100]
    forest = [_sorted_pushes(rng, n, length, parity_tail=n // 3) for n in sizes]
    for ignore in (True, False):
        got = trees.nmt_roots(forest, ignore, ctx)
        want = [pyref.nmt_root_generic(t, ignore) for t in forest]
        assert got == want


def test_nmt_roots_push_order(ctx):
    rng = np.random.default_rng(3)
    good = _sorted_pushes(rng, 8, 64)
    bad = list(good)
    bad[5], bad[6] = bad[6], bad[5]
    if bad[5][:29] == bad[6][:29]:
        pytest.skip("equal namespaces")
    with pytest.raises(da.ErrInvalidPushOrder):
        trees.nmt_roots([good, bad, good], True, ctx)
    # odd-sized tree: violation at the promoted last leaf
    bad2 = good[:7]
    bad2[6] = b"\x00" * 29 + bad2[6][29:]
    with pytest.raises(da.ErrInvalidPushOrder):
        trees.nmt_roots([bad2], True, ctx)


def test_namespaced_merkle_tree_class(ctx):
    rng = np.random.default_rng(9)
    t = trees.NamespacedMerkleTree(ctx=ctx)
    pushes = _sorted_pushes(rng, 13, 100)
    for p in pushes:
        t.push(p)
    assert t.root() == pyref.nmt_root_generic(pushes)
    assert trees.NamespacedMerkleTree(ctx=ctx).root() == b"\x00" * 58 + hashlib.sha256(b"").digest()


@pytest.mark.parametrize("k", [1, 2, 4, 16])
def test_wrapper_roots_match_eds_roots(ctx, k):
    """rsmt2d drop-in: wrapper trees pushed with every EDS row and column give
    the oracle's row/column roots."""
    ods = synth.random_blob_square(k, 40 + k)
    eds, rr, cr, _ = oracle.extend_and_dah(ods, k)
    w = 2 * k
    rows = [[eds[r, c].tobytes() for c in range(w)] for r in range(w)]
    cols = [[eds[r, c].tobytes() for r in range(w)] for c in range(w)]
    got = trees.wrapper_roots(k, list(range(w)) + list(range(w)), rows + cols, ctx)
    assert b"".join(got[:w]) == rr.tobytes()
    assert b"".join(got[w:]) == cr.tobytes()
    # class form through the constructor, one tree
    t = trees.new_constructor(k, ctx)(0, 1)
    for s in rows[1]:
        t.push(s)
    assert t.root() == rr[1].tobytes()


def test_wrapper_partial_trees(ctx):
    """Roots of partially pushed wrapper trees (fewer than 2k pushes) equal the
    generic nmt over the prefixed leaves."""
    k = 4
    ods = synth.random_blob_square(k, 5)
    eds, _, _, _ = oracle.extend_and_dah(ods, k)
    forest, axes, want = [], [], []
    for axis_idx, n in [(0, 3), (1, 5), (5, 6), (7, 8), (2, 0)]:
        shares = [eds[axis_idx, c].tobytes() for c in range(n)]
        pushes = [(s[:29] if (c < k and axis_idx < k) else b"\xff" * 29) + s for c, s in enumerate(shares)]
        forest.append(shares)
        axes.append(axis_idx)
        want.append(pyref.nmt_root_generic(pushes, True))
    assert trees.wrapper_roots(k, axes, forest, ctx) == want


def test_wrapper_errors(ctx):
    with pytest.raises(da.DAError, match="pushed past"):
        trees.wrapper_roots(2, [4], [[b"\x00" * 512]], ctx)
    with pytest.raises(da.DAError, match="pushed past"):
        trees.wrapper_roots(2, [0], [[b"\x00" * 512] * 5], ctx)
    with pytest.raises(da.DAError, match="too short"):
        trees.wrapper_roots(2, [0], [[b"\x00" * 20]], ctx)
    unsorted = [b"\x05" * 512, b"\x01" * 512]
    with pytest.raises(da.ErrInvalidPushOrder):
        trees.wrapper_roots(2, [0], [unsorted], ctx)


@pytest.mark.parametrize("item_len", [0, 1, 32, 90, 91, 200])
def test_merkle_roots(ctx, item_len):
    rng = np.random.default_rng(item_len + 1)
    lists = [[bytes(rng.integers(0, 256, item_len, dtype=np.uint8)) for _ in range(n)]
             for n in [0, 1, 2, 3, 5, 8, 13, 64, 100]]
    got = trees.merkle_roots(lists, ctx)
    assert got == [pyref.rfc6962(x) for x in lists]
    # DAH hash identity: HashFromByteSlices(rowRoots || colRoots)
    ods = synth.random_blob_square(4, 1)
    _, rr, cr, dah = oracle.extend_and_dah(ods, 4)
    items = [rr[i].tobytes() for i in range(8)] + [cr[i].tobytes() for i in range(8)]
    assert trees.hash_from_byte_slices(items, ctx) == dah


def test_commitment_golden(ctx):
    got = trees.create_commitment(NS1, b"\xff" * 3 * 512, ctx=ctx)
    assert got.hex() == "3b9e78b6648ec1a241925b31da2ecb50bfc6f4ad552d3279928ca13ebeba8c2b"


def test_commitments_batch_vs_oracle(ctx):
    rng = np.random.default_rng(77)
    blobs = []
    for n in [1, 100, 478, 479, 5000, 40000, 64 * 482 + 7, 200000]:
        ns = trees.namespace_v0(bytes(rng.integers(0, 256, 10, dtype=np.uint8)))
        blobs.append((ns, bytes(rng.integers(0, 256, n, dtype=np.uint8)), 0))
    got = trees.create_commitments(blobs, ctx=ctx)
    assert got == [pyref.create_commitment(ns, d) for ns, d, _ in blobs]
    # a different threshold changes the subtree layout
    got8 = trees.create_commitments(blobs[:5], subtree_root_threshold=8, ctx=ctx)
    assert got8 == [pyref.create_commitment(ns, d, threshold=8) for ns, d, _ in blobs[:5]]
