"""GPU share inclusion proofs (celestia_da.proof; pkg/proof/proof.go:58-165).

The nmt and celestia-core modules are not in this image, so proof bytes are
checked by the structure the reference verifiers rely on (parity unpinned for
the node ORDER): every NMT range proof must re-derive its row root from the
proven shares (nmt VerifyInclusion, restated below with hashlib), and every
row proof must re-derive the data root (merkle Proof.Verify, restated)."""
import hashlib
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import pyref  # noqa: E402
from celestia_da import da, proof, trees  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = da.Context(0)
    yield c
    c.close()


def _verify_nmt(nodes, width, start, end, leaves):
    """Recompute the root of a full tree of `width` leaves from the range's
    leaf nodes and the proof nodes (maximal disjoint subtrees, left to right)."""
    it = iter(nodes)
    lv = iter(leaves)

    def rec(lo, hi):
        if hi <= start or lo >= end:
            return next(it)
        if hi - lo == 1:
            return next(lv)
        mid = (lo + hi) // 2
        return pyref.node(rec(lo, mid), rec(mid, hi))

    root = rec(0, width)
    assert next(it, None) is None and next(lv, None) is None
    return root


def _verify_merkle(p, leaf_item):
    """crypto/merkle computeHashFromAunts."""
    def h_leaf(x):
        return hashlib.sha256(b"\x00" + x).digest()

    def h_inner(a, b):
        return hashlib.sha256(b"\x01" + a + b).digest()

    def rec(index, total, leaf, aunts):
        if total == 1:
            assert not aunts
            return leaf
        split = 1
        while split * 2 < total:
            split *= 2
        if index < split:
            left = rec(index, split, leaf, aunts[:-1])
            return h_inner(left, aunts[-1])
        right = rec(index - split, total - split, leaf, aunts[:-1])
        return h_inner(aunts[-1], right)

    assert p.leaf_hash == h_leaf(leaf_item)
    return rec(p.index, p.total, p.leaf_hash, p.aunts)


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 13, 256, 300])
def test_proofs_from_byte_slices(ctx, n):
    rng = np.random.default_rng(n)
    items = [bytes(rng.integers(0, 256, 90, dtype=np.uint8)) for _ in range(n)]
    root, proofs = proof.proofs_from_byte_slices(items, ctx)
    assert root == pyref.rfc6962(items)
    for i, p in enumerate(proofs):
        assert p.total == n and p.index == i
        assert _verify_merkle(p, items[i]) == root


def test_range_proof_nodes_shape():
    assert proof.range_proof_nodes(8, 0, 8) == []
    assert proof.range_proof_nodes(8, 0, 4) == [(1, 1)]
    assert proof.range_proof_nodes(8, 3, 5) == [(2, 0), (3, 2), (3, 5), (2, 3)]
    assert proof.range_proof_nodes(4, 1, 2) == [(2, 0), (1, 1)]


def _square(k, seed):
    from test_gpu_inclusion import _square_with_blobs
    return _square_with_blobs(k, [3, 9, 40] if k >= 8 else [2, 3], seed)


@pytest.mark.parametrize("k", [4, 8, 32])
def test_share_inclusion_proofs(ctx, k):
    ods, placed = _square(k, k)
    shares = [ods[i].tobytes() for i in range(k * k)]
    eds = da.extend_shares(ods, ctx)
    dah = da.new_data_availability_header(eds)
    data_root = dah.hash()
    w = 2 * k
    cases = [(start, start + len(trees.split_blob(ns, d)), ns) for start, ns, d in placed]
    cases.append((0, k * k, b"\x00" * 29))          # the whole square
    cases.append((k - 1, k + 1, b"\x00" * 29))      # straddles a row boundary
    for start, end, ns in cases:
        sp = proof.new_share_inclusion_proof(shares, ns, (start, end), ctx)
        assert sp.data == shares[start:end]
        assert sp.namespace_id == ns[1:] and sp.namespace_version == ns[0]
        rp = sp.row_proof
        assert rp.start_row == start // k and rp.end_row == (end - 1) // k
        cursor = 0
        for i, (nmtp, row_root, mp) in enumerate(zip(sp.share_proofs, rp.row_roots, rp.proofs)):
            row = rp.start_row + i
            assert row_root == dah.row_roots[row]
            leaves = [pyref.leaf(s[:29], s) for s in sp.data[cursor:cursor + nmtp.end - nmtp.start]]
            cursor += nmtp.end - nmtp.start
            assert _verify_nmt(nmtp.nodes, w, nmtp.start, nmtp.end, leaves) == row_root
            assert _verify_merkle(mp, row_root) == data_root
        assert cursor == len(sp.data)


@pytest.mark.parametrize("k", [4, 8, 32])
def test_share_proofs_validate_with_library_verifiers(ctx, k):
    """ShareProof.Validate (RowProof.Validate + VerifyProof through
    dagpu_merkle_verify / dagpu_nmt_verify_inclusion) accepts every
    single-namespace proof and rejects tampered ones; a range spanning several
    namespaces does not verify (VerifyInclusion prepends one namespace)."""
    ods, placed = _square(k, k + 100)
    shares = [ods[i].tobytes() for i in range(k * k)]
    eds = da.extend_shares(ods, ctx)
    data_root = da.new_data_availability_header(eds).hash()
    for start, ns, d in placed:
        end = start + len(trees.split_blob(ns, d))
        assert proof.parse_namespace(shares, start, end) == ns
        sp = proof.new_share_inclusion_proof(shares, ns, (start, end), ctx)
        sp.validate(data_root)
        with pytest.raises(da.DAError):
            sp.validate(bytes(32))
        bad = list(sp.data)
        bad[0] = bad[0][:200] + bytes([bad[0][200] ^ 1]) + bad[0][201:]
        with pytest.raises(da.DAError, match="share proof failed"):
            proof.ShareProof(bad, sp.share_proofs, sp.namespace_id, sp.row_proof, sp.namespace_version).validate(
                data_root)
        with pytest.raises(da.DAError):
            proof.ShareProof(sp.data[1:], sp.share_proofs, sp.namespace_id, sp.row_proof,
                             sp.namespace_version).validate(data_root)
    whole = proof.new_share_inclusion_proof(shares, b"\x00" * 29, (0, k * k), ctx)
    with pytest.raises(da.DAError, match="share proof failed"):
        whole.validate(data_root)


def test_tx_inclusion_proofs(ctx):
    """proof.NewTxInclusionProof over a square built from txs: every normal tx
    and every PFB is proven under the square's data root."""
    import random
    from celestia_da import square as sq
    from test_square_host import normal_txs, random_blob_txs
    rng = random.Random(21)
    txs = normal_txs(rng, 6, size=700) + random_blob_txs(rng, 5, 3000, blobs_per=2)
    square = sq.construct(txs)
    k = square.size()
    ods = np.frombuffer(b"".join(square.square_bytes()), np.uint8).reshape(k * k, 512)
    data_root = da.new_data_availability_header(da.extend_shares(ods, ctx)).hash()
    for i in range(len(txs)):
        sp = proof.new_tx_inclusion_proof(txs, i, ctx=ctx)
        sp.validate(data_root)
    with pytest.raises(da.DAError):
        proof.new_tx_inclusion_proof(txs, len(txs), ctx=ctx)
