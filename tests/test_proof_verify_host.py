"""The library's host proof verifiers (dagpu_nmt_verify_inclusion = nmt
Proof.VerifyInclusion, dagpu_merkle_verify = crypto/merkle Proof.Verify) on
trees and proofs built by the oracle's pure-Python restatement (pyref).  No
GPU: these are host functions of libdagpu.so."""
import os
import random
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import pyref  # noqa: E402
from celestia_da import da, proof  # noqa: E402


def _nmt_levels(leaf_nodes):
    levels = [list(leaf_nodes)]
    while len(levels[-1]) > 1:
        lv = levels[-1]
        levels.append([pyref.node(lv[i], lv[i + 1]) for i in range(0, len(lv), 2)])
    return levels


def _nmt_proof(levels, width, start, end):
    depth = len(levels) - 1
    return [levels[depth - d][p] for d, p in proof.range_proof_nodes(width, start, end)]


@pytest.mark.parametrize("width", [1, 2, 4, 8, 16, 64])
def test_nmt_verify_inclusion_valid_and_tampered(width):
    rng = random.Random(width)
    # sorted namespaces, a run of 4 equal ones in the middle
    nss = sorted(b"\x00" * 19 + rng.randbytes(10) for _ in range(width))
    lo = width // 3
    for i in range(lo, min(width, lo + 4)):
        nss[i] = nss[lo]
    shares = [nss[i] + rng.randbytes(483) for i in range(width)]
    levels = _nmt_levels([pyref.leaf(s[:29], s) for s in shares])
    root = levels[-1][0]
    for start in range(width):
        for end in range(start + 1, width + 1):
            if len({s[:29] for s in shares[start:end]}) != 1:
                continue
            ns = shares[start][:29]
            p = proof.NMTProof(start, end, _nmt_proof(levels, width, start, end))
            assert p.verify_inclusion(ns, shares[start:end], root), (start, end)
            bad = bytearray(shares[start])
            bad[100] ^= 1
            assert not p.verify_inclusion(ns, [bytes(bad)] + shares[start + 1:end], root)
            assert not proof.NMTProof(start, end + 1, p.nodes).verify_inclusion(ns, shares[start:end], root)
            if p.nodes:
                assert not proof.NMTProof(start, end, p.nodes[1:] + p.nodes[:1] if len(p.nodes) > 1
                                          else [bytes(90)]).verify_inclusion(ns, shares[start:end], root)
                assert not proof.NMTProof(start, end, p.nodes[:-1]).verify_inclusion(ns, shares[start:end], root)
            assert not p.verify_inclusion(ns, shares[start:end], bytes(90))


def test_nmt_verify_parity_half_and_degenerate_ranges():
    """A row of an EDS: Q0 half namespaced, parity half 0xFF (ignoreMax rule)."""
    rng = random.Random(5)
    k = 8
    q0 = sorted(b"\x00" * 19 + rng.randbytes(10) + rng.randbytes(483) for _ in range(k))
    par = [rng.randbytes(512) for _ in range(k)]
    leaves = [pyref.leaf(s[:29], s) for s in q0] + [pyref.leaf(b"\xff" * 29, s) for s in par]
    levels = _nmt_levels(leaves)
    root = levels[-1][0]
    p = proof.NMTProof(k, 2 * k, _nmt_proof(levels, 2 * k, k, 2 * k))
    assert p.verify_inclusion(b"\xff" * 29, par, root)
    p0 = proof.NMTProof(2, 3, _nmt_proof(levels, 2 * k, 2, 3))
    assert p0.verify_inclusion(q0[2][:29], [q0[2]], root)
    assert not proof.NMTProof(3, 3, p0.nodes).verify_inclusion(q0[2][:29], [], root)
    assert not proof.NMTProof(-1, 1, p0.nodes).verify_inclusion(q0[2][:29], [q0[2]] * 2, root)


def _aunts(items, i):
    def rec(lo, hi):
        if hi - lo == 1:
            return []
        split = 1
        while split * 2 < hi - lo:
            split *= 2
        if i < lo + split:
            return rec(lo, lo + split) + [pyref.rfc6962(items[lo + split:hi])]
        return rec(lo + split, hi) + [pyref.rfc6962(items[lo:lo + split])]
    return rec(0, len(items))


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 13, 32])
def test_merkle_verify(n):
    import hashlib
    rng = random.Random(n)
    items = [rng.randbytes(90) for _ in range(n)]
    root = pyref.rfc6962(items)
    for i in range(n):
        p = proof.MerkleProof(n, i, hashlib.sha256(b"\x00" + items[i]).digest(), _aunts(items, i))
        p.verify(root, items[i])
        with pytest.raises(da.DAError):
            p.verify(root, items[(i + 1) % n] + b"x")
        with pytest.raises(da.DAError):  # a flipped aunt bit, or an aunt too many at n == 1
            aunts = [bytes([p.aunts[0][0] ^ 1]) + p.aunts[0][1:]] + p.aunts[1:] if p.aunts else [bytes(32)]
            proof.MerkleProof(n, i, p.leaf_hash, aunts).verify(root, items[i])
        with pytest.raises(da.DAError):
            proof.MerkleProof(n, -1, p.leaf_hash, p.aunts).verify(root, items[i])
        # Proof.Verify compares the proof's own LeafHash with leafHash(leaf)
        with pytest.raises(da.DAError, match="invalid leaf hash"):
            proof.MerkleProof(n, i, bytes(32), p.aunts).verify(root, items[i])


def test_merkle_verify_max_aunts():
    import hashlib
    leaf = b"x"
    p = proof.MerkleProof(2, 0, hashlib.sha256(b"\x00" + leaf).digest(), [bytes(32)] * 101)
    with pytest.raises(da.DAError, match="no more than 100 aunts"):
        p.verify(bytes(32), leaf)


def test_parse_namespace():
    ns_a, ns_b = b"\x00" * 28 + b"\x01", b"\x00" * 28 + b"\x02"
    raw = [ns_a + bytes(483)] * 3 + [ns_b + bytes(483)] * 2
    assert proof.parse_namespace(raw, 0, 3) == ns_a
    assert proof.parse_namespace(raw, 3, 5) == ns_b
    for a, b in ((-1, 2), (0, -1), (3, 2), (0, 6), (2, 4)):
        with pytest.raises(da.DAError):
            proof.parse_namespace(raw, a, b)
