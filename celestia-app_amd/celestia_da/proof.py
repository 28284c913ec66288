"""Share inclusion proofs, host-side mirror of

  proof.NewShareInclusionProof      pkg/proof/proof.go:58-165
  merkle.ProofsFromByteSlices       celestia-core crypto/merkle (used at proof.go:87)
  nmt ProveRange                    nmt v0.20.0 (used at proof.go:139 via the wrapper tree)

The square is extended and hashed on the GPU, every row-tree node stays in HBM
(dagpu_row_nodes_device) and the RFC-6962 tree over rowRoots||colRoots is
built on the GPU with all levels (dagpu_merkle_levels); a proof is then a
selection of stored nodes (index arithmetic on the host, gathered on the
device).  No hashing happens on the host.

nmt's ProveRange emits the roots of the maximal subtrees that do not overlap
[start, end), left to right (its recursive buildRangeProof appends a subtree's
hash when the subtree is disjoint from the range and its parent is not);
merkle proofs list the sibling ("aunt") hashes from the leaf to the root.  The
node ORDER follows nmt v0.20.0 / celestia-core as restated here; the nmt module
is not in this image, so the proof byte layout is "parity unpinned" (the tests
re-derive every row root and the data root from the proofs).
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _abi
from .da import Context, DAError, default_context, extend_shares, new_data_availability_header
from .inclusion import EDSSubTreeRootCacher


@dataclass
class MerkleProof:
    """crypto/merkle Proof: Total, Index, LeafHash, Aunts (leaf to root)."""
    total: int
    index: int
    leaf_hash: bytes
    aunts: List[bytes]


@dataclass
class NMTProof:
    """tmproto.NMTProof: Start, End (exclusive), Nodes (90-B), LeafHash (nil for inclusion)."""
    start: int
    end: int
    nodes: List[bytes]
    leaf_hash: bytes = b""


@dataclass
class RowProof:
    row_roots: List[bytes]
    proofs: List[MerkleProof]
    start_row: int
    end_row: int


@dataclass
class ShareProof:
    data: List[bytes]
    share_proofs: List[NMTProof]
    namespace_id: bytes
    row_proof: RowProof
    namespace_version: int


def merkle_levels(items: Sequence[bytes], ctx: Optional[Context] = None) -> List[List[bytes]]:
    """Every level of the RFC-6962 tree over `items` (level 0 = leaf hashes)."""
    c = ctx or default_context()
    n = len(items)
    if n == 0:
        return []
    ln = len(items[0])
    buf = np.frombuffer(b"".join(items), np.uint8) if ln else np.zeros(1, np.uint8)
    cap = ctypes.c_size_t(2 * n + 64)  # promoted odd nodes add <= log2(n)
    out = np.zeros((2 * n + 64, 32), np.uint8)
    c.check(c._L.dagpu_merkle_levels(c.handle, n, _abi.addr(buf), ln, _abi.addr(out), ctypes.byref(cap)))
    levels, off, cnt = [], 0, n
    while True:
        levels.append([out[off + i].tobytes() for i in range(cnt)])
        off += cnt
        if cnt == 1:
            return levels
        cnt = (cnt + 1) // 2


def proofs_from_byte_slices(items: Sequence[bytes], ctx: Optional[Context] = None
                            ) -> Tuple[bytes, List[MerkleProof]]:
    """merkle.ProofsFromByteSlices: (root, one proof per item)."""
    levels = merkle_levels(items, ctx)
    if not levels:
        raise DAError(_abi.ERR_ARG, "no items")
    proofs = []
    for i in range(len(items)):
        aunts, idx = [], i
        for lv in levels[:-1]:
            sib = idx ^ 1
            if sib < len(lv):  # an odd last node is promoted: no aunt at this level
                aunts.append(lv[sib])
            idx >>= 1
        proofs.append(MerkleProof(len(items), i, levels[0][i], aunts))
    return levels[-1][0], proofs


def range_proof_nodes(width: int, start: int, end: int) -> List[Tuple[int, int]]:
    """(depth, position) of the maximal subtrees of a full tree of `width`
    leaves disjoint from [start, end), left to right (nmt buildRangeProof)."""
    out: List[Tuple[int, int]] = []
    max_depth = int(math.log2(width))

    def rec(lo: int, hi: int, depth: int):
        if hi <= start or lo >= end:
            out.append((depth, lo >> (max_depth - depth)))
            return
        if hi - lo == 1:
            return
        mid = (lo + hi) // 2
        rec(lo, mid, depth + 1)
        rec(mid, hi, depth + 1)

    rec(0, width, 0)
    return out


def prove_row_ranges(cacher: EDSSubTreeRootCacher, ranges: Sequence[Tuple[int, int, int]]) -> List[NMTProof]:
    """ProveRange(start, end) on row trees: ranges = (row, start, end)."""
    reqs, spans = [], []
    for row, s, e in ranges:
        if not (0 <= s < e <= cacher.w):
            raise DAError(_abi.ERR_ARG, f"invalid range: [{s}, {e}) for a tree of {cacher.w} leaves")
        nodes = range_proof_nodes(cacher.w, s, e)
        spans.append((len(reqs), len(nodes)))
        reqs.extend((row, d, p) for d, p in nodes)
    got = cacher.nodes_at([r[0] for r in reqs], [r[1] for r in reqs], [r[2] for r in reqs])
    return [NMTProof(s, e, got[a:a + n]) for (row, s, e), (a, n) in zip(ranges, spans)]


def new_share_inclusion_proof(shares: Sequence[bytes], namespace: bytes, share_range: Tuple[int, int],
                              ctx: Optional[Context] = None) -> ShareProof:
    """NewShareInclusionProof for a data square given as its k*k shares;
    share_range = [start, end) in row-major share order (pre-validated, as in
    the reference)."""
    c = ctx or default_context()
    n = len(shares)
    k = int(math.isqrt(n))
    start, end = share_range
    start_row, end_row = start // k, (end - 1) // k
    start_leaf, end_leaf = start % k, (end - 1) % k
    eds = extend_shares(np.frombuffer(b"".join(shares), np.uint8).reshape(n, 512), c)
    dah = new_data_availability_header(eds)
    _, all_proofs = proofs_from_byte_slices(dah.row_roots + dah.column_roots, c)
    cacher = EDSSubTreeRootCacher(k, eds.data, c)
    ranges, data = [], []
    for i, row in enumerate(range(start_row, end_row + 1)):
        s = start_leaf if i == 0 else 0
        e = end_leaf if row == end_row else k - 1
        ranges.append((row, s, e + 1))
        data.extend(eds.cell(row, j) for j in range(s, e + 1))
    return ShareProof(
        data=data,
        share_proofs=prove_row_ranges(cacher, ranges),
        namespace_id=namespace[1:],
        row_proof=RowProof(dah.row_roots[start_row:end_row + 1], all_proofs[start_row:end_row + 1],
                           start_row, end_row),
        namespace_version=namespace[0],
    )
