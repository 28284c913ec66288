"""Share inclusion proofs, host-side mirror of

  proof.NewShareInclusionProof      pkg/proof/proof.go:58-165
  proof.NewTxInclusionProof         pkg/proof/proof.go:23-54 (square built by celestia_da.square)
  proof.ParseNamespace              pkg/proof/querier.go:123-151
  merkle.ProofsFromByteSlices       celestia-core crypto/merkle (used at proof.go:87)
  nmt ProveRange                    nmt v0.20.0 (used at proof.go:139 via the wrapper tree)
  verification: ShareProof.Validate / VerifyProof, RowProof.Validate (celestia-core
  types/share_proof.go, row_proof.go), merkle Proof.Verify, nmt Proof.VerifyInclusion
  -> dagpu_merkle_verify / dagpu_nmt_verify_inclusion (host code of the library)

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
import hashlib
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _abi
from .da import Context, DAError, default_context, extend_shares, new_data_availability_header
from .inclusion import EDSSubTreeRootCacher


# crypto/merkle MaxAunts (celestia-core v0.34 crypto/merkle/proof.go)
MAX_AUNTS = 100


@dataclass
class MerkleProof:
    """crypto/merkle Proof: Total, Index, LeafHash, Aunts (leaf to root)."""
    total: int
    index: int
    leaf_hash: bytes
    aunts: List[bytes]

    def verify(self, root: bytes, leaf: bytes) -> None:
        """merkle Proof.Verify: raises DAError when the proof does not prove
        `leaf` under `root`."""
        if root is None:
            raise DAError(_abi.ERR_ARG, "invalid root hash: cannot be nil")
        if self.total < 0:
            raise DAError(_abi.ERR_PROOF, "proof total must be positive")
        if self.index < 0:
            raise DAError(_abi.ERR_PROOF, "proof index cannot be negative")
        # Proof.ValidateBasic's MaxAunts bound, and Verify's LeafHash check
        if len(self.aunts) > MAX_AUNTS:
            raise DAError(_abi.ERR_PROOF, f"expected no more than {MAX_AUNTS} aunts, got {len(self.aunts)}")
        want_leaf = hashlib.sha256(b"\x00" + bytes(leaf)).digest()
        if bytes(self.leaf_hash) != want_leaf:
            raise DAError(_abi.ERR_PROOF, f"invalid leaf hash: wanted {want_leaf.hex().upper()} "
                                          f"got {bytes(self.leaf_hash).hex().upper()}")
        # keep every buffer referenced until the call returns (addr() is a raw pointer)
        r, lf, au = _bytes(root), _bytes(leaf), _bytes(b"".join(self.aunts))
        rc = _abi.lib().dagpu_merkle_verify(_abi.addr(r), _abi.addr(lf), len(leaf), self.index, self.total,
                                            _abi.addr(au), len(self.aunts))
        if rc == _abi.ERR_PROOF:
            raise DAError(rc, "invalid root hash")
        if rc:
            raise DAError(rc, "malformed merkle proof")


@dataclass
class NMTProof:
    """tmproto.NMTProof: Start, End (exclusive), Nodes (90-B), LeafHash (nil for inclusion)."""
    start: int
    end: int
    nodes: List[bytes]
    leaf_hash: bytes = b""

    def verify_inclusion(self, namespace: bytes, leaves: Sequence[bytes], root: bytes) -> bool:
        """nmt Proof.VerifyInclusion (IgnoreMaxNamespace): `leaves` are the raw
        shares (the tree prepends `namespace` to each)."""
        if len(namespace) != 29 or len(root) != 90 or any(len(n) != 90 for n in self.nodes):
            return False
        ln = len(leaves[0]) if leaves else 0
        if any(len(x) != ln for x in leaves):
            return False
        nsb, lv, nd, rt = _bytes(namespace), _bytes(b"".join(leaves)), _bytes(b"".join(self.nodes)), _bytes(root)
        rc = _abi.lib().dagpu_nmt_verify_inclusion(_abi.addr(nsb), _abi.addr(lv), len(leaves), ln, self.start,
                                                   self.end, _abi.addr(nd), len(self.nodes), _abi.addr(rt))
        return rc == 0


@dataclass
class RowProof:
    row_roots: List[bytes]
    proofs: List[MerkleProof]
    start_row: int
    end_row: int

    def validate(self, root: bytes) -> None:
        """RowProof.Validate: every row root is proven under the data root."""
        if self.end_row - self.start_row + 1 != len(self.row_roots):
            raise DAError(_abi.ERR_PROOF, "the number of rows is different than the number of row roots")
        if len(self.proofs) != len(self.row_roots):
            raise DAError(_abi.ERR_PROOF, "the number of proofs is different than the number of row roots")
        for p, r in zip(self.proofs, self.row_roots):
            try:
                p.verify(root, r)
            except DAError:
                raise DAError(_abi.ERR_PROOF, "row proof failed to verify") from None


@dataclass
class ShareProof:
    data: List[bytes]
    share_proofs: List[NMTProof]
    namespace_id: bytes
    row_proof: RowProof
    namespace_version: int

    def verify_proof(self) -> bool:
        """ShareProof.VerifyProof: each row's shares under its row root."""
        if self.namespace_version > 255:
            return False
        ns = bytes([self.namespace_version]) + self.namespace_id
        cursor = 0
        for i, p in enumerate(self.share_proofs):
            used = p.end - p.start
            if not p.verify_inclusion(ns, self.data[cursor:cursor + used], self.row_proof.row_roots[i]):
                return False
            cursor += used
        return True

    def validate(self, root: bytes) -> None:
        """ShareProof.Validate: shapes, the row proof under the data root, then
        the share proofs under the row roots."""
        n = sum(p.end - p.start for p in self.share_proofs)
        if len(self.share_proofs) != len(self.row_proof.row_roots):
            raise DAError(_abi.ERR_PROOF, f"the number of share proofs {len(self.share_proofs)} must equal the "
                                          f"number of row roots {len(self.row_proof.row_roots)}")
        if len(self.data) != n:
            raise DAError(_abi.ERR_PROOF, f"the number of shares {len(self.data)} must equal the number of "
                                          f"shares in share proofs {n}")
        for p in self.share_proofs:
            if p.start < 0:
                raise DAError(_abi.ERR_PROOF, f"proof index cannot be negative: {p.start}")
            if p.end - p.start <= 0:
                raise DAError(_abi.ERR_PROOF, f"proof total must be positive: {p.end - p.start}")
        self.row_proof.validate(root)
        if not self.verify_proof():
            raise DAError(_abi.ERR_PROOF, "share proof failed to verify")


def _bytes(b: bytes) -> np.ndarray:
    return np.frombuffer(b, np.uint8) if len(b) else np.zeros(1, np.uint8)


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


def parse_namespace(raw_shares: Sequence[bytes], start_share: int, end_share: int) -> bytes:
    """proof.ParseNamespace (querier.go:123-151): the one namespace of shares
    [start_share, end_share)."""
    if start_share < 0:
        raise DAError(_abi.ERR_ARG, f"start share {start_share} should be positive")
    if end_share < 0:
        raise DAError(_abi.ERR_ARG, f"end share {end_share} should be positive")
    if end_share < start_share:
        raise DAError(_abi.ERR_ARG, f"end share {end_share} cannot be lower than starting share {start_share}")
    if end_share > len(raw_shares):
        raise DAError(_abi.ERR_ARG, f"end share {end_share} is higher than block shares {len(raw_shares)}")
    ns = bytes(raw_shares[start_share][:29])
    for i, share in enumerate(raw_shares[start_share:end_share]):
        if bytes(share[:29]) != ns:
            raise DAError(_abi.ERR_ARG, f"shares range contain different namespaces at index {i}: "
                                        f"{ns.hex()} and {bytes(share[:29]).hex()}")
    return ns


def new_tx_inclusion_proof(txs: Sequence[bytes], tx_index: int, app_version: int = 1,
                           ctx: Optional[Context] = None) -> ShareProof:
    """proof.NewTxInclusionProof: build the square from `txs`, find the tx's
    share range and prove it (the shares of a PFB live in the PFB namespace)."""
    from . import blobtx, shares as sh, square as sq
    if tx_index >= len(txs):
        raise DAError(_abi.ERR_ARG, f"txIndex {tx_index} out of bounds")
    b = sq.Builder(sq.square_size_upper_bound(app_version), app_version, *txs)
    data_square = b.export()
    r = b.find_tx_share_range(tx_index)
    _, is_blob = blobtx.unmarshal_blob_tx(txs[tx_index])
    ns = sh.PAY_FOR_BLOB_NAMESPACE if is_blob else sh.TX_NAMESPACE
    return new_share_inclusion_proof(data_square.square_bytes(), ns, (r.start, r.end), ctx)
