"""Host-side mirror of the reference's tree and commitment interfaces, computed
on the GPU through include/dagpu.h (nmt_forest.hip):

  nmt.NamespacedMerkleTree (nmt v0.20.0: New(sha256, NamespaceIDSize(29),
      IgnoreMaxNamespace), Push, Root)      -> NamespacedMerkleTree, nmt_roots
  wrapper.ErasuredNamespacedMerkleTree / NewConstructor
      (pkg/wrapper/nmt_wrapper.go:55-140)  -> ErasuredNamespacedMerkleTree,
                                               new_constructor, wrapper_roots
  merkle.HashFromByteSlices (celestia-core crypto/merkle)
                                            -> hash_from_byte_slices, merkle_roots
  inclusion.CreateCommitment / CreateCommitments / SubTreeWidth /
      MerkleMountainRangeSizes (pkg/inclusion/commitment.go:19-107,
      blob_share_commitment_rules.go:76-101) -> create_commitment(s), ...
  shares.SplitBlobs for one blob (sparse shares, pkg/shares/split_sparse_shares.go,
      share_builder.go:26-221)              -> split_blob  (host byte layout)

Trees buffer their pushes in host memory; Root() (or the batch functions)
hashes every leaf and level of every tree in one GPU call, which is how the
rsmt2d.Tree drop-in avoids a cgo call per Push.
"""
from __future__ import annotations

import ctypes
import struct
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _abi
from .da import (PARITY_SHARES_NAMESPACE, Context, DAError, ErrInvalidPushOrder,
                 default_context)
from ._abi import HASH_SIZE, NAMESPACE_SIZE, ROOT_SIZE, SHARE_SIZE

# pkg/appconsts: DefaultSubtreeRootThreshold (v1) = 64, ShareInfoBytes = 1,
# SequenceLenBytes = 4, ShareVersionZero = 0
DEFAULT_SUBTREE_ROOT_THRESHOLD = 64
SHARE_INFO_BYTES = 1
SEQUENCE_LEN_BYTES = 4
SUPPORTED_SHARE_VERSIONS = (0,)


def _ctx(ctx: Optional[Context]) -> Context:
    return ctx if ctx is not None else default_context()


def _pack(trees: Sequence[Sequence[bytes]]) -> Tuple[np.ndarray, np.ndarray, int]:
    counts = np.array([len(t) for t in trees], dtype=np.uint32)
    lens = {len(x) for t in trees for x in t}
    if len(lens) > 1:
        raise DAError(_abi.ERR_ARG, "all leaves of one batch must have the same length")
    leaf_len = lens.pop() if lens else 0
    flat = b"".join(x for t in trees for x in t)
    buf = np.frombuffer(flat, dtype=np.uint8) if flat else np.zeros(1, np.uint8)
    return counts, buf, leaf_len


def nmt_roots(trees: Sequence[Sequence[bytes]], ignore_max_namespace: bool = True,
              ctx: Optional[Context] = None) -> List[bytes]:
    """Root() of one nmt per entry of `trees` (each a list of namespaced data
    pushes, ns = first 29 bytes).  Raises ErrInvalidPushOrder like nmt.Push."""
    c = _ctx(ctx)
    counts, buf, leaf_len = _pack(trees)
    roots = np.zeros((max(len(trees), 1), ROOT_SIZE), np.uint8)
    status = np.zeros(max(len(trees), 1), np.int32)
    rc = c._L.dagpu_nmt_roots(c.handle, len(trees), _abi.addr(counts), _abi.addr(buf), leaf_len,
                              _abi.PREFIX_NONE, None, int(ignore_max_namespace), _abi.addr(roots),
                              _abi.addr(status))
    c.check(rc)
    return [roots[i].tobytes() for i in range(len(trees))]


class NamespacedMerkleTree:
    """nmt.NamespacedMerkleTree with NamespaceIDSize 29 and SHA-256.  Push
    validates eagerly (length, push order) as nmt.Push does; Root() runs on the
    GPU."""

    def __init__(self, ignore_max_namespace: bool = True, ctx: Optional[Context] = None):
        self.ignore_max_namespace = ignore_max_namespace
        self.ctx = ctx
        self.leaves: List[bytes] = []

    def push(self, namespaced_data: bytes) -> None:
        d = bytes(namespaced_data)
        if len(d) < NAMESPACE_SIZE:
            raise DAError(_abi.ERR_SHARE_SIZE,
                          f"mismatched namespace size: got: {len(d)}, want >= {NAMESPACE_SIZE}")
        if self.leaves and d[:NAMESPACE_SIZE] < self.leaves[-1][:NAMESPACE_SIZE]:
            raise ErrInvalidPushOrder(
                _abi.ERR_PUSH_ORDER,
                f"invalid push order: last namespace: {self.leaves[-1][:NAMESPACE_SIZE].hex()}, "
                f"pushed: {d[:NAMESPACE_SIZE].hex()}")
        self.leaves.append(d)

    def root(self) -> bytes:
        return nmt_roots([self.leaves], self.ignore_max_namespace, self.ctx)[0]


def wrapper_roots(square_size: int, axis_indices: Sequence[int],
                  trees: Sequence[Sequence[bytes]], ctx: Optional[Context] = None) -> List[bytes]:
    """Root() of one ErasuredNamespacedMerkleTree(square_size, axis_indices[t])
    per entry of `trees` (each the list of raw shares pushed to it)."""
    c = _ctx(ctx)
    counts, buf, leaf_len = _pack(trees)
    axes = np.array(list(axis_indices) or [0], dtype=np.uint32)
    roots = np.zeros((max(len(trees), 1), ROOT_SIZE), np.uint8)
    status = np.zeros(max(len(trees), 1), np.int32)
    rc = c._L.dagpu_wrapper_roots(c.handle, square_size, len(trees), _abi.addr(axes),
                                  _abi.addr(counts), _abi.addr(buf), leaf_len, _abi.addr(roots),
                                  _abi.addr(status))
    c.check(rc)
    return [roots[i].tobytes() for i in range(len(trees))]


class ErasuredNamespacedMerkleTree:
    """wrapper.ErasuredNamespacedMerkleTree (pkg/wrapper/nmt_wrapper.go:25-140):
    Push(share) prepends share[0:29] in Q0 and the parity namespace elsewhere."""

    def __init__(self, square_size: int, axis_index: int, ctx: Optional[Context] = None):
        if square_size == 0:
            raise DAError(_abi.ERR_ARG, "cannot create a ErasuredNamespacedMerkleTree of squareSize == 0")
        self.square_size = square_size
        self.axis_index = axis_index
        self.ctx = ctx
        self.shares: List[bytes] = []

    def _is_quadrant_zero(self) -> bool:
        return len(self.shares) < self.square_size and self.axis_index < self.square_size

    def push(self, data: bytes) -> None:
        k2 = 2 * self.square_size
        if self.axis_index + 1 > k2 or len(self.shares) + 1 > k2:
            raise DAError(_abi.ERR_ARG,
                          f"pushed past predetermined square size: boundary at {k2} index at "
                          f"{self.axis_index} {len(self.shares)}")
        d = bytes(data)
        if len(d) < NAMESPACE_SIZE:
            raise DAError(_abi.ERR_SHARE_SIZE, "data is too short to contain namespace ID")
        ns = d[:NAMESPACE_SIZE] if self._is_quadrant_zero() else PARITY_SHARES_NAMESPACE
        if self.shares:
            prev = self.shares[-1]
            pns = prev[:NAMESPACE_SIZE] if len(self.shares) - 1 < self.square_size and \
                self.axis_index < self.square_size else PARITY_SHARES_NAMESPACE
            if ns < pns:
                raise ErrInvalidPushOrder(_abi.ERR_PUSH_ORDER,
                                          f"invalid push order: last namespace: {pns.hex()}, "
                                          f"pushed: {ns.hex()}")
        self.shares.append(d)

    def root(self) -> bytes:
        return wrapper_roots(self.square_size, [self.axis_index], [self.shares], self.ctx)[0]


def new_constructor(square_size: int, ctx: Optional[Context] = None):
    """wrapper.NewConstructor: returns NewTree(axis, axis_index)."""
    def new_tree(axis: int, axis_index: int) -> ErasuredNamespacedMerkleTree:
        return ErasuredNamespacedMerkleTree(square_size, axis_index, ctx)
    return new_tree


def merkle_roots(lists: Sequence[Sequence[bytes]], ctx: Optional[Context] = None) -> List[bytes]:
    """merkle.HashFromByteSlices of every list (items of one call share a length)."""
    c = _ctx(ctx)
    counts, buf, item_len = _pack(lists)
    out = np.zeros((max(len(lists), 1), HASH_SIZE), np.uint8)
    c.check(c._L.dagpu_merkle_roots(c.handle, len(lists), _abi.addr(counts), _abi.addr(buf),
                                    item_len, _abi.addr(out)))
    return [out[i].tobytes() for i in range(len(lists))]


def hash_from_byte_slices(items: Sequence[bytes], ctx: Optional[Context] = None) -> bytes:
    return merkle_roots([list(items)], ctx)[0]


# ---- blob shares and commitments ------------------------------------------------

def round_up_power_of_two(v: int) -> int:
    r = 1
    while r < v:
        r <<= 1
    return r


def round_down_power_of_two(v: int) -> int:
    if v <= 0:
        raise ValueError(f"input {v} must be positive")
    up = round_up_power_of_two(v)
    return up if up == v else up // 2


def subtree_width(share_count: int, subtree_root_threshold: int = DEFAULT_SUBTREE_ROOT_THRESHOLD) -> int:
    """inclusion.SubTreeWidth, computed by the library (dagpu_subtree_width)."""
    rc = _abi.lib().dagpu_subtree_width(share_count, subtree_root_threshold)
    if rc < 0:
        raise DAError(rc, "invalid share count or threshold")
    return rc


def merkle_mountain_range_sizes(total: int, max_tree: int) -> List[int]:
    """inclusion.MerkleMountainRangeSizes (pkg/inclusion/commitment.go:85-107)."""
    out = []
    while total:
        t = max_tree if total >= max_tree else round_down_power_of_two(total)
        out.append(t)
        total -= t
    return out


def namespace_v0(sub_id: bytes) -> bytes:
    """namespace.MustNewV0 (pkg/namespace/namespace.go:44-69): version 0,
    18 zero bytes, 10-byte sub-ID (left zero padded)."""
    if len(sub_id) > 10:
        raise ValueError(f"subID must be <= 10, but it was {len(sub_id)} bytes")
    return b"\x00" + b"\x00" * 18 + sub_id.rjust(10, b"\x00")


def split_blob(namespace: bytes, data: bytes, share_version: int = 0) -> List[bytes]:
    """Sparse shares of one blob (SparseShareSplitter.Write): namespace | info
    byte (version << 1 | sequence start) | [sequence length, first share] | data,
    last share zero padded to 512 B."""
    if share_version not in SUPPORTED_SHARE_VERSIONS:
        raise DAError(_abi.ERR_ARG, f"unsupported share version: {share_version}")
    if len(namespace) != NAMESPACE_SIZE:
        raise DAError(_abi.ERR_ARG, f"invalid namespace length: {len(namespace)} must be {NAMESPACE_SIZE}")
    out, rest, first = [], bytes(data), True
    while True:
        head = namespace + bytes([(share_version << 1) | int(first)])
        if first:
            head += struct.pack(">I", len(data))
        room = SHARE_SIZE - len(head)
        chunk, rest = rest[:room], rest[room:]
        out.append((head + chunk).ljust(SHARE_SIZE, b"\x00"))
        first = False
        if not rest:
            return out


def create_commitments(blobs: Sequence[Tuple[bytes, bytes, int]],
                       subtree_root_threshold: int = DEFAULT_SUBTREE_ROOT_THRESHOLD,
                       ctx: Optional[Context] = None) -> List[bytes]:
    """inclusion.CreateCommitments for (namespace, data, share_version) blobs;
    every NMT subtree and every per-blob RFC-6962 root in one GPU call."""
    c = _ctx(ctx)
    shares, counts, nss = [], [], []
    for ns, data, ver in blobs:
        s = split_blob(ns, data, ver)
        shares.extend(s)
        counts.append(len(s))
        nss.append(ns)
    n = len(blobs)
    sh = np.frombuffer(b"".join(shares), np.uint8) if shares else np.zeros(1, np.uint8)
    ns_buf = np.frombuffer(b"".join(nss), np.uint8) if nss else np.zeros(1, np.uint8)
    cnt = np.array(counts or [0], dtype=np.uint32)
    out = np.zeros((max(n, 1), HASH_SIZE), np.uint8)
    c.check(c._L.dagpu_blob_commitments(c.handle, n, _abi.addr(ns_buf), _abi.addr(cnt),
                                        _abi.addr(sh), subtree_root_threshold, _abi.addr(out)))
    return [out[i].tobytes() for i in range(n)]


def create_commitment(namespace: bytes, data: bytes, share_version: int = 0,
                      subtree_root_threshold: int = DEFAULT_SUBTREE_ROOT_THRESHOLD,
                      ctx: Optional[Context] = None) -> bytes:
    return create_commitments([(namespace, data, share_version)], subtree_root_threshold, ctx)[0]
