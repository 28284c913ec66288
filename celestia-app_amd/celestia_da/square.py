"""Original data square construction, host-side mirror of
pkg/square:

  Builder (NewBuilder, AppendTx, AppendBlobTx, Export, FindBlobStartingIndex,
      BlobShareLength, FindTxShareRange, GetWrappedPFB)  pkg/square/builder.go
  Build, Construct, Deconstruct, TxShareRange, BlobShareRange, Square,
      Size, EmptySquare, WriteSquare                     pkg/square/square.go
  inclusion.BlobMinSquareSize                            pkg/inclusion/blob_share_commitment_rules.go:76

The square this produces is the ODS the GPU path extends: `square_bytes()`
feeds `da.extend_shares` / `device.DeviceSquares`, and blob commitments can be
read back from the GPU-built EDS with `inclusion.get_commitment`.

`Deconstruct` needs the blob sizes of each PFB; the reference decodes the
cosmos-sdk tx (MsgPayForBlobs.BlobSizes) with a `TxDecoder` argument, and this
mirror takes the same role as a callable `pfb_blob_sizes(tx) -> list[int]`.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

from . import blobtx as btx
from . import shares as sh
from .inclusion import next_share_index
from .trees import subtree_width
from .shares import Blob, Range, Share, ShareError

# pkg/appconsts/v1: SquareSizeUpperBound 128, SubtreeRootThreshold 64;
# initial_consts.go: DefaultGovMaxSquareSize 64
SQUARE_SIZE_UPPER_BOUND = 128
SUBTREE_ROOT_THRESHOLD = 64
DEFAULT_GOV_MAX_SQUARE_SIZE = 64
LATEST_VERSION = 1


def square_size_upper_bound(app_version: int = LATEST_VERSION) -> int:
    return SQUARE_SIZE_UPPER_BOUND


def subtree_root_threshold(app_version: int = LATEST_VERSION) -> int:
    return SUBTREE_ROOT_THRESHOLD


def blob_min_square_size(share_count: int) -> int:
    return sh.round_up_power_of_two(int(math.ceil(math.sqrt(float(share_count)))))


def size(n_shares: int) -> int:
    """square.Size / da.SquareSize."""
    return sh.round_up_power_of_two(int(math.ceil(math.sqrt(float(n_shares)))))


class Square(list):
    """[]shares.Share."""

    def size(self) -> int:
        return size(len(self))

    def equals(self, other: Sequence[Share]) -> bool:
        return len(self) == len(other) and all(a.to_bytes() == b.to_bytes() for a, b in zip(self, other))

    def is_empty(self) -> bool:
        return self.equals(empty_square())

    def wrapped_pfbs(self) -> List[bytes]:
        r = sh.get_share_range_for_namespace(self, sh.PAY_FOR_BLOB_NAMESPACE)
        return sh.parse_txs(self[r.start:r.end])

    def square_bytes(self) -> List[bytes]:
        return sh.to_bytes(self)


def empty_square() -> Square:
    return Square(sh.tail_padding_shares(sh.MIN_SHARE_COUNT))


@dataclass
class Element:
    blob: Blob
    pfb_index: int
    blob_index: int
    num_shares: int
    max_padding: int

    def max_share_offset(self) -> int:
        return self.num_shares + self.max_padding


def _new_element(blob: Blob, pfb_index: int, blob_index: int, threshold: int) -> Element:
    n = sh.sparse_shares_needed(len(blob.data))
    return Element(blob, pfb_index, blob_index, n, subtree_width(n, threshold) - 1)


def _worst_case_share_indexes(blobs: int, app_version: int) -> List[int]:
    m = square_size_upper_bound(app_version)
    return [m * m] * blobs


class Builder:
    def __init__(self, max_square_size: int, app_version: int = LATEST_VERSION, *txs: bytes):
        if max_square_size <= 0:
            raise ShareError("max square size must be strictly positive")
        if not sh.is_power_of_two(max_square_size):
            raise ShareError("max square size must be a power of two")
        self.max_capacity = max_square_size * max_square_size
        self.current_size = 0
        self.txs: List[bytes] = []
        self.pfbs: List[btx.IndexWrapper] = []
        self.blobs: List[Element] = []
        self.tx_counter = sh.CompactShareCounter()
        self.pfb_counter = sh.CompactShareCounter()
        self.done = False
        self.subtree_root_threshold = subtree_root_threshold(app_version)
        self.app_version = app_version
        seen_blob_tx = False
        for idx, tx in enumerate(txs):
            blob_tx, is_blob = btx.unmarshal_blob_tx(tx)
            if is_blob:
                seen_blob_tx = True
                if not self.append_blob_tx(blob_tx):
                    raise ShareError(f"not enough space to append blob tx at index {idx}")
            else:
                if seen_blob_tx:
                    raise ShareError(f"normal tx at index {idx} can not be appended after blob tx")
                if not self.append_tx(tx):
                    raise ShareError(f"not enough space to append tx at index {idx}")

    def _can_fit(self, n: int) -> bool:
        return self.current_size + n <= self.max_capacity

    def append_tx(self, tx: bytes) -> bool:
        diff = self.tx_counter.add(len(tx))
        if self._can_fit(diff):
            self.txs.append(bytes(tx))
            self.current_size += diff
            self.done = False
            return True
        self.tx_counter.revert()
        return False

    def append_blob_tx(self, blob_tx: btx.BlobTx) -> bool:
        iw = btx.IndexWrapper(blob_tx.tx, _worst_case_share_indexes(len(blob_tx.blobs), self.app_version))
        pfb_diff = self.pfb_counter.add(iw.size())
        elems = [_new_element(b, len(self.pfbs), i, self.subtree_root_threshold) for i, b in enumerate(blob_tx.blobs)]
        max_blob_shares = sum(e.max_share_offset() for e in elems)
        if self._can_fit(pfb_diff + max_blob_shares):
            self.blobs.extend(elems)
            self.pfbs.append(iw)
            self.current_size += pfb_diff + max_blob_shares
            self.done = False
            return True
        self.pfb_counter.revert()
        return False

    def is_empty(self) -> bool:
        return self.tx_counter.size() == 0 and self.pfb_counter.size() == 0

    def export(self) -> Square:
        if self.is_empty():
            return empty_square()
        ss = blob_min_square_size(self.current_size)
        self.blobs.sort(key=lambda e: e.blob.namespace())  # stable, like sort.SliceStable
        tx_writer = sh.CompactShareSplitter(sh.TX_NAMESPACE, sh.SHARE_VERSION_ZERO)
        for tx in self.txs:
            tx_writer.write_tx(tx)
        non_reserved_start = self.tx_counter.size() + self.pfb_counter.size()
        cursor = end_of_last_blob = non_reserved_start
        blob_writer = sh.SparseShareSplitter()
        for i, e in enumerate(self.blobs):
            cursor = next_share_index(cursor, e.num_shares, self.subtree_root_threshold)
            if i == 0:
                non_reserved_start = cursor
            padding = cursor - end_of_last_blob
            if padding > e.max_padding:
                raise ShareError(f"blob has {padding} padding shares, but {e.max_padding} was the max possible")
            self.pfbs[e.pfb_index].share_indexes[e.blob_index] = cursor
            if i > 0:
                blob_writer.write_namespace_padding_shares(padding)
            blob_writer.write(e.blob)
            cursor += e.num_shares
            end_of_last_blob = cursor
        pfb_writer = sh.CompactShareSplitter(sh.PAY_FOR_BLOB_NAMESPACE, sh.SHARE_VERSION_ZERO)
        for iw in self.pfbs:
            pfb_writer.write_tx(iw.marshal())
        if self.pfb_counter.size() < pfb_writer.count():
            raise ShareError(f"pfbCounter.Size() < pfbTxWriter.Count(): {self.pfb_counter.size()} < "
                             f"{pfb_writer.count()}")
        square = write_square(tx_writer, pfb_writer, blob_writer, non_reserved_start, ss)
        self.done = True
        return square

    def _pfb_offset(self, pfb_index: int) -> int:
        if pfb_index < len(self.txs):
            raise ShareError(f"pfbIndex {pfb_index} does not match a pfb")
        pfb_index -= len(self.txs)
        if pfb_index >= len(self.pfbs):
            raise ShareError(f"pfbIndex {pfb_index} out of range")
        return pfb_index

    def find_blob_starting_index(self, pfb_index: int, blob_index: int) -> int:
        p = self._pfb_offset(pfb_index)
        if blob_index < 0:
            raise ShareError(f"blobIndex {blob_index} must not be negative")
        if not self.done:
            self.export()
        if blob_index >= len(self.pfbs[p].share_indexes):
            raise ShareError(f"blobIndex {blob_index} out of range")
        return self.pfbs[p].share_indexes[blob_index]

    def blob_share_length(self, pfb_index: int, blob_index: int) -> int:
        p = self._pfb_offset(pfb_index)
        if blob_index < 0:
            raise ShareError(f"blobIndex {blob_index} must not be negative")
        for e in self.blobs:
            if e.pfb_index == p and e.blob_index == blob_index:
                return e.num_shares
        raise ShareError("blob not found")

    def find_tx_share_range(self, tx_index: int) -> Range:
        if not self.done:
            self.export()
        if tx_index < 0:
            raise ShareError(f"txIndex {tx_index} must not be negative")
        if tx_index >= len(self.txs) + len(self.pfbs):
            raise ShareError(f"txIndex {tx_index} out of range")
        txw, pfw = sh.CompactShareCounter(), sh.CompactShareCounter()
        for i in range(tx_index):
            if i < len(self.txs):
                txw.add(len(self.txs[i]))
            else:
                pfw.add(self.pfbs[i - len(self.txs)].size())
        start = txw.size() + pfw.size() - 1
        if tx_index < len(self.txs):
            if txw.remainder == 0:
                start += 1
            txw.add(len(self.txs[tx_index]))
        else:
            if pfw.remainder == 0:
                start += 1
            pfw.add(self.pfbs[tx_index - len(self.txs)].size())
        return Range(start, txw.size() + pfw.size())

    def get_wrapped_pfb(self, tx_index: int) -> btx.IndexWrapper:
        if tx_index < 0:
            raise ShareError(f"txIndex {tx_index} must not be negative")
        if tx_index < len(self.txs):
            raise ShareError(f"txIndex {tx_index} does not match a pfb")
        if tx_index >= len(self.txs) + len(self.pfbs):
            raise ShareError(f"txIndex {tx_index} out of range")
        if not self.done:
            self.export()
        return self.pfbs[tx_index - len(self.txs)]

    def num_pfbs(self) -> int:
        return len(self.pfbs)

    def num_txs(self) -> int:
        return len(self.txs) + len(self.pfbs)


def write_square(tx_writer: sh.CompactShareSplitter, pfb_writer: sh.CompactShareSplitter,
                 blob_writer: sh.SparseShareSplitter, non_reserved_start: int, square_size: int) -> Square:
    total = square_size * square_size
    pfb_start = tx_writer.count()
    padding_start = pfb_start + pfb_writer.count()
    if non_reserved_start < padding_start:
        raise ShareError(f"nonReservedStart {non_reserved_start} is too small to fit all PFBs and txs")
    padding = sh.reserved_padding_shares(non_reserved_start - padding_start)
    end_of_last_blob = non_reserved_start + blob_writer.count()
    if total < end_of_last_blob:
        raise ShareError(f"square size {total} is too small to fit all blobs")
    tx_shares = tx_writer.export()
    pfb_shares = pfb_writer.export()
    square: List[Optional[Share]] = [None] * total
    square[0:len(tx_shares)] = tx_shares
    square[pfb_start:pfb_start + len(pfb_shares)] = pfb_shares
    if blob_writer.count() > 0:
        square[padding_start:padding_start + len(padding)] = padding
        bl = blob_writer.export()
        square[non_reserved_start:non_reserved_start + len(bl)] = bl
    if total > end_of_last_blob:
        tail = sh.tail_padding_shares(total - end_of_last_blob)
        square[end_of_last_blob:] = tail
    if any(s is None for s in square) or len(square) != total:
        # Go leaves zero-valued shares here; the layout rules above never do
        raise ShareError("square has unwritten shares")
    return Square(square)


def build(txs: Sequence[bytes], app_version: int = LATEST_VERSION,
          max_square_size: int = SQUARE_SIZE_UPPER_BOUND) -> Tuple[Square, List[bytes]]:
    """square.Build: the square and the txs that fit (normal txs first)."""
    b = Builder(max_square_size, app_version)
    normal, blob_txs = [], []
    for tx in txs:
        t, is_blob = btx.unmarshal_blob_tx(tx)
        if is_blob:
            if b.append_blob_tx(t):
                blob_txs.append(tx)
        elif b.append_tx(tx):
            normal.append(tx)
    return b.export(), normal + blob_txs


def construct(txs: Sequence[bytes], app_version: int = LATEST_VERSION,
              max_square_size: int = SQUARE_SIZE_UPPER_BOUND) -> Square:
    """square.Construct: every tx must fit, normal txs before blob txs."""
    return Builder(max_square_size, app_version, *txs).export()


def deconstruct(square: Sequence[Share], pfb_blob_sizes: Callable[[bytes], Sequence[int]]) -> List[bytes]:
    """square.Deconstruct: the txs (blob txs re-assembled from the square)."""
    sq = Square(square)
    if sq.is_empty():
        return []
    tr = sh.get_share_range_for_namespace(sq, sh.TX_NAMESPACE)
    if tr.start != 0:
        raise ShareError(f"expected txs to start at index 0, but got {tr.start}")
    wr = sh.get_share_range_for_namespace(sq[tr.end:], sh.PAY_FOR_BLOB_NAMESPACE)
    if wr.is_empty():
        return sh.parse_txs(sq[tr.start:tr.end])
    if wr.start != 0:
        raise ShareError(f"expected PFBs to start directly after non PFBs at index {tr.end}, but got {wr.start}")
    wr.add(tr.end)
    txs = sh.parse_txs(sq[tr.start:tr.end])
    for i, wb in enumerate(sh.parse_txs(sq[wr.start:wr.end])):
        iw, ok = btx.unmarshal_index_wrapper(wb)
        if not ok:
            raise ShareError(f"expected wrapped PFB at index {i}")
        if not iw.share_indexes:
            raise ShareError(f"wrapped PFB {i} has no blobs attached")
        sizes = list(pfb_blob_sizes(iw.tx))
        if len(sizes) != len(iw.share_indexes):
            raise ShareError(f"expected PFB to have {len(iw.share_indexes)} blob sizes, but got {len(sizes)}")
        blobs = []
        for j, si in enumerate(iw.share_indexes):
            parsed = sh.parse_blobs(sq[si:si + sh.sparse_shares_needed(sizes[j])])
            if len(parsed) != 1:
                raise ShareError(f"expected to parse a single blob, but got {len(parsed)}")
            blobs.append(parsed[0])
        txs.append(btx.marshal_blob_tx(iw.tx, *blobs))
    return txs


# ---- native construction (libdagpu: csrc/square.cpp, dagpu_square_construct/_build) ----------

def _pack(txs: Sequence[bytes]):
    import numpy as np
    lens = np.array([len(t) for t in txs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(bytes(t) for t in txs) or b"\x00", dtype=np.uint8).copy()
    return buf, lens


def _native(fn: str, txs, max_square_size: int, threshold: int, kept=None):
    import ctypes

    import numpy as np

    from . import _abi
    L = _abi.lib()
    buf, lens = _pack(txs)
    k = ctypes.c_uint32(0)
    cap = max(1, max_square_size) ** 2 * sh.SHARE_SIZE
    out = np.empty(cap, np.uint8)
    args = [None, _abi.addr(buf), _abi.addr(lens), len(txs), max_square_size, threshold, _abi.addr(out), cap,
            ctypes.addressof(k)]
    if kept is not None:
        args.append(_abi.addr(kept))
    rc = getattr(L, fn)(*args)
    if rc != 0:
        msg = L.dagpu_last_error(None).decode()
        raise ShareError(msg) if rc == _abi.ERR_SQUARE else ValueError(f"{fn}: status {rc}: {msg}")
    return int(k.value), out[:int(k.value) ** 2 * sh.SHARE_SIZE]


def construct_native(txs: Sequence[bytes], max_square_size: int = SQUARE_SIZE_UPPER_BOUND,
                     threshold: int = SUBTREE_ROOT_THRESHOLD):
    """square.Construct in the library's C++ (dagpu_square_construct): (k, ODS
    bytes as a (k*k*512,) uint8 array), byte-identical to construct(txs)."""
    return _native("dagpu_square_construct", txs, max_square_size, threshold)


def build_native(txs: Sequence[bytes], max_square_size: int = SQUARE_SIZE_UPPER_BOUND,
                 threshold: int = SUBTREE_ROOT_THRESHOLD):
    """square.Build in C++ (dagpu_square_build): (k, ODS bytes, kept txs in the
    order Build returns them: normal txs, then blob txs)."""
    import numpy as np
    kept = np.zeros(max(1, len(txs)), np.uint8)
    k, ods = _native("dagpu_square_build", txs, max_square_size, threshold, kept)
    normal = [t for i, t in enumerate(txs) if kept[i] and not btx.unmarshal_blob_tx(t)[1]]
    blob = [t for i, t in enumerate(txs) if kept[i] and btx.unmarshal_blob_tx(t)[1]]
    return k, ods, normal + blob


def tx_share_range(txs: Sequence[bytes], tx_index: int, app_version: int = LATEST_VERSION) -> Range:
    return Builder(square_size_upper_bound(app_version), app_version, *txs).find_tx_share_range(tx_index)


def blob_share_range(txs: Sequence[bytes], tx_index: int, blob_index: int,
                     app_version: int = LATEST_VERSION) -> Range:
    b = Builder(square_size_upper_bound(app_version), app_version, *txs)
    start = b.find_blob_starting_index(tx_index, blob_index)
    return Range(start, start + b.blob_share_length(tx_index, blob_index))
