"""Host-side mirror of the reference's pkg/da + pkg/wrapper + codec interface.

Names, argument meaning and error text follow the Go reference so the parity
tests read like its own tests:
  ExtendShares                 pkg/da/data_availability_header.go:65-75
  NewDataAvailabilityHeader    pkg/da/data_availability_header.go:44-63
  DataAvailabilityHeader.Hash  pkg/da/data_availability_header.go:92-108
  ValidateBasic                pkg/da/data_availability_header.go:134-162
  MinDataAvailabilityHeader    pkg/da/data_availability_header.go:179-190
  SquareSize / RoundUpPowerOfTwo  :205-215
  rsmt2d.Codec (LeoRSCodec)    pkg/appconsts/global_consts.go:92
Every compute step runs on the GPU through include/dagpu.h.
"""
from __future__ import annotations

import ctypes
import math
import threading
from typing import List, Optional, Sequence

import numpy as np

from . import _abi
from ._abi import HASH_SIZE, ROOT_SIZE, SHARE_SIZE

# pkg/appconsts: DefaultSquareSizeUpperBound = 128, MinSquareSize = 1
DEFAULT_SQUARE_SIZE_UPPER_BOUND = 128
MIN_SQUARE_SIZE = 1
MAX_EXTENDED_SQUARE_WIDTH = DEFAULT_SQUARE_SIZE_UPPER_BOUND * 2
MIN_EXTENDED_SQUARE_WIDTH = MIN_SQUARE_SIZE * 2

PARITY_SHARES_NAMESPACE = b"\xff" * 29
TAIL_PADDING_NAMESPACE = b"\xff" * 28 + b"\xfe"


class DAError(Exception):
    """Error raised by the DA path; `code` is the dagpu_status value."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


class ErrInvalidPushOrder(DAError):
    pass


class ErrByzantineData(DAError):
    """rsmt2d ErrByzantineData: axis ("row" / "col") and index of the failing
    axis; rebuilt_axis / rebuilt_index name the row or column whose repair
    failed (the same axis unless a newly completed orthogonal axis failed),
    whose present shares are ErrByzantineData.Shares."""
    axis = None
    index = None
    rebuilt_axis = None
    rebuilt_index = None


class ErrUnrepairableDataSquare(DAError):
    pass


class ErrTooFewShards(DAError):
    pass


_ERR_CLASS = {
    _abi.ERR_TOO_FEW_SHARDS: ErrTooFewShards,
    _abi.ERR_PUSH_ORDER: ErrInvalidPushOrder,
    _abi.ERR_BYZANTINE: ErrByzantineData,
    _abi.ERR_UNREPAIRABLE: ErrUnrepairableDataSquare,
}


class Context:
    """One HIP device context (dagpu_ctx).  Thread-safe (host calls serialise)."""

    def __init__(self, device: int = 0):
        self._L = _abi.lib()
        h = ctypes.c_void_p()
        rc = self._L.dagpu_init(device, ctypes.byref(h))
        if rc != 0:
            raise DAError(rc, f"dagpu_init(device={device}) failed with status {rc}")
        self.handle = h
        self.device = device

    def close(self) -> None:
        if self.handle:
            self._L.dagpu_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_error(self) -> str:
        return self._L.dagpu_last_error(self.handle).decode()

    def repair_stats(self) -> dict:
        """Schedule of the last Repair on this context (dagpu_repair_stats)."""
        out = np.zeros(5, np.int64)
        self.check(self._L.dagpu_repair_stats(self.handle, out.ctypes.data))
        return dict(zip(("rounds", "fills", "reverse_fills", "decodes", "deferred"), (int(x) for x in out)))

    def check(self, rc: int) -> None:
        if rc != 0:
            cls = _ERR_CLASS.get(rc, DAError)
            raise cls(rc, self.last_error())


class PinnedBuffer:
    """Page-locked host memory from dagpu_host_alloc (include/dagpu.h), viewed
    as a flat numpy uint8 array: the input buffer a block-replay caller hands
    to dagpu_extend_batch so its chunked host->device copies run at PCIe speed."""

    def __init__(self, nbytes: int):
        self._L = _abi.lib()
        self.nbytes = int(nbytes)
        p = self._L.dagpu_host_alloc(max(self.nbytes, 1))
        if not p:
            raise MemoryError(f"dagpu_host_alloc({self.nbytes}) failed")
        self.ptr = p
        raw = (ctypes.c_uint8 * max(self.nbytes, 1)).from_address(p)
        self.array = np.frombuffer(raw, dtype=np.uint8)[:self.nbytes]

    def close(self) -> None:
        if self.ptr:
            self.array = None
            self._L.dagpu_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx: Optional[Context] = None
_default_lock = threading.Lock()


def default_context() -> Context:
    global _default_ctx
    with _default_lock:
        if _default_ctx is None:
            _default_ctx = Context(0)
        return _default_ctx


def is_power_of_two(n: int) -> bool:
    """pkg/shares/powers_of_two.go:42-44."""
    return n != 0 and (n & (n - 1)) == 0


def round_up_power_of_two(n: int) -> int:
    r = 1
    while r < n:
        r <<= 1
    return r


def square_size(n_shares: int) -> int:
    """pkg/da/data_availability_header.go:205-207."""
    return round_up_power_of_two(int(math.ceil(math.sqrt(n_shares))))


def _as_matrix(shares) -> np.ndarray:
    if isinstance(shares, np.ndarray):
        a = np.ascontiguousarray(shares, dtype=np.uint8)
        return a.reshape(-1, a.shape[-1]) if a.ndim > 1 else a.reshape(1, -1)
    shares = list(shares)
    if not shares:
        return np.zeros((0, SHARE_SIZE), np.uint8)
    sizes = {len(s) for s in shares}
    if len(sizes) != 1:
        raise DAError(_abi.ERR_SHARE_SIZE, "all chunks must be of equal size")
    return np.frombuffer(b"".join(bytes(s) for s in shares), np.uint8).reshape(len(shares), -1)


class ExtendedDataSquare:
    """EDS held on the host (rsmt2d.ExtendedDataSquare equivalent).

    Row/column roots were computed on the GPU together with the extension; a
    namespace-order failure is reported when the roots are requested, as rsmt2d
    reports it from RowRoots()/ColRoots()."""

    def __init__(self, k: int, data: np.ndarray, row_roots: np.ndarray, col_roots: np.ndarray,
                 dah: bytes, status: int, ctx: Context):
        self.k = k
        self.data = data  # (2k, 2k, 512) uint8
        self._rr = row_roots
        self._cr = col_roots
        self._dah = dah
        self._status = status
        self._ctx = ctx

    def width(self) -> int:
        return 2 * self.k

    def cell(self, r: int, c: int) -> bytes:
        return self.data[r, c].tobytes()

    def row(self, r: int) -> List[bytes]:
        return [self.data[r, c].tobytes() for c in range(2 * self.k)]

    def col(self, c: int) -> List[bytes]:
        return [self.data[r, c].tobytes() for r in range(2 * self.k)]

    def flattened_ods(self) -> List[bytes]:
        return [self.data[r, c].tobytes() for r in range(self.k) for c in range(self.k)]

    def _check(self) -> None:
        if self._status != 0:
            cls = _ERR_CLASS.get(self._status, DAError)
            raise cls(self._status, "invalid push order: namespaces of original data square are not sorted")

    def row_roots(self) -> List[bytes]:
        self._check()
        return [bytes(r) for r in self._rr]

    def col_roots(self) -> List[bytes]:
        self._check()
        return [bytes(r) for r in self._cr]


def extend_shares(shares, ctx: Optional[Context] = None, keep_eds: bool = True) -> ExtendedDataSquare:
    """da.ExtendShares (pkg/da/data_availability_header.go:65-75)."""
    m = _as_matrix(shares)
    n = m.shape[0]
    if not is_power_of_two(n):
        raise DAError(_abi.ERR_NOT_POW2, f"number of shares is not a power of 2: got {n}")
    k = square_size(n)
    if k * k != n:
        raise DAError(_abi.ERR_NOT_SQUARE, "number of chunks must be a square number")
    ctx = ctx or default_context()
    w = 2 * k
    eds = np.empty((w, w, m.shape[1]), np.uint8) if keep_eds else None
    rr = np.empty((w, ROOT_SIZE), np.uint8)
    cr = np.empty((w, ROOT_SIZE), np.uint8)
    dah = np.empty(HASH_SIZE, np.uint8)
    rc = ctx._L.dagpu_extend_shares(ctx.handle, _abi.addr(m), n, m.shape[1], _abi.addr(eds),
                                    _abi.addr(rr), _abi.addr(cr), _abi.addr(dah))
    status = 0
    if rc == _abi.ERR_PUSH_ORDER:
        status = rc
    elif rc != 0:
        ctx.check(rc)
    return ExtendedDataSquare(k, eds, rr, cr, dah.tobytes(), status, ctx)


class DataAvailabilityHeader:
    """pkg/da/data_availability_header.go:31-40."""

    def __init__(self, row_roots: Sequence[bytes] = (), column_roots: Sequence[bytes] = (),
                 _hash: Optional[bytes] = None):
        self.row_roots = [bytes(r) for r in row_roots]
        self.column_roots = [bytes(r) for r in column_roots]
        self._hash = _hash or b""

    def hash(self) -> bytes:
        """Memoised RFC-6962 root of rowRoots || colRoots (:92-108)."""
        if self._hash:
            return self._hash
        w = len(self.row_roots)
        if w != len(self.column_roots):
            raise DAError(_abi.ERR_ARG, "unequal number of row and column roots")
        rr = np.frombuffer(b"".join(self.row_roots), np.uint8) if w else np.zeros(1, np.uint8)
        cr = np.frombuffer(b"".join(self.column_roots), np.uint8) if w else np.zeros(1, np.uint8)
        out = np.zeros(HASH_SIZE, np.uint8)
        rc = _abi.lib().dagpu_dah_hash(_abi.addr(rr), _abi.addr(cr), w, _abi.addr(out))
        if rc != 0:
            raise DAError(rc, "dah hash failed")
        self._hash = out.tobytes()
        return self._hash

    def square_size(self) -> int:
        return len(self.row_roots) // 2

    def is_zero(self) -> bool:
        return len(self.column_roots) == 0 or len(self.row_roots) == 0

    def equals(self, other: "DataAvailabilityHeader") -> bool:
        return self.hash() == other.hash()

    def __str__(self) -> str:
        return self.hash().hex().upper()

    def validate_basic(self) -> None:
        """pkg/da/data_availability_header.go:134-162."""
        if len(self.column_roots) < MIN_EXTENDED_SQUARE_WIDTH or len(self.row_roots) < MIN_EXTENDED_SQUARE_WIDTH:
            raise DAError(_abi.ERR_ARG,
                          f"minimum valid DataAvailabilityHeader has at least {MIN_EXTENDED_SQUARE_WIDTH} row and column roots")
        if len(self.column_roots) > MAX_EXTENDED_SQUARE_WIDTH or len(self.row_roots) > MAX_EXTENDED_SQUARE_WIDTH:
            raise DAError(_abi.ERR_ARG,
                          f"maximum valid DataAvailabilityHeader has at most {MAX_EXTENDED_SQUARE_WIDTH} row and column roots")
        if len(self.column_roots) != len(self.row_roots):
            raise DAError(_abi.ERR_ARG,
                          f"unequal number of row and column roots: row {len(self.row_roots)} col {len(self.column_roots)}")
        if len(self.hash()) != HASH_SIZE:
            raise DAError(_abi.ERR_ARG, f"wrong hash: expected size to be {HASH_SIZE} bytes")

    def to_proto(self) -> bytes:
        """ToProto (pkg/da/data_availability_header.go:110-119) serialised as the
        celestia.core.v1.da.DataAvailabilityHeader message
        (proto/celestia/core/v1/da/data_availability_header.proto): field 1
        repeated bytes row_roots, field 2 repeated bytes column_roots."""
        out = bytearray()
        for tag, roots in ((0x0A, self.row_roots), (0x12, self.column_roots)):
            for r in roots:
                out.append(tag)
                out += _varint(len(r))
                out += r
        return bytes(out)


def _varint(v: int) -> bytes:
    b = bytearray()
    while True:
        if v < 0x80:
            b.append(v)
            return bytes(b)
        b.append((v & 0x7F) | 0x80)
        v >>= 7


def data_availability_header_from_proto(buf: bytes) -> DataAvailabilityHeader:
    """DataAvailabilityHeaderFromProto (:121-132): decode the proto message, then
    ValidateBasic.  Unknown fields are skipped as proto3 requires."""
    rows, cols = [], []
    i, n = 0, len(buf)

    def varint():
        nonlocal i
        v, shift = 0, 0
        while True:
            if i >= n:
                raise DAError(_abi.ERR_ARG, "proto: truncated varint")
            c = buf[i]
            i += 1
            v |= (c & 0x7F) << shift
            if c < 0x80:
                return v
            shift += 7

    while i < n:
        key = varint()
        field, wt = key >> 3, key & 7
        if wt == 2:
            ln = varint()
            if i + ln > n:
                raise DAError(_abi.ERR_ARG, "proto: truncated bytes field")
            val = bytes(buf[i:i + ln])
            i += ln
            if field == 1:
                rows.append(val)
            elif field == 2:
                cols.append(val)
        elif wt == 0:
            varint()
        elif wt == 1:
            i += 8
        elif wt == 5:
            i += 4
        else:
            raise DAError(_abi.ERR_ARG, f"proto: unsupported wire type {wt}")
    dah = DataAvailabilityHeader(rows, cols)
    dah.validate_basic()
    return dah


def nil_dah_hash() -> bytes:
    """(*DataAvailabilityHeader)(nil).Hash() == merkle.HashFromByteSlices(nil)."""
    return DataAvailabilityHeader().hash()


def new_data_availability_header(eds: ExtendedDataSquare) -> DataAvailabilityHeader:
    """da.NewDataAvailabilityHeader (pkg/da/data_availability_header.go:44-63)."""
    rr = eds.row_roots()
    cr = eds.col_roots()
    return DataAvailabilityHeader(rr, cr, eds._dah)


def tail_padding_share() -> bytes:
    """pkg/shares/padding.go:84-90 (TailPaddingShare): ns | info(v0, start) | len 0 | zeros."""
    return TAIL_PADDING_NAMESPACE + b"\x01" + b"\x00" * 4 + b"\x00" * (SHARE_SIZE - 29 - 5)


def min_shares() -> List[bytes]:
    """pkg/da/data_availability_header.go:193-201."""
    return [tail_padding_share()]


def min_data_availability_header(ctx: Optional[Context] = None) -> DataAvailabilityHeader:
    """pkg/da/data_availability_header.go:179-190."""
    eds = extend_shares(min_shares(), ctx)
    return new_data_availability_header(eds)


class LeoRSCodec:
    """rsmt2d.Codec backed by the GPU Leopard encoder (LeoRSCodec equivalent)."""

    def __init__(self, ctx: Optional[Context] = None):
        self._ctx = ctx  # opened on first use, so the host-side checks need no GPU

    @property
    def ctx(self) -> Context:
        if self._ctx is None:
            self._ctx = default_context()
        return self._ctx

    def name(self) -> str:
        return "Leopard"

    def max_chunks(self) -> int:
        """rsmt2d Codec.MaxChunks: the square of the widest codec vector
        (dagpu_max_codec_width()^2 = 32768^2, Leopard GF(2^16)'s 65536 shards,
        as upstream LeoRSCodec reports).  Squares stop earlier: one GPU holds an
        EDS up to dagpu_max_square_width() (include/dagpu.h)."""
        w = int(_abi.lib().dagpu_max_codec_width())
        return w * w

    def encode(self, data: Sequence[bytes]) -> List[bytes]:
        m = _as_matrix(data)
        k, shard = m.shape
        par = np.empty_like(m)
        self.ctx.check(self.ctx._L.dagpu_encode(self.ctx.handle, k, 1, shard, _abi.addr(m), _abi.addr(par)))
        return [par[i].tobytes() for i in range(k)]

    def encode_batch(self, data: np.ndarray) -> np.ndarray:
        """data: (nvec, k, shard) -> parity (nvec, k, shard)."""
        d = np.ascontiguousarray(data, np.uint8)
        nvec, k, shard = d.shape
        par = np.empty_like(d)
        self.ctx.check(self.ctx._L.dagpu_encode(self.ctx.handle, k, nvec, shard, _abi.addr(d), _abi.addr(par)))
        return par

    def decode(self, shards: Sequence[Optional[bytes]]) -> List[bytes]:
        """Leopard Reconstruct: None marks a missing shard; returns all 2k shards."""
        n = len(shards)
        size = next((len(s) for s in shards if s is not None), None)
        if size is None:  # reedsolomon Reconstruct with no shard at all
            raise ErrTooFewShards(_abi.ERR_TOO_FEW_SHARDS, "too few shards given")
        buf = np.zeros((n, size), np.uint8)
        present = np.zeros(n, np.uint8)
        for i, s in enumerate(shards):
            if s is not None:
                buf[i] = np.frombuffer(bytes(s), np.uint8)
                present[i] = 1
        self.ctx.check(self.ctx._L.dagpu_decode(self.ctx.handle, n // 2, 1, size, _abi.addr(buf),
                                                _abi.addr(present)))
        return [buf[i].tobytes() for i in range(n)]


AXIS_NAMES = ("row", "col")


def repair(eds: np.ndarray, present: np.ndarray, row_roots, col_roots,
           ctx: Optional[Context] = None):
    """rsmt2d ExtendedDataSquare.Repair(rowRoots, colRoots) on the GPU.

    eds: (2k, 2k, 512) uint8 with arbitrary bytes in missing cells; present:
    (2k, 2k) bool.  Returns (repaired eds, present after repair).  Raises
    ErrByzantineData (with .axis/.index/.rebuilt_axis/.rebuilt_index, and
    .eds/.present as rsmt2d leaves the square), ErrUnrepairableDataSquare or
    DAError("bad root input: <axis> <i> expected ... got ...")."""
    ctx = ctx or default_context()
    e = np.ascontiguousarray(eds, dtype=np.uint8).copy()
    w = e.shape[0]
    p = np.ascontiguousarray(present, dtype=np.uint8).reshape(w, w).copy()
    rr = np.ascontiguousarray(np.frombuffer(b"".join(bytes(r) for r in row_roots), np.uint8))
    cr = np.ascontiguousarray(np.frombuffer(b"".join(bytes(c) for c in col_roots), np.uint8))
    byz = np.full(4, -1, np.int32)
    rc = ctx._L.dagpu_repair_ex(ctx.handle, w // 2, _abi.addr(e), _abi.addr(p), _abi.addr(rr), _abi.addr(cr),
                                _abi.addr(byz))
    if rc != 0:
        err = _ERR_CLASS.get(rc, DAError)(rc, ctx.last_error())
        if isinstance(err, ErrByzantineData) and byz[0] >= 0:
            err.axis, err.index = AXIS_NAMES[byz[0]], int(byz[1])
            err.rebuilt_axis, err.rebuilt_index = AXIS_NAMES[byz[2]], int(byz[3])
        err.byz = [int(x) for x in byz]
        err.eds, err.present = e, p.astype(bool)
        raise err
    return e, p.astype(bool)


def extend_batch(ods: np.ndarray, ks: Sequence[int], ctx: Optional[Context] = None,
                 want_eds: bool = False):
    """Batched host API (mixed k).  ods: concatenated ODS bytes.  Returns
    (eds or None, row_roots list, col_roots list, dah (n,32), status (n,))."""
    ctx = ctx or default_context()
    ks = np.ascontiguousarray(ks, dtype=np.uint32)
    n = len(ks)
    ods = np.ascontiguousarray(ods, dtype=np.uint8).reshape(-1)
    tot_root = int(sum(2 * int(k) * ROOT_SIZE for k in ks))
    tot_eds = int(sum(4 * int(k) * int(k) * SHARE_SIZE for k in ks))
    eds = np.empty(tot_eds, np.uint8) if want_eds else None
    rr = np.empty(max(tot_root, 1), np.uint8)
    cr = np.empty(max(tot_root, 1), np.uint8)
    dah = np.empty((max(n, 1), HASH_SIZE), np.uint8)
    status = np.zeros(max(n, 1), np.int32)
    rc = ctx._L.dagpu_extend_batch(ctx.handle, _abi.addr(ods), _abi.addr(ks), n, _abi.addr(eds),
                                   _abi.addr(rr), _abi.addr(cr), _abi.addr(dah), _abi.addr(status))
    if rc not in (0, _abi.ERR_PUSH_ORDER):
        ctx.check(rc)
    rrs, crs, off = [], [], 0
    for k in ks:
        w = 2 * int(k)
        rrs.append(rr[off:off + w * ROOT_SIZE].reshape(w, ROOT_SIZE))
        crs.append(cr[off:off + w * ROOT_SIZE].reshape(w, ROOT_SIZE))
        off += w * ROOT_SIZE
    return eds, rrs, crs, dah[:n], status[:n]
