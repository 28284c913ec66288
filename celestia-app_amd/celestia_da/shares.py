"""Share encoding on both sides of the hot path, host-side
mirror of pkg/shares and the namespace constants it uses:

  Share (Namespace, InfoByte, SequenceLen, IsPadding, RawData,
      RawDataUsingReserved)                 pkg/shares/shares.go
  Builder                                   pkg/shares/share_builder.go
  CompactShareSplitter, MarshalDelimitedTx  pkg/shares/split_compact_shares.go
  SparseShareSplitter, SplitBlobs           pkg/shares/split_sparse_shares.go, share_splitting.go
  CompactShareCounter                       pkg/shares/counter.go
  NamespacePaddingShare(s), Tail/Reserved padding
                                            pkg/shares/padding.go
  ParseTxs, ParseBlobs, ParseShares, ShareSequence,
      CompactSharesNeeded, SparseSharesNeeded
                                            pkg/shares/parse*.go, share_sequence.go
  GetShareRangeForNamespace, Range          pkg/shares/namespace.go, range.go
  InfoByte, ReservedBytes, DelimLen, RawTxSize, ParseDelimiter,
      AvailableBytesFrom{Compact,Sparse}Shares
                                            pkg/shares/info_byte.go, reserved_bytes.go, utils.go
  namespace constants / validation          pkg/namespace/consts.go, namespace.go

This is byte bookkeeping that produces the ODS the GPU path extends (and
parses squares the GPU path repaired); it is control-heavy and stays on the
host, as SURVEY.md §8(f)-4 plans.  Namespaces are 29-byte `bytes`
(version || 28-byte ID); shares are 512-byte `bytes` wrapped in `Share`.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

# ---- pkg/appconsts/global_consts.go -----------------------------------------------------
SHARE_SIZE = 512
NAMESPACE_VERSION_SIZE = 1
NAMESPACE_ID_SIZE = 28
NAMESPACE_SIZE = NAMESPACE_VERSION_SIZE + NAMESPACE_ID_SIZE
SHARE_INFO_BYTES = 1
SEQUENCE_LEN_BYTES = 4
COMPACT_SHARE_RESERVED_BYTES = 4
SHARE_VERSION_ZERO = 0
MAX_SHARE_VERSION = 127
SUPPORTED_SHARE_VERSIONS = (SHARE_VERSION_ZERO,)
FIRST_COMPACT_SHARE_CONTENT_SIZE = SHARE_SIZE - NAMESPACE_SIZE - SHARE_INFO_BYTES - SEQUENCE_LEN_BYTES \
    - COMPACT_SHARE_RESERVED_BYTES  # 474
CONTINUATION_COMPACT_SHARE_CONTENT_SIZE = SHARE_SIZE - NAMESPACE_SIZE - SHARE_INFO_BYTES \
    - COMPACT_SHARE_RESERVED_BYTES  # 478
FIRST_SPARSE_SHARE_CONTENT_SIZE = SHARE_SIZE - NAMESPACE_SIZE - SHARE_INFO_BYTES - SEQUENCE_LEN_BYTES  # 478
CONTINUATION_SPARSE_SHARE_CONTENT_SIZE = SHARE_SIZE - NAMESPACE_SIZE - SHARE_INFO_BYTES  # 482
MIN_SQUARE_SIZE = 1
MIN_SHARE_COUNT = MIN_SQUARE_SIZE * MIN_SQUARE_SIZE

# ---- pkg/namespace/consts.go ---------------------------------------------------------------
NAMESPACE_VERSION_ZERO = 0
NAMESPACE_VERSION_MAX = 255
NAMESPACE_VERSION_ZERO_PREFIX_SIZE = 18
NAMESPACE_VERSION_ZERO_ID_SIZE = NAMESPACE_ID_SIZE - NAMESPACE_VERSION_ZERO_PREFIX_SIZE  # 10


def _primary_reserved(last: int) -> bytes:
    return bytes([NAMESPACE_VERSION_ZERO]) + b"\x00" * (NAMESPACE_ID_SIZE - 1) + bytes([last])


def _secondary_reserved(last: int) -> bytes:
    return bytes([NAMESPACE_VERSION_MAX]) + b"\xff" * (NAMESPACE_ID_SIZE - 1) + bytes([last])


TX_NAMESPACE = _primary_reserved(0x01)
INTERMEDIATE_STATE_ROOTS_NAMESPACE = _primary_reserved(0x02)
PAY_FOR_BLOB_NAMESPACE = _primary_reserved(0x04)
PRIMARY_RESERVED_PADDING_NAMESPACE = _primary_reserved(0xFF)
MAX_PRIMARY_RESERVED_NAMESPACE = _primary_reserved(0xFF)
MIN_SECONDARY_RESERVED_NAMESPACE = _secondary_reserved(0x00)
TAIL_PADDING_NAMESPACE = _secondary_reserved(0xFE)
PARITY_SHARES_NAMESPACE = _secondary_reserved(0xFF)


class ShareError(ValueError):
    """Errors the reference returns as `error` from pkg/shares / pkg/namespace."""


def validate_namespace(ns: bytes) -> bytes:
    """namespace.From: 29 bytes, version 0 or 255, version-0 IDs start with 18 zero bytes."""
    if len(ns) != NAMESPACE_SIZE:
        raise ShareError(f"invalid namespace length: {len(ns)} must be {NAMESPACE_SIZE}")
    version, nid = ns[0], ns[1:]
    if version not in (NAMESPACE_VERSION_ZERO, NAMESPACE_VERSION_MAX):
        raise ShareError(f"unsupported namespace version {version}")
    if version == NAMESPACE_VERSION_ZERO and nid[:NAMESPACE_VERSION_ZERO_PREFIX_SIZE] != \
            b"\x00" * NAMESPACE_VERSION_ZERO_PREFIX_SIZE:
        raise ShareError(f"unsupported namespace id with version {version}. ID must start with "
                         f"{NAMESPACE_VERSION_ZERO_PREFIX_SIZE} leading zeros")
    return bytes(ns)


def new_namespace_v0(sub_id: bytes) -> bytes:
    """namespace.NewV0: version 0, 18 zero bytes, sub-ID left-padded to 10 bytes."""
    if len(sub_id) > NAMESPACE_VERSION_ZERO_ID_SIZE:
        raise ShareError(f"subID must be <= {NAMESPACE_VERSION_ZERO_ID_SIZE}, but it was {len(sub_id)} bytes")
    return validate_namespace(b"\x00" + b"\x00" * NAMESPACE_VERSION_ZERO_PREFIX_SIZE
                              + bytes(sub_id).rjust(NAMESPACE_VERSION_ZERO_ID_SIZE, b"\x00"))


def is_tx_namespace(ns: bytes) -> bool:
    return ns == TX_NAMESPACE


def is_pay_for_blob_namespace(ns: bytes) -> bool:
    return ns == PAY_FOR_BLOB_NAMESPACE


def is_compact_namespace(ns: bytes) -> bool:
    """shares.isCompactShare / Share.IsCompactShare: tx and PFB namespaces."""
    return ns == TX_NAMESPACE or ns == PAY_FOR_BLOB_NAMESPACE


def is_reserved_namespace(ns: bytes) -> bool:
    return ns <= MAX_PRIMARY_RESERVED_NAMESPACE or ns >= MIN_SECONDARY_RESERVED_NAMESPACE


# ---- info_byte.go / reserved_bytes.go / utils.go -----------------------------------------

def new_info_byte(version: int, is_sequence_start: bool) -> int:
    if version > MAX_SHARE_VERSION:
        raise ShareError(f"version {version} must be less than or equal to {MAX_SHARE_VERSION}")
    return (version << 1) + (1 if is_sequence_start else 0)


def parse_info_byte(b: int) -> int:
    return new_info_byte(b >> 1, b % 2 == 1)


def new_reserved_bytes(byte_index: int) -> bytes:
    if byte_index >= SHARE_SIZE:
        raise ShareError(f"byte index {byte_index} must be less than share size {SHARE_SIZE}")
    return struct.pack(">I", byte_index)


def parse_reserved_bytes(reserved: bytes) -> int:
    if len(reserved) != COMPACT_SHARE_RESERVED_BYTES:
        raise ShareError(f"reserved bytes must be of length {COMPACT_SHARE_RESERVED_BYTES}")
    idx = struct.unpack(">I", reserved)[0]
    if SHARE_SIZE <= idx:
        raise ShareError(f"byteIndex must be less than share size {SHARE_SIZE}")
    return idx


def put_uvarint(v: int) -> bytes:
    """encoding/binary.PutUvarint."""
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def read_uvarint(buf: bytes) -> Tuple[int, int]:
    """encoding/binary.ReadUvarint over a 10-byte window: (value, bytes read);
    raises on overflow or a truncated varint."""
    x, s = 0, 0
    for i, b in enumerate(buf[:10]):
        if i == 9 and b > 1:
            raise ShareError("binary: varint overflows a 64-bit integer")
        if b < 0x80:
            return x | (b << s), i + 1
        x |= (b & 0x7F) << s
        s += 7
    raise ShareError("unexpected EOF")


def delim_len(size: int) -> int:
    return len(put_uvarint(size))


def raw_tx_size(desired_size: int) -> int:
    """RawTxSize: the tx length that occupies `desired_size` bytes once delimited."""
    return desired_size - delim_len(desired_size)


def marshal_delimited_tx(tx: bytes) -> bytes:
    return put_uvarint(len(tx)) + bytes(tx)


def zero_pad_if_necessary(share: bytes, width: int) -> Tuple[bytes, int]:
    if len(share) >= width:
        return share, 0
    return share + b"\x00" * (width - len(share)), width - len(share)


def parse_delimiter(data: bytes) -> Tuple[bytes, int]:
    """ParseDelimiter: (data after the varint length prefix, unit length)."""
    if len(data) == 0:
        return data, 0
    window, _ = zero_pad_if_necessary(data[:10], 10)
    n_len, _ = read_uvarint(window)
    return data[len(put_uvarint(n_len)):], n_len


def available_bytes_from_compact_shares(n: int) -> int:
    if n <= 0:
        return 0
    if n == 1:
        return FIRST_COMPACT_SHARE_CONTENT_SIZE
    return (n - 1) * CONTINUATION_COMPACT_SHARE_CONTENT_SIZE + FIRST_COMPACT_SHARE_CONTENT_SIZE


def available_bytes_from_sparse_shares(n: int) -> int:
    if n <= 0:
        return 0
    if n == 1:
        return FIRST_SPARSE_SHARE_CONTENT_SIZE
    return (n - 1) * CONTINUATION_SPARSE_SHARE_CONTENT_SIZE + FIRST_SPARSE_SHARE_CONTENT_SIZE


def compact_shares_needed(sequence_len: int) -> int:
    if sequence_len == 0:
        return 0
    if sequence_len < FIRST_COMPACT_SHARE_CONTENT_SIZE:
        return 1
    avail, need = FIRST_COMPACT_SHARE_CONTENT_SIZE, 1
    while avail < sequence_len:
        avail += CONTINUATION_COMPACT_SHARE_CONTENT_SIZE
        need += 1
    return need


def sparse_shares_needed(sequence_len: int) -> int:
    if sequence_len == 0:
        return 0
    if sequence_len < FIRST_SPARSE_SHARE_CONTENT_SIZE:
        return 1
    avail, need = FIRST_SPARSE_SHARE_CONTENT_SIZE, 1
    while avail < sequence_len:
        avail += CONTINUATION_SPARSE_SHARE_CONTENT_SIZE
        need += 1
    return need


def is_power_of_two(v: int) -> bool:
    return v != 0 and v & (v - 1) == 0


def round_up_power_of_two(v: int) -> int:
    r = 1
    while r < v:
        r <<= 1
    return r


def round_up_power_of_two_strict(v: int) -> int:
    r = round_up_power_of_two(v)
    return r * 2 if r == v else r


def round_down_power_of_two(v: int) -> int:
    if v <= 0:
        raise ShareError(f"input {v} must be positive")
    r = round_up_power_of_two(v)
    return r if r == v else r // 2


# ---- range.go ------------------------------------------------------------------------------

@dataclass
class Range:
    start: int = 0
    end: int = 0

    def is_empty(self) -> bool:
        return self.start == 0 and self.end == 0

    def add(self, v: int) -> None:
        self.start += v
        self.end += v


# ---- shares.go -----------------------------------------------------------------------------

class Share:
    """A 512-byte share (shares.Share)."""

    __slots__ = ("data",)

    def __init__(self, data: bytes):
        if len(data) != SHARE_SIZE:
            raise ShareError(f"share data must be {SHARE_SIZE} bytes, got {len(data)}")
        self.data = bytes(data)

    def __eq__(self, other) -> bool:
        return isinstance(other, Share) and self.data == other.data

    def __repr__(self) -> str:
        return f"Share({self.data[:NAMESPACE_SIZE + 5].hex()}...)"

    def to_bytes(self) -> bytes:
        return self.data

    def namespace(self) -> bytes:
        return validate_namespace(self.data[:NAMESPACE_SIZE])

    def info_byte(self) -> int:
        return parse_info_byte(self.data[NAMESPACE_SIZE])

    def version(self) -> int:
        return self.info_byte() >> 1

    def does_support_versions(self, supported: Sequence[int]) -> None:
        v = self.version()
        if v not in supported:
            raise ShareError(f"unsupported share version {v} is not present in the list of supported share "
                             f"versions {list(supported)}")

    def is_sequence_start(self) -> bool:
        return self.info_byte() % 2 == 1

    def is_compact_share(self) -> bool:
        return is_compact_namespace(self.namespace())

    def sequence_len(self) -> int:
        if not self.is_sequence_start():
            return 0
        s = NAMESPACE_SIZE + SHARE_INFO_BYTES
        return struct.unpack(">I", self.data[s:s + SEQUENCE_LEN_BYTES])[0]

    def is_padding(self) -> bool:
        ns = self.namespace()
        namespace_padding = self.is_sequence_start() and self.sequence_len() == 0
        return namespace_padding or ns == TAIL_PADDING_NAMESPACE or ns == PRIMARY_RESERVED_PADDING_NAMESPACE

    def _raw_data_start(self) -> int:
        i = NAMESPACE_SIZE + SHARE_INFO_BYTES
        if self.is_sequence_start():
            i += SEQUENCE_LEN_BYTES
        if self.is_compact_share():
            i += COMPACT_SHARE_RESERVED_BYTES
        return i

    def raw_data(self) -> bytes:
        """Data after namespace, info byte, sequence length and reserved bytes."""
        return self.data[self._raw_data_start():]

    def raw_data_using_reserved(self) -> bytes:
        """Data starting at the first unit that begins in this share (compact
        shares' reserved bytes); empty when no unit starts here."""
        i = NAMESPACE_SIZE + SHARE_INFO_BYTES
        if self.is_sequence_start():
            i += SEQUENCE_LEN_BYTES
        if self.is_compact_share():
            i = parse_reserved_bytes(self.data[i:i + COMPACT_SHARE_RESERVED_BYTES])
        if i == 0:
            return b""
        return self.data[i:]


def to_bytes(shares: Sequence[Share]) -> List[bytes]:
    return [s.data for s in shares]


def from_bytes(raw: Sequence[bytes]) -> List[Share]:
    return [Share(b) for b in raw]


# ---- share_builder.go ----------------------------------------------------------------------

class Builder:
    def __init__(self, namespace: bytes, share_version: int, is_first_share: bool):
        self.namespace = namespace
        self.share_version = share_version
        self.is_first_share = is_first_share
        self.is_compact_share = is_compact_namespace(namespace)
        info = new_info_byte(share_version, is_first_share)
        raw = bytearray(namespace) + bytes([info])
        if is_first_share:
            raw += b"\x00" * SEQUENCE_LEN_BYTES
        if self.is_compact_share:
            raw += b"\x00" * COMPACT_SHARE_RESERVED_BYTES
        self.raw = raw

    def available_bytes(self) -> int:
        return SHARE_SIZE - len(self.raw)

    def import_raw_share(self, raw: bytes) -> "Builder":
        self.raw = bytearray(raw)
        return self

    def add_data(self, data: bytes) -> Optional[bytes]:
        """Append as much of `data` as fits; return the leftover (None if all fit)."""
        left = SHARE_SIZE - len(self.raw)
        if len(data) <= left:
            self.raw += data
            return None
        self.raw += data[:left]
        return data[left:]

    def build(self) -> Share:
        return Share(bytes(self.raw))

    def is_empty_share(self) -> bool:
        expected = NAMESPACE_SIZE + SHARE_INFO_BYTES
        if self.is_compact_share:
            expected += COMPACT_SHARE_RESERVED_BYTES
        if self.is_first_share:
            expected += SEQUENCE_LEN_BYTES
        return len(self.raw) == expected

    def zero_pad_if_necessary(self) -> int:
        padded, n = zero_pad_if_necessary(bytes(self.raw), SHARE_SIZE)
        self.raw = bytearray(padded)
        return n

    def _index_of_reserved_bytes(self) -> int:
        i = NAMESPACE_SIZE + SHARE_INFO_BYTES
        return i + SEQUENCE_LEN_BYTES if self.is_first_share else i

    def maybe_write_reserved_bytes(self) -> None:
        """Point the reserved bytes at the next unit if they are still empty."""
        if not self.is_compact_share:
            raise ShareError("this is not a compact share")
        i = self._index_of_reserved_bytes()
        if parse_reserved_bytes(bytes(self.raw[i:i + COMPACT_SHARE_RESERVED_BYTES])) != 0:
            return
        self.raw[i:i + COMPACT_SHARE_RESERVED_BYTES] = new_reserved_bytes(len(self.raw))

    def write_sequence_len(self, sequence_len: int) -> None:
        if not self.is_first_share:
            raise ShareError("not the first share")
        s = NAMESPACE_SIZE + SHARE_INFO_BYTES
        self.raw[s:s + SEQUENCE_LEN_BYTES] = struct.pack(">I", sequence_len)

    def flip_sequence_start(self) -> None:
        self.raw[NAMESPACE_SIZE] ^= 0x01


# ---- counter.go ----------------------------------------------------------------------------

class CompactShareCounter:
    """Counts the compact shares a sequence of delimited units occupies."""

    def __init__(self):
        self.last_shares = 0
        self.last_remainder = 0
        self.shares = 0
        self.remainder = 0

    def add(self, data_len: int) -> int:
        """Add a unit of `data_len` bytes (before delimiting); return the change
        in the number of shares."""
        data_len += delim_len(data_len)
        self.last_remainder, self.last_shares = self.remainder, self.shares
        if self.shares == 0:
            if data_len >= FIRST_COMPACT_SHARE_CONTENT_SIZE - self.remainder:
                data_len -= FIRST_COMPACT_SHARE_CONTENT_SIZE - self.remainder
                self.shares += 1
                self.remainder = 0
            else:
                self.remainder += data_len
                data_len = 0
        if data_len >= CONTINUATION_COMPACT_SHARE_CONTENT_SIZE - self.remainder:
            data_len -= CONTINUATION_COMPACT_SHARE_CONTENT_SIZE - self.remainder
            self.shares += 1
            self.remainder = 0
        else:
            self.remainder += data_len
            data_len = 0
        if data_len > 0:
            self.shares += data_len // CONTINUATION_COMPACT_SHARE_CONTENT_SIZE
            self.remainder = data_len % CONTINUATION_COMPACT_SHARE_CONTENT_SIZE
        diff = self.shares - self.last_shares
        if self.last_remainder == 0 and self.remainder > 0:
            diff += 1
        elif self.last_remainder > 0 and self.remainder == 0:
            diff -= 1
        return diff

    def revert(self) -> None:
        self.shares, self.remainder = self.last_shares, self.last_remainder

    def size(self) -> int:
        return self.shares if self.remainder == 0 else self.shares + 1


# ---- split_compact_shares.go -----------------------------------------------------------------

class CompactShareSplitter:
    """Writes length-delimited txs (or wrapped PFBs) into compact shares."""

    def __init__(self, namespace: bytes, share_version: int = SHARE_VERSION_ZERO):
        self.namespace = namespace
        self.share_version = share_version
        self.shares: List[Share] = []
        self.builder = Builder(namespace, share_version, True)
        self.done = False
        self.share_ranges: Dict[bytes, Range] = {}  # keyed by tx bytes (TxKey = sha256(tx) in Go)

    def write_tx(self, tx: bytes) -> None:
        start = len(self.shares)
        self._write(marshal_delimited_tx(tx))
        self.share_ranges[bytes(tx)] = Range(start, self.count())

    def _write(self, raw: bytes) -> None:
        if self.done:
            # remove the last share added by Export if it is not empty
            if not self.builder.is_empty_share():
                self.shares = self.shares[:-1]
            self.done = False
        self.builder.maybe_write_reserved_bytes()
        while True:
            left = self.builder.add_data(raw)
            if left is None:
                break
            self._stack_pending()
            raw = left
        if self.builder.available_bytes() == 0:
            self._stack_pending()

    def _stack_pending(self) -> None:
        self.shares.append(self.builder.build())
        self.builder = Builder(self.namespace, self.share_version, False)

    def export(self) -> List[Share]:
        if self._is_empty():
            return []
        if self.done:
            return self.shares
        padding = 0
        if not self.builder.is_empty_share():
            padding = self.builder.zero_pad_if_necessary()
            self._stack_pending()
        self._write_sequence_len(self._sequence_len(padding))
        self.done = True
        return self.shares

    def share_ranges_with_offset(self, offset: int) -> Dict[bytes, Range]:
        return {k: Range(v.start + offset, v.end + offset) for k, v in self.share_ranges.items()}

    def _write_sequence_len(self, sequence_len: int) -> None:
        if self._is_empty():
            return
        b = Builder(self.namespace, self.share_version, True).import_raw_share(self.shares[0].to_bytes())
        b.write_sequence_len(sequence_len)
        self.shares[0] = b.build()

    def _sequence_len(self, padding: int) -> int:
        if not self.shares:
            return 0
        if len(self.shares) == 1:
            return FIRST_COMPACT_SHARE_CONTENT_SIZE - padding
        return FIRST_COMPACT_SHARE_CONTENT_SIZE + (len(self.shares) - 1) * CONTINUATION_COMPACT_SHARE_CONTENT_SIZE \
            - padding

    def _is_empty(self) -> bool:
        return len(self.shares) == 0 and self.builder.is_empty_share()

    def count(self) -> int:
        if not self.builder.is_empty_share() and not self.done:
            return len(self.shares) + 1
        return len(self.shares)


# ---- padding.go ------------------------------------------------------------------------------

def namespace_padding_share(namespace: bytes, share_version: int = SHARE_VERSION_ZERO) -> Share:
    b = Builder(namespace, share_version, True)
    b.write_sequence_len(0)
    b.add_data(b"\x00" * FIRST_SPARSE_SHARE_CONTENT_SIZE)
    return b.build()


def namespace_padding_shares(namespace: bytes, share_version: int, n: int) -> List[Share]:
    if n < 0:
        raise ShareError("n must be positive")
    return [namespace_padding_share(namespace, share_version) for _ in range(n)]


def reserved_padding_shares(n: int) -> List[Share]:
    return namespace_padding_shares(PRIMARY_RESERVED_PADDING_NAMESPACE, SHARE_VERSION_ZERO, n)


def tail_padding_shares(n: int) -> List[Share]:
    return namespace_padding_shares(TAIL_PADDING_NAMESPACE, SHARE_VERSION_ZERO, n)


def tail_padding_share() -> Share:
    return namespace_padding_share(TAIL_PADDING_NAMESPACE, SHARE_VERSION_ZERO)


# ---- blobs (pkg/blob) and split_sparse_shares.go -----------------------------------------

@dataclass
class Blob:
    """blob.Blob: NamespaceId (28 B), Data, ShareVersion, NamespaceVersion."""
    namespace_id: bytes
    data: bytes
    share_version: int = 0
    namespace_version: int = 0

    @staticmethod
    def new(namespace: bytes, data: bytes, share_version: int = 0) -> "Blob":
        return Blob(bytes(namespace[1:]), bytes(data), share_version, namespace[0])

    def namespace(self) -> bytes:
        return bytes([self.namespace_version]) + self.namespace_id

    def validate(self) -> None:
        if len(self.namespace_id) != NAMESPACE_ID_SIZE:
            raise ShareError(f"namespace id must be {NAMESPACE_ID_SIZE} bytes")
        if self.share_version > 255:
            raise ShareError("share version can not be greater than MaxShareVersion")
        if self.namespace_version > NAMESPACE_VERSION_MAX:
            raise ShareError("namespace version can not be greater than MaxNamespaceVersion")
        if len(self.data) == 0:
            raise ShareError("blob data can not be empty")


def sort_blobs(blobs: List[Blob]) -> None:
    """blob.Sort: stable sort by namespace bytes."""
    blobs.sort(key=lambda b: b.namespace())


class SparseShareSplitter:
    def __init__(self):
        self.shares: List[Share] = []

    def write(self, blob: Blob) -> None:
        blob.validate()
        if blob.share_version not in SUPPORTED_SHARE_VERSIONS:
            raise ShareError(f"unsupported share version: {blob.share_version}")
        ns = blob.namespace()
        b = Builder(ns, blob.share_version, True)
        b.write_sequence_len(len(blob.data))
        raw: Optional[bytes] = blob.data
        while raw is not None:
            left = b.add_data(raw)
            if left is None:
                b.zero_pad_if_necessary()
            self.shares.append(b.build())
            b = Builder(ns, blob.share_version, False)
            raw = left

    def write_namespace_padding_shares(self, count: int) -> None:
        if count < 0:
            raise ShareError("cannot write negative namespaced shares")
        if count == 0:
            return
        if not self.shares:
            raise ShareError("cannot write namespace padding shares on an empty SparseShareSplitter")
        last = self.shares[-1]
        self.shares.extend(namespace_padding_shares(last.namespace(), last.version(), count))

    def export(self) -> List[Share]:
        return self.shares

    def count(self) -> int:
        return len(self.shares)


def split_blobs(*blobs: Blob) -> List[Share]:
    w = SparseShareSplitter()
    for b in blobs:
        w.write(b)
    return w.export()


def split_txs(txs: Sequence[bytes], is_index_wrapper) -> Tuple[List[Share], List[Share], Dict[bytes, Range]]:
    """shares.SplitTxs: normal txs into the tx namespace, index-wrapped PFBs into
    the PFB namespace; `is_index_wrapper(tx) -> bool` decides which."""
    tw = CompactShareSplitter(TX_NAMESPACE)
    pw = CompactShareSplitter(PAY_FOR_BLOB_NAMESPACE)
    for tx in txs:
        (pw if is_index_wrapper(tx) else tw).write_tx(tx)
    tx_shares = list(tw.export())
    ranges = tw.share_ranges_with_offset(0)
    pfb_shares = list(pw.export())
    ranges.update(pw.share_ranges_with_offset(len(tx_shares)))
    return tx_shares, pfb_shares, ranges


# ---- parsing (parse.go, parse_compact_shares.go, parse_sparse_shares.go) ------------------

def _parse_raw_data(raw: bytes) -> List[bytes]:
    units = []
    while True:
        actual, unit_len = parse_delimiter(raw)
        if unit_len == 0 or unit_len > len(actual):
            return units
        raw = actual[unit_len:]
        units.append(actual[:unit_len])


def parse_compact_shares(shares: Sequence[Share], supported=SUPPORTED_SHARE_VERSIONS) -> List[bytes]:
    if not shares:
        return []
    for s in shares:
        s.does_support_versions(supported)
    raw = b"".join(s.raw_data_using_reserved() if i == 0 else s.raw_data() for i, s in enumerate(shares))
    return _parse_raw_data(raw)


def parse_txs(shares: Sequence[Share]) -> List[bytes]:
    return parse_compact_shares(shares)


def parse_sparse_shares(shares: Sequence[Share], supported=SUPPORTED_SHARE_VERSIONS) -> List[Blob]:
    if not shares:
        return []
    seqs: List[Tuple[Blob, int]] = []
    for s in shares:
        v = s.version()
        if v not in supported:
            raise ShareError(f"unsupported share version {v} is not present in supported share versions "
                             f"{list(supported)}")
        if s.is_padding():
            continue
        if s.is_sequence_start():
            seqs.append((Blob.new(s.namespace(), s.raw_data(), v), s.sequence_len()))
        else:
            if not seqs:
                raise ShareError(f"continuation share {s!r} without a sequence start share")
            seqs[-1][0].data += s.raw_data()
    out = []
    for blob, n in seqs:
        blob.data = blob.data[:n]
        out.append(blob)
    return out


def parse_blobs(shares: Sequence[Share]) -> List[Blob]:
    return parse_sparse_shares(shares)


@dataclass
class ShareSequence:
    namespace: bytes
    shares: List[Share] = field(default_factory=list)

    def sequence_len(self) -> int:
        if not self.shares:
            raise ShareError("invalid sequence length because share sequence has no shares")
        return self.shares[0].sequence_len()

    def raw_data(self) -> bytes:
        return b"".join(s.raw_data() for s in self.shares)[:self.sequence_len()]

    def is_padding(self) -> bool:
        return len(self.shares) == 1 and self.shares[0].is_padding()

    def valid_sequence_len(self) -> None:
        if not self.shares:
            raise ShareError("invalid sequence length because share sequence has no shares")
        if self.is_padding():
            return
        first = self.shares[0]
        n = compact_shares_needed(first.sequence_len()) if first.is_compact_share() \
            else sparse_shares_needed(first.sequence_len())
        if len(self.shares) != n:
            raise ShareError(f"share sequence has {len(self.shares)} shares but needed {n} shares")


def parse_shares(shares: Sequence[Share], ignore_padding: bool) -> List[ShareSequence]:
    seqs: List[ShareSequence] = []
    cur: Optional[ShareSequence] = None
    for s in shares:
        ns = s.namespace()
        if s.is_sequence_start():
            if cur is not None and cur.shares:
                seqs.append(cur)
            cur = ShareSequence(ns, [s])
        else:
            if cur is None or cur.namespace != ns:
                raise ShareError(f"share sequence has inconsistent namespace IDs with share {s!r}")
            cur.shares.append(s)
    if cur is not None and cur.shares:
        seqs.append(cur)
    for q in seqs:
        q.valid_sequence_len()
    return [q for q in seqs if not (ignore_padding and q.is_padding())]


def get_share_range_for_namespace(shares: Sequence[Share], ns: bytes) -> Range:
    """Range of the shares whose namespace equals `ns` (shares sorted by namespace)."""
    if not shares:
        return Range()
    if ns < shares[0].namespace() or ns > shares[-1].namespace():
        return Range()
    start = -1
    for i, s in enumerate(shares):
        sns = s.namespace()
        if sns > ns and start != -1:
            return Range(start, i)
        if ns == sns and start == -1:
            start = i
    return Range() if start == -1 else Range(start, len(shares))
