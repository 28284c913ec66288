"""Protobuf wire format of the two tx envelopes that square construction reads
and writes, restated for proto3/gogoproto encoding (fields in number order,
zero values omitted, repeated scalars packed):

  blob.Blob      {bytes namespace_id = 1; bytes data = 2; uint32 share_version = 3;
                  uint32 namespace_version = 4;}         proto/celestia/core/v1/blob/blob.proto
  blob.BlobTx    {bytes tx = 1; repeated Blob blobs = 2; string type_id = 3;}   (type_id "BLOB")
      UnmarshalBlobTx / MarshalBlobTx                     pkg/blob/blob.go:56-90
  tmproto.IndexWrapper {bytes tx = 1; repeated uint32 share_indexes = 2; string type_id = 3;}
      (type_id "INDX"; celestia-core v1.29.0-tm-v0.34.29 proto/tendermint/types/types.proto and
      pkg/consts, not vendored in the reference: restated from the published definitions)

The decoder follows gogoproto's generated Unmarshal: unknown fields are
skipped, a wire type that does not match a known field is an error, and
truncated input is an error.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

from .shares import NAMESPACE_ID_SIZE, Blob, put_uvarint

PROTO_BLOB_TX_TYPE_ID = "BLOB"
PROTO_INDEX_WRAPPER_TYPE_ID = "INDX"


class ProtoError(ValueError):
    pass


# ---- wire helpers ------------------------------------------------------------------------

def _key(num: int, wt: int) -> bytes:
    return put_uvarint((num << 3) | wt)


def _bytes_field(num: int, v: bytes) -> bytes:
    return _key(num, 2) + put_uvarint(len(v)) + v if v else b""


def _varint_field(num: int, v: int) -> bytes:
    return _key(num, 0) + put_uvarint(v) if v else b""


def _read_varint(buf: bytes, i: int) -> Tuple[int, int]:
    x, s = 0, 0
    while True:
        if i >= len(buf):
            raise ProtoError("unexpected EOF")
        if s >= 64:
            raise ProtoError("integer overflow")
        b = buf[i]
        i += 1
        x |= (b & 0x7F) << s
        if b < 0x80:
            return x & 0xFFFFFFFFFFFFFFFF, i
        s += 7


def _fields(buf: bytes):
    """Yield (field number, wire type, value) with value = int or bytes."""
    i = 0
    while i < len(buf):
        k, i = _read_varint(buf, i)
        num, wt = k >> 3, k & 7
        if num <= 0:
            raise ProtoError(f"illegal tag {num}")
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 1:
            if i + 8 > len(buf):
                raise ProtoError("unexpected EOF")
            v, i = buf[i:i + 8], i + 8
        elif wt == 2:
            n, i = _read_varint(buf, i)
            if n < 0 or i + n > len(buf):
                raise ProtoError("unexpected EOF")
            v, i = buf[i:i + n], i + n
        elif wt == 5:
            if i + 4 > len(buf):
                raise ProtoError("unexpected EOF")
            v, i = buf[i:i + 4], i + 4
        else:
            raise ProtoError(f"illegal wireType {wt}")
        yield num, wt, v


def _want(wt: int, expect: int, name: str) -> None:
    if wt != expect:
        raise ProtoError(f"wrong wireType = {wt} for field {name}")


# ---- Blob / BlobTx -------------------------------------------------------------------------

def marshal_blob(b: Blob) -> bytes:
    return (_bytes_field(1, b.namespace_id) + _bytes_field(2, b.data)
            + _varint_field(3, b.share_version) + _varint_field(4, b.namespace_version))


def unmarshal_blob(buf: bytes) -> Blob:
    b = Blob(b"", b"", 0, 0)
    for num, wt, v in _fields(buf):
        if num == 1:
            _want(wt, 2, "NamespaceId"); b.namespace_id = bytes(v)
        elif num == 2:
            _want(wt, 2, "Data"); b.data = bytes(v)
        elif num == 3:
            _want(wt, 0, "ShareVersion"); b.share_version = v & 0xFFFFFFFF
        elif num == 4:
            _want(wt, 0, "NamespaceVersion"); b.namespace_version = v & 0xFFFFFFFF
    return b


@dataclass
class BlobTx:
    tx: bytes
    blobs: List[Blob] = field(default_factory=list)
    type_id: str = PROTO_BLOB_TX_TYPE_ID


def marshal_blob_tx(tx: bytes, *blobs: Blob) -> bytes:
    """blob.MarshalBlobTx."""
    out = _bytes_field(1, tx)
    for b in blobs:
        m = marshal_blob(b)
        out += _key(2, 2) + put_uvarint(len(m)) + m
    return out + _bytes_field(3, PROTO_BLOB_TX_TYPE_ID.encode())


def _unmarshal_blob_tx(buf: bytes) -> BlobTx:
    t = BlobTx(b"", [], "")
    for num, wt, v in _fields(buf):
        if num == 1:
            _want(wt, 2, "Tx"); t.tx = bytes(v)
        elif num == 2:
            _want(wt, 2, "Blobs"); t.blobs.append(unmarshal_blob(v))
        elif num == 3:
            _want(wt, 2, "TypeId"); t.type_id = bytes(v).decode("utf-8", "replace")
    return t


def unmarshal_blob_tx(buf: bytes) -> Tuple[BlobTx, bool]:
    """blob.UnmarshalBlobTx: (tx, is_blob_tx)."""
    try:
        t = _unmarshal_blob_tx(buf)
    except ProtoError:
        return BlobTx(b"", [], ""), False
    if t.type_id != PROTO_BLOB_TX_TYPE_ID or not t.blobs:
        return t, False
    if any(len(b.namespace_id) != NAMESPACE_ID_SIZE for b in t.blobs):
        return t, False
    return t, True


# ---- IndexWrapper -------------------------------------------------------------------------

@dataclass
class IndexWrapper:
    tx: bytes
    share_indexes: List[int] = field(default_factory=list)
    type_id: str = PROTO_INDEX_WRAPPER_TYPE_ID

    def marshal(self) -> bytes:
        out = _bytes_field(1, self.tx)
        if self.share_indexes:
            packed = b"".join(put_uvarint(x) for x in self.share_indexes)
            out += _key(2, 2) + put_uvarint(len(packed)) + packed
        return out + _bytes_field(3, self.type_id.encode())

    def size(self) -> int:
        return len(self.marshal())


def unmarshal_index_wrapper(buf: bytes) -> Tuple[Optional[IndexWrapper], bool]:
    """types.UnmarshalIndexWrapper: (wrapper, is_index_wrapper)."""
    iw = IndexWrapper(b"", [], "")
    try:
        for num, wt, v in _fields(buf):
            if num == 1:
                _want(wt, 2, "Tx"); iw.tx = bytes(v)
            elif num == 2:
                if wt == 0:
                    iw.share_indexes.append(v & 0xFFFFFFFF)
                elif wt == 2:
                    j = 0
                    while j < len(v):
                        x, j = _read_varint(v, j)
                        iw.share_indexes.append(x & 0xFFFFFFFF)
                else:
                    raise ProtoError(f"wrong wireType = {wt} for field ShareIndexes")
            elif num == 3:
                _want(wt, 2, "TypeId"); iw.type_id = bytes(v).decode("utf-8", "replace")
    except ProtoError:
        return None, False
    if iw.type_id != PROTO_INDEX_WRAPPER_TYPE_ID:
        return None, False
    return iw, True
