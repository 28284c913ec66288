"""pkg/square mirror (celestia_da/square.py, blobtx.py) against the reference's
test tables: square_test.go (TxShareRange, Size, Construct/Deconstruct parity,
BlobShareRange) and builder_test.go (rejections, FindTxShareRange, blob
positions).  Host logic, no GPU.

Synthetic txs: the reference signs real cosmos-sdk txs (a MsgSend, a
MsgPayForBlobs), which cannot be produced here.  Normal txs are random bytes;
a PFB tx is `b"PFB" || n || varint(blob sizes)` zero-padded to
PFB_BASE + PFB_PER_BLOB * n bytes.  Only the length of a PFB tx influences the
layout, and (PFB_BASE, PFB_PER_BLOB) = (230, 100) lies inside the range for
which every expectation of TestSquareBlobPostions and
TestBuilderRejectsBlobTransactions holds (a 1-blob PFB of 330 B; the scan over
base 150-490 x per-blob 20-150 found 31 such pairs), so those tables pin the
layout rules (NextShareIndex, padding, namespace order, PFB share accounting).
"""
import random

import pytest

from celestia_da import blobtx as bt
from celestia_da import shares as sh
from celestia_da import square as sq

PFB_BASE, PFB_PER_BLOB = 230, 100
NS1 = sh.new_namespace_v0(b"\x01" * 10)
NS2 = sh.new_namespace_v0(b"\x02" * 10)
NS3 = sh.new_namespace_v0(b"\x03" * 10)
A = sh.available_bytes_from_sparse_shares


def pfb_tx(sizes):
    body = b"PFB" + bytes([len(sizes)]) + b"".join(sh.put_uvarint(s) for s in sizes)
    return body.ljust(PFB_BASE + PFB_PER_BLOB * len(sizes), b"\x00")


def pfb_blob_sizes(tx):
    """The TxDecoder role of Deconstruct: blob sizes of a synthetic PFB tx."""
    assert tx[:3] == b"PFB"
    n, i, out = tx[3], 4, []
    for _ in range(n):
        v, used = sh.read_uvarint(tx[i:i + 10])
        out.append(v)
        i += used
    return out


def blob_txs(namespaces, sizes, rng=None):
    rng = rng or random.Random(0)
    out, k = [], 0
    for group in sizes:
        blobs = []
        for s in group:
            blobs.append(sh.Blob.new(namespaces[k], rng.randbytes(s)))
            k += 1
        out.append(bt.marshal_blob_tx(pfb_tx(group), *blobs))
    return out


def normal_txs(rng, n, size=200):
    return [rng.randbytes(size) for _ in range(n)]


def random_blob_txs(rng, n, max_size, blobs_per=1):
    out = []
    for _ in range(n):
        blobs = [sh.Blob.new(sh.new_namespace_v0(rng.randbytes(10)), rng.randbytes(rng.randrange(1, max_size + 1)))
                 for _ in range(blobs_per)]
        out.append(bt.marshal_blob_tx(pfb_tx([len(b.data) for b in blobs]), *blobs))
    return out


def test_blob_tx_proto_roundtrip():
    b = sh.Blob.new(NS1, b"hello", 0)
    raw = bt.marshal_blob_tx(b"tx-bytes", b)
    t, ok = bt.unmarshal_blob_tx(raw)
    assert ok and t.tx == b"tx-bytes" and t.blobs[0] == b and t.type_id == "BLOB"
    assert bt.unmarshal_blob_tx(b"\x0a\x05hello")[1] is False          # no type id / blobs
    assert bt.unmarshal_blob_tx(b"\x0a\x09hello")[1] is False          # truncated
    assert bt.unmarshal_blob_tx(bt.marshal_blob_tx(b"x", sh.Blob(b"\x00" * 27, b"d")))[1] is False
    iw = bt.IndexWrapper(b"abc", [1, 300, 16384])
    back, ok = bt.unmarshal_index_wrapper(iw.marshal())
    assert ok and back == iw and iw.size() == len(iw.marshal())
    assert bt.unmarshal_index_wrapper(b"random tx bytes")[1] is False


@pytest.mark.parametrize("txs,index,want", [
    ([b"\x01"], 0, (0, 1)),
    ([b"\x02" * 600], 0, (0, 2)),
    ([b"\x03" * 1000], 0, (0, 3)),
    ([b"\x01", b"\x02" * 600, b"\x03" * 1000], 2, (1, 4)),
])
def test_tx_share_range(txs, index, want):
    """square_test.go TestSquareTxShareRange."""
    r = sq.tx_share_range(txs, index)
    assert (r.start, r.end) == want


def test_tx_share_range_invalid_index():
    with pytest.raises(sh.ShareError):
        sq.tx_share_range([b"\x01", b"\x02" * 600, b"\x03" * 1000], 3)


@pytest.mark.parametrize("n,want", [(0, 1), (1, 1), (64, 8), (100, 16), (1000, 32), (128 * 128, 128),
                                    (128 * 128 + 1, 256)])
def test_size(n, want):
    """square_test.go TestSize."""
    assert sq.size(n) == want and sh.is_power_of_two(want)


def test_builder_invalid_constructor():
    for bad in (-4, 0, 13):
        with pytest.raises(sh.ShareError):
            sq.Builder(bad)


def test_builder_rejects_transactions():
    """builder_test.go TestBuilderRejectsTransactions (2x2 square)."""
    def new_tx(n):
        return b"\x00" * sh.raw_tx_size(n)
    b = sq.Builder(2)
    assert not b.append_tx(new_tx(sh.available_bytes_from_compact_shares(4) + 1))
    assert b.append_tx(new_tx(sh.available_bytes_from_compact_shares(4)))
    assert not b.append_tx(new_tx(1))


@pytest.mark.parametrize("sizes,added", [
    ([A(3) + 1], False), ([A(3)], True), ([A(2) + 1, A(1)], False), ([A(1), A(1)], True),
    ([A(1), A(1), A(1)], False),  # three blobs make the PFB two shares
])
def test_builder_rejects_blob_transactions(sizes, added):
    b = sq.Builder(2)
    t, ok = bt.unmarshal_blob_tx(blob_txs([NS1] * len(sizes), [sizes])[0])
    assert ok
    assert b.append_blob_tx(t) == added


BLOB_POSITION_CASES = [
    (4, [NS1], [[1]], [[1]]),
    (4, [NS1, NS1], [[100]] * 2, [[2], [3]]),
    (4, [NS1] * 9, [[100]] * 9, [[7], [8], [9], [10], [11], [12], [13], [14], [15]]),
    (4, [NS1] * 3, [[10000], [10000], [1000000]], []),
    (64, [NS1] * 3, [[1000], [10000], [10000]], [[3], [6], [27]]),
    (32, [NS2, NS1, NS1], [[100], [100], [100]], [[5], [3], [4]]),
    (16, [NS1, NS2, NS1], [[100], [900], [900]], [[3], [6], [4]]),
    (4, [NS1, NS3, NS3, NS2], [[100], [1000, 1000], [420]], [[3], [5, 8], [4]]),
    (1, [NS1, NS2, NS3], [[1000]] * 3, []),
    (4, [NS3, NS2, NS1], [[2000], [2000], [5000]], [[7], [2]]),
    (4, [NS3, NS3, NS2, NS1], [[1800, 1000], [22000], [1800]], [[6, 10], [2]]),
    (4, [NS1, NS3, NS3, NS1, NS2, NS2], [[100], [1400, 900, 200, 200], [420]], [[3], [7, 10, 4, 5], [6]]),
    (4, [NS1, NS3, NS3, NS1, NS2, NS2], [[100], [900, 1400, 200, 200], [420]], [[3], [7, 9, 4, 5], [6]]),
    (16, [NS1, NS1], [[100], [A(64)]], [[2], [3]]),
    (16, [NS1, NS1], [[100], [A(64) + 1]], [[2], [4]]),
]


@pytest.mark.parametrize("case", range(len(BLOB_POSITION_CASES)))
def test_square_blob_positions(case):
    """builder_test.go TestSquareBlobPostions: share indexes in the wrapped PFBs."""
    size, nss, sizes, want = BLOB_POSITION_CASES[case]
    b = sq.Builder(size)
    for tx in blob_txs(nss, sizes):
        t, ok = bt.unmarshal_blob_tx(tx)
        assert ok
        b.append_blob_tx(t)
    square = b.export()
    got = []
    for tx in sh.parse_txs(square):
        iw, ok = bt.unmarshal_index_wrapper(tx)
        assert ok
        got.append(iw.share_indexes)
    assert got == want


def test_construct_errors():
    """square_test.go TestSquareConstruction."""
    rng = random.Random(1)
    send = normal_txs(rng, 250)
    pfbs = random_blob_txs(rng, 100, 1024)
    with pytest.raises(sh.ShareError):
        sq.construct(send[:5] + pfbs + send[5:])
    with pytest.raises(sh.ShareError):
        sq.construct(send, max_square_size=2)
    with pytest.raises(sh.ShareError):
        sq.construct(pfbs, max_square_size=2)


@pytest.mark.parametrize("num_txs", [2, 128, 1024])
def test_construct_deconstruct_parity(num_txs):
    """square_test.go TestSquareDeconstruct/ConstructDeconstructParity."""
    rng = random.Random(num_txs)
    txs = normal_txs(rng, num_txs // 2) + random_blob_txs(rng, num_txs // 2, 800)
    square = sq.construct(txs)
    assert sq.deconstruct(square, pfb_blob_sizes) == txs


def test_deconstruct_no_pfbs_pfbs_only_empty():
    rng = random.Random(5)
    txs = normal_txs(rng, 10)
    assert sq.deconstruct(sq.construct(txs), pfb_blob_sizes) == txs
    txs = random_blob_txs(rng, 100, 1024)
    assert sq.deconstruct(sq.construct(txs), pfb_blob_sizes) == txs
    assert sq.deconstruct(sq.empty_square(), pfb_blob_sizes) == []
    assert sq.Builder(4).export().equals(sq.empty_square())


def test_blob_share_range():
    """square_test.go TestSquareBlobShareRange: the range holds the blob's data."""
    rng = random.Random(11)
    txs = random_blob_txs(rng, 10, 1000, blobs_per=3)
    b = sq.Builder(sq.SQUARE_SIZE_UPPER_BOUND, sq.LATEST_VERSION, *txs)
    square = b.export()
    for pfb_idx, tx in enumerate(txs):
        t, _ = bt.unmarshal_blob_tx(tx)
        for blob_idx, blob in enumerate(t.blobs):
            r = sq.blob_share_range(txs, pfb_idx, blob_idx)
            raw = b"".join(s.raw_data() for s in square[r.start:r.end])
            assert blob.data in raw
    for args in ((-1, 0), (0, -1), (10, 0), (0, 10)):
        with pytest.raises(sh.ShareError):
            sq.blob_share_range(txs, *args)


def test_find_tx_share_range():
    """builder_test.go TestBuilderFindTxShareRange."""
    rng = random.Random(12)
    txs = [rng.randbytes(900) for _ in range(5)] + random_blob_txs(rng, 5, 1000)
    b = sq.Builder(sq.SQUARE_SIZE_UPPER_BOUND, sq.LATEST_VERSION, *txs)
    square = b.export()
    size = square.size() ** 2
    last_end = 0
    for idx, tx in enumerate(txs):
        t, is_blob = bt.unmarshal_blob_tx(tx)
        if is_blob:
            tx = t.tx
        r = b.find_tx_share_range(idx)
        if idx == 5:
            assert r.start > last_end - 1
        else:
            assert r.start >= last_end - 1
        assert r.end <= size
        raw = b"".join(s.raw_data() for s in square[r.start:r.end + 1])
        assert tx in raw
        last_end = r.end


def test_build_drops_what_does_not_fit_and_orders_normal_first():
    rng = random.Random(13)
    normal = normal_txs(rng, 5)
    pfbs = random_blob_txs(rng, 5, 3000)
    square, kept = sq.build(pfbs[:2] + normal + pfbs[2:], max_square_size=4)
    assert kept[:5] == normal and all(t in pfbs for t in kept[5:]) and len(kept) < 10
    assert sq.deconstruct(square, pfb_blob_sizes) == kept


def test_split_blob_matches_sparse_splitter():
    from celestia_da.trees import split_blob
    rng = random.Random(2)
    for n in (1, 478, 479, 5000):
        data = rng.randbytes(n)
        assert split_blob(NS2, data) == sh.to_bytes(sh.split_blobs(sh.Blob.new(NS2, data)))
