"""pkg/shares mirror (celestia_da/shares.py) against the reference's own test
tables: counter_test.go, padding_test.go, split_compact_shares_test.go,
share_sequence_test.go, info_byte_test.go, reserved_bytes_test.go, utils_test.go,
powers_of_two_test.go, parse_sparse_shares_test.go.  Host logic, no GPU."""
import random
import struct

import pytest

from celestia_da import shares as sh

F = sh.FIRST_COMPACT_SHARE_CONTENT_SIZE
C = sh.CONTINUATION_COMPACT_SHARE_CONTENT_SIZE
FS = sh.FIRST_SPARSE_SHARE_CONTENT_SIZE
CS = sh.CONTINUATION_SPARSE_SHARE_CONTENT_SIZE
NS1 = sh.new_namespace_v0(b"\x01" * 10)


def test_constants_match_appconsts():
    assert (F, C, FS, CS) == (474, 478, 478, 482)
    assert sh.TX_NAMESPACE == b"\x00" * 28 + b"\x01"
    assert sh.PAY_FOR_BLOB_NAMESPACE == b"\x00" * 28 + b"\x04"
    assert sh.TAIL_PADDING_NAMESPACE == b"\xff" * 28 + b"\xfe"
    assert sh.PARITY_SHARES_NAMESPACE == b"\xff" * 29


def _tx(n, fill=b"a"):
    return fill * n


@pytest.mark.parametrize("txs", [
    [], [_tx(120)], [_tx(F - 2)], [_tx(F - 1)], [_tx(F)], [_tx(F + 1)], [_tx(F), _tx(C - 4)],
    [_tx(100)] * 1000, [_tx(1000)] * 100, [_tx(77)] * 8931,
])
def test_counter_matches_compact_share_splitter(txs):
    """counter_test.go TestCounterMatchesCompactShareSplitter."""
    w = sh.CompactShareSplitter(sh.PAY_FOR_BLOB_NAMESPACE)
    c = sh.CompactShareCounter()
    total = 0
    for tx in txs:
        w.write_tx(tx)
        diff = c.add(len(tx))
        assert w.count() - total == diff
        total = w.count()
        assert total == c.size()
    out = w.export()
    assert len(out) == total == c.size()


def test_counter_revert():
    c = sh.CompactShareCounter()
    assert c.size() == 0
    c.add(F - 2)
    c.add(1)
    assert c.size() == 2
    c.revert()
    assert c.size() == 1


def _pad(b):
    return b.ljust(sh.SHARE_SIZE, b"\x00")


def test_padding_shares():
    """padding_test.go: namespace / reserved / tail padding share bytes."""
    tail = _pad(sh.TAIL_PADDING_NAMESPACE + b"\x01" + b"\x00" * 4)
    assert sh.namespace_padding_share(NS1).to_bytes() == _pad(NS1 + b"\x01" + b"\x00" * 4)
    assert all(s.to_bytes() == _pad(NS1 + b"\x01" + b"\x00" * 4) for s in sh.namespace_padding_shares(NS1, 0, 2))
    assert sh.reserved_padding_shares(2)[1].to_bytes() == _pad(sh.PRIMARY_RESERVED_PADDING_NAMESPACE + b"\x01"
                                                               + b"\x00" * 4)
    assert sh.tail_padding_share().to_bytes() == tail
    assert [s.to_bytes() for s in sh.tail_padding_shares(2)] == [tail, tail]
    with pytest.raises(sh.ShareError):
        sh.namespace_padding_shares(NS1, 0, -1)


def _generate_tx(num_shares):
    if num_shares == 0:
        return b""
    if num_shares == 1:
        return b"\x01" * sh.raw_tx_size(F)
    return b"\x02" * sh.raw_tx_size(F + (num_shares - 1) * C)


@pytest.mark.parametrize("txs,want", [
    ([], 0), ([b"\x00"], 1), ([b"\x01" * 100], 1), ([b"\x01" * sh.raw_tx_size(F + 1)], 2),
    ([_generate_tx(1)], 1), ([_generate_tx(2)], 2), ([_generate_tx(20)], 20),
])
def test_compact_splitter_count(txs, want):
    """split_compact_shares_test.go TestCount."""
    css = sh.CompactShareSplitter(sh.TX_NAMESPACE)
    for tx in txs:
        css.write_tx(tx)
    assert css.count() == want


def test_compact_splitter_export_write_bytes():
    """split_compact_shares_test.go TestExport_write: exact share bytes."""
    one = _pad(sh.TX_NAMESPACE + bytes([1, 0, 0, 0, 1, 0, 0, 0, 0x26, 0xF]))
    first = (sh.TX_NAMESPACE + bytes([1, 0, 0, 2, 0, 0, 0, 0, 0x26])).ljust(sh.SHARE_SIZE, b"\x0f")
    cont = _pad(sh.TX_NAMESPACE + bytes([0, 0, 0, 0, 0]) + b"\x0f" * (29 + 1 + 4 + 4))
    for writes, want in [([], []), ([b"\x0f"], [one]), ([b"\x0f" * 512], [first, cont])]:
        css = sh.CompactShareSplitter(sh.TX_NAMESPACE)
        for w in writes:
            css._write(w)
        got = [s.to_bytes() for s in css.export()]
        assert got == want
        assert [s.to_bytes() for s in css.export()] == got  # idempotent
        assert len(got) == css.count()


def test_compact_splitter_share_ranges():
    """split_compact_shares_test.go TestExport (share ranges per tx)."""
    one, two, three = b"\x01", b"\x02" * 600, b"\x03" * 1000
    exactly_one = b"\x04" * sh.raw_tx_size(F)
    exactly_two = b"\x05" * sh.raw_tx_size(F + C)
    cases = [
        ([], {}, 0),
        ([one], {one: (0, 1)}, 0),
        ([two], {two: (0, 2)}, 0),
        ([three], {three: (0, 3)}, 0),
        ([one, two, three], {one: (0, 1), two: (0, 2), three: (1, 4)}, 0),
        ([exactly_one], {exactly_one: (0, 1)}, 0),
        ([exactly_two], {exactly_two: (0, 2)}, 0),
        ([exactly_two, exactly_one], {exactly_two: (0, 2), exactly_one: (2, 3)}, 0),
        ([exactly_one, exactly_two], {exactly_one: (0, 1), exactly_two: (1, 3)}, 0),
        ([exactly_one, exactly_two], {exactly_one: (10, 11), exactly_two: (11, 13)}, 10),
    ]
    for txs, want, off in cases:
        css = sh.CompactShareSplitter(sh.TX_NAMESPACE)
        for tx in txs:
            css.write_tx(tx)
        got = {k: (v.start, v.end) for k, v in css.share_ranges_with_offset(off).items()}
        assert got == want


def test_write_after_export():
    """split_compact_shares_test.go TestWriteAfterExport (share counts)."""
    a = b"\x0f" * sh.raw_tx_size(F)
    b = b"\x0f" * sh.raw_tx_size(C * 2)
    c = b"\x0f" * sh.raw_tx_size(C)
    css = sh.CompactShareSplitter(sh.TX_NAMESPACE)
    counts = [len(css.export())]
    for tx in (a, b, c, b"\x0f"):
        css.write_tx(tx)
        counts.append(len(css.export()))
    counts.append(len(css.export()))
    assert counts == [0, 1, 3, 4, 5, 5]


def test_compact_parse_roundtrip():
    """ParseTxs(SplitTxs(txs)) == txs over random tx sets; one sequence per namespace."""
    rng = random.Random(7)
    for _ in range(20):
        txs = [rng.randbytes(rng.randrange(1, 2000)) for _ in range(rng.randrange(1, 30))]
        css = sh.CompactShareSplitter(sh.TX_NAMESPACE)
        for tx in txs:
            css.write_tx(tx)
        out = css.export()
        assert len(out) == sh.compact_shares_needed(out[0].sequence_len())
        assert sh.parse_txs(out) == txs
        seqs = sh.parse_shares(out, ignore_padding=False)
        assert len(seqs) == 1 and seqs[0].namespace == sh.TX_NAMESPACE


@pytest.mark.parametrize("n,want", [(0, 0), (1, 1), (2, 1), (F, 1), (F + 1, 2), (F + C, 2), (F + 100 * C, 101)])
def test_compact_shares_needed(n, want):
    assert sh.compact_shares_needed(n) == want


@pytest.mark.parametrize("n,want", [(0, 0), (1, 1), (2, 1), (FS, 1), (FS + 1, 2), (FS + CS, 2), (FS + C * 2, 3),
                                    (FS + C * 99, 100), (1000, 3), (10000, 21), (100000, 208)])
def test_sparse_shares_needed(n, want):
    assert sh.sparse_shares_needed(n) == want


def test_info_byte():
    for v in (0, 1, 2, 127):
        for start in (True, False):
            ib = sh.new_info_byte(v, start)
            assert ib >> 1 == v and (ib % 2 == 1) == start
    for v in (128, 255):
        with pytest.raises(sh.ShareError):
            sh.new_info_byte(v, False)
    for b, v, start in [(0b0, 0, False), (0b1, 0, True), (0b10, 1, False), (0b11, 1, True), (0b101, 2, True),
                        (0xFF, 127, True)]:
        ib = sh.parse_info_byte(b)
        assert (ib >> 1, ib % 2 == 1) == (v, start)


def test_reserved_bytes():
    """reserved_bytes_test.go."""
    for raw, want in [(b"\x00\x00\x00\x00", 0), (b"\x00\x00\x00\x02", 2), (b"\x00\x00\x00\x80", 128),
                      (b"\x00\x00\x01\x00", 256), (b"\x00\x00\x01\xff", 511)]:
        assert sh.parse_reserved_bytes(raw) == want
        assert sh.new_reserved_bytes(want) == raw
    for bad in (b"", b"\x01", b"\x03\x03\x03", b"\x00" * 5, b"\x00\x00\x03\xe8"):
        with pytest.raises(sh.ShareError):
            sh.parse_reserved_bytes(bad)
    for bad in (512, 1000):
        with pytest.raises(sh.ShareError):
            sh.new_reserved_bytes(bad)


def test_zero_pad_and_delimiter():
    assert sh.zero_pad_if_necessary(b"\x01\x02\x03", 6) == (b"\x01\x02\x03\x00\x00\x00", 3)
    assert sh.zero_pad_if_necessary(b"\x01\x02\x03", 3) == (b"\x01\x02\x03", 0)
    assert sh.zero_pad_if_necessary(b"\x01\x02\x03", 2) == (b"\x01\x02\x03", 0)
    rng = random.Random(1)
    for i in range(100):
        tx = rng.randbytes(i)
        rest, n = sh.parse_delimiter(sh.marshal_delimited_tx(tx))
        assert n == i and rest == tx


def test_powers_of_two():
    assert [sh.round_up_power_of_two(v) for v in (-1, 0, 1, 2, 3, 4, 5, 8, 9)] == [1, 1, 1, 2, 4, 4, 8, 8, 16]
    assert [sh.round_down_power_of_two(v) for v in (1, 2, 3, 4, 5, 8, 9)] == [1, 2, 2, 4, 4, 8, 8]
    with pytest.raises(sh.ShareError):
        sh.round_down_power_of_two(0)
    assert [sh.round_up_power_of_two_strict(v) for v in (1, 2, 3, 4, 5, 8)] == [2, 4, 4, 8, 8, 16]
    assert [sh.is_power_of_two(v) for v in (0, 1, 2, 3, 4, 6, 64)] == [False, True, True, False, True, False, True]


def test_sparse_split_and_parse():
    """SparseShareSplitter + parseSparseShares (incl. namespace padding), and the
    first-share layout used by commitments."""
    rng = random.Random(3)
    blobs = [sh.Blob.new(sh.new_namespace_v0(bytes([i + 1]) * 10), rng.randbytes(n))
             for i, n in enumerate([1, FS, FS + 1, 5000, 1234])]
    w = sh.SparseShareSplitter()
    for i, b in enumerate(blobs):
        w.write(b)
        if i == 1:
            w.write_namespace_padding_shares(2)
    out = w.export()
    assert len(out) == sum(sh.sparse_shares_needed(len(b.data)) for b in blobs) + 2
    parsed = sh.parse_blobs(out)
    assert [(p.namespace(), p.data) for p in parsed] == [(b.namespace(), b.data) for b in blobs]
    first = out[0].to_bytes()
    assert first[:29] == blobs[0].namespace() and first[29] == 1 and struct.unpack(">I", first[30:34])[0] == 1
    with pytest.raises(sh.ShareError):
        sh.SparseShareSplitter().write_namespace_padding_shares(1)
    with pytest.raises(sh.ShareError):
        sh.SparseShareSplitter().write(sh.Blob(b"\x00" * 28, b""))


def test_share_accessors_and_ranges():
    txs = [b"\x07" * 700, b"\x08" * 30]
    css = sh.CompactShareSplitter(sh.TX_NAMESPACE)
    for t in txs:
        css.write_tx(t)
    tx_shares = css.export()
    blob_shares = sh.split_blobs(sh.Blob.new(NS1, b"\x09" * 600))
    square = tx_shares + blob_shares + sh.tail_padding_shares(3)
    assert tx_shares[0].is_compact_share() and not blob_shares[0].is_compact_share()
    assert tx_shares[0].is_sequence_start() and not tx_shares[1].is_sequence_start()
    assert tx_shares[1].sequence_len() == 0
    assert sh.tail_padding_shares(1)[0].is_padding() and not blob_shares[0].is_padding()
    r = sh.get_share_range_for_namespace(square, NS1)
    assert (r.start, r.end) == (len(tx_shares), len(tx_shares) + len(blob_shares))
    assert sh.get_share_range_for_namespace(square, sh.PAY_FOR_BLOB_NAMESPACE).is_empty()
    seqs = sh.parse_shares(square, ignore_padding=True)
    assert [q.namespace for q in seqs] == [sh.TX_NAMESPACE, NS1]
    assert seqs[1].raw_data() == b"\x09" * 600
    with pytest.raises(sh.ShareError):
        sh.Share(b"\x00" * 511)
    with pytest.raises(sh.ShareError):
        sh.validate_namespace(b"\x01" + b"\x00" * 28)  # unsupported version
