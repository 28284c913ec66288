"""Native square construction (csrc/square.cpp: dagpu_square_construct /
dagpu_square_build) against the Python mirror of pkg/square
(celestia_da/square.py), which tests/test_square_host.py pins to the
reference's square_test.go / builder_test.go tables: the same ODS bytes for
every table case and for random blocks (normal txs, blob txs with 1-3 blobs,
namespaces repeating and out of order, sizes across share boundaries), the
same errors with the same messages, and the time of a full 128 x 128 square.
Host only, no GPU.
"""
import random
import time

import numpy as np
import pytest

from celestia_da import blobtx as bt
from celestia_da import shares as sh
from celestia_da import square as sq

from test_square_host import (BLOB_POSITION_CASES, NS1, blob_txs, normal_txs,  # noqa: F401
                              random_blob_txs, pfb_tx)


def _python_ods(txs, max_square_size=128):
    s = sq.construct(txs, max_square_size=max_square_size)
    return s.size(), np.frombuffer(b"".join(s.square_bytes()), np.uint8)


def _same(txs, max_square_size=128):
    k, ods = sq.construct_native(txs, max_square_size)
    pk, pods = _python_ods(txs, max_square_size)
    assert k == pk and ods.shape == pods.shape and (ods == pods).all()
    return k


def test_empty_and_tiny():
    assert _same([]) == 1
    assert _same([b"\x01"]) == 1
    assert _same([b""]) == 1
    assert _same([b"\x02" * 600, b"\x03" * 1000]) == 2


@pytest.mark.parametrize("n", [1, 473, 474, 475, 477, 478, 479, 952, 953, 956, 957, 5000])
def test_compact_boundaries(n):
    """Tx lengths around the first/continuation compact share capacities."""
    rng = random.Random(n)
    _same([rng.randbytes(n)])
    _same([rng.randbytes(n), rng.randbytes(3), rng.randbytes(n)])


@pytest.mark.parametrize("case", range(len(BLOB_POSITION_CASES)))
def test_blob_position_cases(case):
    size, nss, sizes, _ = BLOB_POSITION_CASES[case]
    txs = blob_txs(nss, sizes)
    try:
        want = _python_ods(txs, size)
    except sh.ShareError as e:
        with pytest.raises(sh.ShareError, match=str(e)):
            sq.construct_native(txs, size)
        return
    k, ods = sq.construct_native(txs, size)
    assert k == want[0] and (ods == want[1]).all()


@pytest.mark.parametrize("seed", range(12))
def test_random_blocks(seed):
    rng = random.Random(seed)
    n_normal = rng.randrange(0, 200)
    txs = [rng.randbytes(rng.choice([1, 50, 300, 477, 1000, 3000])) for _ in range(n_normal)]
    nss = [sh.new_namespace_v0(bytes([rng.randrange(1, 6)]) * 10) for _ in range(8)]
    for _ in range(rng.randrange(0, 80)):
        blobs = [sh.Blob.new(rng.choice(nss), rng.randbytes(rng.choice([1, 477, 478, 479, 960, 2000, 20000])))
                 for _ in range(rng.randrange(1, 4))]
        txs.append(bt.marshal_blob_tx(pfb_tx([len(b.data) for b in blobs]), *blobs))
    try:
        want = _python_ods(txs)
    except sh.ShareError as e:
        with pytest.raises(sh.ShareError, match=str(e)):
            sq.construct_native(txs)
        return
    k, ods = sq.construct_native(txs)
    assert k == want[0] and (ods == want[1]).all()


def test_construct_errors_match():
    """square_test.go TestSquareConstruction rejections, same messages."""
    rng = random.Random(1)
    send = normal_txs(rng, 250)
    pfbs = random_blob_txs(rng, 100, 1024)
    for txs, m in ((send[:5] + pfbs + send[5:], 128), (send, 2), (pfbs, 2)):
        with pytest.raises(sh.ShareError) as want:
            sq.construct(txs, max_square_size=m)
        with pytest.raises(sh.ShareError) as got:
            sq.construct_native(txs, m)
        assert str(got.value) == str(want.value)
    for bad in (0, 13):
        with pytest.raises(sh.ShareError, match="max square size must be"):
            sq.construct_native([b"x"], bad)


def test_invalid_blobs():
    """Blob validation inside the splitter: empty data and unsupported share
    versions fail as the mirror fails; a non-blob proto stays a normal tx."""
    for blob in (sh.Blob(NS1[1:], b""), sh.Blob(NS1[1:], b"d", share_version=1)):
        tx = bt.marshal_blob_tx(b"pfb", blob)
        with pytest.raises(sh.ShareError) as want:
            sq.construct([tx])
        with pytest.raises(sh.ShareError) as got:
            sq.construct_native([tx])
        assert str(got.value) == str(want.value)
    # 27-byte namespace ID: not a blob tx -> a normal tx
    odd = bt.marshal_blob_tx(b"x", sh.Blob(b"\x00" * 27, b"d"))
    _same([odd])


def test_build_matches():
    rng = random.Random(13)
    normal = normal_txs(rng, 5)
    pfbs = random_blob_txs(rng, 5, 3000)
    txs = pfbs[:2] + normal + pfbs[2:]
    want_sq, want_kept = sq.build(txs, max_square_size=4)
    k, ods, kept = sq.build_native(txs, max_square_size=4)
    assert kept == want_kept and k == want_sq.size()
    assert (ods == np.frombuffer(b"".join(want_sq.square_bytes()), np.uint8)).all()


def test_full_square_time():
    """A full 128 x 128 square (2,000 normal txs + 2,000 blob txs): the C++
    path takes milliseconds where the mirror takes ~0.2 s."""
    rng = random.Random(99)
    txs = [rng.randbytes(300) for _ in range(2000)]
    nss = sorted(sh.new_namespace_v0(rng.randbytes(10)) for _ in range(64))
    for i in range(2000):
        data = rng.randbytes(rng.randrange(1500, 3000))
        txs.append(bt.marshal_blob_tx(pfb_tx([len(data)]), sh.Blob.new(nss[i % 64], data)))
    k = _same(txs)
    assert k == 128
    best = min(_timed(txs) for _ in range(5))
    print(f"native full-square construction: {best * 1e3:.2f} ms")
    assert best < 0.05


def _timed(txs):
    t0 = time.perf_counter()
    sq.construct_native(txs)
    return time.perf_counter() - t0


def test_argument_errors_carry_this_calls_message():
    # a stale message from an earlier failure must not leak into the next
    # argument error of a context-free call
    import ctypes

    import numpy as np
    from celestia_da import _abi
    L = _abi.lib()
    with pytest.raises(sh.ShareError if hasattr(sh, "ShareError") else Exception):
        sq.construct_native([b"x" * 400] * 20, max_square_size=1)  # an earlier failure with a message
    assert L.dagpu_last_error(None).decode().startswith("not enough space")
    out = np.empty(512, np.uint8)
    k = ctypes.c_uint32(0)
    rc = L.dagpu_square_construct(None, None, None, 0, 64, 0, _abi.addr(out), 512, ctypes.addressof(k))
    assert rc == _abi.ERR_ARG
    assert L.dagpu_last_error(None).decode() == "subtree_root_threshold must be > 0"
    lens = np.array([4], np.uint64)
    rc = L.dagpu_square_build(None, None, _abi.addr(lens), 1, 64, 64, _abi.addr(out), 512, ctypes.addressof(k), None)
    assert rc == _abi.ERR_ARG
    assert L.dagpu_last_error(None).decode() == "txs and tx_lens are required when ntx > 0"
