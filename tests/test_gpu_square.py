"""A square built by the pkg/square mirror goes through the GPU path: extend +
DAH match the oracle, and every blob's commitment read back from the GPU-built
EDS (GetCommitment over the cached row trees) equals CreateCommitment of the
blob — the reference's TestSquareShareCommitments (pkg/square/square_test.go)
with the synthetic txs of test_square_host.py."""
import os
import random
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import oracle  # noqa: E402
import pyref  # noqa: E402
from celestia_da import blobtx as bt  # noqa: E402
from celestia_da import da, inclusion as inc, shares as sh, square as sq, trees  # noqa: E402
from test_square_host import normal_txs, pfb_blob_sizes, random_blob_txs  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = da.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("num_txs,blobs_per,max_size,seed", [(10, 3, 800, 1), (40, 2, 4000, 2), (4, 1, 60000, 3)])
def test_square_share_commitments(ctx, num_txs, blobs_per, max_size, seed):
    rng = random.Random(seed)
    txs = normal_txs(rng, num_txs) + random_blob_txs(rng, num_txs, max_size, blobs_per)
    b = sq.Builder(sq.SQUARE_SIZE_UPPER_BOUND, sq.LATEST_VERSION, *txs)
    square = b.export()
    k = square.size()
    ods = np.frombuffer(b"".join(square.square_bytes()), np.uint8).reshape(k * k, 512)
    eds = da.extend_shares(ods, ctx)
    dah = da.new_data_availability_header(eds)
    if k <= 32:
        _, rr, cr, h = oracle.extend_and_dah(ods, k, want_eds=False)
        assert dah.hash() == h
    cacher = inc.EDSSubTreeRootCacher(k, eds.data, ctx)
    checked = 0
    for pfb_index in range(num_txs):
        wpfb = b.get_wrapped_pfb(pfb_index + num_txs)
        sizes = pfb_blob_sizes(wpfb.tx)
        blob_tx, ok = bt.unmarshal_blob_tx(txs[pfb_index + num_txs])
        assert ok
        for blob_index, share_index in enumerate(wpfb.share_indexes):
            blob = blob_tx.blobs[blob_index]
            got = inc.get_commitment(cacher, dah, share_index, sh.sparse_shares_needed(sizes[blob_index]))
            assert got == trees.create_commitment(blob.namespace(), blob.data, ctx=ctx)
            if len(blob.data) <= 5000:
                assert got == pyref.create_commitment(blob.namespace(), blob.data)
            checked += 1
    assert checked == num_txs * blobs_per
    # the square round-trips through the txs it was built from
    assert sq.deconstruct(square, pfb_blob_sizes) == txs


@pytest.mark.parametrize("n_normal,n_blob,max_size,seed", [(2000, 2000, 3000, 7), (30, 12, 9000, 8), (0, 0, 1, 9)])
def test_native_construct_to_dah(ctx, n_normal, n_blob, max_size, seed):
    """txs -> DataHash with the native constructor (dagpu_square_construct,
    csrc/square.cpp) feeding the GPU path, as app/extend_block.go:14-22 does
    per block: the ODS equals the Python mirror's, the DAH equals the oracle's."""
    import time
    rng = random.Random(seed)
    txs = normal_txs(rng, n_normal, 300) + random_blob_txs(rng, n_blob, max_size)
    t0 = time.perf_counter()
    k, ods = sq.construct_native(txs)
    t_native = time.perf_counter() - t0
    want = sq.construct(txs)
    assert k == want.size()
    assert (ods == np.frombuffer(b"".join(want.square_bytes()), np.uint8)).all()
    dah = da.new_data_availability_header(da.extend_shares(ods.reshape(k * k, 512), ctx))
    _, _, _, h = oracle.extend_and_dah(ods.reshape(k * k, 512), k, nthreads=16, want_eds=False)
    assert dah.hash() == h
    print(f"k={k}: native construct {t_native * 1e3:.2f} ms (incl. Python packing)")
