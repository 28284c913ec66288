"""GPU parity of the EDS-side commitment path (celestia_da.inclusion):
row-tree nodes exported by dagpu_row_nodes_device, getSubTreeRoot walks and
GetCommitment (pkg/inclusion/get_commit.go:12-30), checked against the
oracle's NMT restatement and against CreateCommitment of the same blobs
(the reference's TestEDSSubRootCacher / TestGetCommit pattern)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import oracle  # noqa: E402
import pyref  # noqa: E402
from celestia_da import da, inclusion as inc, trees  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = da.Context(0)
    yield c
    c.close()


def _square_with_blobs(k, blob_lens, seed, threshold=64):
    """Row-major ODS: a few low-namespace shares, then blobs (sorted namespaces)
    at NextShareIndex positions with namespace padding, tail padding last."""
    rng = np.random.default_rng(seed)
    nss = sorted(trees.namespace_v0(bytes(rng.integers(1, 256, 10, dtype=np.uint8))) for _ in blob_lens)
    shares = [b"\x00" * 28 + b"\x01" + bytes(rng.integers(0, 256, 483, dtype=np.uint8)) for _ in range(3)]
    placed = []
    prev_ns = shares[-1][:29]
    for ns, n in zip(nss, blob_lens):
        data = bytes(rng.integers(0, 256, max(1, n * 482 - 100), dtype=np.uint8))
        bs = trees.split_blob(ns, data)
        assert len(bs) == n
        start = inc.next_share_index(len(shares), n, threshold)
        while len(shares) < start:
            shares.append(prev_ns + b"\x00" * 483)
        placed.append((start, ns, data))
        shares.extend(bs)
        prev_ns = ns
    assert len(shares) <= k * k
    while len(shares) < k * k:
        shares.append(da.tail_padding_share())
    return np.frombuffer(b"".join(shares), np.uint8).reshape(k * k, 512), placed


@pytest.mark.parametrize("k,blob_lens", [(4, [1, 2, 3]), (8, [5, 11, 1]), (32, [64, 65, 100, 3]),
                                         (64, [300, 1, 129, 700])])
def test_get_commitment_matches_create_commitment(ctx, k, blob_lens):
    ods, placed = _square_with_blobs(k, blob_lens, seed=k)
    eds = da.extend_shares(ods, ctx)
    dah = da.new_data_availability_header(eds)
    cacher = inc.EDSSubTreeRootCacher(k, eds.data, ctx)
    for start, ns, data in placed:
        n = len(trees.split_blob(ns, data))
        got = inc.get_commitment(cacher, dah, start, n)
        assert got == trees.create_commitment(ns, data, ctx=ctx)
        assert got == pyref.create_commitment(ns, data)


def test_sub_tree_roots_match_oracle(ctx):
    k = 8
    ods, _ = _square_with_blobs(k, [4, 9], seed=3)
    eds, rr, _, _ = oracle.extend_and_dah(ods, k)
    dah = da.DataAvailabilityHeader([rr[i].tobytes() for i in range(2 * k)],
                                    [bytes(90)] * (2 * k))
    cacher = inc.EDSSubTreeRootCacher(k, eds, ctx)
    w = 2 * k
    rng = np.random.default_rng(1)
    for _ in range(40):
        row = int(rng.integers(0, w))
        depth = int(rng.integers(0, 5))
        pos = int(rng.integers(0, 1 << depth))
        width = w >> depth
        leaves = [pyref.leaf(eds[row, c, :29].tobytes() if (row < k and c < k) else b"\xff" * 29,
                             eds[row, c].tobytes()) for c in range(pos * width, (pos + 1) * width)]
        path = inc.gen_sub_tree_root_path(depth, pos)
        assert cacher.get_sub_tree_root(dah, row, path) == pyref.nmt_root(leaves)
    assert cacher.get_sub_tree_root(dah, 3, []) == rr[3].tobytes()


def test_cacher_errors(ctx):
    k = 4
    ods, _ = _square_with_blobs(k, [2], seed=9)
    eds = da.extend_shares(ods, ctx)
    dah = da.new_data_availability_header(eds)
    cacher = inc.EDSSubTreeRootCacher(k, eds.data, ctx)
    with pytest.raises(da.DAError, match="row exceeds range"):
        cacher.get_sub_tree_root(dah, 8, [inc.WALK_LEFT])
    bad = da.DataAvailabilityHeader([bytes(90)] * 8, dah.column_roots)
    with pytest.raises(da.DAError, match="did not find sub tree root"):
        cacher.get_sub_tree_root(bad, 0, [inc.WALK_LEFT])
    small = da.DataAvailabilityHeader(dah.row_roots[:4], dah.column_roots[:4])
    with pytest.raises(da.DAError, match="unexpected number of row roots"):
        cacher.get_sub_tree_root(small, 0, [])
    with pytest.raises(da.DAError, match="doesn't fit"):
        inc.get_commitment(cacher, dah, 15, 2)
