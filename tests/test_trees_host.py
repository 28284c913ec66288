"""CPU tests for the host side of the tree / commitment interfaces
(celestia_da.trees) and the oracle restatement they are checked against.

Golden vectors from the reference's own tests:
  TestCreateCommitment        pkg/inclusion/commitment_test.go:64-82
  TestSubTreeWidth            pkg/inclusion/blob_share_commitment_rules_test.go:407-470
  Test_MerkleMountainRangeHeights  pkg/inclusion/commitment_test.go:15-62
"""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import pyref  # noqa: E402
from celestia_da import trees  # noqa: E402

NS1 = trees.namespace_v0(b"\x01" * 10)
GOLDEN_COMMITMENT = bytes([0x3b, 0x9e, 0x78, 0xb6, 0x64, 0x8e, 0xc1, 0xa2, 0x41, 0x92, 0x5b, 0x31, 0xda, 0x2e,
                           0xcb, 0x50, 0xbf, 0xc6, 0xf4, 0xad, 0x55, 0x2d, 0x32, 0x79, 0x92, 0x8c, 0xa1, 0x3e,
                           0xbe, 0xba, 0x8c, 0x2b])

# (shareCount, want) with DefaultSubtreeRootThreshold = 64, DefaultSquareSizeUpperBound = 128
SUBTREE_WIDTH_CASES = [(0, 1), (1, 1), (2, 1), (64, 1), (65, 2), (63, 1), (128, 2), (129, 4), (191, 4),
                       (256, 4), (320, 8), (64 * 128 - 1, 128)]
MMR_CASES = [(11, 4, [4, 4, 2, 1]), (2, 64, [2]), (64, 8, [8] * 8), (19, 8, [8, 8, 2, 1])]


def test_oracle_commitment_golden():
    assert pyref.create_commitment(NS1, b"\xff" * 1536) == GOLDEN_COMMITMENT


@pytest.mark.parametrize("count,want", SUBTREE_WIDTH_CASES)
def test_subtree_width(count, want):
    assert pyref.subtree_width(count) == want
    assert trees.subtree_width(count) == want  # library (dagpu_subtree_width), no GPU


@pytest.mark.parametrize("total,sq,want", MMR_CASES)
def test_mmr_sizes(total, sq, want):
    assert pyref.mmr_sizes(total, sq) == want
    assert trees.merkle_mountain_range_sizes(total, sq) == want


@pytest.mark.parametrize("n", [0, 1, 477, 478, 479, 960, 961, 1536, 5000])
def test_split_blob_matches_oracle(n):
    data = bytes((i * 7 + 3) & 0xFF for i in range(n))
    got = trees.split_blob(NS1, data)
    assert got == pyref.sparse_shares(NS1, data)
    assert all(len(s) == 512 for s in got)
    assert got[0][29] == 1 and all(s[29] == 0 for s in got[1:])
    assert int.from_bytes(got[0][30:34], "big") == n


def test_split_blob_rejects_unsupported_version():
    with pytest.raises(Exception, match="unsupported share version"):
        trees.split_blob(NS1, b"\xff" * 100, share_version=1)


def test_wrapper_push_errors_on_host():
    t = trees.ErasuredNamespacedMerkleTree(2, 0)
    with pytest.raises(Exception, match="too short"):
        t.push(b"\x00" * 28)
    for _ in range(4):
        t.push(b"\x00" * 512)
    with pytest.raises(Exception, match="pushed past predetermined square size"):
        t.push(b"\x00" * 512)
    with pytest.raises(Exception, match="squareSize == 0"):
        trees.ErasuredNamespacedMerkleTree(0, 0)


def test_nmt_push_order_on_host():
    t = trees.NamespacedMerkleTree()
    t.push(b"\x02" * 40)
    with pytest.raises(trees.ErrInvalidPushOrder):
        t.push(b"\x01" * 40)
