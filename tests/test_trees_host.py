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


# ---- DataAvailabilityHeader proto (pkg/da/data_availability_header.go:110-132,
# TestDataAvailabilityHeaderProtoConversion :101-134) -------------------------------

def _proto_class():
    """The reference's .proto message built at run time with the protobuf
    runtime (an independent encoder to check the hand-written wire format)."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    fdp = descriptor_pb2.FileDescriptorProto(name="dah_test.proto", package="celestia.core.v1.da", syntax="proto3")
    m = fdp.message_type.add(name="DataAvailabilityHeader")
    for num, name in ((1, "row_roots"), (2, "column_roots")):
        m.field.add(name=name, number=num, type=descriptor_pb2.FieldDescriptorProto.TYPE_BYTES,
                    label=descriptor_pb2.FieldDescriptorProto.LABEL_REPEATED)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    desc = pool.FindMessageTypeByName("celestia.core.v1.da.DataAvailabilityHeader")
    return message_factory.GetMessageClass(desc)


def test_dah_proto_round_trip():
    import numpy as np
    import oracle
    from celestia_da import da, synth

    mind = da.DataAvailabilityHeader(*_min_roots())
    k = 128
    _, rr, cr, _ = oracle.extend_and_dah(synth.random_blob_square(k, 1), k, nthreads=8, want_eds=False)
    big = da.DataAvailabilityHeader([rr[i].tobytes() for i in range(2 * k)], [cr[i].tobytes() for i in range(2 * k)])
    cls = _proto_class()
    for dah in (mind, big):
        wire = dah.to_proto()
        back = da.data_availability_header_from_proto(wire)
        assert back.row_roots == dah.row_roots and back.column_roots == dah.column_roots
        assert back.hash() == dah.hash()
        ref = cls(row_roots=dah.row_roots, column_roots=dah.column_roots)
        assert ref.SerializeToString() == wire
        assert da.data_availability_header_from_proto(ref.SerializeToString()).hash() == dah.hash()
    with pytest.raises(da.DAError, match="minimum valid"):
        da.data_availability_header_from_proto(b"")


def _min_roots():
    import oracle
    from celestia_da import da
    import numpy as np
    share = np.frombuffer(da.tail_padding_share(), np.uint8).reshape(1, 512)
    _, rr, cr, _ = oracle.extend_and_dah(share, 1)
    return [rr[i].tobytes() for i in range(2)], [cr[i].tobytes() for i in range(2)]
