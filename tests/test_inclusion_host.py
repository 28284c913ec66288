"""CPU tests of the path arithmetic behind GetCommitment / EDSSubTreeRootCacher
(celestia_da.inclusion), against the reference's own test tables:
  Test_calculateSubTreeRootCoordinates  pkg/inclusion/paths_test.go:12-317
  Test_calculateCommitPaths             pkg/inclusion/paths_test.go:341-440
  TestNextShareIndex                    pkg/inclusion/blob_share_commitment_rules_test.go:148-295
"""
import pytest

from celestia_da import inclusion as inc

L, R = inc.WALK_LEFT, inc.WALK_RIGHT

# (start, end, maxDepth, minDepth, expected [(depth, position)])
COORD_CASES = [
    (0, 4, 3, 1, [(1, 0)]), (4, 8, 3, 1, [(1, 1)]), (3, 5, 3, 3, [(3, 3), (3, 4)]), (3, 4, 3, 3, [(3, 3)]),
    (3, 6, 3, 2, [(3, 3), (2, 2)]), (1, 7, 3, 2, [(3, 1), (2, 1), (2, 2), (3, 6)]),
    (1, 7, 3, 3, [(3, 1), (3, 2), (3, 3), (3, 4), (3, 5), (3, 6)]), (0, 5, 3, 1, [(1, 0), (3, 4)]),
    (0, 7, 3, 1, [(1, 0), (2, 2), (3, 6)]), (0, 8, 3, 0, [(0, 0)]), (0, 32, 7, 2, [(2, 0)]),
    (0, 33, 7, 2, [(2, 0), (7, 32)]), (0, 31, 7, 3, [(3, 0), (4, 2), (5, 6), (6, 14), (7, 30)]),
    (0, 64, 7, 1, [(1, 0)]), (0, 1, 2, 2, [(2, 0)]),
]

# (squareSize, start, blobLen, [(path index, row, instructions)])
COMMIT_PATH_CASES = [
    (2, 2, 2, [(0, 1, [L]), (1, 1, [R])]),
    (4, 2, 2, [(0, 0, [R, L]), (1, 0, [R, R])]),
    (4, 3, 2, [(0, 0, [R, R]), (1, 1, [L, L])]),
    (128, 8252, 1, [(0, 64, [L, R, R, R, R, L, L])]),
    (128, 0, 8193, [(31, 31, [])]),
    (128, 0, 8192, [(31, 31, [])]),
    (128, 0, 64, [(31, 0, [L, L, R, R, R, R, R])]),
    (128, 0, 65, [(31, 0, [L, R, R, R, R, R]), (32, 0, [R, L, L, L, L, L, L])]),
]

# (cursor, blobLen, squareSize, expectedIndex)
NEXT_INDEX_CASES = [(0, 4, 4, 0), (1, 2, 4, 1), (2, 2, 4, 2), (3, 4, 8, 3), (3, 5, 8, 3), (3, 2, 8, 3),
                    (1, 12, 16, 1), (10291, 1, 128, 10291), (11, 2, 8, 11), (11, 11, 8, 11), (11, 64, 64, 11),
                    (64, 65, 128, 64), (64, 63, 128, 64), (1, 63, 16, 1), (1, 16256, 128, 128),
                    (1, 8192, 128, 128), (1, 4096, 128, 64), (1, 8193, 128, 128)]


@pytest.mark.parametrize("start,end,maxd,mind,want", COORD_CASES)
def test_sub_tree_root_coordinates(start, end, maxd, mind, want):
    got = inc.calculate_sub_tree_root_coordinates(maxd, mind, start, end)
    assert [(c.depth, c.position) for c in got] == want


def test_gen_sub_tree_root_path():
    assert inc.gen_sub_tree_root_path(0, 0) == []
    assert inc.gen_sub_tree_root_path(1, 0) == [L]
    assert inc.gen_sub_tree_root_path(3, 4) == [R, L, L]
    assert inc.gen_sub_tree_root_path(7, 30) == [L, L, R, R, R, R, L]


@pytest.mark.parametrize("sq,start,blob_len,want", COMMIT_PATH_CASES)
def test_commitment_paths(sq, start, blob_len, want):
    paths = inc.calculate_commitment_paths(sq, start, blob_len)
    for idx, row, instr in want:
        assert paths[idx].row == row
        assert paths[idx].instructions == instr


@pytest.mark.parametrize("cursor,blob_len,sq,want", NEXT_INDEX_CASES)
def test_next_share_index(cursor, blob_len, sq, want):
    assert inc.next_share_index(cursor, blob_len) == want


def test_fits_in_square():
    assert inc.fits_in_square(0, 4, 64, 4, 4, 4, 4) == (True, 16)
    assert inc.fits_in_square(1, 4, 64, 4, 4, 4, 4)[0] is False
    assert inc.fits_in_square(3, 2, 64) == (True, 0)
