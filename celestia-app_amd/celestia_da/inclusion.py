"""Host-side mirror of pkg/inclusion's EDS-side commitment path:

  EDSSubTreeRootCacher / getSubTreeRoot   pkg/inclusion/nmt_caching.go:81-128
  GetCommitment                           pkg/inclusion/get_commit.go:12-30
  calculateCommitmentPaths, genSubTreeRootPath, calculateSubTreeRootCoordinates
                                          pkg/inclusion/paths.go
  NextShareIndex, BlobSharesUsedNonInteractiveDefaults, FitsInSquare
                                          pkg/inclusion/blob_share_commitment_rules.go:10-75

The reference caches every row-tree inner node through an nmt.NodeVisitor while
rsmt2d builds the roots, then walks the cache from the DAH row root.  Here the
GPU hashes every node of every row tree once (dagpu_row_nodes_device) and keeps
them in HBM; a walk is index arithmetic on the full binary tree (row trees of
an EDS have 2k leaves, a power of two), and subtree roots are gathered on the
device (dagpu_row_nodes_gather_device).  The path arithmetic is host logic.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _abi
from .da import Context, DAError, DataAvailabilityHeader, default_context
from .trees import DEFAULT_SUBTREE_ROOT_THRESHOLD, hash_from_byte_slices, subtree_width

WALK_LEFT = False
WALK_RIGHT = True


# ---- blob_share_commitment_rules.go ------------------------------------------------

def round_up_by_multiple_of(cursor: int, v: int) -> int:
    return cursor if cursor % v == 0 else (cursor // v + 1) * v


def next_share_index(cursor: int, blob_share_len: int,
                     subtree_root_threshold: int = DEFAULT_SUBTREE_ROOT_THRESHOLD) -> int:
    """NextShareIndex: first index >= cursor aligned to the blob's subtree width."""
    return round_up_by_multiple_of(cursor, subtree_width(blob_share_len, subtree_root_threshold))


def blob_shares_used_non_interactive_defaults(cursor: int, subtree_root_threshold: int,
                                              *blob_share_lens: int):
    start = cursor
    indexes = []
    for n in blob_share_lens:
        cursor = next_share_index(cursor, n, subtree_root_threshold)
        indexes.append(cursor)
        cursor += n
    return cursor - start, indexes


def fits_in_square(cursor: int, square_size: int, subtree_root_threshold: int, *blob_share_lens: int):
    if not blob_share_lens:
        return cursor <= square_size * square_size, 0
    cursor = next_share_index(cursor, blob_share_lens[0], subtree_root_threshold)
    used, _ = blob_shares_used_non_interactive_defaults(cursor, subtree_root_threshold, *blob_share_lens)
    return cursor + used <= square_size * square_size, used


# ---- paths.go -------------------------------------------------------------------------

@dataclass(frozen=True)
class Coord:
    depth: int
    position: int

    def climb(self) -> "Coord":
        return Coord(self.depth - 1, self.position // 2)

    def can_climb_right(self, min_depth: int) -> bool:
        return self.position % 2 == 0 and self.depth > min_depth


@dataclass
class Path:
    instructions: List[bool]
    row: int


def calculate_sub_tree_root_coordinates(max_depth: int, min_depth: int, start: int, end: int) -> List[Coord]:
    """Minimal set of subtree roots covering leaves [start, end) of a full
    binary tree of depth max_depth, no root above min_depth (paths.go)."""
    coords: List[Coord] = []
    leaf = start
    node = Coord(max_depth, start)
    last_node, last_leaf, span = node, leaf, 1

    def reset():
        nonlocal last_node, last_leaf, node, span
        last_node, last_leaf = node, leaf
        node = Coord(max_depth, leaf)
        span = 1

    while True:
        if leaf + 1 == end:
            coords.append(node)
            return coords
        if leaf + 1 > end:
            coords.append(last_node)
            leaf = last_leaf + 1
            reset()
        elif not node.can_climb_right(min_depth):
            coords.append(node)
            leaf += 1
            reset()
        else:
            last_leaf, last_node = leaf, node
            leaf += span
            span *= 2
            node = node.climb()


def gen_sub_tree_root_path(depth: int, pos: int) -> List[bool]:
    return [WALK_RIGHT if (pos >> i) & 1 else WALK_LEFT for i in range(depth - 1, -1, -1)]


def calculate_commitment_paths(square_size: int, start: int, blob_share_len: int,
                               subtree_root_threshold: int = DEFAULT_SUBTREE_ROOT_THRESHOLD) -> List[Path]:
    start = next_share_index(start, blob_share_len, subtree_root_threshold)
    start_row, end_row = start // square_size, (start + blob_share_len - 1) // square_size
    norm_start = start % square_size
    norm_end = (start + blob_share_len) - end_row * square_size
    max_depth = int(math.log2(square_size))
    out: List[Path] = []
    for i in range(start_row, end_row + 1):
        s, e = 0, square_size
        if i == start_row:
            s = norm_start
        if i == end_row:
            e = norm_end
        sub_max = int(math.log2(subtree_width(blob_share_len, subtree_root_threshold)))
        for c in calculate_sub_tree_root_coordinates(max_depth, max_depth - sub_max, s, e):
            out.append(Path(gen_sub_tree_root_path(c.depth, c.position), i))
    return out


# ---- the cacher -------------------------------------------------------------------------

class EDSSubTreeRootCacher:
    """Every row-tree node of one EDS, resident in HBM (96-B records).

    Built from an EDS already on the device (`d_eds`, (2k)^2*512 bytes) or from
    host bytes (uploaded once)."""

    def __init__(self, k: int, eds, ctx: Optional[Context] = None, device: int = 0):
        self.ctx = ctx or default_context()
        self.k = k
        self.w = 2 * k
        L = self.ctx._L
        dev = torch.device("cuda", device)
        if isinstance(eds, torch.Tensor) and eds.is_cuda:
            d_eds = eds.reshape(-1)
        else:
            d_eds = torch.from_numpy(np.ascontiguousarray(eds, dtype=np.uint8).reshape(-1)).to(dev)
        if d_eds.numel() != self.w * self.w * 512:
            raise DAError(_abi.ERR_ARG, "EDS size does not match k")
        self.nodes = torch.empty(L.dagpu_row_nodes_size(k), dtype=torch.uint8, device=d_eds.device)
        ws = torch.empty(L.dagpu_row_nodes_workspace_size(k), dtype=torch.uint8, device=d_eds.device)
        self.ctx.check(L.dagpu_row_nodes_device(self.ctx.handle, k, d_eds.data_ptr(), self.nodes.data_ptr(),
                                                ws.data_ptr(), torch.cuda.current_stream().cuda_stream))

    def nodes_at(self, rows: Sequence[int], depths: Sequence[int], positions: Sequence[int]) -> List[bytes]:
        n = len(rows)
        if n == 0:
            return []
        req = torch.tensor(np.stack([rows, depths, positions], axis=1).astype(np.uint32).view(np.int32),
                           device=self.nodes.device)
        out = torch.empty(n * _abi.ROOT_SIZE, dtype=torch.uint8, device=self.nodes.device)
        self.ctx.check(self.ctx._L.dagpu_row_nodes_gather_device(
            self.ctx.handle, self.k, self.nodes.data_ptr(), n, req.data_ptr(), out.data_ptr(),
            torch.cuda.current_stream().cuda_stream))
        host = out.cpu().numpy()
        return [host[i * 90:(i + 1) * 90].tobytes() for i in range(n)]

    def get_sub_tree_roots(self, dah: DataAvailabilityHeader, requests: Sequence[Path]) -> List[bytes]:
        """getSubTreeRoot for many (row, path) pairs; same errors as the reference."""
        if self.w != len(dah.row_roots):
            raise DAError(_abi.ERR_ARG, "data availability header has unexpected number of row roots: "
                                        f"expected {self.w} got {len(dah.row_roots)}")
        rows = [p.row for p in requests]
        for r in rows:
            if r >= self.w:
                raise DAError(_abi.ERR_ARG, f"row exceeds range of cache: max {self.w} got {r}")
        depth_max = int(math.log2(self.w))
        for p in requests:
            if len(p.instructions) > depth_max:
                raise DAError(_abi.ERR_ARG, "did not find sub tree root: path longer than the tree")
        roots = self.nodes_at(sorted(set(rows)), [0] * len(set(rows)), [0] * len(set(rows)))
        root_of = dict(zip(sorted(set(rows)), roots))
        for r in set(rows):  # the walk starts from the DAH row root
            if root_of[r] != dah.row_roots[r]:
                raise DAError(_abi.ERR_ARG, f"did not find sub tree root: {dah.row_roots[r].hex()}")
        depths = [len(p.instructions) for p in requests]
        pos = [sum((1 << (len(p.instructions) - 1 - i)) for i, b in enumerate(p.instructions) if b)
               for p in requests]
        return self.nodes_at(rows, depths, pos)

    def get_sub_tree_root(self, dah: DataAvailabilityHeader, row: int, path: Sequence[bool]) -> bytes:
        return self.get_sub_tree_roots(dah, [Path(list(path), row)])[0]


def get_commitment(cacher: EDSSubTreeRootCacher, dah: DataAvailabilityHeader, start: int,
                   blob_share_len: int,
                   subtree_root_threshold: int = DEFAULT_SUBTREE_ROOT_THRESHOLD) -> bytes:
    """GetCommitment (get_commit.go:12-30): the share commitment of a blob laid
    out at `start` in the original data square, from the cached row trees."""
    square_size = len(dah.row_roots) // 2
    if start + blob_share_len > square_size * square_size:
        raise DAError(_abi.ERR_ARG, "cannot get commitment for blob that doesn't fit in square")
    paths = calculate_commitment_paths(square_size, start, blob_share_len, subtree_root_threshold)
    # prepend WalkLeft: the subtree roots live in the original-data half of each row
    reqs = [Path([WALK_LEFT] + p.instructions, p.row) for p in paths]
    roots = cacher.get_sub_tree_roots(dah, reqs)
    return hash_from_byte_slices(roots, cacher.ctx)
