"""One oversized square split over P GPUs (BASELINE configs[4] stress square;
SURVEY.md §8e), one process per GPU.

The result is the square's ordinary EDS row/column roots and DAH
(da.ExtendShares + NewDataAvailabilityHeader, pkg/da/data_availability_header.go:44-108);
the split only changes placement.  Rank g owns Q0 rows [g*k/P, (g+1)*k/P) and,
after ONE all-to-all (RCCL over xGMI), EDS columns [g*2k/P, (g+1)*2k/P).  The
five steps are documented in include/dagpu.h; the kernels are split.cpp /
nmt_forest.hip / rs_gf16.hip.  The collectives are torch.distributed calls on
device tensors (backend "nccl" = RCCL); a gloo group stages through host memory.

`extend_split_local` runs all P parts in one process on one GPU, with the
all-to-all done as device copies: the single-GPU check of every kernel and of
the block layout the collective sees.
"""
from __future__ import annotations

import contextlib
from typing import List, Optional, Sequence, Tuple

import torch

from . import _abi
from .da import Context, DAError, ErrInvalidPushOrder
from ._abi import ROOT_SIZE, SHARE_SIZE

REC = 96  # row-subtree record: minNs[32] | maxNs[32] | digest[32]


def _stream(s: Optional[torch.cuda.Stream]) -> int:
    return (s or torch.cuda.current_stream()).cuda_stream


def _on(stream: Optional[torch.cuda.Stream]):
    """The library's split steps only queue work on `stream` (no host sync
    inside them), so every torch-side step between them -- copies, cat/clone,
    status reads, the torch.distributed collectives -- must run in that
    stream's order too: torch's current stream for the block."""
    return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()


class SplitPart:
    """Device buffers and steps of one rank (part) of a split square."""

    def __init__(self, k: int, parts: int, part: int, ctx: Context, device: torch.device):
        if parts < 1 or parts & (parts - 1) or parts > k:
            raise DAError(_abi.ERR_ARG, "parts must be a power of two <= k")
        self.k, self.parts, self.part, self.ctx = k, parts, part, ctx
        self.w = 2 * k
        self.W = self.w // parts
        self.rows = k // parts
        L = ctx._L
        ws = L.dagpu_split_workspace_size(k, parts)
        if ws == 0:
            if k == 2 * L.dagpu_max_square_width() and parts < 8:  # include/dagpu.h DAGPU_MAX_SPLIT_WIDTH
                raise DAError(_abi.ERR_UNSUPPORTED,
                              f"split square k = {k} needs >= 8 parts (its EDS is 512 GiB)")
            raise DAError(_abi.ERR_ARG, f"invalid split k={k} parts={parts}")
        u8 = dict(dtype=torch.uint8, device=device)
        self.ws = torch.empty(ws, **u8)
        self.slab = torch.empty(self.w * self.W * SHARE_SIZE, **u8)
        # one part: the rows' send block is the top of its own slab (no exchange)
        self.send = (self.slab[: self.rows * self.w * SHARE_SIZE] if parts == 1
                     else torch.empty(self.rows * self.w * SHARE_SIZE, **u8))
        self.col_roots = torch.empty(self.W * ROOT_SIZE, **u8)
        self.row_sub = torch.empty(self.w * REC, **u8)
        self.status = torch.zeros(1, dtype=torch.int32, device=device)

    @property
    def slab_top(self) -> torch.Tensor:
        """Rows 0..k-1 of the column slab: the all-to-all receive buffer."""
        return self.slab[: self.k * self.W * SHARE_SIZE]

    def step_rows(self, ods_rows: torch.Tensor, stream=None) -> None:
        assert ods_rows.numel() == self.rows * self.k * SHARE_SIZE and ods_rows.is_contiguous()
        self.ctx.check(self.ctx._L.dagpu_split_rows_device(
            self.ctx.handle, self.k, self.parts, self.part, ods_rows.data_ptr(), self.send.data_ptr(),
            self.status.data_ptr(), self.ws.data_ptr(), _stream(stream)))

    def step_cols(self, stream=None) -> None:
        self.ctx.check(self.ctx._L.dagpu_split_cols_device(
            self.ctx.handle, self.k, self.parts, self.part, self.slab.data_ptr(), self.col_roots.data_ptr(),
            self.row_sub.data_ptr(), self.status.data_ptr(), self.ws.data_ptr(), _stream(stream)))

    def step_finish(self, row_sub_all: torch.Tensor, col_roots_all: torch.Tensor,
                    stream=None) -> Tuple[torch.Tensor, torch.Tensor]:
        assert row_sub_all.numel() == self.parts * self.w * REC
        assert col_roots_all.numel() == self.w * ROOT_SIZE
        row_roots = torch.empty(self.w * ROOT_SIZE, dtype=torch.uint8, device=self.slab.device)
        dah = torch.empty(32, dtype=torch.uint8, device=self.slab.device)
        self.ctx.check(self.ctx._L.dagpu_split_finish_device(
            self.ctx.handle, self.k, self.parts, row_sub_all.data_ptr(), col_roots_all.data_ptr(),
            row_roots.data_ptr(), dah.data_ptr(), self.ws.data_ptr(), _stream(stream)))
        return row_roots, dah


def _check_status(status: int) -> None:
    if status & 1:
        raise ErrInvalidPushOrder(_abi.ERR_PUSH_ORDER,
                                  "invalid push order: namespaces of original data square are not sorted")


def extend_split_local(ods: torch.Tensor, k: int, parts: int, ctx: Context,
                       stream=None) -> Tuple[bytes, bytes, bytes]:
    """All P parts in this process on one GPU (all-to-all as device copies).
    ods: k*k*512 B device tensor.  Returns (row_roots, col_roots, dah) bytes."""
    with _on(stream):
        return _extend_split_local(ods, k, parts, ctx, stream)


def _extend_split_local(ods, k, parts, ctx, stream):
    dev = ods.device
    ps = [SplitPart(k, parts, g, ctx, dev) for g in range(parts)]
    rows_b = ps[0].rows * k * SHARE_SIZE
    for g, p in enumerate(ps):
        p.step_rows(ods[g * rows_b:(g + 1) * rows_b], stream)
    blk = ps[0].rows * ps[0].W * SHARE_SIZE
    for h, ph in enumerate(ps):  # rank h receives block h of every rank g, in rank order
        for g, pg in enumerate(ps):
            dst, src = ph.slab_top[g * blk:(g + 1) * blk], pg.send[h * blk:(h + 1) * blk]
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src)
    for p in ps:
        p.step_cols(stream)
    row_sub_all = torch.cat([p.row_sub for p in ps])
    col_all = torch.cat([p.col_roots for p in ps])
    status = max(int(p.status.item()) for p in ps)
    rr, dah = ps[0].step_finish(row_sub_all, col_all, stream)
    torch.cuda.synchronize(dev)
    _check_status(status)
    return rr.cpu().numpy().tobytes(), col_all.cpu().numpy().tobytes(), dah.cpu().numpy().tobytes()


# ---- the collectives (torch.distributed; nccl = RCCL over xGMI) -------------

def all_to_all_blocks(dist, out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """Equal-split all-to-all: block h of `inp` goes to rank h; `out` receives
    the blocks of ranks 0..P-1 in rank order.  gloo stages through host memory;
    dist=None is the single-rank case."""
    if dist is None:
        if out.data_ptr() != inp.data_ptr():  # one part: send block and slab top are one buffer
            out.copy_(inp)
        return
    if dist.get_backend(group) == "nccl" or out.device.type == "cpu":
        dist.all_to_all_single(out, inp, group=group)
        return
    o, i = out.cpu(), inp.cpu()
    dist.all_to_all_single(o, i, group=group)
    out.copy_(o)


def all_gather_flat(dist, out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """Rank-ordered concatenation of every rank's `inp` into `out`."""
    if dist is None:
        out.copy_(inp)
        return
    if dist.get_backend(group) == "nccl" or out.device.type == "cpu":
        dist.all_gather_into_tensor(out, inp, group=group)
        return
    parts = [torch.empty_like(inp, device="cpu") for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, inp.cpu(), group=group)
    out.copy_(torch.cat(parts))


def max_status(dist, status: torch.Tensor, group=None) -> int:
    if dist is None:
        return int(status.item())
    if dist.get_backend(group) == "nccl" or status.device.type == "cpu":
        t = status.clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        return int(t.item())
    t = status.cpu()
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def extend_split_distributed(dist, part: SplitPart, ods_rows: torch.Tensor, group=None,
                             stream=None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """One rank's share of the split: `ods_rows` are this rank's k/P Q0 rows
    (device).  Returns device tensors (row_roots 2k*90, col_roots 2k*90, dah 32),
    identical on every rank.  Raises ErrInvalidPushOrder like NewDAH.  With a
    `stream`, everything (the library steps, the collectives and the status
    read) runs in that stream's order."""
    with _on(stream):
        return _extend_split_distributed(dist, part, ods_rows, group, stream)


def _extend_split_distributed(dist, part, ods_rows, group, stream):
    part.step_rows(ods_rows, stream)
    all_to_all_blocks(dist, part.slab_top, part.send, group)
    part.step_cols(stream)
    own = dist is None
    if own:  # one part: its own records and roots are the gathered arrays
        row_sub_all, col_all = part.row_sub, part.col_roots
    else:
        row_sub_all = torch.empty(part.parts * part.row_sub.numel(), dtype=torch.uint8, device=part.slab.device)
        col_all = torch.empty(part.parts * part.col_roots.numel(), dtype=torch.uint8, device=part.slab.device)
        all_gather_flat(dist, row_sub_all, part.row_sub, group)
        all_gather_flat(dist, col_all, part.col_roots, group)
    rr, dah = part.step_finish(row_sub_all, col_all, stream)
    if own:  # the caller's copy (the part's buffer is rewritten by its next square)
        col_all = col_all.clone()
    # the status read-back is this step's one host wait, after all of it is queued
    status = max_status(dist, part.status, group)
    _check_status(status)
    return rr, col_all, dah


# ---- width routing (ExtendShares above one GPU's widest square) -------------

MIN_WIDE_PARTS = 8  # include/dagpu.h DAGPU_MAX_SPLIT_WIDTH: k = 16384 over >= 8 parts


def route(k: int, world: int) -> str:
    """Where `da.ExtendShares` of width k runs on a job of `world` GPUs
    (pkg/da/data_availability_header.go:65-75 puts no upper bound on k):
    "single" -- each rank extends whole squares (k <= dagpu_max_square_width());
    "split"  -- the square is split over all ranks (k = 16384 needs >= 8).
    Raises DAError(ERR_UNSUPPORTED) where neither path serves k."""
    if k < 1 or k & (k - 1):
        raise DAError(_abi.ERR_ARG, f"square width must be a power of two: got {k}")
    L = _abi.lib()
    if k <= L.dagpu_max_square_width():
        return "single"
    if k == 2 * L.dagpu_max_square_width() and world >= MIN_WIDE_PARTS and world & (world - 1) == 0:
        return "split"
    raise DAError(_abi.ERR_UNSUPPORTED,
                  f"square width k = {k} needs the split path over >= {MIN_WIDE_PARTS} GPUs (a power of two); "
                  f"this job has {world}" if k == 2 * L.dagpu_max_square_width()
                  else f"square width k = {k} is not supported (widest: {2 * L.dagpu_max_square_width()})")


def extend_wide_distributed(dist, k: int, ods_rows: torch.Tensor, ctx: Context, group=None,
                            stream=None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """ExtendShares + NewDataAvailabilityHeader of one square wider than a
    single GPU serves: this rank's k / world Q0 rows in, the square's row roots,
    column roots and DAH out (identical on every rank).  The part's buffers
    live for the call only (a 64 GiB slab per rank at k = 16384, P = 8)."""
    world = dist.get_world_size(group) if dist is not None else 1
    rank = dist.get_rank(group) if dist is not None else 0
    if route(k, world) != "split":
        raise DAError(_abi.ERR_ARG, f"k = {k} fits one GPU: use the single-GPU entry points")
    part = SplitPart(k, world, rank, ctx, ods_rows.device)
    try:
        return extend_split_distributed(dist, part, ods_rows, group, stream)
    finally:
        del part
