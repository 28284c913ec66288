"""Device-resident batched pipeline (block replay / sync batches).

PyTorch is used only as the device allocator and stream provider; the work is
the HIP kernels behind dagpu_extend_batch_device (include/dagpu.h).  Inputs are
already resident in HBM and only the roots/DAH (or nothing) come back.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _abi
from .da import Context, DAError, default_context

ROOT = _abi.ROOT_SIZE


def _stream_handle(stream: Optional[torch.cuda.Stream]) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


class DeviceSquares:
    """n squares of width k resident on one GPU.

    ods:  (n, k*k*512) uint8   eds: (n, 4k^2*512) uint8
    row_roots/col_roots: (n, 2k, 90)   dah: (n, 32)   status: (n,) int32
    """

    def __init__(self, k: int, n: int, device: int = 0, ctx: Optional[Context] = None,
                 with_ods: bool = True, in_place: bool = False):
        self.k, self.n = int(k), int(n)
        self.ctx = ctx or default_context()
        dev = torch.device("cuda", device)
        w = 2 * self.k
        # in_place: the ODS lives in Q0 of the EDS buffer itself (rows at the EDS
        # row pitch), the zero-copy input of dagpu_extend_batch_device (d_ods = NULL)
        self.in_place = bool(in_place)
        self.ods = (torch.empty((n, self.k * self.k * 512), dtype=torch.uint8, device=dev)
                    if with_ods and not in_place else None)
        self.eds = torch.empty((n, w * w * 512), dtype=torch.uint8, device=dev)
        self.row_roots = torch.empty((n, w, ROOT), dtype=torch.uint8, device=dev)
        self.col_roots = torch.empty((n, w, ROOT), dtype=torch.uint8, device=dev)
        self.dah = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        self.status = torch.zeros((n,), dtype=torch.int32, device=dev)
        ws = self.ctx._L.dagpu_workspace_size(self.k, self.n)
        self.workspace = torch.empty((ws,), dtype=torch.uint8, device=dev)
        # tensors of started repairs, held until their join (dagpu_repair_start:
        # the buffers must stay valid until the joined stream has passed the repair)
        self._held = {}

    def q0(self) -> torch.Tensor:
        """(n, k, k*512) view of Q0 inside the EDS buffer."""
        w = 2 * self.k
        return self.eds.view(self.n, w, w * 512)[:, :self.k, :self.k * 512]

    def load_ods(self, ods) -> None:
        """Copy n ODS (anything viewable as (n, k*k*512) uint8) to where extend()
        reads them: self.ods, or Q0 of the EDS when in_place."""
        src = ods if isinstance(ods, torch.Tensor) else torch.from_numpy(ods)
        src = src.reshape(self.n, self.k, self.k * 512)
        if self.in_place:
            self.q0().copy_(src)
        else:
            self.ods.view(self.n, self.k, self.k * 512).copy_(src)

    def _ck(self, rc: int) -> None:
        if rc != 0:
            raise DAError(rc, self.ctx.last_error())

    def extend(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        """ODS -> EDS -> roots -> DAH, enqueued on `stream` (no sync)."""
        L = self.ctx._L
        self._ck(L.dagpu_extend_batch_device(
            self.ctx.handle, self.k, self.n, _abi.addr(self.ods), _abi.addr(self.eds),
            _abi.addr(self.row_roots), _abi.addr(self.col_roots), _abi.addr(self.dah),
            _abi.addr(self.status), _abi.addr(self.workspace), _stream_handle(stream)))

    def extend_from(self, ods: torch.Tensor, stream: Optional[torch.cuda.Stream] = None) -> int:
        """Extend the first m = ods.shape[0] (<= n) squares taking their ODS
        from `ods` ((m, k*k*512) uint8 on this device, e.g. a window of a
        resident block-replay shard) instead of self.ods.  Returns m."""
        m = int(ods.shape[0])
        if m > self.n or ods.dtype != torch.uint8 or ods.device != self.eds.device \
                or not ods.is_contiguous() or ods.numel() != m * self.k * self.k * 512:
            raise ValueError("ods must be a contiguous (m <= n, k*k*512) uint8 tensor on this device")
        L = self.ctx._L
        self._ck(L.dagpu_extend_batch_device(
            self.ctx.handle, self.k, m, _abi.addr(ods), _abi.addr(self.eds),
            _abi.addr(self.row_roots), _abi.addr(self.col_roots), _abi.addr(self.dah),
            _abi.addr(self.status), _abi.addr(self.workspace), _stream_handle(stream)))
        return m

    def extend_rs(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        self._ck(self.ctx._L.dagpu_extend_rs_device(
            self.ctx.handle, self.k, self.n, _abi.addr(self.ods), _abi.addr(self.eds),
            _stream_handle(stream)))

    def repair(self, present: torch.Tensor, status: torch.Tensor, workspace: torch.Tensor,
               stream: Optional[torch.cuda.Stream] = None, byz: Optional[torch.Tensor] = None) -> None:
        """Device-resident rsmt2d Repair of self.eds against self.row/col_roots.
        present: (n, (2k)^2) uint8, updated in place; status: (n,) int32;
        byz (optional): (n, 4) int32 on the device -> failing axis per square
        (dagpu_repair_batch_device_ex)."""
        L = self.ctx._L
        if byz is None:
            self._ck(L.dagpu_repair_batch_device(
                self.ctx.handle, self.k, self.n, _abi.addr(self.eds), _abi.addr(present),
                _abi.addr(self.row_roots), _abi.addr(self.col_roots), _abi.addr(status),
                _abi.addr(workspace), _stream_handle(stream)))
            return
        if byz.dtype != torch.int32 or byz.numel() != 4 * self.n or byz.device != self.eds.device:
            raise ValueError("byz must be an (n, 4) int32 tensor on this device")
        self._ck(L.dagpu_repair_batch_device_ex(
            self.ctx.handle, self.k, self.n, _abi.addr(self.eds), _abi.addr(present),
            _abi.addr(self.row_roots), _abi.addr(self.col_roots), _abi.addr(status), _abi.addr(byz),
            _abi.addr(workspace), _stream_handle(stream)))

    def repair_start(self, present: torch.Tensor, status: torch.Tensor, workspace: torch.Tensor,
                     stream: Optional[torch.cuda.Stream] = None, first: int = 0, count: Optional[int] = None) -> int:
        """dagpu_repair_start on squares [first, first + count) (default all):
        returns at once with a handle for repair_join; the crossword runs on a
        library worker thread and stream forked from `stream`.  present /
        status / workspace as repair() (status and present indexed from
        `first`; workspace sized for `count` squares)."""
        import ctypes
        count = self.n - first if count is None else count
        w = 2 * self.k
        h = ctypes.c_uint64(0)
        self._ck(self.ctx._L.dagpu_repair_start(
            self.ctx.handle, self.k, count, self.eds.data_ptr() + first * w * w * 512,
            present.data_ptr() + first * w * w, self.row_roots.data_ptr() + first * w * ROOT,
            self.col_roots.data_ptr() + first * w * ROOT, status.data_ptr() + 4 * first, workspace.data_ptr(),
            _stream_handle(stream), ctypes.byref(h)))
        # the repair runs on the library's stream: keep its tensors (a temporary
        # workspace included) out of the caching allocator until the join
        self._held[h.value] = (present, status, workspace)
        return h.value

    def repair_join(self, handle: int, stream: Optional[torch.cuda.Stream] = None) -> None:
        """dagpu_repair_join: `stream` waits for the started repair.  The tensors
        held since repair_start are released in `stream`'s order: record_stream
        makes the caching allocator wait for the work queued on the join stream
        (which includes the repair) before it reuses their blocks, whichever
        stream allocated them."""
        js = stream if stream is not None else torch.cuda.current_stream()
        try:
            self._ck(self.ctx._L.dagpu_repair_join(self.ctx.handle, handle, int(js.cuda_stream)))
        finally:
            for t in self._held.pop(handle, ()):
                t.record_stream(js)

    def repair_workspace(self, count: Optional[int] = None) -> torch.Tensor:
        ws = self.ctx._L.dagpu_repair_workspace_size(self.k, self.n if count is None else count)
        return torch.empty((ws,), dtype=torch.uint8, device=self.eds.device)

    def roots(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        self._ck(self.ctx._L.dagpu_roots_device(
            self.ctx.handle, self.k, self.n, _abi.addr(self.eds), _abi.addr(self.row_roots),
            _abi.addr(self.col_roots), _abi.addr(self.dah), _abi.addr(self.status),
            _abi.addr(self.workspace), _stream_handle(stream)))
