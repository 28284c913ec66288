"""ctypes binding of include/dagpu.h (libdagpu.so, built for gfx950).

The product path: every compute call goes through the HIP library.  If the
library is missing this module raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# DAGPU_LIB selects another build of the same library (A/B runs of kernel variants)
LIB_PATH = os.environ.get("DAGPU_LIB") or os.path.join(_PKG_ROOT, "libdagpu.so")

SHARE_SIZE = 512
NAMESPACE_SIZE = 29
ROOT_SIZE = 90
HASH_SIZE = 32

OK = 0
ERR_NOT_POW2 = -1
ERR_NOT_SQUARE = -2
ERR_SHARE_SIZE = -3
ERR_PUSH_ORDER = -4
ERR_TOO_FEW_SHARDS = -5
ERR_UNREPAIRABLE = -6
ERR_BYZANTINE = -7
ERR_BAD_ROOTS = -8
ERR_ARG = -9
ERR_DEVICE = -10
ERR_UNSUPPORTED = -11
ERR_PROOF = -12
ERR_SQUARE = -13

# Every symbol include/dagpu.h declares (checked by tests/test_abi_cpu.py).
EXPORTS = (
    "dagpu_version",
    "dagpu_max_square_width",
    "dagpu_max_codec_width",
    "dagpu_init",
    "dagpu_destroy",
    "dagpu_last_error",
    "dagpu_nmt_verify_inclusion",
    "dagpu_merkle_verify",
    "dagpu_host_alloc",
    "dagpu_host_free",
    "dagpu_host_register",
    "dagpu_host_unregister",
    "dagpu_extend_shares",
    "dagpu_extend_batch",
    "dagpu_workspace_size",
    "dagpu_extend_batch_device",
    "dagpu_extend_rs_device",
    "dagpu_roots_device",
    "dagpu_roots",
    "dagpu_encode",
    "dagpu_decode",
    "dagpu_repair_workspace_size",
    "dagpu_repair_batch_device",
    "dagpu_repair_batch_device_ex",
    "dagpu_repair_start",
    "dagpu_repair_join",
    "dagpu_repair",
    "dagpu_repair_ex",
    "dagpu_square_construct",
    "dagpu_square_build",
    "dagpu_profile_enable",
    "dagpu_profile_read",
    "dagpu_profile_stages",
    "dagpu_repair_stats",
    "dagpu_dah_hash",
    "dagpu_nmt_roots",
    "dagpu_wrapper_roots",
    "dagpu_merkle_roots",
    "dagpu_merkle_levels",
    "dagpu_subtree_width",
    "dagpu_blob_commitments",
    "dagpu_split_workspace_size",
    "dagpu_split_rows_device",
    "dagpu_split_cols_device",
    "dagpu_split_finish_device",
    "dagpu_row_nodes_size",
    "dagpu_row_nodes_workspace_size",
    "dagpu_row_nodes_device",
    "dagpu_row_nodes_gather_device",
)

PREFIX_NONE = 0
PREFIX_SELF = 1
PREFIX_PARITY = 2
PREFIX_FLAGS = 3

PROFILE_KERNELS = ("rs_row", "rs_col", "nmt_leaves", "nmt_trees", "dah", "decode", "repair_fill")
# dagpu_profile_stages (include/dagpu.h DAGPU_STAGE_*)
STAGES = ("start", "uploaded", "rs_rows", "rs_cols", "leaves", "trees", "dah", "results", "eds_top", "eds_bottom")

_lib = None

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
i32p = ctypes.POINTER(ctypes.c_int32)
vp = ctypes.c_void_p
sz = ctypes.c_size_t


class _Unbound:
    """Stand-in for an entry point an older build (DAGPU_LIB A/B runs) lacks."""

    def __init__(self, name):
        self.name = name

    def __call__(self, *a):
        raise AttributeError(f"{LIB_PATH}: no symbol {self.name}")


class _Tolerant:
    """An alternate build under A/B (DAGPU_LIB): symbols it lacks stay unbound."""

    def __init__(self, L):
        object.__setattr__(self, "_L", L)

    def __getattr__(self, name):
        try:
            return getattr(self._L, name)
        except AttributeError:
            u = _Unbound(name)
            object.__setattr__(self, name, u)
            return u


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"HIP extension not built: {LIB_PATH} missing (run __graft_entry__.build())")
        # Load PyTorch's bundled HIP runtime first when torch is installed:
        # libdagpu.so and torch then share ONE libamdhip64.so.7 (same soname).
        # Loading /opt/rocm's copy first would make torch bind to it and fail
        # its own device init ("No HIP GPUs are available").
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        if os.environ.get("DAGPU_LIB"):
            L = _Tolerant(L)
        L.dagpu_version.restype = ctypes.c_int
        L.dagpu_max_square_width.restype = ctypes.c_uint32
        L.dagpu_max_codec_width.restype = ctypes.c_uint32
        L.dagpu_init.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
        L.dagpu_destroy.argtypes = [vp]
        L.dagpu_destroy.restype = None
        L.dagpu_last_error.argtypes = [vp]
        L.dagpu_last_error.restype = ctypes.c_char_p
        i64 = ctypes.c_int64
        L.dagpu_nmt_verify_inclusion.argtypes = [vp, vp, sz, sz, i64, i64, vp, sz, vp]
        L.dagpu_merkle_verify.argtypes = [vp, vp, sz, i64, i64, vp, sz]
        L.dagpu_host_alloc.argtypes = [sz]
        L.dagpu_host_alloc.restype = vp
        L.dagpu_host_free.argtypes = [vp]
        L.dagpu_host_free.restype = None
        L.dagpu_host_register.argtypes = [vp, sz]
        L.dagpu_host_unregister.argtypes = [vp]
        L.dagpu_extend_shares.argtypes = [vp, vp, sz, sz, vp, vp, vp, vp]
        L.dagpu_extend_batch.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp]
        L.dagpu_workspace_size.argtypes = [ctypes.c_uint32, sz]
        L.dagpu_workspace_size.restype = sz
        L.dagpu_extend_batch_device.argtypes = [vp, ctypes.c_uint32, sz, vp, vp, vp, vp, vp, vp,
                                                vp, vp]
        L.dagpu_extend_rs_device.argtypes = [vp, ctypes.c_uint32, sz, vp, vp, vp]
        L.dagpu_roots_device.argtypes = [vp, ctypes.c_uint32, sz, vp, vp, vp, vp, vp, vp, vp]
        L.dagpu_roots.argtypes = [vp, ctypes.c_uint32, vp, vp, vp, vp]
        L.dagpu_encode.argtypes = [vp, ctypes.c_uint32, sz, sz, vp, vp]
        L.dagpu_decode.argtypes = [vp, ctypes.c_uint32, sz, sz, vp, vp]
        L.dagpu_repair_batch_device.argtypes = [vp, ctypes.c_uint32, sz, vp, vp, vp, vp, vp, vp,
                                                vp]
        L.dagpu_repair_workspace_size.argtypes = [ctypes.c_uint32, sz]
        L.dagpu_repair_workspace_size.restype = sz
        L.dagpu_repair.argtypes = [vp, ctypes.c_uint32, vp, vp, vp, vp]
        L.dagpu_profile_stages.argtypes = [vp, vp]
        L.dagpu_repair_stats.argtypes = [vp, vp]
        L.dagpu_repair_ex.argtypes = [vp, ctypes.c_uint32, vp, vp, vp, vp, vp]
        L.dagpu_square_construct.argtypes = [vp, vp, vp, sz, ctypes.c_uint32, ctypes.c_uint32, vp, sz, vp]
        L.dagpu_square_build.argtypes = [vp, vp, vp, sz, ctypes.c_uint32, ctypes.c_uint32, vp, sz, vp, vp]
        L.dagpu_repair_batch_device_ex.argtypes = [vp, ctypes.c_uint32, sz, vp, vp, vp, vp, vp, vp,
                                                   vp, vp]
        L.dagpu_repair_start.argtypes = [vp, ctypes.c_uint32, sz, vp, vp, vp, vp, vp, vp, vp,
                                         ctypes.POINTER(ctypes.c_uint64)]
        L.dagpu_repair_join.argtypes = [vp, ctypes.c_uint64, vp]
        L.dagpu_dah_hash.argtypes = [vp, vp, sz, vp]
        L.dagpu_nmt_roots.argtypes = [vp, sz, vp, vp, sz, ctypes.c_int, vp, ctypes.c_int, vp, vp]
        L.dagpu_wrapper_roots.argtypes = [vp, ctypes.c_uint64, sz, vp, vp, vp, sz, vp, vp]
        L.dagpu_merkle_roots.argtypes = [vp, sz, vp, vp, sz, vp]
        L.dagpu_merkle_levels.argtypes = [vp, sz, vp, sz, vp, ctypes.POINTER(sz)]
        L.dagpu_subtree_width.argtypes = [ctypes.c_uint64, ctypes.c_uint32]
        L.dagpu_blob_commitments.argtypes = [vp, sz, vp, vp, vp, ctypes.c_uint32, vp]
        L.dagpu_split_workspace_size.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.dagpu_split_workspace_size.restype = sz
        L.dagpu_split_rows_device.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, vp, vp,
                                              vp, vp, vp]
        L.dagpu_split_cols_device.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, vp, vp,
                                              vp, vp, vp, vp]
        L.dagpu_split_finish_device.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp, vp, vp, vp]
        L.dagpu_row_nodes_size.argtypes = [ctypes.c_uint32]
        L.dagpu_row_nodes_size.restype = sz
        L.dagpu_row_nodes_workspace_size.argtypes = [ctypes.c_uint32]
        L.dagpu_row_nodes_workspace_size.restype = sz
        L.dagpu_row_nodes_device.argtypes = [vp, ctypes.c_uint32, vp, vp, vp, vp]
        L.dagpu_row_nodes_gather_device.argtypes = [vp, ctypes.c_uint32, vp, sz, vp, vp, vp]
        L.dagpu_profile_enable.argtypes = [vp, ctypes.c_int]
        L.dagpu_profile_read.argtypes = [vp, vp, vp, ctypes.c_int]
        _lib = L
    return _lib


def addr(buf) -> int:
    """Address of a numpy array / bytearray / torch tensor (device or host)."""
    if buf is None:
        return 0
    if hasattr(buf, "data_ptr"):
        return buf.data_ptr()
    if hasattr(buf, "ctypes"):
        return buf.ctypes.data
    if isinstance(buf, bytearray):
        return ctypes.addressof((ctypes.c_char * len(buf)).from_buffer(buf))
    raise TypeError(f"unsupported buffer type {type(buf)}")
