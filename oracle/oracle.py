"""ctypes binding for the CPU oracle (oracle/da_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package
(celestia-app_amd/).  See da_oracle.h for what it restates and where.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, "_build")

SHARE_SIZE = 512
NS_SIZE = 29
NODE_SIZE = 90

ERRORS = {
    -1: "number of shares is not a power of 2",
    -2: "number of chunks must be a square number",
    -3: "invalid shard size",
    -4: "invalid push order",
    -5: "too few shards given",
    -6: "failed to solve data square",
    -7: "byzantine data",
    -8: "bad root input",
    -9: "invalid argument",
}


class OracleError(Exception):
    def __init__(self, code: int):
        super().__init__(f"oracle error {code}: {ERRORS.get(code, '?')}")
        self.code = code


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_libs: dict = {}


def lib(portable: bool = False) -> ctypes.CDLL:
    name = "libda_oracle_portable.so" if portable else "libda_oracle.so"
    if name not in _libs:
        path = os.path.join(_BUILD, name)
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.orc_init.restype = None
        L.orc_sha256.argtypes = [u8p, ctypes.c_size_t, u8p]
        L.orc_encode.argtypes = [ctypes.c_int, ctypes.c_size_t, u8p, u8p]
        L.orc_decode.argtypes = [ctypes.c_int, ctypes.c_size_t, u8p, u8p]
        L.orc_extend_square.argtypes = [ctypes.c_int, u8p, u8p]
        L.orc_compute_roots.argtypes = [ctypes.c_int, u8p, u8p, u8p, ctypes.c_int]
        L.orc_rfc6962_root.argtypes = [u8p, ctypes.c_size_t, ctypes.c_size_t, u8p]
        L.orc_dah_hash.argtypes = [u8p, u8p, ctypes.c_size_t, u8p]
        L.orc_extend_and_dah.argtypes = [ctypes.c_int, u8p, u8p, u8p, u8p, u8p, ctypes.c_int]
        L.orc_repair.argtypes = [ctypes.c_int, u8p, u8p, u8p, u8p]
        L.orc_repair_ex.argtypes = [ctypes.c_int, u8p, u8p, u8p, u8p, ctypes.POINTER(ctypes.c_int32)]
        L.orc_nmt_leaf.argtypes = [u8p, u8p, ctypes.c_size_t, u8p]
        L.orc_nmt_node.argtypes = [u8p, u8p, u8p]
        L.orc_nmt_root_from_leaves.argtypes = [u8p, ctypes.c_size_t, u8p]
        L.orc_axis_root.argtypes = [ctypes.c_int, u8p, ctypes.c_int, ctypes.c_int, u8p]
        for n in ("orc_gf8_log", "orc_gf8_exp", "orc_gf8_skew", "orc_gf8_logwalsh"):
            getattr(L, n).restype = u8p
        for n in ("orc_gf16_log", "orc_gf16_exp", "orc_gf16_skew"):
            getattr(L, n).restype = ctypes.POINTER(ctypes.c_uint16)
        L.orc_init()
        _libs[name] = L
    return _libs[name]


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _u8(x) -> np.ndarray:
    if isinstance(x, (bytes, bytearray)):
        return np.frombuffer(bytes(x), dtype=np.uint8).copy()
    return np.ascontiguousarray(x, dtype=np.uint8)


def _check(rc: int) -> None:
    if rc != 0:
        raise OracleError(rc)


def sha256(data: bytes, portable: bool = False) -> bytes:
    a = _u8(data) if len(data) else np.zeros(1, np.uint8)
    out = np.zeros(32, np.uint8)
    lib(portable).orc_sha256(_p(a), len(data), _p(out))
    return out.tobytes()


def gf8_tables():
    L = lib()
    return (
        np.ctypeslib.as_array(L.orc_gf8_log(), (256,)).copy(),
        np.ctypeslib.as_array(L.orc_gf8_exp(), (256,)).copy(),
        np.ctypeslib.as_array(L.orc_gf8_skew(), (255,)).copy(),
        np.ctypeslib.as_array(L.orc_gf8_logwalsh(), (256,)).copy(),
    )


def gf16_tables():
    L = lib()
    return (
        np.ctypeslib.as_array(L.orc_gf16_log(), (65536,)).copy(),
        np.ctypeslib.as_array(L.orc_gf16_exp(), (65536,)).copy(),
        np.ctypeslib.as_array(L.orc_gf16_skew(), (65535,)).copy(),
    )


def encode(data: np.ndarray) -> np.ndarray:
    """data: (k, shard) uint8 -> parity (k, shard)."""
    data = _u8(data)
    k, shard = data.shape
    par = np.zeros_like(data)
    _check(lib().orc_encode(k, shard, _p(data), _p(par)))
    return par


def decode(shards: np.ndarray, present: np.ndarray) -> np.ndarray:
    """shards: (2k, shard); present: (2k,) bool.  Returns repaired copy."""
    s = _u8(shards).copy()
    pr = np.ascontiguousarray(present, dtype=np.uint8)
    _check(lib().orc_decode(s.shape[0] // 2, s.shape[1], _p(s), _p(pr)))
    return s


def extend_square(ods: np.ndarray, k: int) -> np.ndarray:
    ods = _u8(ods).reshape(k * k, SHARE_SIZE)
    eds = np.zeros((2 * k) * (2 * k) * SHARE_SIZE, np.uint8)
    _check(lib().orc_extend_square(k, _p(ods), _p(eds)))
    return eds.reshape(2 * k, 2 * k, SHARE_SIZE)


def compute_roots(eds: np.ndarray, k: int, nthreads: int = 1):
    eds = _u8(eds)
    w = 2 * k
    rr = np.zeros((w, NODE_SIZE), np.uint8)
    cr = np.zeros((w, NODE_SIZE), np.uint8)
    _check(lib().orc_compute_roots(k, _p(eds), _p(rr), _p(cr), nthreads))
    return rr, cr


def rfc6962_root(items) -> bytes:
    out = np.zeros(32, np.uint8)
    if len(items) == 0:
        lib().orc_rfc6962_root(_p(np.zeros(1, np.uint8)), 0, 0, _p(out))
        return out.tobytes()
    ln = len(items[0])
    a = _u8(b"".join(items))
    lib().orc_rfc6962_root(_p(a), len(items), ln, _p(out))
    return out.tobytes()


def dah_hash(row_roots: np.ndarray, col_roots: np.ndarray) -> bytes:
    rr, cr = _u8(row_roots), _u8(col_roots)
    out = np.zeros(32, np.uint8)
    lib().orc_dah_hash(_p(rr), _p(cr), rr.shape[0], _p(out))
    return out.tobytes()


def extend_and_dah(ods: np.ndarray, k: int, nthreads: int = 1, want_eds: bool = True):
    """Returns (eds or None, row_roots, col_roots, dah)."""
    ods = _u8(ods).reshape(k * k, SHARE_SIZE)
    w = 2 * k
    eds = np.zeros((w, w, SHARE_SIZE), np.uint8) if want_eds else None
    rr = np.zeros((w, NODE_SIZE), np.uint8)
    cr = np.zeros((w, NODE_SIZE), np.uint8)
    dah = np.zeros(32, np.uint8)
    L = lib()
    eptr = _p(eds) if want_eds else ctypes.POINTER(ctypes.c_uint8)()
    _check(L.orc_extend_and_dah(k, _p(ods), eptr, _p(rr), _p(cr), _p(dah), nthreads))
    return eds, rr, cr, dah.tobytes()


def repair(eds: np.ndarray, present: np.ndarray, k: int, row_roots, col_roots):
    e = _u8(eds).copy()
    pr = np.ascontiguousarray(present, dtype=np.uint8).copy()
    rc = lib().orc_repair(k, _p(e), _p(pr), _p(_u8(row_roots)), _p(_u8(col_roots)))
    return rc, e


def repair_ex(eds: np.ndarray, present: np.ndarray, k: int, row_roots, col_roots):
    """orc_repair_ex: (status, eds, present, byz) with byz = [axis, index,
    rebuilt axis, rebuilt index] (-1 = none); eds/present as rsmt2d leaves them."""
    e = _u8(eds).copy()
    pr = np.ascontiguousarray(present, dtype=np.uint8).copy()
    byz = np.full(4, -1, np.int32)
    rc = lib().orc_repair_ex(k, _p(e), _p(pr), _p(_u8(row_roots)), _p(_u8(col_roots)),
                             byz.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return rc, e, pr, [int(x) for x in byz]


def nmt_leaf(ns: bytes, data: bytes) -> bytes:
    out = np.zeros(NODE_SIZE, np.uint8)
    lib().orc_nmt_leaf(_p(_u8(ns)), _p(_u8(data)), len(data), _p(out))
    return out.tobytes()


def nmt_root(leaf_nodes) -> bytes:
    out = np.zeros(NODE_SIZE, np.uint8)
    if len(leaf_nodes) == 0:
        lib().orc_nmt_root_from_leaves(_p(np.zeros(1, np.uint8)), 0, _p(out))
    else:
        a = _u8(b"".join(leaf_nodes))
        lib().orc_nmt_root_from_leaves(_p(a), len(leaf_nodes), _p(out))
    return out.tobytes()


# --- SIMD CPU baseline (da_simd.c; bench.py cpu_baseline "simd-port") ---------

def simd_lib() -> ctypes.CDLL:
    if "simd" not in _libs:
        path = os.path.join(_BUILD, "libda_simd.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.simd_isa.restype = ctypes.c_char_p
        L.simd_extend_and_dah.argtypes = [ctypes.c_int, u8p, u8p, u8p, u8p, u8p, ctypes.c_int]
        _libs["simd"] = L
    return _libs["simd"]


def simd_isa() -> str:
    return simd_lib().simd_isa().decode()


class SimdSquare:
    """Reusable buffers for simd_extend_and_dah (the EDS the Go path returns)."""

    def __init__(self, k: int):
        w = 2 * k
        self.k = k
        self.eds = np.empty((w, w, SHARE_SIZE), np.uint8)
        self.rr = np.empty((w, NODE_SIZE), np.uint8)
        self.cr = np.empty((w, NODE_SIZE), np.uint8)
        self.dah = np.empty(32, np.uint8)

    def run(self, ods: np.ndarray, nthreads: int):
        o = _u8(ods)
        _check(simd_lib().simd_extend_and_dah(self.k, _p(o), _p(self.eds), _p(self.rr), _p(self.cr),
                                              _p(self.dah), nthreads))
        return self.eds, self.rr, self.cr, self.dah.tobytes()
