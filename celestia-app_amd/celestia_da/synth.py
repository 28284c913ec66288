"""Synthetic inputs of the shape the reference benchmarks/tests use.

random_blob_square: "random-namespace blob shares" as produced by
test/util/testfactory/common.go:36-46 (GenerateRandNamespacedRawData): 512
random bytes per share, bytes [0:29] overwritten by a random blob namespace
(version 0, 18 zero bytes, 10 random bytes, not reserved --
pkg/namespace/random_blob.go:22-30), then all shares sorted bytewise.
The PRNG is numpy PCG64 with the given seed (the reference uses tmrand).

constant_square: pkg/da/data_availability_header_test.go:247-263 generateShares
(namespace MustNewV0([1]*10) followed by 0xFF*483, all shares identical).
"""
from __future__ import annotations

import numpy as np

SHARE = 512


def random_blob_square(k: int, seed: int) -> np.ndarray:
    """(k*k, 512) uint8, sorted bytewise (so every Q0 row/column is NMT-ordered)."""
    rng = np.random.default_rng(seed)
    n = k * k
    s = rng.integers(0, 256, size=(n, SHARE), dtype=np.uint8)
    s[:, 0] = 0          # namespace version 0
    s[:, 1:19] = 0       # NamespaceVersionZeroPrefix (18 zero bytes)
    # reserved iff ID <= 0x00..00FF: the first 9 of the 10 random bytes all zero
    reserved = ~s[:, 19:28].any(axis=1)
    s[reserved, 19] = 1
    return sort_shares(s)


def sort_shares(s: np.ndarray) -> np.ndarray:
    """Bytewise lexicographic sort of rows (bytes.Compare order)."""
    # big-endian 64-bit words compare like the bytes they hold; the first 8
    # words (64 bytes) decide unless two rows share them, then sort on all
    words = s.view(">u8")
    order = np.lexsort(words[:, :8].T[::-1])
    w8 = words[order, :8]
    if (w8[1:] == w8[:-1]).all(axis=1).any():
        order = np.lexsort(words.T[::-1])
    return np.ascontiguousarray(s[order])


_FAST = None


def _fast_lib():
    """libdasynth.so (csrc/synth.cpp): the multithreaded generator for large
    runs of distinct squares (block replay, the 4096-square mixed batch)."""
    global _FAST
    if _FAST is None:
        import ctypes
        import os
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "libdasynth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C celestia-app_amd` (or __graft_entry__.build())")
        lib = ctypes.CDLL(path)
        lib.dasynth_blob_squares.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
        lib.dasynth_blob_squares.restype = ctypes.c_int
        _FAST = lib
    return _FAST


def blob_squares(k: int, seed: int, first: int, count: int, out: np.ndarray = None,
                 threads: int = 0) -> np.ndarray:
    """Squares first..first+count-1 of the seeded run `seed` (random blob
    shares, sorted; see csrc/synth.cpp), as (count, k*k*512) uint8.  Square i
    is the same bytes whichever (first, count) window produces it.  `out` may
    be a caller buffer (e.g. page-locked) of at least that many bytes."""
    n = count * k * k * SHARE
    if out is None:
        out = np.empty((count, k * k * SHARE), np.uint8)
    if out.nbytes < n or not out.flags["C_CONTIGUOUS"]:
        raise ValueError("out must be a contiguous buffer of count*k*k*512 bytes")
    rc = _fast_lib().dasynth_blob_squares(k, seed, first, count, out.ctypes.data, threads)
    if rc != 0:
        raise ValueError("dasynth_blob_squares: bad argument")
    return out.reshape(-1)[:n].reshape(count, k * k * SHARE)


def constant_square(k: int) -> np.ndarray:
    ns = bytes([0]) + bytes(18) + bytes([1] * 10)
    share = ns + b"\xff" * (SHARE - len(ns))
    return np.tile(np.frombuffer(share, np.uint8), (k * k, 1))


def tail_padding_square(k: int) -> np.ndarray:
    ns = b"\xff" * 28 + b"\xfe"
    share = ns + b"\x01" + b"\x00" * 4 + b"\x00" * (SHARE - 34)
    return np.tile(np.frombuffer(share, np.uint8), (k * k, 1))


def block_txs(n_normal: int, n_blob: int, seed: int, normal_size: int = 300,
              blob_sizes=(1500, 3000), n_namespaces: int = 64):
    """A synthetic block for square construction (pkg/square): n_normal random
    txs of normal_size bytes, then n_blob BlobTx protos (pkg/blob/blob.go wire
    format) with one blob each, data sizes uniform in blob_sizes, namespaces
    drawn from n_namespaces version-0 IDs.  The PFB tx inside each BlobTx is a
    stand-in of the signed MsgPayForBlobs the reference would carry (only its
    length affects the layout): b"PFB" | 1 | varint(size), zero padded to 330 B."""
    import random

    from . import blobtx, shares
    rng = random.Random(seed)
    txs = [rng.randbytes(normal_size) for _ in range(n_normal)]
    nss = sorted(shares.new_namespace_v0(rng.randbytes(10)) for _ in range(n_namespaces))
    for i in range(n_blob):
        data = rng.randbytes(rng.randrange(blob_sizes[0], blob_sizes[1]))
        pfb = (b"PFB\x01" + shares.put_uvarint(len(data))).ljust(330, b"\x00")
        txs.append(blobtx.marshal_blob_tx(pfb, shares.Blob.new(nss[i % n_namespaces], data)))
    return txs
