"""The bit-sliced GF(2^8) encode (csrc/leo8_sliced.hpp + rs_gf8_sliced.hip)
checked on the CPU: tests/emu/sliced_emu.hip runs the kernel's own per-lane
transform code on the host, with the workgroup's loads, LDS layout exchanges
and stores as plain loops, against the oracle's Leopard encode
(oracle/da_oracle.c, pinned to the reference's golden vectors)."""
import ctypes
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import oracle  # noqa: E402

EMU = os.path.join(os.path.dirname(__file__), "emu", "libsliced_emu.so")


@pytest.fixture(scope="module")
def emu():
    if not os.path.exists(EMU):
        pytest.skip("emulator not built (make -C celestia-app_amd emu)")
    L = ctypes.CDLL(EMU)
    L.sliced_emu_encode.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p]
    L.sliced2_emu_encode.argtypes = [ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p]
    L.sliced_emu_bop3.restype = ctypes.c_uint32
    L.sliced_emu_bop3.argtypes = [ctypes.c_uint32] * 3 + [ctypes.c_int]
    return L


def test_bitop3_truth_tables(emu):
    # v_bitop3_b32: S0 = 0xF0, S1 = 0xCC, S2 = 0xAA (LLVM's encoding for gfx950)
    for tt in (0x96, 0x78, 0xB4, 0x28):
        assert emu.sliced_emu_bop3(0xF0F0F0F0, 0xCCCCCCCC, 0xAAAAAAAA, tt) == tt * 0x01010101


@pytest.mark.parametrize("k", [16, 32, 64, 128])
@pytest.mark.parametrize("shard", [512, 1024])
def test_sliced_encode_matches_oracle(emu, k, shard):
    rng = np.random.default_rng(k * 7 + shard)
    data = rng.integers(0, 256, (k, shard), dtype=np.uint8)
    parity = np.zeros_like(data)
    assert emu.sliced_emu_encode(k, shard, data.ctypes.data, parity.ctypes.data) == 0
    assert np.array_equal(parity, oracle.encode(data))


@pytest.mark.parametrize("k", [16, 128])
def test_sliced_encode_structured_inputs(emu, k):
    """Zero, constant and single-bit data (each bit of each element alone)."""
    shard = 512
    cases = [np.zeros((k, shard), np.uint8), np.full((k, shard), 0xFF, np.uint8)]
    one = np.zeros((k, shard), np.uint8)
    for e in range(0, k, max(1, k // 8)):
        for bit in range(8):
            one[e, (e * 8 + bit) * 3 % shard] |= 1 << bit
    cases.append(one)
    for data in cases:
        parity = np.zeros_like(data)
        emu.sliced_emu_encode(k, shard, data.ctypes.data, parity.ctypes.data)
        assert np.array_equal(parity, oracle.encode(data))


def test_sliced_rejects_unsupported(emu):
    buf = np.zeros((8, 512), np.uint8)
    assert emu.sliced_emu_encode(8, 512, buf.ctypes.data, buf.ctypes.data) == -1
    assert emu.sliced_emu_encode(16, 100, buf.ctypes.data, buf.ctypes.data) == -1


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_sliced2_encode_matches_oracle(emu, seed):
    """The two-vector k = 128 layout (lane element bit, wave-bit branches;
    leo8_encode_sliced2_kernel) on random and structured data."""
    k, shard = 128, 512 * (1 + seed % 2)
    rng = np.random.default_rng(900 + seed)
    cases = [rng.integers(0, 256, (k, shard), dtype=np.uint8)]
    if seed == 0:
        one = np.zeros((k, shard), np.uint8)
        for e in range(k):
            one[e, (e * 5) % shard] = 1 << (e % 8)
        cases += [one, np.full((k, shard), 0xFF, np.uint8)]
    for data in cases:
        parity = np.zeros_like(data)
        assert emu.sliced2_emu_encode(shard, data.ctypes.data, parity.ctypes.data) == 0
        assert np.array_equal(parity, oracle.encode(data))


def _dec_case(rng, shard, npresent):
    k = 128
    data = rng.integers(0, 256, (k, shard), dtype=np.uint8)
    full = np.concatenate([data, oracle.encode(data)])
    present = np.zeros(2 * k, np.uint8)
    present[rng.choice(2 * k, npresent, replace=False)] = 1
    return full, present


@pytest.mark.parametrize("seed,npresent", [(0, 128), (1, 128), (2, 129), (3, 200), (4, 255)])
def test_sliced_decode_matches_oracle(emu, seed, npresent):
    """The bit-sliced k = 128 decoder (rs_decode_sliced.hip: power-basis
    error-locator multiplies, layouts A/B with two lane element bits, formal
    derivative through the LDS originals) rebuilds every erased shard exactly
    as the oracle's Leopard reconstruct does."""
    emu.sliced_dec_emu.argtypes = [ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p]
    rng = np.random.default_rng(4000 + seed)
    shard = 512 * (1 + seed % 2)
    full, present = _dec_case(rng, shard, npresent)
    damaged = full * present[:, None]
    want = oracle.decode(damaged, present.astype(bool))
    assert np.array_equal(want, full)
    got = damaged.copy()
    assert emu.sliced_dec_emu(shard, got.ctypes.data, present.ctypes.data) == 0
    assert np.array_equal(got, full)


def test_sliced_decode_structured_patterns(emu):
    """Maximal erasure of the data half, of the parity half, and of every
    other shard."""
    emu.sliced_dec_emu.argtypes = [ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p]
    rng = np.random.default_rng(77)
    k, shard = 128, 512
    data = rng.integers(0, 256, (k, shard), dtype=np.uint8)
    full = np.concatenate([data, oracle.encode(data)])
    for present in (np.r_[np.zeros(k), np.ones(k)], np.r_[np.ones(k), np.zeros(k)],
                    np.tile([1, 0], k)):
        present = present.astype(np.uint8)
        got = full * present[:, None]
        assert emu.sliced_dec_emu(shard, got.ctypes.data, present.ctypes.data) == 0
        assert np.array_equal(got, full)


@pytest.mark.parametrize("seed", [0, 1])
def test_sliced2_reverse_fill_matches_oracle_decode(emu, seed):
    """The Repair reverse fill (leo8_encode_sliced2_kernel<true, true>: IFFT
    at skew offset 0, FFT at offset k) rebuilds the data
    half from a complete parity half exactly as the oracle's Leopard
    reconstruct does with the whole data half erased."""
    emu.sliced2_emu_reverse.argtypes = [ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p]
    k, shard = 128, 512 * (1 + seed)
    rng = np.random.default_rng(5100 + seed)
    cases = [rng.integers(0, 256, (k, shard), dtype=np.uint8)]
    if seed == 0:
        cases += [np.full((k, shard), 0xFF, np.uint8), np.zeros((k, shard), np.uint8)]
    for data in cases:
        parity = oracle.encode(data)
        full = np.concatenate([data, parity])
        present = np.r_[np.zeros(k), np.ones(k)].astype(bool)
        assert np.array_equal(oracle.decode(full * present[:, None], present)[:k], data)
        got = np.zeros_like(data)
        assert emu.sliced2_emu_reverse(shard, parity.ctypes.data, got.ctypes.data) == 0
        assert np.array_equal(got, data)
