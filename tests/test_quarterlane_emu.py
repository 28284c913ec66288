"""Host emulation of the round-6 quarter-lane GF(2^16) k = 512 decoder's data
movement (csrc/rs_gf16.hip leo16_decode_q_kernel): n = 1024 elements over
8 waves x 32 registers x 4 lane quarters (a lane quarter = 16 lanes = 128 B of
a shard), so a workgroup of 512 threads holds one 128-B piece of a vector and
two workgroups share a CU.  Layouts (q = wave, j = register, ql = quarter):
  S  e = (j >> 3) + 4 (j & 7) + 32 ql + 128 q   loads, stores, pre/post
                                                multiplies, layers on bits 0, 1
  B  e = ql + 4 j + 128 q                        layers on bits 2-6
  T  e = ql + 4 (j & 3) + 16 q + 128 (j >> 2)    layers on bits 7-9, derivative
S <-> B is a 4 x 4 transpose of (j >> 3, ql) per register group j & 7
(v_permlane32_swap then v_permlane16_swap), B <-> T the 8 x 8 LDS transpose of
q with j >> 2.  Checked here on one symbol column against the plain Leopard
loops (test_halflane_emu's references); the kernel itself bit-exact against
the oracle on the GPU (tests/test_gpu_gf16.py)."""
import pytest

from test_halflane_emu import SKEW, bfly, ref_derivative, ref_fft, ref_ifft  # noqa: F401

import numpy as np

NQ = 8


def e_s(q, j, ql):
    return (j >> 3) + 4 * (j & 7) + 32 * ql + 128 * q


def e_b(q, j, ql):
    return ql + 4 * j + 128 * q


def e_t(q, j, ql):
    return ql + 4 * (j & 3) + 16 * q + 128 * (j >> 2)


def permlane32_swap(a, b):
    # rows (16 lanes) 2,3 of a <-> rows 0,1 of b
    return [a[0], a[1], b[0], b[1]], [a[2], a[3], b[2], b[3]]


def permlane16_swap(a, b):
    # odd rows of a <-> even rows of b
    return [a[0], b[0], a[2], b[2]], [a[1], b[1], a[3], b[3]]


def swap_sb(R):
    """S <-> B (its own inverse): per register group g, registers g + 8u."""
    for reg in R:
        for g in range(8):
            r0, r1, r2, r3 = reg[g], reg[g + 8], reg[g + 16], reg[g + 24]
            r0, r2 = permlane32_swap(r0, r2)
            r1, r3 = permlane32_swap(r1, r3)
            r0, r1 = permlane16_swap(r0, r1)
            r2, r3 = permlane16_swap(r2, r3)
            reg[g], reg[g + 8], reg[g + 16], reg[g + 24] = r0, r1, r2, r3


def xpose_bt(R):
    """B <-> T: wave q, register (jj << 2) | r <-> wave jj, register (q << 2) | r."""
    S = [[None] * 32 for _ in range(NQ)]
    for q in range(NQ):
        for jj in range(NQ):
            for r in range(4):
                S[jj][(q << 2) | r] = list(R[q][(jj << 2) | r])
    return S


def layer_s(R, b, inv):
    """Layers on element bits 0 (registers j, j + 8) and 1 (j, j + 16) in S:
    per-lane positions (the quarter is element bits 5-6)."""
    d = 1 << b
    for q, reg in enumerate(R):
        for j in range(32):
            if (j >> 3) & d:
                continue
            for ql in range(4):
                e = e_s(q, j, ql)
                pos = (e & ~(2 * d - 1)) + d - 1
                w = [reg[j][ql], reg[j + 8 * d][ql]]
                bfly(w, 0, 1, pos, inv)
                reg[j][ql], reg[j + 8 * d][ql] = w


def layer_b(R, b, inv):
    """Layers on bits 2-6 in B: registers j, j + 2^(b-2); position from the
    register bits above and q (wave-uniform)."""
    rd = 1 << (b - 2)
    d = 1 << b
    for q, reg in enumerate(R):
        for j in range(32):
            if j & rd:
                continue
            pos = ((128 * q + 4 * j) & ~(2 * d - 1)) + d - 1
            for ql in range(4):
                assert (e_b(q, j, ql) & ~(2 * d - 1)) + d - 1 == pos
                w = [reg[j][ql], reg[j + rd][ql]]
                bfly(w, 0, 1, pos, inv)
                reg[j][ql], reg[j + rd][ql] = w


def layer_t(R, b, inv):
    """Layers on bits 7-9 in T: registers j, j + 4 * 2^(b-7); compile-time positions."""
    rd = 4 << (b - 7)
    d = 1 << b
    for q, reg in enumerate(R):
        for j in range(32):
            if j & rd:
                continue
            pos = ((128 * (j >> 2)) & ~(2 * d - 1)) + d - 1
            for ql in range(4):
                assert (e_t(q, j, ql) & ~(2 * d - 1)) + d - 1 == pos
                w = [reg[j][ql], reg[j + rd][ql]]
                bfly(w, 0, 1, pos, inv)
                reg[j][ql], reg[j + rd][ql] = w


def derivative_t(R):
    """D(x)_e = x_e ^ XOR_{s: bit s of e = 0} x_{e | 2^s}: register bits (2, 3,
    7, 8, 9) in place, wave bits (4-6) and quarter bits (0-1: lanes ^ 16, ^ 32)
    from the staged originals."""
    orig = [[list(x) for x in reg] for reg in R]
    for c, reg in enumerate(R):
        for j in range(32):
            for ql in range(4):
                acc = orig[c][j][ql]
                for bit in (1, 2, 4, 8, 16):
                    if not j & bit:
                        acc ^= orig[c][j | bit][ql]
                for wb in (1, 2, 4):
                    if not c & wb:
                        acc ^= orig[c | wb][j][ql]
                for qb in (1, 2):
                    if not ql & qb:
                        acc ^= orig[c][j][ql | qb]
                reg[j][ql] = acc


def gather(R, f):
    out = {}
    for q, reg in enumerate(R):
        for j in range(32):
            for ql in range(4):
                out[f(q, j, ql)] = reg[j][ql]
    return [out[e] for e in range(len(out))]


def test_quarter_layouts_are_bijections_and_swaps_map():
    for f in (e_s, e_b, e_t):
        assert {f(q, j, ql) for q in range(NQ) for j in range(32) for ql in range(4)} == set(range(1024))
    R = [[[e_s(q, j, ql) for ql in range(4)] for j in range(32)] for q in range(NQ)]
    swap_sb(R)
    assert all(R[q][j][ql] == e_b(q, j, ql) for q in range(NQ) for j in range(32) for ql in range(4))
    T = xpose_bt(R)
    assert all(T[q][j][ql] == e_t(q, j, ql) for q in range(NQ) for j in range(32) for ql in range(4))


@pytest.mark.parametrize("seed", [1, 2])
def test_quarterlane_decoder_equals_leopard_loops(seed):
    rng = np.random.default_rng(seed)
    n = 1024
    x = [int(v) for v in rng.integers(0, 65536, n)]
    ref = list(x)
    ref_ifft(ref, 0)
    ref_derivative(ref)
    ref_fft(ref, 0)
    R = [[[x[e_s(q, j, ql)] for ql in range(4)] for j in range(32)] for q in range(NQ)]
    layer_s(R, 0, True)
    layer_s(R, 1, True)
    swap_sb(R)
    for b in range(2, 7):
        layer_b(R, b, True)
    R = xpose_bt(R)
    for b in (7, 8, 9):
        layer_t(R, b, True)
    derivative_t(R)
    for b in (9, 8, 7):
        layer_t(R, b, False)
    R = xpose_bt(R)
    for b in range(6, 1, -1):
        layer_b(R, b, False)
    swap_sb(R)
    layer_s(R, 1, False)
    layer_s(R, 0, False)
    assert gather(R, e_s) == ref


# --- the quarter-lane k = 512 encoder (leo16_encode_q_kernel): m = 512 over 4
# waves; S and B as the decoder's, T e = ql + 4 (j & 7) + 32 q + 128 (j >> 3)
# (B <-> T: the 4 x 4 transpose of q with j >> 3, LR = 3)
NQE = 4


def e_te(q, j, ql):
    return ql + 4 * (j & 7) + 32 * q + 128 * (j >> 3)


def xpose_bt_e(R):
    S = [[None] * 32 for _ in range(NQE)]
    for q in range(NQE):
        for jj in range(NQE):
            for r in range(8):
                S[jj][(q << 3) | r] = list(R[q][(jj << 3) | r])
    return S


def layer_s_off(R, b, off, inv):
    d = 1 << b
    for q, reg in enumerate(R):
        for j in range(32):
            if (j >> 3) & d:
                continue
            for ql in range(4):
                e = e_s(q, j, ql)
                w = [reg[j][ql], reg[j + 8 * d][ql]]
                bfly(w, 0, 1, off + (e & ~(2 * d - 1)) + d - 1, inv)
                reg[j][ql], reg[j + 8 * d][ql] = w


def layer_b_off(R, b, off, inv):
    rd, d = 1 << (b - 2), 1 << b
    for q, reg in enumerate(R):
        for jb in range(0, 32, 2 * rd):
            pos = off + 128 * q + 4 * jb + d - 1
            for j in range(jb, jb + rd):
                for ql in range(4):
                    assert off + (e_b(q, j, ql) & ~(2 * d - 1)) + d - 1 == pos
                    w = [reg[j][ql], reg[j + rd][ql]]
                    bfly(w, 0, 1, pos, inv)
                    reg[j][ql], reg[j + rd][ql] = w


def layer_te(R, b, off, inv):
    """bits 7, 8 in T: registers j, j + 8 << (b - 7); position off + 128 (jb >> 3) + d - 1"""
    rd, d = 8 << (b - 7), 1 << b
    for q, reg in enumerate(R):
        for jb in range(0, 32, 2 * rd):
            pos = off + 128 * (jb >> 3) + d - 1
            for j in range(jb, jb + rd):
                for ql in range(4):
                    assert off + (e_te(q, j, ql) & ~(2 * d - 1)) + d - 1 == pos
                    w = [reg[j][ql], reg[j + rd][ql]]
                    bfly(w, 0, 1, pos, inv)
                    reg[j][ql], reg[j + rd][ql] = w


@pytest.mark.parametrize("rev", [False, True])
def test_quarterlane_encoder_equals_leopard_loops(rev):
    rng = np.random.default_rng(11 + rev)
    m = 512
    io, fo = (0, m) if rev else (m, 0)
    x = [int(v) for v in rng.integers(0, 65536, m)]
    ref = list(x)
    ref_ifft(ref, io)
    ref_fft(ref, fo)
    R = [[[x[e_s(q, j, ql)] for ql in range(4)] for j in range(32)] for q in range(NQE)]
    layer_s_off(R, 0, io, True)
    layer_s_off(R, 1, io, True)
    swap_sb(R)
    for b in range(2, 7):
        layer_b_off(R, b, io, True)
    R = xpose_bt_e(R)
    layer_te(R, 7, io, True)
    layer_te(R, 8, io, True)  # (merged with the next in the kernel)
    layer_te(R, 8, fo, False)
    layer_te(R, 7, fo, False)
    R = xpose_bt_e(R)
    for b in range(6, 1, -1):
        layer_b_off(R, b, fo, False)
    swap_sb(R)
    layer_s_off(R, 1, fo, False)
    layer_s_off(R, 0, fo, False)
    got = []
    for e in range(m):
        q, j, ql = _inv_s(e)
        got.append(R[q][j][ql])
    assert got == ref


def _inv_s(e):
    return e >> 7, (e & 3) * 8 + ((e >> 2) & 7), (e >> 5) & 3


def test_encoder_layout_bijections():
    assert {e_te(q, j, ql) for q in range(NQE) for j in range(32) for ql in range(4)} == set(range(512))
    assert all(e_s(*_inv_s(e)) == e for e in range(512))
    R = [[[e_b(q, j, ql) for ql in range(4)] for j in range(32)] for q in range(NQE)]
    T = xpose_bt_e(R)
    assert all(T[q][j][ql] == e_te(q, j, ql) for q in range(NQE) for j in range(32) for ql in range(4))


# --- k = 256 (n = 512) through the same decoder template: 4 waves, T as the
# encoder's (LR = 3: e = ql + 4 (j & 7) + 32 q + 128 (j >> 3)), layers on bits 7-8
def derivative_te(R):
    orig = [[list(x) for x in reg] for reg in R]
    for c, reg in enumerate(R):
        for j in range(32):
            for ql in range(4):
                acc = orig[c][j][ql]
                for bit in (1, 2, 4, 8, 16):
                    if not j & bit:
                        acc ^= orig[c][j | bit][ql]
                for wb in (1, 2):
                    if not c & wb:
                        acc ^= orig[c | wb][j][ql]
                for qb in (1, 2):
                    if not ql & qb:
                        acc ^= orig[c][j][ql | qb]
                reg[j][ql] = acc


@pytest.mark.parametrize("seed", [3, 4])
def test_quarterlane_decoder_k256_equals_leopard_loops(seed):
    rng = np.random.default_rng(seed)
    n = 512
    x = [int(v) for v in rng.integers(0, 65536, n)]
    ref = list(x)
    ref_ifft(ref, 0)
    ref_derivative(ref)
    ref_fft(ref, 0)
    R = [[[x[e_s(q, j, ql)] for ql in range(4)] for j in range(32)] for q in range(NQE)]
    layer_s_off(R, 0, 0, True)
    layer_s_off(R, 1, 0, True)
    swap_sb(R)
    for b in range(2, 7):
        layer_b_off(R, b, 0, True)
    R = xpose_bt_e(R)
    layer_te(R, 7, 0, True)
    layer_te(R, 8, 0, True)
    derivative_te(R)
    layer_te(R, 8, 0, False)
    layer_te(R, 7, 0, False)
    R = xpose_bt_e(R)
    for b in range(6, 1, -1):
        layer_b_off(R, b, 0, False)
    swap_sb(R)
    layer_s_off(R, 1, 0, False)
    layer_s_off(R, 0, 0, False)
    got = []
    for e in range(n):
        q, j, ql = _inv_s(e)
        got.append(R[q][j][ql])
    assert got == ref


# --- k = 1024 (n = 2048) through the same decoder template: 16 waves (1,024
# threads, one workgroup per CU), T e = ql + 4 (j & 1) + 8 q + 128 (j >> 1)
# (B <-> T: the 16 x 16 transpose of q with j >> 1, LR = 1), layers on bits 7-10
NQ1K = 16


def e_t1k(q, j, ql):
    return ql + 4 * (j & 1) + 8 * q + 128 * (j >> 1)


def xpose_bt_1k(R):
    S = [[None] * 32 for _ in range(NQ1K)]
    for q in range(NQ1K):
        for jj in range(NQ1K):
            for r in range(2):
                S[jj][(q << 1) | r] = list(R[q][(jj << 1) | r])
    return S


def layer_t1k(R, b, inv):
    """bits 7-10 in T: registers j, j + 2 << (b - 7); position 128 (jb >> 1) + d - 1"""
    rd, d = 2 << (b - 7), 1 << b
    for q, reg in enumerate(R):
        for jb in range(0, 32, 2 * rd):
            pos = 128 * (jb >> 1) + d - 1
            for j in range(jb, jb + rd):
                for ql in range(4):
                    assert (e_t1k(q, j, ql) & ~(2 * d - 1)) + d - 1 == pos
                    w = [reg[j][ql], reg[j + rd][ql]]
                    bfly(w, 0, 1, pos, inv)
                    reg[j][ql], reg[j + rd][ql] = w


def derivative_t1k(R):
    orig = [[list(x) for x in reg] for reg in R]
    for c, reg in enumerate(R):
        for j in range(32):
            for ql in range(4):
                acc = orig[c][j][ql]
                for bit in (1, 2, 4, 8, 16):
                    if not j & bit:
                        acc ^= orig[c][j | bit][ql]
                for wb in (1, 2, 4, 8):
                    if not c & wb:
                        acc ^= orig[c | wb][j][ql]
                for qb in (1, 2):
                    if not ql & qb:
                        acc ^= orig[c][j][ql | qb]
                reg[j][ql] = acc


def test_k1024_layout_bijections():
    assert {e_t1k(q, j, ql) for q in range(NQ1K) for j in range(32) for ql in range(4)} == set(range(2048))
    assert {e_s(q, j, ql) for q in range(NQ1K) for j in range(32) for ql in range(4)} == set(range(2048))
    R = [[[e_b(q, j, ql) for ql in range(4)] for j in range(32)] for q in range(NQ1K)]
    T = xpose_bt_1k(R)
    assert all(T[q][j][ql] == e_t1k(q, j, ql) for q in range(NQ1K) for j in range(32) for ql in range(4))


def test_quarterlane_decoder_k1024_equals_leopard_loops():
    rng = np.random.default_rng(21)
    n = 2048
    x = [int(v) for v in rng.integers(0, 65536, n)]
    ref = list(x)
    ref_ifft(ref, 0)
    ref_derivative(ref)
    ref_fft(ref, 0)
    R = [[[x[e_s(q, j, ql)] for ql in range(4)] for j in range(32)] for q in range(NQ1K)]
    layer_s_off(R, 0, 0, True)
    layer_s_off(R, 1, 0, True)
    swap_sb(R)
    for b in range(2, 7):
        layer_b_off(R, b, 0, True)
    R = xpose_bt_1k(R)
    for b in (7, 8, 9, 10):
        layer_t1k(R, b, True)
    derivative_t1k(R)
    for b in (10, 9, 8, 7):
        layer_t1k(R, b, False)
    R = xpose_bt_1k(R)
    for b in range(6, 1, -1):
        layer_b_off(R, b, 0, False)
    swap_sb(R)
    layer_s_off(R, 1, 0, False)
    layer_s_off(R, 0, 0, False)
    got = []
    for e in range(n):
        q, j, ql = _inv_s(e)
        got.append(R[q][j][ql])
    assert got == ref


# --- the k = 1024 encoder (leo16_encode_q_kernel<1024>): m = 1024 over 8 waves,
# T as the k = 512 decoder's (LR = 2), layers on bits 7, 8 and the merged bit 9
def layer_te2(R, b, off, inv):
    rd, d = 4 << (b - 7), 1 << b
    for q, reg in enumerate(R):
        for jb in range(0, 32, 2 * rd):
            pos = off + 128 * (jb >> 2) + d - 1
            for j in range(jb, jb + rd):
                for ql in range(4):
                    assert off + (e_t(q, j, ql) & ~(2 * d - 1)) + d - 1 == pos
                    w = [reg[j][ql], reg[j + rd][ql]]
                    bfly(w, 0, 1, pos, inv)
                    reg[j][ql], reg[j + rd][ql] = w


@pytest.mark.parametrize("rev", [False, True])
def test_quarterlane_encoder_m1024_equals_leopard_loops(rev):
    rng = np.random.default_rng(31 + rev)
    m = 1024
    io, fo = (0, m) if rev else (m, 0)
    x = [int(v) for v in rng.integers(0, 65536, m)]
    ref = list(x)
    ref_ifft(ref, io)
    ref_fft(ref, fo)
    R = [[[x[e_s(q, j, ql)] for ql in range(4)] for j in range(32)] for q in range(NQ)]
    layer_s_off(R, 0, io, True)
    layer_s_off(R, 1, io, True)
    swap_sb(R)
    for b in range(2, 7):
        layer_b_off(R, b, io, True)
    R = xpose_bt(R)
    for b in (7, 8, 9):
        layer_te2(R, b, io, True)
    for b in (9, 8, 7):  # (bit 9 merged with the IFFT's in the kernel: registers j, j + 16)
        layer_te2(R, b, fo, False)
    R = xpose_bt(R)
    for b in range(6, 1, -1):
        layer_b_off(R, b, fo, False)
    swap_sb(R)
    layer_s_off(R, 1, fo, False)
    layer_s_off(R, 0, fo, False)
    got = []
    for e in range(m):
        q, j, ql = _inv_s(e)
        got.append(R[q][j][ql])
    assert got == ref


# --- the k = 2048 encoder (leo16_encode_q_kernel<2048>): m = 2048 over 16
# waves, T as the k = 1024 decoder's (LR = 1), layers on bits 7-9 and the merged bit 10
def layer_t1k_off(R, b, off, inv):
    rd, d = 2 << (b - 7), 1 << b
    for q, reg in enumerate(R):
        for jb in range(0, 32, 2 * rd):
            pos = off + 128 * (jb >> 1) + d - 1
            for j in range(jb, jb + rd):
                for ql in range(4):
                    assert off + (e_t1k(q, j, ql) & ~(2 * d - 1)) + d - 1 == pos
                    w = [reg[j][ql], reg[j + rd][ql]]
                    bfly(w, 0, 1, pos, inv)
                    reg[j][ql], reg[j + rd][ql] = w


@pytest.mark.parametrize("rev", [False, True])
def test_quarterlane_encoder_m2048_equals_leopard_loops(rev):
    rng = np.random.default_rng(41 + rev)
    m = 2048
    io, fo = (0, m) if rev else (m, 0)
    x = [int(v) for v in rng.integers(0, 65536, m)]
    ref = list(x)
    ref_ifft(ref, io)
    ref_fft(ref, fo)
    R = [[[x[e_s(q, j, ql)] for ql in range(4)] for j in range(32)] for q in range(NQ1K)]
    layer_s_off(R, 0, io, True)
    layer_s_off(R, 1, io, True)
    swap_sb(R)
    for b in range(2, 7):
        layer_b_off(R, b, io, True)
    R = xpose_bt_1k(R)
    for b in (7, 8, 9, 10):
        layer_t1k_off(R, b, io, True)
    for b in (10, 9, 8, 7):  # (bit 10 merged with the IFFT's in the kernel: registers j, j + 16)
        layer_t1k_off(R, b, fo, False)
    R = xpose_bt_1k(R)
    for b in range(6, 1, -1):
        layer_b_off(R, b, fo, False)
    swap_sb(R)
    layer_s_off(R, 1, fo, False)
    layer_s_off(R, 0, fo, False)
    got = []
    for e in range(m):
        q, j, ql = _inv_s(e)
        got.append(R[q][j][ql])
    assert got == ref
