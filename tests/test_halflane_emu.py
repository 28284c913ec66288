"""Host emulation of the round-5 half-lane GF(2^16) kernels' data movement
(csrc/rs_gf16.hip leo16_decode_h1k_kernel, k = 512 decode over n = 1024
elements, and leo16_encode_h_kernel, k = 512 encode over m = 512): the same
layouts S / B / T (two elements per register, one per half wave), the
permlane32 swap S <-> B, the LDS transpose B <-> T, the skew position of
every butterfly, the closed-form formal derivative with its half-bit term and
the merged last-IFFT / first-FFT encoder layer (k = 256 too: n = 512 decode, m = 256
encode) -- on one symbol column, against
the plain Leopard loops (klauspost/reedsolomon v1.11.8 leopard.go
ifftDITDecoder / ifftDITEncoder, formalDerivative, fftDIT; SURVEY.md Appendix
A.5-A.6).  The field arithmetic is the same on every symbol column, so one
column pins the index mapping; the kernels themselves are checked bit-exact
against the oracle on the GPU (tests/test_gpu_gf16.py)."""
import numpy as np
import pytest

MOD = 65535


def _tables():
    # leopard.go initLUTs / initFFTSkew for GF(2^16) (as csrc/gf16_host.hpp)
    cantor = [0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
              0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E]
    exp = np.zeros(65536, np.int64)
    log = np.zeros(65536, np.int64)
    state = 1
    for i in range(MOD):
        exp[state] = i
        state <<= 1
        if state >= 65536:
            state ^= 0x1002D
    exp[0] = MOD
    log[0] = 0
    for i in range(16):
        width = 1 << i
        log[width:2 * width] = log[:width] ^ cantor[i]
    log = exp[log]
    exp2 = np.zeros(65536, np.int64)
    exp2[log] = np.arange(65536)
    exp2[MOD] = exp2[0]
    exp = exp2

    def add_mod(a, b):
        s = a + b
        return (s + (s >> 16)) & 0xFFFF

    def mullog(a, lb):
        return 0 if a == 0 else int(exp[add_mod(int(log[a]), lb)])

    skew = np.zeros(65536, np.int64)
    temp = [1 << i for i in range(1, 16)]
    for m in range(15):
        step = 1 << (m + 1)
        skew[(1 << m) - 1] = 0
        for i in range(m, 15):
            s = 1 << (i + 1)
            for j in range((1 << m) - 1, s, step):
                skew[j + s] = skew[j] ^ temp[i]
        temp[m] = MOD - int(log[mullog(temp[m], int(log[temp[m] ^ 1]))])
        for i in range(m + 1, 15):
            temp[i] = mullog(temp[i], add_mod(int(log[temp[i] ^ 1]), temp[m]))
    skew[:MOD] = log[skew[:MOD]]
    return log, exp, skew


LOG, EXP, SKEW = _tables()


def mul(a: int, lm: int) -> int:
    if a == 0:
        return 0
    s = int(LOG[a]) + lm
    return int(EXP[(s + (s >> 16)) & 0xFFFF])


def bfly(w, i, j, pos, inv):
    lm = int(SKEW[pos])
    if inv:  # ifftDIT2: y ^= x; x ^= y * skew
        w[j] ^= w[i]
        if lm != MOD:
            w[i] ^= mul(w[j], lm)
    else:  # fftDIT2: x ^= y * skew; y ^= x
        if lm != MOD:
            w[i] ^= mul(w[j], lm)
        w[j] ^= w[i]


def ref_ifft(w, off):
    """ifftDITDecoder (off = 0) / ifftDITEncoder (off = m), radix-2 layers:
    butterfly (e, e + d) at skew index off + block start + d - 1."""
    n = len(w)
    d = 1
    while d < n:
        for r in range(0, n, 2 * d):
            for i in range(r, r + d):
                bfly(w, i, i + d, off + r + d - 1, True)
        d *= 2


def ref_fft(w, off):
    n = len(w)
    d = n // 2
    while d >= 1:
        for r in range(0, n, 2 * d):
            for i in range(r, r + d):
                bfly(w, i, i + d, off + r + d - 1, False)
        d //= 2


def ref_derivative(w):  # leopard.go formalDerivative
    n = len(w)
    for i in range(1, n):
        width = ((i ^ (i - 1)) + 1) >> 1
        for t in range(width):
            w[i - width + t] ^= w[i + t]


# --- the half-lane kernels' layouts: R[q][j][hl] ---
def e_s(q, j, hl):
    return 64 * q + 2 * (j & 15) + (j >> 4) + 32 * hl


def e_b(q, j, hl):
    return 64 * q + 2 * j + hl


def e_t(q, j, hl, lr):
    return hl | (j & ((1 << lr) - 1)) << 1 | q << (lr + 1) | (j >> lr) << 6


def swap_sb(R):
    for reg in R:
        for j in range(16):
            a, b = reg[j], reg[j + 16]
            reg[j], reg[j + 16] = [a[0], b[0]], [a[1], b[1]]


def xpose_bt(R, lr):
    nq = len(R)
    S = [[[None, None] for _ in range(32)] for _ in range(nq)]
    for q in range(nq):
        for jj in range(nq):
            for r in range(1 << lr):
                S[jj][(q << lr) | r] = list(R[q][(jj << lr) | r])
    return S


def layer0_s(R, off, inv):
    for q, reg in enumerate(R):
        for j in range(16):
            for hl in range(2):
                pos = off + 64 * q + 2 * j + 32 * hl
                w = [reg[j][hl], reg[j + 16][hl]]
                bfly(w, 0, 1, pos, inv)
                reg[j][hl], reg[j + 16][hl] = w


def layer_b(R, d, off, inv):
    rd = d // 2
    for q, reg in enumerate(R):
        for r in range(0, 64, 2 * d):
            pos = off + 64 * q + r + d - 1
            for e in range(r, r + d, 2):
                for hl in range(2):
                    w = [reg[e // 2][hl], reg[e // 2 + rd][hl]]
                    bfly(w, 0, 1, pos, inv)
                    reg[e // 2][hl], reg[e // 2 + rd][hl] = w


def layer_t(R, d, lr, off, inv):
    rd = (d // 64) << lr
    n = 64 << (5 - lr)
    for reg in R:
        for blk in range(0, n, 2 * d):
            for j in range(32):
                if j & rd or (((j >> lr) << 6) & ~(2 * d - 1)) != blk:
                    continue
                for hl in range(2):
                    w = [reg[j][hl], reg[j + rd][hl]]
                    bfly(w, 0, 1, off + blk + d - 1, inv)
                    reg[j][hl], reg[j + rd][hl] = w


def derivative_t(R, lr):
    orig = [[list(x) for x in reg] for reg in R]
    nq = len(R)
    for c, reg in enumerate(R):
        for j in range(32):
            for hl in range(2):
                acc = orig[c][j][hl]
                for bit in (1, 2, 4, 8, 16):
                    if not j & bit:
                        acc ^= orig[c][j | bit][hl]
                for wb in (1, 2, 4, 8):
                    if wb < nq and not c & wb:
                        acc ^= orig[c | wb][j][hl]
                if hl == 0:
                    acc ^= orig[c][j][1]
                reg[j][hl] = acc


def gather(R, f):
    out = {}
    for q, reg in enumerate(R):
        for j in range(32):
            for hl in range(2):
                out[f(q, j, hl)] = reg[j][hl]
    return [out[e] for e in range(len(out))]


def test_layout_maps_are_bijections():
    for nq, lr in ((16, 1), (8, 2), (4, 3)):
        n = 64 * nq
        for f in (e_s, e_b, lambda q, j, hl: e_t(q, j, hl, lr)):
            es = {f(q, j, hl) for q in range(nq) for j in range(32) for hl in range(2)}
            assert es == set(range(n))


@pytest.mark.parametrize("k,seed", [(512, 1), (512, 2), (256, 3)])
def test_halflane_decoder_equals_leopard_loops(k, seed):
    rng = np.random.default_rng(seed)
    n = 2 * k
    nq, lr = n // 64, (1 if n == 1024 else 2)
    x = [int(v) for v in rng.integers(0, 65536, n)]
    ref = list(x)
    ref_ifft(ref, 0)
    ref_derivative(ref)
    ref_fft(ref, 0)
    # kernel order: load in S, IFFT bit 0 in S, swap to B, bits 1-5, transpose
    # to T, bits 6.., derivative, FFT .. 6, transpose, 5-1, swap, bit 0
    R = [[[x[e_s(q, j, 0)], x[e_s(q, j, 1)]] for j in range(32)] for q in range(nq)]
    layer0_s(R, 0, True)
    swap_sb(R)
    for d in (2, 4, 8, 16, 32):
        layer_b(R, d, 0, True)
    R = xpose_bt(R, lr)
    tds = [d for d in (64, 128, 256, 512) if d < n]
    for d in tds:
        layer_t(R, d, lr, 0, True)
    derivative_t(R, lr)
    for d in reversed(tds):
        layer_t(R, d, lr, 0, False)
    R = xpose_bt(R, lr)
    for d in (32, 16, 8, 4, 2):
        layer_b(R, d, 0, False)
    swap_sb(R)
    layer0_s(R, 0, False)
    assert gather(R, e_s) == ref


@pytest.mark.parametrize("m,rev", [(512, False), (512, True), (256, False), (256, True)])
def test_halflane_encoder_equals_leopard_loops(m, rev):
    rng = np.random.default_rng(7 + rev + m)
    nq, lr = m // 64, (2 if m == 512 else 3)
    io, fo = (0, m) if rev else (m, 0)
    x = [int(v) for v in rng.integers(0, 65536, m)]
    ref = list(x)
    ref_ifft(ref, io)
    ref_fft(ref, fo)
    R = [[[x[e_s(q, j, 0)], x[e_s(q, j, 1)]] for j in range(32)] for q in range(nq)]
    layer0_s(R, io, True)
    swap_sb(R)
    for d in (2, 4, 8, 16, 32):
        layer_b(R, d, io, True)
    R = xpose_bt(R, lr)
    tds = [d for d in (64, 128) if d < m // 2]
    for d in tds:
        layer_t(R, d, lr, io, True)
    # merged dist-m/2 layers (registers j, j + 16 in T): y ^= x; x ^= y (A ^ B); y ^= x
    h = m // 2
    a, b = int(SKEW[io + h - 1]), int(SKEW[fo + h - 1])
    for reg in R:
        for j in range(16):
            for hl in range(2):
                xx, yy = reg[j][hl], reg[j + 16][hl]
                yy ^= xx
                xx ^= (mul(yy, a) if a != MOD else 0) ^ (mul(yy, b) if b != MOD else 0)
                yy ^= xx
                reg[j][hl], reg[j + 16][hl] = xx, yy
    for d in reversed(tds):
        layer_t(R, d, lr, fo, False)
    R = xpose_bt(R, lr)
    for d in (32, 16, 8, 4, 2):
        layer_b(R, d, fo, False)
    swap_sb(R)
    layer0_s(R, fo, False)
    assert gather(R, e_s) == ref


# ---- the decoders' per-element 3/3/2 product table (mul16x_table_to) --------

def perm(hi: int, lo: int, sel: int) -> int:
    """v_perm_b32 (__builtin_amdgcn_perm(hi, lo, sel)): selector byte 0-3 picks
    a byte of lo, 4-7 of hi, 0x0C gives 0x00 (the only other value used)."""
    src = lo | (hi << 32)
    out = 0
    for i in range(4):
        s = (sel >> (8 * i)) & 0xFF
        b = 0 if s == 0x0C else (src >> (8 * s)) & 0xFF
        assert s <= 7 or s == 0x0C
        out |= b << (8 * i)
    return out


def table332_device(lm: int):
    """mul16x_table_to: the 16 products (1 << b) * exp(lm), then each group's
    entries by XOR and v_perm byte packing."""
    pb = [mul(1 << b, lm) for b in range(16)]
    t = [0] * 20

    def quad(p0, p1):
        q = p0 ^ p1
        lo = perm(q, perm(p1, p0, 0x0C04000C), 0x04020100)
        hi = perm(q, perm(p1, p0, 0x0C05010C), 0x05020100)
        return lo, hi

    def grp3(b0, base):
        lo, hi = quad(pb[b0], pb[b0 + 1])
        t[base] = lo
        t[base + 1] = lo ^ perm(pb[b0 + 2], pb[b0 + 2], 0x00000000)
        t[base + 2] = hi
        t[base + 3] = hi ^ perm(pb[b0 + 2], pb[b0 + 2], 0x01010101)

    def grp2(b0, base):
        t[base], t[base + 1] = quad(pb[b0], pb[b0 + 1])

    grp3(0, 0)
    grp3(3, 4)
    grp2(6, 8)
    grp3(8, 10)
    grp3(11, 14)
    grp2(14, 18)
    return t


def table332_host(lm: int):
    """The host builder's definition (ensure_tables tab332): entry e2 of group g
    = (e2 << shift) * c, low byte in the lo pool, high byte in the hi pool."""
    t = [0] * 20
    shift, width, base = [0, 3, 6, 8, 11, 14], [3, 3, 2, 3, 3, 2], [0, 4, 8, 10, 14, 18]
    for g in range(6):
        for e2 in range(1, 1 << width[g]):
            prod = mul(e2 << shift[g], lm)
            lo_dw = base[g] + (e2 >> 2) if width[g] == 3 else base[g]
            hi_dw = base[g] + 2 + (e2 >> 2) if width[g] == 3 else base[g] + 1
            t[lo_dw] |= (prod & 0xFF) << (8 * (e2 & 3))
            t[hi_dw] |= ((prod >> 8) & 0xFF) << (8 * (e2 & 3))
    return t


def mul16x(ylo: int, yhi: int, t):
    """mul16x_add_t with zero accumulators (mul16x_by) on 4 symbols: symbol i =
    byte i of ylo (low) | byte i of yhi (high)."""
    s = [ylo & 0x07070707, (ylo >> 3) & 0x07070707, (ylo >> 6) & 0x03030303,
         yhi & 0x07070707, (yhi >> 3) & 0x07070707, (yhi >> 6) & 0x03030303]
    lo = (perm(t[1], t[0], s[0]) ^ perm(t[5], t[4], s[1]) ^ perm(t[8], t[8], s[2]) ^
          perm(t[11], t[10], s[3]) ^ perm(t[15], t[14], s[4]) ^ perm(t[18], t[18], s[5]))
    hi = (perm(t[3], t[2], s[0]) ^ perm(t[7], t[6], s[1]) ^ perm(t[9], t[9], s[2]) ^
          perm(t[13], t[12], s[3]) ^ perm(t[17], t[16], s[4]) ^ perm(t[19], t[19], s[5]))
    return lo, hi


@pytest.mark.parametrize("lm", [0, 1, 2, 255, 256, 4097, 40000, 65534])
def test_device_table332_equals_host_definition(lm):
    rng = np.random.default_rng(lm)
    t = table332_device(lm)
    assert t == table332_host(lm)
    for _ in range(64):
        syms = [int(x) for x in rng.integers(0, 65536, 4)]
        ylo = sum((v & 0xFF) << (8 * i) for i, v in enumerate(syms))
        yhi = sum((v >> 8) << (8 * i) for i, v in enumerate(syms))
        lo, hi = mul16x(ylo, yhi, t)
        got = [((lo >> (8 * i)) & 0xFF) | (((hi >> (8 * i)) & 0xFF) << 8) for i in range(4)]
        assert got == [mul(v, lm) for v in syms]


@pytest.mark.parametrize("nq,threads,off", [(16, 1024, 0), (8, 512, 0), (8, 512, 512), (4, 256, 256)])
def test_lds_position_tables_map(nq, threads, off):
    """Round 6: the bit-0 layers read their tables from an LDS image instead of
    the constant tables.  The image holds position OFF + 2 i at i x 80 B; its
    global_load_lds fills (cooperative: pos_tables_to_lds, chunk c = i x
    threads + 64 q + lane; per wave: pos_tables_wave, chunks 160 q ..) copy
    16-B chunk c of table c // 5 to LDS byte 16 c, and layer0_sl reads table
    32 q + j + 16 hl for the pair (j, j + 16) of half hl -- the position
    layer0_s computes, OFF + 64 q + 2 j + 32 hl."""
    tab = 80
    ntab = nq * 32
    image = {}
    for c0 in range(0, 5 * ntab, 64):  # cooperative fill, wave-linear
        for lane in range(64):
            c = c0 + lane
            src = (off + 2 * (c // 5)) * tab + (c % 5) * 16
            image[16 * c] = src
    for q in range(nq):  # per-wave fill covers the same chunks
        for i in range(3):
            for lane in range(64 if i < 2 else 32):
                c = 160 * q + 64 * i + lane
                assert image[16 * c] == (off + 2 * (c // 5)) * tab + (c % 5) * 16
    for q in range(nq):
        for j in range(16):
            for hl in range(2):
                idx = 32 * q + j + 16 * hl
                pos = off + 64 * q + 2 * j + 32 * hl
                for part in range(5):
                    assert image[idx * tab + 16 * part] == pos * tab + 16 * part
