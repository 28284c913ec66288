// leo8_sliced.hpp -- bit-sliced Leopard GF(2^8) encode transform (the per-lane
// part of rs_gf8_sliced.hip), shared with the host emulation that checks it on
// the CPU (tools/sliced_emu.hip, tests/test_sliced_emu.py).
//
// Restates the same transform as rs_gf8.hip -- klauspost/reedsolomon v1.11.8
// leopardFF8.encode (ifftDITEncoder8 then fftDIT8 with m = k) -- in a
// different data layout.
//
// Bit-sliced data.  A lane owns 32 byte columns of an element (shard).  It
// keeps them as 8 "planes": plane p is one dword whose 32 bits are bit p of
// each of the 32 bytes.  Adding field elements is still XOR.  Multiplying by a
// field constant c is GF(2)-linear in the bits, so it is an 8x8 bit matrix:
//   out plane i = XOR over j with M_c[i][j] = 1 of plane j,
// where column j of M_c is c * 2^j.  Only full-rate VALU ops are used: v_xor
// and v_bitop3 (xor3, and-xor).  The packed-byte kernel needs v_perm, and any
// v_perm in the stream drops it to half issue rate (profiles/issue_bench_r01.log).
//
// Compile-time skews.  The FFT skew of layer m (butterfly distance D = 2^m) for
// the block starting at element b is fftSkew8[D - 1 + off], with off = b (FFT)
// or k + b (IFFT).  As field elements these skews are GF(2)-linear in off
// (initFFTSkew8 builds them as skew[j + s] = skew[j] ^ temp[i]), so
//   skew(off1 ^ off2) = skew(off1) ^ skew(off2)
// and the multiply matrix splits the same way: M_(a ^ b) = M_a ^ M_b.
//
// Two layouts of the k = 2^n elements over NW = k/16 waves, 16 registers each:
//   A: wave = e >> 4,        register = e & 15   (pair bits 0..3 local)
//   B: wave = e & (NW - 1),  register = e >> (n - 4)  (pair bits n-4..n-1 local)
// In B every bit above a layer's pair bit is a register bit, so every skew is
// a compile-time constant (the matrix folds into a chain of xor3 ops: about 24
// ops per 32-byte butterfly, against 13 v_perm-class ops per 4 bytes before).
// In A the layers below n-4 have skews that also depend on the wave bits:
// skew = C (register bits, compile-time) ^ W (wave bits, one value per layer
// per wave).  W's matrix is loaded into 64 SGPR masks and each matrix entry
// costs one v_bitop3: x_i ^= y_j & (C_ij ? ~W_ij : W_ij).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "gf_const.hpp"

namespace dagpu {
namespace sliced {

constexpr uint8_t gmul(uint8_t a, uint8_t c) {
  if (a == 0 || c == 0) return 0;
  return kGf8.exp[gf8_add_mod(kGf8.log[a], kGf8.log[c])];
}

// skew of table index idx as a field element (log kGf8Mod = element 0)
constexpr uint8_t skew_elem(int idx) {
  const int l = kGf8.skew[idx];
  return l == kGf8Mod ? 0 : kGf8.exp[l];
}

// row[c][i] bit j = bit i of c * 2^j
struct Gf8Mat {
  uint8_t row[256][8];
};
constexpr Gf8Mat make_mat() {
  Gf8Mat m{};
  for (int c = 0; c < 256; c++)
    for (int j = 0; j < 8; j++) {
      const uint8_t col = gmul((uint8_t)(1u << j), (uint8_t)c);
      for (int i = 0; i < 8; i++)
        if ((col >> i) & 1) m.row[c][i] |= (uint8_t)(1u << j);
    }
  return m;
}
inline constexpr Gf8Mat kMat = make_mat();

// Runtime part of the layout-A skews: W(m, w) = skew(D - 1 + 16 w), the same
// for the IFFT and the FFT.  Masks: [m][w][8 i + j] = ~0 if bit i of W * 2^j.
constexpr int kMaxAL = 3;   // layers below n - 4 for k = 128
constexpr int kMaxWav = 8;  // waves for k = 128
struct WMasks {
  uint32_t m[kMaxAL][kMaxWav][64];
};
constexpr WMasks make_wmasks() {
  WMasks t{};
  for (int m = 0; m < kMaxAL; m++)
    for (int w = 0; w < kMaxWav; w++) {
      const uint8_t W = skew_elem((1 << m) - 1 + 16 * w);
      for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) t.m[m][w][8 * i + j] = ((kMat.row[W][i] >> j) & 1) ? 0xFFFFFFFFu : 0u;
    }
  return t;
}
inline constexpr WMasks kWMasksHost = make_wmasks();

// v_bitop3_b32 truth tables (S0 = 0xF0, S1 = 0xCC, S2 = 0xAA)
constexpr uint8_t kXor3 = 0x96;    // a ^ b ^ c
constexpr uint8_t kXorAnd = 0x78;  // a ^ (b & c)
constexpr uint8_t kXorAndN = 0xB4; // a ^ (b & ~c)
constexpr uint8_t kSelect = 0xD8;      // c ? b : a (per bit)

#if defined(__HIP_DEVICE_COMPILE__)
#define SL_BOP3(a, b, c, tt) __builtin_amdgcn_bitop3_b32((a), (b), (c), (tt))
// keeps the scheduler from hoisting the next layer's 64 mask loads (SGPR spills)
#define SL_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define SL_FENCE() ((void)0)
__host__ inline uint32_t sl_bop3_host(uint32_t a, uint32_t b, uint32_t c, uint8_t tt) {
  uint32_t r = 0;
  for (int k = 0; k < 8; k++)
    if ((tt >> k) & 1) r |= ((k & 4) ? a : ~a) & ((k & 2) ? b : ~b) & ((k & 1) ? c : ~c);
  return r;
}
#define SL_BOP3(a, b, c, tt) sl_bop3_host((a), (b), (c), (tt))
#endif

// 8x8 bit transpose of the bytes of 8 dwords, 4 byte positions at once:
// afterwards d[p] byte q bit w = old d[w] byte q bit p.  Its own inverse.
// Each swap of a pair is two shifts and two v_bitop3 bit selects (4 fast ops;
// the xor-swap form t = (hi >> s ^ lo) & m; lo ^= t; hi ^= t << s takes 5).
__host__ __device__ __forceinline__ void swap_bits(uint32_t& hi, uint32_t& lo, int s, uint32_t m) {
  const uint32_t h = hi, l = lo;
  lo = SL_BOP3(l, h >> s, m, kSelect);         // lo with its m bits taken from hi >> s
  hi = SL_BOP3(h, l << s, m << s, kSelect);    // hi with its m << s bits taken from lo << s
}
__host__ __device__ __forceinline__ void transpose8(uint32_t (&d)[8]) {
#pragma unroll
  for (int w = 0; w < 4; w++) swap_bits(d[w], d[w + 4], 4, 0x0F0F0F0Fu);
#pragma unroll
  for (int w0 = 0; w0 < 8; w0 += 4)
#pragma unroll
    for (int w = w0; w < w0 + 2; w++) swap_bits(d[w], d[w + 2], 2, 0x33333333u);
#pragma unroll
  for (int w = 0; w < 8; w += 2) swap_bits(d[w], d[w + 1], 1, 0x55555555u);
}

// Compile-time loop: f(std::integral_constant<int, I>{}) for I = 0 .. N-1, so
// every index, skew and matrix row is a constant expression (a #pragma unroll
// of these nests exceeds the unroller's budget and leaves the register arrays
// dynamically indexed, i.e. in scratch).
template <typename F, int... I>
__host__ __device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__host__ __device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__host__ __device__ __forceinline__ void xor8(uint32_t (&y)[8], const uint32_t (&x)[8]) {
  static_for<8>([&](auto p) { y[p] ^= x[p]; });
}

// x ^= C * y for a compile-time element C: per output plane, its set matrix
// bits are consumed two at a time by xor3.
template <int R, int J>
__host__ __device__ __forceinline__ uint32_t xor_row(uint32_t acc, const uint32_t (&y)[8]) {
  if constexpr (J >= 8) {
    return acc;
  } else if constexpr (!((R >> J) & 1)) {
    return xor_row<R, J + 1>(acc, y);
  } else {
    constexpr int rest = R & ~((2 << J) - 1);  // set bits above J
    if constexpr (rest == 0) {
      return acc ^ y[J];
    } else {
      constexpr int J2 = __builtin_ctz(rest);
      return xor_row<R & ~((2 << J2) - 1), J2 + 1>(SL_BOP3(acc, y[J], y[J2], kXor3), y);
    }
  }
}
template <int C>
__host__ __device__ __forceinline__ void muladd_ct_rows(uint32_t (&x)[8], const uint32_t (&y)[8]) {
  static_for<8>([&](auto i) { x[i] = xor_row<kMat.row[C][i], 0>(x[i], y); });
}

// Shared XOR subexpressions for x ^= C * y (round 3).  Row by row the product
// costs sum_i ceil(|row_i| / 2) three-input XORs (acc + two planes each): 17.9
// on average over the encoder's skews.  A plane triple (or pair) that several
// rows contain can be XOR-ed once into a temporary that those rows then take
// as one term; make_slp extracts them greedily (largest saving first, temps
// may contain temps) at compile time: 13.9 per multiply on average.  Symbols
// 0..7 are the planes y[j], 8.. the temporaries.
struct Slp {
  int ntmp;
  int8_t tmp[8][3];   // operands of temp t (-1 = none: a pair)
  int nterm[8];
  int8_t term[8][16];
};
// acc: rows accumulate into x (row cost ceil(n / 2)); otherwise they are
// summed from scratch (cost floor(n / 2): the first term starts the sum).
constexpr int slp_row_cost(int n, bool acc) { return acc ? (n + 1) / 2 : n / 2; }
constexpr Slp make_slp(int c, bool acc) {
  Slp p{};
  bool has[8][16] = {};
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 8; j++) has[i][j] = (kMat.row[c][i] >> j) & 1;
  int nsym = 8;
  auto cnt = [&](int i) {
    int n = 0;
    for (int s = 0; s < nsym; s++) n += has[i][s];
    return n;
  };
  while (nsym < 16) {
    int best = 0, ba = -1, bb = -1, bc = -1;
    for (int a = 0; a < nsym; a++)
      for (int b = a + 1; b < nsym; b++)
        for (int c3 = b; c3 <= nsym; c3++) {  // c3 == nsym: the pair (a, b)
          const bool pair = c3 == nsym;
          if (!pair && c3 == b) continue;
          const int len = pair ? 2 : 3;
          int sav = -1;  // the temporary's own op
          for (int i = 0; i < 8; i++) {
            if (!(has[i][a] && has[i][b] && (pair || has[i][c3]))) continue;
            const int n = cnt(i);
            sav += slp_row_cost(n, acc) - slp_row_cost(n - len + 1, acc);
          }
          if (sav > best) {
            best = sav;
            ba = a;
            bb = b;
            bc = pair ? -1 : c3;
          }
        }
    if (best <= 0) break;
    const int t = nsym - 8;
    p.tmp[t][0] = (int8_t)ba;
    p.tmp[t][1] = (int8_t)bb;
    p.tmp[t][2] = (int8_t)bc;
    for (int i = 0; i < 8; i++) {
      if (!(has[i][ba] && has[i][bb] && (bc < 0 || has[i][bc]))) continue;
      has[i][ba] = has[i][bb] = false;
      if (bc >= 0) has[i][bc] = false;
      has[i][nsym] = true;
    }
    nsym++;
  }
  p.ntmp = nsym - 8;
  for (int i = 0; i < 8; i++) {
    p.nterm[i] = 0;
    for (int s = 0; s < nsym; s++)
      if (has[i][s]) p.term[i][p.nterm[i]++] = (int8_t)s;
  }
  return p;
}
template <int C, bool ACC = true>
struct SlpOf {
  static constexpr Slp v = make_slp(C, ACC);
};

#ifndef DAGPU_SLP
#define DAGPU_SLP 1  // 0: row-by-row products (A/B builds)
#endif
template <int C>
__host__ __device__ __forceinline__ void muladd_ct(uint32_t (&x)[8], const uint32_t (&y)[8]) {
  if constexpr (!DAGPU_SLP || C == 0) {
    muladd_ct_rows<C>(x, y);
  } else {
    constexpr Slp P = SlpOf<C>::v;
    uint32_t sym[8 + 8];
    static_for<8>([&](auto j) { sym[j] = y[j]; });
    static_for<8>([&](auto t) {
      if constexpr (t < P.ntmp) {
        constexpr int a = P.tmp[t][0], b = P.tmp[t][1], c3 = P.tmp[t][2];
        if constexpr (c3 < 0) sym[8 + t] = sym[a] ^ sym[b];
        else sym[8 + t] = SL_BOP3(sym[a], sym[b], sym[c3], kXor3);
      }
    });
    static_for<8>([&](auto i) {
      constexpr int n = P.nterm[i];
      uint32_t acc = x[i];
      static_for<(n + 1) / 2>([&](auto q) {
        constexpr int t0 = P.term[i][2 * q];
        if constexpr (2 * q + 1 < n) {
          constexpr int t1 = P.term[i][2 * q + 1];
          acc = SL_BOP3(acc, sym[t0], sym[t1], kXor3);
        } else {
          acc ^= sym[t0];
        }
      });
      x[i] = acc;
    });
  }
}

// x ^= (C ^ W) * y: C compile-time, W given by its 64 masks (wave-uniform)
template <int C>
__host__ __device__ __forceinline__ void muladd_rt(uint32_t (&x)[8], const uint32_t (&y)[8], const uint32_t* wm) {
  static_for<8>([&](auto i) {
    uint32_t acc = x[i];
    static_for<8>([&](auto j) {
      if constexpr ((kMat.row[C][i] >> j) & 1)
        acc = SL_BOP3(acc, y[j], wm[8 * i + j], kXorAndN);
      else
        acc = SL_BOP3(acc, y[j], wm[8 * i + j], kXorAnd);
    });
    x[i] = acc;
  });
}

template <int K>
struct Geo {
  static constexpr int n = __builtin_ctz(K);
  static constexpr int NB = n - 4;      // wave bits
  static constexpr int NW = K / 16;     // waves
  static_assert(K >= 16 && K <= 128 && (K & (K - 1)) == 0, "sliced encode: k = 16..128");
};

// IFFT layers m = 0 .. n-5 in layout A (wave wa), distance D = 2^m:
// ifftDIT28 y ^= x; x ^= skew * y.  Compile-time part of the skew: element
// k + (register block start); runtime part: W(m, wa) from wm_base[m * wstride].
template <int K, int IO = K>
__host__ __device__ __forceinline__ void ifft_A(uint32_t (&v)[16][8], const uint32_t* wm_base, int wstride) {
  static_for<Geo<K>::NB>([&](auto m) {
    constexpr int D = 1 << m;
    SL_FENCE();
    const uint32_t* wm = wm_base + m * wstride;
    static_for<16>([&](auto j) {
      if constexpr (!(j & D)) {
        constexpr int c = skew_elem(D - 1 + IO + (j & ~(2 * D - 1)));
        xor8(v[j + D], v[j]);
        muladd_rt<c>(v[j], v[j + D], wm);
      }
    });
  });
}

// FFT layers m = n-5 .. 0 in layout A: fftDIT28 x ^= skew * y; y ^= x.
template <int K, int FO = 0>
__host__ __device__ __forceinline__ void fft_A(uint32_t (&v)[16][8], const uint32_t* wm_base, int wstride) {
  static_for<Geo<K>::NB>([&](auto mm) {
    constexpr int m = Geo<K>::NB - 1 - mm;
    constexpr int D = 1 << m;
    SL_FENCE();
    const uint32_t* wm = wm_base + m * wstride;
    static_for<16>([&](auto j) {
      if constexpr (!(j & D)) {
        constexpr int c = skew_elem(D - 1 + FO + (j & ~(2 * D - 1)));
        muladd_rt<c>(v[j], v[j + D], wm);
        xor8(v[j + D], v[j]);
      }
    });
  });
}

// IFFT layers m = n-4 .. n-1 in layout B: element e = wb + NW * i, the block
// start b = NW * (i with register bits <= m - NB cleared) -- compile-time.
template <int K, int IO = K>
__host__ __device__ __forceinline__ void ifft_B(uint32_t (&v)[16][8]) {
  constexpr int NB = Geo<K>::NB, NW = Geo<K>::NW;
  static_for<4>([&](auto rb) {
    constexpr int D = 1 << (rb + NB), R = 1 << rb;
    static_for<16>([&](auto i) {
      if constexpr (!(i & R)) {
        constexpr int c = skew_elem(D - 1 + IO + NW * (i & ~(2 * R - 1)));
        xor8(v[i + R], v[i]);
        muladd_ct<c>(v[i], v[i + R]);
      }
    });
  });
}

template <int K, int FO = 0>
__host__ __device__ __forceinline__ void fft_B(uint32_t (&v)[16][8]) {
  constexpr int NB = Geo<K>::NB, NW = Geo<K>::NW;
  static_for<4>([&](auto rr) {
    constexpr int rb = 3 - rr;
    constexpr int D = 1 << (rb + NB), R = 1 << rb;
    static_for<16>([&](auto i) {
      if constexpr (!(i & R)) {
        constexpr int c = skew_elem(D - 1 + FO + NW * (i & ~(2 * R - 1)));
        muladd_ct<c>(v[i], v[i + R]);
        xor8(v[i + R], v[i]);
      }
    });
  });
}

// ifft_B then fft_B with their adjacent middle layers fused (round 3): the
// IFFT's last layer and the FFT's first act on the same pairs (i, i + 8), so
//   y ^= x; x ^= c1 y;  x ^= c2 y; y ^= x   ==   y ^= x; x ^= (c1 ^ c2) y; y ^= x
// (multiplication distributes over field addition; a "skip" skew is element 0):
// one constant multiply per pair instead of two.  Skew offsets IO (IFFT) and
// FO (FFT): K and 0 for the encode, 0 and K for the reverse fill.
template <int K, int IO = K, int FO = 0>
__host__ __device__ __forceinline__ void ifft_fft_B(uint32_t (&v)[16][8]) {
  constexpr int NB = Geo<K>::NB, NW = Geo<K>::NW;
  static_for<3>([&](auto rb) {  // IFFT layers n-4 .. n-2
    constexpr int D = 1 << (rb + NB), R = 1 << rb;
    static_for<16>([&](auto i) {
      if constexpr (!(i & R)) {
        constexpr int c = skew_elem(D - 1 + IO + NW * (i & ~(2 * R - 1)));
        xor8(v[i + R], v[i]);
        muladd_ct<c>(v[i], v[i + R]);
      }
    });
  });
  {  // IFFT layer n-1 + FFT layer n-1 (pairs (i, i + 8); block start 0 for i < 8)
    constexpr int D = 1 << (3 + NB);
    static_for<8>([&](auto i) {
      constexpr int c = skew_elem(D - 1 + IO) ^ skew_elem(D - 1 + FO);
      xor8(v[i + 8], v[i]);
      muladd_ct<c>(v[i], v[i + 8]);
      xor8(v[i + 8], v[i]);
    });
  }
  static_for<3>([&](auto rr) {  // FFT layers n-2 .. n-4
    constexpr int rb = 2 - rr;
    constexpr int D = 1 << (rb + NB), R = 1 << rb;
    static_for<16>([&](auto i) {
      if constexpr (!(i & R)) {
        constexpr int c = skew_elem(D - 1 + FO + NW * (i & ~(2 * R - 1)));
        muladd_ct<c>(v[i], v[i + R]);
        xor8(v[i + R], v[i]);
      }
    });
  });
}

// ---------------------------------------------------------------------------
// Two-vector layout for k = 128 (rs_gf8_sliced.hip leo8_encode_sliced2_kernel).
// A 4-wave workgroup holds 2 vectors (128 KB) instead of 4 (256 KB), so two
// workgroups fit a CU and one loads / stores while the other transforms (the
// 4-vector kernel runs one 8-wave workgroup per CU with its phases serialised).
// Lane l = eb * 32 + vv * 16 + t: t = column block, vv = vector, eb = one
// ELEMENT bit carried by the lane.
//   A: e = j + 16 eb + 32 w   (j = register, w = wave)   -- IFFT/FFT layers 0..2
//   B: e = eb + 2 w + 8 i     (i = register)             -- layers 3..6, the same
//      register stride as Geo<128>'s layout B, so ifft_B/fft_B<128> apply as is.
// In A the skew of layer m for element e splits, by the GF(2)-linearity of the
// FFT skews in the block offset (checked by skew_split_ok below), into
//   C(register bits, with the IFFT's +k) ^ eb S16 ^ w0 S32 ^ w1 S64,
// S_b = skew(2^m - 1 + b): C is folded at compile time, the wave bits are
// wave-uniform branches around compile-time matrices, the lane bit multiplies
// a lane-masked copy of y by a compile-time matrix.
// ---------------------------------------------------------------------------
constexpr bool skew_split_ok() {
  for (int m = 0; m < 7; m++) {
    const int D = 1 << m;
    for (int b = 0; b < 256; b += 2 * D) {
      if (D - 1 + b >= 255) continue;
      uint8_t want = 0;
      for (int bit = m + 1; bit < 8; bit++)
        if ((b >> bit) & 1) want ^= skew_elem(D - 1 + (1 << bit));
      if (skew_elem(D - 1 + b) != want) return false;
    }
  }
  return true;
}
static_assert(skew_split_ok(), "FFT skews must be GF(2)-linear in the block offset");

// t = C * y from scratch (no accumulator): the first set bit of a row is the
// plane itself, the rest are consumed two at a time by xor3.
template <int R>
__host__ __device__ __forceinline__ uint32_t row_sum(const uint32_t (&y)[8]) {
  constexpr int J = __builtin_ctz(R);
  return xor_row<R & ~((2 << J) - 1), J + 1>(y[J], y);
}
// x ^= (C * y) & mask: the lane-bit part of a layout-A skew.  One and-xor per
// output plane on top of the row sums (cheaper than masking the 8 inputs).
template <int C>
__host__ __device__ __forceinline__ void muladd_ct_lane(uint32_t (&x)[8], const uint32_t (&y)[8], uint32_t mask) {
  if constexpr (!DAGPU_SLP || C == 0) {
    static_for<8>([&](auto i) {
      constexpr int R = kMat.row[C][i];
      if constexpr (R != 0) x[i] = SL_BOP3(x[i], row_sum<R>(y), mask, kXorAnd);
    });
  } else {  // row sums from scratch over shared temporaries (SlpOf<C, false>)
    constexpr Slp P = SlpOf<C, false>::v;
    uint32_t sym[8 + 8];
    static_for<8>([&](auto j) { sym[j] = y[j]; });
    static_for<8>([&](auto t) {
      if constexpr (t < P.ntmp) {
        constexpr int a = P.tmp[t][0], b = P.tmp[t][1], c3 = P.tmp[t][2];
        if constexpr (c3 < 0) sym[8 + t] = sym[a] ^ sym[b];
        else sym[8 + t] = SL_BOP3(sym[a], sym[b], sym[c3], kXor3);
      }
    });
    static_for<8>([&](auto i) {
      constexpr int n = P.nterm[i];
      if constexpr (n > 0) {
        uint32_t sum = sym[P.term[i][0]];
        static_for<n / 2>([&](auto q) {
          constexpr int t0 = P.term[i][1 + 2 * q];
          if constexpr (2 * q + 2 < n) {
            constexpr int t1 = P.term[i][2 + 2 * q];
            sum = SL_BOP3(sum, sym[t0], sym[t1], kXor3);
          } else {
            sum ^= sym[t0];
          }
        });
        x[i] = SL_BOP3(x[i], sum, mask, kXorAnd);
      }
    });
  }
}

#ifndef DAGPU_WSPEC
#define DAGPU_WSPEC 1  // 0: wave terms as uniform branches around extra multiplies (A/B builds)
#endif
// f(integral_constant<W>) for the wave-uniform index w in 0..3: the wave bits of
// a layout-A skew then fold into the compile-time element, one multiply per
// butterfly on every wave (the branch form costs popcount(w) extra multiplies,
// and the workgroup waits at its barriers for wave 3).
template <typename F>
__host__ __device__ __forceinline__ void wave_switch4(int w, F&& f) {
  switch (w) {
    case 0: f(std::integral_constant<int, 0>{}); break;
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    default: f(std::integral_constant<int, 3>{}); break;
  }
}

// IFFT layers 0..NL-1 in the two-vector layout A (K = 128), wave w, lane mask of eb.
template <int K, int NL = 3, int IO = K>
__host__ __device__ __forceinline__ void ifft_A2(uint32_t (&v)[16][8], int w, uint32_t ebmask) {
  static_assert(K == 128, "two-vector layout: k = 128");
  if constexpr (DAGPU_WSPEC) {
    static_for<NL>([&](auto m) {
      constexpr int D = 1 << m;
      SL_FENCE();
      static_for<16>([&](auto j) {
        if constexpr (!(j & D)) xor8(v[j + D], v[j]);
      });
      wave_switch4(w, [&](auto W) {
        static_for<16>([&](auto j) {
          if constexpr (!(j & D)) muladd_ct<skew_elem(D - 1 + IO + (j & ~(2 * D - 1)) + 32 * W)>(v[j], v[j + D]);
        });
      });
      static_for<16>([&](auto j) {
        if constexpr (!(j & D)) muladd_ct_lane<skew_elem(D - 1 + 16)>(v[j], v[j + D], ebmask);
      });
    });
    return;
  }
  static_for<NL>([&](auto m) {
    constexpr int D = 1 << m;
    SL_FENCE();
    static_for<16>([&](auto j) {
      if constexpr (!(j & D)) {
        constexpr int c = skew_elem(D - 1 + IO + (j & ~(2 * D - 1)));
        xor8(v[j + D], v[j]);
        muladd_ct<c>(v[j], v[j + D]);
      }
    });
    if (w & 1) {
      static_for<16>([&](auto j) {
        if constexpr (!(j & D)) muladd_ct<skew_elem(D - 1 + 32)>(v[j], v[j + D]);
      });
    }
    if (w & 2) {
      static_for<16>([&](auto j) {
        if constexpr (!(j & D)) muladd_ct<skew_elem(D - 1 + 64)>(v[j], v[j + D]);
      });
    }
    static_for<16>([&](auto j) {
      if constexpr (!(j & D)) muladd_ct_lane<skew_elem(D - 1 + 16)>(v[j], v[j + D], ebmask);
    });
  });
}

// FFT layers NL-1..0 in the two-vector layout A.
template <int K, int NL = 3, int FO = 0>
__host__ __device__ __forceinline__ void fft_A2(uint32_t (&v)[16][8], int w, uint32_t ebmask) {
  static_assert(K == 128, "two-vector layout: k = 128");
  if constexpr (DAGPU_WSPEC) {
    static_for<NL>([&](auto mm) {
      constexpr int m = NL - 1 - mm;
      constexpr int D = 1 << m;
      SL_FENCE();
      wave_switch4(w, [&](auto W) {
        static_for<16>([&](auto j) {
          if constexpr (!(j & D)) muladd_ct<skew_elem(D - 1 + FO + (j & ~(2 * D - 1)) + 32 * W)>(v[j], v[j + D]);
        });
      });
      static_for<16>([&](auto j) {
        if constexpr (!(j & D)) muladd_ct_lane<skew_elem(D - 1 + 16)>(v[j], v[j + D], ebmask);
      });
      static_for<16>([&](auto j) {
        if constexpr (!(j & D)) xor8(v[j + D], v[j]);
      });
    });
    return;
  }
  static_for<NL>([&](auto mm) {
    constexpr int m = NL - 1 - mm;
    constexpr int D = 1 << m;
    SL_FENCE();
    static_for<16>([&](auto j) {
      if constexpr (!(j & D)) muladd_ct<skew_elem(D - 1 + FO + (j & ~(2 * D - 1)))>(v[j], v[j + D]);
    });
    if (w & 1) {
      static_for<16>([&](auto j) {
        if constexpr (!(j & D)) muladd_ct<skew_elem(D - 1 + 32)>(v[j], v[j + D]);
      });
    }
    if (w & 2) {
      static_for<16>([&](auto j) {
        if constexpr (!(j & D)) muladd_ct<skew_elem(D - 1 + 64)>(v[j], v[j + D]);
      });
    }
    static_for<16>([&](auto j) {
      if constexpr (!(j & D)) muladd_ct_lane<skew_elem(D - 1 + 16)>(v[j], v[j + D], ebmask);
    });
    static_for<16>([&](auto j) {
      if constexpr (!(j & D)) xor8(v[j + D], v[j]);
    });
  });
}


// Two-vector layout A* (K = 128): e = eb + 2 r + 32 w, the lane bit is element
// bit 0 (a wave-local transpose of A).  Layers 1..2 pair register bits 0..1 of
// r; their skews depend on element bits above the pair bit only, so the lane
// bit drops out: C(register bits) ^ w0 S32 ^ w1 S64, no lane term.
template <int K, int IO = K>
__host__ __device__ __forceinline__ void ifft_As2(uint32_t (&v)[16][8], int w) {
  static_assert(K == 128, "two-vector layout: k = 128");
  if constexpr (DAGPU_WSPEC) {
    static_for<2>([&](auto mm) {
      constexpr int m = 1 + mm;
      constexpr int D = 1 << m, R = D >> 1;
      SL_FENCE();
      static_for<16>([&](auto r) {
        if constexpr (!(r & R)) xor8(v[r + R], v[r]);
      });
      wave_switch4(w, [&](auto W) {
        static_for<16>([&](auto r) {
          if constexpr (!(r & R)) muladd_ct<skew_elem(D - 1 + IO + ((2 * r) & ~(2 * D - 1)) + 32 * W)>(v[r], v[r + R]);
        });
      });
    });
    return;
  }
  static_for<2>([&](auto mm) {
    constexpr int m = 1 + mm;
    constexpr int D = 1 << m, R = D >> 1;
    SL_FENCE();
    static_for<16>([&](auto r) {
      if constexpr (!(r & R)) {
        constexpr int c = skew_elem(D - 1 + IO + ((2 * r) & ~(2 * D - 1)));
        xor8(v[r + R], v[r]);
        muladd_ct<c>(v[r], v[r + R]);
      }
    });
    if (w & 1) {
      static_for<16>([&](auto r) {
        if constexpr (!(r & R)) muladd_ct<skew_elem(D - 1 + 32)>(v[r], v[r + R]);
      });
    }
    if (w & 2) {
      static_for<16>([&](auto r) {
        if constexpr (!(r & R)) muladd_ct<skew_elem(D - 1 + 64)>(v[r], v[r + R]);
      });
    }
  });
}

template <int K, int FO = 0>
__host__ __device__ __forceinline__ void fft_As2(uint32_t (&v)[16][8], int w) {
  static_assert(K == 128, "two-vector layout: k = 128");
  if constexpr (DAGPU_WSPEC) {
    static_for<2>([&](auto mm) {
      constexpr int m = 2 - mm;
      constexpr int D = 1 << m, R = D >> 1;
      SL_FENCE();
      wave_switch4(w, [&](auto W) {
        static_for<16>([&](auto r) {
          if constexpr (!(r & R)) muladd_ct<skew_elem(D - 1 + FO + ((2 * r) & ~(2 * D - 1)) + 32 * W)>(v[r], v[r + R]);
        });
      });
      static_for<16>([&](auto r) {
        if constexpr (!(r & R)) xor8(v[r + R], v[r]);
      });
    });
    return;
  }
  static_for<2>([&](auto mm) {
    constexpr int m = 2 - mm;
    constexpr int D = 1 << m, R = D >> 1;
    SL_FENCE();
    static_for<16>([&](auto r) {
      if constexpr (!(r & R)) muladd_ct<skew_elem(D - 1 + FO + ((2 * r) & ~(2 * D - 1)))>(v[r], v[r + R]);
    });
    if (w & 1) {
      static_for<16>([&](auto r) {
        if constexpr (!(r & R)) muladd_ct<skew_elem(D - 1 + 32)>(v[r], v[r + R]);
      });
    }
    if (w & 2) {
      static_for<16>([&](auto r) {
        if constexpr (!(r & R)) muladd_ct<skew_elem(D - 1 + 64)>(v[r], v[r + R]);
      });
    }
    static_for<16>([&](auto r) {
      if constexpr (!(r & R)) xor8(v[r + R], v[r]);
    });
  });
}

// ---------------------------------------------------------------------------
// Bit-sliced decode for k = 128 (rs_decode_sliced.hip leo8_decode128_sliced_kernel):
// leopard8.go reconstruct's IFFT_256 and FFT_256 (decoder skew index b + D - 1,
// no +k offset) on n = 256 work elements, one vector per 4-wave workgroup.
// Lane l = t + 16 eb: t = 32-byte column block, eb = TWO element bits; wave w.
//   A:  e = j + 16 eb + 64 w  (j = register)  -- layers 0..1
//   A*: e = eb + 4 r + 64 w   (r = register)  -- layers 2..3 (wave-local transpose of A)
//   B:  e = eb + 4 w + 16 i   (i = register)  -- layers 4..7, skews compile-time
// In A the skew of layer m splits (skew_split_ok, bits up to 7) into
//   C(j) ^ eb0 S16 ^ eb1 S32 ^ w0 S64 ^ w1 S128,  S_x = skew(2^m - 1 + x);
// in A* the lane bits are element bits 0..1, below the pair bit, so only the
// wave terms remain.
// ---------------------------------------------------------------------------

// Decoder layers 0..NL-1 in layout A (IFFT ascending, FFT descending).
// IFFT butterfly (ifftDIT8): y ^= x; x ^= skew * y.  FFT (fftDIT8): x ^= skew * y; y ^= x.
template <bool IFFT, int NL>
__host__ __device__ __forceinline__ void dec_A(uint32_t (&v)[16][8], int w, uint32_t eb0mask, uint32_t eb1mask) {
  if constexpr (DAGPU_WSPEC) {
    static_for<NL>([&](auto mm) {
      constexpr int m = IFFT ? (int)mm : NL - 1 - (int)mm;
      constexpr int D = 1 << m;
      SL_FENCE();
      if constexpr (IFFT) {
        static_for<16>([&](auto j) {
          if constexpr (!(j & D)) xor8(v[j + D], v[j]);
        });
      }
      wave_switch4(w, [&](auto W) {
        static_for<16>([&](auto j) {
          if constexpr (!(j & D)) muladd_ct<skew_elem(D - 1 + (j & ~(2 * D - 1)) + 64 * W)>(v[j], v[j + D]);
        });
      });
      static_for<16>([&](auto j) {
        if constexpr (!(j & D)) muladd_ct_lane<skew_elem(D - 1 + 16)>(v[j], v[j + D], eb0mask);
      });
      static_for<16>([&](auto j) {
        if constexpr (!(j & D)) muladd_ct_lane<skew_elem(D - 1 + 32)>(v[j], v[j + D], eb1mask);
      });
      if constexpr (!IFFT) {
        static_for<16>([&](auto j) {
          if constexpr (!(j & D)) xor8(v[j + D], v[j]);
        });
      }
    });
    return;
  }
  static_for<NL>([&](auto mm) {
    constexpr int m = IFFT ? (int)mm : NL - 1 - (int)mm;
    constexpr int D = 1 << m;
    SL_FENCE();
    if constexpr (IFFT) {
      static_for<16>([&](auto j) {
        if constexpr (!(j & D)) xor8(v[j + D], v[j]);
      });
    }
    static_for<16>([&](auto j) {
      if constexpr (!(j & D)) muladd_ct<skew_elem(D - 1 + (j & ~(2 * D - 1)))>(v[j], v[j + D]);
    });
    if (w & 1) {
      static_for<16>([&](auto j) {
        if constexpr (!(j & D)) muladd_ct<skew_elem(D - 1 + 64)>(v[j], v[j + D]);
      });
    }
    if (w & 2) {
      static_for<16>([&](auto j) {
        if constexpr (!(j & D)) muladd_ct<skew_elem(D - 1 + 128)>(v[j], v[j + D]);
      });
    }
    static_for<16>([&](auto j) {
      if constexpr (!(j & D)) muladd_ct_lane<skew_elem(D - 1 + 16)>(v[j], v[j + D], eb0mask);
    });
    static_for<16>([&](auto j) {
      if constexpr (!(j & D)) muladd_ct_lane<skew_elem(D - 1 + 32)>(v[j], v[j + D], eb1mask);
    });
    if constexpr (!IFFT) {
      static_for<16>([&](auto j) {
        if constexpr (!(j & D)) xor8(v[j + D], v[j]);
      });
    }
  });
}

// Decoder layers 2..3 in layout A*: register bit (m - 2) of r is element bit m,
// block start b = 4 (r with register bits <= m - 2 cleared) + 64 w.
template <bool IFFT>
__host__ __device__ __forceinline__ void dec_Astar(uint32_t (&v)[16][8], int w) {
  if constexpr (DAGPU_WSPEC) {
    static_for<2>([&](auto mm) {
      constexpr int rb = IFFT ? (int)mm : 1 - (int)mm;
      constexpr int D = 4 << rb, R = 1 << rb;
      SL_FENCE();
      if constexpr (IFFT) {
        static_for<16>([&](auto r) {
          if constexpr (!(r & R)) xor8(v[r + R], v[r]);
        });
      }
      wave_switch4(w, [&](auto W) {
        static_for<16>([&](auto r) {
          if constexpr (!(r & R)) muladd_ct<skew_elem(D - 1 + 4 * (r & ~(2 * R - 1)) + 64 * W)>(v[r], v[r + R]);
        });
      });
      if constexpr (!IFFT) {
        static_for<16>([&](auto r) {
          if constexpr (!(r & R)) xor8(v[r + R], v[r]);
        });
      }
    });
    return;
  }
  static_for<2>([&](auto mm) {
    constexpr int rb = IFFT ? (int)mm : 1 - (int)mm;
    constexpr int D = 4 << rb, R = 1 << rb;
    SL_FENCE();
    if constexpr (IFFT) {
      static_for<16>([&](auto r) {
        if constexpr (!(r & R)) xor8(v[r + R], v[r]);
      });
    }
    static_for<16>([&](auto r) {
      if constexpr (!(r & R)) muladd_ct<skew_elem(D - 1 + 4 * (r & ~(2 * R - 1)))>(v[r], v[r + R]);
    });
    if (w & 1) {
      static_for<16>([&](auto r) {
        if constexpr (!(r & R)) muladd_ct<skew_elem(D - 1 + 64)>(v[r], v[r + R]);
      });
    }
    if (w & 2) {
      static_for<16>([&](auto r) {
        if constexpr (!(r & R)) muladd_ct<skew_elem(D - 1 + 128)>(v[r], v[r + R]);
      });
    }
    if constexpr (!IFFT) {
      static_for<16>([&](auto r) {
        if constexpr (!(r & R)) xor8(v[r + R], v[r]);
      });
    }
  });
}

// Decoder layers 4..7 in layout B: register bit rb of i is element bit 4 + rb,
// block start b = 16 (i with register bits <= rb cleared) -- compile-time.
template <bool IFFT>
__host__ __device__ __forceinline__ void dec_B(uint32_t (&v)[16][8]) {
  static_for<4>([&](auto rr) {
    constexpr int rb = IFFT ? (int)rr : 3 - (int)rr;
    constexpr int D = 16 << rb, R = 1 << rb;
    SL_FENCE();
    static_for<16>([&](auto i) {
      if constexpr (!(i & R)) {
        constexpr int c = skew_elem(D - 1 + 16 * (i & ~(2 * R - 1)));
        if constexpr (IFFT) {
          xor8(v[i + R], v[i]);
          muladd_ct<c>(v[i], v[i + R]);
        } else {
          muladd_ct<c>(v[i], v[i + R]);
          xor8(v[i + R], v[i]);
        }
      }
    });
  });
}

// Formal derivative (leopard8.go: for i in 1..n-1, work[i-lowbit(i), i) ^=
// work[i, i+lowbit(i))) in closed form: D(x)_e = x_e ^ XOR over bits s with
// e_s = 0 of x_(e | 2^s), ORIGINAL x.  The register bits of the layout are
// applied in place in ascending register order (v[j | 2^sb] > j is still
// original when j is processed); the caller adds the other bits' terms.
// Planes [P0, P0 + NP).
template <int P0, int NP>
__host__ __device__ __forceinline__ void deriv_local(uint32_t (&v)[16][8]) {
  static_for<16>([&](auto j) {
    static_for<4>([&](auto sb) {
      if constexpr (!((j >> sb) & 1)) {
        static_for<NP>([&](auto p) { v[j][P0 + p] ^= v[j | (1 << sb)][P0 + p]; });
      }
    });
  });
}

// x * exp(lm) on PACKED bytes (before the bit transpose / after the inverse
// one), with the 3/3/2-bit byte tables of gf_const.hpp: tb = t8[lm][0..3]
// (c * (0..7) as lo | hi, c * ((0..7) << 3) as lo | hi) and t2 = t8[lm][4]
// (c * ((0..3) << 6)), all zero for a missing shard.  Per dword: three v_perm
// lookups (an 8-byte pool each for the two 3-bit groups), five index ops and
// one xor3 -- 9 ops for 4 bytes (72 per 32 bytes; the bit-plane power-basis
// multiply took ~136, four 2-bit lookups 104).
typedef unsigned int tab4 __attribute__((ext_vector_type(4)));
__host__ __device__ __forceinline__ uint32_t perm8v(uint32_t hi, uint32_t lo, uint32_t idx) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(hi, lo, idx);
#else
  uint32_t r = 0;
  for (int b = 0; b < 4; b++) {
    const uint32_t i = (idx >> (8 * b)) & 7u;
    r |= (((i < 4 ? lo : hi) >> (8 * (i & 3))) & 0xFFu) << (8 * b);
  }
  return r;
#endif
}
__host__ __device__ __forceinline__ void mul_packed(uint32_t (&d)[8], const tab4 tb, uint32_t t2) {
  static_for<8>([&](auto i) {
    const uint32_t y = d[i];
    const uint32_t p0 = perm8v(tb.y, tb.x, y & 0x07070707u);
    const uint32_t p1 = perm8v(tb.w, tb.z, (y >> 3) & 0x07070707u);
    const uint32_t p2 = perm8v(t2, t2, (y >> 6) & 0x03030303u);
    d[i] = SL_BOP3(p0, p1, p2, kXor3);
  });
}
__host__ __device__ inline tab4 mul_table(int lm) {  // lm < 0: the zero multiplier
  if (lm < 0) return (tab4){0u, 0u, 0u, 0u};
  return (tab4){kGf8.t8[lm][0], kGf8.t8[lm][1], kGf8.t8[lm][2], kGf8.t8[lm][3]};
}
__host__ __device__ inline uint32_t mul_table2(int lm) { return lm < 0 ? 0u : kGf8.t8[lm][4]; }

}  // namespace sliced
}  // namespace dagpu
