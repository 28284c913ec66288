// gf_const.hpp -- compile-time Leopard GF(2^8) constants for the gfx950 kernels.
//
// Restates klauspost/reedsolomon v1.11.8 leopard8.go (initLUTs8, initFFTSkew8,
// mul8LUTs), the field the reference's default codec uses
// (pkg/appconsts/global_consts.go:92 DefaultCodec = rsmt2d.NewLeoRSCodec ->
// reedsolomon.New(k, k, WithLeopardGF(true)), GF(2^8) while 2k <= 256).
//
// Everything here is constexpr: the encode kernels are fully unrolled per k,
// so every skew value and every multiply table folds to an immediate.
//
// Multiply-by-constant on four packed bytes uses v_perm_b32 as a byte-table
// lookup.  Multiplication by a fixed field element is GF(2)-linear in the bit
// representation, so  c*x = T0[x&7] ^ T1[(x>>3)&7] ^ T2[x>>6]  with 8-, 8- and
// 4-entry byte tables (t8).  An 8-entry table spans two dwords; gfx950 VOP3
// reads at most one scalar operand, so the second dword is moved into a VGPR
// right before use by an inline-asm v_mov (left to itself the compiler hoists
// those constants and keeps them live: 256 VGPRs at k=128).  The 4 x 2-bit
// form (t, one SGPR per v_perm) is used for runtime multipliers.
// Measured (tools/rs_bench.hip, k=128): 3/3/2 form 13.5 % faster than 2x4.
#pragma once
#include <stdint.h>

namespace dagpu {

constexpr int kGf8Bits = 8;
constexpr int kGf8Order = 256;
constexpr int kGf8Mod = 255;

struct Gf8Const {
  uint8_t log[256];
  uint8_t exp[256];
  uint8_t skew[255];
  uint8_t walsh[256];  // logWalsh8 = FWHT(log with [0] = 0), decode only
  // perm tables per log_m: t[g][lm] = bytes c*(v << 2g), v = 0..3
  uint32_t t[4][256];
  // 3/3/2-bit tables per log_m: t8[lm] = {c*(0..3), c*(4..7), c*((0..3)<<3),
  // c*((4..7)<<3), c*((0..3)<<6)}
  uint32_t t8[256][5];
};

constexpr uint8_t gf8_add_mod(unsigned a, unsigned b) {
  unsigned s = a + b;
  return (uint8_t)(s + (s >> 8));
}

constexpr Gf8Const make_gf8_const() {
  Gf8Const g{};
  const uint8_t cantor[8] = {1, 214, 152, 146, 86, 200, 88, 230};
  unsigned state = 1;
  for (unsigned i = 0; i < 255; i++) {
    g.exp[state] = (uint8_t)i;
    state <<= 1;
    if (state >= 256) state ^= 0x11D;
  }
  g.exp[0] = 255;
  g.log[0] = 0;
  for (int i = 0; i < 8; i++) {
    int width = 1 << i;
    for (int j = 0; j < width; j++) g.log[j + width] = (uint8_t)(g.log[j] ^ cantor[i]);
  }
  for (int i = 0; i < 256; i++) g.log[i] = g.exp[g.log[i]];
  for (int i = 0; i < 256; i++) g.exp[g.log[i]] = (uint8_t)i;
  g.exp[255] = g.exp[0];

  auto mullog = [&](uint8_t a, uint8_t lb) -> uint8_t {
    if (a == 0) return 0;
    return g.exp[gf8_add_mod(g.log[a], lb)];
  };

  uint8_t temp[7] = {};
  for (int i = 1; i < 8; i++) temp[i - 1] = (uint8_t)(1 << i);
  for (int i = 0; i < 255; i++) g.skew[i] = 0;
  for (int m = 0; m < 7; m++) {
    int step = 1 << (m + 1);
    g.skew[(1 << m) - 1] = 0;
    for (int i = m; i < 7; i++) {
      int s = 1 << (i + 1);
      for (int j = (1 << m) - 1; j < s; j += step) g.skew[j + s] = (uint8_t)(g.skew[j] ^ temp[i]);
    }
    temp[m] = (uint8_t)(255 - g.log[mullog(temp[m], g.log[temp[m] ^ 1])]);
    for (int i = m + 1; i < 7; i++) {
      uint8_t sum = gf8_add_mod(g.log[temp[i] ^ 1], temp[m]);
      temp[i] = mullog(temp[i], sum);
    }
  }
  for (int i = 0; i < 255; i++) g.skew[i] = g.log[g.skew[i]];

  // logWalsh8: fwht8(log with [0] = 0, m = mtrunc = 256)
  {
    for (int i = 0; i < 256; i++) g.walsh[i] = g.log[i];
    g.walsh[0] = 0;
    auto addm = [](unsigned a, unsigned b) -> uint8_t { unsigned s = a + b; return (uint8_t)(s + (s >> 8)); };
    auto subm = [](unsigned a, unsigned b) -> uint8_t { unsigned d = a - b; return (uint8_t)(d + (d >> 8)); };
    for (int dist = 1, dist4 = 4; dist4 <= 256; dist = dist4, dist4 <<= 2) {
      for (int r = 0; r < 256; r += dist4) {
        for (int i = r; i < r + dist; i++) {
          uint8_t t0 = g.walsh[i], t1 = g.walsh[i + dist], t2 = g.walsh[i + 2 * dist], t3 = g.walsh[i + 3 * dist];
          uint8_t a0 = addm(t0, t1), a1 = subm(t0, t1), a2 = addm(t2, t3), a3 = subm(t2, t3);
          g.walsh[i] = addm(a0, a2); g.walsh[i + 2 * dist] = subm(a0, a2);
          g.walsh[i + dist] = addm(a1, a3); g.walsh[i + 3 * dist] = subm(a1, a3);
        }
      }
    }
  }

  for (int lm = 0; lm < 256; lm++) {
    uint32_t a[8] = {}, b[8] = {}, c[4] = {};
    for (int x = 0; x < 8; x++) {
      a[x] = mullog((uint8_t)x, (uint8_t)lm);
      b[x] = mullog((uint8_t)(x << 3), (uint8_t)lm);
    }
    for (int x = 0; x < 4; x++) c[x] = mullog((uint8_t)(x << 6), (uint8_t)lm);
    g.t8[lm][0] = a[0] | a[1] << 8 | a[2] << 16 | a[3] << 24;
    g.t8[lm][1] = a[4] | a[5] << 8 | a[6] << 16 | a[7] << 24;
    g.t8[lm][2] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
    g.t8[lm][3] = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
    g.t8[lm][4] = c[0] | c[1] << 8 | c[2] << 16 | c[3] << 24;
    for (int grp = 0; grp < 4; grp++) {
      uint32_t v = 0;
      for (int x = 0; x < 4; x++) v |= (uint32_t)mullog((uint8_t)(x << (2 * grp)), (uint8_t)lm) << (8 * x);
      g.t[grp][lm] = v;
    }
  }
  return g;
}

inline constexpr Gf8Const kGf8 = make_gf8_const();

// Sanity: first skew entries quoted in SURVEY.md Appendix A.1.
static_assert(kGf8.skew[0] == 255 && kGf8.skew[2] == 85 && kGf8.skew[4] == 17 &&
                  kGf8.skew[8] == 153 && kGf8.skew[14] == 187,
              "Leopard GF(2^8) FFT skew mismatch");

}  // namespace dagpu
