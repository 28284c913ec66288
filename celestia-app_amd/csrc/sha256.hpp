// sha256.hpp -- SHA-256 compression for gfx950 (one message per lane).
//
// Replaces Go crypto/sha256 as used by nmt v0.20.0 NmtHasher (leaf/node hashes,
// mirror test/util/malicious/hasher.go:186-309) and celestia-core
// crypto/merkle (pkg/da/data_availability_header.go:92-108).
//
// Op budget per round on CDNA4: 6 v_alignbit (rotates) + 2 v_bitop3 (xor3) +
// 1 v_bitop3 (Ch) + 1 v_bitop3 (Maj) + 4 adds (v_add3).  The message schedule
// uses v_alignbit + shift + v_bitop3 + v_add3.  All 64 rounds are unrolled and
// the circular 16-word schedule stays in VGPRs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dagpu {

// Each helper falls back to plain C when its operands are compile-time
// constants, so rounds whose inputs are all constant (the parity-namespace
// prefix of a parity leaf, the 0xFF prefix of a node whose left child is all
// parity) fold away entirely instead of being issued with literal operands.
#define DAGPU_CONST3(a, b, c) (__builtin_constant_p(a) && __builtin_constant_p(b) && __builtin_constant_p(c))
__device__ __forceinline__ uint32_t rotr32(uint32_t x, int n) {
  if (__builtin_constant_p(x)) return (x >> n) | (x << (32 - n));
  return __builtin_amdgcn_alignbit(x, x, n);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  if (DAGPU_CONST3(a, b, c)) return a ^ b ^ c;
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// bitop3 truth-table index = (src0 << 2) | (src1 << 1) | src2
__device__ __forceinline__ uint32_t sha_ch(uint32_t e, uint32_t f, uint32_t g) {
  if (DAGPU_CONST3(e, f, g)) return (e & f) ^ (~e & g);
  return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
}
__device__ __forceinline__ uint32_t sha_maj(uint32_t a, uint32_t b, uint32_t c) {
  if (DAGPU_CONST3(a, b, c)) return (a & b) ^ (a & c) ^ (b & c);
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}
__device__ __forceinline__ uint32_t bswap32(uint32_t x) {
  return __builtin_amdgcn_perm(x, x, 0x00010203u);
}

// Round constants.  Rounds 0-15 fold them to immediates; rounds 16-63 run as a
// rolled loop (3 x 16 rounds, keeps the code ~1/4 the size of a full unroll so
// kernels with 9 compressions stay inside the instruction cache) and read them
// with scalar loads.
static __constant__ const uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
    0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
    0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
    0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
    0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
    0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
    0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
    0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};

__device__ __forceinline__ void sha256_init(uint32_t (&st)[8]) {
  st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
  st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}

#define DAGPU_SHA_ROUND(a, b, c, d, e, f, g, h, kw)                         \
  do {                                                                     \
    const uint32_t t1_ = h + xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25)) + \
                         sha_ch(e, f, g) + (kw);                           \
    const uint32_t t2_ = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22)) +    \
                         sha_maj(a, b, c);                                 \
    d += t1_;                                                              \
    h = t1_ + t2_;                                                         \
  } while (0)

// Round constants as compile-time values, for the fully unrolled form.
struct ShaK {
  static constexpr uint32_t v[64] = {
      0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
      0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
      0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
      0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
      0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
      0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
      0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
      0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
};

// One compression.  w[] holds the 16 big-endian message words of the block and
// is clobbered (used as the circular schedule).  Register renaming instead of
// the 8-variable shuffle: round i uses the rotated (a..h) assignment.
// FULL = all 64 rounds unrolled: for blocks with compile-time message words
// (a constant namespace prefix, the padding block) the schedule words that
// depend only on constants fold too -- in the rolled form rounds 16-63 are
// one loop body and fold nothing.  Costs code size, so only those blocks use it.
#ifndef DAGPU_SHA_FULL
#define DAGPU_SHA_FULL 1  // 0: every block rolled (A/B builds)
#endif
template <bool FULL>
__device__ __forceinline__ void sha256_compress_t(uint32_t (&st)[8], uint32_t (&w)[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
  uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int j = 0; j < 16; j += 8) {
    DAGPU_SHA_ROUND(a, b, c, d, e, f, g, h, ShaK::v[j + 0] + w[j + 0]);
    DAGPU_SHA_ROUND(h, a, b, c, d, e, f, g, ShaK::v[j + 1] + w[j + 1]);
    DAGPU_SHA_ROUND(g, h, a, b, c, d, e, f, ShaK::v[j + 2] + w[j + 2]);
    DAGPU_SHA_ROUND(f, g, h, a, b, c, d, e, ShaK::v[j + 3] + w[j + 3]);
    DAGPU_SHA_ROUND(e, f, g, h, a, b, c, d, ShaK::v[j + 4] + w[j + 4]);
    DAGPU_SHA_ROUND(d, e, f, g, h, a, b, c, ShaK::v[j + 5] + w[j + 5]);
    DAGPU_SHA_ROUND(c, d, e, f, g, h, a, b, ShaK::v[j + 6] + w[j + 6]);
    DAGPU_SHA_ROUND(b, c, d, e, f, g, h, a, ShaK::v[j + 7] + w[j + 7]);
  }
  auto schedule16 = [&]() {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
      const uint32_t s0 = xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
      w[j] = w[j] + s0 + w[(j + 9) & 15] + s1;
    }
  };
  if constexpr (FULL && DAGPU_SHA_FULL) {
#pragma unroll
    for (int it = 16; it < 64; it += 16) {
      schedule16();
#pragma unroll
      for (int j = 0; j < 16; j += 8) {
        DAGPU_SHA_ROUND(a, b, c, d, e, f, g, h, ShaK::v[it + j + 0] + w[j + 0]);
        DAGPU_SHA_ROUND(h, a, b, c, d, e, f, g, ShaK::v[it + j + 1] + w[j + 1]);
        DAGPU_SHA_ROUND(g, h, a, b, c, d, e, f, ShaK::v[it + j + 2] + w[j + 2]);
        DAGPU_SHA_ROUND(f, g, h, a, b, c, d, e, ShaK::v[it + j + 3] + w[j + 3]);
        DAGPU_SHA_ROUND(e, f, g, h, a, b, c, d, ShaK::v[it + j + 4] + w[j + 4]);
        DAGPU_SHA_ROUND(d, e, f, g, h, a, b, c, ShaK::v[it + j + 5] + w[j + 5]);
        DAGPU_SHA_ROUND(c, d, e, f, g, h, a, b, ShaK::v[it + j + 6] + w[j + 6]);
        DAGPU_SHA_ROUND(b, c, d, e, f, g, h, a, ShaK::v[it + j + 7] + w[j + 7]);
      }
    }
  } else {
#pragma unroll 1
    for (int it = 16; it < 64; it += 16) {
      schedule16();
#pragma unroll
      for (int j = 0; j < 16; j += 8) {
        DAGPU_SHA_ROUND(a, b, c, d, e, f, g, h, kSha256K[it + j + 0] + w[j + 0]);
        DAGPU_SHA_ROUND(h, a, b, c, d, e, f, g, kSha256K[it + j + 1] + w[j + 1]);
        DAGPU_SHA_ROUND(g, h, a, b, c, d, e, f, kSha256K[it + j + 2] + w[j + 2]);
        DAGPU_SHA_ROUND(f, g, h, a, b, c, d, e, kSha256K[it + j + 3] + w[j + 3]);
        DAGPU_SHA_ROUND(e, f, g, h, a, b, c, d, kSha256K[it + j + 4] + w[j + 4]);
        DAGPU_SHA_ROUND(d, e, f, g, h, a, b, c, kSha256K[it + j + 5] + w[j + 5]);
        DAGPU_SHA_ROUND(c, d, e, f, g, h, a, b, kSha256K[it + j + 6] + w[j + 6]);
        DAGPU_SHA_ROUND(b, c, d, e, f, g, h, a, kSha256K[it + j + 7] + w[j + 7]);
      }
    }
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

__device__ __forceinline__ void sha256_compress(uint32_t (&st)[8], uint32_t (&w)[16]) {
  sha256_compress_t<false>(st, w);
}

}  // namespace dagpu
