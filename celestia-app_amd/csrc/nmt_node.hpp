// nmt_node.hpp -- NMT node helpers shared by the square pipeline (nmt.hip) and
// the generic forest engine (nmt_forest.hip).  A node in registers is 24 dwords
// in memory byte order: minNs (29 B zero padded to 8 dwords), maxNs, digest.
// HashNode message layout follows nmt v0.20.0 NmtHasher.HashNode (mirror:
// test/util/malicious/hasher.go:271-297): 0x01 | left(90) | right(90).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "sha256.hpp"

namespace dagpu {

// v_perm_b32 selector byte 0x0C produces 0x00.
#define PZ 0x0Cu

// ---------------------------------------------------------------------------
// Node helpers.  A node in registers/LDS: 24 dwords in memory byte order:
// [0..7] minNs (29 B, zero padded), [8..15] maxNs, [16..23] digest bytes.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool ns_is_parity(const uint32_t (&ns)[8]) {
  uint32_t acc = ns[0] & ns[1] & ns[2] & ns[3] & ns[4] & ns[5] & ns[6];
  return acc == 0xFFFFFFFFu && (ns[7] & 0xFFu) == 0xFFu;
}

// lexicographic a < b over 29 bytes
__device__ __forceinline__ bool ns_less(const uint32_t (&x)[8], const uint32_t (&y)[8]) {
  int res = 0;  // -1 less, 1 greater, 0 equal so far
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t xa = bswap32(i == 7 ? (x[i] & 0xFFu) : x[i]);
    const uint32_t ya = bswap32(i == 7 ? (y[i] & 0xFFu) : y[i]);
    if (res == 0) res = (xa < ya) ? -1 : ((xa > ya) ? 1 : 0);
  }
  return res < 0;
}

// OR `src` (NDW little-endian dwords, zero padded) into byte buffer m at OFF.
template <int OFF, int NDW, int MW>
__device__ __forceinline__ void put_bytes(uint32_t (&m)[MW], const uint32_t (&src)[NDW]) {
  constexpr int al = OFF & 3;
  constexpr int d0 = OFF >> 2;
#pragma unroll
  for (int i = 0; i < NDW; i++) {
    if constexpr (al == 0) {
      m[d0 + i] |= src[i];
    } else {
      m[d0 + i] |= src[i] << (8 * al);
      if (d0 + i + 1 < MW) m[d0 + i + 1] |= src[i] >> (32 - 8 * al);
    }
  }
}

// v_perm_b32 with a plain-C fallback when both sources are compile-time
// constants (parity namespace words), so constant message words fold.
__device__ __forceinline__ uint32_t perm_c(uint32_t s0, uint32_t s1, uint32_t sel) {
  if (__builtin_constant_p(s0) && __builtin_constant_p(s1)) {
    const uint64_t v = ((uint64_t)s0 << 32) | s1;
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint32_t sb = (sel >> (8 * i)) & 0xFFu;
      const uint32_t byte = sb < 8 ? (uint32_t)(v >> (8 * sb)) & 0xFFu : sb == 12 ? 0u : 0xFFu;
      r |= byte << (8 * i);
    }
    return r;
  }
  return __builtin_amdgcn_perm(s0, s1, sel);
}

// Byte m of the HashNode message 0x01 | L.min(29) | L.max(29) | L.d(32) |
// R.min(29) | R.max(29) | R.d(32) | SHA padding (181 B, 3 blocks): part 0..5
// and byte within the part, or part -1 with a constant value.
struct NodeByte {
  int part, q, cval;
};
constexpr NodeByte node_byte(int m) {
  constexpr int off[6] = {1, 30, 59, 91, 120, 149}, len[6] = {29, 29, 32, 29, 29, 32};
  if (m == 0) return {-1, 0, 0x01};
  for (int p = 0; p < 6; p++)
    if (m >= off[p] && m < off[p] + len[p]) return {p, m - off[p], 0};
  if (m == 181) return {-1, 0, 0x80};
  if (m >= 184 && m < 192) {  // 64-bit big-endian bit length 181 * 8 = 1448
    const unsigned long long bits = 181ull * 8ull;
    return {-1, 0, (int)((bits >> (8 * (191 - m))) & 0xFF)};
  }
  return {-1, 0, 0};
}

// Big-endian message word J built with v_perm_b32 straight from the parts'
// little-endian dwords: one perm when its 4 bytes come from <= 2 source
// dwords, two when from 3 (a 29-byte namespace's last byte plus its neighbours),
// plus an OR for the 0x01 / 0x80 bytes.  (Round 2 shifted and OR-ed every
// dword into place and byte-swapped each word: ~3 ops per word.)
template <int J, class G>
__device__ __forceinline__ uint32_t node_word(const G& get) {
  struct Src {
    int part, d;
  };
  struct Plan {
    Src src[3];
    int nsrc;
    int which[4];  // per output byte (0 = LSB = message byte 4J+3): source slot, -1 = constant
    int sb[4];     // byte within that source dword
    uint32_t cword;  // constant bytes
  };
  constexpr Plan P = [] {
    Plan pl{};
    pl.nsrc = 0;
    pl.cword = 0;
    for (int i = 0; i < 4; i++) {
      const NodeByte nb = node_byte(4 * J + 3 - i);
      if (nb.part < 0) {
        pl.which[i] = -1;
        pl.sb[i] = 0;
        pl.cword |= (uint32_t)nb.cval << (8 * i);
        continue;
      }
      const int d = nb.q >> 2;
      int slot = -1;
      for (int t = 0; t < pl.nsrc; t++)
        if (pl.src[t].part == nb.part && pl.src[t].d == d) slot = t;
      if (slot < 0) {
        slot = pl.nsrc++;
        pl.src[slot] = {nb.part, d};
      }
      pl.which[i] = slot;
      pl.sb[i] = nb.q & 3;
    }
    return pl;
  }();
  if constexpr (P.nsrc == 0) {
    return P.cword;
  } else if constexpr (P.nsrc <= 2) {
    // perm(S0 = src[1] (bytes 4..7), S1 = src[0] (bytes 0..3))
    constexpr uint32_t sel = [] {
      uint32_t s = 0;
      for (int i = 0; i < 4; i++) {
        const uint32_t v = P.which[i] < 0 ? 0x0Cu : (uint32_t)(P.which[i] == 0 ? P.sb[i] : 4 + P.sb[i]);
        s |= v << (8 * i);
      }
      return s;
    }();
    const uint32_t s1 = get(P.src[0].part, P.src[0].d);
    const uint32_t s0 = P.nsrc == 2 ? get(P.src[1].part, P.src[1].d) : s1;
    const uint32_t w = perm_c(s0, s1, sel);
    return P.cword ? (w | P.cword) : w;
  } else {
    // t = perm(src[1], src[0]) for their bytes; then perm(t, src[2])
    constexpr uint32_t sel1 = [] {
      uint32_t s = 0;
      for (int i = 0; i < 4; i++) {
        const uint32_t v = (P.which[i] == 0) ? (uint32_t)P.sb[i] : (P.which[i] == 1) ? 4u + P.sb[i] : 0x0Cu;
        s |= v << (8 * i);
      }
      return s;
    }();
    constexpr uint32_t sel2 = [] {
      uint32_t s = 0;
      for (int i = 0; i < 4; i++) {
        const uint32_t v = (P.which[i] == 2) ? (uint32_t)P.sb[i] : (P.which[i] < 0) ? 0x0Cu : 4u + i;
        s |= v << (8 * i);
      }
      return s;
    }();
    const uint32_t t = perm_c(get(P.src[1].part, P.src[1].d), get(P.src[0].part, P.src[0].d), sel1);
    const uint32_t w = perm_c(t, get(P.src[2].part, P.src[2].d), sel2);
    return P.cword ? (w | P.cword) : w;
  }
}

template <int B, class G, bool F>
__device__ __forceinline__ void static_for_words(const G& get, uint32_t (&st)[8], std::bool_constant<F>) {
  uint32_t m[16];
  [&]<int... I>(std::integer_sequence<int, I...>) {
    ((m[I] = node_word<16 * B + I>(get)), ...);
  }(std::make_integer_sequence<int, 16>{});
  sha256_compress_t<F>(st, m);
}

// NMT HashNode message 0x01 | L.min | L.max | L.d | R.min | R.max | R.d
// (181 B, 3 SHA blocks).  get(P, i): P = 0..5 -> Lmn, Lmx, Ld, Rmn, Rmx, Rd
// (8 little-endian dwords in memory byte order; namespace bytes 29..31 are
// never read).  FULLn: block n runs fully unrolled, for callers whose get()
// returns compile-time constants in that block (all-parity children).
template <bool FULL0 = false, bool FULL1 = false, bool FULL2 = false, class G>
__device__ __forceinline__ void sha_node_msg(const G& get, uint32_t (&st)[8]) {
  sha256_init(st);
  static_for_words<0>(get, st, std::bool_constant<FULL0>{});
  static_for_words<1>(get, st, std::bool_constant<FULL1>{});
  static_for_words<2>(get, st, std::bool_constant<FULL2>{});
}

__device__ __forceinline__ void load_digest(const uint8_t* p, uint32_t (&d)[8]) {
  const uint4* q = (const uint4*)p;
  const uint4 x0 = q[0], x1 = q[1];
  d[0] = x0.x; d[1] = x0.y; d[2] = x0.z; d[3] = x0.w;
  d[4] = x1.x; d[5] = x1.y; d[6] = x1.z; d[7] = x1.w;
}

__device__ __forceinline__ void write_root(uint8_t* dst, const uint32_t (&mn)[8], const uint32_t (&mx)[8],
                                           const uint32_t (&dg)[8]) {
  // 90 B at a 2-byte aligned address: 45 halfword stores
  uint16_t* d16 = (uint16_t*)dst;
#pragma unroll
  for (int h = 0; h < 45; h++) {
    uint32_t lo, hi;
    const int b0 = 2 * h, b1 = 2 * h + 1;
    auto byte_at = [&](int b) -> uint32_t {
      if (b < 29) return (mn[b >> 2] >> (8 * (b & 3))) & 0xFFu;
      if (b < 58) { const int q = b - 29; return (mx[q >> 2] >> (8 * (q & 3))) & 0xFFu; }
      const int q = b - 58;
      return (dg[q >> 2] >> (8 * (q & 3))) & 0xFFu;
    };
    lo = byte_at(b0);
    hi = byte_at(b1);
    d16[h] = (uint16_t)(lo | (hi << 8));
  }
}

// SHA-256 state of the leaf message 0x00 | P | share for a 512-B share at
// `src` (16-B aligned), P = share[0:29] when q0 else the parity namespace.
// ns receives share[0:29] (zero padded to 8 dwords) for the caller's tables.
__device__ __forceinline__ void share_leaf_sha256(const uint4* src, bool q0, uint32_t (&st)[8],
                                                  uint32_t (&ns)[8]) {
  uint4 cur[8];
  auto stage = [&](int sg) {
#pragma unroll
    for (int q = 0; q < 8; q++) cur[q] = src[8 * sg + q];
  };
  // one SHA block from 5 consecutive uint4 (dwords 16b-8 .. 16b+8 of the share)
  auto mid_block = [&](const uint4& u0, const uint4& u1, const uint4& u2, const uint4& u3, const uint4& u4) {
    const uint32_t d[20] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w, u2.x, u2.y,
                            u2.z, u2.w, u3.x, u3.y, u3.z, u3.w, u4.x, u4.y, u4.z, u4.w};
    uint32_t m[16];
#pragma unroll
    for (int j = 0; j < 16; j++) m[j] = __builtin_amdgcn_perm(d[j], d[j + 1], 0x06070001u);
    sha256_compress(st, m);
  };
  sha256_init(st);
  stage(0);
  {  // block 0: 0x00 | P(29) | share[0:34]
    uint32_t m[16];
    const uint4 q0v = cur[0], q1v = cur[1], q2v = cur[2];
    const uint32_t d[12] = {q0v.x, q0v.y, q0v.z, q0v.w, q1v.x, q1v.y,
                            q1v.z, q1v.w, q2v.x, q2v.y, q2v.z, q2v.w};
#pragma unroll
    for (int j = 0; j < 7; j++) ns[j] = d[j];
    ns[7] = d[7] & 0xFFu;
#pragma unroll
    for (int j = 8; j < 16; j++) m[j] = __builtin_amdgcn_perm(d[j - 8], d[j - 7], 0x06070001u);
    const uint32_t m7lo = __builtin_amdgcn_perm(d[0], d[0], (PZ << 24) | (PZ << 16) | 0x0001u);
    if (q0) {
      m[0] = __builtin_amdgcn_perm(d[0], d[0], (PZ << 24) | 0x000102u);
#pragma unroll
      for (int j = 1; j <= 6; j++) m[j] = __builtin_amdgcn_perm(d[j - 1], d[j], 0x07000102u);
      m[7] = __builtin_amdgcn_perm(d[6], d[7], (0x0700u << 16) | (PZ << 8) | PZ) | m7lo;
      sha256_compress(st, m);
    } else {
      // parity leaf (wave-uniform): words 0..6 are the constant prefix
      // 0x00 | 0xFF*27, so rounds 0..6 fold at compile time (own call site)
      m[0] = 0x00FFFFFFu;
#pragma unroll
      for (int j = 1; j <= 6; j++) m[j] = 0xFFFFFFFFu;
      m[7] = 0xFFFF0000u | m7lo;
      sha256_compress_t<true>(st, m);
    }
  }
  mid_block(cur[2], cur[3], cur[4], cur[5], cur[6]);  // block 1
  uint4 prev0 = cur[6], prev1 = cur[7];
#pragma unroll 1
  for (int s2 = 1; s2 <= 3; s2++) {  // blocks 2 s2 and 2 s2 + 1
    stage(s2);
    mid_block(prev0, prev1, cur[0], cur[1], cur[2]);
    mid_block(cur[2], cur[3], cur[4], cur[5], cur[6]);
    prev0 = cur[6];
    prev1 = cur[7];
  }
  {  // block 8: share[482:512] | 0x80 | zeros | bit length
    uint32_t m[16];
    const uint32_t d[8] = {prev0.x, prev0.y, prev0.z, prev0.w, prev1.x, prev1.y, prev1.z, prev1.w};
#pragma unroll
    for (int j = 0; j < 7; j++) m[j] = __builtin_amdgcn_perm(d[j], d[j + 1], 0x06070001u);
    m[7] = __builtin_amdgcn_perm(d[7], d[7], (0x0607u << 16) | (PZ << 8) | PZ) | 0x8000u;
#pragma unroll
    for (int j = 8; j < 15; j++) m[j] = 0u;
    m[15] = 542u * 8u;
    sha256_compress_t<true>(st, m);  // words 8..15 constant: their schedule terms fold
  }
}

}  // namespace dagpu
