// nmt_node.hpp -- NMT node helpers shared by the square pipeline (nmt.hip) and
// the generic forest engine (nmt_forest.hip).  A node in registers is 24 dwords
// in memory byte order: minNs (29 B zero padded to 8 dwords), maxNs, digest.
// HashNode message layout follows nmt v0.20.0 NmtHasher.HashNode (mirror:
// test/util/malicious/hasher.go:271-297): 0x01 | left(90) | right(90).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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

// Window form: OR part P (8 dwords fetched through get(P, i)) placed at message
// byte OFF into the 16-word window of SHA block B.  Only dwords that land in the
// window are fetched, so each block pulls just the source words it needs.
template <int OFF, int B, int P, class G>
__device__ __forceinline__ void put_part_win(uint32_t (&m)[16], const G& get) {
  constexpr int al = OFF & 3;
  constexpr int d0 = OFF >> 2;
  constexpr int lo = 16 * B, hi = 16 * B + 16;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int p0 = d0 + i, p1 = d0 + i + 1;
    const bool in0 = p0 >= lo && p0 < hi;
    const bool in1 = al != 0 && p1 >= lo && p1 < hi;
    if (in0 || in1) {
      const uint32_t v = get(P, i);
      if (in0) m[p0 - lo] |= al ? (v << (8 * al)) : v;
      if (in1) m[p1 - lo] |= v >> (32 - 8 * al);
    }
  }
}

// NMT HashNode message 0x01 | L.min | L.max | L.d | R.min | R.max | R.d
// (181 B, 3 SHA blocks).  get(P, i): P = 0..5 -> Lmn, Lmx, Ld, Rmn, Rmx, Rd.
template <class G>
__device__ __forceinline__ void sha_node_msg(const G& get, uint32_t (&st)[8]) {
  sha256_init(st);
#pragma unroll
  for (int blk = 0; blk < 3; blk++) {
    uint32_t m[16];
#pragma unroll
    for (int j = 0; j < 16; j++) m[j] = 0;
    if (blk == 0) m[0] = 0x01u;
    if (blk == 0) { put_part_win<1, 0, 0>(m, get); put_part_win<30, 0, 1>(m, get); put_part_win<59, 0, 2>(m, get); }
    if (blk == 1) {
      put_part_win<59, 1, 2>(m, get); put_part_win<91, 1, 3>(m, get); put_part_win<120, 1, 4>(m, get);
    }
    if (blk == 2) {
      put_part_win<120, 2, 4>(m, get); put_part_win<149, 2, 5>(m, get);
      m[45 - 32] |= 0x80u << 8;  // byte 181
    }
#pragma unroll
    for (int j = 0; j < 16; j++) m[j] = bswap32(m[j]);
    if (blk == 2) { m[14] = 0; m[15] = 181u * 8u; }
    sha256_compress(st, m);
  }
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
      sha256_compress(st, m);
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
    sha256_compress(st, m);
  }
}

}  // namespace dagpu
