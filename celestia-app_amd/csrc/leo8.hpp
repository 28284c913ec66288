// leo8.hpp -- Leopard GF(2^8) butterflies and multiplies shared by the encode
// (rs_gf8.hip) and decode (rs_decode.hip) kernels.  Restates the element-wise
// operations of klauspost/reedsolomon v1.11.8 leopard8.go (mulAdd8/refMulAdd8,
// ifftDIT28, fftDIT28, mulgf8) on 4 packed bytes per lane.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf_const.hpp"

namespace dagpu {

#ifndef DAGPU_MUL3
#define DAGPU_MUL3 0
#endif

// 8-entry byte-table lookup: table = {lo (entries 0..3), hi (entries 4..7)}.
// The hi dword is moved into the result register right before the v_perm in
// ONE asm statement, so it is never hoisted or kept live (gfx950 VOP3 reads at
// most one scalar operand).  Not volatile: the per-lane index is an input, so
// only truly identical lookups can be merged.
__device__ __forceinline__ uint32_t perm8(uint32_t lo, uint32_t hi, uint32_t idx) {
  uint32_t r;
  asm("v_mov_b32 %0, %2\n\tv_perm_b32 %0, %0, %3, %1" : "=&v"(r) : "v"(idx), "s"(hi), "s"(lo));
  return r;
}

// x ^= y * exp(log_m) for a COMPILE-TIME log_m  (leopard8.go mulAdd8 /
// refMulAdd8).  DAGPU_MUL3 = 0: 4 x 2-bit lookups (7 index ops, 4 v_perm,
// 2 v_bitop3); = 1: 3/3/2-bit lookups (5 index ops, 2 v_mov, 3 v_perm,
// v_bitop3 + v_xor).
__device__ __forceinline__ void gf8_muladd(uint32_t& x, uint32_t y, const int lm) {
#if DAGPU_MUL3
  const uint32_t p0 = perm8(kGf8.t8[lm][0], kGf8.t8[lm][1], y & 0x07070707u);
  const uint32_t p1 = perm8(kGf8.t8[lm][2], kGf8.t8[lm][3], (y >> 3) & 0x07070707u);
  const uint32_t p2 = __builtin_amdgcn_perm(kGf8.t8[lm][4], kGf8.t8[lm][4], (y >> 6) & 0x03030303u);
  x = __builtin_amdgcn_bitop3_b32(x, p0, p1, 0x96) ^ p2;
#else
  const uint32_t p0 = __builtin_amdgcn_perm(kGf8.t[0][lm], kGf8.t[0][lm], y & 0x03030303u);
  const uint32_t p1 = __builtin_amdgcn_perm(kGf8.t[1][lm], kGf8.t[1][lm], (y >> 2) & 0x03030303u);
  const uint32_t p2 = __builtin_amdgcn_perm(kGf8.t[2][lm], kGf8.t[2][lm], (y >> 4) & 0x03030303u);
  const uint32_t p3 = __builtin_amdgcn_perm(kGf8.t[3][lm], kGf8.t[3][lm], (y >> 6) & 0x03030303u);
  x = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(x, p0, p1, 0x96), p2, p3, 0x96);
#endif
}

// Raw buffer resource over [base, base + 2^31) built from wave-uniform values
// (guide T8/T20): every shard access is buffer_load/store with voffset = lane
// column and soffset = shard offset (SGPR), so no per-shard VGPR address.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  const uint64_t p = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  void* bp = (void*)(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(bp, (short)0, 0x7FFFFFFF, 0x00020000);
}

// ifftDIT28: y ^= x; x ^= y*log_m (multiply skipped when log_m == 255)
__device__ __forceinline__ void ifft2(uint32_t& x, uint32_t& y, const int lm) {
  y ^= x;
  if (lm != kGf8Mod) gf8_muladd(x, y, lm);
}
// fftDIT28: x ^= y*log_m; y ^= x
__device__ __forceinline__ void fft2(uint32_t& x, uint32_t& y, const int lm) {
  if (lm != kGf8Mod) gf8_muladd(x, y, lm);
  y ^= x;
}


}  // namespace dagpu
