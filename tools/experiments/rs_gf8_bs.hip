// EXPERIMENT (not built): bit-sliced k=128 encoder.  Measured on MI355X: VALU
// instructions 250M -> 108M per launch, but 1.6x SLOWER (rs_row 0.40 -> 0.63 ms,
// rs_col 0.67 -> 1.08 ms): 205 VGPRs = one 8-wave workgroup per CU, and the two
// LDS transposes (32 barriers) serialise its load and compute phases
// (SQ_WAIT_INST_ANY 219M -> 500M).  Needs gf_const.hpp bscnt/bsidx tables.
// rs_gf8_bs.hip -- bit-sliced Leopard GF(2^8) encode for k = 128 on gfx950.
//
// Same transform as rs_gf8.hip (klauspost/reedsolomon v1.11.8 leopard8.go
// ifftDITEncoder8 + fftDIT8, the codec rsmt2d v0.11.0 calls 3k times per
// square), computed on BIT PLANES: a thread owns one 32-byte column group of a
// vector, and each of its elements is held as 8 dwords where dword p carries bit
// p of all 32 bytes.  Multiplication by a fixed field element is GF(2)-linear,
// so x ^= c*y becomes, per output plane, the XOR of the input planes selected by
// c's 8x8 bit matrix (compile-time: every skew folds into an XOR schedule,
// ~2.5 three-input XORs per plane).  A butterfly on 32 bytes costs ~28 VALU
// ops instead of ~104 with per-byte v_perm table lookups.
//
// k = 128 elements x 8 planes do not fit one thread, so eight waves share a
// column group: in the "block" layout wave q holds elements 16q .. 16q+15
// (index bits 0-3 local); an 8x8 block transpose through LDS moves to the
// "transposed" layout where wave q holds the elements whose bits 1-3 equal q
// (bits 0 and 4-6 local).  IFFT layers 1..8 and FFT layers 8..1 run in block
// layout with skews that depend on q (one code path per wave, wave-uniform
// switch); IFFT layers 16..64 and FFT layers 64..16 run transposed, where the
// skews do not depend on q.
//   load 32 B x 16 elements -> bit-transpose -> block IFFT -> LDS transpose ->
//   transposed IFFT/FFT -> LDS transpose -> block FFT -> bit-transpose -> store
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"
#include "leo8.hpp"

namespace dagpu {

namespace {

constexpr int kBsK = 128;
constexpr int kBsE = 16;        // elements per thread
constexpr int kBsParts = 8;     // waves per column group
constexpr int kBsVecs = 4;      // vectors per workgroup (64 lanes = 4 vectors x 16 groups)

struct P8 {
  uint32_t p[8];
};

__device__ __forceinline__ uint32_t bx3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// x ^= exp(lm) * y on bit planes (lm compile-time after unrolling)
__device__ __forceinline__ void bs_muladd(P8& x, const P8& y, const int lm) {
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int n = kGf8.bscnt[lm][j];
    uint32_t acc = x.p[j];
#pragma unroll
    for (int t = 0; t < 8; t += 2) {
      if (t + 1 < n) acc = bx3(acc, y.p[kGf8.bsidx[lm][j][t]], y.p[kGf8.bsidx[lm][j][t + 1]]);
      else if (t < n) acc ^= y.p[kGf8.bsidx[lm][j][t]];
    }
    x.p[j] = acc;
  }
}

__device__ __forceinline__ void bs_xor(P8& y, const P8& x) {
#pragma unroll
  for (int j = 0; j < 8; j++) y.p[j] ^= x.p[j];
}

// ifftDIT28 / fftDIT28 on bit planes (multiply skipped when lm == 255)
__device__ __forceinline__ void bs_ifft2(P8& x, P8& y, const int lm) {
  bs_xor(y, x);
  if (lm != kGf8Mod) bs_muladd(x, y, lm);
}
__device__ __forceinline__ void bs_fft2(P8& x, P8& y, const int lm) {
  if (lm != kGf8Mod) bs_muladd(x, y, lm);
  bs_xor(y, x);
}

// 8x8 bit transpose in every byte lane of 8 dwords (an involution): afterwards
// dword p holds bit p of byte 4m+n at bit position 8n+m.
__device__ __forceinline__ void bit_transpose(P8& d) {
#pragma unroll
  for (int m = 0; m < 4; m++) {
    const uint32_t t = __builtin_amdgcn_bitop3_b32(d.p[m] >> 4, d.p[m + 4], 0x0F0F0F0Fu, 0x28);  // (a^b)&c
    d.p[m] ^= t << 4;
    d.p[m + 4] ^= t;
  }
#pragma unroll
  for (int mm = 0; mm < 4; mm++) {  // m = 0, 1, 4, 5
    const int m = mm + (mm & 2);
    const uint32_t t = __builtin_amdgcn_bitop3_b32(d.p[m] >> 2, d.p[m + 2], 0x33333333u, 0x28);
    d.p[m] ^= t << 2;
    d.p[m + 2] ^= t;
  }
#pragma unroll
  for (int m = 0; m < 8; m += 2) {
    const uint32_t t = __builtin_amdgcn_bitop3_b32(d.p[m] >> 1, d.p[m + 1], 0x55555555u, 0x28);
    d.p[m] ^= t << 1;
    d.p[m + 1] ^= t;
  }
}

// Block layout, wave Q (elements 16Q + j): IFFT radix-4 steps dist 1 and 4
// (ifftDITEncoder8, skew index K-1+iend).
template <int Q, int D>
__device__ __forceinline__ void block_ifft_step(P8 (&w)[kBsE]) {
#pragma unroll
  for (int r = 0; r < kBsE; r += 4 * D) {
    const int iend = 16 * Q + r + D;
    const int l01 = kGf8.skew[kBsK - 1 + iend];
    const int l02 = kGf8.skew[kBsK - 1 + iend + D];
    const int l23 = kGf8.skew[kBsK - 1 + iend + 2 * D];
#pragma unroll
    for (int i = r; i < r + D; i++) {
      bs_ifft2(w[i], w[i + D], l01);
      bs_ifft2(w[i + 2 * D], w[i + 3 * D], l23);
      bs_ifft2(w[i], w[i + 2 * D], l02);
      bs_ifft2(w[i + D], w[i + 3 * D], l02);
    }
  }
}

template <int Q>
__device__ __forceinline__ void block_ifft(P8 (&w)[kBsE]) {
  block_ifft_step<Q, 1>(w);
  block_ifft_step<Q, 4>(w);
}

// Block layout, wave Q: the distance-8 sub-layer of the FFT dist4 = 32 step
// (skew[16Q + 7] for both of its halves), the dist4 = 8 step and the final
// radix-2 layer (fftDIT8, skew index iend - 1).
template <int Q>
__device__ __forceinline__ void block_fft(P8 (&w)[kBsE]) {
  constexpr int l8 = kGf8.skew[16 * Q + 7];
#pragma unroll
  for (int j = 0; j < 8; j++) bs_fft2(w[j], w[j + 8], l8);
#pragma unroll
  for (int r = 0; r < kBsE; r += 8) {
    const int iend = 16 * Q + r + 2;
    const int l01 = kGf8.skew[iend - 1], l02 = kGf8.skew[iend + 1], l23 = kGf8.skew[iend + 3];
#pragma unroll
    for (int i = r; i < r + 2; i++) {
      bs_fft2(w[i], w[i + 4], l02);
      bs_fft2(w[i + 2], w[i + 6], l02);
      bs_fft2(w[i], w[i + 2], l01);
      bs_fft2(w[i + 4], w[i + 6], l23);
    }
  }
#pragma unroll
  for (int r = 0; r < kBsE; r += 2) bs_fft2(w[r], w[r + 1], kGf8.skew[16 * Q + r]);
}

// Transposed layout: slot s = (h << 1) | b0 holds element 16h + 2q + b0.
__device__ __forceinline__ void transposed_layers(P8 (&w)[kBsE]) {
  // IFFT radix-4 dist 16 (bits 4, 5), groups r = 64 g6
#pragma unroll
  for (int g6 = 0; g6 < 2; g6++) {
    const int iend = 64 * g6 + 16;
    const int l01 = kGf8.skew[kBsK - 1 + iend];
    const int l02 = kGf8.skew[kBsK - 1 + iend + 16];
    const int l23 = kGf8.skew[kBsK - 1 + iend + 32];
#pragma unroll
    for (int b0 = 0; b0 < 2; b0++) {
      const int sb = 8 * g6 + b0;
      bs_ifft2(w[sb], w[sb + 2], l01);
      bs_ifft2(w[sb + 4], w[sb + 6], l23);
      bs_ifft2(w[sb], w[sb + 4], l02);
      bs_ifft2(w[sb + 2], w[sb + 6], l02);
    }
  }
  {  // IFFT last layer, dist 64 (bit 6)
    constexpr int lm = kGf8.skew[kBsK - 1 + 64];
#pragma unroll
    for (int s = 0; s < 8; s++) bs_ifft2(w[s], w[s + 8], lm);
  }
  {  // FFT dist4 = 128, dist = 32: bit 6 then bit 5
    constexpr int l01 = kGf8.skew[31], l02 = kGf8.skew[63], l23 = kGf8.skew[95];
#pragma unroll
    for (int s = 0; s < 4; s++) {
      bs_fft2(w[s], w[s + 8], l02);
      bs_fft2(w[s + 4], w[s + 12], l02);
      bs_fft2(w[s], w[s + 4], l01);
      bs_fft2(w[s + 8], w[s + 12], l23);
    }
  }
#pragma unroll
  for (int gr = 0; gr < 4; gr++) {  // FFT dist4 = 32 step, first sub-layer (bit 4)
    const int l02 = kGf8.skew[32 * gr + 15];
#pragma unroll
    for (int b0 = 0; b0 < 2; b0++) bs_fft2(w[4 * gr + b0], w[4 * gr + b0 + 2], l02);
  }
}

// 8x8 block transpose between layouts: element (wave h, slot 2c + b0) <->
// (wave c, slot 2h + b0); one bit plane per LDS round.
__device__ __forceinline__ void lds_transpose(P8 (&w)[kBsE], uint32_t* lds, int q, int lane) {
  // lds[((dst * 8 + src) * 2 + b0) * 64 + lane]
#pragma unroll
  for (int p = 0; p < 8; p++) {
#pragma unroll
    for (int c = 0; c < kBsParts; c++)
#pragma unroll
      for (int b0 = 0; b0 < 2; b0++) lds[((c * kBsParts + q) * 2 + b0) * 64 + lane] = w[2 * c + b0].p[p];
    __syncthreads();
#pragma unroll
    for (int c = 0; c < kBsParts; c++)
#pragma unroll
      for (int b0 = 0; b0 < 2; b0++) w[2 * c + b0].p[p] = lds[((q * kBsParts + c) * 2 + b0) * 64 + lane];
    __syncthreads();
  }
}

// The whole per-wave program for part Q.  Each part is its own straight-line
// path (a shared body with a q-switch around the block phases made the
// register allocator merge eight large cases: 256 VGPRs + spills).
template <int Q>
__device__ __forceinline__ void run_part(const EncodeArgs& a, long first_vec, int lane, uint32_t* lds) {
  constexpr int q = Q;
  const int vv = lane >> 4, g = lane & 15;
  const long total = a.nsq * a.nvec;
  const bool active = first_vec + vv < total;
  const long sq0 = first_vec / a.nvec, vec0 = first_vec % a.nvec;  // the 4 vectors share one square
  const auto in_rsrc = make_rsrc(a.in + sq0 * a.in_sq_stride + vec0 * a.in_vec_stride);
  const uint32_t voff_in = active ? (uint32_t)(vv * a.in_vec_stride + g * 32) : (uint32_t)(g * 32);
  const uint32_t is = (uint32_t)a.in_shard_stride;
  const uint32_t ebase = 16u * (uint32_t)q;
  P8 w[kBsE];
#pragma unroll
  for (int j = 0; j < kBsE; j++) {
    const uint32_t so = (ebase + j) * is;
#pragma unroll
    for (int p = 0; p < 8; p++) w[j].p[p] = __builtin_amdgcn_raw_buffer_load_b32(in_rsrc, voff_in + 4 * p, so, 0);
  }
  if (a.copy && active) {
    const auto cp = make_rsrc(a.copy + sq0 * a.copy_sq_stride + vec0 * a.copy_vec_stride);
    const uint32_t voff = (uint32_t)(vv * a.copy_vec_stride + g * 32);
    const uint32_t cs = (uint32_t)a.copy_shard_stride;
#pragma unroll
    for (int j = 0; j < kBsE; j++)
#pragma unroll
      for (int p = 0; p < 8; p++)
        __builtin_amdgcn_raw_buffer_store_b32(w[j].p[p], cp, voff + 4 * p, (ebase + j) * cs, 0);
  }
#pragma unroll
  for (int j = 0; j < kBsE; j++) bit_transpose(w[j]);
  block_ifft<Q>(w);
  lds_transpose(w, lds, q, lane);
  transposed_layers(w);
  lds_transpose(w, lds, q, lane);
  block_fft<Q>(w);
#pragma unroll
  for (int j = 0; j < kBsE; j++) bit_transpose(w[j]);
  if (!active) return;
  const auto out_rsrc = make_rsrc(a.out + sq0 * a.out_sq_stride + vec0 * a.out_vec_stride);
  const uint32_t voff = (uint32_t)(vv * a.out_vec_stride + g * 32);
  const uint32_t os = (uint32_t)a.out_shard_stride;
  if (a.mismatch) {  // prerepairSanityCheck: parity must equal Encode(data)
    uint32_t diff = 0;
#pragma unroll
    for (int j = 0; j < kBsE; j++)
#pragma unroll
      for (int p = 0; p < 8; p++)
        diff |= w[j].p[p] ^ __builtin_amdgcn_raw_buffer_load_b32(out_rsrc, voff + 4 * p, (ebase + j) * os, 0);
    if (diff) atomicOr(&a.mismatch[sq0], a.mismatch_bit);
    return;
  }
#pragma unroll
  for (int j = 0; j < kBsE; j++)
#pragma unroll
    for (int p = 0; p < 8; p++)
      __builtin_amdgcn_raw_buffer_store_b32(w[j].p[p], out_rsrc, voff + 4 * p, (ebase + j) * os, 0);
}


// One workgroup = 8 waves (parts) x 64 lanes (4 vectors x 16 column groups).
__global__ __launch_bounds__(512) void leo8_encode_bs128_kernel(EncodeArgs a) {
  __shared__ uint32_t lds[kBsParts * kBsParts * 2 * 64];  // 32 KiB
  const long first_vec = (long)blockIdx.x * kBsVecs;
  const int lane = threadIdx.x & 63;
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
    case 0: run_part<0>(a, first_vec, lane, lds); break;
    case 1: run_part<1>(a, first_vec, lane, lds); break;
    case 2: run_part<2>(a, first_vec, lane, lds); break;
    case 3: run_part<3>(a, first_vec, lane, lds); break;
    case 4: run_part<4>(a, first_vec, lane, lds); break;
    case 5: run_part<5>(a, first_vec, lane, lds); break;
    case 6: run_part<6>(a, first_vec, lane, lds); break;
    default: run_part<7>(a, first_vec, lane, lds); break;
  }
}

}  // namespace

// k = 128 squares: bit-sliced kernel when the vector count per square is a
// multiple of 4 and shards are exactly 512 B (the square pipeline); the caller
// falls back to the per-byte kernel otherwise.
bool leo8_bs128_applicable(const EncodeArgs& a) {
  return a.shard_bytes == 512 && a.nchunk == 1 && a.nvec % kBsVecs == 0 && !a.vec_flags;
}

hipError_t launch_leo8_encode_bs128(const EncodeArgs& a, hipStream_t s) {
  const long blocks = a.nsq * a.nvec / kBsVecs;
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(leo8_encode_bs128_kernel, dim3((unsigned)blocks), dim3(512), 0, s, a);
  return hipGetLastError();
}

}  // namespace dagpu
