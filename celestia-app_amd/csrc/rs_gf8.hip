// rs_gf8.hip -- Leopard GF(2^8) Reed-Solomon encode on gfx950.
//
// Replaces the hot loop of klauspost/reedsolomon v1.11.8 leopardFF8.encode
// (ifftDITEncoder8 + fftDIT8), which rsmt2d v0.11.0 ComputeExtendedDataSquare
// calls 3k times per square (pkg/da/data_availability_header.go:74, codec from
// pkg/appconsts/global_consts.go:92).
//
// Mapping: every byte column of a 512-B share is an independent GF(2^8)
// codeword, so one thread owns one DWORD column (4 byte lanes) of one vector
// (row or column of the square) and keeps all k shard dwords of that column in
// VGPRs.  The whole IFFT_m -> FFT_m transform then runs register-resident, fully
// unrolled per k (template), every skew constant folded to an immediate.
// HBM traffic is the algorithmic minimum: each data dword read once, each parity
// dword written once (plus the Q0 copy in the row pass, which replaces the
// ODS->EDS memcpy).  Loads/stores are 256 B contiguous per wave instruction.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf_const.hpp"
#include "kernels.hpp"

namespace dagpu {

// x ^= y * exp(log_m)    (leopard8.go mulAdd8 / refMulAdd8): 7 index ops,
// 4 v_perm_b32 (one SGPR table each), 2 v_bitop3 xor3.
__device__ __forceinline__ void gf8_muladd(uint32_t& x, uint32_t y, const int lm) {
  const uint32_t p0 = __builtin_amdgcn_perm(kGf8.t[0][lm], kGf8.t[0][lm], y & 0x03030303u);
  const uint32_t p1 = __builtin_amdgcn_perm(kGf8.t[1][lm], kGf8.t[1][lm], (y >> 2) & 0x03030303u);
  const uint32_t p2 = __builtin_amdgcn_perm(kGf8.t[2][lm], kGf8.t[2][lm], (y >> 4) & 0x03030303u);
  const uint32_t p3 = __builtin_amdgcn_perm(kGf8.t[3][lm], kGf8.t[3][lm], (y >> 6) & 0x03030303u);
  x = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(x, p0, p1, 0x96), p2, p3, 0x96);
}

// Raw buffer resource over [base, base + 2^31): all offsets used by one block
// (k shards at stride <= 2k*512 B) stay far below that.
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

// ifftDITEncoder8 with m = mtrunc = K, skewLUT = fftSkew8[m-1:]
template <int K, int DIST>
__device__ __forceinline__ void ifft_enc_layers(uint32_t (&w)[K]) {
  if constexpr (DIST * 4 <= K) {
#pragma unroll
    for (int r = 0; r < K; r += DIST * 4) {
      const int iend = r + DIST;
      const int l01 = kGf8.skew[K - 1 + iend];
      const int l02 = kGf8.skew[K - 1 + iend + DIST];
      const int l23 = kGf8.skew[K - 1 + iend + 2 * DIST];
#pragma unroll
      for (int i = r; i < iend; i++) {
        ifft2(w[i], w[i + DIST], l01);
        ifft2(w[i + 2 * DIST], w[i + 3 * DIST], l23);
        ifft2(w[i], w[i + 2 * DIST], l02);
        ifft2(w[i + DIST], w[i + 3 * DIST], l02);
      }
    }
    ifft_enc_layers<K, DIST * 4>(w);
  } else if constexpr (DIST < K) {
    const int lm = kGf8.skew[K - 1 + DIST];
#pragma unroll
    for (int i = 0; i < DIST; i++) ifft2(w[i], w[i + DIST], lm);
  }
}

// fftDIT8 with mtrunc = m = K, skewLUT = fftSkew8[:] (index iend-1)
template <int K, int DIST4>
__device__ __forceinline__ void fft_layers(uint32_t (&w)[K]) {
  constexpr int DIST = DIST4 >> 2;
  if constexpr (DIST != 0) {
#pragma unroll
    for (int r = 0; r < K; r += DIST4) {
      const int iend = r + DIST;
      const int l01 = kGf8.skew[iend - 1];
      const int l02 = kGf8.skew[iend + DIST - 1];
      const int l23 = kGf8.skew[iend + 2 * DIST - 1];
#pragma unroll
      for (int i = r; i < iend; i++) {
        fft2(w[i], w[i + 2 * DIST], l02);
        fft2(w[i + DIST], w[i + 3 * DIST], l02);
        fft2(w[i], w[i + DIST], l01);
        fft2(w[i + 2 * DIST], w[i + 3 * DIST], l23);
      }
    }
    fft_layers<K, DIST>(w);
  } else if constexpr (DIST4 == 2) {
#pragma unroll
    for (int r = 0; r < K; r += 2) fft2(w[r], w[r + 1], kGf8.skew[r]);
  }
}

// One block = 128 threads = 512 bytes (128 dword columns) of one vector.
// Block index (flattened) = (square * nvec + vec) * nchunk + chunk.
// Occupancy target per k: k=128 holds 128 data VGPRs per lane and the
// scheduler wants ~230 at full unroll, so k=128 runs at 2 waves/SIMD (3 spills);
// smaller k fit 4-8 waves.
template <int K>
struct EncOcc { static constexpr int waves = K >= 128 ? 2 : (K >= 64 ? 4 : 8); };

template <int K>
__global__ __launch_bounds__(128)
__attribute__((amdgpu_waves_per_eu(EncOcc<K>::waves, 8))) void leo8_encode_kernel(EncodeArgs a) {
  const long blk = blockIdx.x;
  const int chunk = (int)(blk % a.nchunk);
  const long sv = blk / a.nchunk;
  const long vec = sv % a.nvec;
  const long sq = sv / a.nvec;
  const uint32_t col = (uint32_t)chunk * 512u + threadIdx.x * 4u;  // byte offset inside shard
  if (col >= (uint32_t)a.shard_bytes) return;

  // Buffer descriptors built from wave-uniform values (guide T8/T20): each
  // shard access is buffer_load/store with voffset = col (shared by all k
  // shards) and soffset = i*stride (SGPR), so no per-shard VGPR address.
  const auto in_rsrc = make_rsrc(a.in + sq * a.in_sq_stride + vec * a.in_vec_stride);
  const uint32_t in_stride = (uint32_t)a.in_shard_stride;
  uint32_t w[K];
#pragma unroll
  for (int i = 0; i < K; i++)
    w[i] = __builtin_amdgcn_raw_buffer_load_b32(in_rsrc, col, i * in_stride, 0);

  if (a.copy) {
    const auto cp_rsrc = make_rsrc(a.copy + sq * a.copy_sq_stride + vec * a.copy_vec_stride);
    const uint32_t cp_stride = (uint32_t)a.copy_shard_stride;
#pragma unroll
    for (int i = 0; i < K; i++) __builtin_amdgcn_raw_buffer_store_b32(w[i], cp_rsrc, col, i * cp_stride, 0);
  }

  ifft_enc_layers<K, 1>(w);
  fft_layers<K, K>(w);

  const auto out_rsrc = make_rsrc(a.out + sq * a.out_sq_stride + vec * a.out_vec_stride);
  const uint32_t out_stride = (uint32_t)a.out_shard_stride;
#pragma unroll
  for (int i = 0; i < K; i++) __builtin_amdgcn_raw_buffer_store_b32(w[i], out_rsrc, col, i * out_stride, 0);
}

template <int K>
static hipError_t launch_k(const EncodeArgs& a, hipStream_t s) {
  const long blocks = a.nsq * a.nvec * a.nchunk;
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(leo8_encode_kernel<K>, dim3((unsigned)blocks), dim3(128), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_leo8_encode(int k, const EncodeArgs& a, hipStream_t s) {
  switch (k) {
    case 1: return launch_k<1>(a, s);
    case 2: return launch_k<2>(a, s);
    case 4: return launch_k<4>(a, s);
    case 8: return launch_k<8>(a, s);
    case 16: return launch_k<16>(a, s);
    case 32: return launch_k<32>(a, s);
    case 64: return launch_k<64>(a, s);
    case 128: return launch_k<128>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dagpu
