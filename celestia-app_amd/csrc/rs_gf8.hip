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

#include "kernels.hpp"
#include "leo8.hpp"

namespace dagpu {

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
  if (a.vec_flags && a.vec_flags[sv] == 0) return;  // uniform
  const uint32_t col = (uint32_t)chunk * 512u + threadIdx.x * 4u;  // byte offset inside shard
  if (col >= (uint32_t)a.shard_bytes) return;

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
  if (a.mismatch) {  // prerepairSanityCheck: parity must equal Encode(data)
    uint32_t diff = 0;
#pragma unroll
    for (int i = 0; i < K; i++) diff |= w[i] ^ __builtin_amdgcn_raw_buffer_load_b32(out_rsrc, col, i * out_stride, 0);
    if (diff) atomicOr(&a.mismatch[sq], a.mismatch_bit);
    return;
  }
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
