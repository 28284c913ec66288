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

// Variant choice measured with tools/rs_bench2.cpp (k=128, 64-square batch,
// row/col pass ms): 2-bit mul unsplit 0.399/0.769, split 0.368/0.745,
// 3/3/2-bit mul unsplit 0.371/0.719 (chosen), split 0.421/0.822.
#ifndef DAGPU_MUL3
#define DAGPU_MUL3 1
#endif
#ifndef DAGPU_ENC_SPLIT
#define DAGPU_ENC_SPLIT 0
#endif
#ifndef DAGPU_ENC_WAVES128
#define DAGPU_ENC_WAVES128 2
#endif
// Scheduling fence after every radix-4 group at k = 128 (keeps the scheduler
// from interleaving groups): rs_bench2 row/col 0.382/0.744 -> 0.367/0.718 ms.
#ifndef DAGPU_ENC_FENCE
#define DAGPU_ENC_FENCE 1
#endif
#if DAGPU_ENC_FENCE
#define ENC_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define ENC_FENCE() ((void)0)
#endif

#include "kernels.hpp"
#include "leo8.hpp"

namespace dagpu {

// ifftDITEncoder8 (m = mtrunc = K, skewLUT = fftSkew8[m-1:], i.e. skew offset
// IO = K; the reverse fill's IFFT has IO = 0) restricted to the E elements
// [BASE, BASE+E) one thread holds: every radix-4 group that fits inside the
// slice; the trailing radix-2 layer only when the slice is the whole vector.
template <int K, int IO, int E, int BASE, int DIST>
__device__ __forceinline__ void ifft_enc_local(uint32_t (&w)[E]) {
  if constexpr (DIST * 4 <= E) {
#pragma unroll
    for (int r = 0; r < E; r += DIST * 4) {
      const int iend = BASE + r + DIST;  // global index
      const int l01 = kGf8.skew[IO - 1 + iend];
      const int l02 = kGf8.skew[IO - 1 + iend + DIST];
      const int l23 = kGf8.skew[IO - 1 + iend + 2 * DIST];
#pragma unroll
      for (int i = r; i < r + DIST; i++) {
        ifft2(w[i], w[i + DIST], l01);
        ifft2(w[i + 2 * DIST], w[i + 3 * DIST], l23);
        ifft2(w[i], w[i + 2 * DIST], l02);
        ifft2(w[i + DIST], w[i + 3 * DIST], l02);
      }
      if constexpr (K >= 128) ENC_FENCE();
    }
    ifft_enc_local<K, IO, E, BASE, DIST * 4>(w);
  } else if constexpr (E == K && DIST < K) {
    const int lm = kGf8.skew[IO - 1 + DIST];
#pragma unroll
    for (int i = 0; i < DIST; i++) ifft2(w[i], w[i + DIST], lm);
  }
}

// fftDIT8 (mtrunc = m, skewLUT = fftSkew8[:], index iend-1: skew offset FO = 0;
// the reverse fill's FFT has FO = K) restricted to the slice [BASE, BASE+E):
// radix-4 steps with dist4 <= E, then the final radix-2 layer when the
// transform size is 2 * 4^j.
template <int FO, int E, int BASE, int DIST4>
__device__ __forceinline__ void fft_local(uint32_t (&w)[E]) {
  constexpr int DIST = DIST4 >> 2;
  if constexpr (DIST != 0) {
#pragma unroll
    for (int r = 0; r < E; r += DIST4) {
      const int iend = BASE + r + DIST;
      const int l01 = kGf8.skew[FO + iend - 1];
      const int l02 = kGf8.skew[FO + iend + DIST - 1];
      const int l23 = kGf8.skew[FO + iend + 2 * DIST - 1];
#pragma unroll
      for (int i = r; i < r + DIST; i++) {
        fft2(w[i], w[i + 2 * DIST], l02);
        fft2(w[i + DIST], w[i + 3 * DIST], l02);
        fft2(w[i], w[i + DIST], l01);
        fft2(w[i + 2 * DIST], w[i + 3 * DIST], l23);
      }
      if constexpr (E >= 128) ENC_FENCE();
    }
    fft_local<FO, E, BASE, DIST>(w);
  } else if constexpr (DIST4 == 2) {
#pragma unroll
    for (int r = 0; r < E; r += 2) fft2(w[r], w[r + 1], kGf8.skew[FO + BASE + r]);
  }
}

// Encode one dword column of one vector, half HH of H.  With H == 2 (k = 128)
// the 128 elements of a column are split over two thread halves of the same
// workgroup (waves 0-1: elements 0..63, waves 2-3: 64..127; each half runs its
// own code with its own folded skews).  All layers are local except the
// IFFT's last radix-2 layer (distance 64) and the FFT's first sub-layer
// (distance 64); they are adjacent, so one chunked LDS exchange gives each half
// both operands and each computes the pair result it keeps.
template <int K, int H, int HH, bool REV>
__device__ __forceinline__ void encode_half(const EncodeArgs& a, long sq, long vec, int t, bool active,
                                            uint32_t (*xch)[16][128]) {
  constexpr int E = K / H;
  // inactive columns (shard < 512 B) read column 0 (valid memory, result
  // unused) so the loads stay branch-free; they skip every store
  const uint32_t col = active ? (uint32_t)t * 4u : 0u;
  const auto in_rsrc = make_rsrc(a.in + sq * a.in_sq_stride + vec * a.in_vec_stride);
  const uint32_t in_stride = (uint32_t)a.in_shard_stride;
  uint32_t w[E];
#pragma unroll
  for (int j = 0; j < E; j++)
    w[j] = __builtin_amdgcn_raw_buffer_load_b32(in_rsrc, col, (HH * E + j) * in_stride, 0);

  if (a.copy && active) {
    const auto cp_rsrc = make_rsrc(a.copy + sq * a.copy_sq_stride + vec * a.copy_vec_stride);
    const uint32_t cp_stride = (uint32_t)a.copy_shard_stride;
#pragma unroll
    for (int j = 0; j < E; j++)
      __builtin_amdgcn_raw_buffer_store_b32(w[j], cp_rsrc, col, (HH * E + j) * cp_stride, 0);
  }

  if constexpr (H == 1) {
    ifft_enc_local<K, REV ? 0 : K, K, 0, 1>(w);
    fft_local<REV ? K : 0, K, 0, K>(w);
  } else {
    static_assert(K == 128 && H == 2 && !REV, "split encode is specialised for the k = 128 forward encode");
    ifft_enc_local<K, K, E, HH * E, 1>(w);  // distances 1..32 (radix-4 dist 1, 4, 16)
    constexpr int L1 = kGf8.skew[K - 1 + 64];  // IFFT trailing layer, pairs (i, i+64)
    constexpr int L2 = kGf8.skew[63];          // FFT first radix-4 (dist 32), sub-layer (i, i+64)
#pragma unroll
    for (int c = 0; c < E / 16; c++) {
#pragma unroll
      for (int q = 0; q < 16; q++) xch[HH][q][t] = w[16 * c + q];
      __syncthreads();
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const uint32_t o = xch[1 - HH][q][t];
        uint32_t x = HH == 0 ? w[16 * c + q] : o;
        uint32_t y = HH == 0 ? o : w[16 * c + q];
        ifft2(x, y, L1);  // y ^= x; x ^= y*L1
        fft2(x, y, L2);   // x ^= y*L2; y ^= x
        w[16 * c + q] = HH == 0 ? x : y;
      }
      __syncthreads();
    }
    // rest of the first FFT radix-4 step: (i, i+32) lower with skew[31],
    // (i+64, i+96) upper with skew[95]
    constexpr int LA = HH == 0 ? kGf8.skew[31] : kGf8.skew[95];
#pragma unroll
    for (int i = 0; i < 32; i++) fft2(w[i], w[i + 32], LA);
    fft_local<0, E, HH * E, 32>(w);  // radix-4 dist 8, 2 (dist4 32, 8) + final radix-2
  }

  if (!active) return;
  const auto out_rsrc = make_rsrc(a.out + sq * a.out_sq_stride + vec * a.out_vec_stride);
  const uint32_t out_stride = (uint32_t)a.out_shard_stride;
  if (a.mismatch) {  // prerepairSanityCheck: parity must equal Encode(data)
    uint32_t diff = 0;
#pragma unroll
    for (int j = 0; j < E; j++)
      diff |= w[j] ^ __builtin_amdgcn_raw_buffer_load_b32(out_rsrc, col, (HH * E + j) * out_stride, 0);
    if (diff) {
      atomicOr(&a.mismatch[sq], a.mismatch_bit);
      if (a.mismatch_vec) a.mismatch_vec[sq * a.nvec + vec] = 1;
    }
    return;
  }
  if (a.out_present) {  // Repair fill: store the missing shards of the out half, compare given ones
    uint32_t diff = 0;
#pragma unroll
    for (int j = 0; j < E; j++) {
      if (fill_given(a, sq, vec, HH * E + j))  // wave-uniform
        diff |= w[j] ^ __builtin_amdgcn_raw_buffer_load_b32(out_rsrc, col, (HH * E + j) * out_stride, 0);
      else
        __builtin_amdgcn_raw_buffer_store_b32(w[j], out_rsrc, col, (HH * E + j) * out_stride, 0);
    }
    if (diff) a.redo[sq * a.nvec + vec] = 1;
    return;
  }
#pragma unroll
  for (int j = 0; j < E; j++)
    __builtin_amdgcn_raw_buffer_store_b32(w[j], out_rsrc, col, (HH * E + j) * out_stride, 0);
}

template <int K>
struct EncSplit { static constexpr int H = (K >= 128 && DAGPU_ENC_SPLIT) ? 2 : 1; };
template <int K>
struct EncOcc { static constexpr int waves = K >= 128 ? DAGPU_ENC_WAVES128 : (K >= 64 ? 3 : 8); };

// One block = 128*H threads = 512 bytes (128 dword columns) of one vector.
// Block index (flattened) = (square * nvec + vec) * nchunk + chunk.
template <int K, bool REV>
__global__ __launch_bounds__(128 * EncSplit<K>::H)
__attribute__((amdgpu_waves_per_eu(EncOcc<K>::waves, 8))) void leo8_encode_kernel(EncodeArgs a) {
  constexpr int H = REV ? 1 : EncSplit<K>::H;
  const long blk = blockIdx.x;
  const int chunk = (int)(blk % a.nchunk);
  const long sv = blk / a.nchunk;
  const long vec = sv % a.nvec;
  const long sq = sv / a.nvec;
  if (vec_skipped(a, sv)) return;  // uniform
  const int t = threadIdx.x & 127;
  // chunks of 512 B: shift the column window inside the shard
  EncodeArgs b = a;
  const long coff = (long)chunk * 512;
  b.in += coff;
  b.out += coff;
  if (b.copy) b.copy += coff;
  const bool active = coff + t * 4 < a.shard_bytes;
  if constexpr (H == 1) {
    if (!active) return;
    encode_half<K, 1, 0, REV>(b, sq, vec, t, true, nullptr);
  } else {
    // every thread reaches the exchange barriers; inactive columns skip memory
    __shared__ uint32_t xch[2][16][128];
    const int h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 7);  // wave-uniform
    if (h == 0) encode_half<K, H, 0, false>(b, sq, vec, t, active, xch);
    else encode_half<K, H, 1, false>(b, sq, vec, t, active, xch);
  }
}

template <int K>
static hipError_t launch_k(const EncodeArgs& a, hipStream_t s) {
  const long blocks = a.nsq * a.nvec * a.nchunk;
  if (blocks <= 0) return hipSuccess;
  if (a.reverse) {
    if (!a.out_present) return hipErrorInvalidValue;  // reverse transform: Repair fill only
    hipLaunchKernelGGL((leo8_encode_kernel<K, true>), dim3((unsigned)blocks), dim3(128), 0, s, a);
  } else {
    hipLaunchKernelGGL((leo8_encode_kernel<K, false>), dim3((unsigned)blocks), dim3(128 * EncSplit<K>::H), 0, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_leo8_encode(int k, const EncodeArgs& a, hipStream_t s) {
  if (leo8_sliced_applicable(k, a)) return launch_leo8_encode_sliced(k, a, s);
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
