// rs_gf8_sliced.hip -- bit-sliced Leopard GF(2^8) Reed-Solomon encode on gfx950
// (k = 16..128), the default for the row and column passes of ExtendShares.
//
// Replaces the same hot loop as rs_gf8.hip: klauspost/reedsolomon v1.11.8
// leopardFF8.encode (ifftDITEncoder8 + fftDIT8), called 3k times per square by
// rsmt2d v0.11.0 ComputeExtendedDataSquare (pkg/da/data_availability_header.go:74).
// The transform itself (bit-sliced planes, compile-time and wave-split skews)
// is in leo8_sliced.hpp; this file holds the memory side.
//
// One workgroup = NW = k/16 waves = 4 vectors x one 512-B chunk of their shards.
// Lane l handles vector 4g + (l >> 4) and bytes [16t, 16t+16) + [256+16t, +16)
// of the chunk, t = l & 15: two 16-B loads per element, 256 B contiguous per 16
// lanes.  Each element's 32 bytes are bit-transposed into 8 planes in
// registers (16 elements x 8 planes = 128 VGPRs).  Layout A (wave = element
// >> 4) for the IFFT's low layers, one LDS exchange to layout B (wave =
// element & (NW-1)) for the high layers of the IFFT and the FFT, one exchange
// back for the FFT's low layers, planes transposed back and stored.  LDS:
// k x 64 lanes x 16 B (128 KB at k = 128), two passes of 4 planes per exchange.
// HBM traffic is the algorithmic minimum (each data byte read once, each
// parity byte written once, plus the Q0 copy of the row pass).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "kernels.hpp"
#include "leo8.hpp"
#include "leo8_sliced.hpp"

namespace dagpu {

using namespace sliced;

// Two copies of the mask table, one for the IFFT and one for the FFT: with one
// table the compiler merges the two layers' identical loads and keeps all 192
// masks live across the middle of the kernel (SGPR spills through v_writelane).
__constant__ WMasks kWMasksIfft = make_wmasks();
__constant__ WMasks kWMasksFft = make_wmasks();

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Exchange between layouts through LDS: every wave writes its registers at the
// element slots of layout FROM and reads back the slots of layout TO.  Slot of
// element e for lane l: lds[e * 64 + l] (16 B = 4 planes); two passes of 4
// planes.  The caller guarantees a barrier before the first write.
template <int K, bool A_TO_B>
__device__ __forceinline__ void exchange(uint32_t (&v)[16][8], u32x4* lds, int wave, int lane) {
  constexpr int NW = Geo<K>::NW;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    if (h) __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int e = A_TO_B ? 16 * wave + r : wave + NW * r;
      u32x4 q = {v[r][4 * h], v[r][4 * h + 1], v[r][4 * h + 2], v[r][4 * h + 3]};
      lds[e * 64 + lane] = q;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int e = A_TO_B ? wave + NW * r : 16 * wave + r;
      const u32x4 q = lds[e * 64 + lane];
      v[r][4 * h] = q.x;
      v[r][4 * h + 1] = q.y;
      v[r][4 * h + 2] = q.z;
      v[r][4 * h + 3] = q.w;
    }
  }
}

template <int K>
__global__ __launch_bounds__(64 * Geo<K>::NW) __attribute__((amdgpu_waves_per_eu(2, 2)))
void leo8_encode_sliced_kernel(EncodeArgs a) {
  constexpr int NW = Geo<K>::NW;
  __shared__ u32x4 lds[NW > 1 ? K * 64 : 1];
  // Block order: XCD x (blocks x, x+8, ... on gfx950's round-robin dispatch)
  // takes one contiguous eighth of the work (profiles/sliced_modes_r01.log: with
  // non-temporal stores, row/col 1.27/2.21 -> 1.21/2.09 ms per 256 squares).
  const long ngrp = a.nvec >> 2;
  const long nblk = a.nsq * ngrp * a.nchunk;
  long blk = blockIdx.x;
  if ((nblk & 7) == 0) blk = (blk & 7) * (nblk >> 3) + (blk >> 3);
  const long chunk = blk % a.nchunk;
  const long sg = blk / a.nchunk;
  const long grp = sg % ngrp;
  const long sq = sg / ngrp;
  constexpr int st_aux = 2;  // non-temporal stores: nothing in this launch re-reads them
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int vs = lane >> 4, t = lane & 15;

  uint32_t v[16][8];
  {
    const auto rsrc = make_rsrc(a.in + sq * a.in_sq_stride + grp * 4 * a.in_vec_stride + chunk * 512);
    const uint32_t voff = (uint32_t)(vs * a.in_vec_stride) + 16u * t;
    const uint32_t sstride = (uint32_t)a.in_shard_stride;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t soff = (uint32_t)(16 * wave + j) * sstride;
      const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, soff, 0);
      const u32x4 hi = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + 256u, soff, 0);
      v[j][0] = lo.x; v[j][1] = lo.y; v[j][2] = lo.z; v[j][3] = lo.w;
      v[j][4] = hi.x; v[j][5] = hi.y; v[j][6] = hi.z; v[j][7] = hi.w;
    }
  }
  if (a.copy) {  // row pass: the data shards also go to Q0 of the EDS
    const auto rsrc = make_rsrc(a.copy + sq * a.copy_sq_stride + grp * 4 * a.copy_vec_stride + chunk * 512);
    const uint32_t voff = (uint32_t)(vs * a.copy_vec_stride) + 16u * t;
    const uint32_t sstride = (uint32_t)a.copy_shard_stride;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t soff = (uint32_t)(16 * wave + j) * sstride;
      const u32x4 lo = {v[j][0], v[j][1], v[j][2], v[j][3]};
      const u32x4 hi = {v[j][4], v[j][5], v[j][6], v[j][7]};
      __builtin_amdgcn_raw_buffer_store_b128(lo, rsrc, voff, soff, st_aux);
      __builtin_amdgcn_raw_buffer_store_b128(hi, rsrc, voff + 256u, soff, st_aux);
    }
  }
#pragma unroll
  for (int j = 0; j < 16; j++) transpose8(v[j]);

  ifft_A<K>(v, &kWMasksIfft.m[0][wave][0], kMaxWav * 64);
  if constexpr (NW > 1) exchange<K, true>(v, lds, wave, lane);
  ifft_fft_B<K>(v);
  if constexpr (NW > 1) {
    __syncthreads();
    exchange<K, false>(v, lds, wave, lane);
  }
  fft_A<K>(v, &kWMasksFft.m[0][wave][0], kMaxWav * 64);

#pragma unroll
  for (int j = 0; j < 16; j++) transpose8(v[j]);
  const auto rsrc = make_rsrc(a.out + sq * a.out_sq_stride + grp * 4 * a.out_vec_stride + chunk * 512);
  const uint32_t voff = (uint32_t)(vs * a.out_vec_stride) + 16u * t;
  const uint32_t sstride = (uint32_t)a.out_shard_stride;
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const uint32_t soff = (uint32_t)(16 * wave + j) * sstride;
    const u32x4 lo = {v[j][0], v[j][1], v[j][2], v[j][3]};
    const u32x4 hi = {v[j][4], v[j][5], v[j][6], v[j][7]};
    __builtin_amdgcn_raw_buffer_store_b128(lo, rsrc, voff, soff, st_aux);
    __builtin_amdgcn_raw_buffer_store_b128(hi, rsrc, voff + 256u, soff, st_aux);
  }
}


// ---------------------------------------------------------------------------
// k = 128, two vectors per 4-wave workgroup (leo8_sliced.hpp "two-vector
// layout"): 128 KB of state per workgroup instead of 256 KB, so two workgroups
// share a CU (VGPRs 2 x 1 wave/SIMD, LDS 2 x 64 KB) and one workgroup's loads
// and stores overlap the other's transform.  Lane l: t = l & 15 (column block),
// vv = (l >> 4) & 1 (vector), eb = l >> 5 (element bit).  LDS slot of element e
// for lane (vv, t): e * 32 + vv * 16 + t, 4 planes per pass, two passes.
// ---------------------------------------------------------------------------
// A* <-> B through the workgroup's lds: A* holds element e = eb + 2 r + 32 w.
template <bool S_TO_B>
__device__ __forceinline__ void exchange2s(uint32_t (&v)[16][8], u32x4* lds, int w, int eb, int col) {
#pragma unroll
  for (int h = 0; h < 2; h++) {
    if (h) __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int e = S_TO_B ? eb + 2 * r + 32 * w : eb + 2 * w + 8 * r;
      lds[e * 32 + col] = (u32x4){v[r][4 * h], v[r][4 * h + 1], v[r][4 * h + 2], v[r][4 * h + 3]};
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int e = S_TO_B ? eb + 2 * w + 8 * r : eb + 2 * r + 32 * w;
      const u32x4 q = lds[e * 32 + col];
      v[r][4 * h] = q.x;
      v[r][4 * h + 1] = q.y;
      v[r][4 * h + 2] = q.z;
      v[r][4 * h + 3] = q.w;
    }
  }
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A <-> A*: the wave's own 32 elements swap element bit 0 (register bit in A)
// with element bit 4 (the lane bit eb in A), through the wave's quarter of lds
// (16 KB per half of 4 planes); a wave's LDS operations complete in order, so
// wave-scope fences separate the phases.
template <bool A_TO_S>
__device__ __forceinline__ void transpose_wave2(uint32_t (&v)[16][8], u32x4* lds, int w, int eb, int col) {
  u32x4* q = lds + w * 32 * 32;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    if (h) wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int e = A_TO_S ? r + 16 * eb : eb + 2 * r;
      q[e * 32 + col] = (u32x4){v[r][4 * h], v[r][4 * h + 1], v[r][4 * h + 2], v[r][4 * h + 3]};
    }
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int e = A_TO_S ? eb + 2 * r : r + 16 * eb;
      const u32x4 x = q[e * 32 + col];
      v[r][4 * h] = x.x;
      v[r][4 * h + 1] = x.y;
      v[r][4 * h + 2] = x.z;
      v[r][4 * h + 3] = x.w;
    }
  }
}

// The k = 128 two-vector transform: layer 0 in A (lane term), layers 1..2 in
// A* (element bit 0 in the lane: no lane term), layers 3..6 in B (compile-time
// skews), and back.  Skew offsets IO / FO: K / 0 for the encode, 0 / K for the
// reverse fill (parity half -> data half, EncodeArgs.reverse).
template <int IO, int FO>
__device__ __forceinline__ void transform2(uint32_t (&v)[16][8], u32x4* lds, int w, int eb, int col, uint32_t ebmask) {
  constexpr int K = 128;
  ifft_A2<K, 1, IO>(v, w, ebmask);
  transpose_wave2<true>(v, lds, w, eb, col);
  ifft_As2<K, IO>(v, w);
  __syncthreads();  // every wave's wave-local reads are done before the exchange writes
  exchange2s<true>(v, lds, w, eb, col);
  ifft_fft_B<K, IO, FO>(v);
  __syncthreads();
  exchange2s<false>(v, lds, w, eb, col);
  fft_As2<K, FO>(v, w);
  __syncthreads();  // other waves' last exchange reads of this wave's quarter are done
  transpose_wave2<false>(v, lds, w, eb, col);
  fft_A2<K, 1, FO>(v, w, ebmask);
}

// FILL (Repair fill mode, EncodeArgs): block = (pair of same-square vectors
// from pair_list, chunk); each half of the lanes takes its own vector (a -1
// entry: the lanes load the partner's data and store nothing); a shard of the
// half being rebuilt is stored where it is missing, a given one is compared
// (redo on a difference).  REV: the reverse fill (EncodeArgs.reverse: `in` is
// the parity half, `out` the data half).
template <bool FILL, bool REV = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void leo8_encode_sliced2_kernel(EncodeArgs a) {
  constexpr int K = 128;
  __shared__ u32x4 lds[K * 32];  // 64 KB
  const int lane = threadIdx.x & 63;
  const int t = lane & 15, vv = (lane >> 4) & 1, eb = lane >> 5;
  long chunk, sq, vbase, vlane;  // vector = vbase (block-uniform) + vlane (this lane)
  int fill_v = -1;               // FILL: this lane's flattened vector, -1 = none
  if constexpr (FILL) {
    chunk = blockIdx.x % a.nchunk;
    const long g = blockIdx.x / a.nchunk;
    if (g >= *a.pair_count) return;  // uniform
    const int v0 = a.pair_list[2 * g], v1 = a.pair_list[2 * g + 1];
    sq = v0 / a.nvec;
    fill_v = vv ? v1 : v0;
    vbase = 0;
    vlane = (fill_v >= 0 ? fill_v : v0) - sq * a.nvec;
  } else {
    const long ngrp = a.nvec >> 1;
    const long nblk = a.nsq * ngrp * a.nchunk;
    long blk = blockIdx.x;
    if ((nblk & 7) == 0) blk = (blk & 7) * (nblk >> 3) + (blk >> 3);  // one eighth per XCD
    chunk = blk % a.nchunk;
    const long sg = blk / a.nchunk;
    const long grp = sg % ngrp;
    sq = sg / ngrp;
    vbase = grp * 2;
    vlane = vv;
  }
  constexpr int st_aux = 2;  // non-temporal stores
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ebmask = eb ? 0xFFFFFFFFu : 0u;

  // layout A: register j holds element j + 16 eb + 32 w; the lane part of the
  // element offset (16 eb) goes into voffset, the wave part into soffset
  uint32_t v[16][8];
  {
    const auto rsrc = make_rsrc(a.in + sq * a.in_sq_stride + vbase * a.in_vec_stride + chunk * 512);
    const uint32_t sstride = (uint32_t)a.in_shard_stride;
    const uint32_t voff = (uint32_t)(vlane * a.in_vec_stride) + (uint32_t)(16 * eb) * sstride + 16u * t;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t soff = (uint32_t)(j + 32 * w) * sstride;
      const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, soff, 0);
      const u32x4 hi = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + 256u, soff, 0);
      v[j][0] = lo.x; v[j][1] = lo.y; v[j][2] = lo.z; v[j][3] = lo.w;
      v[j][4] = hi.x; v[j][5] = hi.y; v[j][6] = hi.z; v[j][7] = hi.w;
    }
  }
  if (!FILL && a.copy) {  // row pass: the data shards also go to Q0 of the EDS
    const auto rsrc = make_rsrc(a.copy + sq * a.copy_sq_stride + vbase * a.copy_vec_stride + chunk * 512);
    const uint32_t sstride = (uint32_t)a.copy_shard_stride;
    const uint32_t voff = (uint32_t)(vlane * a.copy_vec_stride) + (uint32_t)(16 * eb) * sstride + 16u * t;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t soff = (uint32_t)(j + 32 * w) * sstride;
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){v[j][0], v[j][1], v[j][2], v[j][3]}, rsrc, voff, soff, st_aux);
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){v[j][4], v[j][5], v[j][6], v[j][7]}, rsrc, voff + 256u, soff,
                                             st_aux);
    }
  }
#pragma unroll
  for (int j = 0; j < 16; j++) transpose8(v[j]);

  const int col = vv * 16 + t;
  transform2<REV ? 0 : K, REV ? K : 0>(v, lds, w, eb, col, ebmask);
#if defined(DAGPU_RS_PAD) && DAGPU_RS_PAD > 0
  {  // A/B instrument only: DAGPU_RS_PAD x 128 extra fast-class VALU ops per lane, results unchanged
    const uint32_t z = __builtin_amdgcn_readfirstlane((uint32_t)(a.nchunk - 1));  // 0 at run time
#pragma unroll
    for (int r = 0; r < DAGPU_RS_PAD; r++)
#pragma unroll
      for (int j = 0; j < 16; j++)
#pragma unroll
        for (int p = 0; p < 8; p++) v[j][p] ^= z * (uint32_t)(2654435761u * (r + 1) + 97u * j + p);
  }
#endif

#pragma unroll
  for (int j = 0; j < 16; j++) transpose8(v[j]);
  const auto rsrc = make_rsrc(a.out + sq * a.out_sq_stride + vbase * a.out_vec_stride + chunk * 512);
  const uint32_t sstride = (uint32_t)a.out_shard_stride;
  const uint32_t voff = (uint32_t)(vlane * a.out_vec_stride) + (uint32_t)(16 * eb) * sstride + 16u * t;
  if constexpr (FILL) {
    if (fill_v < 0) return;
    uint32_t diff = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t soff = (uint32_t)(j + 32 * w) * sstride;
      if (fill_given(a, sq, vlane, j + 16 * eb + 32 * w)) {
        const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, soff, 0);
        const u32x4 hi = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + 256u, soff, 0);
        diff |= (lo.x ^ v[j][0]) | (lo.y ^ v[j][1]) | (lo.z ^ v[j][2]) | (lo.w ^ v[j][3]);
        diff |= (hi.x ^ v[j][4]) | (hi.y ^ v[j][5]) | (hi.z ^ v[j][6]) | (hi.w ^ v[j][7]);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128((u32x4){v[j][0], v[j][1], v[j][2], v[j][3]}, rsrc, voff, soff, 0);
        __builtin_amdgcn_raw_buffer_store_b128((u32x4){v[j][4], v[j][5], v[j][6], v[j][7]}, rsrc, voff + 256u, soff,
                                               0);
      }
    }
    if (diff) a.redo[fill_v] = 1;
    return;
  }
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const uint32_t soff = (uint32_t)(j + 32 * w) * sstride;
    __builtin_amdgcn_raw_buffer_store_b128((u32x4){v[j][0], v[j][1], v[j][2], v[j][3]}, rsrc, voff, soff, st_aux);
    __builtin_amdgcn_raw_buffer_store_b128((u32x4){v[j][4], v[j][5], v[j][6], v[j][7]}, rsrc, voff + 256u, soff,
                                           st_aux);
  }
}

template <int K>
static hipError_t launch_sliced_k(const EncodeArgs& a, hipStream_t s) {
  const long blocks = a.nsq * (a.nvec / 4) * a.nchunk;
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(leo8_encode_sliced_kernel<K>, dim3((unsigned)blocks), dim3(64 * Geo<K>::NW), 0, s, a);
  return hipGetLastError();
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// The sliced kernel covers the ExtendShares / Codec shapes: k = 16..128, whole
// 512-B chunks, vectors in groups of 4, 16-B aligned rows, no compare mode or
// vector mask.  DAGPU_ENC_SLICED=0 selects the packed-byte kernel for A/B runs.
bool leo8_sliced_applicable(int k, const EncodeArgs& a) {
  const char* e = sw(SW_ENC_SLICED);
  const bool enabled = !(e && e[0] == '0');
  if (!enabled || k < 16 || k > 128) return false;
  if (a.shard_bytes <= 0 || a.shard_bytes % 512 || a.nvec % 4 || a.vec_flags || a.mismatch || a.out_present ||
      a.reverse)
    return false;
  if (a.nchunk * 512 != a.shard_bytes) return false;
  const long strides[] = {a.in_sq_stride, a.in_vec_stride, a.in_shard_stride, a.out_sq_stride,
                          a.out_vec_stride, a.out_shard_stride};
  for (long st : strides)
    if (st % 16) return false;
  if (!aligned16(a.in) || !aligned16(a.out)) return false;
  if (a.copy && (!aligned16(a.copy) || a.copy_sq_stride % 16 || a.copy_vec_stride % 16 || a.copy_shard_stride % 16))
    return false;
  // buffer offsets (voffset + soffset) must stay below the 2^31 range
  const long lim = 1L << 31;
  if (3 * a.in_vec_stride + 512 + (long)k * a.in_shard_stride >= lim) return false;
  if (3 * a.out_vec_stride + 512 + (long)k * a.out_shard_stride >= lim) return false;
  if (a.copy && 3 * a.copy_vec_stride + 512 + (long)k * a.copy_shard_stride >= lim) return false;
  return true;
}

// DAGPU_ENC_SLICED2=0 keeps k = 128 on the 4-vector kernel (A/B runs).
static bool sliced2_enabled() {
  const char* e = sw(SW_ENC_SLICED2);
  return !(e && e[0] == '0');
}

hipError_t launch_leo8_encode_sliced(int k, const EncodeArgs& a, hipStream_t s) {
  // (leo8_sliced_applicable has checked the shapes: nvec % 4 == 0, offsets < 2^31)
  if (k == 128 && sliced2_enabled()) {
    const long blocks = a.nsq * (a.nvec / 2) * a.nchunk;
    if (blocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(leo8_encode_sliced2_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  switch (k) {
    case 16: return launch_sliced_k<16>(a, s);
    case 32: return launch_sliced_k<32>(a, s);
    case 64: return launch_sliced_k<64>(a, s);
    case 128: return launch_sliced_k<128>(a, s);
    default: return hipErrorInvalidValue;
  }
}

// Repair fill at k = 128 over a pair list (EncodeArgs fill fields; grid for the
// worst case, blocks past *pair_count return).  Same shape limits as the
// sliced encoder: whole 512-B chunks, 16-B aligned strides, offsets < 2^31.
bool leo8_fill_sliced_applicable(const EncodeArgs& a) {
  if (a.shard_bytes <= 0 || a.shard_bytes % 512 || a.nchunk * 512 != a.shard_bytes) return false;
  const long strides[] = {a.in_sq_stride, a.in_vec_stride, a.in_shard_stride, a.out_sq_stride,
                          a.out_vec_stride, a.out_shard_stride};
  for (long st : strides)
    if (st % 16) return false;
  if (!aligned16(a.in) || !aligned16(a.out)) return false;
  const long lim = 1L << 31;
  return (a.nvec - 1) * a.in_vec_stride + 512 + 128L * a.in_shard_stride < lim &&
         (a.nvec - 1) * a.out_vec_stride + 512 + 128L * a.out_shard_stride < lim;
}

hipError_t launch_leo8_fill_sliced(const EncodeArgs& a, long max_pairs, hipStream_t s) {
  const long blocks = max_pairs * a.nchunk;
  if (blocks <= 0) return hipSuccess;
  if (a.reverse) hipLaunchKernelGGL((leo8_encode_sliced2_kernel<true, true>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  else hipLaunchKernelGGL((leo8_encode_sliced2_kernel<true, false>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace dagpu
