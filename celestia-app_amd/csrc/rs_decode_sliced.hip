// rs_decode_sliced.hip -- bit-sliced Leopard GF(2^8) reconstruct for k = 128 on
// gfx950, the default decode of ExtendedDataSquare.Repair's row and column
// passes (and of the codec entry) whenever the shards are whole 512-B chunks.
//
// Replaces the same hot loop as rs_decode.hip's leo8_decode128_kernel:
// klauspost/reedsolomon v1.11.8 leopardFF8.reconstruct, reached from rsmt2d
// v0.11.0 LeoRSCodec.Decode.  Per vector of
// n = 256 work elements ([parity 128][data 128]) with >= 128 present:
//   work[i] = present ? shard * exp(errLocs[i]) : 0
//   IFFT_256 (decoder skews skew[b + D - 1]); formal derivative; FFT_256
//   missing shard = work[pos] * exp(255 - errLocs[pos])
// (error locators from leo8_errlocs_kernel, shared across equal patterns).
//
// Layout: one 4-wave workgroup = one vector x one 512-B chunk of its shards;
// lane l = t + 16 eb holds bytes [16t, 16t+16) + [256+16t, +16) of 16 elements
// as 8 bit planes (leo8_sliced.hpp "bit-sliced decode"):
//   A:  e = j + 16 eb + 64 w  -- load, premultiply, IFFT layers 0..1
//   A*: e = eb + 4 r + 64 w   -- IFFT layers 2..3 (no lane term in the skews)
//   B:  e = eb + 4 w + 16 i   -- IFFT layers 4..7, formal derivative, FFT 7..4
//   A*, A                     -- FFT layers 3..2, 1..0, postmultiply, store
// Every op of the transform is a full-rate v_xor / v_bitop3 / shift; the
// error-locator multiplies run on the packed bytes before the bit transpose and
// after the inverse one (mul_packed: three v_perm lookups of 3/3/2-bit tables per
// dword, fewer ops than on the planes).  LDS: 64 KB, three workgroup passes (A*->B, derivative,
// B->A*) and two wave-local ones (A<->A*), each in two halves of 4 planes;
// the derivative's cross-lane and cross-wave terms (element bits 0..3 in B)
// are read from the originals written to LDS, its register bits (4..7) are
// applied in place.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "kernels.hpp"
#include "leo8.hpp"
#include "leo8_sliced.hpp"

namespace dagpu {

using namespace sliced;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// element held in register r of lane group eb, wave w
__device__ __forceinline__ int elemA(int r, int eb, int w) { return r + 16 * eb + 64 * w; }
__device__ __forceinline__ int elemS(int r, int eb, int w) { return eb + 4 * r + 64 * w; }  // A*
__device__ __forceinline__ int elemB(int r, int eb, int w) { return eb + 4 * w + 16 * r; }

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A <-> A*: the wave's own 64 elements change between register and lane bits,
// through the wave's quarter of lds (16 KB per half of 4 planes); a wave's LDS
// operations complete in order, so a wave-scope fence separates the phases.
template <bool A_TO_S>
__device__ __forceinline__ void dec_transpose_wave(uint32_t (&v)[16][8], u32x4* lds, int w, int eb, int t) {
  u32x4* q = lds + w * 64 * 16;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    if (h) wave_sync_lds();
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int e = (A_TO_S ? elemA(r, eb, 0) : elemS(r, eb, 0));
      q[e * 16 + t] = (u32x4){v[r][4 * h], v[r][4 * h + 1], v[r][4 * h + 2], v[r][4 * h + 3]};
    }
    wave_sync_lds();
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int e = (A_TO_S ? elemS(r, eb, 0) : elemA(r, eb, 0));
      const u32x4 x = q[e * 16 + t];
      v[r][4 * h] = x.x;
      v[r][4 * h + 1] = x.y;
      v[r][4 * h + 2] = x.z;
      v[r][4 * h + 3] = x.w;
    }
  }
}

// A* <-> B through the workgroup's lds (element slots e * 16 + t).
template <bool S_TO_B>
__device__ __forceinline__ void dec_exchange(uint32_t (&v)[16][8], u32x4* lds, int w, int eb, int t) {
#pragma unroll
  for (int h = 0; h < 2; h++) {
    __syncthreads();  // previous readers of lds are done
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int e = S_TO_B ? elemS(r, eb, w) : elemB(r, eb, w);
      lds[e * 16 + t] = (u32x4){v[r][4 * h], v[r][4 * h + 1], v[r][4 * h + 2], v[r][4 * h + 3]};
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int e = S_TO_B ? elemB(r, eb, w) : elemS(r, eb, w);
      const u32x4 q = lds[e * 16 + t];
      v[r][4 * h] = q.x;
      v[r][4 * h + 1] = q.y;
      v[r][4 * h + 2] = q.z;
      v[r][4 * h + 3] = q.w;
    }
  }
}

// Formal derivative in layout B.  Per half (4 planes): originals to LDS, then
// per register i ascending: register bits in place (deriv_local), element bits
// 0..3 (eb0, eb1, w0, w1) from the partners' originals in LDS where this
// element's bit is 0.
template <int H>
__device__ __forceinline__ void dec_derivative_half(uint32_t (&v)[16][8], u32x4* lds, int w, int eb, int t) {
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; r++)
    lds[elemB(r, eb, w) * 16 + t] = (u32x4){v[r][4 * H], v[r][4 * H + 1], v[r][4 * H + 2], v[r][4 * H + 3]};
  __syncthreads();
  deriv_local<4 * H, 4>(v);
  auto add = [&](int delta) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const u32x4 q = lds[(elemB(r, eb, w) + delta) * 16 + t];
      v[r][4 * H] ^= q.x;
      v[r][4 * H + 1] ^= q.y;
      v[r][4 * H + 2] ^= q.z;
      v[r][4 * H + 3] ^= q.w;
    }
  };
  if (!(eb & 1)) add(1);
  if (!(eb & 2)) add(2);
  if (!(w & 1)) add(4);
  if (!(w & 2)) add(8);
}

// DAGPU_PHASE_PROBE builds only (tools/phase_probe.py): lane 0 of waves 0 and 3
// stamp s_memtime at the phase boundaries, [block][wave 0 / 3][phase].
#ifdef DAGPU_PHASE_PROBE
constexpr int kProbe8Phases = 14;
__device__ uint64_t g_probe8[8192 * 2 * kProbe8Phases];
#define DEC8_PROBE(i)                                                                           \
  do {                                                                                          \
    if ((threadIdx.x & 63) == 0 && (w == 0 || w == 3) && blk < 8192)                            \
      g_probe8[(blk * 2 + (w == 3)) * kProbe8Phases + (i)] = __builtin_amdgcn_s_memtime();      \
  } while (0)
#else
#define DEC8_PROBE(i) ((void)0)
#endif

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void leo8_decode128_sliced_kernel(DecodeArgs a) {
  constexpr int K = 128;
  __shared__ u32x4 lds[256 * 16];  // 64 KB
  __shared__ tab4 mtab[257];       // packed-byte multiply tables per log value; [256] = zero
  __shared__ uint32_t mtab2[257];
  const long blk = blockIdx.x;
  const long chunk = blk % a.nchunk;  // 512-B chunks
  const long v = blk / a.nchunk;      // flattened (square, vector)
  if (a.flags[v] == 0) return;        // uniform: nothing to decode for this vector
  mtab[threadIdx.x] = mul_table((int)threadIdx.x);
  mtab2[threadIdx.x] = mul_table2((int)threadIdx.x);
  if (threadIdx.x == 0) {
    mtab[256] = mul_table(-1);
    mtab2[256] = 0u;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t = lane & 15, eb = lane >> 4;
  DEC8_PROBE(0);
  const long sq = v / a.nvec, vec = v % a.nvec;
  const uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
  const uint8_t* err = a.err + err_vec(a, v) * 256;
  const u32x4 errq = *(const u32x4*)(err + 16 * eb + 64 * w);  // errLocs of this lane's 16 elements
  auto err_of = [&](int j) -> uint32_t {
    const uint32_t d = j < 4 ? errq.x : j < 8 ? errq.y : j < 12 ? errq.z : errq.w;
    return (d >> (8 * (j & 3))) & 0xFFu;
  };
  // work index e -> shard: [parity K][data K]; e < K exactly for waves 0, 1
  const int shard0 = 64 * w + (w < 2 ? K : -K);  // shard of element j + 16 eb + 64 w is shard0 + 16 eb + j
  const auto rsrc = make_rsrc(a.data + sq * a.sq_stride + vec * a.vec_stride + chunk * 512);
  const uint32_t sstride = (uint32_t)a.shard_stride;
  const uint32_t voff = (uint32_t)(16 * eb) * sstride + 16u * t;

  uint32_t v_[16][8];
  uint32_t miss = 0;
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const int shard = shard0 + 16 * eb + j;
    const bool p = pres[(long)shard * a.p_shard_stride] != 0;
    miss |= (uint32_t)!p << j;
    const uint32_t soff = (uint32_t)(shard0 + j) * sstride;
    const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, soff, 0);
    const u32x4 hi = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + 256u, soff, 0);
    v_[j][0] = lo.x; v_[j][1] = lo.y; v_[j][2] = lo.z; v_[j][3] = lo.w;
    v_[j][4] = hi.x; v_[j][5] = hi.y; v_[j][6] = hi.z; v_[j][7] = hi.w;
  }
#pragma unroll
  for (int j = 0; j < 16; j++) {
    // present: shard * exp(errLocs); missing: 0 -- on packed bytes, then planes
    const uint32_t ti = ((miss >> j) & 1) ? 256u : err_of(j);
    mul_packed(v_[j], mtab[ti], mtab2[ti]);
    transpose8(v_[j]);
  }
  DEC8_PROBE(1);
  const uint32_t eb0mask = (eb & 1) ? 0xFFFFFFFFu : 0u, eb1mask = (eb & 2) ? 0xFFFFFFFFu : 0u;
  // layers 2..3 in A* instead of A: no lane terms (repair 19.5-19.7 -> 19.3 ms per 256 squares)
  dec_A<true, 2>(v_, w, eb0mask, eb1mask);
  DEC8_PROBE(2);
  dec_transpose_wave<true>(v_, lds, w, eb, t);
  DEC8_PROBE(3);
  dec_Astar<true>(v_, w);
  DEC8_PROBE(4);
  dec_exchange<true>(v_, lds, w, eb, t);
  DEC8_PROBE(5);
  dec_B<true>(v_);
  DEC8_PROBE(6);
  dec_derivative_half<0>(v_, lds, w, eb, t);
  dec_derivative_half<1>(v_, lds, w, eb, t);
  DEC8_PROBE(7);
  dec_B<false>(v_);
  DEC8_PROBE(8);
  dec_exchange<false>(v_, lds, w, eb, t);
  DEC8_PROBE(9);
  dec_Astar<false>(v_, w);
  DEC8_PROBE(10);
  __syncthreads();  // other waves' last reads of this wave's quarter of lds are done
  dec_transpose_wave<false>(v_, lds, w, eb, t);
  DEC8_PROBE(11);
  dec_A<false, 2>(v_, w, eb0mask, eb1mask);
  DEC8_PROBE(12);
  // missing shard = work * exp(255 - errLocs)
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const bool m = (miss >> j) & 1;
    if (!__any(m)) continue;  // uniform: no lane of this wave lost element j
    transpose8(v_[j]);
    mul_packed(v_[j], mtab[255u - err_of(j)], mtab2[255u - err_of(j)]);
    if (m) {
      const uint32_t soff = (uint32_t)(shard0 + j) * sstride;
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){v_[j][0], v_[j][1], v_[j][2], v_[j][3]}, rsrc, voff, soff, 0);
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){v_[j][4], v_[j][5], v_[j][6], v_[j][7]}, rsrc, voff + 256u,
                                             soff, 0);
    }
  }
  DEC8_PROBE(13);
}

// DAGPU_DEC_SLICED=0 keeps k = 128 on the packed-byte decoder (A/B runs;
// read per launch through sw(), see switches.hpp).
static bool dec_sliced_enabled() {
  const char* e = sw(SW_DEC_SLICED);
  return !(e && e[0] == '0');
}

bool leo8_decode_sliced_applicable(const DecodeArgs& a) {
  if (!dec_sliced_enabled() || a.k != 128) return false;
  if (a.shard_bytes <= 0 || a.shard_bytes % 512 || a.nchunk * 512 != a.shard_bytes) return false;
  if (((uintptr_t)a.data & 15) || a.sq_stride % 16 || a.vec_stride % 16 || a.shard_stride % 16) return false;
  // voffset (48 shard strides + 512) and soffset (256 shard strides) below 2^31
  if (256L * a.shard_stride + 512 >= (1L << 31)) return false;
  return true;
}

hipError_t launch_leo8_decode128_sliced(const DecodeArgs& a, hipStream_t s) {
  const long blocks = a.nsq * a.nvec * a.nchunk;
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(leo8_decode128_sliced_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace dagpu

#ifdef DAGPU_PHASE_PROBE
extern "C" int dagpu_debug_probe8(int op, uint64_t* out, size_t n) {
  if (op == 0) {
    static uint64_t zero[8192 * 2 * dagpu::kProbe8Phases];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(dagpu::g_probe8), zero, sizeof zero);
  }
  if (n > 8192 * 2 * (size_t)dagpu::kProbe8Phases) n = 8192 * 2 * (size_t)dagpu::kProbe8Phases;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(dagpu::g_probe8), n * sizeof(uint64_t));
}
#endif
