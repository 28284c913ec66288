// rs_decode.hip -- Leopard GF(2^8) reconstruct (decode) on gfx950.
//
// Replaces klauspost/reedsolomon v1.11.8 leopardFF8.reconstruct, reached from
// rsmt2d v0.11.0 LeoRSCodec.Decode inside ExtendedDataSquare.Repair
// (solveCrosswordRow/Col -> rebuildShares), SURVEY.md §3.5 and §8a row A11.
//
// Per vector of n = 2k shards with >= k present:
//   1. error locator (kernel 1, one wave per vector, four per workgroup):
//        errLocs[i] = 1 for each missing position (work layout: [parity k][data k]),
//        FWHT(errLocs, mtrunc = n); errLocs[i] = errLocs[i]*logWalsh[i] mod 255;
//        FWHT(errLocs, 256)
//   2. decode (kernel 2, one thread per dword column of the vector):
//        work[i] = present ? shard*errLocs[i] : 0
//        IFFT_n (decoder skew: fftSkew[iend-1]) ; formal derivative ; FFT_n
//        missing shard = work[pos] * (255 - errLocs[pos])
// The transform runs register-resident exactly like the encoder: one thread
// holds all n elements of its dword column for k <= 64, and for k = 128 four
// waves share a column (leo8_decode128_kernel, layout transposes through LDS).
// Runtime multiplies (error locators) read the 2-bit lookup tables from an LDS
// copy with a wave-uniform index; presence comes from wave ballots.
// MDS codes have a unique decoding, so any correct decoder is bit-exact; this
// one is also step-for-step the reference algorithm.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"
#include "leo8.hpp"

namespace dagpu {

// ---------------------------------------------------------------------------
// Kernel 1: error locators.  One 64-thread block per vector.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t add_mod8(uint32_t a, uint32_t b) {
  const uint32_t s = a + b;
  return (s + (s >> 8)) & 0xFFu;
}
__device__ __forceinline__ uint32_t sub_mod8(uint32_t a, uint32_t b) {
  const uint32_t d = a - b;
  return (d + (d >> 8)) & 0xFFu;
}

// fwht8(data, m = 256, mtrunc) by one wave: 4 radix-4 passes, 64 groups of 4
// each.  Only this wave touches e, and a wave's LDS operations complete in
// order, so a wave-scope fence is the barrier between passes.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void fwht256_wave(uint32_t* e, int mtrunc, int g) {
#pragma unroll
  for (int dist = 1; dist <= 64; dist *= 4) {
    const int dist4 = dist * 4;
    const int r = (g / dist) * dist4;
    const int i = r + (g % dist);
    if (r < mtrunc) {
      const uint32_t t0 = e[i], t1 = e[i + dist], t2 = e[i + 2 * dist], t3 = e[i + 3 * dist];
      const uint32_t a0 = add_mod8(t0, t1), a1 = sub_mod8(t0, t1);
      const uint32_t a2 = add_mod8(t2, t3), a3 = sub_mod8(t2, t3);
      e[i] = add_mod8(a0, a2);
      e[i + 2 * dist] = sub_mod8(a0, a2);
      e[i + dist] = add_mod8(a1, a3);
      e[i + 3 * dist] = sub_mod8(a1, a3);
    }
    wave_sync();
  }
}

// One wave per vector, four vectors per workgroup; the decodable count goes
// to the global counter once per workgroup (one atomic per vector on a single
// address cost 0.27 ms per launch at 65,536 vectors).
constexpr int kErrVecs = 4;
__global__ __launch_bounds__(64 * kErrVecs) void leo8_errlocs_kernel(DecodeArgs a) {
  __shared__ uint32_t e_all[kErrVecs][256];
  __shared__ int blk_cnt;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (threadIdx.x == 0) blk_cnt = 0;
  __syncthreads();
  const long v = (long)blockIdx.x * kErrVecs + wave;  // flattened (square, vector)
  // locators_only: flagged vectors that compute their head's locators (uniform per wave)
  bool skip = v >= a.nsq * a.nvec || (a.locators_only && !a.flags[v]);
  const long hv = skip ? v : err_head_checked_wave(a, v, lane);
  skip = skip || (a.locators_only && !err_computes(a, v, hv));
  if (!skip) {
    uint32_t* e = e_all[wave];
    const long sq = v / a.nvec, vec = v % a.nvec;
    const int k = a.k, n = 2 * k;
    const uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
    int cnt = 0;
    for (int i = lane; i < 256; i += 64) {
      uint32_t x = 0;
      if (i < k) x = pres[(long)(k + i) * a.p_shard_stride] ? 0u : 1u;          // parity k+i -> work i
      else if (i < n) x = pres[(long)(i - k) * a.p_shard_stride] ? 0u : 1u;     // data i-k -> work i
      e[i] = x;
      if (i < n) cnt += (x == 0);
    }
    bool decode = true;
    if (!a.locators_only) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);  // present shards
      decode = cnt >= k && cnt < n && vec_selected(a, v);
      if (lane == 0) {
        a.flags[v] = decode ? 1 : 0;
        if (cnt < k && a.too_few) atomicOr(a.too_few, 1);
        if (decode) atomicAdd(&blk_cnt, 1);
      }
    }
    // uniform per wave; a vector sharing an earlier vector's erasure pattern
    // uses that vector's locators
    if (decode && err_computes(a, v, hv)) {
      wave_sync();
      fwht256_wave(e, n, lane);
      for (int i = lane; i < 256; i += 64) e[i] = (e[i] * kGf8.walsh[i]) % 255u;
      wave_sync();
      fwht256_wave(e, 256, lane);
      uint8_t* out = a.err + hv * 256;
      for (int i = lane; i < n; i += 64) out[i] = (uint8_t)e[i];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && blk_cnt && a.ndecodable) atomicAdd(a.ndecodable, blk_cnt);
}

// ---------------------------------------------------------------------------
// Kernel 2: decode.  N = 2K work elements; thread half h holds [h*E, (h+1)*E).
// ---------------------------------------------------------------------------
// ifftDITDecoder8 radix-4 layers entirely inside this half (dist4 <= E).
template <int N, int E, int BASE, int DIST>
__device__ __forceinline__ void ifft_dec_local(uint32_t (&w)[E]) {
  if constexpr (DIST * 4 <= E) {
#pragma unroll
    for (int r = 0; r < E; r += DIST * 4) {
      const int iend = BASE + r + DIST;  // global index
      const int l01 = kGf8.skew[iend - 1];
      const int l02 = kGf8.skew[iend + DIST - 1];
      const int l23 = kGf8.skew[iend + 2 * DIST - 1];
#pragma unroll
      for (int i = r; i < r + DIST; i++) {
        ifft2(w[i], w[i + DIST], l01);
        ifft2(w[i + 2 * DIST], w[i + 3 * DIST], l23);
        ifft2(w[i], w[i + 2 * DIST], l02);
        ifft2(w[i + DIST], w[i + 3 * DIST], l02);
      }
    }
    ifft_dec_local<N, E, BASE, DIST * 4>(w);
  } else if constexpr (E == N && DIST < N) {
    // one layer left (N = 2 * 4^j), only when the whole vector is local
    const int lm = kGf8.skew[DIST - 1];
#pragma unroll
    for (int i = 0; i < DIST; i++) ifft2(w[i], w[i + DIST], lm);
  }
}

// fftDIT8 radix-4 layers with dist4 <= E (inside this half), then the final
// radix-2 layer when it exists.
template <int N, int E, int BASE, int DIST4>
__device__ __forceinline__ void fft_dec_local(uint32_t (&w)[E]) {
  constexpr int DIST = DIST4 >> 2;
  if constexpr (DIST != 0) {
#pragma unroll
    for (int r = 0; r < E; r += DIST4) {
      const int iend = BASE + r + DIST;
      const int l01 = kGf8.skew[iend - 1];
      const int l02 = kGf8.skew[iend + DIST - 1];
      const int l23 = kGf8.skew[iend + 2 * DIST - 1];
#pragma unroll
      for (int i = r; i < r + DIST; i++) {
        fft2(w[i], w[i + 2 * DIST], l02);
        fft2(w[i + DIST], w[i + 3 * DIST], l02);
        fft2(w[i], w[i + DIST], l01);
        fft2(w[i + 2 * DIST], w[i + 3 * DIST], l23);
      }
    }
    fft_dec_local<N, E, BASE, DIST>(w);
  } else if constexpr (DIST4 == 2) {
#pragma unroll
    for (int r = 0; r < E; r += 2) fft2(w[r], w[r + 1], kGf8.skew[BASE + r]);
  }
}

// formal derivative steps i in (0, E) of a half: work[i-width, i) ^= work[i, i+width)
template <int E>
__device__ __forceinline__ void derivative_local(uint32_t (&w)[E]) {
#pragma unroll
  for (int i = 1; i < E; i++) {
    const int width = ((i ^ (i - 1)) + 1) >> 1;
#pragma unroll
    for (int j = 0; j < width; j++) w[i - width + j] ^= w[i + j];
  }
}

template <int K>
struct DecOcc { static constexpr int waves = K >= 64 ? 2 : (K >= 32 ? 4 : 8); };

__device__ __forceinline__ uint32_t gf8_mul_lds(uint32_t y, const uint4* tab, uint32_t lm);

// Decode of one dword column for k <= 64 (n = 2k <= 128 elements per thread,
// the whole transform register-resident).  Presence comes from wave ballots and
// the error locators from one per-lane byte load + v_readlane (wave-uniform),
// the runtime multiplies from the LDS copy of the lookup tables.
template <int K>
__device__ __forceinline__ void decode_small(const DecodeArgs& a, long v, int lane, uint32_t col, bool active,
                                             const uint4* tab) {
  constexpr int N = 2 * K;
  constexpr int NB = (N + 63) / 64;  // 64-element ballot words
  const long sq = v / a.nvec, vec = v % a.nvec;
  uint8_t* base = a.data + sq * a.sq_stride + vec * a.vec_stride;
  const auto rsrc = make_rsrc(base);
  const uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
  const uint8_t* err = a.err + err_vec(a, v) * 256;
  const uint32_t ss = (uint32_t)a.shard_stride;
  uint64_t pm[NB];
  uint32_t e8[NB];
#pragma unroll
  for (int c = 0; c < NB; c++) {
    const int i = 64 * c + lane;
    const int sh = i < K ? K + i : i - K;
    pm[c] = __ballot(i < N && pres[(long)(i < N ? sh : 0) * a.p_shard_stride] != 0);
    e8[c] = i < N ? err[i] : 0u;
  }
  // 1. work[i] = present ? shard * errLocs[i] : 0   ([parity K][data K])
  uint32_t w[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    const int sh = i < K ? K + i : i - K;
    const bool p = (pm[i >> 6] >> (i & 63)) & 1;
    uint32_t x = 0;
    if (p && active) x = __builtin_amdgcn_raw_buffer_load_b32(rsrc, col, (uint32_t)sh * ss, 0);
    w[i] = p ? gf8_mul_lds(x, tab, __builtin_amdgcn_readlane(e8[i >> 6], i & 63)) : 0u;
  }
  ifft_dec_local<N, N, 0, 1>(w);
  derivative_local<N>(w);
  fft_dec_local<N, N, 0, N>(w);
  if (!active) return;
#pragma unroll
  for (int pos = 0; pos < N; pos++) {  // missing shard = work[pos] * (255 - errLocs[pos])
    const int sh = pos < K ? pos + K : pos - K;
    if (((pm[pos >> 6] >> (pos & 63)) & 1) == 0) {
      const uint32_t y = gf8_mul_lds(w[pos], tab, 255u - __builtin_amdgcn_readlane(e8[pos >> 6], pos & 63));
      __builtin_amdgcn_raw_buffer_store_b32(y, rsrc, col, (uint32_t)sh * ss, 0);
    }
  }
}

// One block = 2 waves x 64 dword columns = 512 B of one vector.
template <int K>
__global__ __launch_bounds__(128)
__attribute__((amdgpu_waves_per_eu(DecOcc<K>::waves, 8))) void leo8_decode_kernel(DecodeArgs a) {
  const long blk = blockIdx.x;
  const int chunk = (int)(blk % a.nchunk);
  const long v = blk / a.nchunk;  // flattened (square, vector)
  if (a.flags[v] == 0) return;   // uniform: nothing to decode for this vector
  __shared__ uint4 tab[256];
  for (int i = threadIdx.x; i < 256; i += 128)
    tab[i] = make_uint4(kGf8.t[0][i], kGf8.t[1][i], kGf8.t[2][i], kGf8.t[3][i]);
  __syncthreads();
  const int t = threadIdx.x;
  const uint32_t col = (uint32_t)chunk * 512u + (uint32_t)t * 4u;
  decode_small<K>(a, v, t & 63, col, col < (uint32_t)a.shard_bytes, tab);
}

// ---------------------------------------------------------------------------
// k = 128 (n = 256) decode over FOUR wave-parts per dword column (64 elements
// per thread, no spills).  Element index bits: 0-5 are local in the "block"
// layout (part q holds i = 64q + j), bits 4-5 become the part index in the
// "transposed" layout (part q holds i = 64a + 16q + b, slot 16a + b), where
// bits 0-3 and 6-7 are local.  Both layout changes are the same 4x4 block
// transpose through LDS.  Schedule:
//   block:      premultiply, IFFT layers 1..32
//   transpose
//   transposed: IFFT layers 64, 128 (constants independent of q), formal
//               derivative, FFT layers 128, 64
//   transpose
//   block:      FFT layers 32..1, postmultiply of missing shards
// The formal derivative (leopard8.go FormalDerivative: for i in 1..n-1,
// work[i-w, i) ^= work[i, i+w), w = lowbit(i)) has the closed form
//   D(x)_e = x_e ^ XOR_{s : bit s of e == 0} x_{e | 2^s}   (original x),
// so the local bits are applied in place in ascending order and the two part
// bits (4, 5) come from the partner parts' original values via LDS.
// ---------------------------------------------------------------------------
constexpr int kD4Threads = 256;

// 4x4 (part, 16-element group) transpose in 4 chunks of 4 group-slots:
// element 16c + b of part q <-> element 16q + b of part c.
template <int Q>
__device__ __forceinline__ void xpose4(uint32_t (&w)[64], uint32_t (*xch)[4][4][64], int lane) {
#pragma unroll
  for (int h = 0; h < 4; h++) {
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
      for (int bb = 0; bb < 4; bb++) xch[c][Q][bb][lane] = w[16 * c + 4 * h + bb];
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
      for (int bb = 0; bb < 4; bb++) w[16 * c + 4 * h + bb] = xch[Q][c][bb][lane];
    __syncthreads();
  }
}

// Runtime multiply y * exp(lm) from the LDS copy of the 2-bit lookup tables
// (tab[lm] = kGf8.t[0..3][lm]); lm is wave-uniform, so the ds_read broadcasts.
__device__ __forceinline__ uint32_t gf8_mul_lds(uint32_t y, const uint4* tab, uint32_t lm) {
  const uint4 t = tab[lm];
  const uint32_t p0 = __builtin_amdgcn_perm(t.x, t.x, y & 0x03030303u);
  const uint32_t p1 = __builtin_amdgcn_perm(t.y, t.y, (y >> 2) & 0x03030303u);
  const uint32_t p2 = __builtin_amdgcn_perm(t.z, t.z, (y >> 4) & 0x03030303u);
  const uint32_t p3 = __builtin_amdgcn_perm(t.w, t.w, (y >> 6) & 0x03030303u);
  return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(p0, p1, p2, 0x96), p3, 0u, 0x96);
}

template <int Q>
__device__ __forceinline__ void decode128_part(const DecodeArgs& a, long v, int lane, uint32_t col, bool active,
                                               uint32_t (*xch)[4][4][64], const uint4* tab) {
  constexpr int K = 128, N = 256;
  const long sq = v / a.nvec, vec = v % a.nvec;
  uint8_t* base = a.data + sq * a.sq_stride + vec * a.vec_stride;
  const auto rsrc = make_rsrc(base);
  const uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
  const uint8_t* err = a.err + err_vec(a, v) * 256;
  const uint32_t ss = (uint32_t)a.shard_stride;
  // presence of the shard behind work index i: bit (i & 63) of pm[i >> 6]
  // (wave-uniform ballots); this part's error locators, one per lane
  uint64_t pm[4];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const int i = 64 * c + lane;
    const int sh = i < K ? K + i : i - K;
    pm[c] = __ballot(pres[(long)sh * a.p_shard_stride] != 0);
  }
  const uint32_t my_err = err[64 * Q + lane];

  uint32_t w[64];
#pragma unroll
  for (int j = 0; j < 64; j++) {  // work[i] = present ? shard * errLocs[i] : 0, [parity K][data K]
    const int i = 64 * Q + j;
    const int sh = i < K ? K + i : i - K;
    const bool p = (pm[Q] >> j) & 1;
    uint32_t x = 0;
    if (p && active) x = __builtin_amdgcn_raw_buffer_load_b32(rsrc, col, (uint32_t)sh * ss, 0);
    w[j] = p ? gf8_mul_lds(x, tab, __builtin_amdgcn_readlane(my_err, j)) : 0u;
  }
  ifft_dec_local<N, 64, 64 * Q, 1>(w);  // IFFT layers 1..32
  xpose4<Q>(w, xch, lane);
  {  // IFFT radix-4 step dist 64 (iend = 64): layers 64 then 128
    constexpr int l01 = kGf8.skew[63], l02 = kGf8.skew[127], l23 = kGf8.skew[191];
#pragma unroll
    for (int b = 0; b < 16; b++) {
      ifft2(w[b], w[16 + b], l01);
      ifft2(w[32 + b], w[48 + b], l23);
      ifft2(w[b], w[32 + b], l02);
      ifft2(w[16 + b], w[48 + b], l02);
    }
  }
  {  // formal derivative; slot 16a + b is element 64a + 16Q + b
    uint32_t t[64];
    uint32_t (*xd)[64] = &xch[0][0][0];  // [4 parts * 16 slots][64 lanes] per chunk
#pragma unroll
    for (int h = 0; h < 4; h++) {  // cross bits 4 (part ^ 1) and 5 (part ^ 2), original values
#pragma unroll
      for (int u = 0; u < 16; u++) xd[Q * 16 + u][lane] = w[16 * h + u];
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 16; u++) {
        uint32_t acc = 0;
        if constexpr ((Q & 1) == 0) acc ^= xd[(Q | 1) * 16 + u][lane];
        if constexpr ((Q & 2) == 0) acc ^= xd[(Q | 2) * 16 + u][lane];
        t[16 * h + u] = acc;
      }
      __syncthreads();
    }
    // local bits 0-3 (slot bits 0-3) and 6-7 (slot bits 4-5), ascending in place
#pragma unroll
    for (int j = 0; j < 64; j++) {
      uint32_t acc = w[j] ^ t[j];
#pragma unroll
      for (int sb = 0; sb < 6; sb++)
        if (((j >> sb) & 1) == 0) acc ^= w[j | (1 << sb)];
      w[j] = acc;
    }
  }
  {  // FFT radix-4 step dist4 = 256, dist = 64 (iend = 64): layers 128 then 64
    constexpr int l01 = kGf8.skew[63], l02 = kGf8.skew[127], l23 = kGf8.skew[191];
#pragma unroll
    for (int b = 0; b < 16; b++) {
      fft2(w[b], w[32 + b], l02);
      fft2(w[16 + b], w[48 + b], l02);
      fft2(w[b], w[16 + b], l01);
      fft2(w[32 + b], w[48 + b], l23);
    }
  }
  xpose4<Q>(w, xch, lane);
  fft_dec_local<N, 64, 64 * Q, 64>(w);  // FFT layers 32..1
  if (!active) return;
#pragma unroll
  for (int j = 0; j < 64; j++) {  // missing shard s = work[pos] * (255 - errLocs[pos])
    const int pos = 64 * Q + j;
    const int sh = pos < K ? pos + K : pos - K;
    if (((pm[Q] >> j) & 1) == 0) {  // shard sh (work index pos) was missing
      const uint32_t y = gf8_mul_lds(w[j], tab, 255u - __builtin_amdgcn_readlane(my_err, j));
      __builtin_amdgcn_raw_buffer_store_b32(y, rsrc, col, (uint32_t)sh * ss, 0);
    }
  }
}

// One block = 4 waves (parts) x 64 dword columns = 256 B of one vector.
__global__ __launch_bounds__(kD4Threads) __attribute__((amdgpu_waves_per_eu(3, 8)))
void leo8_decode128_kernel(DecodeArgs a, int nchunk256) {
  const long blk = blockIdx.x;
  const int chunk = (int)(blk % nchunk256);
  const long v = blk / nchunk256;
  if (a.flags[v] == 0) return;  // uniform
  __shared__ uint32_t xch[4][4][4][64];
  __shared__ uint4 tab[256];
  tab[threadIdx.x] = make_uint4(kGf8.t[0][threadIdx.x], kGf8.t[1][threadIdx.x], kGf8.t[2][threadIdx.x],
                                kGf8.t[3][threadIdx.x]);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t col = (uint32_t)chunk * 256u + (uint32_t)lane * 4u;
  const bool active = col < (uint32_t)a.shard_bytes;
  switch (q) {
    case 0: decode128_part<0>(a, v, lane, col, active, xch, tab); break;
    case 1: decode128_part<1>(a, v, lane, col, active, xch, tab); break;
    case 2: decode128_part<2>(a, v, lane, col, active, xch, tab); break;
    default: decode128_part<3>(a, v, lane, col, active, xch, tab); break;
  }
}

// Marks rebuilt shards present (separate launch so decode kernels of the same
// pass read a stable presence map).
__global__ __launch_bounds__(256) void mark_present_kernel(DecodeArgs a) {
  const long v = blockIdx.x;
  if (a.flags[v] == 0) return;
  const long sq = v / a.nvec, vec = v % a.nvec;
  uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
  for (int i = threadIdx.x; i < 2 * a.k; i += 256) pres[(long)i * a.p_shard_stride] = 1;
  if (threadIdx.x == 0 && a.progress) atomicAdd(a.progress, 1);
}

template <int K>
static hipError_t launch_dec(const DecodeArgs& a, hipStream_t s) {
  const long blocks = a.nsq * a.nvec * a.nchunk;
  hipLaunchKernelGGL((leo8_decode_kernel<K>), dim3((unsigned)blocks), dim3(128), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_leo8_errlocs(const DecodeArgs& a, hipStream_t s) {
  const long nv = a.nsq * a.nvec;
  if (nv <= 0) return hipSuccess;
  hipLaunchKernelGGL(leo8_errlocs_kernel, dim3((unsigned)((nv + kErrVecs - 1) / kErrVecs)), dim3(64 * kErrVecs), 0,
                     s, a);
  return hipGetLastError();
}

hipError_t launch_leo8_decode_only(const DecodeArgs& a, hipStream_t s, bool mark_present) {
  const long nv = a.nsq * a.nvec;
  if (nv <= 0) return hipSuccess;
  hipError_t e = hipSuccess;
  switch (a.k) {
    case 1: e = launch_dec<1>(a, s); break;
    case 2: e = launch_dec<2>(a, s); break;
    case 4: e = launch_dec<4>(a, s); break;
    case 8: e = launch_dec<8>(a, s); break;
    case 16: e = launch_dec<16>(a, s); break;
    case 32: e = launch_dec<32>(a, s); break;
    case 64: e = launch_dec<64>(a, s); break;
    case 128: {
      if (leo8_decode_sliced_applicable(a)) {
        e = launch_leo8_decode128_sliced(a, s);
        break;
      }
      const long nc = (a.shard_bytes + 255) / 256;
      hipLaunchKernelGGL(leo8_decode128_kernel, dim3((unsigned)(nv * nc)), dim3(kD4Threads), 0, s, a, (int)nc);
      e = hipGetLastError();
      break;
    }
    default: return hipErrorInvalidValue;
  }
  if (e != hipSuccess) return e;
  if (mark_present) {
    hipLaunchKernelGGL(mark_present_kernel, dim3((unsigned)nv), dim3(256), 0, s, a);
    e = hipGetLastError();
  }
  return e;
}

hipError_t launch_leo8_decode(const DecodeArgs& a, hipStream_t s, bool mark_present) {
  hipError_t e = launch_leo8_errlocs(a, s);
  if (e != hipSuccess) return e;
  return launch_leo8_decode_only(a, s, mark_present);
}

}  // namespace dagpu
