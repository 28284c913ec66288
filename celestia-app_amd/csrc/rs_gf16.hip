// rs_gf16.hip -- Leopard GF(2^16) encode / reconstruct on gfx950, used when a
// vector has 2k > 256 shards (k = 256, 512: the C5 stress squares).
//
// Replaces klauspost/reedsolomon v1.11.8 leopardFF16 (leopard.go encode /
// reconstruct), which rsmt2d v0.11.0 LeoRSCodec selects for
// dataShards + parityShards > 256.  Field: poly
// 0x1002D, Cantor basis; a symbol is the byte pair (b[i], b[i+32]) inside every
// 64-byte block of a shard (leopard.go refMulAdd).  Parity unpinned: no
// reference golden vector exists for k > 128; the kernels are checked against
// the oracle's GF(2^16) restatement and by erase/decode round trips.
//
// Kernels.  k = 256 and 512 run register-resident half-lane kernels
// (leo16_encode_h_kernel, leo16_decode_h_kernel: a lane holds 4 symbols of two
// elements, one per half wave, and multiplies by 3/3/2-split v_perm product
// tables); wider squares the LDS-slice kernels of rs_gf16_wide.hip.  A decode
// whose shard size is not a multiple of 256 B (codec API) takes the generic
// leo16_decode_kernel: one 256-thread workgroup per 64-B column block, the
// n = 2k elements of 32 symbols as uint16 rows in LDS, log/exp multiplies
// through 128 KiB tables in global memory (L2-resident).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <vector>

#include "gf16_host.hpp"
#include "kernels.hpp"
#include "leo8.hpp"
#include "sha256.hpp"

namespace dagpu {

namespace {

constexpr int kThreads16 = 256;
constexpr uint32_t kMod16 = 65535u;

__device__ uint16_t g_log16[65536];
__device__ uint16_t g_exp16[65536];
__device__ uint16_t g_skew16[65536];
// Folded Walsh weights for the n-point error-locator transform (n = 2k =
// 512, 1024): g_wfold16[n == 1024][r] = sum_q walsh[q*n + r] mod 65535.
__device__ uint16_t g_wfold16[3][2048];

__device__ __forceinline__ uint32_t mul16(uint32_t a, uint32_t lm) {
  if (a == 0) return 0;
  uint32_t s = (uint32_t)g_log16[a] + lm;
  s = (s + (s >> 16)) & 0xFFFFu;
  return g_exp16[s];
}

__device__ __forceinline__ uint32_t add_mod16(uint32_t a, uint32_t b) {
  const uint32_t s = a + b;
  return (s + (s >> 16)) & 0xFFFFu;
}
__device__ __forceinline__ uint32_t sub_mod16(uint32_t a, uint32_t b) {
  const uint32_t d = a - b;  // wraps: (d + (d >> 16)) mod 2^16 matches leopard subMod
  return (d + (d >> 16)) & 0xFFFFu;
}

// 64-B block <-> 32 LDS symbols.  Thread q (0..7) of a row moves lo dword q
// (symbols 4q..4q+3, low bytes) and hi dword q (same symbols, high bytes).
__device__ __forceinline__ void block_to_lds(uint16_t* row, uint32_t lo, uint32_t hi, int q) {
  uint32_t* r32 = (uint32_t*)row;
  r32[2 * q] = __builtin_amdgcn_perm(hi, lo, 0x05010400u);
  r32[2 * q + 1] = __builtin_amdgcn_perm(hi, lo, 0x07030602u);
}
__device__ __forceinline__ void lds_to_block(const uint16_t* row, uint32_t& lo, uint32_t& hi, int q) {
  const uint32_t* r32 = (const uint32_t*)row;
  const uint32_t s0 = r32[2 * q], s1 = r32[2 * q + 1];
  lo = __builtin_amdgcn_perm(s1, s0, 0x06040200u);
  hi = __builtin_amdgcn_perm(s1, s0, 0x07050301u);
}

// One radix-2 step over m elements: pair p -> (i, j, log multiplier).
template <bool INV, class PairFn>
__device__ __forceinline__ void step16(uint16_t* w, int npairs, PairFn pair) {
  for (int t = threadIdx.x; t < npairs * 32; t += kThreads16) {
    const int p = t >> 5, s = t & 31;
    int i, j;
    uint32_t lm;
    pair(p, i, j, lm);
    uint32_t x = w[i * 32 + s], y = w[j * 32 + s];
    if (INV) {
      y ^= x;
      if (lm != kMod16) x ^= mul16(y, lm);
    } else {
      if (lm != kMod16) x ^= mul16(y, lm);
      y ^= x;
    }
    w[i * 32 + s] = (uint16_t)x;
    w[j * 32 + s] = (uint16_t)y;
  }
  __syncthreads();
}

// ifftDITEncoder / ifftDITDecoder over m elements (mtrunc = m), skew index
// base + iend (encoder: base = m - 1 on fftSkew; decoder: base = -1).
__device__ void ifft16(uint16_t* w, int m, int base) {
  int dist = 1, dist4 = 4;
  while (dist4 <= m) {
    const int d = dist, d4 = dist4;
    // first butterflies: (i, i+d) with l01, (i+2d, i+3d) with l23
    step16<true>(w, m / 2, [&](int p, int& i, int& j, uint32_t& lm) {
      const int r = (p / (2 * d)) * d4, q = p % (2 * d), iend = r + d;
      if (q < d) { i = r + q; lm = g_skew16[base + iend]; }
      else { i = r + d + q; lm = g_skew16[base + iend + 2 * d]; }  // r + 2d + (q - d)
      j = i + d;
    });
    // second: (i, i+2d), (i+d, i+3d) with l02
    step16<true>(w, m / 2, [&](int p, int& i, int& j, uint32_t& lm) {
      const int r = (p / (2 * d)) * d4, q = p % (2 * d), iend = r + d;
      i = r + q;  // q < d: r + q ; q >= d: r + d + (q - d) == r + q
      j = i + 2 * d;
      lm = g_skew16[base + iend + d];
    });
    dist = dist4;
    dist4 <<= 2;
  }
  if (dist < m) {
    const int d = dist;
    step16<true>(w, d, [&](int p, int& i, int& j, uint32_t& lm) {
      i = p;
      j = p + d;
      lm = g_skew16[base + d];
    });
  }
}

// fftDIT over m elements (mtrunc = m), skew index fo + iend - 1 (encode:
// fo = 0; reverse fill: fo = m).
__device__ void fft16(uint16_t* w, int m, int fo) {
  int dist4 = m, dist = m >> 2;
  while (dist != 0) {
    const int d = dist, d4 = dist4;
    step16<false>(w, m / 2, [&](int p, int& i, int& j, uint32_t& lm) {
      const int r = (p / (2 * d)) * d4, q = p % (2 * d), iend = r + d;
      i = r + q;
      j = i + 2 * d;
      lm = g_skew16[fo + iend + d - 1];
    });
    step16<false>(w, m / 2, [&](int p, int& i, int& j, uint32_t& lm) {
      const int r = (p / (2 * d)) * d4, q = p % (2 * d), iend = r + d;
      if (q < d) { i = r + q; lm = g_skew16[fo + iend - 1]; }
      else { i = r + d + q; lm = g_skew16[fo + iend + 2 * d - 1]; }
      j = i + d;
    });
    dist4 = dist;
    dist >>= 2;
  }
  if (dist4 == 2) {
    step16<false>(w, m / 2, [&](int p, int& i, int& j, uint32_t& lm) {
      i = 2 * p;
      j = i + 1;
      lm = g_skew16[fo + i];
    });
  }
}

// The same locators from n-point transforms (n = 2k <= 1024).  The erasure
// vector is zero past n, so its 65536-point FWHT is n-periodic (popcount(i & j)
// only sees the low log2(n) bits of j when i < n), and only the first n
// outputs of the second transform are used, which sum the products over j = r
// (mod n): out = FWHT_n(FWHT_n(e) * wfold), wfold[r] = sum_q walsh[q*n + r]
// (mod 65535; a ring identity, so the values stay congruent to the reference's).
// One 256-thread workgroup per vector, 2 x log4(n) radix-4 stages in 4 KiB of
// LDS instead of 2 x 8 over 128 KiB (round 2: ~200 us per launch, set by the
// one head vector of each square's erasure pattern).
constexpr int kFoldThreads = 256;

template <int N>
__device__ __forceinline__ void fwht_n(uint32_t* e) {
  int dist = 1;
  if constexpr ((__builtin_ctz(N) & 1) != 0) {  // odd log2: one radix-2 stage first
    for (int g = threadIdx.x; g < N / 2; g += kFoldThreads) {
      const int i = 2 * g;
      const uint32_t t0 = e[i], t1 = e[i + 1];
      e[i] = add_mod16(t0, t1);
      e[i + 1] = sub_mod16(t0, t1);
    }
    __syncthreads();
    dist = 2;
  }
  for (; dist < N; dist <<= 2) {
    const int dist4 = dist << 2;
    for (int g = threadIdx.x; g < N / 4; g += kFoldThreads) {
      const int r = (g / dist) * dist4;
      const int i = r + (g % dist);
      const uint32_t t0 = e[i], t1 = e[i + dist], t2 = e[i + 2 * dist], t3 = e[i + 3 * dist];
      const uint32_t a0 = add_mod16(t0, t1), a1 = sub_mod16(t0, t1);
      const uint32_t a2 = add_mod16(t2, t3), a3 = sub_mod16(t2, t3);
      e[i] = add_mod16(a0, a2);
      e[i + 2 * dist] = sub_mod16(a0, a2);
      e[i + dist] = add_mod16(a1, a3);
      e[i + 3 * dist] = sub_mod16(a1, a3);
    }
    __syncthreads();
  }
}

constexpr int kTab16x = 20;  // dwords per 3/3/2 product table (mul16x_add_t)
__device__ __forceinline__ void mul16x_table_to(uint32_t* out, uint32_t lm);

template <int N>
__global__ __launch_bounds__(kFoldThreads) void leo16_errlocs_fold_kernel(DecodeArgs a) {
  __shared__ uint32_t e[N];
  __shared__ int cnt_s;
  const long v = blockIdx.x;
  const long sq = v / a.nvec, vec = v % a.nvec;
  constexpr int k = N / 2;
  const uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
  if (a.locators_only && !a.flags[v]) return;  // uniform
  const long hv = err_head_checked_block(a, v);
  if (a.locators_only && !err_computes(a, v, hv)) return;  // uniform
  if (threadIdx.x == 0) cnt_s = 0;
  __syncthreads();
  int cnt = 0;
  uint32_t miss = 0;  // bit r: element threadIdx.x + r * kFoldThreads is missing
  for (int i = threadIdx.x, r = 0; i < N; i += kFoldThreads, r++) {
    const uint32_t x = i < k ? (pres[(long)(k + i) * a.p_shard_stride] ? 0u : 1u)   // parity k+i -> work i
                             : (pres[(long)(i - k) * a.p_shard_stride] ? 0u : 1u);  // data i-k -> work i
    e[i] = x;
    miss |= x << r;
    cnt += (x == 0);
  }
  atomicAdd(&cnt_s, cnt);
  __syncthreads();
  const int present = cnt_s;
  bool decode = true;
  if (!a.locators_only) {
    decode = present >= k && present < N && vec_selected(a, v);
    if (threadIdx.x == 0) {
      a.flags[v] = decode ? 1 : 0;
      if (present < k && a.too_few) atomicOr(a.too_few, 1);
      if (decode && a.ndecodable) atomicAdd(a.ndecodable, 1);
    }
  }
  if (!decode) return;  // uniform
  if (!err_computes(a, v, hv)) return;  // shares an earlier vector's locators
  fwht_n<N>(e);
  const uint16_t* wf = g_wfold16[N == 512 ? 0 : N == 1024 ? 1 : 2];
  for (int i = threadIdx.x; i < N; i += kFoldThreads) e[i] = (e[i] * (uint32_t)wf[i]) % kMod16;
  __syncthreads();
  fwht_n<N>(e);
  uint16_t* out = (uint16_t*)(a.err + hv * (long)rs_err_bytes(k));
  for (int i = threadIdx.x; i < N; i += kFoldThreads) out[i] = (uint16_t)e[i];
  // Round 6: the half-lane decoders' per-element product tables, built here
  // once per erasure pattern (not in every decoder workgroup: 16 random exp
  // gathers per element were the decoder's slowest phase, tools/phase_probe.py
  // dec512h) -- exp(errLoc) for a present element (premultiply), exp(-errLoc)
  // for a missing one (postmultiply), element-major, 80 B each: the LDS image
  // the decoder copies with global_load_lds.
  uint32_t* tabs = (uint32_t*)(a.err + hv * (long)rs_err_bytes(k) + rs_err_tab_off(k));
  for (int i = threadIdx.x, r = 0; i < N; i += kFoldThreads, r++) {
    const uint32_t lm = e[i] & 0xFFFFu;
    mul16x_table_to(tabs + (long)i * kTab16x, ((miss >> r) & 1) ? kMod16 - lm : lm);
  }
}

// ---------------------------------------------------------------------------
// Decode: one 256-thread workgroup per (vector, 64-B column block); LDS holds
// work (n rows) and the formal-derivative output (n rows).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads16) void leo16_decode_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t w16[];
  const int k = a.k, n = 2 * k;
  const long nblk = a.shard_bytes / 64;
  const long blk = blockIdx.x % nblk;
  const long v = blockIdx.x / nblk;
  if (a.flags[v] == 0) return;  // uniform
  const long sq = v / a.nvec, vec = v % a.nvec;
  uint8_t* base = a.data + sq * a.sq_stride + vec * a.vec_stride + blk * 64;
  const uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
  const uint16_t* err = (const uint16_t*)(a.err + err_vec(a, v) * (long)rs_err_bytes(k));
  uint16_t* work = w16;
  uint16_t* der = w16 + n * 32;
  // work[i] = shard(pos(i)) * errLocs[i], zero if missing; layout [parity k][data k]
  for (int t = threadIdx.x; t < n * 8; t += kThreads16) {
    const int i = t >> 3, q = t & 7;
    const int shard = i < k ? k + i : i - k;
    uint32_t lo = 0, hi = 0;
    if (pres[(long)shard * a.p_shard_stride]) {
      const uint32_t* src = (const uint32_t*)(base + (long)shard * a.shard_stride);
      lo = src[q];
      hi = src[q + 8];
    }
    block_to_lds(work + i * 32, lo, hi, q);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < n * 32; t += kThreads16) {
    const int i = t >> 5;
    work[t] = (uint16_t)mul16(work[t], err[i]);
  }
  __syncthreads();
  ifft16(work, n, -1);
  // formal derivative: every read in the reference's sequential loop sees an
  // original value, so der[x] = work[x] ^ XOR_{b: bit b of x == 0} work[x + 2^b]
  for (int t = threadIdx.x; t < n * 32; t += kThreads16) {
    const int x = t >> 5, s = t & 31;
    uint32_t acc = work[t];
    for (int b = 1; b < n; b <<= 1)
      if ((x & b) == 0) acc ^= work[(x + b) * 32 + s];
    der[t] = (uint16_t)acc;
  }
  __syncthreads();
  fft16(der, n, 0);
  // reveal erasures: shard = work[pos] * (65535 - errLocs[pos])
  for (int t = threadIdx.x; t < n * 32; t += kThreads16) {
    const int i = t >> 5;
    const int shard = i < k ? k + i : i - k;
    if (!pres[(long)shard * a.p_shard_stride]) der[t] = (uint16_t)mul16(der[t], kMod16 - err[i]);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < n * 8; t += kThreads16) {
    const int i = t >> 3, q = t & 7;
    const int shard = i < k ? k + i : i - k;
    if (pres[(long)shard * a.p_shard_stride]) continue;
    uint32_t lo, hi;
    lds_to_block(der + i * 32, lo, hi, q);
    uint32_t* dst = (uint32_t*)(base + (long)shard * a.shard_stride);
    dst[q] = lo;
    dst[q + 8] = hi;
  }
}

__global__ __launch_bounds__(256) void mark_present16_kernel(DecodeArgs a) {
  const long v = blockIdx.x;
  if (a.flags[v] == 0) return;
  const long sq = v / a.nvec, vec = v % a.nvec;
  uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
  for (int i = threadIdx.x; i < 2 * a.k; i += 256) pres[(long)i * a.p_shard_stride] = 1;
  if (threadIdx.x == 0 && a.progress) atomicAdd(a.progress, 1);
}

// ---------------------------------------------------------------------------
// Register-resident GF(2^16) transforms (k = 256, 512; the half-lane kernels
// below).  Multiplies by a skew use per-position product tables read with
// scalar loads (the position is wave-uniform); a position whose skew is 65535
// (leopard "skip") has an all-zero table.
// ---------------------------------------------------------------------------
// a wave-uniform value the compiler cannot see through: values derived from it
// in one phase are not kept live (in SGPRs, then spilled) for the next
__device__ __forceinline__ int opaque_s(int x) {
  asm volatile("" : "+s"(x));
  return x;
}

// Positions < 2m = 1024 cover every encoder skew index (IFFT m-1+iend+2d <
// 2m, FFT iend-1 < m) and every k = 512 decoder one (iend - 1 < n).
// __constant__ so that the wave-uniform table reads become scalar loads.
constexpr int kTabPos = 4096;  // skew positions of the register kernels (decoders n <= 2048, encoders 2m <= 4096)

// 3/3/2 split (round 5): each byte of y in groups of 3, 3 and 2 bits, so a
// symbol takes 6 lookups per output byte instead of 8.  A 3-bit group indexes
// an 8-byte pool, i.e. two table dwords (perm(t[2i+1], t[2i], sel): selector
// bytes 0-3 pick from t[2i], 4-7 from t[2i+1]); the 2-bit group a 4-byte one
// (the same SGPR twice, no VGPR copy).  Per 4 symbols: 12 v_perm, 6 selectors
// from 4 shift / and pairs (2 plain ands), 6 xor3 = 28 ops (the 2-bit split:
// 16 v_perm, 14 selector ops, 8 xor3 = 38) plus, per table and phase, a VGPR
// copy of one dword of each of the 8 two-dword pools (a VOP3 reads one SGPR).
// Table (20 dwords per skew position, kTab16x):
//   [0,1] group 0 (y bits 0-2) -> product lo byte   [2,3] -> hi byte
//   [4,5] group 1 (bits 3-5) lo / [6,7] hi           [8] group 2 (bits 6-7) lo, [9] hi
//   [10..13] group 3 (bits 8-10), [14..17] group 4 (bits 11-13), [18, 19] group 5 (bits 14-15)
// entry e of a group at byte e of its pool: product (e << shift) * c.
__constant__ uint32_t g_ptab16x[kTabPos * kTab16x];
__constant__ uint32_t g_ptab16x_merged[4 * kTab16x];

__device__ __forceinline__ void mul16x_add_t(uint32_t& xlo, uint32_t& xhi, uint32_t ylo, uint32_t yhi,
                                             const uint32_t* t) {
  const uint32_t s0 = ylo & 0x07070707u, s1 = (ylo >> 3) & 0x07070707u, s2 = (ylo >> 6) & 0x03030303u;
  const uint32_t s3 = yhi & 0x07070707u, s4 = (yhi >> 3) & 0x07070707u, s5 = (yhi >> 6) & 0x03030303u;
  using B = uint32_t;
  const B l0 = __builtin_amdgcn_perm(t[1], t[0], s0), h0 = __builtin_amdgcn_perm(t[3], t[2], s0);
  const B l1 = __builtin_amdgcn_perm(t[5], t[4], s1), h1 = __builtin_amdgcn_perm(t[7], t[6], s1);
  const B l2 = __builtin_amdgcn_perm(t[8], t[8], s2), h2 = __builtin_amdgcn_perm(t[9], t[9], s2);
  const B l3 = __builtin_amdgcn_perm(t[11], t[10], s3), h3 = __builtin_amdgcn_perm(t[13], t[12], s3);
  const B l4 = __builtin_amdgcn_perm(t[15], t[14], s4), h4 = __builtin_amdgcn_perm(t[17], t[16], s4);
  const B l5 = __builtin_amdgcn_perm(t[18], t[18], s5), h5 = __builtin_amdgcn_perm(t[19], t[19], s5);
  xlo = xor3(xor3(xor3(xlo, l0, l1), l2, l3), l4, l5);
  xhi = xor3(xor3(xor3(xhi, h0, h1), h2, h3), h4, h5);
}

__device__ __forceinline__ void mul16_add(uint32_t& xlo, uint32_t& xhi, uint32_t ylo, uint32_t yhi, int pos) {
  mul16x_add_t(xlo, xhi, ylo, yhi, g_ptab16x + pos * kTab16x);
}
#define MERGED_TAB(m) (g_ptab16x_merged + kTab16x * (m))
#define MERGED_MUL mul16x_add_t

// NS elements per lane, 4 symbols each as a low-byte and a high-byte dword
template <int NS>
struct W16n {
  uint32_t lo[NS], hi[NS];
};

// ifftDIT2: y ^= x; x ^= y * skew[pos]
template <class W>
__device__ __forceinline__ void ifft2_16(W& w, int i, int j, int pos) {
  w.lo[j] ^= w.lo[i];
  w.hi[j] ^= w.hi[i];
  mul16_add(w.lo[i], w.hi[i], w.lo[j], w.hi[j], pos);
}
// fftDIT2: x ^= y * skew[pos]; y ^= x
template <class W>
__device__ __forceinline__ void fft2_16(W& w, int i, int j, int pos) {
  mul16_add(w.lo[i], w.hi[i], w.lo[j], w.hi[j], pos);
  w.lo[j] ^= w.lo[i];
  w.hi[j] ^= w.hi[i];
}

// the merged last-IFFT / first-FFT butterfly: y ^= x; x ^= y (A ^ B); y ^= x
template <class W>
__device__ __forceinline__ void ifft_fft2_16(W& w, int i, int j, const uint32_t* t) {
  w.lo[j] ^= w.lo[i];
  w.hi[j] ^= w.hi[i];
  MERGED_MUL(w.lo[i], w.hi[i], w.lo[j], w.hi[j], t);
  w.lo[j] ^= w.lo[i];
  w.hi[j] ^= w.hi[i];
}

// log of the element 1 << b (the decoders' per-element table builder)
__constant__ uint16_t g_logbit16[16];

// tok: a value written by the previous phase.  A table position passes through
// an asm that reads it, so no scalar table load is hoisted above that point and
// the tables of a layer are not all live at once (round 4: 848 v_writelane +
// 848 v_readlane spills without it, profiles/gf16_dec512_tok_r04.log).
__device__ __forceinline__ int opaque_tok(int x, uint32_t tok) {
  asm volatile("" : "+s"(x) : "v"(tok));
  return x;
}

// DAGPU_PHASE_PROBE builds (tools/phase_probe.py, never the product library):
// lane 0 of the first and last wave stamp s_memtime at the phase boundaries.
#ifdef DAGPU_PHASE_PROBE
constexpr int kProbePhases = 14;
__device__ uint64_t g_probe[8192 * 2 * kProbePhases];
__device__ uint64_t g_probe_e[8192 * 2 * kProbePhases];  // the half-lane encoders'
// half-lane kernels: waves 0 and QL (the last) of the first 8192 workgroups
#define H_PROBE(buf, i, QL)                                                                      \
  do {                                                                                          \
    if ((threadIdx.x & 63) == 0 && (q == 0 || q == (QL)) && blockIdx.x < 8192)                  \
      buf[(blockIdx.x * 2 + (q == (QL))) * kProbePhases + (i)] = __builtin_amdgcn_s_memtime();  \
  } while (0)
#else
#define H_PROBE(buf, i, QL) ((void)0)
#endif

// ---------------------------------------------------------------------------
// k = 512 / 256 decoder, round 5 (leo16_decode_h_kernel<K>): unpacked symbols with
// the 3/3/2 multiply (mul16x_add_t, 28 ops per 4 symbols) instead of the
// packed 2-bit one (22 ops per 2 symbols).  Unpacked, a lane holds 4 symbols of
// an element in 2 VGPRs, so 1,024 elements x 64 lanes would need the CU's
// whole register file; instead each register holds TWO elements, one per half
// wave (lanes 0-31 / 32-63, both halves the same 256 B of their shards):
// 16 waves x 32 register pairs x 2 halves = 1,024 elements, 64 data VGPRs.
// The half is element bit 0, so every layer but bit 0's has one skew position
// per register (the position depends on the bits above the layer's only).
// Layouts (q = wave, j = register pair, hl = lane half):
//   B  e = 64 q + 2 j + hl            layers on bits 1-5 (register bits 0-4)
//   T  e = hl | (j & 1) << 1 | q << 2 | (j >> 1) << 6
//                                     layers on bits 6-9, the formal derivative
//   S  e = 64 q + 2 (j & 15) + (j >> 4) + 32 hl
//                                     loads, stores, pre/post multiplies and the
//                                     bit-0 layer: pair (j, j + 16) is (x, y)
// S <-> B is one v_permlane32_swap per register pair (j, j + 16); B <-> T a
// 16 x 16 LDS transpose of q with j >> 1.  In S the two halves of a register
// belong to different bit-0 butterflies, so that layer's tables are per lane:
// 20 dwords read from g_ptab16x with vector loads (the other layers' come
// from SGPRs).  Pre/post multiplies: the decoders' 16-dword LDS tables
// (mul16_table_to), read per lane.
// ---------------------------------------------------------------------------
using W32 = W16n<32>;

// e of register j, lane half hl, in layout S (within the wave's 64 elements)
__device__ __forceinline__ constexpr int s_local(int j, int hl) { return 2 * (j & 15) + (j >> 4) + 32 * hl; }

// layout S <-> B: halves between registers j and j + 16
__device__ __forceinline__ void swap_sb(W32& w) {
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const auto l = __builtin_amdgcn_permlane32_swap(w.lo[j], w.lo[j + 16], false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(w.hi[j], w.hi[j + 16], false, false);
    w.lo[j] = l[0];
    w.lo[j + 16] = l[1];
    w.hi[j] = h[0];
    w.hi[j + 16] = h[1];
  }
}

// a skew position's 3/3/2 table into VGPRs (pos differs between the halves)
// (buffer loads: one 32-bit offset per lane instead of a 64-bit address)
__device__ __forceinline__ void lane_tab(int pos, uint32_t (&t)[kTab16x]) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const auto r = make_rsrc(g_ptab16x);
  const uint32_t off = (uint32_t)pos * (uint32_t)(kTab16x * 4);
#pragma unroll
  for (int i = 0; i < kTab16x / 4; i++) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off + 16u * i, 0, 0);
    t[4 * i] = v.x;
    t[4 * i + 1] = v.y;
    t[4 * i + 2] = v.z;
    t[4 * i + 3] = v.w;
  }
}

// bit-0 layer in layout S: x = register j, y = register j + 16 (j < 16), the
// pair's position = e of x (ifftDITDecoder / fftDIT: iend - 1 = block start)
// (the position passes through an asm that reads the pair's data: the IFFT's
// and the FFT's loads of the same tables are neither merged nor hoisted, which
// kept all 16 tables live through the kernel)
__device__ __forceinline__ int opaque_v(int x, uint32_t tok) {
  asm volatile("" : "+v"(x) : "v"(tok));
  return x;
}
// OFF: skew offset of the transform (decoder 0; encoder IFFT IO, FFT FO --
// ifftDITEncoder's index IO - 1 + iend is OFF + block start + dist - 1 too)
template <bool INV, int OFF = 0>
__device__ __forceinline__ void layer0_s(W32& w, int q, int hl) {
#pragma unroll
  for (int j = 0; j < 16; j++) {
    uint32_t t[kTab16x];
    // pair j's table is loaded once pair j - 1 is done: one table live at a time
    lane_tab(opaque_v(OFF + 64 * q + 2 * j + 32 * hl, w.lo[j > 0 ? j - 1 : 0]), t);
    if constexpr (INV) {  // ifftDIT2: y ^= x; x ^= y * skew
      w.lo[j + 16] ^= w.lo[j];
      w.hi[j + 16] ^= w.hi[j];
      mul16x_add_t(w.lo[j], w.hi[j], w.lo[j + 16], w.hi[j + 16], t);
    } else {  // fftDIT2: x ^= y * skew; y ^= x
      mul16x_add_t(w.lo[j], w.hi[j], w.lo[j + 16], w.hi[j + 16], t);
      w.lo[j + 16] ^= w.lo[j];
      w.hi[j + 16] ^= w.hi[j];
    }
    // computed here: otherwise the compiler sinks each pair's multiply to the
    // first use of its result and keeps the loaded tables live until then
    asm volatile("" : "+v"(w.lo[j]), "+v"(w.hi[j]), "+v"(w.lo[j + 16]), "+v"(w.hi[j + 16]));
  }
}

// a butterfly's results computed where it stands (the scheduler otherwise
// sinks multiplies toward their consumers and spills their operands)
__device__ __forceinline__ void pin_pair(W32& w, int i, int j) {
  asm volatile("" : "+v"(w.lo[i]), "+v"(w.hi[i]), "+v"(w.lo[j]), "+v"(w.hi[j]));
}

// One layer on element bit b >= 1 in layout B (dist D = 1 << b, registers j
// and j + D / 2): butterflies grouped by skew position (block of 2 D elements,
// position = block start + D - 1), one table per group.
template <bool INV, int D, int OFF = 0>
__device__ __forceinline__ void layer_b(W32& w, int q) {
  constexpr int RD = D / 2;
#pragma unroll
  for (int r = 0; r < 64; r += 2 * D) {
    const int pos = opaque_tok(OFF + 64 * q + r + D - 1, w.lo[r / 2]);
#pragma unroll
    for (int e = r; e < r + D; e += 2) {
      if constexpr (INV) ifft2_16(w, e / 2, e / 2 + RD, pos);
      else fft2_16(w, e / 2, e / 2 + RD, pos);
      pin_pair(w, e / 2, e / 2 + RD);
    }
  }
}

// One layer on element bit b >= 6 in layout T (LR low register bits stay
// element bits 1..LR, the wave holds the next 5 - LR, register bits LR.. are
// element bits 6..; decoder n = 1024: LR = 1, encoder m = 512: LR = 2):
// positions are compile-time (bits above b are register bits).  The block at
// OFF + blk = 0 has position D - 1, whose skew is log 0 (the only zero skews are
// at 2^m - 1): Leopard skips its multiply, and so does this (y ^= x alone, in
// the IFFT and the FFT butterfly) -- half of the layer at 2 D = n / 2, all of
// the top layer.
template <bool INV, int D, int LR = 1, int OFF = 0>
__device__ __forceinline__ void layer_t(W32& w) {
  constexpr int RD = (D / 64) << LR;
  constexpr int N = 64 << (5 - LR);  // elements of the transform
#pragma unroll
  for (int blk = 0; blk < N; blk += 2 * D) {  // element block start (bits > b)
    const bool zero = OFF + blk == 0;  // compile-time once unrolled
    const int jf = (blk >> 6) << LR;  // first register of the block
    const int pos = zero ? 0 : opaque_tok(OFF + blk + D - 1, w.lo[jf]);  // loaded here, not hoisted / merged
#pragma unroll
    for (int j = 0; j < 32; j++) {
      if (j & RD) continue;
      if ((((j >> LR) << 6) & ~(2 * D - 1)) != blk) continue;
      if (zero) {
        w.lo[j + RD] ^= w.lo[j];
        w.hi[j + RD] ^= w.hi[j];
      } else if constexpr (INV) {
        ifft2_16(w, j, j + RD, pos);
      } else {
        fft2_16(w, j, j + RD, pos);
      }
      pin_pair(w, j, j + RD);
    }
  }
}

// B <-> T: wave q, register (jj << LR) | r  <->  wave jj, register (q << LR) | r
// (NQ = 32 >> LR waves); RPR values of r per LDS round (NQ * NQ * RPR * 256 B)
template <int LR = 1, int RPR = 1>
__device__ __forceinline__ void xpose_bt(W32& w, uint32_t* lds, int q, int lane) {
  constexpr int NQ = 32 >> LR;
#pragma unroll
  for (int r0 = 0; r0 < (1 << LR); r0 += RPR) {
#pragma unroll
    for (int lh = 0; lh < 2; lh++) {
#pragma unroll
      for (int c = 0; c < NQ; c++)
#pragma unroll
        for (int u = 0; u < RPR; u++)
          lds[((c * NQ + q) * RPR + u) * 64 + lane] = lh ? w.hi[(c << LR) | (r0 + u)] : w.lo[(c << LR) | (r0 + u)];
      __syncthreads();
#pragma unroll
      for (int c = 0; c < NQ; c++)
#pragma unroll
        for (int u = 0; u < RPR; u++) {
          const uint32_t v = lds[((q * NQ + c) * RPR + u) * 64 + lane];
          if (lh) w.hi[(c << LR) | (r0 + u)] = v;
          else w.lo[(c << LR) | (r0 + u)] = v;
        }
      __syncthreads();
    }
  }
}

// xpose_bt over two LDS buffers of one round each (round r in buffer (B0 + r)
// & 1, buffer 1 at lds + NQ * NQ * RPR * 64): a barrier between a round's
// writes and reads, none after the reads -- the next round writes the other
// buffer, and the one after it writes this buffer only past the next round's
// barrier, which every wave reaches after its reads here (round 6: the k = 512
// decoder's transposes and derivative 8 -> 4 barriers each).
template <int LR, int RPR, int B0>
__device__ __forceinline__ void xpose_bt_db(W32& w, uint32_t* lds, int q, int lane) {
  constexpr int NQ = 32 >> LR;
  constexpr int RW = NQ * NQ * RPR * 64;  // dwords per round
#pragma unroll
  for (int r0 = 0; r0 < (1 << LR); r0 += RPR) {
#pragma unroll
    for (int lh = 0; lh < 2; lh++) {
      uint32_t* buf = lds + ((B0 + 2 * (r0 / RPR) + lh) & 1) * RW;
#pragma unroll
      for (int c = 0; c < NQ; c++)
#pragma unroll
        for (int u = 0; u < RPR; u++)
          buf[((c * NQ + q) * RPR + u) * 64 + lane] = lh ? w.hi[(c << LR) | (r0 + u)] : w.lo[(c << LR) | (r0 + u)];
      __syncthreads();
#pragma unroll
      for (int c = 0; c < NQ; c++)
#pragma unroll
        for (int u = 0; u < RPR; u++) {
          const uint32_t v = buf[((q * NQ + c) * RPR + u) * 64 + lane];
          if (lh) w.hi[(c << LR) | (r0 + u)] = v;
          else w.lo[(c << LR) | (r0 + u)] = v;
        }
    }
  }
}

// Formal derivative in layout T, D(x)_e = x_e ^ XOR_{s: bit s of e = 0} x_{e | 2^s}:
// register bits (element bits 1..LR and 6..) in place in ascending register
// order, wave bits (LR+1 .. 5) and the half bit (0, lanes 0-31 read lane + 32)
// from the originals staged in LDS, 8 register pairs per round (NQ waves).
// DB: two buffers of one round each, alternating as in xpose_bt_db (round r in
// buffer r & 1, no barrier after a round's reads); otherwise one buffer.
template <int NQ, bool DB = false>
__device__ __forceinline__ void derivative_t(W32& w, uint32_t* lds0, int c, int lane, uint32_t lowmask) {
  constexpr int B = 8;
#pragma unroll
  for (int s0 = 0; s0 < 32; s0 += B) {
    uint32_t* lds = lds0 + (DB ? ((s0 / B) & 1) * (NQ * B * 2 * 64) : 0);
#pragma unroll
    for (int u = 0; u < B; u++) {
      lds[((c * B + u) * 2) * 64 + lane] = w.lo[s0 + u];
      lds[((c * B + u) * 2 + 1) * 64 + lane] = w.hi[s0 + u];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < B; u++) {
      const int j = s0 + u;
      uint32_t alo = w.lo[j], ahi = w.hi[j];
#pragma unroll
      for (int bit = 1; bit < 32; bit <<= 1)
        if ((j & bit) == 0) {
          alo ^= w.lo[j | bit];
          ahi ^= w.hi[j | bit];
        }
#pragma unroll
      for (int wb = 1; wb < NQ; wb <<= 1)
        if ((c & wb) == 0) {
          alo ^= lds[(((c | wb) * B + u) * 2) * 64 + lane];
          ahi ^= lds[(((c | wb) * B + u) * 2 + 1) * 64 + lane];
        }
      // bit 0: lanes 0-31 (hl = 0) add their partner's (lane + 32) original
      alo ^= lds[((c * B + u) * 2) * 64 + (lane ^ 32)] & lowmask;
      ahi ^= lds[((c * B + u) * 2 + 1) * 64 + (lane ^ 32)] & lowmask;
      asm volatile("" : "+v"(alo), "+v"(ahi));  // one register's partner reads in flight at a time
      w.lo[j] = alo;
      w.hi[j] = ahi;
    }
    if constexpr (!DB) __syncthreads();
  }
}

// ONE product table per element, in the 3/3/2 format of mul16x_add_t (round 5):
// exp(errLoc) for a present element (premultiply), exp(-errLoc) for a missing
// one (postmultiply).  A missing element's loaded bytes are zero (or zeroed)
// and a present one is never stored, so neither needs the other table.  From
// the 16 products pb[b] = (1 << b) * exp(lm): a 3-bit group's entries 0..3 are
// (0, p0, p1, p0 ^ p1) and entries 4..7 those XOR p2 (GF(2)-linear multiply).
__device__ __forceinline__ void mul16x_table_to(uint32_t* out, uint32_t lm) {
  uint32_t pb[16];
#pragma unroll
  for (int b = 0; b < 16; b++) {
    uint32_t sidx = (uint32_t)g_logbit16[b] + lm;
    sidx = (sidx + (sidx >> 16)) & 0xFFFFu;
    pb[b] = g_exp16[sidx];
  }
  uint32_t t[kTab16x];
  // entries 0..3 of a group over basis products p0, p1: low bytes, high bytes
  auto quad = [&](uint32_t p0, uint32_t p1, uint32_t& lo, uint32_t& hi) {
    const uint32_t q = p0 ^ p1;
    lo = __builtin_amdgcn_perm(q, __builtin_amdgcn_perm(p1, p0, 0x0C04000Cu), 0x04020100u);
    hi = __builtin_amdgcn_perm(q, __builtin_amdgcn_perm(p1, p0, 0x0C05010Cu), 0x05020100u);
  };
  auto grp3 = [&](int b0, int base) {
    uint32_t lo, hi;
    quad(pb[b0], pb[b0 + 1], lo, hi);
    t[base] = lo;
    t[base + 1] = lo ^ __builtin_amdgcn_perm(pb[b0 + 2], pb[b0 + 2], 0x00000000u);
    t[base + 2] = hi;
    t[base + 3] = hi ^ __builtin_amdgcn_perm(pb[b0 + 2], pb[b0 + 2], 0x01010101u);
  };
  auto grp2 = [&](int b0, int base) { quad(pb[b0], pb[b0 + 1], t[base], t[base + 1]); };
  grp3(0, 0);
  grp3(3, 4);
  grp2(6, 8);
  grp3(8, 10);
  grp3(11, 14);
  grp2(14, 18);
  uint4* o = (uint4*)out;
#pragma unroll
  for (int i = 0; i < kTab16x / 4; i++) o[i] = make_uint4(t[4 * i], t[4 * i + 1], t[4 * i + 2], t[4 * i + 3]);
}
__device__ __forceinline__ void mul16x_table_from(const uint32_t* tab, int e, uint32_t (&t)[kTab16x]) {
  const uint4* q = (const uint4*)(tab + e * kTab16x);
#pragma unroll
  for (int h = 0; h < kTab16x / 4; h++) {
    const uint4 v = q[h];
    t[4 * h] = v.x;
    t[4 * h + 1] = v.y;
    t[4 * h + 2] = v.z;
    t[4 * h + 3] = v.w;
  }
}
// (xl, xh) *= the table's multiplier
__device__ __forceinline__ void mul16x_by(uint32_t& xl, uint32_t& xh, const uint32_t (&t)[kTab16x]) {
  uint32_t zl = 0u, zh = 0u;
  mul16x_add_t(zl, zh, xl, xh, t);
  xl = zl;
  xh = zh;
}

// K = 512 (n = 1024, 16 waves, LR = 1) and, round 5, K = 256 (n = 512, 8 waves,
// LR = 2: 512 threads at <= 128 VGPRs and 72 KiB of LDS, two workgroups per CU).
// Dynamic LDS, round 6:
//   K = 512 (one workgroup per CU, 160 KiB): buffers A = [0, 64 KiB) and
//     B = [64, 128 KiB) of the double-buffered transposes and derivative
//     (xpose_bt_db), the n x 80-B tables at [80, 160 KiB) -- at the start for
//     the premultiply and reloaded after the last transpose for the
//     postmultiply (the first round that writes B follows a barrier every wave
//     reaches after its premultiply);
//   K = 256: [0, n x 64 B) single-buffered staging, then the n x 80-B tables.
// bit-0 layer in layout S with its tables from LDS (round 6): `posl` holds the
// tables of the even positions OFF + 2 i at i x 80 B (pos_tables_to_lds), so a
// lane reads its pair's table with ds_read_b128 (the two halves of a wave read
// two tables) instead of five buffer loads from the constant tables per pair,
// whose latency each pair waited for (one table live at a time).
template <bool INV>
__device__ __forceinline__ void layer0_sl(W32& w, int q, int hl, const uint32_t* posl) {
#pragma unroll
  for (int j = 0; j < 16; j++) {
    uint32_t t[kTab16x];
    mul16x_table_from(posl, opaque_v(32 * q + j + 16 * hl, w.lo[j > 0 ? j - 1 : 0]), t);
    if constexpr (INV) {
      w.lo[j + 16] ^= w.lo[j];
      w.hi[j + 16] ^= w.hi[j];
      mul16x_add_t(w.lo[j], w.hi[j], w.lo[j + 16], w.hi[j + 16], t);
    } else {
      mul16x_add_t(w.lo[j], w.hi[j], w.lo[j + 16], w.hi[j + 16], t);
      w.lo[j + 16] ^= w.lo[j];
      w.hi[j + 16] ^= w.hi[j];
    }
    asm volatile("" : "+v"(w.lo[j]), "+v"(w.hi[j]), "+v"(w.lo[j + 16]), "+v"(w.hi[j + 16]));
  }
}

typedef __attribute__((address_space(3))) void* lds_vptr;
typedef __attribute__((address_space(1))) void* glb_vptr;
// The constant tables of the NPOS even positions OFF, OFF + 2, .. into LDS
// (i x 80 B) with global_load_lds, THREADS threads: 16-B chunk c (table c / 5,
// part c % 5) lane-linear within each wave.
template <int NPOS, int THREADS, int OFF>
__device__ __forceinline__ void pos_tables_to_lds(uint32_t* dst, int q, int lane) {
  constexpr int NCH = NPOS * 5;
  static_assert(NCH % 64 == 0, "whole waves of chunks");
  const uint8_t* src = (const uint8_t*)(const void*)g_ptab16x;
#pragma unroll
  for (int i = 0; i < (NCH + THREADS - 1) / THREADS; i++) {
    const int c0 = i * THREADS + 64 * q;  // the wave's first chunk (uniform)
    if (c0 < NCH) {
      const int c = c0 + lane;
      const uint8_t* g = src + (long)(OFF + 2 * (c / 5)) * (kTab16x * 4) + (c % 5) * 16;
      __builtin_amdgcn_global_load_lds((glb_vptr)g, (lds_vptr)(dst + c0 * 4), 16, 0, 0);
    }
  }
}

// The tables of one wave's 32 bit-0-layer positions OFF + 2 i, i in [32 q, 32 q + 32)
// (the half-lane encoders' layout S), into the LDS image of pos_tables_to_lds by
// the wave itself: 160 chunks of 16 B, so the wave needs no workgroup barrier,
// only its own vmcnt wait (wait_dma) before reading them.
template <int OFF>
__device__ __forceinline__ void pos_tables_wave(uint32_t* dst, int q, int lane) {
  const uint8_t* src = (const uint8_t*)(const void*)g_ptab16x;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const int c0 = 160 * q + 64 * i;  // uniform
    const int c = c0 + lane;
    if (i < 2 || lane < 32) {
      const uint8_t* g = src + (long)(OFF + 2 * (c / 5)) * (kTab16x * 4) + (c % 5) * 16;
      __builtin_amdgcn_global_load_lds((glb_vptr)g, (lds_vptr)(dst + c0 * 4), 16, 0, 0);
    }
  }
}
__device__ __forceinline__ void wait_dma() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <int K>
constexpr size_t dec_h_tab_off() { return K == 512 ? 80 * 1024 : (size_t)(2 * K) * 64; }
template <int K>
constexpr size_t dec_h_lds_bytes() { return dec_h_tab_off<K>() + (size_t)(2 * K) * kTab16x * sizeof(uint32_t); }
static_assert(dec_h_lds_bytes<512>() == 160 * 1024 && dec_h_lds_bytes<256>() == 72 * 1024, "decoder LDS");

// The n x 80-B table image of vector v's erasure pattern (leo16_errlocs_fold_kernel)
// into LDS with global_load_lds (no VGPRs, 5 x 16 B per thread): chunk
// c = i * 2K + thread, lane-linear within each wave as the DMA writes it.
template <int K>
__device__ __forceinline__ void dec_h_load_tables(uint32_t* tab, const uint8_t* img, int q, int lane) {
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const long c = (long)i * (2 * K) + 64 * q;  // the wave's first chunk
    __builtin_amdgcn_global_load_lds((glb_vptr)(img + (c + lane) * 16), (lds_vptr)(tab + c * 4), 16, 0, 0);
  }
}

// A missing shard's load gets an out-of-range voffset (the buffer returns 0
// without touching memory), halving a maximal-erasure vector's load traffic
// (+0.4 %, profiles/gf16_skip_ab_r05.log).  (8-byte lane-pair loads with a DPP
// swap, half the vector-memory instructions, measured no faster:
// profiles/gf16_load64_ab_r05.log.)
template <int K>
__global__ __launch_bounds__(2 * K) __attribute__((amdgpu_waves_per_eu(4, 4))) void leo16_decode_h_kernel(
    DecodeArgs a) {
  constexpr int NQ = K / 32, LR = K == 512 ? 1 : 2, RPR = K == 512 ? 1 : 2;
  static_assert(2 * K * kTab16x * 4 == 5 * 16 * 2 * K, "five 16-B chunks per thread");
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn_lds[];
  uint32_t* lds = dyn_lds;
  uint32_t* tab = dyn_lds + dec_h_tab_off<K>() / 4;
  const long blk = blockIdx.x;
  const int piece = (int)(blk % a.nchunk);  // nchunk = 256-B pieces of the shard
  const long v = blk / a.nchunk;
  if (a.flags[v] == 0) return;  // uniform
  const long sq = v / a.nvec, vec = v % a.nvec;
  const int lane = threadIdx.x & 63;
  const int hl = lane >> 5;
  const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lowmask = hl ? 0u : 0xFFFFFFFFu;
  H_PROBE(g_probe, 0, NQ - 1);
  // lane (hl, c): 64-B block c >> 3 of this 256-B piece, symbols 4 (c & 7) .. +3
  const uint32_t col = (uint32_t)piece * 256u + (uint32_t)((lane & 31) >> 3) * 64u + (uint32_t)(lane & 7) * 4u;
  const uint32_t voff = col + (uint32_t)hl * 32u * (uint32_t)a.shard_stride;  // upper half: shard + 32
  const auto rsrc = make_rsrc(a.data + sq * a.sq_stride + vec * a.vec_stride);
  const uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
  const uint8_t* img = a.err + err_vec(a, v) * rs_err_bytes(K) + rs_err_tab_off(K);
  dec_h_load_tables<K>(tab, img, q, lane);
  pos_tables_to_lds<K, 2 * K, 0>(lds, q, lane);  // the bit-0 layers' tables into the staging area
  const int my_i = 64 * q + lane;
  const int my_shard = my_i < K ? K + my_i : my_i - K;
  const uint64_t pm = __builtin_amdgcn_ballot_w64(pres[(long)my_shard * a.p_shard_stride] != 0);
  W32 w;
  const int q_ld = opaque_s(q);
  const uint32_t pmh_ld = hl ? (uint32_t)(pm >> 32) : (uint32_t)pm;
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const int i = 64 * q_ld + s_local(j, 0);
    const int shard = i < K ? K + i : i - K;
    const uint32_t so = (uint32_t)shard * (uint32_t)a.shard_stride;
    // missing: voffset >= 2^31 > num_records (soffset < 2^30 here), so out of range
    const uint32_t vj = ((pmh_ld >> s_local(j, 0)) & 1) ? voff : (voff | 0x80000000u);
    w.lo[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, vj, so, 0);
    w.hi[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, vj + 32u, so, 0);
  }
  // every wave's table DMA has landed (an explicit vmcnt(0): hipcc's barrier
  // fence waits only for lgkmcnt here, checked in the ISA) before any wave reads
  wait_dma();
  __syncthreads();
  H_PROBE(g_probe, 1, NQ - 1);
  const int q_pm = opaque_s(q);
#pragma unroll
  for (int j = 0; j < 32; j++) {
    uint32_t t[kTab16x];
    mul16x_table_from(tab, 64 * q_pm + s_local(j, 0) + 32 * hl, t);
    uint32_t xl = w.lo[j], xh = w.hi[j];
    mul16x_by(xl, xh, t);
    asm volatile("" : "+v"(xl), "+v"(xh));  // one element's table live at a time
    w.lo[j] = xl;
    w.hi[j] = xh;
  }
  H_PROBE(g_probe, 2, NQ - 1);
  // ---- IFFT (ifftDITDecoder, skew index iend - 1) ----
  layer0_sl<true>(w, q, hl, lds);
  swap_sb(w);
  H_PROBE(g_probe, 3, NQ - 1);
  layer_b<true, 2>(w, q);
  layer_b<true, 4>(w, q);
  layer_b<true, 8>(w, q);
  layer_b<true, 16>(w, q);
  layer_b<true, 32>(w, q);
  H_PROBE(g_probe, 4, NQ - 1);
  __syncthreads();  // every wave's reads of the position tables are done
  if constexpr (K == 512) xpose_bt_db<LR, RPR, 0>(w, lds, q, lane);  // rounds A B A B
  else xpose_bt<LR, RPR>(w, lds, q, lane);
  H_PROBE(g_probe, 5, NQ - 1);
  layer_t<true, 64, LR>(w);
  layer_t<true, 128, LR>(w);
  layer_t<true, 256, LR>(w);
  if constexpr (K == 512) layer_t<true, 512, LR>(w);
  H_PROBE(g_probe, 6, NQ - 1);
  derivative_t<NQ, K == 512>(w, lds, q, lane, lowmask);  // A B A B
  H_PROBE(g_probe, 7, NQ - 1);
  // ---- FFT (fftDIT, skew index iend - 1) ----
  if constexpr (K == 512) layer_t<false, 512, LR>(w);
  layer_t<false, 256, LR>(w);
  layer_t<false, 128, LR>(w);
  layer_t<false, 64, LR>(w);
  H_PROBE(g_probe, 8, NQ - 1);
  if constexpr (K == 512) {
    xpose_bt_db<LR, RPR, 0>(w, lds, q, lane);  // A B A B
    // every wave's reads of B are done: the tables come back over it while the
    // B and S layers run (their DMA is waited for at the barrier below)
    __syncthreads();
  } else {
    xpose_bt<LR, RPR>(w, lds, q, lane);
  }
  if constexpr (K == 512) dec_h_load_tables<K>(tab, img, q, lane);  // (K = 256: never overwritten)
  pos_tables_to_lds<K, 2 * K, 0>(lds, q, lane);
  H_PROBE(g_probe, 9, NQ - 1);
  layer_b<false, 32>(w, q);
  layer_b<false, 16>(w, q);
  layer_b<false, 8>(w, q);
  layer_b<false, 4>(w, q);
  layer_b<false, 2>(w, q);
  H_PROBE(g_probe, 10, NQ - 1);
  swap_sb(w);
  wait_dma();  // the tables' DMA has landed in every wave before any reads them
  __syncthreads();
  layer0_sl<false>(w, q, hl, lds);
  H_PROBE(g_probe, 11, NQ - 1);
  // erased shards = work * (65535 - errLocs), per lane; a register whose two
  // elements are both given is skipped (wave-uniform)
  uint64_t pm_e = pm;
  int q_e = q;
  asm volatile("" : "+s"(pm_e), "+s"(q_e));
  const uint32_t pmh = hl ? (uint32_t)(pm_e >> 32) : (uint32_t)pm_e;
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const int l0 = s_local(j, 0);
    if (((pm_e >> l0) & 1) && ((pm_e >> (l0 + 32)) & 1)) continue;  // uniform
    uint32_t t[kTab16x];
    mul16x_table_from(tab, 64 * q_e + l0 + 32 * hl, t);
    uint32_t xl = w.lo[j], xh = w.hi[j];
    mul16x_by(xl, xh, t);
    asm volatile("" : "+v"(xl), "+v"(xh));
    const int i = 64 * q_e + l0;
    const int shard = i < K ? K + i : i - K;
    const uint32_t so = (uint32_t)shard * (uint32_t)a.shard_stride;
    if (!((pmh >> l0) & 1)) {
      __builtin_amdgcn_raw_buffer_store_b32(xl, rsrc, voff, so, 0);
      __builtin_amdgcn_raw_buffer_store_b32(xh, rsrc, voff + 32u, so, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  H_PROBE(g_probe, 12, NQ - 1);
}

// ---------------------------------------------------------------------------
// k = 512 decoder, round 6 (leo16_decode_q_kernel): QUARTER lanes, so that two
// workgroups share a CU and one's barrier waits, loads and stores overlap the
// other's butterflies (leo16_decode_h_kernel's 1,024 threads own a CU alone;
// verdict r05: 0.59 VALU instructions per clock per CU, 37 % of wave cycles
// waiting).  A lane quarter (16 lanes) holds 128 B of a shard -- lane l: quarter
// ql = l >> 4, 64-B block (l >> 3) & 1, symbols 4 (l & 7) .. +3 -- and every
// register four elements, one per quarter: 8 waves x 32 registers x 4 quarters
// = the n = 1024 elements of one 128-B piece in 64 data VGPRs at <= 128 VGPRs,
// 512 threads and 64 KiB of LDS per workgroup.  Layouts (q = wave, j = register):
//   S  e = (j >> 3) + 4 (j & 7) + 32 ql + 128 q   loads, stores, pre/post
//                                                 multiplies, layers on bits 0, 1
//   B  e = ql + 4 j + 128 q                        layers on bits 2-6
//   T  e = ql + 4 (j & 3) + 16 q + 128 (j >> 2)    layers on bits 7-9, derivative
// S <-> B: a 4 x 4 transpose of (j >> 3, ql) per register group j & 7
// (v_permlane32_swap, then v_permlane16_swap); B <-> T: xpose_bt_db (LR = 2,
// NQ = 8 waves).  In S the quarters of a register are different butterflies,
// so the bit-0 and bit-1 layers read per-lane tables, from LDS images each
// wave fills for its own positions (pos_tables_wave-style).  The erasure
// multiplies read the head's per-element table image (leo16_errlocs_fold_kernel)
// per lane from L2.  Host emulation of the layouts: tests/test_quarterlane_emu.py.
// ---------------------------------------------------------------------------
using WQ = W16n<32>;

__device__ __forceinline__ constexpr int q_elem_s(int j, int ql) { return (j >> 3) + 4 * (j & 7) + 32 * ql; }

// S <-> B (its own inverse): per register group g, registers g, g+8, g+16, g+24
__device__ __forceinline__ void swap_sb_q(WQ& w) {
#pragma unroll
  for (int g = 0; g < 8; g++) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      uint32_t* v = h ? w.hi : w.lo;
      const auto a = __builtin_amdgcn_permlane32_swap(v[g], v[g + 16], false, false);
      const auto b = __builtin_amdgcn_permlane32_swap(v[g + 8], v[g + 24], false, false);
      const auto c = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
      const auto d = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
      v[g] = c[0];
      v[g + 8] = c[1];
      v[g + 16] = d[0];
      v[g + 24] = d[1];
    }
  }
}

// A table from a per-lane byte offset into an LDS image
__device__ __forceinline__ void lds_tab(const uint32_t* img, uint32_t byte_off, uint32_t (&t)[kTab16x]) {
  const uint4* p = (const uint4*)((const uint8_t*)img + byte_off);
#pragma unroll
  for (int h = 0; h < kTab16x / 4; h++) {
    const uint4 v = p[h];
    t[4 * h] = v.x;
    t[4 * h + 1] = v.y;
    t[4 * h + 2] = v.z;
    t[4 * h + 3] = v.w;
  }
}

// Layer on element bit b (0 or 1) in S: x = register j, y = j + 8 (b = 0) /
// j + 16 (b = 1).  Position (e & ~(2d - 1)) + d - 1 per lane; the wave's images:
// bit 0 at img0 + (e(x) - 128 q) / 2 * 80, bit 1 at img1 + (e(x) - 128 q) / 4 * 80.
template <bool INV, int B, bool FRESH = false>
__device__ __forceinline__ void layer_s_q(WQ& w, int ql, const uint32_t* img) {
  constexpr int RD = 8 << B;  // register distance of the pair
  // FRESH (k = 1024's FFT side): a fresh quarter index, so that the table
  // offsets are not the IFFT's, held (spilled) across the kernel
  if constexpr (FRESH) asm volatile("" : "+v"(ql));
#pragma unroll
  for (int j = 0; j < 32; j++) {
    if ((j >> 3) & (1 << B)) continue;
    const int le = q_elem_s(j, 0) + 32 * ql;  // e(x) - 128 q
    uint32_t t[kTab16x];
    lds_tab(img, (uint32_t)opaque_v((le >> (B + 1)) * (kTab16x * 4), w.lo[j > 0 ? j - 1 : 0]), t);
    if constexpr (INV) {
      w.lo[j + RD] ^= w.lo[j];
      w.hi[j + RD] ^= w.hi[j];
      mul16x_add_t(w.lo[j], w.hi[j], w.lo[j + RD], w.hi[j + RD], t);
    } else {
      mul16x_add_t(w.lo[j], w.hi[j], w.lo[j + RD], w.hi[j + RD], t);
      w.lo[j + RD] ^= w.lo[j];
      w.hi[j + RD] ^= w.hi[j];
    }
    asm volatile("" : "+v"(w.lo[j]), "+v"(w.hi[j]), "+v"(w.lo[j + RD]), "+v"(w.hi[j + RD]));
  }
}

// Layer on element bit b in 2..6 in B: registers j, j + 2^(b-2); position
// 128 q + 4 jb + d - 1 for the register block jb (wave-uniform, scalar tables)
template <bool INV, int B, int OFF = 0>
__device__ __forceinline__ void layer_b_q(WQ& w, int q) {
  constexpr int RD = 1 << (B - 2), D = 1 << B;
#pragma unroll
  for (int jb = 0; jb < 32; jb += 2 * RD) {
    const int pos = opaque_tok(OFF + 128 * q + 4 * jb + D - 1, w.lo[jb]);
#pragma unroll
    for (int j = jb; j < jb + RD; j++) {
      if constexpr (INV) ifft2_16(w, j, j + RD, pos);
      else fft2_16(w, j, j + RD, pos);
      pin_pair(w, j, j + RD);
    }
  }
}

// Layer on element bit b in 7..9 in T: registers j, j + 4 * 2^(b-7);
// compile-time positions 128 (jb >> 2) + d - 1; block start 0 is a zero skew
template <bool INV, int B, int LR = 2>
__device__ __forceinline__ void layer_t_q(WQ& w) {
  constexpr int RD = (1 << LR) << (B - 7), D = 1 << B;
#pragma unroll
  for (int jb = 0; jb < 32; jb += 2 * RD) {
    const bool zero = jb == 0;
    const int pos = zero ? 0 : opaque_tok(128 * (jb >> LR) + D - 1, w.lo[jb]);
#pragma unroll
    for (int j = jb; j < 32; j++) {
      if ((j & ~(2 * RD - 1)) != jb || (j & RD)) continue;
      if (zero) {
        w.lo[j + RD] ^= w.lo[j];
        w.hi[j + RD] ^= w.hi[j];
      } else if constexpr (INV) {
        ifft2_16(w, j, j + RD, pos);
      } else {
        fft2_16(w, j, j + RD, pos);
      }
      pin_pair(w, j, j + RD);
    }
  }
}

// Formal derivative in T: register bits (element bits 2, 3, 7-9) in place in
// ascending register order; wave bits (4-6) and quarter bits (0: lane ^ 16,
// 1: lane ^ 32) from the originals staged in LDS, 8 registers per round in two
// alternating 32-KiB buffers (no barrier after a round's reads).
template <int NQ = 8>
__device__ __forceinline__ void derivative_tq(WQ& w, uint32_t* lds0, int c, int lane) {
  constexpr int B = 8, RW = NQ * B * 2 * 64;
  const uint32_t m16 = ((lane >> 4) & 1) ? 0u : 0xFFFFFFFFu, m32 = ((lane >> 5) & 1) ? 0u : 0xFFFFFFFFu;
#pragma unroll
  for (int s0 = 0; s0 < 32; s0 += B) {
    uint32_t* lds = lds0 + ((s0 / B) & 1) * RW;
#pragma unroll
    for (int u = 0; u < B; u++) {
      lds[((c * B + u) * 2) * 64 + lane] = w.lo[s0 + u];
      lds[((c * B + u) * 2 + 1) * 64 + lane] = w.hi[s0 + u];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < B; u++) {
      const int j = s0 + u;
      uint32_t alo = w.lo[j], ahi = w.hi[j];
#pragma unroll
      for (int bit = 1; bit < 32; bit <<= 1)
        if ((j & bit) == 0) {
          alo ^= w.lo[j | bit];
          ahi ^= w.hi[j | bit];
        }
#pragma unroll
      for (int wb = 1; wb < NQ; wb <<= 1)
        if ((c & wb) == 0) {
          alo ^= lds[(((c | wb) * B + u) * 2) * 64 + lane];
          ahi ^= lds[(((c | wb) * B + u) * 2 + 1) * 64 + lane];
        }
      const uint32_t* me = lds + ((c * B + u) * 2) * 64;
      alo ^= (me[lane ^ 16] & m16) ^ (me[lane ^ 32] & m32);
      ahi ^= (me[64 + (lane ^ 16)] & m16) ^ (me[64 + (lane ^ 32)] & m32);
      asm volatile("" : "+v"(alo), "+v"(ahi));
      w.lo[j] = alo;
      w.hi[j] = ahi;
    }
  }
}

// The wave's S-layer tables into its LDS images: bit 0, the 64 even positions
// 128 q + 2 i, at img0 = lds + q * 64 * 80 B; bit 1, the 32 positions
// 128 q + 4 i + 1, at img1 = lds + 40 KiB + q * 32 * 80 B (global_load_lds,
// 16-B chunks lane-linear; the wave waits for its own DMA before reading).
// (OFF: the transform's skew offset; IMG1: byte offset of the bit-1 images =
// 5 KiB x waves; the decoder: OFF = 0, 8 waves)
template <int OFF = 0, int IMG1 = 40 * 1024>
__device__ __forceinline__ void q_pos_tables(uint32_t* lds, int q, int lane) {
  const uint8_t* src = (const uint8_t*)(const void*)g_ptab16x;
  asm volatile("" : "+v"(lane));  // the two calls' addresses are not kept live in between
  uint32_t* img0 = lds + q * 64 * kTab16x;
  uint32_t* img1 = lds + IMG1 / 4 + q * 32 * kTab16x;
#pragma unroll
  for (int i = 0; i < 5; i++) {  // 320 chunks
    const int c = 64 * i + lane;
    const uint8_t* g = src + (long)(OFF + 128 * q + 2 * (c / 5)) * (kTab16x * 4) + (c % 5) * 16;
    __builtin_amdgcn_global_load_lds((glb_vptr)g, (lds_vptr)(img0 + 64 * i * 4), 16, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 3; i++) {  // 160 chunks
    const int c = 64 * i + lane;
    if (i < 2 || lane < 32) {
      const uint8_t* g = src + (long)(OFF + 128 * q + 4 * (c / 5) + 1) * (kTab16x * 4) + (c % 5) * 16;
      __builtin_amdgcn_global_load_lds((glb_vptr)g, (lds_vptr)(img1 + 64 * i * 4), 16, 0, 0);
    }
  }
}

// K = 512 (8 waves, T e = ql + 4 (j & 3) + 16 q + 128 (j >> 2), bits 7-9) and
// K = 256 (4 waves, T as the encoder's: e = ql + 4 (j & 7) + 32 q + 128 (j >> 3),
// bits 7-8; four workgroups per CU, the half-lane k = 256 decoder: two)
template <int K>
__global__ __launch_bounds__(K) __attribute__((amdgpu_waves_per_eu(4, 4))) void leo16_decode_q_kernel(
    DecodeArgs a) {
  constexpr int NQ = K / 64, LR = K == 1024 ? 1 : K == 512 ? 2 : 3, RPR = K == 1024 ? 1 : K == 512 ? 2 : 4,
                IMG1 = NQ * 5 * 1024;
  // two rounds of the transposes / derivative (K = 512: 32 KiB each, 256: 16
  // KiB); the S-layer images (NQ x 7.5 KiB) in the same space before the first
  // transpose and after the last
  __shared__ __attribute__((aligned(16))) uint32_t lds[K * 32];
  const uint32_t* img0_base = lds;
  const uint32_t* img1_base = lds + IMG1 / 4;
  const long blk = blockIdx.x;
  const int piece = (int)(blk % a.nchunk);  // nchunk = 128-B pieces of the shard
  const long v = blk / a.nchunk;
  if (a.flags[v] == 0) return;  // uniform
  const long sq = v / a.nvec, vec = v % a.nvec;
  const int lane = threadIdx.x & 63;
  const int ql = lane >> 4;
  const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  q_pos_tables<0, IMG1>(lds, q, lane);
  const uint32_t col = (uint32_t)piece * 128u + (uint32_t)((lane >> 3) & 1) * 64u + (uint32_t)(lane & 7) * 4u;
  const uint32_t voff = col + (uint32_t)ql * 32u * (uint32_t)a.shard_stride;  // quarter ql: shard + 32 ql
  const auto rsrc = make_rsrc(a.data + sq * a.sq_stride + vec * a.vec_stride);
  const uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
  const auto trs = make_rsrc(a.err + err_vec(a, v) * rs_err_bytes(K) + rs_err_tab_off(K));
  // presence of the wave's 128 elements, li = e - 128 q = 32 ql + m(j) with
  // m(j) = q_elem_s(j, 0) < 32: the lane's 32 registers are bits 32 ql .. +31
  // (pw, per lane), and allq bit m = all four quarters of register m present
  const int e0 = 128 * q + lane, e1 = e0 + 64;
  const uint64_t pm0 = __builtin_amdgcn_ballot_w64(pres[(long)(e0 < K ? K + e0 : e0 - K) * a.p_shard_stride] != 0);
  const uint64_t pm1 = __builtin_amdgcn_ballot_w64(pres[(long)(e1 < K ? K + e1 : e1 - K) * a.p_shard_stride] != 0);
  const uint32_t pw0 = (uint32_t)pm0, pw1 = (uint32_t)(pm0 >> 32), pw2 = (uint32_t)pm1, pw3 = (uint32_t)(pm1 >> 32);
  const uint32_t pw = ql == 0 ? pw0 : ql == 1 ? pw1 : ql == 2 ? pw2 : pw3;
  uint32_t allq = pw0 & pw1 & pw2 & pw3;
  WQ w;
  const int q_ld = opaque_s(q);
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const int i = 128 * q_ld + q_elem_s(j, 0);  // quarter 0's element
    const int shard = i < K ? K + i : i - K;
    const uint32_t so = (uint32_t)shard * (uint32_t)a.shard_stride;
    const uint32_t vj = ((pw >> q_elem_s(j, 0)) & 1) ? voff : (voff | 0x80000000u);
    w.lo[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, vj, so, 0);
    w.hi[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, vj + 32u, so, 0);
  }
  // premultiply: every element by its table (present: exp(errLoc); a missing
  // element's bytes are zero, so its postmultiply table leaves them zero)
  const int q_pm = opaque_s(q);
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const uint32_t e = (uint32_t)(128 * q_pm + q_elem_s(j, ql));
    uint32_t t[kTab16x];
    {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int h = 0; h < kTab16x / 4; h++) {
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(trs, e * (kTab16x * 4) + 16u * h, 0, 0);
        t[4 * h] = x.x;
        t[4 * h + 1] = x.y;
        t[4 * h + 2] = x.z;
        t[4 * h + 3] = x.w;
      }
    }
    uint32_t xl = w.lo[j], xh = w.hi[j];
    mul16x_by(xl, xh, t);
    asm volatile("" : "+v"(xl), "+v"(xh));
    w.lo[j] = xl;
    w.hi[j] = xh;
  }
  // ---- IFFT (ifftDITDecoder, skew index iend - 1) ----
  wait_dma();
  layer_s_q<true, 0>(w, ql, img0_base + q * 64 * kTab16x);
  layer_s_q<true, 1>(w, ql, img1_base + q * 32 * kTab16x);
  swap_sb_q(w);
  layer_b_q<true, 2>(w, q);
  layer_b_q<true, 3>(w, q);
  layer_b_q<true, 4>(w, q);
  layer_b_q<true, 5>(w, q);
  layer_b_q<true, 6>(w, q);
  __syncthreads();  // every wave's reads of its S-layer images are done
  xpose_bt_db<LR, RPR, 0>(w, lds, q, lane);  // rounds A B A B
  layer_t_q<true, 7, LR>(w);
  layer_t_q<true, 8, LR>(w);
  if constexpr (K >= 512) layer_t_q<true, 9, LR>(w);
  if constexpr (K >= 1024) layer_t_q<true, 10, LR>(w);
  derivative_tq<NQ>(w, lds, q, lane);  // A B A B
  // ---- FFT (fftDIT, skew index iend - 1) ----
  if constexpr (K >= 1024) layer_t_q<false, 10, LR>(w);
  if constexpr (K >= 512) layer_t_q<false, 9, LR>(w);
  layer_t_q<false, 8, LR>(w);
  layer_t_q<false, 7, LR>(w);
  xpose_bt_db<LR, RPR, 0>(w, lds, q, lane);  // A B A B
  __syncthreads();  // every wave's reads of B are done: the images come back over it
  q_pos_tables<0, IMG1>(lds, q, lane);
  layer_b_q<false, 6>(w, q);
  layer_b_q<false, 5>(w, q);
  layer_b_q<false, 4>(w, q);
  layer_b_q<false, 3>(w, q);
  layer_b_q<false, 2>(w, q);
  swap_sb_q(w);
  wait_dma();
  layer_s_q<false, 1, K == 1024>(w, ql, img1_base + q * 32 * kTab16x);
  layer_s_q<false, 0, K == 1024>(w, ql, img0_base + q * 64 * kTab16x);
  // erased shards = work * (65535 - errLocs): the stored table of a missing
  // element; a register whose four elements are all given is skipped (uniform)
  const int q_e = opaque_s(q);
  asm volatile("" : "+s"(allq));
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const int l0 = q_elem_s(j, 0);
    if ((allq >> l0) & 1) continue;  // uniform
    const uint32_t e = (uint32_t)(128 * q_e + q_elem_s(j, ql));
    uint32_t t[kTab16x];
    {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int h = 0; h < kTab16x / 4; h++) {
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(trs, e * (kTab16x * 4) + 16u * h, 0, 0);
        t[4 * h] = x.x;
        t[4 * h + 1] = x.y;
        t[4 * h + 2] = x.z;
        t[4 * h + 3] = x.w;
      }
    }
    uint32_t xl = w.lo[j], xh = w.hi[j];
    mul16x_by(xl, xh, t);
    asm volatile("" : "+v"(xl), "+v"(xh));
    const int i = 128 * q_e + l0;
    const int shard = i < K ? K + i : i - K;
    const uint32_t so = (uint32_t)shard * (uint32_t)a.shard_stride;
    if (!((pw >> l0) & 1)) {
      __builtin_amdgcn_raw_buffer_store_b32(xl, rsrc, voff, so, 0);
      __builtin_amdgcn_raw_buffer_store_b32(xh, rsrc, voff + 32u, so, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// ---------------------------------------------------------------------------
// k = 512 encoder, round 6 (leo16_encode_q_kernel): the quarter-lane layouts of
// leo16_decode_q_kernel over m = 512 elements -- 4 waves (256 threads) x 32
// registers x 4 quarters, one 128-B piece of a vector per workgroup, 32 KiB of
// LDS -- so FOUR workgroups share a CU (the half-lane encoder: two).
//   S, B as the decoder's;  T  e = ql + 4 (j & 7) + 32 q + 128 (j >> 3)
// (B <-> T: xpose_bt_db with LR = 3, NQ = 4).  The last IFFT layer and the
// first FFT layer (bit 8, registers j, j + 16 in T) are merged as in the other
// encoders.  Host emulation: tests/test_quarterlane_emu.py.
// ---------------------------------------------------------------------------
// bits >= 7 in T: registers j, j + (1 << LR) << (b - 7); position OFF + 128 (jb >> LR) + d - 1
template <bool INV, int B, int OFF, int LR = 3>
__device__ __forceinline__ void layer_te_q(WQ& w) {
  constexpr int RD = (1 << LR) << (B - 7), D = 1 << B;
#pragma unroll
  for (int jb = 0; jb < 32; jb += 2 * RD) {
    const bool zero = OFF + 128 * (jb >> LR) == 0;
    const int pos = zero ? 0 : opaque_tok(OFF + 128 * (jb >> LR) + D - 1, w.lo[jb]);
#pragma unroll
    for (int j = jb; j < jb + RD; j++) {
      if (zero) {
        w.lo[j + RD] ^= w.lo[j];
        w.hi[j + RD] ^= w.hi[j];
      } else if constexpr (INV) {
        ifft2_16(w, j, j + RD, pos);
      } else {
        fft2_16(w, j, j + RD, pos);
      }
      pin_pair(w, j, j + RD);
    }
  }
}

// M = 1024 (k = 1024, round 6): 8 waves (512 threads), T as the k = 512
// decoder's (LR = 2: e = ql + 4 (j & 3) + 16 q + 128 (j >> 2)), layers on bits
// 7, 8 and the merged bit 9; 64 KiB of LDS, two workgroups per CU.  M = 2048:
// 16 waves, T as the k = 1024 decoder's (LR = 1), bits 7-9 and the merged 10,
// 128 KiB of LDS, one workgroup per CU.
template <int M, bool REV>
__global__ __launch_bounds__(M / 2) __attribute__((amdgpu_waves_per_eu(4, 4))) void leo16_encode_q_kernel(
    EncodeArgs a) {
  constexpr int IO = REV ? 0 : M, FO = REV ? M : 0;
  constexpr int NQ = M / 128, LR = M == 2048 ? 1 : M == 1024 ? 2 : 3, RPR = M == 2048 ? 1 : M == 1024 ? 2 : 4;
  // two transpose rounds (xpose_bt_db; M = 512: 16 KiB each, 1024: 32 KiB); the
  // S-layer images (NQ x 7.5 KiB: bit 0 at q x 5 KiB, bit 1 at IMG1 + q x 2.5
  // KiB) in the same space before the first transpose and after the last
  __shared__ __attribute__((aligned(16))) uint32_t lds[M == 2048 ? 32768 : M == 1024 ? 16384 : 8192];
  constexpr int IMG1 = NQ * 5 * 1024;
  const long blk = blockIdx.x;
  const int piece = (int)(blk % a.nchunk);  // nchunk = 128-B pieces of the shard
  const long sv = blk / a.nchunk;
  const long vec = sv % a.nvec;
  const long sq = sv / a.nvec;
  if (vec_skipped(a, sv)) return;  // uniform
  const int lane = threadIdx.x & 63;
  const int ql = lane >> 4;
  const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t col = (uint32_t)piece * 128u + (uint32_t)((lane >> 3) & 1) * 64u + (uint32_t)(lane & 7) * 4u;
  const bool active = col < (uint32_t)a.shard_bytes;
  q_pos_tables<IO, IMG1>(lds, q, lane);
  const uint32_t cl = active ? col : 0u;  // inactive lanes read valid memory, store nothing
  // M = 2048: the wave's first element in the buffer base (a column vector of a
  // k = 2048 EDS spans 4 GiB, past the 32-bit buffer offsets)
  constexpr int QW = M == 2048 ? 0 : 128;  // element offset of the wave left in the offsets
  const long wb = M == 2048 ? 128L * q : 0L;
  WQ w;
  {
    const auto in_rsrc = make_rsrc(a.in + sq * a.in_sq_stride + vec * a.in_vec_stride + wb * a.in_shard_stride);
    const uint32_t vin = cl + (uint32_t)ql * 32u * (uint32_t)a.in_shard_stride;  // quarter ql: shard + 32 ql
    const int q_ld = opaque_s(q);
#pragma unroll
    for (int j = 0; j < 32; j++) {
      const uint32_t so = (uint32_t)(QW * q_ld + q_elem_s(j, 0)) * (uint32_t)a.in_shard_stride;
      w.lo[j] = __builtin_amdgcn_raw_buffer_load_b32(in_rsrc, vin, so, 0);
      w.hi[j] = __builtin_amdgcn_raw_buffer_load_b32(in_rsrc, vin + 32u, so, 0);
    }
    if (a.copy && active) {  // Q0 placement
      const auto cp = make_rsrc(a.copy + sq * a.copy_sq_stride + vec * a.copy_vec_stride + wb * a.copy_shard_stride);
      const uint32_t vcp = col + (uint32_t)ql * 32u * (uint32_t)a.copy_shard_stride;
#pragma unroll
      for (int j = 0; j < 32; j++) {
        const uint32_t so = (uint32_t)(QW * q_ld + q_elem_s(j, 0)) * (uint32_t)a.copy_shard_stride;
        __builtin_amdgcn_raw_buffer_store_b32(w.lo[j], cp, vcp, so, 0);
        __builtin_amdgcn_raw_buffer_store_b32(w.hi[j], cp, vcp + 32u, so, 0);
      }
    }
  }
  // Repair fill: which out-half shards are given, read before the transform;
  // the lane's 32 registers are bits 32 ql .. +31 of the wave's 128 (gw)
  uint32_t gw = 0;
  if (a.out_present) {
    const uint64_t g0 = __builtin_amdgcn_ballot_w64(fill_given(a, sq, vec, 128 * q + lane));
    const uint64_t g1 = __builtin_amdgcn_ballot_w64(fill_given(a, sq, vec, 128 * q + 64 + lane));
    gw = ql == 0 ? (uint32_t)g0 : ql == 1 ? (uint32_t)(g0 >> 32) : ql == 2 ? (uint32_t)g1 : (uint32_t)(g1 >> 32);
  }
  // ---- IFFT (ifftDITEncoder, skew index IO - 1 + iend) ----
  wait_dma();
  layer_s_q<true, 0>(w, ql, lds + q * 64 * kTab16x);
  layer_s_q<true, 1>(w, ql, lds + IMG1 / 4 + q * 32 * kTab16x);
  swap_sb_q(w);
  layer_b_q<true, 2, IO>(w, q);
  layer_b_q<true, 3, IO>(w, q);
  layer_b_q<true, 4, IO>(w, q);
  layer_b_q<true, 5, IO>(w, q);
  layer_b_q<true, 6, IO>(w, q);
  __syncthreads();  // every wave's reads of its S-layer images are done
  xpose_bt_db<LR, RPR, 0>(w, lds, q, lane);  // rounds A B A B
  layer_te_q<true, 7, IO, LR>(w);
  if constexpr (M >= 1024) layer_te_q<true, 8, IO, LR>(w);
  if constexpr (M >= 2048) layer_te_q<true, 9, IO, LR>(w);
  // last IFFT layer (top bit, skew IO + M/2 - 1) merged with the first FFT
  // layer (top bit, skew FO + M/2 - 1): registers j, j + 16
#pragma unroll
  for (int j = 0; j < 16; j++) {
    ifft_fft2_16(w, j, j + 16, MERGED_TAB(M == 2048 ? 3 : M == 1024 ? 2 : 1));
    pin_pair(w, j, j + 16);
  }
  // ---- FFT (fftDIT, skew index FO + iend - 1) ----
  if constexpr (M >= 2048) layer_te_q<false, 9, FO, LR>(w);
  if constexpr (M >= 1024) layer_te_q<false, 8, FO, LR>(w);
  layer_te_q<false, 7, FO, LR>(w);
  xpose_bt_db<LR, RPR, 0>(w, lds, q, lane);  // A B A B
  __syncthreads();  // every wave's reads of B are done: the images come back over it
  q_pos_tables<FO, IMG1>(lds, q, lane);
  layer_b_q<false, 6, FO>(w, q);
  layer_b_q<false, 5, FO>(w, q);
  layer_b_q<false, 4, FO>(w, q);
  layer_b_q<false, 3, FO>(w, q);
  layer_b_q<false, 2, FO>(w, q);
  swap_sb_q(w);
  wait_dma();
  layer_s_q<false, 1>(w, ql, lds + IMG1 / 4 + q * 32 * kTab16x);
  layer_s_q<false, 0>(w, ql, lds + q * 64 * kTab16x);
  if (!active) return;
  // ---- store: compare (prerepairSanityCheck), Repair fill, or plain ----
  const auto out_rsrc = make_rsrc(a.out + sq * a.out_sq_stride + vec * a.out_vec_stride + wb * a.out_shard_stride);
  const uint32_t vout = col + (uint32_t)ql * 32u * (uint32_t)a.out_shard_stride;
  const int q_st = opaque_s(q);
  if (a.mismatch) {
    uint32_t diff = 0;
#pragma unroll
    for (int j = 0; j < 32; j++) {
      const uint32_t so = (uint32_t)(QW * q_st + q_elem_s(j, 0)) * (uint32_t)a.out_shard_stride;
      diff |= w.lo[j] ^ __builtin_amdgcn_raw_buffer_load_b32(out_rsrc, vout, so, 0);
      diff |= w.hi[j] ^ __builtin_amdgcn_raw_buffer_load_b32(out_rsrc, vout + 32u, so, 0);
    }
    if (diff) {
      atomicOr(&a.mismatch[sq], a.mismatch_bit);
      if (a.mismatch_vec) a.mismatch_vec[sq * a.nvec + vec] = 1;
    }
    return;
  }
  if (a.out_present) {  // store the missing shards of the out half, compare given ones
    uint32_t diff = 0;
#pragma unroll
    for (int j = 0; j < 32; j++) {
      const uint32_t so = (uint32_t)(QW * q_st + q_elem_s(j, 0)) * (uint32_t)a.out_shard_stride;
      if ((gw >> q_elem_s(j, 0)) & 1) {
        diff |= w.lo[j] ^ __builtin_amdgcn_raw_buffer_load_b32(out_rsrc, vout, so, 0);
        diff |= w.hi[j] ^ __builtin_amdgcn_raw_buffer_load_b32(out_rsrc, vout + 32u, so, 0);
      } else {
        __builtin_amdgcn_raw_buffer_store_b32(w.lo[j], out_rsrc, vout, so, 0);
        __builtin_amdgcn_raw_buffer_store_b32(w.hi[j], out_rsrc, vout + 32u, so, 0);
      }
    }
    if (diff) a.redo[sv] = 1;
    return;
  }
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const uint32_t so = (uint32_t)(QW * q_st + q_elem_s(j, 0)) * (uint32_t)a.out_shard_stride;
    __builtin_amdgcn_raw_buffer_store_b32(w.lo[j], out_rsrc, vout, so, 0);
    __builtin_amdgcn_raw_buffer_store_b32(w.hi[j], out_rsrc, vout + 32u, so, 0);
  }
}

// ---------------------------------------------------------------------------
// k = 512 encoder, round 5 (leo16_encode_h_kernel): the half-lane layouts of
// leo16_decode_h_kernel over m = 512 elements -- 8 waves (512 threads) x 32
// register pairs x 2 halves, 64 data VGPRs within the 128 of 4 waves per SIMD
// -- so TWO workgroups share a CU and one's loads and stores overlap the
// other's transform (leo16_encode_reg32_kernel's 16 waves filled a CU alone
// and left its load and store phases bare).  A workgroup covers 256 B of its
// vector's shards.  Layouts as the decoder's, with T for LR = 2:
//   T  e = hl | (j & 3) << 1 | q << 3 | (j >> 2) << 6.
// The last IFFT layer and the first FFT layer (both dist 256, registers j and
// j + 16 in T) are merged as in the other encoders.
// ---------------------------------------------------------------------------
// M = 256 (round 5 too): 4 waves (256 threads), T with three low register
// bits, the merged dist-128 layer; four workgroups per CU.
template <int M, bool REV>
__global__ __launch_bounds__(M) __attribute__((amdgpu_waves_per_eu(4, 4))) void leo16_encode_h_kernel(
    EncodeArgs a) {
  constexpr int IO = REV ? 0 : M, FO = REV ? M : 0;
  constexpr int LR = M == 512 ? 2 : 3, RPR = M == 512 ? 2 : 8;
  // M = 512: two 32-KiB transpose rounds (xpose_bt_db, round 6: 8 -> 4
  // barriers per transpose), 64 KiB, so two workgroups still share a CU;
  // M = 256 keeps one (32 KiB: four workgroups per CU)
  constexpr bool DB = M == 512;
  __shared__ __attribute__((aligned(16))) uint32_t lds[(DB ? 2 : 1) * 8 * 8 * 2 * 64];
  const long blk = blockIdx.x;
  const int piece = (int)(blk % a.nchunk);  // nchunk = 256-B pieces of the shard
  const long sv = blk / a.nchunk;
  const long vec = sv % a.nvec;
  const long sq = sv / a.nvec;
  if (vec_skipped(a, sv)) return;  // uniform
  const int lane = threadIdx.x & 63;
  const int hl = lane >> 5;
  const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t col = (uint32_t)piece * 256u + (uint32_t)((lane & 31) >> 3) * 64u + (uint32_t)(lane & 7) * 4u;
  const bool active = col < (uint32_t)a.shard_bytes;
  H_PROBE(g_probe_e, 0, M / 64 - 1);
  pos_tables_wave<IO>(lds, q, lane);  // this wave's IFFT bit-0 tables (round 6)
  const uint32_t cl = active ? col : 0u;  // inactive lanes read valid memory, store nothing
  W32 w;
  {
    const auto in_rsrc = make_rsrc(a.in + sq * a.in_sq_stride + vec * a.in_vec_stride);
    const uint32_t vin = cl + (uint32_t)hl * 32u * (uint32_t)a.in_shard_stride;  // upper half: shard + 32
    const int q_ld = opaque_s(q);
#pragma unroll
    for (int j = 0; j < 32; j++) {
      const uint32_t so = (uint32_t)(64 * q_ld + s_local(j, 0)) * (uint32_t)a.in_shard_stride;
      w.lo[j] = __builtin_amdgcn_raw_buffer_load_b32(in_rsrc, vin, so, 0);
      w.hi[j] = __builtin_amdgcn_raw_buffer_load_b32(in_rsrc, vin + 32u, so, 0);
    }
    if (a.copy && active) {  // Q0 placement
      const auto cp = make_rsrc(a.copy + sq * a.copy_sq_stride + vec * a.copy_vec_stride);
      const uint32_t vcp = col + (uint32_t)hl * 32u * (uint32_t)a.copy_shard_stride;
#pragma unroll
      for (int j = 0; j < 32; j++) {
        const uint32_t so = (uint32_t)(64 * q_ld + s_local(j, 0)) * (uint32_t)a.copy_shard_stride;
        __builtin_amdgcn_raw_buffer_store_b32(w.lo[j], cp, vcp, so, 0);
        __builtin_amdgcn_raw_buffer_store_b32(w.hi[j], cp, vcp + 32u, so, 0);
      }
    }
  }
  // Repair fill: which out-half shards are given (element 64 q + lane), read
  // before the transform so that the store loop does not wait on presence loads
  const uint64_t given = a.out_present ? __builtin_amdgcn_ballot_w64(fill_given(a, sq, vec, 64 * q + lane)) : 0ull;
  H_PROBE(g_probe_e, 1, M / 64 - 1);
  // ---- IFFT (ifftDITEncoder, skew index IO - 1 + iend) ----
  wait_dma();
  layer0_sl<true>(w, q, hl, lds);
  swap_sb(w);
  H_PROBE(g_probe_e, 2, M / 64 - 1);
  layer_b<true, 2, IO>(w, q);
  layer_b<true, 4, IO>(w, q);
  layer_b<true, 8, IO>(w, q);
  layer_b<true, 16, IO>(w, q);
  layer_b<true, 32, IO>(w, q);
  H_PROBE(g_probe_e, 3, M / 64 - 1);
  __syncthreads();  // every wave's reads of its bit-0 tables are done before the staging is rewritten
  if constexpr (DB) xpose_bt_db<LR, RPR, 0>(w, lds, q, lane);  // rounds A B A B
  else xpose_bt<LR, RPR>(w, lds, q, lane);
  H_PROBE(g_probe_e, 4, M / 64 - 1);
  layer_t<true, 64, LR, IO>(w);
  if constexpr (M == 512) layer_t<true, 128, LR, IO>(w);
  // last IFFT layer (dist M / 2, skew IO - 1 + M / 2) merged with the first FFT
  // layer (dist M / 2, skew FO + M / 2 - 1): registers j, j + 16
#pragma unroll
  for (int j = 0; j < 16; j++) {
    ifft_fft2_16(w, j, j + 16, MERGED_TAB(M == 512 ? 1 : 0));
    pin_pair(w, j, j + 16);
  }
  // ---- FFT (fftDIT, skew index FO + iend - 1) ----
  if constexpr (M == 512) layer_t<false, 128, LR, FO>(w);
  layer_t<false, 64, LR, FO>(w);
  H_PROBE(g_probe_e, 5, M / 64 - 1);
  if constexpr (DB) xpose_bt_db<LR, RPR, 0>(w, lds, q, lane);  // A B A B
  else xpose_bt<LR, RPR>(w, lds, q, lane);                      // (ends with a barrier)
  // the FFT bit-0 tables into A (DB: its last reads, round 2's, precede round
  // 3's barrier), landing while the B layers run
  pos_tables_wave<FO>(lds, q, lane);
  H_PROBE(g_probe_e, 6, M / 64 - 1);
  layer_b<false, 32, FO>(w, q);
  layer_b<false, 16, FO>(w, q);
  layer_b<false, 8, FO>(w, q);
  layer_b<false, 4, FO>(w, q);
  layer_b<false, 2, FO>(w, q);
  H_PROBE(g_probe_e, 7, M / 64 - 1);
  swap_sb(w);
  wait_dma();
  layer0_sl<false>(w, q, hl, lds);
  H_PROBE(g_probe_e, 8, M / 64 - 1);
  if (!active) return;
  // ---- store: compare (prerepairSanityCheck), Repair fill, or plain ----
  const auto out_rsrc = make_rsrc(a.out + sq * a.out_sq_stride + vec * a.out_vec_stride);
  const uint32_t vout = col + (uint32_t)hl * 32u * (uint32_t)a.out_shard_stride;
  const int q_st = opaque_s(q);
  if (a.mismatch) {
    uint32_t diff = 0;
#pragma unroll
    for (int j = 0; j < 32; j++) {
      const uint32_t so = (uint32_t)(64 * q_st + s_local(j, 0)) * (uint32_t)a.out_shard_stride;
      diff |= w.lo[j] ^ __builtin_amdgcn_raw_buffer_load_b32(out_rsrc, vout, so, 0);
      diff |= w.hi[j] ^ __builtin_amdgcn_raw_buffer_load_b32(out_rsrc, vout + 32u, so, 0);
    }
    if (diff) {
      atomicOr(&a.mismatch[sq], a.mismatch_bit);
      if (a.mismatch_vec) a.mismatch_vec[sq * a.nvec + vec] = 1;
    }
    return;
  }
  if (a.out_present) {  // store the missing shards of the out half, compare given ones
    uint64_t g = given;
    asm volatile("" : "+s"(g));
    const uint32_t gh = hl ? (uint32_t)(g >> 32) : (uint32_t)g;
    uint32_t diff = 0;
#pragma unroll
    for (int j = 0; j < 32; j++) {
      const int l0 = s_local(j, 0);
      const uint32_t so = (uint32_t)(64 * q_st + l0) * (uint32_t)a.out_shard_stride;
      if ((gh >> l0) & 1) {
        diff |= w.lo[j] ^ __builtin_amdgcn_raw_buffer_load_b32(out_rsrc, vout, so, 0);
        diff |= w.hi[j] ^ __builtin_amdgcn_raw_buffer_load_b32(out_rsrc, vout + 32u, so, 0);
      } else {
        __builtin_amdgcn_raw_buffer_store_b32(w.lo[j], out_rsrc, vout, so, 0);
        __builtin_amdgcn_raw_buffer_store_b32(w.hi[j], out_rsrc, vout + 32u, so, 0);
      }
    }
    if (diff) a.redo[sv] = 1;
    return;
  }
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const uint32_t so = (uint32_t)(64 * q_st + s_local(j, 0)) * (uint32_t)a.out_shard_stride;
    __builtin_amdgcn_raw_buffer_store_b32(w.lo[j], out_rsrc, vout, so, 0);
    __builtin_amdgcn_raw_buffer_store_b32(w.hi[j], out_rsrc, vout + 32u, so, 0);
  }
  H_PROBE(g_probe_e, 9, M / 64 - 1);
}

// Tables are module globals: upload once per device.
std::mutex g_tab_mu;
bool g_tab_done[64];

hipError_t ensure_tables() {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> g(g_tab_mu);
  if (g_tab_done[dev]) return hipSuccess;
  static const gf16::Tables t = gf16::make_tables();
  if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_log16), t.log.data(), 65536 * 2)) != hipSuccess) return e;
  if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_exp16), t.exp.data(), 65536 * 2)) != hipSuccess) return e;
  if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_skew16), t.skew.data(), 65536 * 2)) != hipSuccess) return e;
  {
    std::vector<uint16_t> wf(3 * 2048, 0);
    for (int f = 0; f < 3; f++) {
      const int n = 512 << f;
      for (int r = 0; r < n; r++) {
        uint64_t acc = 0;
        for (int q = 0; q < 65536 / n; q++) acc += t.walsh[(size_t)q * n + r];
        wf[(size_t)f * 2048 + r] = (uint16_t)(acc % kMod16);
      }
    }
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_wfold16), wf.data(), wf.size() * 2)) != hipSuccess) return e;
  }
  {
    // merged encoder tables: the element exp(skew[p]) ^ exp(skew[q]) (skew kMod16 = element 0)
    auto elem = [&](int pos) -> unsigned { return t.skew[pos] == kMod16 ? 0u : (unsigned)t.exp[t.skew[pos]]; };
    const int pairs[4][2] = {{383, 127}, {767, 255}, {1535, 511}, {3071, 1023}};  // m = 256 .. 2048
    // 3/3/2-split tables (mul16x_add_t): per skew position and for the two merged elements
    auto tab332 = [&](unsigned c, uint32_t* out) {  // c = field element (0: zero table)
      for (int i = 0; i < kTab16x; i++) out[i] = 0;
      if (!c) return;
      const unsigned lc = t.log[c];
      static const int shift[6] = {0, 3, 6, 8, 11, 14}, width[6] = {3, 3, 2, 3, 3, 2};
      static const int base[6] = {0, 4, 8, 10, 14, 18};
      for (int g = 0; g < 6; g++)
        for (int e2 = 1; e2 < (1 << width[g]); e2++) {
          const unsigned x = (unsigned)e2 << shift[g];
          unsigned sidx = (unsigned)t.log[x] + lc;
          sidx = (sidx + (sidx >> 16)) & 0xFFFFu;
          const unsigned prod = t.exp[sidx];
          const int lo_dw = width[g] == 3 ? base[g] + (e2 >> 2) : base[g];
          const int hi_dw = width[g] == 3 ? base[g] + 2 + (e2 >> 2) : base[g] + 1;
          out[lo_dw] |= (prod & 0xFFu) << (8 * (e2 & 3));
          out[hi_dw] |= ((prod >> 8) & 0xFFu) << (8 * (e2 & 3));
        }
    };
    std::vector<uint32_t> px((size_t)kTabPos * kTab16x, 0u);
    for (int pos = 0; pos < kTabPos; pos++)
      if (t.skew[pos] != kMod16) tab332((unsigned)t.exp[t.skew[pos]], px.data() + (size_t)pos * kTab16x);
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_ptab16x), px.data(), px.size() * 4)) != hipSuccess) return e;
    std::vector<uint32_t> mx(4 * kTab16x, 0u);
    for (int m = 0; m < 4; m++) tab332(elem(pairs[m][0]) ^ elem(pairs[m][1]), mx.data() + (size_t)m * kTab16x);
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_ptab16x_merged), mx.data(), mx.size() * 4)) != hipSuccess) return e;
    uint16_t lb[16];
    for (int b = 0; b < 16; b++) lb[b] = (uint16_t)t.log[1u << b];
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_logbit16), lb, sizeof lb)) != hipSuccess) return e;
  }
  // > 64 KiB of dynamic LDS: the generic decoder (k = 512: 128 KiB) and the half-lane ones
  if ((e = hipFuncSetAttribute((const void*)leo16_decode_kernel,  // k <= 512 here (wider: rs_gf16_wide.hip)
                               hipFuncAttributeMaxDynamicSharedMemorySize, 512 * 256)) != hipSuccess)
    return e;
  if ((e = hipFuncSetAttribute((const void*)leo16_decode_h_kernel<512>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)dec_h_lds_bytes<512>())) != hipSuccess)
    return e;
  if ((e = hipFuncSetAttribute((const void*)leo16_decode_h_kernel<256>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)dec_h_lds_bytes<256>())) != hipSuccess)
    return e;
  g_tab_done[dev] = true;
  return hipSuccess;
}

bool gf16_k_ok(int k) { return k >= 256 && k <= 512 && (k & (k - 1)) == 0; }

}  // namespace

// Wide squares (k > 512) and DAGPU_GF16_WIDE=1 (A/B of the wide kernels at
// k = 256 / 512): the LDS-slice kernels of rs_gf16_wide.hip.
static bool wide_forced() {
  const char* e = sw(SW_GF16_WIDE);
  return e && e[0] == '1';
}
static bool use_wide(int k) { return k > 512 || wide_forced(); }

// k = 256 / 512 encoders: the half-lane kernels, one workgroup per 256-B piece
// of a vector's shards (a last partial piece: inactive lanes store nothing)
hipError_t launch_leo16_encode(int k, const EncodeArgs& a, hipStream_t s) {
  if ((k == 1024 || k == 2048) && a.shard_bytes % 64 == 0 && !wide_forced()) {
    // k = 1024 / 2048: the quarter-lane encoder, 8 / 16 waves (two workgroups / one per CU), 128-B pieces
    if (a.reverse && !a.out_present) return hipErrorInvalidValue;
    hipError_t e = ensure_tables();
    if (e != hipSuccess) return e;
    EncodeArgs b = a;
    b.nchunk = (a.shard_bytes + 127) / 128;
    const long qb = b.nsq * b.nvec * b.nchunk;
    if (qb <= 0) return hipSuccess;
    if (k == 2048) {
      if (a.reverse) hipLaunchKernelGGL((leo16_encode_q_kernel<2048, true>), dim3((unsigned)qb), dim3(1024), 0, s, b);
      else hipLaunchKernelGGL((leo16_encode_q_kernel<2048, false>), dim3((unsigned)qb), dim3(1024), 0, s, b);
    } else if (a.reverse) {
      hipLaunchKernelGGL((leo16_encode_q_kernel<1024, true>), dim3((unsigned)qb), dim3(512), 0, s, b);
    } else {
      hipLaunchKernelGGL((leo16_encode_q_kernel<1024, false>), dim3((unsigned)qb), dim3(512), 0, s, b);
    }
    return hipGetLastError();
  }
  if (use_wide(k)) return launch_leo16w_encode(k, a, s);
  if (!gf16_k_ok(k) || a.shard_bytes % 64) return hipErrorInvalidValue;
  if (a.reverse && !a.out_present) return hipErrorInvalidValue;  // reverse transform: Repair fill only
  hipError_t e = ensure_tables();
  if (e != hipSuccess) return e;
  EncodeArgs b = a;
  b.nchunk = (a.shard_bytes + 255) / 256;
  const long hb = b.nsq * b.nvec * b.nchunk;
  if (hb <= 0) return hipSuccess;
  if (k == 512) {
#ifndef DAGPU_ENC512_HALF  // (A/B builds: the half-lane k = 512 encoder)
    b.nchunk = (a.shard_bytes + 127) / 128;  // quarter-lane encoder, 128-B pieces, four workgroups per CU
    const long qb = b.nsq * b.nvec * b.nchunk;
    if (a.reverse) hipLaunchKernelGGL((leo16_encode_q_kernel<512, true>), dim3((unsigned)qb), dim3(256), 0, s, b);
    else hipLaunchKernelGGL((leo16_encode_q_kernel<512, false>), dim3((unsigned)qb), dim3(256), 0, s, b);
#else
    if (a.reverse) hipLaunchKernelGGL((leo16_encode_h_kernel<512, true>), dim3((unsigned)hb), dim3(512), 0, s, b);
    else hipLaunchKernelGGL((leo16_encode_h_kernel<512, false>), dim3((unsigned)hb), dim3(512), 0, s, b);
#endif
  } else {
    if (a.reverse) hipLaunchKernelGGL((leo16_encode_h_kernel<256, true>), dim3((unsigned)hb), dim3(256), 0, s, b);
    else hipLaunchKernelGGL((leo16_encode_h_kernel<256, false>), dim3((unsigned)hb), dim3(256), 0, s, b);
  }
  return hipGetLastError();
}

hipError_t launch_leo16_errlocs(const DecodeArgs& a, hipStream_t s) {
  if (a.k > 1024) return launch_leo16w_errlocs(a, s);
  if (!gf16_k_ok(a.k) && a.k != 1024) return hipErrorInvalidValue;
  hipError_t e = ensure_tables();
  if (e != hipSuccess) return e;
  const long nv = a.nsq * a.nvec;
  if (nv <= 0) return hipSuccess;
  if (a.k == 256)
    hipLaunchKernelGGL(leo16_errlocs_fold_kernel<512>, dim3((unsigned)nv), dim3(kFoldThreads), 0, s, a);
  else if (a.k == 512)
    hipLaunchKernelGGL(leo16_errlocs_fold_kernel<1024>, dim3((unsigned)nv), dim3(kFoldThreads), 0, s, a);
  else  // k = 1024: the quarter-lane decoder's 80-B tables (the wide decoder reads the locators)
    hipLaunchKernelGGL(leo16_errlocs_fold_kernel<2048>, dim3((unsigned)nv), dim3(kFoldThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_leo16_decode_only(const DecodeArgs& a, hipStream_t s, bool mark_present) {
  if (a.k == 1024 && a.shard_bytes % 128 == 0 && !wide_forced()) {
    // k = 1024: the quarter-lane decoder, 16 waves (one workgroup per CU), 128-B pieces
    hipError_t e = ensure_tables();
    if (e != hipSuccess) return e;
    const long nv = a.nsq * a.nvec;
    if (nv <= 0) return hipSuccess;
    DecodeArgs b = a;
    b.nchunk = a.shard_bytes / 128;
    hipLaunchKernelGGL(leo16_decode_q_kernel<1024>, dim3((unsigned)(nv * b.nchunk)), dim3(1024), 0, s, b);
    if ((e = hipGetLastError()) != hipSuccess || !mark_present) return e;
    hipLaunchKernelGGL(mark_present16_kernel, dim3((unsigned)nv), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  if (use_wide(a.k)) return launch_leo16w_decode_only(a, s, mark_present);
  if (!gf16_k_ok(a.k) || a.shard_bytes % 64) return hipErrorInvalidValue;
  hipError_t e = ensure_tables();
  if (e != hipSuccess) return e;
  const long nv = a.nsq * a.nvec;
  if (nv <= 0) return hipSuccess;
  if (a.shard_bytes % 256 == 0) {  // half-lane decoders, 256-B pieces
    DecodeArgs b = a;
    b.nchunk = a.shard_bytes / 256;
    const long grid = nv * b.nchunk;
    if (a.k == 512) {
#ifndef DAGPU_DEC512_HALF  // (A/B builds: the half-lane k = 512 decoder)
      b.nchunk = a.shard_bytes / 128;  // quarter-lane decoder, 128-B pieces, two workgroups per CU
      hipLaunchKernelGGL(leo16_decode_q_kernel<512>, dim3((unsigned)(nv * b.nchunk)), dim3(512), 0, s, b);
#else
      hipLaunchKernelGGL((leo16_decode_h_kernel<512>), dim3((unsigned)grid), dim3(1024), dec_h_lds_bytes<512>(), s, b);
#endif
    } else {
#ifdef DAGPU_DEC256_QUARTER  // (A/B builds: the quarter-lane k = 256 decoder, four workgroups per CU:
      // 2,533-2,540 vs 2,551-2,562 squares/s for the half-lane one, profiles/gf16_q256_ab_r06.log)
      b.nchunk = a.shard_bytes / 128;
      hipLaunchKernelGGL(leo16_decode_q_kernel<256>, dim3((unsigned)(nv * b.nchunk)), dim3(256), 0, s, b);
#else
      hipLaunchKernelGGL((leo16_decode_h_kernel<256>), dim3((unsigned)grid), dim3(512), dec_h_lds_bytes<256>(), s, b);
#endif
    }
  } else {  // shard sizes off the 256-B grid (codec API): the generic LDS decoder
    const long blocks = nv * (a.shard_bytes / 64);
    hipLaunchKernelGGL(leo16_decode_kernel, dim3((unsigned)blocks), dim3(kThreads16),
                       (size_t)a.k * 2 * 64 * 2, s, a);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (mark_present) {
    hipLaunchKernelGGL(mark_present16_kernel, dim3((unsigned)nv), dim3(256), 0, s, a);
    e = hipGetLastError();
  }
  return e;
}

// Error-locator sharing.  err_key[v] = 32-bit hash of vector v's erasure
// pattern (its 2k presence flags, as 64-flag masks mixed with their index);
// err_head[v] = the first u <= v of v's square with the same key whose flags
// equal v's one by one (a key collision falls back to v itself), whose
// locators v then uses.  (Rounds 2-3 shared locators only along runs of equal
// neighbours: under the maximal erasure pattern the kept rows are scattered, so
// about half of them computed their own.)
//
// Two launches: the keys over a grid of (square, vector) blocks, so a few
// large squares (k = 512 Repair: 2 squares x 1024 vectors x 1024 flags per
// axis) still fill the chip, then one workgroup per square finds the heads.
// Flag layouts: p_shard_stride == 1 (row axis, codec API): one wave per
// vector, 64 flags per ballot; otherwise (column axis, where adjacent vectors
// are adjacent bytes) one lane per vector, its 64-flag groups split over the
// 16 waves of the block and XOR-ed in LDS.
__device__ __forceinline__ uint32_t key_mix(uint64_t m, int g) {
  uint64_t x = m + 0x9E3779B97F4A7C15ull * (uint64_t)(g + 1);
  x ^= x >> 31;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 29;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 32;
  return (uint32_t)x;
}

__device__ __forceinline__ void errloc_key_rows_block(const DecodeArgs& a, long bid) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long gv = bid * 16 + wave;  // wave-uniform
  if (gv >= a.nsq * a.nvec) return;
  const long sq = gv / a.nvec;
  const long v = gv - sq * a.nvec;
  const uint8_t* pv = a.present + sq * a.p_sq_stride + v * a.p_vec_stride;
  const int n = 2 * a.k;
  uint32_t key = 0;
  for (int g = 0; 64 * g < n; g++) {
    const int i = 64 * g + lane;
    const uint64_t m = __builtin_amdgcn_ballot_w64(i < n && pv[i] != 0);
    key ^= key_mix(m, g);
  }
  if (lane == 0) a.err_key[gv] = a.key_collide ? 0x5A5A5A5A : (int32_t)key;
}

__device__ __forceinline__ void errloc_key_cols_block(const DecodeArgs& a, long bid, uint32_t* acc) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long nb = (a.nvec + 63) / 64;
  const long sq = bid / nb;
  const long v = (bid - sq * nb) * 64 + lane;
  const int n = 2 * a.k;
  if (threadIdx.x < 64) acc[threadIdx.x] = 0;
  __syncthreads();
  if (v < a.nvec) {
    const uint8_t* pv = a.present + sq * a.p_sq_stride + v * a.p_vec_stride;
    uint32_t key = 0;
    for (int g = wave; 64 * g < n; g += 16) {
      uint64_t m = 0;
      for (int j = 0; j < 64 && 64 * g + j < n; j++)
        m |= (uint64_t)(pv[(long)(64 * g + j) * a.p_shard_stride] != 0) << j;
      key ^= key_mix(m, g);
    }
    if (key) atomicXor(&acc[lane], key);
  }
  __syncthreads();
  if (wave == 0 && v < a.nvec) a.err_key[sq * a.nvec + v] = a.key_collide ? 0x5A5A5A5A : (int32_t)acc[lane];
}

static long errloc_key_blocks(const DecodeArgs& a) {
  return a.p_shard_stride == 1 ? (a.nsq * a.nvec + 15) / 16 : a.nsq * ((a.nvec + 63) / 64);
}

// keys of a0 (blocks < nb0), then of a1 (one launch for both axes of a Repair round)
__global__ __launch_bounds__(1024) void errloc_key_kernel(DecodeArgs a0, DecodeArgs a1, long nb0) {
  __shared__ uint32_t acc[64];
  const bool second = (long)blockIdx.x >= nb0;
  const DecodeArgs& a = second ? a1 : a0;
  const long bid = second ? (long)blockIdx.x - nb0 : (long)blockIdx.x;
  if (a.p_shard_stride == 1) errloc_key_rows_block(a, bid);
  else errloc_key_cols_block(a, bid, acc);
}

// One workgroup per square (nvec <= kMaxHeadVec): keys in LDS, candidate head =
// the first vector with an equal key; squares of a0 (blocks < a0.nsq), then of a1.
constexpr int kMaxHeadVec = 2 * kMaxK;
__global__ __launch_bounds__(1024) void errloc_heads_kernel(DecodeArgs a0, DecodeArgs a1) {
  extern __shared__ int32_t key[];  // nvec
  const bool second = (long)blockIdx.x >= a0.nsq;
  const DecodeArgs& a = second ? a1 : a0;
  const long sq = second ? (long)blockIdx.x - a0.nsq : (long)blockIdx.x;
  const int nvec = (int)a.nvec;
  const long v0 = sq * a.nvec;
  for (int t = threadIdx.x; t < nvec; t += 1024) key[t] = a.err_key[v0 + t];
  __syncthreads();
  for (int t = threadIdx.x; t < nvec; t += 1024) {
    const int32_t kt = key[t];
    int u = 0;
    while (key[u] != kt) u++;  // ends at t at the latest
    a.err_head[v0 + t] = (int32_t)(v0 + u);
  }
}

// Candidate heads of a (and of a1 when given, e.g. both axes of a Repair round
// ahead of the axis choice); the flag-by-flag check of each candidate is the
// locator kernels' err_head_checked_*.
hipError_t launch_errloc_heads2(const DecodeArgs& a, const DecodeArgs* a1, hipStream_t s) {
  if (!a.err_key || !a.err_head) return hipSuccess;
  if (a1 && (!a1->err_key || !a1->err_head || a1->nsq <= 0 || a1->nvec <= 0)) return hipErrorInvalidValue;
  const long nv = a.nsq * a.nvec;
  if (nv <= 0) return hipSuccess;
  if (a.nvec > kMaxHeadVec || (a1 && a1->nvec > kMaxHeadVec)) return hipErrorInvalidValue;
  const DecodeArgs& b = a1 ? *a1 : a;
  const long nb0 = errloc_key_blocks(a), nb1 = a1 ? errloc_key_blocks(b) : 0;
  hipLaunchKernelGGL(errloc_key_kernel, dim3((unsigned)(nb0 + nb1)), dim3(1024), 0, s, a, b, nb0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const long nvec = a1 && b.nvec > a.nvec ? b.nvec : a.nvec;
  hipLaunchKernelGGL(errloc_heads_kernel, dim3((unsigned)(a.nsq + (a1 ? b.nsq : 0))), dim3(1024),
                     (size_t)nvec * 4, s, a, b);
  return hipGetLastError();
}

hipError_t launch_errloc_heads(const DecodeArgs& a, hipStream_t s) { return launch_errloc_heads2(a, nullptr, s); }

hipError_t launch_rs_prepare(int k) {
  if (k <= 128) return hipSuccess;  // GF(2^8): constexpr tables
  hipError_t e = ensure_tables();
  if (e == hipSuccess) e = leo16w_prepare();
  return e;
}

// Field dispatch used by the host runtime: GF(2^8) for 2k <= 256, else GF(2^16).
hipError_t launch_rs_encode(int k, const EncodeArgs& a, hipStream_t s) {
  return k <= 128 ? launch_leo8_encode(k, a, s) : launch_leo16_encode(k, a, s);
}
hipError_t launch_rs_errlocs_only(const DecodeArgs& a, hipStream_t s) {
  return a.k <= 128 ? launch_leo8_errlocs(a, s) : launch_leo16_errlocs(a, s);
}
hipError_t launch_rs_errlocs(const DecodeArgs& a, hipStream_t s) {
  hipError_t e = launch_errloc_heads(a, s);
  if (e != hipSuccess) return e;
  return launch_rs_errlocs_only(a, s);
}
hipError_t launch_rs_decode_only(const DecodeArgs& a, hipStream_t s, bool mark_present) {
  return a.k <= 128 ? launch_leo8_decode_only(a, s, mark_present)
                    : launch_leo16_decode_only(a, s, mark_present);
}
hipError_t launch_rs_decode(const DecodeArgs& a, hipStream_t s, bool mark_present) {
  hipError_t e = launch_rs_errlocs(a, s);
  if (e != hipSuccess) return e;
  return launch_rs_decode_only(a, s, mark_present);
}

}  // namespace dagpu

#ifdef DAGPU_PHASE_PROBE
// probe builds only: op 0 clears the stamps, op 1 copies n of them to out
// op 0: zero both buffers; 1: read the decoders' stamps; 2: the half-lane encoders'
extern "C" int dagpu_debug_probe(int op, uint64_t* out, size_t n) {
  if (op == 0) {
    static uint64_t zero[8192 * 2 * dagpu::kProbePhases];
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(dagpu::g_probe), zero, sizeof zero);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(dagpu::g_probe_e), zero, sizeof zero);
    return (int)e;
  }
  if (n > 8192 * 2 * (size_t)dagpu::kProbePhases) n = 8192 * 2 * (size_t)dagpu::kProbePhases;
  if (op == 2) return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(dagpu::g_probe_e), n * sizeof(uint64_t));
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(dagpu::g_probe), n * sizeof(uint64_t));
}
#endif
