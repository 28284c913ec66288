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
// Layout.  One 256-thread workgroup transforms one 64-byte column block of one
// vector: the m (encode) or n = 2k (decode) elements of 32 symbols live in LDS
// as uint16 rows of 64 B.  Every radix-2 butterfly step is a pass over
// (pair, symbol) items with a barrier between steps; the 32 lanes of a pair
// share one skew constant.  The multiply is log/exp through 128 KiB tables in
// global memory (L2-resident), so this path is latency/L2 bound, not VALU
// bound -- adequate for the stress sizes, where SHA-256 over the 2-4x larger
// square dominates anyway.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "gf16_host.hpp"
#include "kernels.hpp"

namespace dagpu {

namespace {

constexpr int kThreads16 = 256;
constexpr uint32_t kMod16 = 65535u;

__device__ uint16_t g_log16[65536];
__device__ uint16_t g_exp16[65536];
__device__ uint16_t g_skew16[65536];
__device__ uint16_t g_walsh16[65536];

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

// fftDIT over m elements (mtrunc = m), skew index iend - 1.
__device__ void fft16(uint16_t* w, int m) {
  int dist4 = m, dist = m >> 2;
  while (dist != 0) {
    const int d = dist, d4 = dist4;
    step16<false>(w, m / 2, [&](int p, int& i, int& j, uint32_t& lm) {
      const int r = (p / (2 * d)) * d4, q = p % (2 * d), iend = r + d;
      i = r + q;
      j = i + 2 * d;
      lm = g_skew16[iend + d - 1];
    });
    step16<false>(w, m / 2, [&](int p, int& i, int& j, uint32_t& lm) {
      const int r = (p / (2 * d)) * d4, q = p % (2 * d), iend = r + d;
      if (q < d) { i = r + q; lm = g_skew16[iend - 1]; }
      else { i = r + d + q; lm = g_skew16[iend + 2 * d - 1]; }
      j = i + d;
    });
    dist4 = dist;
    dist >>= 2;
  }
  if (dist4 == 2) {
    step16<false>(w, m / 2, [&](int p, int& i, int& j, uint32_t& lm) {
      i = 2 * p;
      j = i + 1;
      lm = g_skew16[i];
    });
  }
}

// ---------------------------------------------------------------------------
// Encode: parity = FFT_m(IFFT_m(data)), m = k.  Same EncodeArgs addressing as
// the GF(2^8) encoder, including Q0 placement and compare mode.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads16) void leo16_encode_kernel(EncodeArgs a, int k) {
  extern __shared__ __attribute__((aligned(16))) uint16_t w16[];  // k rows of 32 symbols
  const long nblk = a.shard_bytes / 64;
  const long blk = blockIdx.x % nblk;
  const long v = blockIdx.x / nblk;
  const long sq = v / a.nvec, vec = v % a.nvec;
  if (a.vec_flags && a.vec_flags[v] == 0) return;  // uniform
  const uint8_t* in = a.in + sq * a.in_sq_stride + vec * a.in_vec_stride + blk * 64;
  for (int t = threadIdx.x; t < k * 8; t += kThreads16) {
    const int e = t >> 3, q = t & 7;
    const uint32_t* src = (const uint32_t*)(in + (long)e * a.in_shard_stride);
    const uint32_t lo = src[q], hi = src[q + 8];
    block_to_lds(w16 + e * 32, lo, hi, q);
    if (a.copy) {
      uint32_t* dst = (uint32_t*)(a.copy + sq * a.copy_sq_stride + vec * a.copy_vec_stride +
                                  (long)e * a.copy_shard_stride + blk * 64);
      dst[q] = lo;
      dst[q + 8] = hi;
    }
  }
  __syncthreads();
  ifft16(w16, k, k - 1);
  fft16(w16, k);
  uint8_t* out = a.out + sq * a.out_sq_stride + vec * a.out_vec_stride + blk * 64;
  bool diff = false;
  for (int t = threadIdx.x; t < k * 8; t += kThreads16) {
    const int e = t >> 3, q = t & 7;
    uint32_t lo, hi;
    lds_to_block(w16 + e * 32, lo, hi, q);
    uint32_t* dst = (uint32_t*)(out + (long)e * a.out_shard_stride);
    if (a.mismatch) {
      diff |= (dst[q] != lo) || (dst[q + 8] != hi);
    } else {
      dst[q] = lo;
      dst[q + 8] = hi;
    }
  }
  if (a.mismatch && __builtin_amdgcn_ballot_w64(diff) != 0 && (threadIdx.x & 63) == 0)
    atomicOr(a.mismatch + sq, a.mismatch_bit);
}

// ---------------------------------------------------------------------------
// Error locators: one 1024-thread workgroup per vector, FWHT over the whole
// 65536-entry field in LDS (128 KiB of uint16).  The reference's first FWHT
// truncates at mtrunc = 2k; entries past 2k are zero, so the full transform is
// the same function.  Values are only congruent mod 65535 to the reference's
// (partial reduction), which is all their use as log multipliers needs.
// ---------------------------------------------------------------------------
constexpr int kErrThreads = 1024;
constexpr int kErrLds = 65536 * 2 + 16;

__device__ void fwht65536(uint16_t* e) {
  for (int dist = 1; dist < 65536; dist <<= 2) {
    const int dist4 = dist << 2;
    for (int g = threadIdx.x; g < 16384; g += kErrThreads) {
      const int r = (g / dist) * dist4;
      const int i = r + (g % dist);
      const uint32_t t0 = e[i], t1 = e[i + dist], t2 = e[i + 2 * dist], t3 = e[i + 3 * dist];
      const uint32_t a0 = add_mod16(t0, t1), a1 = sub_mod16(t0, t1);
      const uint32_t a2 = add_mod16(t2, t3), a3 = sub_mod16(t2, t3);
      e[i] = (uint16_t)add_mod16(a0, a2);
      e[i + 2 * dist] = (uint16_t)sub_mod16(a0, a2);
      e[i + dist] = (uint16_t)add_mod16(a1, a3);
      e[i + 3 * dist] = (uint16_t)sub_mod16(a1, a3);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kErrThreads) void leo16_errlocs_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t e16[];  // 65536 entries + counter
  int& cnt_s = *(int*)(e16 + 65536);
  const long v = blockIdx.x;
  const long sq = v / a.nvec, vec = v % a.nvec;
  const int k = a.k, n = 2 * k;
  const uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
  if (threadIdx.x == 0) cnt_s = 0;
  __syncthreads();
  int cnt = 0;
  for (int i = threadIdx.x; i < 65536; i += kErrThreads) {
    uint32_t x = 0;
    if (i < k) x = pres[(long)(k + i) * a.p_shard_stride] ? 0u : 1u;       // parity k+i -> work i
    else if (i < n) x = pres[(long)(i - k) * a.p_shard_stride] ? 0u : 1u;  // data i-k -> work i
    e16[i] = (uint16_t)x;
    if (i < n) cnt += (x == 0);
  }
  atomicAdd(&cnt_s, cnt);
  __syncthreads();
  const int present = cnt_s;
  const bool decode = present >= k && present < n;
  if (threadIdx.x == 0) {
    a.flags[v] = decode ? 1 : 0;
    if (present < k && a.too_few) atomicOr(a.too_few, 1);
    if (decode && a.ndecodable) atomicAdd(a.ndecodable, 1);
  }
  if (!decode) return;  // uniform
  fwht65536(e16);
  for (int i = threadIdx.x; i < 65536; i += kErrThreads)
    e16[i] = (uint16_t)(((uint32_t)e16[i] * (uint32_t)g_walsh16[i]) % kMod16);
  __syncthreads();
  fwht65536(e16);
  uint16_t* out = (uint16_t*)(a.err + v * (long)rs_err_bytes(k));
  for (int i = threadIdx.x; i < n; i += kErrThreads) out[i] = e16[i];
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
  const uint16_t* err = (const uint16_t*)(a.err + v * (long)rs_err_bytes(k));
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
  fft16(der, n);
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
  if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_walsh16), t.walsh.data(), 65536 * 2)) != hipSuccess) return e;
  // > 64 KiB of dynamic LDS (errlocs 128 KiB, k = 512 decode 128 KiB)
  if ((e = hipFuncSetAttribute((const void*)leo16_errlocs_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize, kErrLds)) != hipSuccess)
    return e;
  if ((e = hipFuncSetAttribute((const void*)leo16_decode_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize, kMaxK * 256)) != hipSuccess)
    return e;
  g_tab_done[dev] = true;
  return hipSuccess;
}

bool gf16_k_ok(int k) { return k >= 256 && k <= kMaxK && (k & (k - 1)) == 0; }

}  // namespace

hipError_t launch_leo16_encode(int k, const EncodeArgs& a, hipStream_t s) {
  if (!gf16_k_ok(k) || a.shard_bytes % 64) return hipErrorInvalidValue;
  hipError_t e = ensure_tables();
  if (e != hipSuccess) return e;
  const long blocks = a.nsq * a.nvec * (a.shard_bytes / 64);
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(leo16_encode_kernel, dim3((unsigned)blocks), dim3(kThreads16),
                     (size_t)k * 64, s, a, k);
  return hipGetLastError();
}

hipError_t launch_leo16_errlocs(const DecodeArgs& a, hipStream_t s) {
  if (!gf16_k_ok(a.k)) return hipErrorInvalidValue;
  hipError_t e = ensure_tables();
  if (e != hipSuccess) return e;
  const long nv = a.nsq * a.nvec;
  if (nv <= 0) return hipSuccess;
  hipLaunchKernelGGL(leo16_errlocs_kernel, dim3((unsigned)nv), dim3(kErrThreads), kErrLds, s, a);
  return hipGetLastError();
}

hipError_t launch_leo16_decode_only(const DecodeArgs& a, hipStream_t s, bool mark_present) {
  if (!gf16_k_ok(a.k) || a.shard_bytes % 64) return hipErrorInvalidValue;
  hipError_t e = ensure_tables();
  if (e != hipSuccess) return e;
  const long nv = a.nsq * a.nvec;
  if (nv <= 0) return hipSuccess;
  const long blocks = nv * (a.shard_bytes / 64);
  hipLaunchKernelGGL(leo16_decode_kernel, dim3((unsigned)blocks), dim3(kThreads16),
                     (size_t)a.k * 2 * 64 * 2, s, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (mark_present) {
    hipLaunchKernelGGL(mark_present16_kernel, dim3((unsigned)nv), dim3(256), 0, s, a);
    e = hipGetLastError();
  }
  return e;
}

// Field dispatch used by the host runtime: GF(2^8) for 2k <= 256, else GF(2^16).
hipError_t launch_rs_encode(int k, const EncodeArgs& a, hipStream_t s) {
  return k <= 128 ? launch_leo8_encode(k, a, s) : launch_leo16_encode(k, a, s);
}
hipError_t launch_rs_errlocs(const DecodeArgs& a, hipStream_t s) {
  return a.k <= 128 ? launch_leo8_errlocs(a, s) : launch_leo16_errlocs(a, s);
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
