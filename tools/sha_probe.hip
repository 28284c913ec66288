// sha_probe.hip -- three SHA-256 compression formulations on gfx950 and the
// issue rates they rest on.
//   rot 0: v_alignbit rotates + v_add3 (the production sha256.hpp: slow-class
//          VALU ops, ~1 wave-instruction/clk/CU)
//   rot 1: fast-class ops only (v_lshrrev/v_lshlrev + v_bitop3 + 2-input
//          v_add_u32), forced with inline asm so the compiler cannot re-fuse
//          shifts into v_alignbit or adds into v_add3
//   rot 2: rotates as the low half of a 64-bit shift of the pair {x, x}
//          (v_lshrrev_b64), 2-input adds
// plus single-opcode rates (16 chains per lane, 8 waves/SIMD) for the ops these
// need, and a cross-wave mix: half the waves of every workgroup issue only a
// slow op, the other half only a fast one.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/sha_probe.hip -o tools/sha_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include <stdlib.h>

static __constant__ const uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

template <int N>
__device__ __forceinline__ uint32_t shr(uint32_t x) {
  uint32_t r;
  asm("v_lshrrev_b32 %0, %1, %2" : "=v"(r) : "i"(N), "v"(x));
  return r;
}
template <int N>
__device__ __forceinline__ uint32_t shl(uint32_t x) {
  uint32_t r;
  asm("v_lshlrev_b32 %0, %1, %2" : "=v"(r) : "i"(N), "v"(x));
  return r;
}
__device__ __forceinline__ uint32_t add2(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t xr(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <int N>
__device__ __forceinline__ uint32_t rot64(uint64_t p) {
  uint64_t r;
  asm("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "i"(N), "v"(p));
  return (uint32_t)r;
}
__device__ __forceinline__ uint64_t pair(uint32_t x) {
  return ((uint64_t)x << 32) | x;  // one v_mov of x into the high half
}

// slow-class (VOP3-only) forms: a ^ b = v_xad_u32(a, b, 0); (a ^ b) + c = v_xad_u32(a, b, c);
// x >> n = v_alignbit_b32(0, x, n); a + b = v_add3_u32(a, b, 0); Ch = v_bfi_b32(e, f, g)
__device__ __forceinline__ uint32_t xad(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint32_t xad0(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_xad_u32 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t add3s(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint32_t add2s(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_add3_u32 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t x, uint32_t y) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(x), "v"(y));
  return r;
}
template <int N>
__device__ __forceinline__ uint32_t rots(uint32_t x) {
  uint32_t r;
  asm("v_alignbit_b32 %0, %1, %1, %2" : "=v"(r) : "v"(x), "i"(N));
  return r;
}
template <int N>
__device__ __forceinline__ uint32_t shrs(uint32_t x) {
  uint32_t r;
  asm("v_alignbit_b32 %0, 0, %1, %2" : "=v"(r) : "v"(x), "i"(N));
  return r;
}

// Sigma functions in the three forms.
template <int ROT, int A, int B, int C>
__device__ __forceinline__ uint32_t big_sigma(uint32_t x) {
  if constexpr (ROT == 0) {
    return x3(__builtin_amdgcn_alignbit(x, x, A), __builtin_amdgcn_alignbit(x, x, B),
              __builtin_amdgcn_alignbit(x, x, C));
  } else if constexpr (ROT == 1) {
    // (x >> A ^ x >> B ^ x >> C) = (x ^ x >> (B-A) ^ x >> (C-A)) >> A, same on the left
    const uint32_t r = shr<A>(x3(x, shr<B - A>(x), shr<C - A>(x)));
    const uint32_t l = shl<32 - C>(x3(x, shl<C - B>(x), shl<C - A>(x)));
    return xr(r, l);
  } else {
    const uint64_t p = pair(x);
    return x3(rot64<A>(p), rot64<B>(p), rot64<C>(p));
  }
}
template <int ROT, int A, int B, int S>
__device__ __forceinline__ uint32_t small_sigma(uint32_t x) {
  if constexpr (ROT == 0) {
    return x3(__builtin_amdgcn_alignbit(x, x, A), __builtin_amdgcn_alignbit(x, x, B), x >> S);
  } else if constexpr (ROT == 1) {
    // x>>A ^ x>>B ^ x>>S = (x ^ x>>(B-A)) >> A ^ x >> S ; left: (x << (32-B)) ^ (x << (32-A))
    const uint32_t r = x3(shr<A>(xr(x, shr<B - A>(x))), shr<S>(x), shl<32 - A>(x));
    return xr(r, shl<32 - B>(x));
  } else {
    const uint64_t p = pair(x);
    return x3(rot64<A>(p), rot64<B>(p), shr<S>(x));
  }
}
template <int ROT>
__device__ __forceinline__ uint32_t add3x(uint32_t a, uint32_t b, uint32_t c) {
  if constexpr (ROT == 0) return a + b + c;  // v_add3
  return add2(add2(a, b), c);
}

// rot 3: slow-class ops only -- 16 per round
__device__ __forceinline__ void round_slow(uint32_t a, uint32_t b, uint32_t c, uint32_t& d, uint32_t e,
                                           uint32_t f, uint32_t g, uint32_t& h, uint32_t kw) {
  const uint32_t u = xad(xad0(rots<6>(e), rots<11>(e)), rots<25>(e), h);  // h + Sigma1(e)
  const uint32_t t1 = add3s(u, bfi(e, f, g), kw);
  const uint32_t maj = bfi(xad0(a, b), c, a);
  const uint32_t t2 = xad(xad0(rots<2>(a), rots<13>(a)), rots<22>(a), maj);  // Sigma0(a) + Maj
  d = add2s(d, t1);
  h = add2s(t1, t2);
}
__device__ __forceinline__ void compress_slow(uint32_t (&st)[8], uint32_t (&w)[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll 1
  for (int it = 0; it < 64; it += 16) {
    if (it) {
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
        const uint32_t s0w = xad(xad0(rots<7>(w15), rots<18>(w15)), shrs<3>(w15), w[j]);
        const uint32_t s1w = xad(xad0(rots<17>(w2), rots<19>(w2)), shrs<10>(w2), w[(j + 9) & 15]);
        w[j] = add2s(s0w, s1w);
      }
    }
#pragma unroll
    for (int j = 0; j < 16; j += 8) {
      round_slow(a, b, c, d, e, f, g, h, add2s(kK[it + j + 0], w[j + 0]));
      round_slow(h, a, b, c, d, e, f, g, add2s(kK[it + j + 1], w[j + 1]));
      round_slow(g, h, a, b, c, d, e, f, add2s(kK[it + j + 2], w[j + 2]));
      round_slow(f, g, h, a, b, c, d, e, add2s(kK[it + j + 3], w[j + 3]));
      round_slow(e, f, g, h, a, b, c, d, add2s(kK[it + j + 4], w[j + 4]));
      round_slow(d, e, f, g, h, a, b, c, add2s(kK[it + j + 5], w[j + 5]));
      round_slow(c, d, e, f, g, h, a, b, add2s(kK[it + j + 6], w[j + 6]));
      round_slow(b, c, d, e, f, g, h, a, add2s(kK[it + j + 7], w[j + 7]));
    }
  }
  st[0] = add2s(st[0], a); st[1] = add2s(st[1], b); st[2] = add2s(st[2], c); st[3] = add2s(st[3], d);
  st[4] = add2s(st[4], e); st[5] = add2s(st[5], f); st[6] = add2s(st[6], g); st[7] = add2s(st[7], h);
}

template <int ROT>
__device__ __forceinline__ void round_(uint32_t a, uint32_t b, uint32_t c, uint32_t& d, uint32_t e,
                                       uint32_t f, uint32_t g, uint32_t& h, uint32_t kw) {
  const uint32_t t1 = add3x<ROT>(add2(h, kw), big_sigma<ROT, 6, 11, 25>(e),
                                 __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA));
  const uint32_t t2 = add3x<ROT>(big_sigma<ROT, 2, 13, 22>(a), __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8), 0);
  d = add2(d, t1);
  h = add2(t1, t2);
}

template <int ROT>
__device__ __forceinline__ void compress(uint32_t (&st)[8], uint32_t (&w)[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll 1
  for (int it = 0; it < 64; it += 16) {
    if (it) {
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const uint32_t s0 = small_sigma<ROT, 7, 18, 3>(w[(j + 1) & 15]);
        const uint32_t s1 = small_sigma<ROT, 17, 19, 10>(w[(j + 14) & 15]);
        w[j] = add2(add3x<ROT>(w[j], s0, w[(j + 9) & 15]), s1);
      }
    }
#pragma unroll
    for (int j = 0; j < 16; j += 8) {
      round_<ROT>(a, b, c, d, e, f, g, h, add2(kK[it + j + 0], w[j + 0]));
      round_<ROT>(h, a, b, c, d, e, f, g, add2(kK[it + j + 1], w[j + 1]));
      round_<ROT>(g, h, a, b, c, d, e, f, add2(kK[it + j + 2], w[j + 2]));
      round_<ROT>(f, g, h, a, b, c, d, e, add2(kK[it + j + 3], w[j + 3]));
      round_<ROT>(e, f, g, h, a, b, c, d, add2(kK[it + j + 4], w[j + 4]));
      round_<ROT>(d, e, f, g, h, a, b, c, add2(kK[it + j + 5], w[j + 5]));
      round_<ROT>(c, d, e, f, g, h, a, b, add2(kK[it + j + 6], w[j + 6]));
      round_<ROT>(b, c, d, e, f, g, h, a, add2(kK[it + j + 7], w[j + 7]));
    }
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

template <int ROT>
__global__ __launch_bounds__(256) void sha_kernel(uint32_t* out, int iters, uint32_t seed) {
  uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; i++) m[i] = seed + threadIdx.x * 16 + i + blockIdx.x;
  for (int it = 0; it < iters; it++) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = ROT == 3 ? xad0(m[i], st[i & 7]) : m[i] ^ st[i & 7];
    if constexpr (ROT == 3) compress_slow(st, w);
    else compress<ROT>(st, w);
  }
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; i++) out[t * 8 + i] = st[i];
}


// ---- split compression: round waves + schedule helper waves ----
// 512-thread workgroup: waves 0-3 run the 64 rounds (slow-class ops only),
// wave 4+r computes round wave r's message schedule W[16..63] + K with
// fast-class ops only (HELPER_FAST) and hands it over through LDS, 16 words
// at a time (two slots).  Four workgroup barriers per block.
template <bool HELPER_FAST>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(8, 8))) void sha_split_kernel(uint32_t* out, int iters, uint32_t seed) {
  __shared__ uint4 raw[4][4][64];      // [pair][quad][lane] W[0..15] of the current block
  __shared__ uint4 slot[4][2][4][64];  // [pair][slot][quad][lane] W[t]+K[t], 16 words
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int pr = wave & 3;
  const bool helper = wave >= 4;
  const long msg = (long)blockIdx.x * 256 + pr * 64 + lane;
  uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; i++) m[i] = seed + (uint32_t)(msg & 255) * 16 + i + blockIdx.x;
  uint32_t a, b, c, d, e, f, g, h;
  uint32_t w[16];
  for (int it = 0; it < iters; it++) {
    if (!helper) {
#pragma unroll
      for (int i = 0; i < 16; i++) w[i] = m[i] ^ st[i & 7];
#pragma unroll
      for (int q = 0; q < 4; q++) raw[pr][q][lane] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
      a = st[0]; b = st[1]; c = st[2]; d = st[3]; e = st[4]; f = st[5]; g = st[6]; h = st[7];
    }
    __syncthreads();
#pragma unroll 1
    for (int ch = 0; ch < 4; ch++) {
      if (helper) {
        if (ch == 0) {
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const uint4 v = raw[pr][q][lane];
            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
          }
        }
        if (ch < 3) {
#pragma unroll
          for (int j = 0; j < 16; j++) {
            if constexpr (HELPER_FAST) {
              const uint32_t s0 = small_sigma<1, 7, 18, 3>(w[(j + 1) & 15]);
              const uint32_t s1 = small_sigma<1, 17, 19, 10>(w[(j + 14) & 15]);
              w[j] = add2(add2(add2(w[j], s0), w[(j + 9) & 15]), s1);
            } else {
              const uint32_t s0 = small_sigma<0, 7, 18, 3>(w[(j + 1) & 15]);
              const uint32_t s1 = small_sigma<0, 17, 19, 10>(w[(j + 14) & 15]);
              w[j] = w[j] + s0 + w[(j + 9) & 15] + s1;
            }
          }
          uint32_t kw[16];
#pragma unroll
          for (int j = 0; j < 16; j++) kw[j] = HELPER_FAST ? add2(kK[16 * (ch + 1) + j], w[j]) : kK[16 * (ch + 1) + j] + w[j];
#pragma unroll
          for (int q = 0; q < 4; q++) slot[pr][ch & 1][q][lane] = make_uint4(kw[4 * q], kw[4 * q + 1], kw[4 * q + 2], kw[4 * q + 3]);
        }
      } else {
        uint32_t kw[16];
        if (ch == 0) {
#pragma unroll
          for (int j = 0; j < 16; j++) kw[j] = kK[j] + w[j];
        } else {
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const uint4 v = slot[pr][(ch - 1) & 1][q][lane];
            kw[4 * q] = v.x; kw[4 * q + 1] = v.y; kw[4 * q + 2] = v.z; kw[4 * q + 3] = v.w;
          }
        }
#pragma unroll
        for (int j = 0; j < 16; j += 8) {
          round_<0>(a, b, c, d, e, f, g, h, kw[j + 0]);
          round_<0>(h, a, b, c, d, e, f, g, kw[j + 1]);
          round_<0>(g, h, a, b, c, d, e, f, kw[j + 2]);
          round_<0>(f, g, h, a, b, c, d, e, kw[j + 3]);
          round_<0>(e, f, g, h, a, b, c, d, kw[j + 4]);
          round_<0>(d, e, f, g, h, a, b, c, kw[j + 5]);
          round_<0>(c, d, e, f, g, h, a, b, kw[j + 6]);
          round_<0>(b, c, d, e, f, g, h, a, kw[j + 7]);
        }
      }
      if (ch < 3) __syncthreads();
    }
    if (!helper) {
      st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
    }
  }
  if (!helper) {
#pragma unroll
    for (int i = 0; i < 8; i++) out[msg * 8 + i] = st[i];
  }
}

// ---- co-issue: SHA waves (rot 0 mixed or rot 3 slow-only) beside fast-only waves ----
// 512-thread workgroup: waves 0-3 run `iters` compressions (MODE & 1: SHA on),
// waves 4-7 run `fiters` x 64 dependent-chain v_bitop3 over 16 chains (MODE & 2: fast on).
template <int ROT, int MODE>
__global__ __launch_bounds__(512) void coissue_kernel(uint32_t* out, int iters, int fiters, uint32_t seed) {
  const int wave = threadIdx.x >> 6;
  uint32_t acc = 0;
  if (wave < 4) {
    if (MODE & 1) {
      uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                        0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
      uint32_t m[16];
#pragma unroll
      for (int i = 0; i < 16; i++) m[i] = seed + threadIdx.x * 16 + i + blockIdx.x;
      for (int it = 0; it < iters; it++) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = ROT == 3 ? xad0(m[i], st[i & 7]) : m[i] ^ st[i & 7];
        if constexpr (ROT == 3) compress_slow(st, w);
        else compress<ROT>(st, w);
      }
      acc = st[0] ^ st[5];
    }
  } else if (MODE & 2) {
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = seed ^ (threadIdx.x * 16 + i);
    for (int it = 0; it < fiters; it++) {
#pragma unroll
      for (int r = 0; r < 4; r++)
#pragma unroll
        for (int i = 0; i < 16; i++)
          asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(v[(i + 3) & 15]), "v"(v[(i + 7) & 15]));
    }
#pragma unroll
    for (int i = 0; i < 16; i++) acc ^= v[i];
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// ---- single-opcode rates ----
#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define S_(x) #x
enum { OP_XOR, OP_ALIGN, OP_LSHR64, OP_LSHL64, OP_MOV64, OP_ALIGNBYTE, OP_OR, OP_SUB, OP_ADDCO,
       OP_MUL24, OP_LSHLADD64, OP_NOT, OP_CNDMASK, OP_PKMOV, OP_COUNT };
static const char* kOpNames[] = {"v_xor_b32", "v_alignbit_b32", "v_lshrrev_b64", "v_lshlrev_b64",
                                 "v_mov_b64", "v_alignbyte_b32", "v_or_b32", "v_sub_u32",
                                 "v_add_co_u32", "v_mul_u32_u24", "v_lshl_add_u64", "v_not_b32",
                                 "v_cndmask_b32", "v_pk_mov_b32"};

template <int OP>
__global__ __launch_bounds__(256) void op_kernel(uint32_t* out, int iters, uint32_t seed) {
  uint64_t r[8];
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = ((uint64_t)(seed ^ threadIdx.x) << 32) | (seed + i * 77 + threadIdx.x);
  const uint32_t c1 = seed * 3 + 0x01020304u;
  const uint64_t c2 = 0x0706050403020100ull + seed;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int rep = 0; rep < 8; rep++) {
#pragma unroll
      for (int i = 0; i < 8; i++) {
        uint32_t lo = (uint32_t)r[i], hi = (uint32_t)(r[i] >> 32);
        if constexpr (OP == OP_XOR) {
          asm volatile("v_xor_b32 %0, %0, %2\n v_xor_b32 %1, %1, %2" : "+v"(lo), "+v"(hi) : "v"(c1));
        } else if constexpr (OP == OP_ALIGN) {
          asm volatile("v_alignbit_b32 %0, %0, %2, 7\n v_alignbit_b32 %1, %1, %2, 7" : "+v"(lo), "+v"(hi) : "v"(c1));
        } else if constexpr (OP == OP_ALIGNBYTE) {
          asm volatile("v_alignbyte_b32 %0, %0, %2, 1\n v_alignbyte_b32 %1, %1, %2, 1" : "+v"(lo), "+v"(hi) : "v"(c1));
        } else if constexpr (OP == OP_OR) {
          asm volatile("v_or_b32 %0, %0, %2\n v_or_b32 %1, %1, %2" : "+v"(lo), "+v"(hi) : "v"(c1));
        } else if constexpr (OP == OP_SUB) {
          asm volatile("v_sub_u32 %0, %0, %2\n v_sub_u32 %1, %1, %2" : "+v"(lo), "+v"(hi) : "v"(c1));
        } else if constexpr (OP == OP_ADDCO) {
          asm volatile("v_add_co_u32 %0, vcc, %0, %2\n v_add_co_u32 %1, vcc, %1, %2" : "+v"(lo), "+v"(hi) : "v"(c1) : "vcc");
        } else if constexpr (OP == OP_MUL24) {
          asm volatile("v_mul_u32_u24 %0, %0, %2\n v_mul_u32_u24 %1, %1, %2" : "+v"(lo), "+v"(hi) : "v"(c1));
        } else if constexpr (OP == OP_NOT) {
          asm volatile("v_not_b32 %0, %0\n v_not_b32 %1, %1" : "+v"(lo), "+v"(hi));
        } else if constexpr (OP == OP_CNDMASK) {
          asm volatile("v_cndmask_b32 %0, %0, %2, vcc\n v_cndmask_b32 %1, %1, %2, vcc" : "+v"(lo), "+v"(hi) : "v"(c1) : "vcc");
        }
        if constexpr (OP == OP_LSHR64) {
          asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(r[i]));
        } else if constexpr (OP == OP_LSHL64) {
          asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(r[i]));
        } else if constexpr (OP == OP_MOV64) {
          asm volatile("v_mov_b64 %0, %1" : "=v"(r[i]) : "v"(r[(i + 1) & 7]));
        } else if constexpr (OP == OP_LSHLADD64) {
          asm volatile("v_lshl_add_u64 %0, %0, 3, %1" : "+v"(r[i]) : "v"(c2));
        } else if constexpr (OP == OP_PKMOV) {
          asm volatile("v_pk_mov_b32 %0, %0, %1 op_sel:[1,0]" : "+v"(r[i]) : "v"(c2));
        } else {
          r[i] = ((uint64_t)hi << 32) | lo;
        }
      }
    }
  }
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) acc ^= r[i];
  if (acc == 0x123456789ull) out[blockIdx.x] = (uint32_t)acc;
}
// instructions per lane per iteration
static int op_instr(int op) {
  switch (op) {
    case OP_LSHR64: case OP_LSHL64: case OP_MOV64: case OP_LSHLADD64: case OP_PKMOV: return 64;
    default: return 128;
  }
}

// cross-wave mix: waves 0-3 of a 512-thread workgroup issue SLOW (v_alignbit)
// only, waves 4-7 FAST (v_xor) only; MODE 0 = all slow, 1 = all fast, 2 = half/half
template <int MODE>
__global__ __launch_bounds__(512) void mix_kernel(uint32_t* out, int iters, uint32_t seed) {
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; i++) v[i] = seed ^ (threadIdx.x * 16 + i);
  const uint32_t c1 = seed * 3 + 0x01020304u;
  const bool slow = MODE == 0 || (MODE == 2 && (threadIdx.x >> 6) < 4);
  if (slow) {
    for (int it = 0; it < iters; it++) {
#define SL(i) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(v[i]) : "v"(c1));
      R16(SL) R16(SL) R16(SL) R16(SL)
    }
  } else {
    for (int it = 0; it < iters; it++) {
#define FA(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[i]) : "v"(c1));
      R16(FA) R16(FA) R16(FA) R16(FA)
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) acc ^= v[i];
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

static float time_ms(void (*launch)(uint32_t*, int), uint32_t* out, int iters) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch(out, 2);
  (void)hipEventRecord(a, 0);
  launch(out, iters);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms;
}

static int g_blocks;
template <int ROT>
static void launch_sha(uint32_t* out, int iters) {
  hipLaunchKernelGGL(sha_kernel<ROT>, dim3(g_blocks), dim3(256), 0, 0, out, iters, 1u);
}
static void launch_sha_capped(uint32_t* out, int iters) {  // 48 KB LDS per 256-thread WG: 3 WGs/CU
  hipLaunchKernelGGL(sha_kernel<0>, dim3(g_blocks), dim3(256), 48 * 1024, 0, out, iters, 1u);
}
static int g_fiters = 200;
template <int ROT, int MODE>
static void launch_co(uint32_t* out, int iters) {
  hipLaunchKernelGGL((coissue_kernel<ROT, MODE>), dim3(g_blocks / 2), dim3(512), 0, 0, out, iters, g_fiters, 1u);
}
template <bool F>
static void launch_split(uint32_t* out, int iters) {
  hipLaunchKernelGGL(sha_split_kernel<F>, dim3(g_blocks), dim3(512), 0, 0, out, iters, 1u);
}
template <int OP>
static void launch_op(uint32_t* out, int iters) {
  hipLaunchKernelGGL(op_kernel<OP>, dim3(g_blocks), dim3(256), 0, 0, out, iters, 1u);
}
template <int MODE>
static void launch_mix(uint32_t* out, int iters) {
  hipLaunchKernelGGL(mix_kernel<MODE>, dim3(g_blocks / 2), dim3(512), 0, 0, out, iters, 1u);
}


// ---- mixed formulations: workgroups alternate between two SHA formulations so
// that every SIMD holds waves of both (slow-class rot 0/3 beside fast-class rot 1).
// Workgroup b uses RB when (b & 3) < NB, else RA.
template <int RA, int RB, int NB>
__global__ __launch_bounds__(256) void sha_mix_kernel(uint32_t* out, int iters, uint32_t seed) {
  uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; i++) m[i] = seed + threadIdx.x * 16 + i + blockIdx.x;
  if ((int)(blockIdx.x & 3) < NB) {
    for (int it = 0; it < iters; it++) {
      uint32_t w[16];
#pragma unroll
      for (int i = 0; i < 16; i++) w[i] = RB == 3 ? xad0(m[i], st[i & 7]) : m[i] ^ st[i & 7];
      if constexpr (RB == 3) compress_slow(st, w);
      else compress<RB>(st, w);
    }
  } else {
    for (int it = 0; it < iters; it++) {
      uint32_t w[16];
#pragma unroll
      for (int i = 0; i < 16; i++) w[i] = RA == 3 ? xad0(m[i], st[i & 7]) : m[i] ^ st[i & 7];
      if constexpr (RA == 3) compress_slow(st, w);
      else compress<RA>(st, w);
    }
  }
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; i++) out[t * 8 + i] = st[i];
}
template <int RA, int RB, int NB>
static void launch_shamix(uint32_t* out, int iters) {
  hipLaunchKernelGGL((sha_mix_kernel<RA, RB, NB>), dim3(g_blocks), dim3(256), 0, 0, out, iters, 1u);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int ncu = p.multiProcessorCount;
  g_blocks = ncu * 16;  // 16 x 256 threads per CU: 16 waves per SIMD requested
  uint32_t* out;
  (void)hipMalloc(&out, (size_t)g_blocks * 256 * 8 * 4);
  std::vector<uint32_t> h0((size_t)g_blocks * 256 * 8), h1(h0.size()), h2(h0.size());
  const double clk = 2.4e9;
  if (getenv("SHA_MIX_ONLY")) {
    const int iters = 100;
    const double comp = (double)g_blocks * 256 * iters;
    auto line = [&](const char* name, void (*fn)(uint32_t*, int)) {
      const float ms = time_ms(fn, out, iters);
      (void)hipMemcpy(h1.data(), out, h1.size() * 4, hipMemcpyDeviceToHost);
      printf("{\"sha_mix\":\"%s\",\"ms\":%.3f,\"gcompr_per_s\":%.2f}\n", name, ms, comp / ms / 1e6);
    };
    line("rot0_all", launch_sha<0>);
    line("rot1_all", launch_sha<1>);
    line("rot3_all", launch_sha<3>);
    line("rot0+rot1_1of4", launch_shamix<0, 1, 1>);
    line("rot0+rot1_2of4", launch_shamix<0, 1, 2>);
    line("rot0+rot1_3of4", launch_shamix<0, 1, 3>);
    line("rot3+rot1_1of4", launch_shamix<3, 1, 1>);
    line("rot3+rot1_2of4", launch_shamix<3, 1, 2>);
    line("rot3+rot1_3of4", launch_shamix<3, 1, 3>);
    line("rot0+rot3_2of4", launch_shamix<0, 3, 2>);
    return 0;
  }
  auto op_line = [&](int op, void (*fn)(uint32_t*, int)) {
    const int iters = 400;
    const float ms = time_ms(fn, out, iters);
    const double wi = (double)g_blocks * 4 * iters * op_instr(op);
    printf("{\"op\":\"%s\",\"ms\":%.3f,\"wave_instr_per_clk_per_cu_at_2.4GHz\":%.3f}\n", kOpNames[op], ms,
           wi / ncu / (ms * 1e-3) / clk);
  };
  op_line(OP_XOR, launch_op<OP_XOR>);
  op_line(OP_ALIGN, launch_op<OP_ALIGN>);
  op_line(OP_LSHR64, launch_op<OP_LSHR64>);
  op_line(OP_LSHL64, launch_op<OP_LSHL64>);
  op_line(OP_MOV64, launch_op<OP_MOV64>);
  op_line(OP_ALIGNBYTE, launch_op<OP_ALIGNBYTE>);
  op_line(OP_OR, launch_op<OP_OR>);
  op_line(OP_SUB, launch_op<OP_SUB>);
  op_line(OP_ADDCO, launch_op<OP_ADDCO>);
  op_line(OP_MUL24, launch_op<OP_MUL24>);
  op_line(OP_LSHLADD64, launch_op<OP_LSHLADD64>);
  op_line(OP_NOT, launch_op<OP_NOT>);
  op_line(OP_CNDMASK, launch_op<OP_CNDMASK>);
  op_line(OP_PKMOV, launch_op<OP_PKMOV>);
  {
    const int iters = 400;
    const float m0 = time_ms(launch_mix<0>, out, iters), m1 = time_ms(launch_mix<1>, out, iters),
                m2 = time_ms(launch_mix<2>, out, iters);
    printf("{\"probe\":\"cross_wave_mix\",\"all_slow_ms\":%.3f,\"all_fast_ms\":%.3f,\"half_half_ms\":%.3f,"
           "\"additive_prediction_ms\":%.3f}\n", m0, m1, m2, 0.5 * (m0 + m1));
  }
  {
    const int it = 40;
    for (int fi : {100, 200, 400}) {
      g_fiters = fi;
      const float f = time_ms(launch_co<0, 2>, out, it);
      const float s0 = time_ms(launch_co<0, 1>, out, it), b0 = time_ms(launch_co<0, 3>, out, it);
      const float s3 = time_ms(launch_co<3, 1>, out, it), b3 = time_ms(launch_co<3, 3>, out, it);
      printf("{\"coissue\":true,\"fast_iters\":%d,\"fast_alone_ms\":%.3f,\"sha_mixed_alone_ms\":%.3f,"
             "\"sha_mixed_with_fast_ms\":%.3f,\"sha_slowonly_alone_ms\":%.3f,\"sha_slowonly_with_fast_ms\":%.3f}\n",
             fi, f, s0, b0, s3, b3);
    }
  }
  const int iters = 100;
  const double comp = (double)g_blocks * 256 * iters;
  float ms[4];
  ms[0] = time_ms(launch_sha<0>, out, iters);
  (void)hipMemcpy(h0.data(), out, h0.size() * 4, hipMemcpyDeviceToHost);
  ms[1] = time_ms(launch_sha<1>, out, iters);
  (void)hipMemcpy(h1.data(), out, h1.size() * 4, hipMemcpyDeviceToHost);
  ms[2] = time_ms(launch_sha<2>, out, iters);
  (void)hipMemcpy(h2.data(), out, h2.size() * 4, hipMemcpyDeviceToHost);
  ms[3] = time_ms(launch_sha<3>, out, iters);
  {
    std::vector<uint32_t> h3(h0.size());
    (void)hipMemcpy(h3.data(), out, h3.size() * 4, hipMemcpyDeviceToHost);
    printf("{\"sha_rot\":3,\"ms\":%.3f,\"gcompr_per_s\":%.2f,\"same_digests\":%s}\n", ms[3], comp / ms[3] / 1e6,
           h3 == h0 ? "true" : "false");
  }
  bool same = h0 == h1 && h0 == h2;
  {
    const float mss = time_ms(launch_sha_capped, out, iters);
    printf("{\"sha_rot\":0,\"waves_per_simd\":3,\"ms\":%.3f,\"gcompr_per_s\":%.2f}\n", mss, comp / mss / 1e6);
  }
  for (int r = 0; r < 2; r++) {
    const float mss = time_ms(r ? launch_split<true> : launch_split<false>, out, iters);
    (void)hipMemcpy(h1.data(), out, h1.size() * 4, hipMemcpyDeviceToHost);
    const bool ok = h0 == h1;
    same = same && ok;
    printf("{\"sha_split\":\"%s\",\"ms\":%.3f,\"gcompr_per_s\":%.2f,\"same_digests\":%s}\n",
           r ? "helper_fast" : "helper_slow", mss, comp / mss / 1e6, ok ? "true" : "false");
  }
  for (int r = 0; r < 3; r++)
    printf("{\"sha_rot\":%d,\"ms\":%.3f,\"gcompr_per_s\":%.2f,\"same_digests\":%s}\n", r, ms[r],
           comp / ms[r] / 1e6, same ? "true" : "false");
  return same ? 0 : 1;
}
