// rs_bench.hip -- A/B microbenchmark of GF(2^8) encode-kernel variants at
// k=128 on contiguous vectors (row-pass shape), one process, interleaved runs
// (guide §5.4 rule 24).  Variants:
//   mul 0: 4 x 2-bit v_perm lookups (one SGPR table each)      [production]
//   mul 1: 3-bit/3-bit/2-bit lookups, second table dword forced into a VGPR
//          by an inline-asm v_mov right before use (no hoisting)
// and occupancy targets 2 / 3 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/rs_bench.hip -o tools/rs_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../celestia-app_amd/csrc/leo8.hpp"

using namespace dagpu;

struct Tab8 {
  uint32_t v[256][5];
};
constexpr Tab8 make_tab8() {
  Tab8 t{};
  for (int lm = 0; lm < 256; lm++) {
    auto mul = [&](int x) -> uint32_t {
      // c * x via the 2-bit tables (linear)
      uint32_t r = 0;
      for (int g = 0; g < 4; g++) r ^= (kGf8.t[g][lm] >> (8 * ((x >> (2 * g)) & 3))) & 0xFF;
      return r;
    };
    uint32_t a[8], b[8], c[4];
    for (int x = 0; x < 8; x++) { a[x] = mul(x); b[x] = mul(x << 3); }
    for (int x = 0; x < 4; x++) c[x] = mul(x << 6);
    t.v[lm][0] = a[0] | a[1] << 8 | a[2] << 16 | a[3] << 24;
    t.v[lm][1] = a[4] | a[5] << 8 | a[6] << 16 | a[7] << 24;
    t.v[lm][2] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
    t.v[lm][3] = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
    t.v[lm][4] = c[0] | c[1] << 8 | c[2] << 16 | c[3] << 24;
  }
  return t;
}
inline constexpr Tab8 kT8 = make_tab8();

template <int MV>
__device__ __forceinline__ void muladd_c(uint32_t& x, uint32_t y, const int lm) {
  if constexpr (MV == 0) {
    gf8_muladd(x, y, lm);
  } else {
    uint32_t v0, v1;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v0) : "s"(kT8.v[lm][1]));
    asm volatile("v_mov_b32 %0, %1" : "=v"(v1) : "s"(kT8.v[lm][3]));
    const uint32_t p0 = __builtin_amdgcn_perm(v0, kT8.v[lm][0], y & 0x07070707u);
    const uint32_t p1 = __builtin_amdgcn_perm(v1, kT8.v[lm][2], (y >> 3) & 0x07070707u);
    const uint32_t p2 = __builtin_amdgcn_perm(kT8.v[lm][4], kT8.v[lm][4], (y >> 6) & 0x03030303u);
    x = __builtin_amdgcn_bitop3_b32(x, p0, p1, 0x96) ^ p2;
  }
}

template <int MV>
__device__ __forceinline__ void ifft2v(uint32_t& x, uint32_t& y, const int lm) {
  y ^= x;
  if (lm != kGf8Mod) muladd_c<MV>(x, y, lm);
}
template <int MV>
__device__ __forceinline__ void fft2v(uint32_t& x, uint32_t& y, const int lm) {
  if (lm != kGf8Mod) muladd_c<MV>(x, y, lm);
  y ^= x;
}

template <int MV, int K, int DIST>
__device__ __forceinline__ void ifft_l(uint32_t (&w)[K]) {
  if constexpr (DIST * 4 <= K) {
#pragma unroll
    for (int r = 0; r < K; r += DIST * 4) {
      const int iend = r + DIST;
      const int l01 = kGf8.skew[K - 1 + iend], l02 = kGf8.skew[K - 1 + iend + DIST],
                l23 = kGf8.skew[K - 1 + iend + 2 * DIST];
#pragma unroll
      for (int i = r; i < iend; i++) {
        ifft2v<MV>(w[i], w[i + DIST], l01);
        ifft2v<MV>(w[i + 2 * DIST], w[i + 3 * DIST], l23);
        ifft2v<MV>(w[i], w[i + 2 * DIST], l02);
        ifft2v<MV>(w[i + DIST], w[i + 3 * DIST], l02);
      }
    }
    ifft_l<MV, K, DIST * 4>(w);
  } else if constexpr (DIST < K) {
    const int lm = kGf8.skew[K - 1 + DIST];
#pragma unroll
    for (int i = 0; i < DIST; i++) ifft2v<MV>(w[i], w[i + DIST], lm);
  }
}
template <int MV, int K, int DIST4>
__device__ __forceinline__ void fft_l(uint32_t (&w)[K]) {
  constexpr int DIST = DIST4 >> 2;
  if constexpr (DIST != 0) {
#pragma unroll
    for (int r = 0; r < K; r += DIST4) {
      const int iend = r + DIST;
      const int l01 = kGf8.skew[iend - 1], l02 = kGf8.skew[iend + DIST - 1], l23 = kGf8.skew[iend + 2 * DIST - 1];
#pragma unroll
      for (int i = r; i < iend; i++) {
        fft2v<MV>(w[i], w[i + 2 * DIST], l02);
        fft2v<MV>(w[i + DIST], w[i + 3 * DIST], l02);
        fft2v<MV>(w[i], w[i + DIST], l01);
        fft2v<MV>(w[i + 2 * DIST], w[i + 3 * DIST], l23);
      }
    }
    fft_l<MV, K, DIST>(w);
  } else if constexpr (DIST4 == 2) {
#pragma unroll
    for (int r = 0; r < K; r += 2) fft2v<MV>(w[r], w[r + 1], kGf8.skew[r]);
  }
}

template <int MV, int WAVES>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(WAVES, 8))) void enc(
    const uint8_t* in, uint8_t* out) {
  constexpr int K = 128;
  const long vec = blockIdx.x;
  const uint32_t col = threadIdx.x * 4u;
  const auto ir = make_rsrc(in + vec * K * 512);
  uint32_t w[K];
#pragma unroll
  for (int i = 0; i < K; i++) w[i] = __builtin_amdgcn_raw_buffer_load_b32(ir, col, i * 512u, 0);
  ifft_l<MV, K, 1>(w);
  fft_l<MV, K, K>(w);
  const auto orr = make_rsrc(out + vec * K * 512);
#pragma unroll
  for (int i = 0; i < K; i++) __builtin_amdgcn_raw_buffer_store_b32(w[i], orr, col, i * 512u, 0);
}

int main() {
  const long nvec = 16384;
  const size_t bytes = nvec * 128 * 512;
  uint8_t *in, *out0, *out1;
  (void)hipMalloc(&in, bytes);
  (void)hipMalloc(&out0, bytes);
  (void)hipMalloc(&out1, bytes);
  uint8_t* h = (uint8_t*)malloc(bytes);
  for (size_t i = 0; i < bytes; i++) h[i] = (uint8_t)(i * 2654435761u >> 13);
  (void)hipMemcpy(in, h, bytes, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  struct V { const char* name; void (*k)(const uint8_t*, uint8_t*); uint8_t* o; };
  V vs[] = {{"perm2bit_w2", enc<0, 2>, out0}, {"perm3bit_asm_w2", enc<1, 2>, out1},
            {"perm2bit_w3", enc<0, 3>, out0}, {"perm3bit_asm_w3", enc<1, 3>, out1}};
  double best[4] = {1e9, 1e9, 1e9, 1e9};
  for (int rep = 0; rep < 5; rep++) {
    for (int v = 0; v < 4; v++) {
      hipLaunchKernelGGL(vs[v].k, dim3(nvec), dim3(128), 0, 0, in, vs[v].o);
      (void)hipEventRecord(a, 0);
      hipLaunchKernelGGL(vs[v].k, dim3(nvec), dim3(128), 0, 0, in, vs[v].o);
      (void)hipEventRecord(b, 0);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      if (ms < best[v]) best[v] = ms;
    }
  }
  uint8_t* h0 = (uint8_t*)malloc(bytes);
  uint8_t* h1 = (uint8_t*)malloc(bytes);
  (void)hipMemcpy(h0, out0, bytes, hipMemcpyDeviceToHost);
  (void)hipMemcpy(h1, out1, bytes, hipMemcpyDeviceToHost);
  const int same = memcmp(h0, h1, bytes) == 0;
  for (int v = 0; v < 4; v++)
    printf("{\"variant\":\"%s\",\"ms\":%.3f,\"alg_GBs\":%.1f,\"outputs_equal\":%d}\n", vs[v].name, best[v],
           2.0 * bytes / (best[v] * 1e-3) / 1e9, same);
  return 0;
}
