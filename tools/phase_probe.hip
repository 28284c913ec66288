// phase_probe.hip -- does a phase of slow-class VALU instructions (v_perm) slow
// down a LATER phase of fast-class ones (v_bitop3) in the same wave?  The issue
// bench (profiles/issue_bench_r01.log) shows that interleaving them runs every
// instruction at the slow rate; a decoder that does its byte-domain multiplies
// (v_perm) before and after a bit-sliced transform (v_bitop3 only) needs the
// phases to be independent.  Prints ms for: fast only, slow only, slow then
// fast, and fast interleaved 1:4 with slow, 16 chains per lane, 8 waves/SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/phase_probe.hip -o tools/phase_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define S(i) #i
#define FAST(i) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(v[(i + 3) & 15]), "v"(v[(i + 7) & 15]));
#define SLOW(i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(v[(i + 3) & 15]), "v"(sel));

template <int NSLOW, int NFAST, bool MIX>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; i++) v[i] = seed ^ (threadIdx.x * 16 + i);
  const uint32_t sel = 0x01020304u + seed;
  if constexpr (MIX) {
#pragma unroll 1
    for (int r = 0; r < NSLOW; r++) {
#pragma unroll
      for (int i = 0; i < 16; i++) {
        SLOW(i)
        FAST(i) FAST((i + 5) & 15) FAST((i + 9) & 15) FAST((i + 13) & 15)
      }
    }
  } else {
#pragma unroll 1
    for (int r = 0; r < NSLOW; r++) {
#pragma unroll
      for (int i = 0; i < 16; i++) { SLOW(i) }
    }
#pragma unroll 1
    for (int r = 0; r < NFAST; r++) {
#pragma unroll
      for (int i = 0; i < 16; i++) { FAST(i) }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) acc += v[i];
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <int NSLOW, int NFAST, bool MIX>
static void run(const char* name, uint32_t* out, hipEvent_t a, hipEvent_t b) {
  const int blocks = 256 * 16;  // 8 waves/SIMD
  hipLaunchKernelGGL((k<NSLOW, NFAST, MIX>), dim3(blocks), dim3(256), 0, 0, out, 1u);
  (void)hipEventRecord(a, 0);
  hipLaunchKernelGGL((k<NSLOW, NFAST, MIX>), dim3(blocks), dim3(256), 0, 0, out, 1u);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  printf("{\"probe\":\"%s\",\"slow_instr_per_lane\":%d,\"fast_instr_per_lane\":%d,\"ms\":%.3f}\n", name,
         NSLOW * 16, (MIX ? 4 * NSLOW : NFAST) * 16, ms);
}

int main() {
  uint32_t* out;
  (void)hipMalloc(&out, 1 << 20);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  run<0, 400, false>("fast_only", out, a, b);
  run<100, 0, false>("slow_only", out, a, b);
  run<100, 400, false>("slow_then_fast", out, a, b);
  run<100, 0, true>("interleaved_1_slow_4_fast", out, a, b);
  return 0;
}
