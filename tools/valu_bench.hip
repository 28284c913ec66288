// valu_bench.hip -- measures the practical VALU ceilings of MI355X used by
// bench.py's roofline (SURVEY.md §8d asks to confirm the int32 estimate).
//   op tests: 16 independent chains per lane of one instruction kind, no
//             memory, 8 waves/SIMD -> lane-ops/s per instruction kind.
//   sha:      the production sha256_compress (csrc/sha256.hpp) looped on
//             register data -> compressions/s with no memory traffic.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/valu_bench.hip -o tools/valu_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../celestia-app_amd/csrc/sha256.hpp"

using namespace dagpu;

enum Op { XOR = 0, ADD, ALIGNBIT, BITOP3, ADD3, PERM, FMA_F32, PK_FMA_F32 };
static const char* kNames[] = {"v_xor_b32", "v_add_u32", "v_alignbit_b32", "v_bitop3_b32",
                               "v_add3_u32", "v_perm_b32", "v_fma_f32", "v_pk_fma_f32"};

template <int OP>
__global__ __launch_bounds__(256) void op_kernel(uint32_t* out, int iters, uint32_t seed) {
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; i++) v[i] = seed ^ (threadIdx.x * 16 + i);
  const uint32_t s1 = seed * 3 + 1, s2 = seed * 7 + 5;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
#pragma unroll
      for (int i = 0; i < 16; i++) {
        uint32_t x = v[i];
        // xor/add chains go through inline asm: plain C lets the compiler fold
        // the 8 rounds algebraically (r01 reported v_xor_b32 above the issue peak)
        if constexpr (OP == XOR) asm volatile("v_xor_b32 %0, %1, %2" : "=v"(x) : "v"(x), "v"(v[(i + 3) & 15]));
        if constexpr (OP == ADD) asm volatile("v_add_u32 %0, %1, %2" : "=v"(x) : "v"(x), "v"(v[(i + 3) & 15]));
        if constexpr (OP == ALIGNBIT) x = __builtin_amdgcn_alignbit(x, v[(i + 3) & 15], 7);
        if constexpr (OP == BITOP3) x = __builtin_amdgcn_bitop3_b32(x, v[(i + 3) & 15], v[(i + 7) & 15], 0x96);
        if constexpr (OP == ADD3) x = x + v[(i + 3) & 15] + v[(i + 7) & 15];
        if constexpr (OP == PERM) x = __builtin_amdgcn_perm(x, v[(i + 3) & 15], s1);
        if constexpr (OP == FMA_F32) x = __float_as_uint(__builtin_fmaf(__uint_as_float(x), 1.0001f, __uint_as_float(v[(i + 3) & 15])));
        if constexpr (OP == PK_FMA_F32) {
          typedef float f2 __attribute__((ext_vector_type(2)));
          f2 a = {__uint_as_float(x), __uint_as_float(v[(i + 1) & 15])};
          f2 b = {__uint_as_float(v[(i + 3) & 15]), __uint_as_float(v[(i + 5) & 15])};
          f2 c = __builtin_elementwise_fma(a, (f2){1.0001f, 0.9999f}, b);
          x = __float_as_uint(c.x) ^ __float_as_uint(c.y);
        }
        v[i] = x;
      }
    }
  }
  uint32_t acc = s2;
#pragma unroll
  for (int i = 0; i < 16; i++) acc += v[i];
  if (acc == 0x12345678u) out[blockIdx.x] = acc;  // keep live
}

__global__ __launch_bounds__(256) void sha_kernel(uint32_t* out, int iters, uint32_t seed) {
  uint32_t st[8];
  sha256_init(st);
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; i++) m[i] = seed + threadIdx.x * 16 + i + blockIdx.x;
  for (int it = 0; it < iters; it++) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = m[i] ^ st[i & 7];
    sha256_compress(st, w);
  }
  uint32_t acc = st[0] ^ st[1] ^ st[2] ^ st[3] ^ st[4] ^ st[5] ^ st[6] ^ st[7];
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <int OP>
static void run_op(uint32_t* out, hipEvent_t a, hipEvent_t b, int blocks) {
  const int iters = 1000;
  hipLaunchKernelGGL(op_kernel<OP>, dim3(blocks), dim3(256), 0, 0, out, 10, 1u);
  (void)hipEventRecord(a, 0);
  hipLaunchKernelGGL(op_kernel<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, 1u);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  const double wave_instr = (double)blocks * 4 * iters * 8 * 16;  // 4 waves per block
  const double lane_ops = wave_instr * 64;
  // wave-instructions per CU per ns -> per clock at the nominal 2.4 GHz
  printf("{\"test\":\"%s\",\"ms\":%.3f,\"T_lane_ops\":%.2f,\"wave_instr_per_clk_per_cu_at_2.4GHz\":%.3f}\n",
         kNames[OP], ms, lane_ops / ms / 1e9, wave_instr / 256 / (ms * 1e-3) / 2.4e9);
}

int main() {
  uint32_t* out;
  (void)hipMalloc(&out, 1 << 20);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int blocks = 256 * 16;  // 16 workgroups of 256 threads per CU (8 waves/SIMD max)
  run_op<XOR>(out, a, b, blocks);
  run_op<ADD>(out, a, b, blocks);
  run_op<ALIGNBIT>(out, a, b, blocks);
  run_op<BITOP3>(out, a, b, blocks);
  run_op<ADD3>(out, a, b, blocks);
  run_op<PERM>(out, a, b, blocks);
  run_op<FMA_F32>(out, a, b, blocks);
  run_op<PK_FMA_F32>(out, a, b, blocks);
  run_op<XOR>(out, a, b, blocks);
  for (int rep = 0; rep < 2; rep++) {
    const int iters = 200;
    hipLaunchKernelGGL(sha_kernel, dim3(blocks), dim3(256), 0, 0, out, 2, 1u);
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(sha_kernel, dim3(blocks), dim3(256), 0, 0, out, iters, 1u);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    double comp = (double)blocks * 256 * iters;
    printf("{\"test\":\"sha256_compress\",\"ms\":%.3f,\"gcompr_per_s\":%.2f,\"tops_at_1384\":%.2f}\n",
           ms, comp / ms / 1e6, comp * 1384 / ms / 1e9);
  }
  return 0;
}
