// overlap_probe.hip -- feasibility probe for RS/SHA overlap on MI355X.
//
// Question: if the RS encoder were lean (1 wave per SIMD per workgroup, ~100
// VGPRs, little or no LDS), would the hardware dispatcher co-schedule it with
// the SHA leaf work launched on another stream, and would the pair finish in
// about max(T_sha + RS issue share, T_rs) instead of T_sha + T_rs?
//
// sha: leaf-shaped SHA work: each lane reads 9 x 64 B and runs 9 compressions
//      (csrc/sha256.hpp), 256-thread workgroups; optional dynamic LDS caps its
//      occupancy (lds_kb per workgroup).
// rs:  RS-shaped memory/VALU work: a 4-wave workgroup reads one 64 KB "vector"
//      (k = 128 shards x 512 B), does `ops` fast xor/bitop3 ops per data dword
//      group, writes 64 KB.
// Prints ms alone and concurrent (two non-blocking streams).
// argv: <sha LDS KB> <rs variant> [sha WG size] [sha persistent WGs per CU] [work queue 0/1] [variant 5: rs WGs per CU]
// rs variant 5 = rs2 as a persistent grid taking groups from a counter; 6 = rs6 (8-wave, 2 vectors,
// ~90 VGPRs), 7 = rs6 as a persistent grid
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/overlap_probe.hip -o tools/overlap_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../celestia-app_amd/csrc/sha256.hpp"

using namespace dagpu;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(6))) void sha_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                  long n) {
  extern __shared__ uint32_t cap[];  // occupancy cap only
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t st[8];
  sha256_init(st);
  const u32x4* p = (const u32x4*)(in + i * 144);
  // one block prefetched ahead (~80 VGPRs, like nmt_leaf_kernel)
  u32x4 nx[4];
#pragma unroll
  for (int q = 0; q < 4; q++) nx[q] = p[q];
#pragma unroll
  for (int b = 0; b < 9; b++) {  // unrolled: ~9 compression sites of code, like nmt_leaf_kernel's 27 KB
    uint32_t w[16];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      w[4 * q] = nx[q].x; w[4 * q + 1] = nx[q].y; w[4 * q + 2] = nx[q].z; w[4 * q + 3] = nx[q].w;
    }
    if (b + 1 < 9) {
#pragma unroll
      for (int q = 0; q < 4; q++) nx[q] = p[(b + 1) * 4 + q];
    }
    sha256_compress(st, w);
  }
  if (threadIdx.x == 0 && n < 0) cap[0] = st[0];
  out[i] = st[0] ^ st[7];
}

// persistent form: a fixed grid (wgs_per_cu x CUs) strides over the leaves, so
// the SHA work holds a bounded number of wave slots without claiming LDS
__global__ __launch_bounds__(256) void sha_persist_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                          long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    uint32_t st[8];
    sha256_init(st);
    const u32x4* p = (const u32x4*)(in + i * 144);
    u32x4 nx[4];
#pragma unroll
    for (int q = 0; q < 4; q++) nx[q] = p[q];
#pragma unroll
    for (int b = 0; b < 9; b++) {
      uint32_t w[16];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        w[4 * q] = nx[q].x; w[4 * q + 1] = nx[q].y; w[4 * q + 2] = nx[q].z; w[4 * q + 3] = nx[q].w;
      }
      if (b + 1 < 9) {
#pragma unroll
        for (int q = 0; q < 4; q++) nx[q] = p[(b + 1) * 4 + q];
      }
      sha256_compress(st, w);
    }
    out[i] = st[0] ^ st[7];
  }
}

// work-queue form: a fixed grid, each workgroup grabs 256 leaves at a time from
// a counter, so workgroups that become resident late simply take less work
__global__ __launch_bounds__(256) void sha_queue_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                        long n, unsigned long long* counter) {
  __shared__ long base_s;
  for (;;) {
    if (threadIdx.x == 0) base_s = (long)atomicAdd(counter, 256ull);
    __syncthreads();
    const long base = base_s;
    __syncthreads();
    if (base >= n) return;
    const long i = base + threadIdx.x;
    if (i < n) {
      uint32_t st[8];
      sha256_init(st);
      const u32x4* p = (const u32x4*)(in + i * 144);
      u32x4 nx[4];
#pragma unroll
      for (int q = 0; q < 4; q++) nx[q] = p[q];
#pragma unroll
      for (int b = 0; b < 9; b++) {
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          w[4 * q] = nx[q].x; w[4 * q + 1] = nx[q].y; w[4 * q + 2] = nx[q].z; w[4 * q + 3] = nx[q].w;
        }
        if (b + 1 < 9) {
#pragma unroll
          for (int q = 0; q < 4; q++) nx[q] = p[(b + 1) * 4 + q];
        }
        sha256_compress(st, w);
      }
      out[i] = st[0] ^ st[7];
    }
  }
}

template <int OPS>
__global__ __launch_bounds__(256) void rs_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, long nvec) {
  const long v = blockIdx.x;
  if (v >= nvec) return;
  const u32x4* src = in + v * 4096;  // 64 KB per vector (64 data dwords per lane)
  u32x4* dst = out + v * 4096;
  u32x4 d[16];
#pragma unroll
  for (int j = 0; j < 16; j++) d[j] = src[j * 256 + threadIdx.x];
  uint32_t x[64];
#pragma unroll
  for (int j = 0; j < 16; j++) { x[4 * j] = d[j].x; x[4 * j + 1] = d[j].y; x[4 * j + 2] = d[j].z; x[4 * j + 3] = d[j].w; }
#pragma unroll 1
  for (int r = 0; r < OPS; r++) {
#pragma unroll
    for (int j = 0; j < 64; j++) {
      const uint32_t a = x[(j + 1) & 63], b = x[(j + 7) & 63];
      asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[j]) : "v"(a), "v"(b));
    }
  }
#pragma unroll
  for (int j = 0; j < 16; j++) dst[j * 256 + threadIdx.x] = (u32x4){x[4 * j], x[4 * j + 1], x[4 * j + 2], x[4 * j + 3]};
}


// rs2: the L1 shape -- a 4-wave workgroup holds 128 KB (two 64-KB vectors):
// 128 data dwords per lane (~200 VGPRs), one 64-KB LDS exchange (2 passes).
template <int OPS>
__device__ __forceinline__ void rs2_body(const u32x4* __restrict__ in, u32x4* __restrict__ out, long v, u32x4* lds);
template <int OPS>
__global__ __launch_bounds__(256) void rs2_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, long ngrp) {
  __shared__ u32x4 lds[4096];  // 64 KB
  const long v = blockIdx.x;
  if (v >= ngrp) return;
  rs2_body<OPS>(in, out, v, lds);
}
// persistent rs2: a fixed grid takes groups from a counter
template <int OPS>
__global__ __launch_bounds__(256) void rs2_queue_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, long ngrp,
                                                        unsigned long long* counter) {
  __shared__ u32x4 lds[4096];  // 64 KB
  __shared__ long v_s;
  for (;;) {
    __syncthreads();
    if (threadIdx.x == 0) v_s = (long)atomicAdd(counter, 1ull);
    __syncthreads();
    const long v = v_s;
    if (v >= ngrp) return;
    rs2_body<OPS>(in, out, v, lds);
  }
}
template <int OPS>
__device__ __forceinline__ void rs2_body(const u32x4* __restrict__ in, u32x4* __restrict__ out, long v, u32x4* lds) {
  const u32x4* src = in + v * 8192;  // 128 KB per group
  u32x4* dst = out + v * 8192;
  uint32_t x[128];
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const u32x4 d = src[j * 256 + threadIdx.x];
    x[4 * j] = d.x; x[4 * j + 1] = d.y; x[4 * j + 2] = d.z; x[4 * j + 3] = d.w;
  }
#pragma unroll 1
  for (int r = 0; r < OPS; r++) {
#pragma unroll
    for (int j = 0; j < 128; j++) {
      const uint32_t a = x[(j + 1) & 127], b = x[(j + 7) & 127];
      asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[j]) : "v"(a), "v"(b));
    }
    if (r == OPS / 2) {  // one exchange through LDS, two passes of 64 dwords
#pragma unroll
      for (int h = 0; h < 2; h++) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 16; j++)
          lds[j * 256 + threadIdx.x] = (u32x4){x[64 * h + 4 * j], x[64 * h + 4 * j + 1], x[64 * h + 4 * j + 2], x[64 * h + 4 * j + 3]};
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 16; j++) {
          const u32x4 q = lds[j * 256 + (threadIdx.x ^ 64)];
          x[64 * h + 4 * j] = q.x; x[64 * h + 4 * j + 1] = q.y; x[64 * h + 4 * j + 2] = q.z; x[64 * h + 4 * j + 3] = q.w;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 32; j++) dst[j * 256 + threadIdx.x] = (u32x4){x[4 * j], x[4 * j + 1], x[4 * j + 2], x[4 * j + 3]};
}

// rs3: lean registers (64 data dwords) + one 64-KB LDS exchange (L2 shape)
template <int OPS>
__global__ __launch_bounds__(256) void rs3_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, long nvec) {
  __shared__ u32x4 lds[4096];  // 64 KB
  const long v = blockIdx.x;
  if (v >= nvec) return;
  const u32x4* src = in + v * 4096;
  u32x4* dst = out + v * 4096;
  uint32_t x[64];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const u32x4 d = src[j * 256 + threadIdx.x];
    x[4 * j] = d.x; x[4 * j + 1] = d.y; x[4 * j + 2] = d.z; x[4 * j + 3] = d.w;
  }
#pragma unroll 1
  for (int r = 0; r < OPS; r++) {
#pragma unroll
    for (int j = 0; j < 64; j++) {
      const uint32_t a = x[(j + 1) & 63], b = x[(j + 7) & 63];
      asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[j]) : "v"(a), "v"(b));
    }
    if (r == OPS / 3 || r == 2 * OPS / 3) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 16; j++) lds[j * 256 + threadIdx.x] = (u32x4){x[4 * j], x[4 * j + 1], x[4 * j + 2], x[4 * j + 3]};
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const u32x4 q = lds[j * 256 + (threadIdx.x ^ 64)];
        x[4 * j] = q.x; x[4 * j + 1] = q.y; x[4 * j + 2] = q.z; x[4 * j + 3] = q.w;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 16; j++) dst[j * 256 + threadIdx.x] = (u32x4){x[4 * j], x[4 * j + 1], x[4 * j + 2], x[4 * j + 3]};
}

// rs4: fat registers (128 data dwords, two 64-KB vectors per workgroup), no LDS
template <int OPS>
__global__ __launch_bounds__(256) void rs4_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, long ngrp) {
  const long v = blockIdx.x;
  if (v >= ngrp) return;
  const u32x4* src = in + v * 8192;
  u32x4* dst = out + v * 8192;
  uint32_t x[128];
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const u32x4 d = src[j * 256 + threadIdx.x];
    x[4 * j] = d.x; x[4 * j + 1] = d.y; x[4 * j + 2] = d.z; x[4 * j + 3] = d.w;
  }
#pragma unroll 1
  for (int r = 0; r < OPS; r++) {
#pragma unroll
    for (int j = 0; j < 128; j++) {
      const uint32_t a = x[(j + 1) & 127], b = x[(j + 7) & 127];
      asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[j]) : "v"(a), "v"(b));
    }
  }
#pragma unroll
  for (int j = 0; j < 32; j++) dst[j * 256 + threadIdx.x] = (u32x4){x[4 * j], x[4 * j + 1], x[4 * j + 2], x[4 * j + 3]};
}

// rs5: variant 0 with the op loop fully unrolled (~60 KB of straight-line code,
// the size of a real k = 128 encoder) -- does instruction-cache pressure spoil
// the overlap with the SHA kernel?
template <int OPS>
__global__ __launch_bounds__(256) void rs5_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, long nvec) {
  const long v = blockIdx.x;
  if (v >= nvec) return;
  const u32x4* src = in + v * 4096;
  u32x4* dst = out + v * 4096;
  uint32_t x[64];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const u32x4 d = src[j * 256 + threadIdx.x];
    x[4 * j] = d.x; x[4 * j + 1] = d.y; x[4 * j + 2] = d.z; x[4 * j + 3] = d.w;
  }
#pragma unroll
  for (int r = 0; r < OPS; r++) {
#pragma unroll
    for (int j = 0; j < 64; j++) {
      const uint32_t a = x[(j + 1) & 63], b = x[(j + 7) & 63];
      asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[j]) : "v"(a), "v"(b));
    }
  }
#pragma unroll
  for (int j = 0; j < 16; j++) dst[j * 256 + threadIdx.x] = (u32x4){x[4 * j], x[4 * j + 1], x[4 * j + 2], x[4 * j + 3]};
}


// rs6: the low-VGPR shape -- an 8-wave workgroup holds 2 vectors (128 KB):
// 64 data dwords per lane (~90 VGPRs, 4 waves/SIMD), one 64-KB LDS exchange in
// two halves; OPS x 64 bitop3 per lane (OPS = 55: the real encoder's VALU work
// per byte spread over twice the waves).
template <int OPS>
__device__ __forceinline__ void rs6_body(const u32x4* __restrict__ in, u32x4* __restrict__ out, long g, u32x4* lds) {
  const u32x4* src = in + g * 8192;  // 128 KB per group
  u32x4* dst = out + g * 8192;
  uint32_t x[64];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const u32x4 d = src[j * 512 + threadIdx.x];
    x[4 * j] = d.x; x[4 * j + 1] = d.y; x[4 * j + 2] = d.z; x[4 * j + 3] = d.w;
  }
#pragma unroll 1
  for (int r = 0; r < OPS; r++) {
#pragma unroll
    for (int j = 0; j < 64; j++) {
      const uint32_t a = x[(j + 1) & 63], b = x[(j + 7) & 63];
      asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[j]) : "v"(a), "v"(b));
    }
    if (r == OPS / 2) {
#pragma unroll
      for (int h = 0; h < 2; h++) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 8; j++)
          lds[j * 512 + threadIdx.x] = (u32x4){x[32 * h + 4 * j], x[32 * h + 4 * j + 1], x[32 * h + 4 * j + 2], x[32 * h + 4 * j + 3]};
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const u32x4 q = lds[j * 512 + (threadIdx.x ^ 64)];
          x[32 * h + 4 * j] = q.x; x[32 * h + 4 * j + 1] = q.y; x[32 * h + 4 * j + 2] = q.z; x[32 * h + 4 * j + 3] = q.w;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 16; j++) dst[j * 512 + threadIdx.x] = (u32x4){x[4 * j], x[4 * j + 1], x[4 * j + 2], x[4 * j + 3]};
}
template <int OPS>
__global__ __launch_bounds__(512) void rs6_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, long ngrp) {
  __shared__ u32x4 lds[4096];  // 64 KB
  if ((long)blockIdx.x >= ngrp) return;
  rs6_body<OPS>(in, out, blockIdx.x, lds);
}
template <int OPS>
__global__ __launch_bounds__(512) void rs6_queue_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, long ngrp,
                                                        unsigned long long* counter) {
  __shared__ u32x4 lds[4096];
  __shared__ long g_s;
  for (;;) {
    __syncthreads();
    if (threadIdx.x == 0) g_s = (long)atomicAdd(counter, 1ull);
    __syncthreads();
    const long g = g_s;
    if (g >= ngrp) return;
    rs6_body<OPS>(in, out, g, lds);
  }
}

int main(int argc, char** argv) {
  const long ncell = 256L * 65536;  // leaves per 256-square step
  const long nvec = 256L * 384;  // RS vectors per step (k = 128, 64 KB each)
  const int lds_kb = argc > 1 ? atoi(argv[1]) : 0;
  uint32_t *shin, *shout;
  u32x4 *rin, *rout;
  (void)hipMalloc(&shin, ncell * 576);
  (void)hipMalloc(&shout, ncell * 4);
  (void)hipMalloc(&rin, nvec * 65536);
  (void)hipMalloc(&rout, nvec * 65536);
  (void)hipMemset(shin, 1, ncell * 576);
  (void)hipMemset(rin, 2, nvec * 65536);
  hipStream_t sa, sb;
  (void)hipStreamCreateWithFlags(&sa, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&sb, hipStreamNonBlocking);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int shab = argc > 3 ? atoi(argv[3]) : 256;  // sha workgroup size
  const int persist = argc > 4 ? atoi(argv[4]) : 0;  // SHA workgroups per CU (persistent grid), 0 = off
  const int queue = argc > 5 ? atoi(argv[5]) : 0;  // 1: the persistent grid takes work from a queue
  const int rs_wgs = argc > 6 ? atoi(argv[6]) : 1;  // variant 5: persistent rs2 workgroups per CU
  unsigned long long* counter;
  unsigned long long* rcounter;
  (void)hipMalloc(&counter, 8);
  (void)hipMalloc(&rcounter, 8);
  auto sha = [&](hipStream_t s) {
    if (persist > 0 && queue) {
      (void)hipMemsetAsync(counter, 0, 8, s);
      hipLaunchKernelGGL(sha_queue_kernel, dim3(256 * persist), dim3(256), 0, s, shin, shout, ncell, counter);
      return;
    }
    if (persist > 0) {
      hipLaunchKernelGGL(sha_persist_kernel, dim3(256 * persist), dim3(256), 0, s, shin, shout, ncell);
      return;
    }
    hipLaunchKernelGGL(sha_kernel, dim3((unsigned)((ncell + shab - 1) / shab)), dim3(shab), lds_kb * 1024, s, shin, shout, ncell);
  };
  const int variant = argc > 2 ? atoi(argv[2]) : 0;
  auto rs = [&](hipStream_t s) {
    if (variant == 0) hipLaunchKernelGGL(rs_kernel<52>, dim3((unsigned)nvec), dim3(256), 0, s, rin, rout, nvec);
    else if (variant == 1) hipLaunchKernelGGL(rs2_kernel<55>, dim3((unsigned)(nvec / 2)), dim3(256), 0, s, rin, rout, nvec / 2);
    else if (variant == 2) hipLaunchKernelGGL(rs3_kernel<52>, dim3((unsigned)nvec), dim3(256), 0, s, rin, rout, nvec);
    else if (variant == 3) hipLaunchKernelGGL(rs4_kernel<55>, dim3((unsigned)(nvec / 2)), dim3(256), 0, s, rin, rout, nvec / 2);
    else if (variant == 6) hipLaunchKernelGGL(rs6_kernel<55>, dim3((unsigned)(nvec / 2)), dim3(512), 0, s, rin, rout, nvec / 2);
    else if (variant == 7) {
      (void)hipMemsetAsync(rcounter, 0, 8, s);
      hipLaunchKernelGGL(rs6_queue_kernel<55>, dim3((unsigned)(256 * rs_wgs)), dim3(512), 0, s, rin, rout, nvec / 2, rcounter);
    }
    else if (variant == 5) {
      (void)hipMemsetAsync(rcounter, 0, 8, s);
      hipLaunchKernelGGL(rs2_queue_kernel<55>, dim3((unsigned)(256 * rs_wgs)), dim3(256), 0, s, rin, rout, nvec / 2, rcounter);
    }
    else hipLaunchKernelGGL(rs5_kernel<90>, dim3((unsigned)nvec), dim3(256), 0, s, rin, rout, nvec);
  };
  auto timeit = [&](const char* name, auto fn) {
    fn();
    (void)hipDeviceSynchronize();
    float best = 1e9;
    for (int rep = 0; rep < 5; rep++) {
      (void)hipEventRecord(e0, 0);
      fn();
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("{\"probe\":\"%s\",\"variant\":%d,\"sha_wg\":%d,\"lds_kb\":%d,\"sha_persist_wg_per_cu\":%d,\"queue\":%d,\"ms\":%.3f}\n", name,
           variant, shab, lds_kb, persist, queue, best);
    fflush(stdout);
  };
  // the default stream (0) is blocking w.r.t. nothing here: sa/sb are non-blocking,
  // so bracket the concurrent pair with events joined on stream 0
  hipEvent_t ja, jb;
  (void)hipEventCreateWithFlags(&ja, hipEventDisableTiming);
  (void)hipEventCreateWithFlags(&jb, hipEventDisableTiming);
  auto both = [&]() {
    (void)hipEventRecord(ja, 0);
    (void)hipStreamWaitEvent(sa, ja, 0);
    (void)hipStreamWaitEvent(sb, ja, 0);
    rs(sb);
    sha(sa);
    (void)hipEventRecord(ja, sa);
    (void)hipEventRecord(jb, sb);
    (void)hipStreamWaitEvent(0, ja, 0);
    (void)hipStreamWaitEvent(0, jb, 0);
  };
  timeit("sha_alone", [&]() { sha(0); });
  timeit("rs_alone", [&]() { rs(0); });
  timeit("serial", [&]() { rs(0); sha(0); });
  timeit("concurrent", both);
  return 0;
}
