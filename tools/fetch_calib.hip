// fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE against a known byte
// count for the access patterns of this repo's kernels (MI355X_MICROARCH.md:
// "other access widths are uncalibrated").  Each kernel reads every byte of a
// 2 GiB buffer exactly once and writes 4 B per lane.
//   A  lane-per-share, 16 B/lane loads at a 512-B lane stride (leaf kernel r01)
//   B  4 lanes x 16 B contiguous per share, 16 shares per instruction (LDS-staged leaf)
//   C  4 B/lane, 256 B contiguous per wave instruction (RS encoder buffer loads)
//   D  16 B/lane fully contiguous (reference streaming pattern of the guide)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void kA(const uint4* p, uint32_t* out) {  // 1 lane = 1 share (32 uint4)
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  const uint4* s = p + g * 32;
  uint32_t acc = 0;
#pragma unroll 4
  for (int i = 0; i < 32; i++) { uint4 v = s[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  out[g] = acc;
}
__global__ void kB(const uint4* p, uint32_t* out) {  // wave = 64 shares, staged 64 B per step
  const long wave = ((long)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  uint32_t acc = 0;
  for (int st = 0; st < 8; st++)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const long share = wave * 64 + (lane >> 2) + 16 * j;
      uint4 v = p[share * 32 + 4 * st + (lane & 3)];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  out[(long)blockIdx.x * 256 + threadIdx.x] = acc;
}
__global__ void kC(const uint32_t* p, uint32_t* out, long nvec) {  // 128 lanes x 4 B = 512 B rows
  const long g = (long)blockIdx.x * 128 + threadIdx.x;
  const uint32_t* s = p + (long)blockIdx.x * 128 * 64 + threadIdx.x;
  uint32_t acc = 0;
#pragma unroll 8
  for (int i = 0; i < 64; i++) acc ^= s[i * 128];
  out[g] = acc;
}
__global__ void kD(const uint4* p, uint32_t* out) {
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  const long n = (long)gridDim.x * 256;
  uint32_t acc = 0;
  for (int i = 0; i < 32; i++) { uint4 v = p[g + i * n]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  out[g] = acc;
}

int main() {
  const size_t bytes = 2ull << 30;
  uint4* p;
  uint32_t* out;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&out, bytes / 64) != hipSuccess) return 1;
  hipMemset(p, 1, bytes);
  const long shares = bytes / 512;
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(kA, dim3(shares / 256), dim3(256), 0, 0, p, out);
    hipLaunchKernelGGL(kB, dim3(shares / 256), dim3(256), 0, 0, p, out);
    hipLaunchKernelGGL(kC, dim3(bytes / 4 / (128 * 64)), dim3(128), 0, 0, (const uint32_t*)p, out, 0L);
    hipLaunchKernelGGL(kD, dim3(bytes / 16 / 32 / 256), dim3(256), 0, 0, p, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("read %zu bytes per kernel launch\n", bytes);
  return 0;
}
