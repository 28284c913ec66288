// d2h_probe.hip -- which device->host copy path does HIP take for each kind
// of host memory, and does it steal CUs from a concurrent kernel?
// (the single-square EDS download ran as
// __amd_rocclr_copyBuffer blit kernels that stretched the NMT kernels.)
//
// For each host-memory kind: D2H of `mb` MiB alone, a CU-filling busy kernel
// alone, then both at once on two streams; prints the elapsed times.  Run
// under `rocprofv3 --kernel-trace --stats` to see which kinds spawn blit
// kernels (copyBuffer) instead of using the SDMA engines.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

// every lane spins ~`iters` dependent integer ops: a stand-in for the leaf kernel
__global__ __launch_bounds__(256) void busy_kernel(uint32_t* out, int iters) {
  uint32_t x = threadIdx.x * 2654435761u + blockIdx.x;
  for (int i = 0; i < iters; i++) x = (x << 7 | x >> 25) + 0x9e3779b9u * (x ^ i);
  if (x == 0x12345678u) out[blockIdx.x] = x;  // never true in practice; keeps x live
}

struct Kind {
  const char* name;
  void* p;
  bool reg;
};

int main(int argc, char** argv) {
  const size_t mb = argc > 1 ? (size_t)atol(argv[1]) : 16;
  const int iters = argc > 2 ? atoi(argv[2]) : 40000;
  const size_t bytes = mb << 20;
  printf("HSA_ENABLE_SDMA=%s bytes=%zu\n", getenv("HSA_ENABLE_SDMA") ? getenv("HSA_ENABLE_SDMA") : "(unset)", bytes);
  void* d_src;
  uint32_t* d_out;
  CK(hipMalloc(&d_src, bytes));
  CK(hipMalloc(&d_out, 1 << 20));
  CK(hipMemset(d_src, 0x5a, bytes));
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  hipEvent_t a0, a1, b0, b1;
  CK(hipEventCreate(&a0));
  CK(hipEventCreate(&a1));
  CK(hipEventCreate(&b0));
  CK(hipEventCreate(&b1));

  Kind kinds[6];
  int nk = 0;
  void* p;
  CK(hipHostMalloc(&p, bytes, hipHostMallocDefault));
  kinds[nk++] = {"hipHostMalloc(Default)", p, false};
  CK(hipHostMalloc(&p, bytes, hipHostMallocNonCoherent));
  kinds[nk++] = {"hipHostMalloc(NonCoherent)", p, false};
  CK(hipHostMalloc(&p, bytes, hipHostMallocCoherent));
  kinds[nk++] = {"hipHostMalloc(Coherent)", p, false};
  p = aligned_alloc(4096, bytes);
  memset(p, 0, bytes);
  CK(hipHostRegister(p, bytes, hipHostRegisterDefault));
  kinds[nk++] = {"malloc+hipHostRegister", p, true};
  p = aligned_alloc(4096, bytes);
  memset(p, 0, bytes);
  kinds[nk++] = {"pageable", p, false};

  const int blocks = 256 * 8;
  for (int r = 0; r < 2; r++) {  // round 0 warms up
    for (int i = 0; i < nk; i++) {
      float t_copy = 0, t_busy = 0, t_copy_c = 0, t_busy_c = 0;
      // copy alone
      CK(hipEventRecord(b0, sb));
      CK(hipMemcpyAsync(kinds[i].p, d_src, bytes, hipMemcpyDeviceToHost, sb));
      CK(hipEventRecord(b1, sb));
      CK(hipStreamSynchronize(sb));
      CK(hipEventElapsedTime(&t_copy, b0, b1));
      // busy alone
      CK(hipEventRecord(a0, sa));
      hipLaunchKernelGGL(busy_kernel, dim3(blocks), dim3(256), 0, sa, d_out, iters);
      CK(hipEventRecord(a1, sa));
      CK(hipStreamSynchronize(sa));
      CK(hipEventElapsedTime(&t_busy, a0, a1));
      // both: the busy kernel first, the copy right behind it on the other stream
      CK(hipEventRecord(a0, sa));
      hipLaunchKernelGGL(busy_kernel, dim3(blocks), dim3(256), 0, sa, d_out, iters);
      CK(hipEventRecord(a1, sa));
      CK(hipEventRecord(b0, sb));
      CK(hipMemcpyAsync(kinds[i].p, d_src, bytes, hipMemcpyDeviceToHost, sb));
      CK(hipEventRecord(b1, sb));
      CK(hipDeviceSynchronize());
      CK(hipEventElapsedTime(&t_busy_c, a0, a1));
      CK(hipEventElapsedTime(&t_copy_c, b0, b1));
      if (r == 1)
        printf("%-28s copy %.3f ms (%.1f GB/s) | busy %.3f ms | concurrent: busy %.3f ms, copy %.3f ms\n",
               kinds[i].name, t_copy, bytes / (t_copy * 1e-3) / 1e9, t_busy, t_busy_c, t_copy_c);
    }
  }
  // also H2D from each kind (the upload side of the single-square call)
  for (int i = 0; i < nk; i++) {
    float t = 0;
    for (int r = 0; r < 2; r++) {
      CK(hipEventRecord(b0, sb));
      CK(hipMemcpyAsync(d_src, kinds[i].p, bytes, hipMemcpyHostToDevice, sb));
      CK(hipEventRecord(b1, sb));
      CK(hipStreamSynchronize(sb));
      CK(hipEventElapsedTime(&t, b0, b1));
    }
    printf("%-28s H2D %.3f ms (%.1f GB/s)\n", kinds[i].name, t, bytes / (t * 1e-3) / 1e9);
  }
  return 0;
}
