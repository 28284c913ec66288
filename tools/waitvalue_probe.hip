// Probe of the stream-ordering primitives the asynchronous Repair relies on:
// stream A waits on a 32/64-bit word (hipStreamWaitValue*), stream B (or the
// host) releases it.  Each case has a watchdog: a wait not released within
// 5 s prints HANG and the process exits (the run is a probe, not a test).
//   hipcc --offload-arch=gfx950 -O2 tools/waitvalue_probe.hip -o tools/waitvalue_probe
//   ./tools/waitvalue_probe <case>   case: sig32 sig64 dev32 host32
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <chrono>
#include <thread>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      printf("%s -> %s\n", #x, hipGetErrorString(e_));                        \
      fflush(stdout);                                                         \
      _exit(2);                                                               \
    }                                                                         \
  } while (0)

static bool wait_stream(hipStream_t s, double secs) {
  auto t0 = std::chrono::steady_clock::now();
  while (hipStreamQuery(s) == hipErrorNotReady) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > secs) return false;
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  return true;
}

int main(int argc, char** argv) {
  const char* c = argc > 1 ? argv[1] : "sig32";
  int can = 0;
  CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0));
  printf("case %s: hipDeviceAttributeCanUseStreamWaitValue = %d\n", c, can);
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  void* p = nullptr;
  const bool is64 = !strcmp(c, "sig64");
  if (!strcmp(c, "dev32")) CK(hipMalloc(&p, 8));
  else if (!strcmp(c, "host32")) CK(hipHostMalloc(&p, 8, hipHostMallocDefault));
  else CK(hipExtMallocWithFlags(&p, 8, hipMallocSignalMemory));
  CK(hipMemsetAsync(p, 0, 8, b));
  CK(hipStreamSynchronize(b));
  int* marker = nullptr;
  CK(hipHostMalloc((void**)&marker, 4, hipHostMallocDefault));
  *marker = 0;
  for (uint32_t gen = 1; gen <= 3; gen++) {
    if (is64) CK(hipStreamWaitValue64(a, p, gen, hipStreamWaitValueEq, ~0ull));
    else CK(hipStreamWaitValue32(a, p, gen, hipStreamWaitValueEq, 0xFFFFFFFFu));
    CK(hipMemsetAsync(marker, (int)gen, 1, a));  // runs once the wait has passed
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    const bool early = hipStreamQuery(a) == hipSuccess;
    if (!strcmp(c, "host32")) {
      __atomic_store_n((uint32_t*)p, gen, __ATOMIC_RELEASE);
    } else if (is64) {
      CK(hipStreamWriteValue64(b, p, gen, 0));
    } else {
      CK(hipStreamWriteValue32(b, p, gen, 0));
    }
    const bool ok = wait_stream(a, 5.0);
    printf("  gen %u: passed before release: %s, after release: %s, marker %d\n", gen, early ? "YES (bad)" : "no",
           ok ? "yes" : "HANG", ok ? (int)(*(volatile unsigned char*)marker) : -1);
    fflush(stdout);
    if (!ok) _exit(3);
  }
  printf("case %s ok\n", c);
  return 0;
}
