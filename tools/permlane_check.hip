// permlane_check.hip -- prints the lane mapping of v_permlane16_swap /
// v_permlane32_swap and DPP row_ror:8 on gfx950 (used by the bit-sliced encoder).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
__global__ void k(uint32_t* o) {
  const uint32_t l = threadIdx.x;
  uint32_t a = l, b = 100 + l;
  auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  auto s = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  uint32_t d = __builtin_amdgcn_update_dpp(0u, a, 0x128, 0xF, 0xF, false);
  o[l] = r[0]; o[64 + l] = r[1]; o[128 + l] = s[0]; o[192 + l] = s[1]; o[256 + l] = d;
}
int main() {
  uint32_t* d; (void)hipMalloc(&d, 320 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  uint32_t h[320]; (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  const char* nm[5] = {"pl32.a", "pl32.b", "pl16.a", "pl16.b", "ror8"};
  for (int t = 0; t < 5; t++) { printf("%s:", nm[t]); for (int i = 0; i < 64; i++) printf(" %u", h[t * 64 + i]); printf("\n"); }
  return 0;
}
