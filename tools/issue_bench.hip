// issue_bench.hip -- VALU issue cost per opcode on gfx950, in shader clocks,
// as a function of waves per SIMD.  Each wave runs 16 independent register
// chains of ONE opcode (inline asm, so the instruction count is exact) and
// stamps s_memtime / s_memrealtime around the loop; the in-kernel clock is
// d(memtime)/d(memrealtime) x 100 MHz (MI355X_MICROARCH.md 'DVFS give-back' 6).
// Output per (op, waves/SIMD): cycles per instruction per wave and the SIMD's
// instruction throughput = waves / that.  Used to pick instruction forms for the
// SHA-256 and GF(2^8) kernels (DESIGN.md "Issue costs").
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/issue_bench.hip -o tools/issue_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
#define S(x) #x
#define ALIGNBIT(i) "v_alignbit_b32 %" S(i) ", %" S(i) ", %16, 7\n"
#define ALIGNSELF(i) "v_alignbit_b32 %" S(i) ", %" S(i) ", %" S(i) ", 7\n"
#define BITOP3(i) "v_bitop3_b32 %" S(i) ", %" S(i) ", %16, %17 bitop3:0x96\n"
#define XOR(i) "v_xor_b32 %" S(i) ", %" S(i) ", %16\n"
#define ADD(i) "v_add_u32 %" S(i) ", %" S(i) ", %16\n"
#define ADD3(i) "v_add3_u32 %" S(i) ", %" S(i) ", %16, %17\n"
#define PERM(i) "v_perm_b32 %" S(i) ", %" S(i) ", %16, %17\n"
#define LSHR(i) "v_lshrrev_b32 %" S(i) ", 3, %" S(i) "\n"
#define AND(i) "v_and_b32 %" S(i) ", %16, %" S(i) "\n"
#define LSHLOR(i) "v_lshl_or_b32 %" S(i) ", %" S(i) ", 7, %16\n"
#define XAD(i) "v_xad_u32 %" S(i) ", %" S(i) ", %16, %17\n"
#define OR3(i) "v_or3_b32 %" S(i) ", %" S(i) ", %16, %17\n"
#define MOV(i) "v_mov_b32 %" S(i) ", %16\n"
#define AND_E64(i) "v_and_b32_e64 %" S(i) ", %16, %" S(i) "\n"
#define BFE(i) "v_bfe_u32 %" S(i) ", %" S(i) ", 3, 8\n"
#define PKADD16(i) "v_pk_add_u16 %" S(i) ", %" S(i) ", %16\n"
#define MIX_PB(i) "v_perm_b32 %" S(i) ", %" S(i) ", %16, %17\nv_bitop3_b32 %" S(i) ", %" S(i) ", %16, %17 bitop3:0x96\n"
#define MIX_AX(i) "v_alignbit_b32 %" S(i) ", %" S(i) ", %16, 7\nv_xor_b32 %" S(i) ", %" S(i) ", %16\n"
#define MIX_AB(i) "v_alignbit_b32 %" S(i) ", %" S(i) ", %16, 7\nv_bitop3_b32 %" S(i) ", %" S(i) ", %16, %17 bitop3:0x96\n"
#define MIX_PX(i) "v_perm_b32 %" S(i) ", %" S(i) ", %16, %17\nv_xor_b32 %" S(i) ", %" S(i) ", %16\n"

#define P8(X) X(0, 8) X(1, 9) X(2, 10) X(3, 11) X(4, 12) X(5, 13) X(6, 14) X(7, 15)
#define Q4(X) X(0, 4, 8, 12) X(1, 5, 9, 13) X(2, 6, 10, 14) X(3, 7, 11, 15)
// independent mixes: the slow op and the fast op(s) work on different chains
#define PB_IND2(i, j) "v_perm_b32 %" S(i) ", %" S(i) ", %16, %17\nv_bitop3_b32 %" S(j) ", %" S(j) ", %16, %17 bitop3:0x96\n"
#define MIX_PB_IND(i) PB_IND2(i, i)
#define AX_IND2(i, j) "v_alignbit_b32 %" S(i) ", %" S(i) ", %16, 7\nv_xor_b32 %" S(j) ", %" S(j) ", %16\n"
#define S1F3(a, b, c, d) "v_alignbit_b32 %" S(a) ", %" S(a) ", %16, 7\nv_xor_b32 %" S(b) ", %" S(b) ", %16\nv_add_u32 %" S(c) ", %" S(c) ", %16\nv_bitop3_b32 %" S(d) ", %" S(d) ", %16, %17 bitop3:0x96\n"
#define S2F2(a, b, c, d) "v_alignbit_b32 %" S(a) ", %" S(a) ", %16, 7\nv_xor_b32 %" S(b) ", %" S(b) ", %16\nv_perm_b32 %" S(c) ", %" S(c) ", %16, %17\nv_bitop3_b32 %" S(d) ", %" S(d) ", %16, %17 bitop3:0x96\n"
#define S1F1_4(a, b, c, d) "v_alignbit_b32 %" S(a) ", %" S(a) ", %16, 7\nv_xor_b32 %" S(b) ", %" S(b) ", %16\nv_alignbit_b32 %" S(c) ", %" S(c) ", %16, 7\nv_bitop3_b32 %" S(d) ", %" S(d) ", %16, %17 bitop3:0x96\n"

#define PL32_2(i, j) "v_permlane32_swap_b32 %" S(i) ", %" S(j) "\n"
#define PL16_2(i, j) "v_permlane16_swap_b32 %" S(i) ", %" S(j) "\n"
#define DPPXOR(i) "v_xor_b32_dpp %" S(i) ", %16, %" S(i) " row_ror:8 row_mask:0xf bank_mask:0xf\n"
#define CNDDPP(i) "v_cndmask_b32_dpp %" S(i) ", %16, %" S(i) ", vcc row_ror:8 row_mask:0xf bank_mask:0xf\n"
#define BODY_S1F7 ALIGNBIT(0) XOR(1) ADD(2) BITOP3(3) XOR(4) AND(5) ADD(6) XOR(7) ALIGNBIT(8) XOR(9) ADD(10) BITOP3(11) XOR(12) AND(13) ADD(14) XOR(15)
#define BODY_S1F15 ALIGNBIT(0) XOR(1) ADD(2) BITOP3(3) XOR(4) AND(5) ADD(6) XOR(7) LSHR(8) XOR(9) ADD(10) BITOP3(11) XOR(12) AND(13) ADD(14) XOR(15)
#define BODY_PL32 P8(PL32_2) P8(PL32_2)
#define BODY_PL16 P8(PL16_2) P8(PL16_2)
#define BODY_DPPXOR R16(DPPXOR)
#define BODY_CNDDPP R16(CNDDPP)
#define BODY_FASTMIX XOR(0) ADD(1) BITOP3(2) LSHR(3) AND(4) XOR(5) BITOP3(6) ADD(7) XOR(8) ADD(9) BITOP3(10) LSHR(11) AND(12) XOR(13) BITOP3(14) ADD(15)
#define BODY_BSMIX BITOP3(0) BITOP3(1) XOR(2) BITOP3(3) DPPXOR(4) BITOP3(5) XOR(6) BITOP3(7) BITOP3(8) BITOP3(9) XOR(10) BITOP3(11) LSHR(12) BITOP3(13) XOR(14) BITOP3(15)

#define OPS(X)                                                                                 \
  X(ALIGNBIT, 1) X(ALIGNSELF, 1) X(BITOP3, 1) X(XOR, 1) X(ADD, 1) X(ADD3, 1) X(PERM, 1)        \
  X(LSHR, 1) X(AND, 1) X(LSHLOR, 1) X(XAD, 1) X(OR3, 1) X(MOV, 1) X(AND_E64, 1) X(BFE, 1)      \
  X(PKADD16, 1) X(MIX_PB, 2) X(MIX_AX, 2) X(MIX_AB, 2) X(MIX_PX, 2) \
  X(PB_IND, 2) X(AX_IND, 2) X(S1F3, 4) X(S2F2, 4) X(S1F1, 4) \
  X(S1F7, 1) X(S1F15, 1) X(PL32, 1) X(PL16, 1) X(DPPXOR, 1) X(CNDDPP, 1) X(FASTMIX, 1) X(BSMIX, 1)

#define BODY_ALIGNBIT R16(ALIGNBIT)
#define BODY_ALIGNSELF R16(ALIGNSELF)
#define BODY_BITOP3 R16(BITOP3)
#define BODY_XOR R16(XOR)
#define BODY_ADD R16(ADD)
#define BODY_ADD3 R16(ADD3)
#define BODY_PERM R16(PERM)
#define BODY_LSHR R16(LSHR)
#define BODY_AND R16(AND)
#define BODY_LSHLOR R16(LSHLOR)
#define BODY_XAD R16(XAD)
#define BODY_OR3 R16(OR3)
#define BODY_MOV R16(MOV)
#define BODY_AND_E64 R16(AND_E64)
#define BODY_BFE R16(BFE)
#define BODY_PKADD16 R16(PKADD16)
#define BODY_MIX_PB R16(MIX_PB)
#define BODY_MIX_AX R16(MIX_AX)
#define BODY_MIX_AB R16(MIX_AB)
#define BODY_MIX_PX R16(MIX_PX)
#define BODY_PB_IND P8(PB_IND2) P8(PB_IND2)
#define BODY_AX_IND P8(AX_IND2) P8(AX_IND2)
#define BODY_S1F3 Q4(S1F3) Q4(S1F3) Q4(S1F3) Q4(S1F3)
#define BODY_S2F2 Q4(S2F2) Q4(S2F2) Q4(S2F2) Q4(S2F2)
#define BODY_S1F1 Q4(S1F1_4) Q4(S1F1_4) Q4(S1F1_4) Q4(S1F1_4)

#define KERNEL(NAME, PER)                                                                      \
  __global__ __launch_bounds__(256) void k_##NAME(uint64_t* out, int iters, uint32_t seed) {   \
    uint32_t r[16];                                                                            \
    for (int i = 0; i < 16; i++) r[i] = seed ^ (threadIdx.x * 16 + i);                         \
    const uint32_t c1 = seed * 3 + 0x01020304u, c2 = 0x07060504u;                              \
    __builtin_amdgcn_s_barrier();                                                              \
    const uint64_t t0 = __builtin_amdgcn_s_memtime();                                          \
    const uint64_t q0 = __builtin_amdgcn_s_memrealtime();                                      \
    for (int it = 0; it < iters; it++) {                                                       \
      asm volatile(BODY_##NAME BODY_##NAME BODY_##NAME BODY_##NAME                                     \
                   : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),   \
                     "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), \
                     "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15])                        \
                   : "v"(c1), "v"(c2));                                                        \
    }                                                                                          \
    const uint64_t t1 = __builtin_amdgcn_s_memtime();                                          \
    const uint64_t q1 = __builtin_amdgcn_s_memrealtime();                                      \
    uint32_t acc = 0;                                                                          \
    for (int i = 0; i < 16; i++) acc ^= r[i];                                                  \
    const long wv = (long)blockIdx.x * 4 + (threadIdx.x >> 6);                                 \
    if ((threadIdx.x & 63) == 0) {                                                             \
      out[wv * 2] = t1 - t0;                                                                   \
      out[wv * 2 + 1] = (q1 - q0) | ((uint64_t)(acc == 0x12345678u) << 63);                    \
    }                                                                                          \
  }
#define DECL(NAME, PER) KERNEL(NAME, PER)
OPS(DECL)

typedef void (*kfn)(uint64_t*, int, uint32_t);

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int ncu = p.multiProcessorCount;
  uint64_t* d;
  const int maxw = 8;
  (void)hipMalloc(&d, sizeof(uint64_t) * 2 * ncu * maxw * 4);
  std::vector<uint64_t> h(2 * ncu * maxw * 4);
  struct K { const char* name; kfn f; int per; };
#define ENTRY(NAME, PER) K{#NAME, k_##NAME, PER},
  K ks[] = {OPS(ENTRY)};
  const int iters = 2000;
  for (auto& k : ks) {
    for (int w : {1, 2, 4, 8}) {
      const int blocks = ncu * w;
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, d, 50, 1u);
      hipEvent_t a, b;
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      (void)hipEventRecord(a, 0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, d, iters, 1u);
      (void)hipEventRecord(b, 0);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      (void)hipMemcpy(h.data(), d, sizeof(uint64_t) * 2 * blocks * 4, hipMemcpyDeviceToHost);
      std::vector<double> cyc, ghz;
      for (int i = 0; i < blocks * 4; i++) {
        const double c = (double)h[2 * i], q = (double)(h[2 * i + 1] & ~(1ull << 63));
        cyc.push_back(c);
        ghz.push_back(c / q * 0.1);
      }
      std::sort(cyc.begin(), cyc.end());
      std::sort(ghz.begin(), ghz.end());
      const double instr = (double)iters * 64 * k.per;
      const double cpi = cyc[cyc.size() / 2] / instr;  // median wave
      const double total = instr * blocks * 4;
      printf("{\"op\":\"%s\",\"waves_per_simd\":%d,\"cyc_per_instr_per_wave\":%.3f,"
             "\"simd_instr_per_clk\":%.3f,\"clock_ghz\":%.3f,\"chip_wave_instr_per_clk_per_cu\":%.3f}\n",
             k.name, w, cpi, w / cpi, ghz[ghz.size() / 2],
             total / (ms * 1e-3) / (ghz[ghz.size() / 2] * 1e9) / ncu);
      (void)hipEventDestroy(a);
      (void)hipEventDestroy(b);
    }
  }
  return 0;
}
