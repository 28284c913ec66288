// repair.hip -- device helpers for rsmt2d ExtendedDataSquare.Repair (v0.11.0):
// axis completeness, root verification and status mapping.  The decode itself
// is rs_decode.hip; the crossword schedule is driven from dagpu.cpp.
//
// Reference semantics: prerepairSanityCheck rejects a complete
// axis whose root differs from the given one ("bad root input") or whose parity
// differs from Encode(data) (ErrByzantineData); solveCrossword rebuilds axes
// with >= k shares and rejects a rebuilt axis whose root differs
// (ErrByzantineData); no progress -> ErrUnrepairableDataSquare.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dagpu.h"
#include "kernels.hpp"

namespace dagpu {

// Axis arrays are laid out [axis][square][idx] (rows block, then columns block)
// so each block doubles as the per-vector flag array of that axis' encode pass.
__device__ __forceinline__ void axis_of(long a, int w, long nsq, long& sq, int& axis, int& idx) {
  axis = (int)(a / (nsq * w));
  const long rem = a - (long)axis * nsq * w;
  sq = rem / w;
  idx = (int)(rem % w);
}

// one wave per axis: complete[axis][sq][idx]
__global__ __launch_bounds__(64) void axis_complete_kernel(const uint8_t* present, int k, long nsq,
                                                            int32_t* complete) {
  const long a = blockIdx.x;
  const int w = 2 * k;
  long sq;
  int axis, idx;
  axis_of(a, w, nsq, sq, axis, idx);
  const uint8_t* p = present + sq * (long)w * w;
  int missing = 0;
  for (int j = threadIdx.x; j < w; j += 64) {
    const long cell = axis == 0 ? (long)idx * w + j : (long)j * w + idx;
    missing |= p[cell] == 0;
  }
  missing = __any(missing);
  if (threadIdx.x == 0) complete[a] = missing ? 0 : 1;
}

hipError_t launch_axis_complete(const uint8_t* present, int k, long nsq, int32_t* complete,
                                hipStream_t s) {
  const long n = nsq * 4L * k;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(axis_complete_kernel, dim3((unsigned)n), dim3(64), 0, s, present, k, nsq, complete);
  return hipGetLastError();
}

// one thread per axis: compare 90-B roots of axes complete after the crossword
__global__ __launch_bounds__(256) void verify_roots_kernel(const uint8_t* exp_rr, const uint8_t* exp_cr,
                                                           const uint8_t* got_rr, const uint8_t* got_cr,
                                                           const int32_t* complete_now,
                                                           const int32_t* complete_before, int k,
                                                           long nsq, int32_t* bits, int32_t* root_bad) {
  const long a = (long)blockIdx.x * 256 + threadIdx.x;
  const int w = 2 * k;
  if (a >= nsq * 2L * w) return;
  long sq;
  int axis, idx;
  axis_of(a, w, nsq, sq, axis, idx);
  root_bad[a] = 0;
  if (!complete_now[a]) {
    atomicOr(&bits[sq], kRepIncomplete);
    return;
  }
  const long off = (sq * w + idx) * kNodeSize;
  const uint16_t* e16 = (const uint16_t*)((axis == 0 ? exp_rr : exp_cr) + off);
  const uint16_t* g16 = (const uint16_t*)((axis == 0 ? got_rr : got_cr) + off);
  uint32_t diff = 0;
#pragma unroll
  for (int h = 0; h < kNodeSize / 2; h++) diff |= (uint32_t)(e16[h] ^ g16[h]);
  if (!diff) return;
  if (complete_before[a]) root_bad[a] = 1;  // untouched by the crossword: pre-repair check
  else atomicOr(&bits[sq], kRepByz);
}

hipError_t launch_verify_roots(const uint8_t* exp_rr, const uint8_t* exp_cr, const uint8_t* got_rr,
                               const uint8_t* got_cr, const int32_t* complete_now,
                               const int32_t* complete_before, int k, long nsq, int32_t* bits,
                               int32_t* root_bad, hipStream_t s) {
  const long n = nsq * 4L * k;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(verify_roots_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, exp_rr,
                     exp_cr, got_rr, got_cr, complete_now, complete_before, k, nsq, bits, root_bad);
  return hipGetLastError();
}

// One workgroup per square.  prerepairSanityCheck first: rsmt2d v0.11.0 runs
// its per-axis checks concurrently (errgroup) and returns whichever fails
// first in time; here the first in launch order wins -- for i = 0..2k-1: row i
// root, col i root, row i parity, col i parity (key = 4i + check) -- which the
// oracle (orc_repair) follows too.  A root failure is "bad root input: <axis>
// <i>", a parity failure ErrByzantineData{axis, i, that axis' shares}.  Then
// the crossword: a failing rebuilt axis (kRepByz) is ErrByzantineData whose
// axis and index the host resolves in rsmt2d's sequential order (dagpu.cpp
// exact_repair); then "no progress" (ErrUnrepairableDataSquare).
__global__ __launch_bounds__(256) void finalize_repair_kernel(const int32_t* bits, const int32_t* complete_before,
                                                              const int32_t* root_bad, const int32_t* parity_bad,
                                                              int k, long nsq, int32_t* status, int32_t* byz) {
  __shared__ int key_s;
  const long sq = blockIdx.x;
  const int w = 2 * k;
  if (threadIdx.x == 0) key_s = 0x7fffffff;
  __syncthreads();
  int key = 0x7fffffff;
  for (int i = threadIdx.x; i < w; i += 256) {
    const long r = sq * w + i, c = (nsq + sq) * w + i;  // [axis][square][idx]
    int kk = 0x7fffffff;
    if (complete_before[c] && parity_bad[c]) kk = 4 * i + 3;
    if (complete_before[r] && parity_bad[r]) kk = 4 * i + 2;
    if (root_bad[c]) kk = 4 * i + 1;
    if (root_bad[r]) kk = 4 * i;
    key = key < kk ? key : kk;
  }
  atomicMin(&key_s, key);
  __syncthreads();
  if (threadIdx.x != 0) return;
  const int b = bits[sq];
  int st = DAGPU_OK, ax = -1, ix = -1;
  if (key_s != 0x7fffffff) {
    st = (key_s & 3) < 2 ? DAGPU_ERR_BAD_ROOTS : DAGPU_ERR_BYZANTINE;
    ax = key_s & 1;
    ix = key_s >> 2;
  } else if (b & kRepByz) {
    st = DAGPU_ERR_BYZANTINE;
  } else if (b & kRepIncomplete) {
    st = DAGPU_ERR_UNREPAIRABLE;
  }
  status[sq] = st;
  if (byz) {
    byz[4 * sq + 0] = ax;
    byz[4 * sq + 1] = ix;
    byz[4 * sq + 2] = ax;
    byz[4 * sq + 3] = ix;
  }
}

hipError_t launch_finalize_repair(const int32_t* bits, const int32_t* complete_before, const int32_t* root_bad,
                                  const int32_t* parity_bad, int k, long nsq, int32_t* status, int32_t* byz,
                                  hipStream_t s) {
  if (nsq <= 0) return hipSuccess;
  hipLaunchKernelGGL(finalize_repair_kernel, dim3((unsigned)nsq), dim3(256), 0, s, bits, complete_before,
                     root_bad, parity_bad, k, nsq, status, byz);
  return hipGetLastError();
}

}  // namespace dagpu
