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
                                                            int32_t* complete, int32_t* ncomplete) {
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
  if (threadIdx.x == 0 && !missing && ncomplete) atomicAdd(ncomplete, 1);
}

// 0x80 in every byte of x that is nonzero (no carries between bytes)
__device__ __forceinline__ uint32_t nonzero_bytes_hi(uint32_t x) {
  return (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}

// Rows, w % 16 == 0 and 16-B aligned presence: L = w / 16 lanes per row, each
// one 16-B load; a row is complete when no lane of its group saw a zero byte.
__global__ __launch_bounds__(256) void axis_complete_rows_kernel(const uint8_t* present, int k, long nsq,
                                                                 int32_t* complete, int32_t* ncomplete) {
  const int w = 2 * k, L = w / 16;
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  const long nrow = nsq * w;
  const long row = t / L;  // square-major: sq * w + r
  bool zero = false;
  if (row < nrow) {
    const uint4 v = ((const uint4*)(present + row * w))[t - row * L];
    zero = (nonzero_bytes_hi(v.x) & nonzero_bytes_hi(v.y) & nonzero_bytes_hi(v.z) & nonzero_bytes_hi(v.w)) !=
           0x80808080u;
  }
  const uint64_t b = __ballot(zero);
  const int lane = threadIdx.x & 63;
  const int g = lane / L;  // L <= 64 and divides 64 (w = 16 .. 1024)
  const uint64_t m = (L == 64 ? ~0ull : ((1ull << L) - 1)) << (g * L);
  const bool done = row < nrow && lane == g * L && !(b & m);
  if (row < nrow && lane == g * L) complete[row] = done ? 1 : 0;
  const uint64_t dm = __ballot(done);
  if (ncomplete && dm && lane == 0) atomicAdd(ncomplete, (int)__popcll(dm));
}

// Columns, w % 4 == 0 and 4-B aligned presence: block = (square, 256 columns);
// lane j holds columns 4j..4j+3 (dword loads, coalesced along the row), the
// four waves take every fourth row, AND-combined in LDS.
// 16 waves split the rows of a 256-column group, 16 loads in flight per lane
// (4 waves walking all w rows one dependent load at a time took ~38 us for two
// k = 512 squares: 8 workgroups on 8 CUs)
constexpr int kColWaves = 16;
__global__ __launch_bounds__(64 * kColWaves) void axis_complete_cols_kernel(const uint8_t* present, int k, long nsq,
                                                                            int32_t* complete, int32_t* ncomplete) {
  __shared__ uint32_t acc_s[kColWaves][64];
  const int w = 2 * k;
  const int ngrp = (w + 255) / 256;
  const long sq = blockIdx.x / ngrp;
  const int grp = (int)(blockIdx.x - sq * ngrp);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = grp * 256 + 4 * lane;  // first of this lane's 4 columns
  uint32_t acc = 0x80808080u;
  if (c < w) {
    const uint8_t* p = present + sq * (long)w * w + c;
#pragma unroll 16
    for (int r = wave; r < w; r += kColWaves) acc &= nonzero_bytes_hi(*(const uint32_t*)(p + (long)r * w));
  }
  acc_s[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && c < w) {
    uint32_t all = acc_s[0][lane];
#pragma unroll
    for (int q = 1; q < kColWaves; q++) all &= acc_s[q][lane];
    int32_t* out = complete + nsq * w + sq * w + c;
    int nc = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int cj = (all >> (8 * j + 7)) & 1;
      out[j] = cj;
      nc += cj;
    }
    if (nc && ncomplete) atomicAdd(ncomplete, nc);
  }
}

hipError_t launch_axis_complete(const uint8_t* present, int k, long nsq, int32_t* complete,
                                hipStream_t s, int32_t* ncomplete) {
  const long n = nsq * 4L * k;
  if (n <= 0) return hipSuccess;
  const int w = 2 * k;
  if (w >= 16 && w <= 1024 && ((uintptr_t)present & 15) == 0) {  // L = w / 16 lanes <= 64
    const long threads = nsq * w * (w / 16);
    hipLaunchKernelGGL(axis_complete_rows_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, present,
                       k, nsq, complete, ncomplete);
    hipLaunchKernelGGL(axis_complete_cols_kernel, dim3((unsigned)(nsq * ((w + 255) / 256))), dim3(64 * kColWaves),
                       0, s, present, k, nsq, complete, ncomplete);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(axis_complete_kernel, dim3((unsigned)n), dim3(64), 0, s, present, k, nsq, complete, ncomplete);
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
                                                              int k, long nsq, int32_t* status, int32_t* byz,
                                                              int32_t* pre_fail) {
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
  if (pre_fail) pre_fail[sq] = key_s != 0x7fffffff;
  if (byz) {
    byz[4 * sq + 0] = ax;
    byz[4 * sq + 1] = ix;
    byz[4 * sq + 2] = ax;
    byz[4 * sq + 3] = ix;
  }
}

hipError_t launch_finalize_repair(const int32_t* bits, const int32_t* complete_before, const int32_t* root_bad,
                                  const int32_t* parity_bad, int k, long nsq, int32_t* status, int32_t* byz,
                                  hipStream_t s, int32_t* pre_fail) {
  if (nsq <= 0) return hipSuccess;
  hipLaunchKernelGGL(finalize_repair_kernel, dim3((unsigned)nsq), dim3(256), 0, s, bits, complete_before,
                     root_bad, parity_bad, k, nsq, status, byz, pre_fail);
  return hipGetLastError();
}

// rsmt2d returns from prerepairSanityCheck before solveCrossword: a square that
// fails it keeps its input presence (the crossword ran beside the check here).
__global__ __launch_bounds__(256) void restore_presence_kernel(uint8_t* present, const uint8_t* p0,
                                                               const int32_t* pre_fail, long per_sq, long nsq) {
  const long n4 = per_sq / 4;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  if (gid >= n4 * nsq) return;
  const long sq = gid / n4;
  if (!pre_fail[sq]) return;
  ((uint32_t*)present)[gid] = ((const uint32_t*)p0)[gid];
}

hipError_t launch_restore_presence(uint8_t* present, const uint8_t* p0, const int32_t* pre_fail, int k, long nsq,
                                   hipStream_t s) {
  const long per = 4L * k * k;  // (2k)^2 flags, a multiple of 4
  const long threads = nsq * (per / 4);
  if (threads <= 0) return hipSuccess;
  hipLaunchKernelGGL(restore_presence_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, present, p0,
                     pre_fail, per, nsq);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Repair shortcut (round 3): fill route and deferral, see kernels.hpp PlanArgs
// and dagpu.cpp repair_device.  A decode rebuilds a vector as the unique
// codeword through its >= k given shares; when its data half (indices < k) is
// complete that codeword is Encode(data half), which the fill encoder computes
// for a fraction of the decoder's work (IFFT_k + FFT_k against the decoder's
// n-point transforms and per-element multiplies).  Given shares of the parity
// half are compared, and a difference sends the vector back to the decoder, so
// every rebuilt vector gets the decoder's bytes.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int nonzero_bytes(uint32_t x) {
  const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);  // 0x80 per zero byte
  return 4 - __builtin_popcount(z);
}

constexpr int kPlanThreads = 256;

// Present shards per vector (all, and of the data half) -> flags, vec_counts,
// *ndecodable.  The layouts of the locator-key kernels (rs_gf16.hip): contiguous
// flags (p_shard_stride == 1, the row axis): 16 lanes per vector, 16 flags per
// lane load; otherwise (column axis) one lane per vector, the 2k flags split
// over the 16 waves of the block and summed in LDS.  (One lane per vector
// throughout took 0.1 ms per launch at k = 512, 2 squares: 2,048 lanes in all.)
// blk_cnt[0] += decodable, blk_cnt[1] += decodable with a complete data or
// parity half (the Repair plan's fill candidates, repair_plan_kernel's f / r)
__device__ __forceinline__ void vec_count_finish(const DecodeArgs& a, long v, int sys, int tot, int* blk_cnt) {
  const int k = a.k, n = 2 * k;
  const bool decode = tot >= k && tot < n && vec_selected(a, v);
  a.flags[v] = decode ? 1 : 0;
  if (a.vec_counts) a.vec_counts[v] = sys | (tot << 16);
  if (tot < k && a.too_few) atomicOr(a.too_few, 1);
  if (decode) atomicAdd(blk_cnt, 1);
  if (decode && (sys == k || tot - sys == k)) atomicAdd(blk_cnt + 1, 1);
}

__device__ __forceinline__ void vec_count_flush(const DecodeArgs& a, const int* blk_cnt) {
  if (threadIdx.x != 0) return;
  if (blk_cnt[0] && a.ndecodable) atomicAdd(a.ndecodable, blk_cnt[0]);
  if (blk_cnt[1] && a.nfill) atomicAdd(a.nfill, blk_cnt[1]);
}

// Rows of the presence map: 16 lanes per row (4 rows per wave) when the row's
// 16-flag loads each lie inside one half (k >= 16, aligned), one row per wave
// otherwise (a wave per row spent most of its time launching and reducing:
// 35 us for 256 k = 128 squares).
__device__ __forceinline__ void vec_count_rows_block(const DecodeArgs& a, long bid, int* blk_cnt) {
  if (threadIdx.x == 0) blk_cnt[0] = blk_cnt[1] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int k = a.k, n = 2 * k;
  const long nv = a.nsq * a.nvec;
  if (k >= 16 && ((uintptr_t)a.present & 15) == 0 && (a.p_vec_stride & 15) == 0 && (a.p_sq_stride & 15) == 0) {
    // a 16-flag load straddling index k would count parity flags as data: k >= 16
    const long v = (bid * 16 + wave) * 4 + (lane >> 4);
    const int sl = lane & 15;
    int sys = 0, tot = 0;
    if (v < nv) {
      const long sq = v / a.nvec;
      const uint4* q = (const uint4*)(a.present + sq * a.p_sq_stride + (v - sq * a.nvec) * a.p_vec_stride);
      for (int j = sl; j < n / 16; j += 16) {
        const uint4 x = q[j];
        const int c = nonzero_bytes(x.x) + nonzero_bytes(x.y) + nonzero_bytes(x.z) + nonzero_bytes(x.w);
        tot += c;
        if (16 * j < k) sys += c;
      }
    }
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) {  // within the 16-lane group
      sys += __shfl_xor(sys, off);
      tot += __shfl_xor(tot, off);
    }
    if (sl == 0 && v < nv) vec_count_finish(a, v, sys, tot, blk_cnt);
  } else {
    const long v = bid * 16 + wave;  // wave-uniform
    if (v < nv) {
      const long sq = v / a.nvec;
      const uint8_t* pres = a.present + sq * a.p_sq_stride + (v - sq * a.nvec) * a.p_vec_stride;
      int sys = 0, tot = 0;
      for (int i = lane; i < n; i += 64) {
        const int c = pres[i] != 0;
        tot += c;
        if (i < k) sys += c;
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        sys += __shfl_xor(sys, off);
        tot += __shfl_xor(tot, off);
      }
      if (lane == 0) vec_count_finish(a, v, sys, tot, blk_cnt);
    }
  }
  __syncthreads();
  vec_count_flush(a, blk_cnt);
}

__device__ __forceinline__ void vec_count_cols_block(const DecodeArgs& a, long bid, int* blk_cnt, int* acc_sys,
                                                     int* acc_tot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long nb = (a.nvec + 63) / 64;
  const long sq = bid / nb;
  const long vec = (bid - sq * nb) * 64 + lane;
  if (threadIdx.x < 64) acc_sys[threadIdx.x] = acc_tot[threadIdx.x] = 0;
  if (threadIdx.x == 0) blk_cnt[0] = blk_cnt[1] = 0;
  __syncthreads();
  const int k = a.k, n = 2 * k;
  if (vec < a.nvec) {
    const uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
    int sys = 0, tot = 0;
#pragma unroll 8
    for (int i = wave; i < n; i += 16) {
      const int c = pres[(long)i * a.p_shard_stride] != 0;
      tot += c;
      if (i < k) sys += c;
    }
    if (sys) atomicAdd(&acc_sys[lane], sys);
    if (tot) atomicAdd(&acc_tot[lane], tot);
  }
  __syncthreads();
  if (wave == 0 && vec < a.nvec) vec_count_finish(a, sq * a.nvec + vec, acc_sys[lane], acc_tot[lane], blk_cnt);
  __syncthreads();
  vec_count_flush(a, blk_cnt);
}

// the 4-rows-per-wave layout of vec_count_rows_block (same condition as the block's)
static bool vec_rows_packed(const DecodeArgs& a) {
  return a.k >= 16 && ((uintptr_t)a.present & 15) == 0 && (a.p_vec_stride & 15) == 0 && (a.p_sq_stride & 15) == 0;
}
static long vec_count_blocks(const DecodeArgs& a) {
  const long nv = a.nsq * a.nvec;
  if (nv <= 0) return 0;
  if (a.p_shard_stride == 1) return vec_rows_packed(a) ? (nv + 63) / 64 : (nv + 15) / 16;
  return a.nsq * ((a.nvec + 63) / 64);
}

__device__ __forceinline__ void vec_count_block(const DecodeArgs& a, long bid, int* blk_cnt, int* acc_sys,
                                                int* acc_tot) {
  if (a.p_shard_stride == 1) vec_count_rows_block(a, bid, blk_cnt);
  else vec_count_cols_block(a, bid, blk_cnt, acc_sys, acc_tot);
}

__global__ __launch_bounds__(1024) void vec_count_kernel(DecodeArgs a) {
  __shared__ int blk_cnt[2];
  __shared__ int acc_sys[64], acc_tot[64];
  vec_count_block(a, blockIdx.x, blk_cnt, acc_sys, acc_tot);
}

hipError_t launch_vec_count(const DecodeArgs& a, hipStream_t s) {
  const long nb = vec_count_blocks(a);
  if (nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(vec_count_kernel, dim3((unsigned)nb), dim3(1024), 0, s, a);
  return hipGetLastError();
}

// Both axes of a Repair round in one launch (blocks [0, nb0) count axis a0,
// the rest a1), plus the round's counter bookkeeping (see RoundCounters):
// block 0 moves the previous plan's deferral count to its read slot and clears
// the plan's counters, and the last block to finish copies the counters to the
// host mailbox, so the host's read needs no copy of its own.
__global__ __launch_bounds__(1024) void vec_count_round_kernel(DecodeArgs a0, DecodeArgs a1, long nb0,
                                                               RoundCounters rc) {
  __shared__ int blk_cnt[2];
  __shared__ int acc_sys[64], acc_tot[64];
  __shared__ int last_s;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    atomicExch(rc.ctr + kCtrDeferredPrev, atomicExch(rc.ctr + kCtrDeferred, 0));
    atomicExch(rc.ctr + kCtrPairs, 0);
    atomicExch(rc.ctr + kCtrPairsRev, 0);
  }
  if ((long)blockIdx.x < nb0) vec_count_block(a0, blockIdx.x, blk_cnt, acc_sys, acc_tot);
  else vec_count_block(a1, blockIdx.x - nb0, blk_cnt, acc_sys, acc_tot);
  if (!rc.host) return;  // uniform
  if (threadIdx.x == 0) {
    // This thread's counter atomics are performed (their completion waited
    // for) before its ticket; no fence: an agent-scope fence here writes back
    // and invalidates the XCD's L2 in every block (2x the launch's time at
    // 2,048 blocks).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last_s = atomicAdd(rc.ctr + kCtrTicket, 1) == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (!last_s || threadIdx.x != 0) return;
  for (int i = 0; i < kCtrRead; i++) rc.host[i] = atomicAdd(rc.ctr + i, 0);
  atomicExch(rc.ctr + kCtrTicket, 0);
  __threadfence_system();  // the counters before the sequence number
  ((volatile int32_t*)rc.host)[kCtrRead] = rc.seq;
}

hipError_t launch_vec_count_round(const DecodeArgs& a0, const DecodeArgs& a1, const RoundCounters& rc,
                                  hipStream_t s) {
  const long nb0 = vec_count_blocks(a0), nb1 = vec_count_blocks(a1);
  if (nb0 + nb1 <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(vec_count_round_kernel, dim3((unsigned)(nb0 + nb1)), dim3(1024), 0, s, a0, a1, nb0, rc);
  return hipGetLastError();
}

__global__ __launch_bounds__(kPlanThreads) void repair_plan_kernel(PlanArgs p) {
  __shared__ int low_ok;
  __shared__ int nfill_s[kPlanThreads], nrev_s[kPlanThreads];
  __shared__ int base_s, rbase_s, total_s, rtotal_s;
  const long sq = blockIdx.x;
  const int k = p.k, w = 2 * k;
  if (threadIdx.x == 0) low_ok = 1;
  __syncthreads();
  // vectors i = threadIdx.x + 256 m, any w
  for (int i = threadIdx.x; i < k; i += kPlanThreads) {
    const int32_t c = p.counts[sq * w + i];
    if (!p.flags[sq * w + i] && (c >> 16) != w) low_ok = 0;
  }
  __syncthreads();
  const bool defer = low_ok && !p.nodefer[sq];
  int nf = 0, nr = 0, nd = 0;
  const long ax0 = (long)p.axis * p.nsq * w + sq * w;  // [axis][sq][idx]
  for (int i = threadIdx.x; i < w; i += kPlanThreads) {
    const long v = sq * w + i;
    const int32_t c = p.counts[v];
    const int sys = c & 0xFFFF, tot = c >> 16;
    const bool dec = p.flags[v] != 0;
    // forward fill: data half complete; reverse fill: parity half complete
    const bool f = dec && sys == k;
    const bool r = dec && !f && tot - sys == k;
    p.fill[v] = f ? 1 : (r ? 2 : 0);
    if (f || r) {
      p.flags[v] = 0;
      p.known[ax0 + i] = 1;
      if (f) nf++;
      else nr++;
    } else if (dec) {
      if (defer && i >= k) {
        p.flags[v] = 0;
        p.deferred[ax0 + i] = 1;
        nd++;
      } else {
        p.known[ax0 + i] = tot == k;
      }
    }
  }
  if (nd) atomicAdd(p.ndeferred, nd);
  if (p.nplan) {
    int ndec = 0;
    for (int i = threadIdx.x; i < w; i += kPlanThreads) ndec += p.flags[sq * w + i] != 0;
    if (nf) atomicAdd(p.nplan + 0, nf);
    if (nr) atomicAdd(p.nplan + 1, nr);
    if (ndec) atomicAdd(p.nplan + 2, ndec);
  }
  if (!p.pair_list) return;
  // pair lists: the square's forward fills in pairs, its reverse fills in
  // pairs in the second list; an odd one is paired with -1
  nfill_s[threadIdx.x] = nf;
  nrev_s[threadIdx.x] = nr;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0, racc = 0;
    for (int t = 0; t < kPlanThreads; t++) {
      const int c = nfill_s[t], rc = nrev_s[t];
      nfill_s[t] = acc;
      nrev_s[t] = racc;
      acc += c;
      racc += rc;
    }
    total_s = acc;
    rtotal_s = racc;
    base_s = acc ? atomicAdd(p.pair_count, (acc + 1) / 2) : 0;
    rbase_s = racc ? atomicAdd(p.pair_count_rev, (racc + 1) / 2) : 0;
  }
  __syncthreads();
  int32_t* out = p.pair_list + 2L * base_s;
  int32_t* rout = p.pair_list_rev + 2L * rbase_s;
  int o = nfill_s[threadIdx.x], ro = nrev_s[threadIdx.x];
  for (int i = threadIdx.x; i < w; i += kPlanThreads) {
    const int32_t fv = p.fill[sq * w + i];
    if (fv == 1) out[o++] = (int32_t)(sq * w + i);
    else if (fv == 2) rout[ro++] = (int32_t)(sq * w + i);
  }
  if (threadIdx.x == 0 && (total_s & 1)) out[total_s] = -1;
  if (threadIdx.x == 0 && (rtotal_s & 1)) rout[rtotal_s] = -1;
}

hipError_t launch_repair_plan(const PlanArgs& p, hipStream_t s) {
  if (p.nsq <= 0) return hipSuccess;
  hipLaunchKernelGGL(repair_plan_kernel, dim3((unsigned)p.nsq), dim3(kPlanThreads), 0, s, p);
  return hipGetLastError();
}

// One workgroup per square: the deferred axes need a codeword check unless
// every row and every column < k is known to be a codeword (then the square is
// G A G^T: every column is one) or every column and every row < k is.
__global__ __launch_bounds__(256) void repair_defer_check_kernel(int32_t* deferred, const int32_t* known, int k,
                                                                  long nsq, int32_t* check, int32_t* nleft) {
  __shared__ int any_def, rows_all, cols_low, cols_all, rows_low;
  const long sq = blockIdx.x;
  const int w = 2 * k;
  if (threadIdx.x == 0) {
    any_def = 0;
    rows_all = cols_low = cols_all = rows_low = 1;
    check[sq] = 0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < w; i += 256) {
    const long r = sq * w + i, c = (nsq + sq) * w + i;
    if (deferred[r] || deferred[c]) any_def = 1;
    if (!known[r]) { rows_all = 0; if (i < k) rows_low = 0; }
    if (!known[c]) { cols_all = 0; if (i < k) cols_low = 0; }
  }
  __syncthreads();
  if (!any_def) return;
  if (!((rows_all && cols_low) || (cols_all && rows_low))) {
    if (threadIdx.x == 0 && nleft) atomicAdd(nleft, 1);  // this square's marks stay for the compare
    return;
  }
  for (int i = threadIdx.x; i < w; i += 256) {
    deferred[sq * w + i] = 0;
    deferred[(nsq + sq) * w + i] = 0;
  }
}

hipError_t launch_repair_defer_check(int32_t* deferred, const int32_t* known, int k, long nsq, int32_t* check,
                                     hipStream_t s, int32_t* nleft) {
  if (nsq <= 0) return hipSuccess;
  hipLaunchKernelGGL(repair_defer_check_kernel, dim3((unsigned)nsq), dim3(256), 0, s, deferred, known, k, nsq,
                     check, nleft);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void mark_flagged_kernel(DecodeArgs a, const int32_t* flags, int32_t* known) {
  const long v = blockIdx.x;
  if (flags[v] == 0) return;
  // a filled vector the decoder redid (a given parity shard differed): not a codeword by construction
  if (known && a.flags[v] && threadIdx.x == 0) known[v] = 0;
  const long sq = v / a.nvec, vec = v % a.nvec;
  uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
  for (int i = threadIdx.x; i < 2 * a.k; i += 256) pres[(long)i * a.p_shard_stride] = 1;
}

// The same over the whole presence map of square-major [sq][r][c] bytes, one
// dword (4 columns) per thread: a row axis marks whole dwords of flagged rows,
// a column axis ORs in the bytes of flagged columns; threads gid < nsq * w
// also do the known[] update of vector gid.  A vector is flagged in flags or
// (optional) flags2; the known[] update follows flags2 when it is given.
// zero4 (optional): four counters cleared for the next Repair round.
__global__ __launch_bounds__(256) void mark_flagged_map_kernel(DecodeArgs a, const int32_t* flags,
                                                               const int32_t* flags2, int32_t* known, int rows,
                                                               int32_t* zero4) {
  const int w = 2 * a.k, w4 = w / 4;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long nv = a.nsq * w;
  if (zero4 && gid < 4) zero4[gid] = 0;
  const int32_t* kf = flags2 ? flags2 : flags;
  if (known && gid < nv && kf[gid] && a.flags[gid]) known[gid] = 0;
  if (gid >= nv * w4) return;
  const long sq = gid / ((long)w * w4);
  const long rem = gid - sq * (long)w * w4;
  const int r = (int)(rem / w4), c = 4 * (int)(rem - (long)r * w4);
  uint32_t* p = (uint32_t*)(a.present + sq * a.p_sq_stride + (long)r * w + c);
  const int32_t* f = flags + sq * w;
  const int32_t* f2 = flags2 ? flags2 + sq * w : nullptr;
  auto flagged = [&](int i) -> bool { return f[i] || (f2 && f2[i]); };
  if (rows) {
    if (flagged(r)) *p = 0x01010101u;
  } else {
    const uint32_t set = (flagged(c) ? 0x1u : 0u) | (flagged(c + 1) ? 0x100u : 0u) |
                         (flagged(c + 2) ? 0x10000u : 0u) | (flagged(c + 3) ? 0x1000000u : 0u);
    if (set) {
      const uint32_t x = *p;
      // a flagged byte becomes exactly 1 (the decoders test presence != 0)
      uint32_t y = x;
#pragma unroll
      for (int j = 0; j < 4; j++)
        if ((set >> (8 * j)) & 1) y = (y & ~(0xFFu << (8 * j))) | (1u << (8 * j));
      *p = y;
    }
  }
}

static bool mark_map_ok(const DecodeArgs& a, bool& rows) {
  const long w = 2L * a.k;
  rows = a.p_vec_stride == w && a.p_shard_stride == 1;
  const bool cols = a.p_vec_stride == 1 && a.p_shard_stride == w;
  return a.nvec == w && w % 4 == 0 && a.p_sq_stride == w * w && (rows || cols) && ((uintptr_t)a.present & 3) == 0;
}

hipError_t launch_rs_mark_present(const DecodeArgs& a, const int32_t* flags, hipStream_t s, int32_t* known) {
  const long nv = a.nsq * a.nvec;
  if (nv <= 0) return hipSuccess;
  bool rows = false;
  if (mark_map_ok(a, rows)) {
    const long w = 2L * a.k;
    const long threads = a.nsq * w * (w / 4);
    hipLaunchKernelGGL(mark_flagged_map_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, a, flags,
                       (const int32_t*)nullptr, known, rows ? 1 : 0, (int32_t*)nullptr);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(mark_flagged_kernel, dim3((unsigned)nv), dim3(256), 0, s, a, flags, known);
  return hipGetLastError();
}

hipError_t launch_rs_mark_round(const DecodeArgs& a, const int32_t* fill, int32_t* known, int32_t* zero4,
                                hipStream_t s) {
  const long nv = a.nsq * a.nvec;
  bool rows = false;
  if (nv > 0 && mark_map_ok(a, rows)) {
    const long w = 2L * a.k;
    const long threads = a.nsq * w * (w / 4);
    hipLaunchKernelGGL(mark_flagged_map_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, a, a.flags,
                       fill, known, rows ? 1 : 0, zero4);
    return hipGetLastError();
  }
  hipError_t e = launch_rs_mark_present(a, a.flags, s, nullptr);
  if (e == hipSuccess && fill) e = launch_rs_mark_present(a, fill, s, known);
  if (e == hipSuccess && zero4) e = hipMemsetAsync(zero4, 0, 4 * sizeof(int32_t), s);
  return e;
}

}  // namespace dagpu
