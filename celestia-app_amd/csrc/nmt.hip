// nmt.hip -- batched NMT (SHA-256) row/column roots and DAH hash on gfx950.
//
// Replaces, per square:
//   * rsmt2d lazy RowRoots()/ColRoots() (pkg/da/data_availability_header.go:45-52)
//     building one ErasuredNamespacedMerkleTree per axis
//     (pkg/wrapper/nmt_wrapper.go:55-124) -> nmt v0.20.0 Push/Root with
//     NmtHasher.HashLeaf/HashNode (mirror test/util/malicious/hasher.go:186-309);
//   * DataAvailabilityHeader.Hash -> merkle.HashFromByteSlices(rows||cols)
//     (pkg/data_availability_header.go:92-108).
//
// The wrapper's namespace rule is symmetric (cell (r,c) keeps its namespace iff
// r<k && c<k, nmt_wrapper.go:103-107,138-140), so a cell's leaf node is the same
// in its row tree and its column tree.  The reference hashes every leaf twice;
// here every leaf is hashed ONCE (kernel 1), and both trees read its digest
// (kernel 2).  Bit-exact: same leaf bytes, same digest.
//
// Kernel 1 (leaves): one lane per cell; 542-B message 0x00|ns|share = 9 SHA
//   blocks; the share is streamed with 16-B loads and re-aligned into big-endian
//   message words with one v_perm_b32 per word.
// Kernel 2 (tree levels): one launch per tree level over ALL 4k trees of ALL
//   squares in the batch (thread = node), so every level runs at full lane
//   occupancy (a per-tree workgroup would idle most lanes in the last levels).
//   A node record is 48 B: digest(32) | minRef | maxRef (cell index of the Q0
//   leaf whose namespace it carries, or PARITY).  Namespace bytes are read from
//   a dense Q0 namespace table written by kernel 1.  Node ranges follow
//   HashNode with ignoreMaxNamespace=true; push order (ErrInvalidPushOrder) is
//   checked on Q0 leaves at level 1.
// Kernel 3 (DAH): one workgroup per square, RFC-6962 over 4k roots.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "kernels.hpp"
#include "nmt_node.hpp"
#include "sha256.hpp"

namespace dagpu {

// ---------------------------------------------------------------------------
// Kernel 1: leaf digests.  digest(r,c) = SHA256(0x00 | P | share), where
// P = share[0:29] if r<k && c<k else 0xFF*29 (ParitySharesNamespace).
// ---------------------------------------------------------------------------
// One lane per leaf.  The share is read one full 128-B line at a time (eight
// back-to-back 16-B loads per lane), so each line is fetched from HBM once even
// though a lane consumes it over two SHA blocks (reading 64 B per block let
// lines be evicted between the halves: +37 % FETCH_SIZE, r01).  Message block b
// needs share uint4 4b-2 .. 4b+2: line s (uint4 8s .. 8s+7) feeds blocks 2s
// and 2s+1, with two uint4 carried over.  An LDS-staged coalesced variant
// (DAGPU_LEAF_LDS) fetches the same bytes but runs ~10 % slower (occupancy).
constexpr int kLeafWave = 256;

__global__ __launch_bounds__(kLeafWave) void nmt_leaf_kernel(SquareArgs a) {
  const int k = a.k;
  const long w = 2L * k;
  const long cells = w * w;
  const long total = cells * a.nsq;
  const long gid = (long)blockIdx.x * kLeafWave + threadIdx.x;
  if (gid >= total) return;
  const long sq = gid / cells;
  const long cell = gid - sq * cells;
  const long r = cell / w, c = cell - (cell / w) * w;
  const bool q0 = (r < k) && (c < k);
  const uint4* src = (const uint4*)(a.eds + sq * a.eds_sq_stride + cell * kShareSize);
  uint32_t st[8], ns[8];
  share_leaf_sha256(src, q0, st, ns);
  if (q0) {  // dense Q0 namespace table (29 B, zero padded to 32)
    uint4* nsp = (uint4*)(a.ns_table + (sq * k * k + r * k + c) * 32);
    nsp[0] = make_uint4(ns[0], ns[1], ns[2], ns[3]);
    nsp[1] = make_uint4(ns[4], ns[5], ns[6], ns[7]);
  }
  uint4* out = (uint4*)(a.digests + gid * kDigest);
  out[0] = make_uint4(bswap32(st[0]), bswap32(st[1]), bswap32(st[2]), bswap32(st[3]));
  out[1] = make_uint4(bswap32(st[4]), bswap32(st[5]), bswap32(st[6]), bswap32(st[7]));
}

__device__ __forceinline__ void load_ns(const uint8_t* share, bool q0, uint32_t (&ns)[8]) {
  if (q0) {
    const uint4* p = (const uint4*)share;
    const uint4 v0 = p[0], v1 = p[1];
    ns[0] = v0.x; ns[1] = v0.y; ns[2] = v0.z; ns[3] = v0.w;
    ns[4] = v1.x; ns[5] = v1.y; ns[6] = v1.z; ns[7] = v1.w & 0xFFu;
  } else {
#pragma unroll
    for (int i = 0; i < 7; i++) ns[i] = 0xFFFFFFFFu;
    ns[7] = 0xFFu;
  }
}

// ---------------------------------------------------------------------------
// Kernel 2: one tree level.  Level L has per = w >> L nodes per tree; a
// square's level-L records are [row trees: w x per, tree-major][column trees:
// per x w, NODE-major], so consecutive lanes of a column level walk across
// columns and read consecutive digests / records (coalesced) just like the
// lanes of a row level walk along a row.
// ---------------------------------------------------------------------------
constexpr uint32_t kParityRef = 0xFFFFFFFFu;

__device__ __forceinline__ void ns_by_ref(const uint8_t* ns_sq, uint32_t ref, uint32_t (&ns)[8]) {
  if (ref == kParityRef) {
#pragma unroll
    for (int i = 0; i < 7; i++) ns[i] = 0xFFFFFFFFu;
    ns[7] = 0xFFu;
  } else {
    const uint4* p = (const uint4*)(ns_sq + (long)ref * 32);
    const uint4 v0 = p[0], v1 = p[1];
    ns[0] = v0.x; ns[1] = v0.y; ns[2] = v0.z; ns[3] = v0.w;
    ns[4] = v1.x; ns[5] = v1.y; ns[6] = v1.z; ns[7] = v1.w;
  }
}

// Level 1: pairs of leaves.  Leaf node = ns | ns | digest; a Q0 leaf whose
// namespace equals the parity namespace gets kParityRef (same bytes).
__device__ __forceinline__ void level_coords(long gid, int w, int per, long& sq, int& axis, int& idx, int& p) {
  const long blk = 2L * w * per;  // records of one square at this level
  sq = gid / blk;
  const long g = gid - sq * blk;
  axis = g >= (long)w * per;
  const long g2 = g - (axis ? (long)w * per : 0);
  if (axis == 0) { idx = (int)(g2 / per); p = (int)(g2 - (long)idx * per); }
  else { p = (int)(g2 / w); idx = (int)(g2 - (long)p * w); }
}

// record index of node (axis, idx, p) of square sq at a level with `per` nodes per tree
__device__ __forceinline__ long level_rec(long sq, int w, int per, int axis, int idx, int p) {
  const long base = sq * 2L * w * per;
  return axis == 0 ? base + (long)idx * per + p : base + (long)w * per + (long)p * w + idx;
}

__global__ __launch_bounds__(256) void nmt_level1_kernel(SquareArgs a, uint8_t* out_rec, int final_level) {
  const int k = a.k;
  const int w = 2 * k;
  const int half = w / 2;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = a.nsq * 2L * w * half;
  if (gid >= total) return;
  long sq;
  int axis, idx, p;
  level_coords(gid, w, half, sq, axis, idx, p);
  const uint8_t* dig = a.digests + sq * (long)w * w * kDigest;
  const uint8_t* ns_sq = a.ns_table + sq * (long)k * k * 32;
  const int j0 = 2 * p, j1 = 2 * p + 1;
  const long cell0 = axis == 0 ? (long)idx * w + j0 : (long)j0 * w + idx;
  const long cell1 = axis == 0 ? (long)idx * w + j1 : (long)j1 * w + idx;
  const bool q00 = (idx < k) && (j0 < k), q01 = (idx < k) && (j1 < k);
  // Q0 ref = r*k + c
  const uint32_t ref0 = q00 ? (axis == 0 ? (uint32_t)(idx * k + j0) : (uint32_t)(j0 * k + idx)) : kParityRef;
  const uint32_t ref1 = q01 ? (axis == 0 ? (uint32_t)(idx * k + j1) : (uint32_t)(j1 * k + idx)) : kParityRef;
  uint32_t nl[8], nr[8], dl[8], dr[8];
  ns_by_ref(ns_sq, ref0, nl);
  ns_by_ref(ns_sq, ref1, nr);
  load_digest(dig + cell0 * kDigest, dl);
  load_digest(dig + cell1 * kDigest, dr);
  if (q01) {  // nmt Push order: ns(j0) <= ns(j1) <= ns(j1+1)
    bool bad = ns_less(nr, nl);
    if (j1 + 1 < k) {
      const uint32_t ref2 = axis == 0 ? (uint32_t)(idx * k + j1 + 1) : (uint32_t)((j1 + 1) * k + idx);
      uint32_t n2[8];
      ns_by_ref(ns_sq, ref2, n2);
      bad |= ns_less(n2, nr);
    }
    if (bad) atomicOr(&a.status[sq], kStatusPushOrder);
  }
  uint32_t st[8];
  const bool lpar = ns_is_parity(nl), rpar = ns_is_parity(nr);
  if (__all(lpar && rpar)) {
    // both children of every node of this wave carry the parity namespace (3/4
    // of all nodes): the namespace words of all three blocks are constant and
    // every block runs fully unrolled so their schedule terms fold as well
    auto get = [&](int P, int i) -> uint32_t {
      return P == 2 ? dl[i] : P == 5 ? dr[i] : 0xFFFFFFFFu;
    };
    sha_node_msg<true, true, true>(get, st);
  } else if (__all(lpar)) {
    // every left leaf of this wave carries the parity namespace: the message's
    // first 56 bytes (0x01 | 0xFF*58) are constant and rounds 0..13 of block 0 fold
    auto get = [&](int P, int i) -> uint32_t {
      return P == 0 || P == 1 ? 0xFFFFFFFFu : P == 2 ? dl[i] : P == 3 || P == 4 ? nr[i] : dr[i];
    };
    sha_node_msg<true>(get, st);
  } else {
    auto get = [&](int P, int i) -> uint32_t {
      return P == 0 || P == 1 ? nl[i] : P == 2 ? dl[i] : P == 3 || P == 4 ? nr[i] : dr[i];
    };
    sha_node_msg(get, st);
  }
  uint32_t dg[8];
#pragma unroll
  for (int i = 0; i < 8; i++) dg[i] = bswap32(st[i]);
  if (final_level) {
    uint8_t* dst = (axis == 0 ? a.row_roots : a.col_roots) + (sq * w + idx) * kNodeSize;
    write_root(dst, nl, rpar ? nl : nr, dg);
  } else {
    const uint32_t lref = lpar ? kParityRef : ref0;
    const uint32_t rref = rpar ? kParityRef : ref1;
    uint4* o = (uint4*)(out_rec + gid * 48);
    o[0] = make_uint4(dg[0], dg[1], dg[2], dg[3]);
    o[1] = make_uint4(dg[4], dg[5], dg[6], dg[7]);
    o[2] = make_uint4(lref, rref == kParityRef ? lref : rref, 0u, 0u);
  }
}

// Levels >= 2: node q of tree t from records 2q, 2q+1 of the previous level.
__global__ __launch_bounds__(256) void nmt_level_kernel(SquareArgs a, const uint8_t* in_rec, uint8_t* out_rec,
                                                        int level, int final_level) {
  const int k = a.k;
  const int w = 2 * k;
  const int per = w >> level;  // nodes per tree at this level
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = a.nsq * 2L * w * per;
  if (gid >= total) return;
  long sq;
  int axis, idx, p;
  level_coords(gid, w, per, sq, axis, idx, p);
  const uint8_t* ns_sq = a.ns_table + sq * (long)k * k * 32;
  const uint4* li = (const uint4*)(in_rec + level_rec(sq, w, 2 * per, axis, idx, 2 * p) * 48);
  const uint4* ri = (const uint4*)(in_rec + level_rec(sq, w, 2 * per, axis, idx, 2 * p + 1) * 48);
  const uint4 l0 = li[0], l1 = li[1], l2 = li[2], r0 = ri[0], r1 = ri[1], r2 = ri[2];
  const uint32_t dl[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
  const uint32_t dr[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
  uint32_t lmn[8], lmx[8], rmn[8], rmx[8];
  ns_by_ref(ns_sq, l2.x, lmn);
  ns_by_ref(ns_sq, l2.y, lmx);
  ns_by_ref(ns_sq, r2.x, rmn);
  ns_by_ref(ns_sq, r2.y, rmx);
  uint32_t st[8];
  if (__all(l2.x == kParityRef && r2.x == kParityRef)) {
    // both children all-parity (3/4 of all nodes): constant namespace words in
    // all three blocks, each fully unrolled so the schedule folds too
    auto get = [&](int P, int i) -> uint32_t {
      return P == 2 ? dl[i] : P == 5 ? dr[i] : 0xFFFFFFFFu;
    };
    sha_node_msg<true, true, true>(get, st);
  } else if (__all(l2.x == kParityRef)) {
    // all-parity left children (min PARITY implies max PARITY): constant
    // 0x01 | 0xFF*58 prefix, rounds 0..13 of block 0 fold
    auto get = [&](int P, int i) -> uint32_t {
      return P <= 1 ? 0xFFFFFFFFu : P == 2 ? dl[i] : P == 3 ? rmn[i] : P == 4 ? rmx[i] : dr[i];
    };
    sha_node_msg<true>(get, st);
  } else {
    auto get = [&](int P, int i) -> uint32_t {
      return P == 0 ? lmn[i] : P == 1 ? lmx[i] : P == 2 ? dl[i] : P == 3 ? rmn[i] : P == 4 ? rmx[i] : dr[i];
    };
    sha_node_msg(get, st);
  }
  uint32_t dg[8];
#pragma unroll
  for (int i = 0; i < 8; i++) dg[i] = bswap32(st[i]);
  const bool rpar = r2.x == kParityRef;
  if (final_level) {
    uint8_t* dst = (axis == 0 ? a.row_roots : a.col_roots) + (sq * w + idx) * kNodeSize;
    if (rpar) write_root(dst, lmn, lmx, dg);
    else write_root(dst, lmn, rmx, dg);
  } else {
    uint4* o = (uint4*)(out_rec + gid * 48);
    o[0] = make_uint4(dg[0], dg[1], dg[2], dg[3]);
    o[1] = make_uint4(dg[4], dg[5], dg[6], dg[7]);
    o[2] = make_uint4(l2.x, rpar ? l2.y : r2.y, 0u, 0u);
  }
}

// ---------------------------------------------------------------------------
// Kernel 3: DAH = RFC-6962 root over rowRoots || colRoots (2w items of 90 B).
// leaf = SHA256(0x00 | root) (91 B, 2 blocks); inner = SHA256(0x01 | l | r).
// One workgroup per square.  The n = 4k leaves go through LDS in chunks of
// C = min(n, 2048): each chunk's leaf digests are reduced to the root of its
// subtree (n and C are powers of two, so every chunk is an exact subtree of
// the RFC-6962 split), the n / C subtree digests (1 up to k = 512, 32 at
// k = 16384) then to the DAH.
// ---------------------------------------------------------------------------
constexpr int kDahThreads = 1024;
constexpr int kDahChunk = 2048;

// RFC-6962 inner levels over cur digests at src (8 dwords each), ping-ponging
// with dst (cur / 2 slots); returns the buffer holding the root.
__device__ uint32_t* rfc_reduce(uint32_t* src, uint32_t* dst, int cur) {
  while (cur > 1) {
    const int next = cur / 2;
    for (int i = threadIdx.x; i < next; i += kDahThreads) {
      uint32_t m[32];
#pragma unroll
      for (int j = 0; j < 32; j++) m[j] = 0;
      uint32_t lft[8], rgt[8];
#pragma unroll
      for (int j = 0; j < 8; j++) { lft[j] = src[(2 * i) * 8 + j]; rgt[j] = src[(2 * i + 1) * 8 + j]; }
      m[0] = 0x01u;
      put_bytes<1>(m, lft);
      put_bytes<33>(m, rgt);
      m[65 >> 2] |= 0x80u << (8 * (65 & 3));
      uint32_t st[8];
      sha256_init(st);
#pragma unroll
      for (int blk = 0; blk < 2; blk++) {
        uint32_t wv[16];
#pragma unroll
        for (int j = 0; j < 16; j++) wv[j] = bswap32(m[16 * blk + j]);
        if (blk == 1) { wv[14] = 0; wv[15] = 65u * 8u; }
        sha256_compress(st, wv);
      }
#pragma unroll
      for (int j = 0; j < 8; j++) dst[i * 8 + j] = bswap32(st[j]);
    }
    __syncthreads();
    uint32_t* t = src;
    src = dst;
    dst = t;
    cur = next;
  }
  return src;
}

// RFC-6962 leaf digest of DAH item li (row roots, then column roots) of square sq
__device__ __forceinline__ void dah_leaf(const SquareArgs& a, long sq, int li, uint32_t* out) {
  const int w = 2 * a.k;
  const uint8_t* root = (li < w ? a.row_roots + (sq * w + li) * kNodeSize
                                : a.col_roots + (sq * w + (li - w)) * kNodeSize);
  // message bytes: [0]=0x00, [1..90]=root, [91]=0x80, len=728 bits
  uint32_t m[32];
#pragma unroll
  for (int j = 0; j < 32; j++) m[j] = 0;
  const uint16_t* r16 = (const uint16_t*)root;  // 2-B aligned (90 B stride)
#pragma unroll
  for (int h = 0; h < 45; h++) {
    const uint32_t v = r16[h];
    const int off = 1 + 2 * h;  // byte offset of this halfword in the message
    m[off >> 2] |= v << (8 * (off & 3));
    if ((off & 3) == 3) m[(off >> 2) + 1] |= v >> 8;
  }
  m[91 >> 2] |= 0x80u << (8 * (91 & 3));
  uint32_t st[8];
  sha256_init(st);
#pragma unroll
  for (int blk = 0; blk < 2; blk++) {
    uint32_t wv[16];
#pragma unroll
    for (int j = 0; j < 16; j++) wv[j] = bswap32(m[16 * blk + j]);
    if (blk == 1) { wv[14] = 0; wv[15] = 91u * 8u; }
    sha256_compress(st, wv);
  }
#pragma unroll
  for (int j = 0; j < 8; j++) out[j] = bswap32(st[j]);
}

__global__ __launch_bounds__(kDahThreads) void dah_kernel(SquareArgs a) {
  // (C + C/2) leaf / level slots, then n / C subtree digests (8 dwords each)
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const long sq = blockIdx.x;
  const int w = 2 * a.k;
  const int n = 2 * w;
  const int C = n < kDahChunk ? n : kDahChunk;
  uint32_t* sub = lds + (C + C / 2) * 8;
  for (int c0 = 0; c0 < n; c0 += C) {
    for (int i = threadIdx.x; i < C; i += kDahThreads) dah_leaf(a, sq, c0 + i, lds + i * 8);
    __syncthreads();
    const uint32_t* r = rfc_reduce(lds, lds + C * 8, C);
    if (threadIdx.x < 8) sub[(c0 / C) * 8 + threadIdx.x] = r[threadIdx.x];
    __syncthreads();
  }
  const uint32_t* root = rfc_reduce(sub, lds, n / C);
  if (threadIdx.x < 8) {
    uint32_t* out = (uint32_t*)(a.dah + sq * 32);
    out[threadIdx.x] = root[threadIdx.x];
  }
}

// Few wide squares (n >= 1024 items, under 64 squares): one workgroup per
// square put the wide lower levels on one CU each (k = 512: 4,096 leaf and
// 4,094 node compressions, ~0.13 ms).  Here the 64-item subtrees go to nsq * n
// / 64 single-wave workgroups (their roots into the digest buffer, free once the
// trees are built) and one workgroup per square reduces the n / 64 subtree roots.
constexpr int kDahSub = 64;
__global__ __launch_bounds__(kDahSub) void dah_sub_kernel(SquareArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t buf[2][kDahSub * 8];
  const int n = 4 * a.k, per = n / kDahSub;
  const long sq = blockIdx.x / per;
  const int b = (int)(blockIdx.x % per);
  const int i = threadIdx.x;
  dah_leaf(a, sq, b * kDahSub + i, buf[0] + i * 8);
  int cur = kDahSub, src = 0;
  while (cur > 1) {
    __syncthreads();  // one wave: orders the level's LDS writes before the next level's reads
    const int next = cur / 2;
    if (i < next) {
      uint32_t m[32];
#pragma unroll
      for (int j = 0; j < 32; j++) m[j] = 0;
      uint32_t lft[8], rgt[8];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        lft[j] = buf[src][(2 * i) * 8 + j];
        rgt[j] = buf[src][(2 * i + 1) * 8 + j];
      }
      m[0] = 0x01u;
      put_bytes<1>(m, lft);
      put_bytes<33>(m, rgt);
      m[65 >> 2] |= 0x80u << (8 * (65 & 3));
      uint32_t st[8];
      sha256_init(st);
#pragma unroll
      for (int blk = 0; blk < 2; blk++) {
        uint32_t wv[16];
#pragma unroll
        for (int j = 0; j < 16; j++) wv[j] = bswap32(m[16 * blk + j]);
        if (blk == 1) { wv[14] = 0; wv[15] = 65u * 8u; }
        sha256_compress(st, wv);
      }
#pragma unroll
      for (int j = 0; j < 8; j++) buf[src ^ 1][i * 8 + j] = bswap32(st[j]);
    }
    src ^= 1;
    cur = next;
  }
  __syncthreads();
  if (i < 8) ((uint32_t*)a.digests)[blockIdx.x * 8 + i] = buf[src][i];
}

__global__ __launch_bounds__(kDahThreads) void dah_top_kernel(SquareArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const long sq = blockIdx.x;
  const int per = 4 * a.k / kDahSub;
  const uint32_t* sub = (const uint32_t*)a.digests + sq * per * 8;
  for (int i = threadIdx.x; i < per * 8; i += kDahThreads) lds[i] = sub[i];
  __syncthreads();
  const uint32_t* root = rfc_reduce(lds, lds + per * 8, per);
  if (threadIdx.x < 8) ((uint32_t*)(a.dah + sq * 32))[threadIdx.x] = root[threadIdx.x];
}

hipError_t launch_nmt_leaves(const SquareArgs& a, hipStream_t s) {
  const long w = 2L * a.k;
  const long total = w * w * a.nsq;
  const long blocks = (total + kLeafWave - 1) / kLeafWave;
  hipLaunchKernelGGL(nmt_leaf_kernel, dim3((unsigned)blocks), dim3(kLeafWave), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_nmt_trees(const SquareArgs& a, hipStream_t s) {
  const int w = 2 * a.k;
  int levels = 0;
  while ((1 << levels) < w) levels++;
  // ping-pong node buffers: level 1 -> recA, 2 -> recB, 3 -> recA, ...
  uint8_t* bufs[2] = {a.rec_a, a.rec_b};
  {
    const long total = a.nsq * 2L * w * (w / 2);
    hipLaunchKernelGGL(nmt_level1_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a,
                       bufs[0], (int)(levels == 1));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  for (int L = 2; L <= levels; L++) {
    const long total = a.nsq * 2L * w * (w >> L);
    hipLaunchKernelGGL(nmt_level_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a,
                       (const uint8_t*)bufs[(L - 2) & 1], bufs[(L - 1) & 1], L, (int)(L == levels));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

size_t nmt_workspace_bytes(int k, long nsq) {
  const size_t w = 2 * (size_t)k;
  const size_t dig = align256(w * w * kDigest * nsq);
  const size_t ns = align256((size_t)k * k * 32 * nsq);
  const size_t ra = align256(nsq * 2 * w * (w / 2) * 48);
  const size_t rb = align256(nsq * 2 * w * (w / 4 > 0 ? w / 4 : 1) * 48);
  return dig + ns + ra + rb;
}

void nmt_workspace_carve(SquareArgs& a, void* ws) {
  const size_t w = 2 * (size_t)a.k;
  uint8_t* p = (uint8_t*)ws;
  a.digests = p;
  p += align256(w * w * kDigest * a.nsq);
  a.ns_table = p;
  p += align256((size_t)a.k * a.k * 32 * a.nsq);
  a.rec_a = p;
  p += align256(a.nsq * 2 * w * (w / 2) * 48);
  a.rec_b = p;
}

static bool dah_split_enabled() {  // DAGPU_DAH_SPLIT=0: one workgroup per square always (A/B)
  const char* e = sw(SW_DAH_SPLIT);
  return !(e && e[0] == '0');
}

hipError_t launch_dah(const SquareArgs& a, hipStream_t s) {
  const int n = 4 * a.k;
  if (a.k > kMaxSplitK) return hipErrorInvalidValue;  // (k = 16384: split squares' finish step)
  if (a.digests && n >= 1024 && a.nsq < 64 && dah_split_enabled()) {
    // the digest buffer (w^2 * 32 B per square) holds the n / 64 subtree roots
    const int per = n / kDahSub;
    hipLaunchKernelGGL(dah_sub_kernel, dim3((unsigned)(a.nsq * per)), dim3(kDahSub), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const size_t lds = (size_t)(per + per / 2) * 8 * sizeof(uint32_t);  // <= 24 KiB (k = 8192)
    hipLaunchKernelGGL(dah_top_kernel, dim3((unsigned)a.nsq), dim3(kDahThreads), lds, s, a);
    return hipGetLastError();
  }
  const int C = n < kDahChunk ? n : kDahChunk;
  const size_t lds = ((size_t)(C + C / 2) + (size_t)(n / C)) * 8 * sizeof(uint32_t);  // <= 97 KiB
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)dah_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(dah_kernel, dim3((unsigned)a.nsq), dim3(kDahThreads), lds, s, a);
  return hipGetLastError();
}

}  // namespace dagpu
