// nmt_forest.hip -- generic batched Merkle forests on gfx950: many independent
// namespaced Merkle trees (nmt v0.20.0) or RFC-6962 trees (celestia-core
// crypto/merkle) of arbitrary, possibly ragged, leaf counts, hashed level by
// level with one lane per node over ALL trees of the batch.
//
// Used by
//   * the rsmt2d.Tree drop-in (ErasuredNamespacedMerkleTree Push/Root,
//     pkg/wrapper/nmt_wrapper.go:93-124) for trees the caller pushes itself;
//   * inclusion.CreateCommitment (pkg/inclusion/commitment.go:19-75): NMT
//     subtree roots over blob shares, then merkle.HashFromByteSlices;
//   * the oversized-square split (split.cpp): NMT subtree roots over a column
//     slab of each row and the top levels above the gathered subtrees.
//
// Leaf message (one lane per leaf):  byte0 | prefix | data
//   NMT leaf:   0x00 | [ns(29)] | data  -> record ns|ns|SHA256(msg)
//               (nmt HashLeaf, mirror test/util/malicious/hasher.go:186-209);
//               prefix = data[0:29] ("self", wrapper Q0 / blob commitment),
//               0xFF*29 ("parity", wrapper Q1..Q3) or none (plain nmt Push).
//   RFC-6962:   0x00 | item          -> 32-B digest (merkle leafHash)
// Inner node: NMT HashNode (hasher.go:271-309) with the ignoreMaxNamespace
// range rule, or RFC-6962 innerHash SHA256(0x01|l|r).  A level with an odd node
// count promotes its last node unchanged, which yields exactly the RFC-6962
// "split at the largest power of two below n" tree (nmt computeRoot,
// merkle.HashFromByteSlices) for every n.
//
// Node records in HBM are 96 B: minNs[32] | maxNs[32] | digest[32] (29-B
// namespaces zero padded) so every field is one pair of 16-B loads.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "forest.hpp"
#include "nmt_node.hpp"
#include "sha256.hpp"

namespace dagpu {

// ---------------------------------------------------------------------------
// Generic message assembly.  The message is  0x00 | P | data  where P is the
// 29-B prefix (pmode self/parity) or empty; data is 4-B aligned.  Words lying
// wholly inside the data region take the fast path (two dword loads + one
// v_perm that both re-aligns and byte-swaps); the few words that straddle the
// prefix, the end of data or the padding are built byte by byte.
// ---------------------------------------------------------------------------
struct MsgShape {
  long off;    // byte offset of data in the message (1 or 30)
  long dlen;   // data bytes
  long mlen;   // message bytes = off + dlen
  long nblk;   // SHA-256 blocks
};

__device__ __forceinline__ MsgShape msg_shape(long dlen, bool has_prefix) {
  MsgShape s;
  s.off = has_prefix ? 1 + kNsSize : 1;
  s.dlen = dlen;
  s.mlen = s.off + dlen;
  s.nblk = (s.mlen + 8) / 64 + 1;
  return s;
}

__device__ __forceinline__ uint32_t data_byte(const uint32_t* d32, long p) {
  return (d32[p >> 2] >> (8 * (p & 3))) & 0xFFu;
}

// message byte p (pmode: 0 none, 1 self, 2 parity)
__device__ __forceinline__ uint32_t msg_byte(const uint32_t* d32, const MsgShape& s, int pmode, long p) {
  if (p == 0) return 0x00u;
  if (p < s.off) return pmode == kPfxParity ? 0xFFu : data_byte(d32, p - 1);
  if (p < s.mlen) return data_byte(d32, p - s.off);
  if (p == s.mlen) return 0x80u;
  const long tot = s.nblk * 64;
  if (p >= tot - 8) {  // 64-bit big-endian bit length
    const uint64_t bits = (uint64_t)s.mlen * 8u;
    return (uint32_t)(bits >> (8 * (tot - 1 - p))) & 0xFFu;
  }
  return 0u;
}

// big-endian message word g
__device__ __forceinline__ uint32_t msg_word(const uint32_t* d32, const MsgShape& s, int pmode, long g) {
  const long lo = 4 * g;
  const long a = lo - s.off;  // data byte under the word's first byte
  if (a >= 0) {
    const long q = a >> 2;
    const uint32_t sh = (uint32_t)(a & 3);
    if (sh == 0 && a + 4 <= s.dlen) return bswap32(d32[q]);
    if (sh != 0 && 4 * q + 8 <= s.dlen) {
      // v_perm: src1 (d[q]) supplies bytes 0-3, src0 (d[q+1]) bytes 4-7; the
      // selector takes bytes sh..sh+3 most-significant first (re-align + bswap)
      return __builtin_amdgcn_perm(d32[q + 1], d32[q], 0x00010203u + sh * 0x01010101u);
    }
  }
  return (msg_byte(d32, s, pmode, lo) << 24) | (msg_byte(d32, s, pmode, lo + 1) << 16) |
         (msg_byte(d32, s, pmode, lo + 2) << 8) | msg_byte(d32, s, pmode, lo + 3);
}

// ---------------------------------------------------------------------------
// Leaves: one lane per leaf.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void forest_leaf_kernel(ForestLeafArgs a) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.nleaves) return;
  const uint32_t* d32 = (const uint32_t*)(a.data + i * a.data_stride);
  int pm = a.pmode;
  if (pm == kPfxFlags) {
    pm = a.pflags[i];
  } else if (pm == kPfxGrid) {
    const long r = a.grid_r0 + i / a.grid_w, c = a.grid_c0 + i % a.grid_w;
    pm = (r < a.grid_k && c < a.grid_k) ? kPfxSelf : kPfxParity;
  }
  uint32_t st[8];
  if (a.dlen == kShareSize && a.pmode != kPfxNone && !a.rfc && (a.data_stride & 15) == 0 &&
      (((uintptr_t)a.data) & 15) == 0) {
    // 512-B shares with a namespace prefix (wrapper cells, blob commitments,
    // split-square slabs): the share-specialised leaf hash of the square pipeline
    uint32_t ns[8];
    share_leaf_sha256((const uint4*)d32, pm == kPfxSelf, st, ns);
    if (pm == kPfxParity) {
#pragma unroll
      for (int j = 0; j < 7; j++) ns[j] = 0xFFFFFFFFu;
      ns[7] = 0xFFu;
    }
    uint4* o = (uint4*)(a.out + i * kRecNmt);
    o[0] = make_uint4(ns[0], ns[1], ns[2], ns[3]);
    o[1] = make_uint4(ns[4], ns[5], ns[6], ns[7]);
    o[2] = o[0];
    o[3] = o[1];
    o[4] = make_uint4(bswap32(st[0]), bswap32(st[1]), bswap32(st[2]), bswap32(st[3]));
    o[5] = make_uint4(bswap32(st[4]), bswap32(st[5]), bswap32(st[6]), bswap32(st[7]));
    return;
  }
  const MsgShape sh = msg_shape(a.dlen, a.pmode != kPfxNone);
  sha256_init(st);
#pragma unroll 1
  for (long b = 0; b < sh.nblk; b++) {
    uint32_t m[16];
#pragma unroll
    for (int j = 0; j < 16; j++) m[j] = msg_word(d32, sh, pm, 16 * b + j);
    sha256_compress(st, m);
  }
  if (a.rfc) {
    uint4* o = (uint4*)(a.out + i * kRecRfc);
    o[0] = make_uint4(bswap32(st[0]), bswap32(st[1]), bswap32(st[2]), bswap32(st[3]));
    o[1] = make_uint4(bswap32(st[4]), bswap32(st[5]), bswap32(st[6]), bswap32(st[7]));
    return;
  }
  uint32_t ns[8];
  if (pm == kPfxParity) {
#pragma unroll
    for (int j = 0; j < 7; j++) ns[j] = 0xFFFFFFFFu;
    ns[7] = 0xFFu;
  } else {
#pragma unroll
    for (int j = 0; j < 7; j++) ns[j] = d32[j];
    ns[7] = d32[7] & 0xFFu;
  }
  uint4* o = (uint4*)(a.out + i * kRecNmt);
  o[0] = make_uint4(ns[0], ns[1], ns[2], ns[3]);
  o[1] = make_uint4(ns[4], ns[5], ns[6], ns[7]);
  o[2] = o[0];
  o[3] = o[1];
  o[4] = make_uint4(bswap32(st[0]), bswap32(st[1]), bswap32(st[2]), bswap32(st[3]));
  o[5] = make_uint4(bswap32(st[4]), bswap32(st[5]), bswap32(st[6]), bswap32(st[7]));
}

// ---------------------------------------------------------------------------
// One inner level over all trees: lane = output node.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load8(const uint8_t* p, uint32_t (&d)[8]) {
  const uint4* q = (const uint4*)p;
  const uint4 x0 = q[0], x1 = q[1];
  d[0] = x0.x; d[1] = x0.y; d[2] = x0.z; d[3] = x0.w;
  d[4] = x1.x; d[5] = x1.y; d[6] = x1.z; d[7] = x1.w;
}

__device__ __forceinline__ void store8(uint8_t* p, const uint32_t (&d)[8]) {
  uint4* q = (uint4*)p;
  q[0] = make_uint4(d[0], d[1], d[2], d[3]);
  q[1] = make_uint4(d[4], d[5], d[6], d[7]);
}

// tree of output node gid: largest t with off[t] <= gid (off has ntrees+1 entries)
__device__ __forceinline__ long find_tree(const int64_t* off, long ntrees, long gid) {
  long lo = 0, hi = ntrees;  // invariant off[lo] <= gid < off[hi]
  while (hi - lo > 1) {
    const long mid = (lo + hi) >> 1;
    if (off[mid] <= gid) lo = mid; else hi = mid;
  }
  return lo;
}

// RFC-6962 inner node SHA256(0x01 | l | r) (65 B, 2 blocks); l, r, out in byte order
__device__ __forceinline__ void rfc_inner(const uint32_t (&l)[8], const uint32_t (&r)[8], uint32_t (&out)[8]) {
  uint32_t m[32];
#pragma unroll
  for (int j = 0; j < 32; j++) m[j] = 0;
  m[0] = 0x01u;
  put_bytes<1>(m, l);
  put_bytes<33>(m, r);
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
  for (int j = 0; j < 8; j++) out[j] = bswap32(st[j]);
}

__device__ __forceinline__ void forest_level_node(const ForestLevelArgs& a, long gid) {
  long t, j;
  if (a.out_off) {
    t = find_tree(a.out_off, a.ntrees, gid);
    j = gid - a.out_off[t];
  } else {
    t = gid / a.out_per;
    j = gid - t * a.out_per;
  }
  const long ibase = a.in_off ? a.in_off[t] : t * a.in_tstride;
  const long icount = a.in_off ? a.in_off[t + 1] - a.in_off[t] : a.in_per;
  const long j0 = 2 * j, j1 = 2 * j + 1;
  const int rec = a.rfc ? kRecRfc : kRecNmt;
  const uint8_t* lp = a.in + (ibase + j0 * a.in_lstride) * rec;
  uint8_t* op = a.out + gid * rec;
  if (j1 >= icount) {  // odd node out: promoted unchanged
    const uint4* src = (const uint4*)lp;
    uint4* dst = (uint4*)op;
    for (int q = 0; q < rec / 16; q++) dst[q] = src[q];
    return;
  }
  const uint8_t* rp = a.in + (ibase + j1 * a.in_lstride) * rec;
  if (a.rfc) {
    uint32_t l[8], r[8], o[8];
    load8(lp, l);
    load8(rp, r);
    rfc_inner(l, r, o);
    store8(op, o);
    return;
  }
  uint32_t lmn[8], lmx[8], ld[8], rmn[8], rmx[8], rd[8];
  load8(lp, lmn); load8(lp + 32, lmx); load8(lp + 64, ld);
  load8(rp, rmn); load8(rp + 32, rmx); load8(rp + 64, rd);
  if (a.check_order) {  // nmt Push: ns(j0) <= ns(j1) <= ns(j1 + 1)
    bool bad = ns_less(rmn, lmn);
    if (j1 + 1 < icount) {
      uint32_t n2[8];
      load8(a.in + (ibase + (j1 + 1) * a.in_lstride) * rec, n2);
      bad |= ns_less(n2, rmn);
    }
    if (bad) atomicOr(&a.status[a.status_shared ? 0 : t], kForestPushOrder);
  }
  uint32_t st[8];
  // A min namespace equal to the parity namespace (the largest) makes the max
  // the parity namespace too.  Waves whose children all carry it (the parity
  // quadrants of a wrapper square / split slab) hash with constant namespace
  // words, as nmt_level_kernel does.
  const bool lpar = ns_is_parity(lmn), rpar = ns_is_parity(rmn);
  if (__all(lpar && rpar)) {
    auto get = [&](int P, int i) -> uint32_t { return P == 2 ? ld[i] : P == 5 ? rd[i] : 0xFFFFFFFFu; };
    sha_node_msg<true, true, true>(get, st);
  } else if (__all(lpar)) {
    auto get = [&](int P, int i) -> uint32_t {
      return P <= 1 ? 0xFFFFFFFFu : P == 2 ? ld[i] : P == 3 ? rmn[i] : P == 4 ? rmx[i] : rd[i];
    };
    sha_node_msg<true>(get, st);
  } else {
    auto get = [&](int P, int i) -> uint32_t {
      return P == 0 ? lmn[i] : P == 1 ? lmx[i] : P == 2 ? ld[i] : P == 3 ? rmn[i] : P == 4 ? rmx[i] : rd[i];
    };
    sha_node_msg(get, st);
  }
  uint32_t dg[8];
#pragma unroll
  for (int i = 0; i < 8; i++) dg[i] = bswap32(st[i]);
  const bool keep_left_max = a.ignore_max && ns_is_parity(rmn);
  store8(op, lmn);
  if (keep_left_max) store8(op + 32, lmx); else store8(op + 32, rmx);
  store8(op + 64, dg);
}

__global__ __launch_bounds__(256) void forest_level_kernel(ForestLevelArgs a) {
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  if (gid < a.total_out) forest_level_node(a, gid);
}

// the same level of two forests in one launch (their nodes back to back)
__global__ __launch_bounds__(256) void forest_level2_kernel(ForestLevelArgs a, ForestLevelArgs b) {
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  if (gid < a.total_out) forest_level_node(a, gid);
  else if (gid - a.total_out < b.total_out) forest_level_node(b, gid - a.total_out);
}

// ---------------------------------------------------------------------------
// Roots.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void forest_roots_kernel(const uint8_t* leaves, const uint8_t* inner,
                                                           const int64_t* root_idx, long ntrees, int rfc,
                                                           int records, uint8_t* out, long stride,
                                                           int64_t ubase, long utstride) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t >= ntrees) return;
  // uniform plan (root_idx null): ubase >= 0 -> inner record ubase + t;
  // -2 -> leaf t * utstride (single-leaf trees); -1 -> empty trees
  const int64_t ix = root_idx ? root_idx[t] : ubase >= 0 ? ubase + t : ubase == -2 ? -(t * utstride) - 2 : -1;
  const int rec = rfc ? kRecRfc : kRecNmt;
  uint32_t mn[8], mx[8], dg[8];
  if (ix == -1) {  // empty tree: SHA256("")
    const uint32_t e[8] = {0x42c4b0e3u, 0x141cfc98u, 0xc8f4fb9au, 0x24b96f99u,
                           0xe441ae27u, 0x4c939b64u, 0x1b9995a4u, 0x55b85278u};
#pragma unroll
    for (int q = 0; q < 8; q++) { mn[q] = 0; mx[q] = 0; dg[q] = e[q]; }
  } else {
    const uint8_t* p = ix >= 0 ? inner + ix * rec : leaves + (-(ix + 2)) * rec;
    if (rfc) {
      load8(p, dg);
    } else {
      load8(p, mn); load8(p + 32, mx); load8(p + 64, dg);
    }
  }
  if (rfc) {
    store8(out + t * stride, dg);
  } else if (records) {
    uint8_t* o = out + t * stride;
    store8(o, mn); store8(o + 32, mx); store8(o + 64, dg);
  } else {
    write_root(out + t * stride, mn, mx, dg);
  }
}

hipError_t launch_forest_leaves(const ForestLeafArgs& a, hipStream_t s) {
  if (a.nleaves <= 0) return hipSuccess;
  hipLaunchKernelGGL(forest_leaf_kernel, dim3((unsigned)((a.nleaves + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_forest_level(const ForestLevelArgs& a, hipStream_t s) {
  if (a.total_out <= 0) return hipSuccess;
  hipLaunchKernelGGL(forest_level_kernel, dim3((unsigned)((a.total_out + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_forest_roots(const uint8_t* leaves, const uint8_t* inner, const int64_t* root_idx,
                               long ntrees, int rfc, int records, uint8_t* out, long out_stride,
                               hipStream_t s) {
  if (ntrees <= 0) return hipSuccess;
  if (out_stride == 0) out_stride = rfc ? kRecRfc : records ? kRecNmt : kNodeSize;
  hipLaunchKernelGGL(forest_roots_kernel, dim3((unsigned)((ntrees + 255) / 256)), dim3(256), 0, s, leaves,
                     inner, root_idx, ntrees, rfc, records, out, out_stride, (int64_t)-1, 0L);
  return hipGetLastError();
}

// Roots of a uniform plan from its shape alone: nothing to upload, so the
// caller's host plan need not outlive the enqueue.
static hipError_t launch_forest_roots_uniform(const ForestPlan& p, const uint8_t* leaves, const uint8_t* inner,
                                              int rfc, int records, uint8_t* out, long out_stride,
                                              hipStream_t s) {
  if (p.ntrees <= 0) return hipSuccess;
  if (out_stride == 0) out_stride = rfc ? kRecRfc : records ? kRecNmt : kNodeSize;
  const int64_t ubase = p.per0 == 0 ? -1 : p.nlevels == 0 ? -2 : (int64_t)p.base[p.nlevels];
  hipLaunchKernelGGL(forest_roots_kernel, dim3((unsigned)((p.ntrees + 255) / 256)), dim3(256), 0, s, leaves,
                     inner, (const int64_t*)nullptr, p.ntrees, rfc, records, out, out_stride, ubase, p.tstride0);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Namespace push-order check over share vectors (nmt Push ErrInvalidPushOrder
// for Q0 rows/columns): element j of vector v at base + v*vec_stride +
// j*elem_stride; ORs `bit` into *status if ns(j+1) < ns(j) anywhere.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ns_order_kernel(const uint8_t* base, long nvec, long nper,
                                                       long vec_stride, long elem_stride, int32_t* status,
                                                       int bit) {
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long pairs = nper - 1;
  if (gid >= nvec * pairs) return;
  const long v = gid / pairs, j = gid - v * pairs;
  const uint8_t* a = base + v * vec_stride + j * elem_stride;
  uint32_t x[8], y[8];
  load8(a, x);
  load8(a + elem_stride, y);
  x[7] &= 0xFFu;
  y[7] &= 0xFFu;
  if (ns_less(y, x)) atomicOr(status, bit);
}

hipError_t launch_ns_order_check(const uint8_t* base, long nvec, long nper, long vec_stride, long elem_stride,
                                 int32_t* status, int bit, hipStream_t s) {
  const long total = nvec * (nper - 1);
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(ns_order_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, base, nvec, nper,
                     vec_stride, elem_stride, status, bit);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Node gather for exported row-tree levels (inclusion.EDSSubTreeRootCacher):
// request r = (row, depth, position); level L = log2(w) - depth; record at
// lvl_off(L) + row * (w >> L) + position with lvl_off(L) = sum_{l<L} w*(w>>l).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void node_gather_kernel(const uint8_t* nodes, int w, int logw, const uint32_t* req,
                                                          long n, uint8_t* out) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  const uint32_t row = req[3 * t], depth = req[3 * t + 1], pos = req[3 * t + 2];
  const int L = logw - (int)depth;
  long off = 0;
  for (int l = 0; l < L; l++) off += (long)w * (w >> l);
  const uint8_t* p = nodes + (off + (long)row * (w >> L) + pos) * kRecNmt;
  uint32_t mn[8], mx[8], dg[8];
  load8(p, mn); load8(p + 32, mx); load8(p + 64, dg);
  write_root(out + t * kNodeSize, mn, mx, dg);
}

// Packed 90-B nodes (minNs | maxNs | digest) -> 96-B records (each field
// zero padded to 32 B), one lane per node.
// One thread per output dword (24 per record): the byte-loop form (one thread
// per record, 96 byte loads and stores that the compiler kept in order since the
// buffers may alias) took 24 us for the 1,024 row roots of a k = 512 split square.
__global__ __launch_bounds__(256) void node_to_rec_kernel(const uint8_t* __restrict__ nodes, long n,
                                                          uint8_t* __restrict__ recs) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t >= n * (kRecNmt / 4)) return;
  const long i = t / (kRecNmt / 4);
  const int j = (int)(t - i * (kRecNmt / 4));  // dword j of the record: field j / 8, bytes 4 (j % 8) ..
  const uint8_t* nd = nodes + i * kNodeSize;
  const int f = j >> 3, off = 4 * (j & 7);
  const uint8_t* src = nd + 29 * f;  // minNs, maxNs, then the digest at 58
  uint32_t v = 0;
#pragma unroll
  for (int b = 0; b < 4; b++) {
    const int o = off + b;
    if (f == 2 || o < 29) v |= (uint32_t)src[o] << (8 * b);
  }
  ((uint32_t*)(recs + i * kRecNmt))[j] = v;
}

hipError_t launch_node_to_rec(const uint8_t* nodes, long n, uint8_t* recs, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const long threads = n * (kRecNmt / 4);
  hipLaunchKernelGGL(node_to_rec_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, nodes, n, recs);
  return hipGetLastError();
}

hipError_t launch_node_gather(const uint8_t* nodes, int w, const uint32_t* req, long n, uint8_t* out,
                              hipStream_t s) {
  if (n <= 0) return hipSuccess;
  int logw = 0;
  while ((1 << logw) < w) logw++;
  hipLaunchKernelGGL(node_gather_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, nodes, w, logw, req,
                     n, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Host planner.
// ---------------------------------------------------------------------------
ForestPlan ForestPlan::uniform_plan(long ntrees, long leaves, long tstride, long lstride) {
  ForestPlan p;
  p.ntrees = ntrees;
  p.uniform = true;
  p.per0 = leaves;
  p.tstride0 = tstride;
  p.lstride0 = lstride;
  p.total.push_back(ntrees * leaves);
  p.base.push_back(0);
  p.per.push_back(leaves);
  long c = leaves, acc = 0;
  while (c > 1) {
    c = (c + 1) / 2;
    p.nlevels++;
    p.per.push_back(c);
    p.total.push_back(ntrees * c);
    p.base.push_back(acc);
    acc += ntrees * c;
  }
  p.inner_records = acc;
  p.root_idx.resize(ntrees);
  for (long t = 0; t < ntrees; t++) {
    if (leaves == 0) p.root_idx[t] = -1;
    else if (p.nlevels == 0) p.root_idx[t] = -(t * tstride) - 2;
    else p.root_idx[t] = p.base[p.nlevels] + t;
  }
  p.finalize();
  return p;
}

ForestPlan ForestPlan::ragged_plan(const std::vector<long>& counts) {
  ForestPlan p;
  const long T = (long)counts.size();
  p.ntrees = T;
  p.uniform = false;
  p.counts0 = counts;
  p.root_idx.assign(T, -1);
  std::vector<long> cur = counts;
  std::vector<int64_t> off(T + 1, 0);
  for (long t = 0; t < T; t++) off[t + 1] = off[t] + cur[t];
  p.off.push_back(off);
  p.total.push_back(off[T]);
  p.base.push_back(0);
  p.per.push_back(0);
  for (long t = 0; t < T; t++)
    if (cur[t] == 1) p.root_idx[t] = -(off[t]) - 2;
  long acc = 0;
  for (;;) {
    bool more = false;
    for (long t = 0; t < T; t++) more |= cur[t] > 1;
    if (!more) break;
    for (long t = 0; t < T; t++) cur[t] = cur[t] > 1 ? (cur[t] + 1) / 2 : 0;
    for (long t = 0; t < T; t++) off[t + 1] = off[t] + cur[t];
    p.nlevels++;
    p.off.push_back(off);
    p.total.push_back(off[T]);
    p.base.push_back(acc);
    p.per.push_back(0);
    for (long t = 0; t < T; t++)
      if (cur[t] == 1) p.root_idx[t] = acc + off[t];
    acc += off[T];
  }
  p.inner_records = acc;
  p.finalize();
  return p;
}

void ForestPlan::finalize() {
  meta.clear();
  meta_off.assign(off.size(), 0);
  for (size_t L = 0; L < off.size(); L++) {
    meta_off[L] = (long)meta.size();
    meta.insert(meta.end(), off[L].begin(), off[L].end());
  }
  meta_root = (long)meta.size();
  meta.insert(meta.end(), root_idx.begin(), root_idx.end());
}

// level L (>= 1) of plan p as kernel arguments
static ForestLevelArgs level_args(const ForestPlan& p, int L, const uint8_t* d_leaves, uint8_t* d_inner,
                                  int64_t* d_meta, int ignore_max, int check_order, int rfc, int32_t* d_status,
                                  int status_shared = 0) {
  const int rec = rfc ? kRecRfc : kRecNmt;
  ForestLevelArgs a{};
  a.in = L == 1 ? d_leaves : d_inner + (long)p.base[L - 1] * rec;
  a.out = d_inner + (long)p.base[L] * rec;
  if (p.uniform) {
    a.in_off = nullptr;
    a.in_tstride = L == 1 ? p.tstride0 : p.per[L - 1];
    a.in_lstride = L == 1 ? p.lstride0 : 1;
    a.in_per = p.per[L - 1];
    a.out_off = nullptr;
    a.out_per = p.per[L];
  } else {
    a.in_off = d_meta + p.meta_off[L - 1];
    a.in_lstride = 1;
    a.out_off = d_meta + p.meta_off[L];
  }
  a.ntrees = p.ntrees;
  a.total_out = p.total[L];
  a.ignore_max = ignore_max;
  a.check_order = check_order && L == 1;
  a.rfc = rfc;
  a.status = d_status;
  a.status_shared = status_shared;
  return a;
}

hipError_t forest_enqueue(const ForestPlan& p, const uint8_t* d_leaves, uint8_t* d_inner, int64_t* d_meta,
                          int ignore_max, int check_order, int rfc, int32_t* d_status, uint8_t* d_roots,
                          int records, long roots_stride, hipStream_t s) {
  if (p.ntrees == 0) return hipSuccess;
  hipError_t e = hipSuccess;
  if (!p.uniform) {  // uniform plans address their levels and roots by shape
    e = hipMemcpyAsync(d_meta, p.meta.data(), p.meta.size() * sizeof(int64_t), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
  }
  for (int L = 1; L <= p.nlevels; L++) {
    e = launch_forest_level(level_args(p, L, d_leaves, d_inner, d_meta, ignore_max, check_order, rfc, d_status), s);
    if (e != hipSuccess) return e;
  }
  if (p.uniform) return launch_forest_roots_uniform(p, d_leaves, d_inner, rfc, records, d_roots, roots_stride, s);
  return launch_forest_roots(d_leaves, d_inner, d_meta + p.meta_root, p.ntrees, rfc, records, d_roots,
                             roots_stride, s);
}

hipError_t forest_enqueue_pair(const ForestJob& x, const ForestJob& y, hipStream_t s) {
  const ForestJob* j[2] = {&x, &y};
  for (int f = 0; f < 2; f++) {
    if (j[f]->p->ntrees == 0 || j[f]->p->uniform) continue;
    hipError_t e = hipMemcpyAsync(j[f]->d_meta, j[f]->p->meta.data(), j[f]->p->meta.size() * sizeof(int64_t),
                                  hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
  }
  const int nl = x.p->nlevels > y.p->nlevels ? x.p->nlevels : y.p->nlevels;
  for (int L = 1; L <= nl; L++) {
    ForestLevelArgs a[2];
    int n = 0;
    for (int f = 0; f < 2; f++)
      if (j[f]->p->ntrees > 0 && L <= j[f]->p->nlevels && j[f]->p->total[L] > 0)
        a[n++] = level_args(*j[f]->p, L, j[f]->d_leaves, j[f]->d_inner, j[f]->d_meta, j[f]->ignore_max,
                            j[f]->check_order, j[f]->rfc, j[f]->d_status, j[f]->status_shared);
    hipError_t e = hipSuccess;
    if (n == 1) {
      e = launch_forest_level(a[0], s);
    } else if (n == 2) {
      const long total = a[0].total_out + a[1].total_out;
      hipLaunchKernelGGL(forest_level2_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a[0], a[1]);
      e = hipGetLastError();
    }
    if (e != hipSuccess) return e;
  }
  for (int f = 0; f < 2; f++) {
    const ForestJob& q = *j[f];
    if (q.p->ntrees == 0) continue;
    if (q.p->uniform) {
      hipError_t e = launch_forest_roots_uniform(*q.p, q.d_leaves, q.d_inner, q.rfc, q.records, q.d_roots,
                                                 q.roots_stride, s);
      if (e != hipSuccess) return e;
      continue;
    }
    hipError_t e = launch_forest_roots(q.d_leaves, q.d_inner, q.d_meta + q.p->meta_root, q.p->ntrees, q.rfc,
                                       q.records, q.d_roots, q.roots_stride, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace dagpu
