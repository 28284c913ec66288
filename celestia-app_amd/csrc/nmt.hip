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
// Kernel 2 (trees): one workgroup builds 512/w trees (w = 2k): level 1 reads
//   leaf digests + namespaces, levels >= 2 run in LDS.  Node namespace ranges
//   follow HashNode with ignoreMaxNamespace=true; push-order (ErrInvalidPushOrder)
//   is checked on Q0 leaves.
// Kernel 3 (DAH): one workgroup per square, RFC-6962 over 4k roots.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"
#include "sha256.hpp"

namespace dagpu {

// v_perm_b32 selector byte 0x0C produces 0x00.
#define PZ 0x0Cu

// ---------------------------------------------------------------------------
// Kernel 1: leaf digests.  digest(r,c) = SHA256(0x00 | P | share), where
// P = share[0:29] if r<k && c<k else 0xFF*29 (ParitySharesNamespace).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void nmt_leaf_kernel(SquareArgs a) {
  const int k = a.k;
  const long w = 2L * k;
  const long cells = w * w;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  if (gid >= cells * a.nsq) return;
  const long sq = gid / cells;
  const long cell = gid - sq * cells;
  const long r = cell / w, c = cell - (cell / w) * w;
  const bool q0 = (r < k) && (c < k);

  // Message 0x00 | P | share (542 B) as big-endian words: word J >= 8 is share
  // bytes 4J-30..4J-27 = perm(dw[J-8], dw[J-7]) (share starts at byte 30).
  const uint4* src = (const uint4*)(a.eds + sq * a.eds_sq_stride + cell * kShareSize);
  uint32_t st[8];
  sha256_init(st);
  uint32_t m[16];
  uint4 carry;
  {  // block 0: 0x00 | P(29) | share[0:34]
    const uint4 q0v = src[0], q1v = src[1], q2v = src[2];
    const uint32_t d[12] = {q0v.x, q0v.y, q0v.z, q0v.w, q1v.x, q1v.y,
                            q1v.z, q1v.w, q2v.x, q2v.y, q2v.z, q2v.w};
    if (q0) {
      m[0] = __builtin_amdgcn_perm(d[0], d[0], (PZ << 24) | 0x000102u);
#pragma unroll
      for (int j = 1; j <= 6; j++) m[j] = __builtin_amdgcn_perm(d[j - 1], d[j], 0x07000102u);
      m[7] = __builtin_amdgcn_perm(d[6], d[7], (0x0700u << 16) | (PZ << 8) | PZ);
    } else {
      m[0] = 0x00FFFFFFu;
#pragma unroll
      for (int j = 1; j <= 6; j++) m[j] = 0xFFFFFFFFu;
      m[7] = 0xFFFF0000u;
    }
    m[7] |= __builtin_amdgcn_perm(d[0], d[0], (PZ << 24) | (PZ << 16) | 0x0001u);
#pragma unroll
    for (int j = 8; j < 16; j++) m[j] = __builtin_amdgcn_perm(d[j - 8], d[j - 7], 0x06070001u);
    sha256_compress(st, m);
    carry = q2v;
  }
  // blocks 1..7: words 16b..16b+15 read dwords 16b-8 .. 16b+8
#pragma unroll 1
  for (int b = 1; b <= 7; b++) {
    const uint4 n0 = src[4 * b - 1], n1 = src[4 * b], n2 = src[4 * b + 1], n3 = src[4 * b + 2];
    const uint32_t d[20] = {carry.x, carry.y, carry.z, carry.w, n0.x, n0.y, n0.z,
                            n0.w,    n1.x,    n1.y,    n1.z,    n1.w, n2.x, n2.y,
                            n2.z,    n2.w,    n3.x,    n3.y,    n3.z, n3.w};
#pragma unroll
    for (int j = 0; j < 16; j++) m[j] = __builtin_amdgcn_perm(d[j], d[j + 1], 0x06070001u);
    sha256_compress(st, m);
    carry = n3;
  }
  {  // block 8: share[482:512] | 0x80 | zeros | bit length
    const uint4 n0 = src[31];
    const uint32_t d[8] = {carry.x, carry.y, carry.z, carry.w, n0.x, n0.y, n0.z, n0.w};
#pragma unroll
    for (int j = 0; j < 7; j++) m[j] = __builtin_amdgcn_perm(d[j], d[j + 1], 0x06070001u);
    m[7] = __builtin_amdgcn_perm(d[7], d[7], (0x0607u << 16) | (PZ << 8) | PZ) | 0x8000u;
#pragma unroll
    for (int j = 8; j < 15; j++) m[j] = 0u;
    m[15] = 542u * 8u;
    sha256_compress(st, m);
  }
  uint4* out = (uint4*)(a.digests + gid * kDigest);
  out[0] = make_uint4(bswap32(st[0]), bswap32(st[1]), bswap32(st[2]), bswap32(st[3]));
  out[1] = make_uint4(bswap32(st[4]), bswap32(st[5]), bswap32(st[6]), bswap32(st[7]));
}

// ---------------------------------------------------------------------------
// Node helpers.  A node in registers/LDS: 24 dwords in memory byte order:
// [0..7] minNs (29 B, zero padded), [8..15] maxNs, [16..23] digest bytes.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool ns_is_parity(const uint32_t (&ns)[8]) {
  uint32_t acc = ns[0] & ns[1] & ns[2] & ns[3] & ns[4] & ns[5] & ns[6];
  return acc == 0xFFFFFFFFu && (ns[7] & 0xFFu) == 0xFFu;
}

// lexicographic a < b over 29 bytes
__device__ __forceinline__ bool ns_less(const uint32_t (&x)[8], const uint32_t (&y)[8]) {
  int res = 0;  // -1 less, 1 greater, 0 equal so far
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t xa = bswap32(i == 7 ? (x[i] & 0xFFu) : x[i]);
    const uint32_t ya = bswap32(i == 7 ? (y[i] & 0xFFu) : y[i]);
    if (res == 0) res = (xa < ya) ? -1 : ((xa > ya) ? 1 : 0);
  }
  return res < 0;
}

// OR `src` (NDW little-endian dwords, zero padded) into byte buffer m at OFF.
template <int OFF, int NDW, int MW>
__device__ __forceinline__ void put_bytes(uint32_t (&m)[MW], const uint32_t (&src)[NDW]) {
  constexpr int al = OFF & 3;
  constexpr int d0 = OFF >> 2;
#pragma unroll
  for (int i = 0; i < NDW; i++) {
    if constexpr (al == 0) {
      m[d0 + i] |= src[i];
    } else {
      m[d0 + i] |= src[i] << (8 * al);
      if (d0 + i + 1 < MW) m[d0 + i + 1] |= src[i] >> (32 - 8 * al);
    }
  }
}

// Window form: OR part P (8 dwords fetched through get(P, i)) placed at message
// byte OFF into the 16-word window of SHA block B.  Only dwords that land in the
// window are fetched, so each block pulls just the source words it needs.
template <int OFF, int B, int P, class G>
__device__ __forceinline__ void put_part_win(uint32_t (&m)[16], const G& get) {
  constexpr int al = OFF & 3;
  constexpr int d0 = OFF >> 2;
  constexpr int lo = 16 * B, hi = 16 * B + 16;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int p0 = d0 + i, p1 = d0 + i + 1;
    const bool in0 = p0 >= lo && p0 < hi;
    const bool in1 = al != 0 && p1 >= lo && p1 < hi;
    if (in0 || in1) {
      const uint32_t v = get(P, i);
      if (in0) m[p0 - lo] |= al ? (v << (8 * al)) : v;
      if (in1) m[p1 - lo] |= v >> (32 - 8 * al);
    }
  }
}

// NMT HashNode message 0x01 | L.min | L.max | L.d | R.min | R.max | R.d
// (181 B, 3 SHA blocks).  get(P, i): P = 0..5 -> Lmn, Lmx, Ld, Rmn, Rmx, Rd.
template <class G>
__device__ __forceinline__ void sha_node_msg(const G& get, uint32_t (&st)[8]) {
  sha256_init(st);
#pragma unroll
  for (int blk = 0; blk < 3; blk++) {
    uint32_t m[16];
#pragma unroll
    for (int j = 0; j < 16; j++) m[j] = 0;
    if (blk == 0) m[0] = 0x01u;
    if (blk == 0) { put_part_win<1, 0, 0>(m, get); put_part_win<30, 0, 1>(m, get); put_part_win<59, 0, 2>(m, get); }
    if (blk == 1) {
      put_part_win<59, 1, 2>(m, get); put_part_win<91, 1, 3>(m, get); put_part_win<120, 1, 4>(m, get);
    }
    if (blk == 2) {
      put_part_win<120, 2, 4>(m, get); put_part_win<149, 2, 5>(m, get);
      m[45 - 32] |= 0x80u << 8;  // byte 181
    }
#pragma unroll
    for (int j = 0; j < 16; j++) m[j] = bswap32(m[j]);
    if (blk == 2) { m[14] = 0; m[15] = 181u * 8u; }
    sha256_compress(st, m);
  }
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

__device__ __forceinline__ void load_digest(const uint8_t* p, uint32_t (&d)[8]) {
  const uint4* q = (const uint4*)p;
  const uint4 x0 = q[0], x1 = q[1];
  d[0] = x0.x; d[1] = x0.y; d[2] = x0.z; d[3] = x0.w;
  d[4] = x1.x; d[5] = x1.y; d[6] = x1.z; d[7] = x1.w;
}

// ---------------------------------------------------------------------------
// Kernel 2: trees.  Tree id t in [0, nsq*2w): sq = t / 2w, axis = (t/w)&1,
// idx = t % w.  tpw = 512/w trees per 256-thread workgroup (w <= 512), so every
// level has at most one node per thread.  Nodes live in LDS as 24 dwords:
// [0..7] minNs, [8..15] maxNs, [16..23] digest (memory byte order).
// ---------------------------------------------------------------------------
constexpr int kTreeThreads = 256;

__global__ __launch_bounds__(kTreeThreads) void nmt_tree_kernel(SquareArgs a, int tpw) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int k = a.k;
  const int w = 2 * k;
  const long tree0 = (long)blockIdx.x * tpw;
  const long ntrees = a.nsq * 2L * w;
  const int half = w / 2;  // level-1 nodes per tree
  const int g = threadIdx.x;

  // ---- level 1: hash pairs of leaves (leaf node = ns | ns | digest) ----
  {
    const int tl = g / half, p = g - tl * half;
    const long t = tree0 + tl;
    uint32_t out[24];
    if (tl < tpw && t < ntrees) {
      const long sq = t / (2L * w);
      const int axis = (int)((t / w) & 1);
      const int idx = (int)(t % w);
      const uint8_t* eds = a.eds + sq * a.eds_sq_stride;
      const uint8_t* dig = a.digests + sq * (long)w * w * kDigest;
      const int j0 = 2 * p, j1 = 2 * p + 1;
      const long cell0 = axis == 0 ? (long)idx * w + j0 : (long)j0 * w + idx;
      const long cell1 = axis == 0 ? (long)idx * w + j1 : (long)j1 * w + idx;
      const bool q00 = (idx < k) && (j0 < k), q01 = (idx < k) && (j1 < k);
      uint32_t nl[8], nr[8], dl[8], dr[8];
      load_ns(eds + cell0 * kShareSize, q00, nl);
      load_ns(eds + cell1 * kShareSize, q01, nr);
      load_digest(dig + cell0 * kDigest, dl);
      load_digest(dig + cell1 * kDigest, dr);
      // nmt Push order: ns(j0) <= ns(j1) <= ns(j1+1); only Q0 leaves can violate
      if (q01) {
        bool bad = ns_less(nr, nl);
        if (j1 + 1 < k) {
          const long cell2 = axis == 0 ? (long)idx * w + j1 + 1 : (long)(j1 + 1) * w + idx;
          uint32_t n2[8];
          load_ns(eds + cell2 * kShareSize, true, n2);
          bad |= ns_less(n2, nr);
        }
        if (bad) atomicOr(&a.status[sq], kStatusPushOrder);
      }
      uint32_t st[8];
      auto get = [&](int P, int i) -> uint32_t {
        return P == 0 || P == 1 ? nl[i] : P == 2 ? dl[i] : P == 3 || P == 4 ? nr[i] : dr[i];
      };
      sha_node_msg(get, st);
      const bool rpar = ns_is_parity(nr);
#pragma unroll
      for (int i = 0; i < 8; i++) {
        out[i] = nl[i];
        out[8 + i] = rpar ? nl[i] : nr[i];
        out[16 + i] = bswap32(st[i]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 24; i++) out[i] = 0;
    }
    uint4* slot = (uint4*)(lds + g * 24);
#pragma unroll
    for (int i = 0; i < 6; i++) slot[i] = make_uint4(out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]);
  }
  __syncthreads();

  // ---- levels >= 2 in LDS: node q of tree tl reads slots 2q, 2q+1 ----
  for (int per_tree = half; per_tree > 1; per_tree >>= 1) {
    const int next = per_tree >> 1;
    const int total = tpw * next;
    uint32_t out[24];
    const bool active = g < total;
    int tl = 0, q = 0;
    if (active) {
      tl = g / next;
      q = g - tl * next;
      const uint32_t* sl = lds + ((long)tl * half + 2 * q) * 24;
      const uint32_t* sr = sl + 24;
      uint32_t st[8];
      auto get = [&](int P, int i) -> uint32_t { return P < 3 ? sl[8 * P + i] : sr[8 * (P - 3) + i]; };
      sha_node_msg(get, st);
      uint32_t rmn[8];
#pragma unroll
      for (int i = 0; i < 8; i++) rmn[i] = sr[i];
      const bool rpar = ns_is_parity(rmn);
#pragma unroll
      for (int i = 0; i < 8; i++) {
        out[i] = sl[i];
        out[8 + i] = rpar ? sl[8 + i] : sr[8 + i];
        out[16 + i] = bswap32(st[i]);
      }
    }
    __syncthreads();
    if (active) {
      uint4* slot = (uint4*)(lds + ((long)tl * half + q) * 24);
#pragma unroll
      for (int i = 0; i < 6; i++) slot[i] = make_uint4(out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]);
    }
    __syncthreads();
  }

  // ---- write roots (90 B each) ----
  for (int e = g; e < tpw * kNodeSize; e += kTreeThreads) {
    const int tl = e / kNodeSize, b = e - tl * kNodeSize;
    const long t = tree0 + tl;
    if (t >= ntrees) continue;
    const long sq = t / (2L * w);
    const int axis = (int)((t / w) & 1);
    const int idx = (int)(t % w);
    const uint32_t* slot = lds + (long)tl * half * 24;
    int word, byte;
    if (b < 29) { word = b >> 2; byte = b & 3; }
    else if (b < 58) { word = 8 + ((b - 29) >> 2); byte = (b - 29) & 3; }
    else { word = 16 + ((b - 58) >> 2); byte = (b - 58) & 3; }
    uint8_t* dst = (axis == 0 ? a.row_roots : a.col_roots) + (sq * w + idx) * kNodeSize;
    dst[b] = (uint8_t)(slot[word] >> (8 * byte));
  }
}

// ---------------------------------------------------------------------------
// Kernel 3: DAH = RFC-6962 root over rowRoots || colRoots (2w items of 90 B).
// leaf = SHA256(0x00 | root) (91 B, 2 blocks); inner = SHA256(0x01 | l | r).
// ---------------------------------------------------------------------------
constexpr int kDahThreads = 256;

__global__ __launch_bounds__(kDahThreads) void dah_kernel(SquareArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];  // n * 8 dwords
  const long sq = blockIdx.x;
  const int w = 2 * a.k;
  const int n = 2 * w;
  for (int i = threadIdx.x; i < n; i += kDahThreads) {
    const uint8_t* root = (i < w ? a.row_roots + (sq * w + i) * kNodeSize
                                 : a.col_roots + (sq * w + (i - w)) * kNodeSize);
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
    for (int j = 0; j < 8; j++) lds[i * 8 + j] = bswap32(st[j]);
  }
  __syncthreads();
  int cur = n;
  while (cur > 1) {
    const int next = cur / 2;
    uint32_t keep[2][8];
    int cnt = 0;
    for (int i = threadIdx.x; i < next; i += kDahThreads, cnt++) {
      uint32_t m[32];
#pragma unroll
      for (int j = 0; j < 32; j++) m[j] = 0;
      uint32_t lft[8], rgt[8];
#pragma unroll
      for (int j = 0; j < 8; j++) { lft[j] = lds[(2 * i) * 8 + j]; rgt[j] = lds[(2 * i + 1) * 8 + j]; }
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
      for (int j = 0; j < 8; j++) keep[cnt & 1][j] = bswap32(st[j]);
    }
    __syncthreads();
    cnt = 0;
    for (int i = threadIdx.x; i < next; i += kDahThreads, cnt++) {
#pragma unroll
      for (int j = 0; j < 8; j++) lds[i * 8 + j] = keep[cnt & 1][j];
    }
    __syncthreads();
    cur = next;
  }
  if (threadIdx.x < 8) {
    uint32_t* dst = (uint32_t*)(a.dah + sq * 32);
    dst[threadIdx.x] = lds[threadIdx.x];
  }
}

hipError_t launch_nmt_leaves(const SquareArgs& a, hipStream_t s) {
  const long w = 2L * a.k;
  const long total = w * w * a.nsq;
  const long blocks = (total + 255) / 256;
  hipLaunchKernelGGL(nmt_leaf_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_nmt_trees(const SquareArgs& a, hipStream_t s) {
  const int w = 2 * a.k;
  if (w > 512) return hipErrorInvalidValue;
  const int tpw = 512 / w;
  const long ntrees = a.nsq * 2L * w;
  const long blocks = (ntrees + tpw - 1) / tpw;
  const size_t lds = (size_t)kTreeThreads * 24 * sizeof(uint32_t);
  hipLaunchKernelGGL(nmt_tree_kernel, dim3((unsigned)blocks), dim3(kTreeThreads), lds, s, a, tpw);
  return hipGetLastError();
}

hipError_t launch_dah(const SquareArgs& a, hipStream_t s) {
  const int n = 4 * a.k;
  if (n > 2 * kDahThreads * 2) return hipErrorInvalidValue;  // keep[2] per thread
  const size_t lds = (size_t)n * 8 * sizeof(uint32_t);
  hipLaunchKernelGGL(dah_kernel, dim3((unsigned)a.nsq), dim3(kDahThreads), lds, s, a);
  return hipGetLastError();
}

}  // namespace dagpu
