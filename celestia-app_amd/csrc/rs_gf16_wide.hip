// rs_gf16_wide.hip -- Leopard GF(2^16) encode / reconstruct for wide squares,
// k = 1024 .. kMaxK (2k = 2048 .. 16384 shards per vector), and for codec
// vectors up to kMaxCodecK (2k = 65536 shards, Leopard's whole field).
//
// Replaces klauspost/reedsolomon v1.11.8 leopardFF16 encode / reconstruct
// (leopard.go), which rsmt2d v0.11.0 LeoRSCodec uses for every width above
// 128; pkg/da/data_availability_header.go:65-75
// ExtendShares itself puts no upper bound on k.  Same arithmetic as the
// register-resident k = 256 / 512 kernels (rs_gf16.hip): a symbol is the byte
// pair (b[i], b[i+32]) of a 64-byte block, IFFT/FFT butterflies with the
// fftSkew multipliers, formal derivative and errLocs multiplies for decode.
// Parity unpinned (no reference vector beyond k = 128): checked against the
// oracle's GF(2^16) restatement and by erase/decode round trips.
//
// Layout.  At these widths one transform (m = k or n = 2k elements) does not
// fit in registers: a workgroup keeps the elements of ONE column slice of ONE
// vector in LDS -- S symbols of every element (S = 32 / 16 / 8 / 4, chosen so
// the slice stays <= 128 KiB) as a low-byte plane and a high-byte plane of
// dwords (4 symbols per dword, element-major, one pad dword per element
// against bank conflicts).  Codec vectors past the widest square (n = 32768 /
// 65536 elements) keep 2 / 1 symbols per element, low and high bytes packed in
// one dword / one 16-bit word (PK = 2 / 1); registers hold them as the same
// lo / hi dwords with zero upper bytes, which every multiply keeps zero.  Each butterfly stage is one pass of radix-4 units
// (4 elements x G dword groups per lane, both layers of the radix-4 step in
// registers, one barrier per stage).  A multiply by a skew constant is the
// 16-dword product table of that skew position (the products of every 2-bit
// group of a symbol, low and high bytes, for v_perm; 1 MiB for all positions
// < 2 kMaxCodecK), loaded once per unit and applied to its G groups.  The decoder's
// per-element errLocs multiplies use one product table per element (exp gathers;
// log/exp gathers per symbol at 4 symbols per element).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <vector>

#include "gf16_host.hpp"
#include "kernels.hpp"
#include "sha256.hpp"

namespace dagpu {

namespace {

constexpr uint32_t kMod = 65535u;
// Threads per workgroup: 512 (8 waves); round 6: the decoders of n >= 4096
// elements 1,024 (16 waves, so that the one workgroup a CU holds -- its LDS slice
// takes up to 160 KiB -- has 4 waves per SIMD to hide its LDS and table latency:
// k = 2048 Repair 18.2 -> 20.2 squares/s; at n = 2048 a wash, and the encoder at
// 1,024 threads slowed the k = 1024 split square 5.0 -> 6.2 ms;
// profiles/gf16_wide_ab_r06.log).
constexpr int kWideThreads = 512;
template <int NG>
constexpr int dec_threads() { return NG <= 4 ? 1024 : 512; }  // (packed slices: NG = 1)
constexpr int kPtabPos = 2 * kMaxCodecK;  // skew positions used by any transform <= 2 kMaxCodecK

struct WideTabs {
  const uint16_t* log;
  const uint16_t* exp;
  const uint32_t* ptab;   // kPtabPos x kTabW dwords
  const uint16_t* wfold;  // folded Walsh weights, n = 2048 .. 2 kMaxCodecK, back to back
};

__device__ __forceinline__ uint32_t xor3w(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// x ^= y * skew[pos] for 4 symbols (lo / hi byte dwords) with the position's
// product table t[kTabW] in registers: the 3/3/2 bit split of rs_gf16.hip
// mul16x_add_t (round 5; 12 v_perm per 4 symbols instead of 16).  Table:
// [0,1] / [2,3] group 0 (y bits 0-2) -> product lo / hi byte, [4..7] group 1
// (bits 3-5), [8] / [9] group 2 (bits 6-7), [10..13] group 3 (bits 8-10),
// [14..17] group 4 (bits 11-13), [18] / [19] group 5 (bits 14-15).
constexpr int kTabW = 20;
__device__ __forceinline__ void pmul_add(uint32_t& xlo, uint32_t& xhi, uint32_t ylo, uint32_t yhi,
                                         const uint32_t (&t)[kTabW]) {
  const uint32_t s0 = ylo & 0x07070707u, s1 = (ylo >> 3) & 0x07070707u, s2 = (ylo >> 6) & 0x03030303u;
  const uint32_t s3 = yhi & 0x07070707u, s4 = (yhi >> 3) & 0x07070707u, s5 = (yhi >> 6) & 0x03030303u;
  const uint32_t l0 = __builtin_amdgcn_perm(t[1], t[0], s0), h0 = __builtin_amdgcn_perm(t[3], t[2], s0);
  const uint32_t l1 = __builtin_amdgcn_perm(t[5], t[4], s1), h1 = __builtin_amdgcn_perm(t[7], t[6], s1);
  const uint32_t l2 = __builtin_amdgcn_perm(t[8], t[8], s2), h2 = __builtin_amdgcn_perm(t[9], t[9], s2);
  const uint32_t l3 = __builtin_amdgcn_perm(t[11], t[10], s3), h3 = __builtin_amdgcn_perm(t[13], t[12], s3);
  const uint32_t l4 = __builtin_amdgcn_perm(t[15], t[14], s4), h4 = __builtin_amdgcn_perm(t[17], t[16], s4);
  const uint32_t l5 = __builtin_amdgcn_perm(t[18], t[18], s5), h5 = __builtin_amdgcn_perm(t[19], t[19], s5);
  xlo = xor3w(xor3w(xor3w(xlo, l0, l1), l2, l3), l4, l5);
  xhi = xor3w(xor3w(xor3w(xhi, h0, h1), h2, h3), h4, h5);
}

// The only zero skews (log 0) below 2^14 sit at positions 2^m - 1 (Leopard
// skips their multiply): the block at offset 0 of every layer, all of the top
// layer.  Leopard's initFFTSkew zeroes FFTSkew[2^m - 1] only for m <= kBits - 2
// = 14 (position 32767 has a nonzero skew), so the bit test is used only below
// 2^14; a position above (ZG: transforms that reach past 2^14 positions, the
// codec vectors past k = 8192) always multiplies, by its table, which is all
// zero where the skew is log 0 (tables() below), so a zero skew there still
// adds nothing.  Square transforms (m, n <= 16384) stay below 2^14.
template <bool ZG>
__device__ __forceinline__ bool zero_skew(int pos) {
  return (!ZG || pos < (1 << 14)) && ((pos + 1) & pos) == 0;
}
__device__ __forceinline__ void load_tab(const WideTabs& T, int pos, uint32_t (&t)[kTabW]) {
  const uint4* p = (const uint4*)(T.ptab + (long)pos * kTabW);
#pragma unroll
  for (int i = 0; i < kTabW / 4; i++) {
    const uint4 v = p[i];
    t[4 * i] = v.x;
    t[4 * i + 1] = v.y;
    t[4 * i + 2] = v.z;
    t[4 * i + 3] = v.w;
  }
}

// The product table (pmul_add format) of exp(lm), for the decoder's per-element
// errLocs multiplies (round 5): the 16 products (1 << b) * exp(lm) (logs of the
// basis from uniform loads, 16 independent exp gathers), then each 3-bit
// group's entries 0..3 = (0, p0, p1, p0 ^ p1) and 4..7 = those ^ p2, packed by
// v_perm (rs_gf16.hip mul16x_table_to, checked in tests/test_halflane_emu.py).
// It replaces a log and an exp gather per symbol (8 dependent gathers per 4
// symbols) with 2 per 4 symbols, all independent.
__device__ __forceinline__ void elem_tab(const WideTabs& T, uint32_t lm, uint32_t (&t)[kTabW]) {
  uint32_t pb[16];
#pragma unroll
  for (int b = 0; b < 16; b++) {
    uint32_t sidx = (uint32_t)T.log[1u << b] + lm;
    sidx = (sidx + (sidx >> 16)) & 0xFFFFu;
    pb[b] = T.exp[sidx];
  }
  auto quad = [&](uint32_t p0, uint32_t p1, uint32_t& lo, uint32_t& hi) {
    const uint32_t q = p0 ^ p1;
    lo = __builtin_amdgcn_perm(q, __builtin_amdgcn_perm(p1, p0, 0x0C04000Cu), 0x04020100u);
    hi = __builtin_amdgcn_perm(q, __builtin_amdgcn_perm(p1, p0, 0x0C05010Cu), 0x05020100u);
  };
  auto grp3 = [&](int b0, int base) {
    uint32_t lo, hi;
    quad(pb[b0], pb[b0 + 1], lo, hi);
    t[base] = lo;
    t[base + 1] = lo ^ __builtin_amdgcn_perm(pb[b0 + 2], pb[b0 + 2], 0x00000000u);
    t[base + 2] = hi;
    t[base + 3] = hi ^ __builtin_amdgcn_perm(pb[b0 + 2], pb[b0 + 2], 0x01010101u);
  };
  grp3(0, 0);
  grp3(3, 4);
  quad(pb[6], pb[7], t[8], t[9]);
  grp3(8, 10);
  grp3(11, 14);
  quad(pb[14], pb[15], t[18], t[19]);
}

// The same table from the element's 16 basis products (1 << b) * exp(lm), as
// leo16w_errlocs_kernel stores them (round 6: two 16-B loads, no gathers).
__device__ __forceinline__ void elem_tab_pb(const uint8_t* pb32, uint32_t (&t)[kTabW]) {
  const uint4 u0 = ((const uint4*)pb32)[0], u1 = ((const uint4*)pb32)[1];
  const uint32_t w[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
  uint32_t pb[16];
#pragma unroll
  for (int b = 0; b < 16; b++) pb[b] = (w[b >> 1] >> (16 * (b & 1))) & 0xFFFFu;
  auto quad = [&](uint32_t p0, uint32_t p1, uint32_t& lo, uint32_t& hi) {
    const uint32_t q = p0 ^ p1;
    lo = __builtin_amdgcn_perm(q, __builtin_amdgcn_perm(p1, p0, 0x0C04000Cu), 0x04020100u);
    hi = __builtin_amdgcn_perm(q, __builtin_amdgcn_perm(p1, p0, 0x0C05010Cu), 0x05020100u);
  };
  auto grp3 = [&](int b0, int base) {
    uint32_t lo, hi;
    quad(pb[b0], pb[b0 + 1], lo, hi);
    t[base] = lo;
    t[base + 1] = lo ^ __builtin_amdgcn_perm(pb[b0 + 2], pb[b0 + 2], 0x00000000u);
    t[base + 2] = hi;
    t[base + 3] = hi ^ __builtin_amdgcn_perm(pb[b0 + 2], pb[b0 + 2], 0x01010101u);
  };
  grp3(0, 0);
  grp3(3, 4);
  quad(pb[6], pb[7], t[8], t[9]);
  grp3(8, 10);
  grp3(11, 14);
  quad(pb[14], pb[15], t[18], t[19]);
}

// (lo, hi) *= the element's factor through its table from the basis products
template <int NG>
__device__ __forceinline__ void mul_elem_pb(const uint8_t* pb32, uint32_t (&lo)[NG], uint32_t (&hi)[NG]) {
  uint32_t t[kTabW];
  elem_tab_pb(pb32, t);
#pragma unroll
  for (int g = 0; g < NG; g++) {
    uint32_t rl = 0, rh = 0;
    pmul_add(rl, rh, lo[g], hi[g], t);
    lo[g] = rl;
    hi[g] = rh;
  }
}

// mulLog on one 16-bit symbol (leopard.go mulLog): a * exp(lm), 0 stays 0
__device__ __forceinline__ uint32_t mul_log(const WideTabs& T, uint32_t a, uint32_t lm) {
  if (a == 0) return 0;
  uint32_t s = (uint32_t)T.log[a] + lm;
  s = (s + (s >> 16)) & 0xFFFFu;
  return T.exp[s];
}

// (lo, hi) *= exp(lm) for one element's NG dword pairs: NG >= 2 through the
// element's product table (16 gathers, k = 1024 Repair 45.9 -> 75.2 squares/s,
// profiles/gf16_widedec_ab_r05.log); NG = 1 (n >= 8192: 4 symbols per element)
// by log/exp gathers per symbol (8, fewer than the table's 16).
template <int NG>
__device__ __forceinline__ void mul_elem(const WideTabs& T, uint32_t (&lo)[NG], uint32_t (&hi)[NG], uint32_t lm) {
  if constexpr (NG >= 2) {
    uint32_t t[kTabW];
    elem_tab(T, lm, t);
#pragma unroll
    for (int g = 0; g < NG; g++) {
      uint32_t rl = 0, rh = 0;
      pmul_add(rl, rh, lo[g], hi[g], t);
      lo[g] = rl;
      hi[g] = rh;
    }
  } else {
#pragma unroll
    for (int g = 0; g < NG; g++) {
      uint32_t rl = 0, rh = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const uint32_t sym = ((lo[g] >> (8 * b)) & 0xFFu) | (((hi[g] >> (8 * b)) & 0xFFu) << 8);
        const uint32_t p = mul_log(T, sym, lm);
        rl |= (p & 0xFFu) << (8 * b);
        rh |= (p >> 8) << (8 * b);
      }
      lo[g] = rl;
      hi[g] = rh;
    }
  }
}

// LDS planes: lo[e * NGP + g], hi[...] (NG = S / 4 dword groups, NGP = NG + 1
// for odd element strides, so lanes on different elements spread over banks;
// NG = 2 is used only at n = 8192, where a pad dword would not fit 160 KiB).
// PK = 2 / 1 (NG = 1): one packed word per element, lo[e] = lo16 | hi16 << 16
// (2 symbols) or ((uint16_t*)lo)[e] = lo8 | hi8 << 8 (1 symbol); hi unused.
template <int NG_, int PK_ = 0>
struct Planes {
  static constexpr int NG = NG_, PK = PK_;
  static_assert(PK == 0 || NG == 1, "packed slices hold one group");
  static constexpr int NGP = NG <= 2 ? NG : NG + 1;
  static constexpr int SYM = PK ? PK : 4 * NG;  // symbols per element in the slice
  uint32_t* lo;
  uint32_t* hi;
  __device__ __forceinline__ int at(int e, int g) const { return e * NGP + g; }
  __device__ __forceinline__ void get(int e, int g, uint32_t& l, uint32_t& h) const {
    if constexpr (PK == 0) {
      l = lo[at(e, g)];
      h = hi[at(e, g)];
    } else if constexpr (PK == 2) {
      const uint32_t d = lo[e];
      l = d & 0xFFFFu;
      h = d >> 16;
    } else {
      const uint32_t d = ((const uint16_t*)lo)[e];
      l = d & 0xFFu;
      h = d >> 8;
    }
  }
  __device__ __forceinline__ void put(int e, int g, uint32_t l, uint32_t h) const {
    if constexpr (PK == 0) {
      lo[at(e, g)] = l;
      hi[at(e, g)] = h;
    } else if constexpr (PK == 2) {
      lo[e] = l | (h << 16);
    } else {
      ((uint16_t*)lo)[e] = (uint16_t)(l | (h << 8));
    }
  }
  // LDS bytes of an n-element slice
  static constexpr size_t bytes(int n) { return PK ? (size_t)n * PK * 2 : (size_t)2 * n * NGP * 4; }
};

// Global memory side of a slice group: p is the group's low-byte dword (4
// symbols at b[i], high bytes at b[i + 32]), or for packed slices its 2 / 1
// low bytes.
template <int PK>
__device__ __forceinline__ void gload(const uint8_t* p, uint32_t& lo, uint32_t& hi) {
  if constexpr (PK == 0) {
    lo = ((const uint32_t*)p)[0];
    hi = ((const uint32_t*)p)[8];
  } else if constexpr (PK == 2) {
    lo = ((const uint16_t*)p)[0];
    hi = ((const uint16_t*)p)[16];
  } else {
    lo = p[0];
    hi = p[32];
  }
}
template <int PK>
__device__ __forceinline__ void gstore(uint8_t* p, uint32_t lo, uint32_t hi) {
  if constexpr (PK == 0) {
    ((uint32_t*)p)[0] = lo;
    ((uint32_t*)p)[8] = hi;
  } else if constexpr (PK == 2) {
    ((uint16_t*)p)[0] = (uint16_t)lo;
    ((uint16_t*)p)[16] = (uint16_t)hi;
  } else {
    p[0] = (uint8_t)lo;
    p[32] = (uint8_t)hi;
  }
}
template <int PK>
__device__ __forceinline__ bool gdiffers(const uint8_t* p, uint32_t lo, uint32_t hi) {
  uint32_t l, h;
  gload<PK>(p, l, h);
  return l != lo || h != hi;
}

// One radix-4 (or radix-2) unit: elements e[0..R), dword groups g0 .. g0+G-1.
template <class PL, int G, int R>
struct Unit {
  uint32_t lo[R][G], hi[R][G];
  __device__ __forceinline__ void load(const PL& P, const int (&e)[R], int g0) {
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
      for (int g = 0; g < G; g++) P.get(e[r], g0 + g, lo[r][g], hi[r][g]);
  }
  __device__ __forceinline__ void store(const PL& P, const int (&e)[R], int g0) const {
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
      for (int g = 0; g < G; g++) P.put(e[r], g0 + g, lo[r][g], hi[r][g]);
  }
  // ifftDIT2: y ^= x; x ^= y * skew (zero: the skew is log 0, no multiply)
  __device__ __forceinline__ void ifft2(int i, int j, const uint32_t (&t)[kTabW], bool zero) {
#pragma unroll
    for (int g = 0; g < G; g++) {
      lo[j][g] ^= lo[i][g];
      hi[j][g] ^= hi[i][g];
    }
    if (!zero) {
#pragma unroll
      for (int g = 0; g < G; g++) pmul_add(lo[i][g], hi[i][g], lo[j][g], hi[j][g], t);
    }
  }
  // fftDIT2: x ^= y * skew; y ^= x
  __device__ __forceinline__ void fft2(int i, int j, const uint32_t (&t)[kTabW], bool zero) {
    if (!zero) {
#pragma unroll
      for (int g = 0; g < G; g++) pmul_add(lo[i][g], hi[i][g], lo[j][g], hi[j][g], t);
    }
#pragma unroll
    for (int g = 0; g < G; g++) {
      lo[j][g] ^= lo[i][g];
      hi[j][g] ^= hi[i][g];
    }
  }
};

// A skew table from a wave-uniform position: scalar loads (constant address
// space), so the table sits in SGPRs instead of five 16-B vector loads per lane.
typedef const __attribute__((address_space(4))) uint32_t* ConstTab;
template <int N>
__device__ __forceinline__ void load_tab_u(const WideTabs& T, int pos, uint32_t (&t)[N]) {
  const ConstTab p = (ConstTab)(T.ptab + (long)__builtin_amdgcn_readfirstlane(pos) * kTabW);
#pragma unroll
  for (int i = 0; i < kTabW; i++) t[i] = p[i];
}

// One radix-4 IFFT step (dist, dist4 = 4 dist) over all units.  UNI: the 64
// units of a wave lie in one block of 4 dist elements (dist * CH >= 64), so
// their three skew positions are wave-uniform and the tables come by scalar loads.
template <class PL, int G, bool UNI, int TH, bool ZG>
__device__ __forceinline__ void ifft_step(const PL& P, const WideTabs& T, int n, int base, int dist) {
  constexpr int CH = PL::NG / G;
  const int dist4 = dist << 2;
  const int units = (n / 4) * CH;
  uint32_t t[kTabW];
  for (int u = threadIdx.x; u < units; u += TH) {
    const int quad = u / CH, g0 = (u - quad * CH) * G;
    const int r = (quad / dist) * dist4, i = r + (quad % dist), iend = r + dist;
    const int e[4] = {i, i + dist, i + 2 * dist, i + 3 * dist};
    Unit<PL, G, 4> x;
    x.load(P, e, g0);
    auto tab = [&](int pos) {
      if constexpr (UNI) load_tab_u(T, pos, t);
      else load_tab(T, pos, t);
    };
    bool z = zero_skew<ZG>(base + iend);
    if (!z) tab(base + iend);
    x.ifft2(0, 1, t, z);
    z = zero_skew<ZG>(base + iend + 2 * dist);
    if (!z) tab(base + iend + 2 * dist);
    x.ifft2(2, 3, t, z);
    z = zero_skew<ZG>(base + iend + dist);
    if (!z) tab(base + iend + dist);
    x.ifft2(0, 2, t, z);
    x.ifft2(1, 3, t, z);
    x.store(P, e, g0);
  }
  __syncthreads();
}

// ifftDITEncoder / ifftDITDecoder over n elements (mtrunc = n), skew index
// base + iend (encoder: base = IO - 1; decoder: -1)
template <class PL, int G, int TH, bool ZG>
__device__ void wide_ifft(const PL& P, const WideTabs& T, int n, int base) {
  constexpr int CH = PL::NG / G;
  int dist = 1, dist4 = 4;
  while (dist4 <= n) {
    if (dist * CH >= 64) ifft_step<PL, G, true, TH, ZG>(P, T, n, base, dist);
    else ifft_step<PL, G, false, TH, ZG>(P, T, n, base, dist);
    dist = dist4;
    dist4 <<= 2;
  }
  if (dist < n) {  // one radix-2 layer left (log2 n odd): one position for all
    const int units = (n / 2) * CH;
    uint32_t t[kTabW];
    const bool z = zero_skew<ZG>(base + dist);
    if (!z) load_tab_u(T, base + dist, t);
    for (int u = threadIdx.x; u < units; u += TH) {
      const int p = u / CH, g0 = (u - p * CH) * G;
      const int e[2] = {p, p + dist};
      Unit<PL, G, 2> x;
      x.load(P, e, g0);
      x.ifft2(0, 1, t, z);
      x.store(P, e, g0);
    }
    __syncthreads();
  }
}

// One radix-4 FFT step (fftDIT, skew index fo + iend - 1); UNI as ifft_step.
template <class PL, int G, bool UNI, int TH, bool ZG>
__device__ __forceinline__ void fft_step(const PL& P, const WideTabs& T, int n, int fo, int dist) {
  constexpr int CH = PL::NG / G;
  const int dist4 = dist << 2;
  const int units = (n / 4) * CH;
  uint32_t t[kTabW];
  for (int u = threadIdx.x; u < units; u += TH) {
    const int quad = u / CH, g0 = (u - quad * CH) * G;
    const int r = (quad / dist) * dist4, i = r + (quad % dist), iend = r + dist;
    const int e[4] = {i, i + dist, i + 2 * dist, i + 3 * dist};
    Unit<PL, G, 4> x;
    x.load(P, e, g0);
    auto tab = [&](int pos) {
      if constexpr (UNI) load_tab_u(T, pos, t);
      else load_tab(T, pos, t);
    };
    bool z = zero_skew<ZG>(fo + iend + dist - 1);
    if (!z) tab(fo + iend + dist - 1);
    x.fft2(0, 2, t, z);
    x.fft2(1, 3, t, z);
    z = zero_skew<ZG>(fo + iend - 1);
    if (!z) tab(fo + iend - 1);
    x.fft2(0, 1, t, z);
    z = zero_skew<ZG>(fo + iend + 2 * dist - 1);
    if (!z) tab(fo + iend + 2 * dist - 1);
    x.fft2(2, 3, t, z);
    x.store(P, e, g0);
  }
  __syncthreads();
}

// fftDIT over n elements (mtrunc = n), skew index fo + iend - 1
template <class PL, int G, int TH, bool ZG>
__device__ void wide_fft(const PL& P, const WideTabs& T, int n, int fo) {
  constexpr int CH = PL::NG / G;
  int dist4 = n, dist = n >> 2;
  while (dist != 0) {
    if (dist * CH >= 64) fft_step<PL, G, true, TH, ZG>(P, T, n, fo, dist);
    else fft_step<PL, G, false, TH, ZG>(P, T, n, fo, dist);
    dist4 = dist;
    dist >>= 2;
  }
  if (dist4 == 2) {
    const int units = (n / 2) * CH;
    uint32_t t[kTabW];
    for (int u = threadIdx.x; u < units; u += TH) {
      const int p = u / CH, g0 = (u - p * CH) * G;
      const int e[2] = {2 * p, 2 * p + 1};
      const bool z = zero_skew<ZG>(fo + 2 * p);
      if (!z) load_tab(T, fo + 2 * p, t);
      Unit<PL, G, 2> x;
      x.load(P, e, g0);
      x.fft2(0, 1, t, z);
      x.store(P, e, g0);
    }
    __syncthreads();
  }
}

// Column slice of a workgroup: blockIdx -> (vector v, 64-B block, slice of
// S symbols: 4 NG, or PK for packed slices).  Consecutive logical blocks (the slices and blocks of one
// vector, which share cache lines) are kept on one XCD: hardware dispatch
// deals workgroups round-robin over the 8 XCDs.
struct SliceCoord {
  long v, blk;
  int sl;
};
template <int S>
__device__ __forceinline__ SliceCoord slice_of(long nblk) {
  constexpr int nsl = 32 / S;
  long b = blockIdx.x;
  const long G = gridDim.x;
  if ((G & 7) == 0) b = (b & 7) * (G >> 3) + (b >> 3);
  SliceCoord c;
  c.sl = (int)(b % nsl);
  b /= nsl;
  c.blk = b % nblk;
  c.v = b / nblk;
  return c;
}

// ---------------------------------------------------------------------------
// Encode: parity = FFT_m(IFFT_m(data)), m = k.  EncodeArgs semantics as the
// other encoders: Q0 placement copy, compare mode (mismatch), Repair fill
// (out_present / redo), reverse fill (IFFT at skew offset 0, FFT at m).
// ---------------------------------------------------------------------------
template <int NG, int G, int PK = 0>
__global__ __launch_bounds__(kWideThreads) void leo16w_encode_kernel(EncodeArgs a, WideTabs T, int k) {
  using PL = Planes<NG, PK>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  PL P{lds, lds + k * PL::NGP};
  const SliceCoord c = slice_of<PL::SYM>(a.shard_bytes / 64);
  const long sq = c.v / a.nvec, vec = c.v % a.nvec;
  if (vec_skipped(a, c.v)) return;  // uniform
  const long col = c.blk * 64 + (long)c.sl * PL::SYM;  // byte of lo dword 0 of this slice
  const uint8_t* in = a.in + sq * a.in_sq_stride + vec * a.in_vec_stride + col;
  uint8_t* cp = a.copy ? a.copy + sq * a.copy_sq_stride + vec * a.copy_vec_stride + col : nullptr;
  for (int t = threadIdx.x; t < k * NG; t += kWideThreads) {
    const int e = t / NG, g = t - e * NG;
    uint32_t lo, hi;
    gload<PK>(in + (long)e * a.in_shard_stride + 4 * g, lo, hi);
    P.put(e, g, lo, hi);
    if (cp) gstore<PK>(cp + (long)e * a.copy_shard_stride + 4 * g, lo, hi);
  }
  __syncthreads();
  // positions up to 2k - 2: past 2^14 only for k >= 16384 (NG = 1 or packed)
  constexpr bool ZG = NG == 1;
  wide_ifft<PL, G, kWideThreads, ZG>(P, T, k, a.reverse ? -1 : k - 1);
  wide_fft<PL, G, kWideThreads, ZG>(P, T, k, a.reverse ? k : 0);
  uint8_t* out = a.out + sq * a.out_sq_stride + vec * a.out_vec_stride + col;
  bool diff = false;
  for (int t = threadIdx.x; t < k * NG; t += kWideThreads) {
    const int e = t / NG, g = t - e * NG;
    uint32_t lo, hi;
    P.get(e, g, lo, hi);
    uint8_t* dst = out + (long)e * a.out_shard_stride + 4 * g;
    if (a.mismatch || (a.out_present && fill_given(a, sq, vec, e))) {
      diff |= gdiffers<PK>(dst, lo, hi);
    } else {
      gstore<PK>(dst, lo, hi);
    }
  }
  if (a.mismatch && diff) {
    atomicOr(a.mismatch + sq, a.mismatch_bit);
    if (a.mismatch_vec) a.mismatch_vec[sq * a.nvec + vec] = 1;
  }
  if (a.out_present && !a.mismatch && diff) a.redo[c.v] = 1;  // Repair fill: a given shard differs
}

// ---------------------------------------------------------------------------
// Error locators (leopard.go reconstruct, first part) from n-point transforms:
// FWHT_n(FWHT_n(e) * wfold), wfold[r] = sum_q logWalsh[q n + r] mod 65535
// (see rs_gf16.hip leo16_errlocs_fold_kernel; n = 2k up to 2 kMaxCodecK here:
// ET = uint32_t LDS words up to n = 32768, uint16_t at 65536 -- every value is
// a residue mod 65535, so 16 bits hold it -- both 128 KiB).
// ---------------------------------------------------------------------------
constexpr int kFoldThreads = 512;

__device__ __forceinline__ uint32_t add_mod(uint32_t a, uint32_t b) {
  const uint32_t s = a + b;
  return (s + (s >> 16)) & 0xFFFFu;
}
__device__ __forceinline__ uint32_t sub_mod(uint32_t a, uint32_t b) {
  const uint32_t d = a - b;
  return (d + (d >> 16)) & 0xFFFFu;
}

template <typename ET>
__device__ void fwht_rt(ET* e, int n) {
  int dist = 1;
  if ((__builtin_ctz(n) & 1) != 0) {  // odd log2: one radix-2 stage first
    for (int g = threadIdx.x; g < n / 2; g += kFoldThreads) {
      const int i = 2 * g;
      const uint32_t t0 = e[i], t1 = e[i + 1];
      e[i] = (ET)add_mod(t0, t1);
      e[i + 1] = (ET)sub_mod(t0, t1);
    }
    __syncthreads();
    dist = 2;
  }
  for (; dist < n; dist <<= 2) {
    const int dist4 = dist << 2;
    for (int g = threadIdx.x; g < n / 4; g += kFoldThreads) {
      const int r = (g / dist) * dist4;
      const int i = r + (g % dist);
      const uint32_t t0 = e[i], t1 = e[i + dist], t2 = e[i + 2 * dist], t3 = e[i + 3 * dist];
      const uint32_t a0 = add_mod(t0, t1), a1 = sub_mod(t0, t1);
      const uint32_t a2 = add_mod(t2, t3), a3 = sub_mod(t2, t3);
      e[i] = (ET)add_mod(a0, a2);
      e[i + 2 * dist] = (ET)sub_mod(a0, a2);
      e[i + dist] = (ET)add_mod(a1, a3);
      e[i + 3 * dist] = (ET)sub_mod(a1, a3);
    }
    __syncthreads();
  }
}

template <typename ET>
__global__ __launch_bounds__(kFoldThreads) void leo16w_errlocs_kernel(DecodeArgs a, WideTabs T, long wf_off) {
  extern __shared__ __attribute__((aligned(16))) uint32_t e_lds[];
  ET* e = (ET*)e_lds;
  // bit r of miss: element threadIdx.x + r * kFoldThreads is missing (n <= 64 *
  // kFoldThreads; the 16-bit build, n = 65536, reads the presence bytes again)
  constexpr bool kMissBits = sizeof(ET) == 4;
  __shared__ int cnt_s;
  const long v = blockIdx.x;
  const long sq = v / a.nvec, vec = v % a.nvec;
  const int k = a.k, n = 2 * k;
  const uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
  if (a.locators_only && !a.flags[v]) return;  // uniform
  const long hv = err_head_checked_block(a, v);
  if (a.locators_only && !err_computes(a, v, hv)) return;  // uniform
  if (threadIdx.x == 0) cnt_s = 0;
  __syncthreads();
  int cnt = 0;
  uint64_t miss = 0;
  auto missing = [&](int i) -> uint32_t {
    return i < k ? (pres[(long)(k + i) * a.p_shard_stride] ? 0u : 1u)   // parity k+i -> work i
                 : (pres[(long)(i - k) * a.p_shard_stride] ? 0u : 1u);  // data i-k -> work i
  };
  for (int i = threadIdx.x, r = 0; i < n; i += kFoldThreads, r++) {
    const uint32_t x = missing(i);
    e[i] = (ET)x;
    if constexpr (kMissBits) miss |= (uint64_t)x << r;
    cnt += (x == 0);
  }
  atomicAdd(&cnt_s, cnt);
  __syncthreads();
  const int present = cnt_s;
  bool decode = true;
  if (!a.locators_only) {
    decode = present >= k && present < n && vec_selected(a, v);
    if (threadIdx.x == 0) {
      a.flags[v] = decode ? 1 : 0;
      if (present < k && a.too_few) atomicOr(a.too_few, 1);
      if (decode && a.ndecodable) atomicAdd(a.ndecodable, 1);
    }
  }
  if (!decode) return;  // uniform
  if (!err_computes(a, v, hv)) return;  // shares an earlier vector's locators
  fwht_rt(e, n);
  const uint16_t* wf = T.wfold + wf_off;
  for (int i = threadIdx.x; i < n; i += kFoldThreads) e[i] = (ET)(((uint32_t)e[i] * (uint32_t)wf[i]) % kMod);
  __syncthreads();
  fwht_rt(e, n);
  uint16_t* out = (uint16_t*)(a.err + hv * (long)rs_err_bytes(k));
  for (int i = threadIdx.x; i < n; i += kFoldThreads) out[i] = (uint16_t)e[i];
  // Round 6: each element's 16 basis products (1 << b) * exp(+-errLoc) -- the
  // premultiply's factor for a present element, the postmultiply's for a missing
  // one -- once per erasure pattern, so the decoder's workgroups (one per
  // column slice) build their tables from two coalesced 16-B loads instead of
  // 16 random exp gathers per element each.
  if (rs_err_elem_bytes(a.k) == 32) {  // (k = 1024: leo16_errlocs_fold_kernel<2048> writes 80-B tables)
    uint4* pbo = (uint4*)(a.err + hv * (long)rs_err_bytes(k) + rs_err_tab_off(k));
    for (int i = threadIdx.x, r = 0; i < n; i += kFoldThreads, r++) {
      const uint32_t lm0 = (uint32_t)e[i] & 0xFFFFu;
      const bool gone = kMissBits ? ((miss >> r) & 1) != 0 : missing(i) != 0;
      const uint32_t lm = gone ? kMod - lm0 : lm0;
      uint32_t p[8];
#pragma unroll
      for (int b = 0; b < 16; b += 2) {
        uint32_t s0 = (uint32_t)T.log[1u << b] + lm, s1 = (uint32_t)T.log[1u << (b + 1)] + lm;
        s0 = (s0 + (s0 >> 16)) & 0xFFFFu;
        s1 = (s1 + (s1 >> 16)) & 0xFFFFu;
        p[b / 2] = (uint32_t)T.exp[s0] | ((uint32_t)T.exp[s1] << 16);
      }
      pbo[2 * i] = make_uint4(p[0], p[1], p[2], p[3]);
      pbo[2 * i + 1] = make_uint4(p[4], p[5], p[6], p[7]);
    }
  }
}

// ---------------------------------------------------------------------------
// Decode: work[i] = shard(pos(i)) * errLocs[i] (0 where missing; layout
// [parity k][data k]) -> ifftDITDecoder -> formal derivative -> fftDIT ->
// erased shard = work[pos] * (65535 - errLocs[pos]).
// The formal derivative D(x)_e = x_e ^ XOR_{b: bit b of e == 0} x_{e + 2^b}
// (the closed form of leopard.go's in-place loop) runs in place: it only reads
// elements above e, so element chunks are processed in ascending order, each
// reading before a barrier and writing after it.
// ---------------------------------------------------------------------------
template <int NG, int G, int PK = 0, int TH = dec_threads<NG>()>
__global__ __launch_bounds__(TH) void leo16w_decode_kernel(DecodeArgs a, WideTabs T) {
  using PL = Planes<NG, PK>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  constexpr int CH = NG / G;
  const int k = a.k, n = 2 * k;
  PL P{lds, lds + n * PL::NGP};
  const SliceCoord c = slice_of<PL::SYM>(a.shard_bytes / 64);
  const long v = c.v;
  if (a.flags[v] == 0) return;  // uniform
  const long sq = v / a.nvec, vec = v % a.nvec;
  const long col = c.blk * 64 + (long)c.sl * PL::SYM;
  uint8_t* base = a.data + sq * a.sq_stride + vec * a.vec_stride + col;
  const uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
  const uint16_t* err = (const uint16_t*)(a.err + err_vec(a, v) * (long)rs_err_bytes(k));
  // k >= 2048: the basis products leo16w_errlocs_kernel stored per element;
  // k <= 1024 has the register kernels' 80-B tables there (this kernel then
  // reads the locators: DAGPU_GF16_WIDE A/B, shards off the 128-B grid)
  const uint8_t* pbase = rs_err_elem_bytes(k) == 32 ? (const uint8_t*)err + rs_err_tab_off(k) : nullptr;
  // one thread per element: its table once, then its NG dword pairs
  for (int i = threadIdx.x; i < n; i += TH) {
    const long shard = i < k ? k + i : i - k;
    if (pres[shard * a.p_shard_stride]) {
      const uint8_t* src = base + shard * a.shard_stride;
      uint32_t lo[NG], hi[NG];
#pragma unroll
      for (int g = 0; g < NG; g++) gload<PK>(src + 4 * g, lo[g], hi[g]);
      if (pbase) mul_elem_pb<NG>(pbase + (long)i * 32, lo, hi);
      else mul_elem<NG>(T, lo, hi, err[i]);
#pragma unroll
      for (int g = 0; g < NG; g++) P.put(i, g, lo[g], hi[g]);
    } else {
#pragma unroll
      for (int g = 0; g < NG; g++) P.put(i, g, 0u, 0u);
    }
  }
  __syncthreads();
  constexpr bool ZG = PK != 0;  // positions below n - 1: past 2^14 only for n >= 32768 (packed)
  wide_ifft<PL, G, TH, ZG>(P, T, n, -1);
  {  // formal derivative, ascending chunks of X elements
    constexpr int X = TH / CH;
    for (int x0 = 0; x0 < n; x0 += X) {
      const int u = threadIdx.x;
      const int x = x0 + u / CH, g0 = (u % CH) * G;
      uint32_t dl[G], dh[G];
      const bool act = x < n;
      if (act) {
#pragma unroll
        for (int g = 0; g < G; g++) P.get(x, g0 + g, dl[g], dh[g]);
        for (int b = 1; b < n; b <<= 1) {
          if (x & b) continue;
#pragma unroll
          for (int g = 0; g < G; g++) {
            uint32_t l, h;
            P.get(x + b, g0 + g, l, h);
            dl[g] ^= l;
            dh[g] ^= h;
          }
        }
      }
      __syncthreads();
      if (act) {
#pragma unroll
        for (int g = 0; g < G; g++) P.put(x, g0 + g, dl[g], dh[g]);
      }
      __syncthreads();
    }
  }
  wide_fft<PL, G, TH, ZG>(P, T, n, 0);
  for (int i = threadIdx.x; i < n; i += TH) {
    const long shard = i < k ? k + i : i - k;
    if (pres[shard * a.p_shard_stride]) continue;
    uint32_t lo[NG], hi[NG];
#pragma unroll
    for (int g = 0; g < NG; g++) P.get(i, g, lo[g], hi[g]);
    if (pbase) mul_elem_pb<NG>(pbase + (long)i * 32, lo, hi);  // (the stored factor is the postmultiply's)
    else mul_elem<NG>(T, lo, hi, kMod - err[i]);
    uint8_t* dst = base + shard * a.shard_stride;
#pragma unroll
    for (int g = 0; g < NG; g++) gstore<PK>(dst + 4 * g, lo[g], hi[g]);
  }
}

__global__ __launch_bounds__(256) void leo16w_mark_present_kernel(DecodeArgs a) {
  const long v = blockIdx.x;
  if (a.flags[v] == 0) return;
  const long sq = v / a.nvec, vec = v % a.nvec;
  uint8_t* pres = a.present + sq * a.p_sq_stride + vec * a.p_vec_stride;
  for (int i = threadIdx.x; i < 2 * a.k; i += 256) pres[(long)i * a.p_shard_stride] = 1;
  if (threadIdx.x == 0 && a.progress) atomicAdd(a.progress, 1);
}

// ---------------------------------------------------------------------------
// Tables: one device copy per device, built on the host from gf16::make_tables.
// ---------------------------------------------------------------------------
std::mutex g_mu;
WideTabs g_tabs[64];
bool g_done[64];

long wfold_offset(int n) {  // n = 2048, 4096, ...: offsets of the folded tables
  long off = 0;
  for (int m = 2048; m < n; m <<= 1) off += m;
  return off;
}

hipError_t tables(WideTabs& out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> g(g_mu);
  if (g_done[dev]) {
    out = g_tabs[dev];
    return hipSuccess;
  }
  static const gf16::Tables t = gf16::make_tables();
  std::vector<uint32_t> pt((size_t)kPtabPos * kTabW, 0u);
  for (int pos = 0; pos < kPtabPos; pos++) {
    const unsigned lm = t.skew[pos];
    if (lm == kMod) continue;  // leopard skips the multiply: zero table
    static const int shift[6] = {0, 3, 6, 8, 11, 14}, width[6] = {3, 3, 2, 3, 3, 2};
    static const int base[6] = {0, 4, 8, 10, 14, 18};
    uint32_t* o = pt.data() + (size_t)pos * kTabW;
    for (int g = 0; g < 6; g++)
      for (int e2 = 1; e2 < (1 << width[g]); e2++) {
        const unsigned x = (unsigned)e2 << shift[g];
        unsigned s = (unsigned)t.log[x] + lm;
        s = (s + (s >> 16)) & 0xFFFFu;
        const unsigned prod = t.exp[s];
        const int lo_dw = width[g] == 3 ? base[g] + (e2 >> 2) : base[g];
        const int hi_dw = width[g] == 3 ? base[g] + 2 + (e2 >> 2) : base[g] + 1;
        o[lo_dw] |= (prod & 0xFFu) << (8 * (e2 & 3));
        o[hi_dw] |= ((prod >> 8) & 0xFFu) << (8 * (e2 & 3));
      }
  }
  std::vector<uint16_t> wf((size_t)wfold_offset(2 * 2 * kMaxCodecK), 0);
  for (int n = 2048; n <= 2 * kMaxCodecK; n <<= 1) {
    const long off = wfold_offset(n);
    for (int r = 0; r < n; r++) {
      uint64_t acc = 0;
      for (int q = 0; q < 65536 / n; q++) acc += t.walsh[(size_t)q * n + r];
      wf[(size_t)(off + r)] = (uint16_t)(acc % kMod);
    }
  }
  void *d_log = nullptr, *d_exp = nullptr, *d_pt = nullptr, *d_wf = nullptr;
  if ((e = hipMalloc(&d_log, 65536 * 2)) != hipSuccess) return e;
  if ((e = hipMalloc(&d_exp, 65536 * 2)) != hipSuccess) return e;
  if ((e = hipMalloc(&d_pt, pt.size() * 4)) != hipSuccess) return e;
  if ((e = hipMalloc(&d_wf, wf.size() * 2)) != hipSuccess) return e;
  if ((e = hipMemcpy(d_log, t.log.data(), 65536 * 2, hipMemcpyHostToDevice)) != hipSuccess) return e;
  if ((e = hipMemcpy(d_exp, t.exp.data(), 65536 * 2, hipMemcpyHostToDevice)) != hipSuccess) return e;
  if ((e = hipMemcpy(d_pt, pt.data(), pt.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) return e;
  if ((e = hipMemcpy(d_wf, wf.data(), wf.size() * 2, hipMemcpyHostToDevice)) != hipSuccess) return e;
  g_tabs[dev] = WideTabs{(const uint16_t*)d_log, (const uint16_t*)d_exp, (const uint32_t*)d_pt,
                         (const uint16_t*)d_wf};
  g_done[dev] = true;
  out = g_tabs[dev];
  return hipSuccess;
}

// Slice width per element count: S = 4 NG symbols, LDS = 2 planes x n x NGP
// dwords <= 160 KiB.  Round 6: the widest slice that fits (n <= 2048: 32
// symbols, 144 KiB; 4096: 16, 160 KiB; 8192: 8 without the pad dword, 128 KiB;
// 16384: 4, 128 KiB; codec vectors 32768: 2 packed, 128 KiB; 65536: 1 packed,
// 128 KiB), so that every skew table a unit loads, every per-element errLocs
// table and every 64-B block's load serve more symbols (round 5: 8 / 4 symbols
// at n = 4096 / 8192; profiles/gf16_wide_ab_r06.log).
int slice_sym(int n) {
  return n <= 2048 ? 32 : n <= 4096 ? 16 : n <= 8192 ? 8 : n <= 16384 ? 4 : n <= 32768 ? 2 : 1;
}

size_t lds_bytes(int n, int ng) {
  const int ngp = ng <= 2 ? ng : ng + 1;  // Planes<NG>::NGP
  return (size_t)2 * n * ngp * sizeof(uint32_t);
}

template <class K>
hipError_t lds_attr(K kernel, size_t bytes) {
  return bytes > 65536 ? hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)bytes)
                       : hipSuccess;
}

template <int NG, int G, int PK = 0>
hipError_t launch_enc(const EncodeArgs& a, const WideTabs& T, int k, hipStream_t s) {
  using PL = Planes<NG, PK>;
  const size_t lds = PL::bytes(k);
  hipError_t e = lds_attr(leo16w_encode_kernel<NG, G, PK>, lds);
  if (e != hipSuccess) return e;
  const long blocks = a.nsq * a.nvec * (a.shard_bytes / 64) * (32 / PL::SYM);
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL((leo16w_encode_kernel<NG, G, PK>), dim3((unsigned)blocks), dim3(kWideThreads), lds, s, a, T, k);
  return hipGetLastError();
}

template <int NG, int G, int PK = 0, int TH = dec_threads<NG>()>
hipError_t launch_dec(const DecodeArgs& a, const WideTabs& T, hipStream_t s) {
  using PL = Planes<NG, PK>;
  const int n = 2 * a.k;
  const size_t lds = PL::bytes(n);
  hipError_t e = lds_attr(leo16w_decode_kernel<NG, G, PK, TH>, lds);
  if (e != hipSuccess) return e;
  const long blocks = a.nsq * a.nvec * (a.shard_bytes / 64) * (32 / PL::SYM);
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL((leo16w_decode_kernel<NG, G, PK, TH>), dim3((unsigned)blocks), dim3(TH), lds, s, a, T);
  return hipGetLastError();
}

// dword groups per radix-4 unit at 32-symbol slices: the decoder 8 (round 6:
// one unit per column of a slice, so a skew table serves 8 groups; k = 1024
// Repair 74.9 -> 81-82 squares/s), the encoder 4 (at 8 it held 136 VGPRs and
// the k = 1024 split square went 5.0 -> 7.2 ms; profiles/gf16_wide_ab_r06.log)
constexpr int WG8 = 8, WG8E = 4;

bool wide_k_ok(int k) { return k >= 256 && k <= kMaxCodecK && (k & (k - 1)) == 0; }

}  // namespace

hipError_t leo16w_prepare() {
  WideTabs T;
  hipError_t e = tables(T);
  // LDS attributes of every instantiation (hipFuncSetAttribute at launch time otherwise)
  const size_t big = 2 * 16384 * 4;  // <= the largest slice any width asks for
  if (e == hipSuccess) e = lds_attr(leo16w_encode_kernel<8, WG8E>, lds_bytes(2048, 8));
  if (e == hipSuccess) e = lds_attr(leo16w_encode_kernel<4, 4>, lds_bytes(4096, 4));
  if (e == hipSuccess) e = lds_attr(leo16w_encode_kernel<2, 2>, lds_bytes(8192, 2));
  if (e == hipSuccess) e = lds_attr(leo16w_encode_kernel<1, 1>, big);
  if (e == hipSuccess) e = lds_attr(leo16w_encode_kernel<1, 1, 2>, Planes<1, 2>::bytes(kMaxCodecK));
  if (e == hipSuccess) e = lds_attr(leo16w_decode_kernel<8, WG8>, lds_bytes(2048, 8));
  if (e == hipSuccess) e = lds_attr(leo16w_decode_kernel<4, 4>, lds_bytes(4096, 4));
  if (e == hipSuccess) e = lds_attr(leo16w_decode_kernel<2, 2>, lds_bytes(8192, 2));
  if (e == hipSuccess) e = lds_attr(leo16w_decode_kernel<1, 1>, big);
  if (e == hipSuccess) e = lds_attr(leo16w_decode_kernel<1, 1, 2>, Planes<1, 2>::bytes(2 * kMaxCodecK / 2));
  if (e == hipSuccess) e = lds_attr(leo16w_decode_kernel<1, 1, 1>, Planes<1, 1>::bytes(2 * kMaxCodecK));
  if (e == hipSuccess) e = lds_attr(leo16w_errlocs_kernel<uint32_t>, (size_t)4 * kMaxCodecK);
  if (e == hipSuccess) e = lds_attr(leo16w_errlocs_kernel<uint16_t>, (size_t)2 * 2 * kMaxCodecK);
  return e;
}

hipError_t launch_leo16w_encode(int k, const EncodeArgs& a, hipStream_t s) {
  if (!wide_k_ok(k) || a.shard_bytes % 64) return hipErrorInvalidValue;
  if (a.reverse && !a.out_present) return hipErrorInvalidValue;
  WideTabs T;
  hipError_t e = tables(T);
  if (e != hipSuccess) return e;
  switch (slice_sym(k)) {
    case 32: return launch_enc<8, WG8E>(a, T, k, s);
    case 16: return launch_enc<4, 4>(a, T, k, s);
    case 8: return launch_enc<2, 2>(a, T, k, s);
    case 4: return launch_enc<1, 1>(a, T, k, s);
    default: return launch_enc<1, 1, 2>(a, T, k, s);  // m = 32768 (k + k = 65536 shards)
  }
}

hipError_t launch_leo16w_errlocs(const DecodeArgs& a, hipStream_t s) {
  if (!wide_k_ok(a.k) || a.k < 1024) return hipErrorInvalidValue;
  WideTabs T;
  hipError_t e = tables(T);
  if (e != hipSuccess) return e;
  const long nv = a.nsq * a.nvec;
  if (nv <= 0) return hipSuccess;
  const int n = 2 * a.k;
  if (n > 32768) {  // n = 65536: 16-bit words (128 KiB)
    const size_t lds = (size_t)n * 2;
    if ((e = lds_attr(leo16w_errlocs_kernel<uint16_t>, lds)) != hipSuccess) return e;
    hipLaunchKernelGGL(leo16w_errlocs_kernel<uint16_t>, dim3((unsigned)nv), dim3(kFoldThreads), lds, s, a, T,
                       wfold_offset(n));
    return hipGetLastError();
  }
  const size_t lds = (size_t)n * 4;
  if ((e = lds_attr(leo16w_errlocs_kernel<uint32_t>, lds)) != hipSuccess) return e;
  hipLaunchKernelGGL(leo16w_errlocs_kernel<uint32_t>, dim3((unsigned)nv), dim3(kFoldThreads), lds, s, a, T,
                     wfold_offset(n));
  return hipGetLastError();
}

hipError_t launch_leo16w_decode_only(const DecodeArgs& a, hipStream_t s, bool mark_present) {
  if (!wide_k_ok(a.k) || a.shard_bytes % 64) return hipErrorInvalidValue;
  WideTabs T;
  hipError_t e = tables(T);
  if (e != hipSuccess) return e;
  const long nv = a.nsq * a.nvec;
  if (nv <= 0) return hipSuccess;
  switch (slice_sym(2 * a.k)) {
    case 32: e = launch_dec<8, WG8>(a, T, s); break;
    case 16: e = launch_dec<4, 4>(a, T, s); break;
    case 8: e = launch_dec<2, 2>(a, T, s); break;
    case 4: e = launch_dec<1, 1>(a, T, s); break;
    case 2: e = launch_dec<1, 1, 2>(a, T, s); break;  // codec k = 16384
    default: e = launch_dec<1, 1, 1>(a, T, s); break;  // codec k = 32768
  }
  if (e != hipSuccess) return e;
  if (mark_present) {
    hipLaunchKernelGGL(leo16w_mark_present_kernel, dim3((unsigned)nv), dim3(256), 0, s, a);
    e = hipGetLastError();
  }
  return e;
}

}  // namespace dagpu
