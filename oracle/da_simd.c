/*
 * da_simd.c -- multithreaded SIMD CPU restatement of the DA hot path: the CPU
 * baseline bench.py reports beside the GPU ("simd-port").
 * TEST/BENCH INFRASTRUCTURE ONLY (see da_oracle.h): only tests/ and bench.py's
 * cpu_baseline leg load it; the product path never links or calls it.
 *
 * Why it exists: the Go reference (da.ExtendShares + NewDataAvailabilityHeader,
 * pkg/da/data_availability_header.go:44-75) cannot be built here (no Go
 * toolchain, modules not vendored), and BASELINE.md's fallback
 * asks for a C restatement at the reference's own speed class:
 *   - GF(2^8) multiply-add as klauspost/reedsolomon v1.11.8 does it on amd64:
 *     GFNI affine (vgf2p8affineqb, one 8x8 bit matrix per log constant) with
 *     AVX-512, else AVX2 split-nibble PSHUFB tables; tables built ONCE per
 *     constant at init, not per call;
 *   - SHA-256 with the x86 SHA extensions, as Go's crypto/sha256 does on
 *     amd64 (OpenSSL's SHA256_* where the CPU lacks them);
 *   - the same work as the reference: rsmt2d v0.11.0 extends Q0 rows -> Q1,
 *     Q0 columns -> Q2, Q2 rows -> Q3 (3k Leopard encodes of k shards), then
 *     builds 4k wrapper NMTs, hashing every leaf in its row tree AND its column
 *     tree (1,573,374 compressions per k=128 square), then the RFC-6962 DAH;
 *   - rows/columns/trees spread over all given threads (rsmt2d's errgroup
 *     goroutines), OpenMP dynamic schedule.
 * Arithmetic (Leopard IFFT/FFT order, skews, NMT rules) follows da_oracle.c,
 * whose tables it reuses; tests/test_cpu_baseline.py checks it bit-exact
 * against the scalar oracle.  GF(2^8) only (k <= 128), the rsmt2d widths the
 * CPU baseline configs use (configs[0] k=64, configs[1] k=128).
 */
#include <immintrin.h>
#include <omp.h>
#include <openssl/sha.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "da_oracle.h"

#define SS ORC_SHARE_SIZE
#define NS ORC_NS_SIZE
#define NODE ORC_NODE_SIZE

/* per log constant: GFNI matrix, and AVX2 nibble tables (lo | hi) */
static uint64_t g_affine[256];
static uint8_t g_nib[256][32];
static int g_isa; /* 2 = AVX-512BW + GFNI, 1 = AVX2 */
static int g_inited;
static int g_shani; /* x86 SHA extensions present */

static void simd_init(void) {
  if (g_inited) return;
  orc_init();
  for (int c = 0; c < 256; c++) {
    /* y = x * exp(c) is GF(2)-linear in x: column j = (1 << j) * exp(c) */
    uint8_t col[8];
    for (int j = 0; j < 8; j++) col[j] = orc_gf8_mullog((uint8_t)(1 << j), (uint8_t)c);
    uint64_t A = 0;
    for (int i = 0; i < 8; i++) {
      uint8_t row = 0;
      for (int j = 0; j < 8; j++) row |= (uint8_t)(((col[j] >> i) & 1) << j);
      A |= (uint64_t)row << (8 * (7 - i)); /* vgf2p8affineqb: byte 7-i = row i */
    }
    g_affine[c] = A;
    for (int v = 0; v < 16; v++) {
      g_nib[c][v] = orc_gf8_mullog((uint8_t)v, (uint8_t)c);
      g_nib[c][16 + v] = orc_gf8_mullog((uint8_t)(v << 4), (uint8_t)c);
    }
  }
  __builtin_cpu_init();
  g_isa = (__builtin_cpu_supports("gfni") && __builtin_cpu_supports("avx512bw")) ? 2 : 1;
  g_shani = __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1");
  g_inited = 1;
}

/* ---- 512-B slice kernels ------------------------------------------------- */
__attribute__((target("avx512f,avx512bw,gfni"))) static void muladd_gfni(uint8_t* x, const uint8_t* y,
                                                                          unsigned lm) {
  const __m512i A = _mm512_set1_epi64((long long)g_affine[lm]);
  for (int i = 0; i < SS; i += 64) {
    __m512i p = _mm512_gf2p8affine_epi64_epi8(_mm512_loadu_si512(y + i), A, 0);
    _mm512_storeu_si512(x + i, _mm512_xor_si512(_mm512_loadu_si512(x + i), p));
  }
}
__attribute__((target("avx512f,avx512bw"))) static void xor_512(uint8_t* d, const uint8_t* s) {
  for (int i = 0; i < SS; i += 64)
    _mm512_storeu_si512(d + i, _mm512_xor_si512(_mm512_loadu_si512(d + i), _mm512_loadu_si512(s + i)));
}
__attribute__((target("avx2"))) static void muladd_avx2(uint8_t* x, const uint8_t* y, unsigned lm) {
  const __m256i lo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)g_nib[lm]));
  const __m256i hi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)(g_nib[lm] + 16)));
  const __m256i m = _mm256_set1_epi8(0x0F);
  for (int i = 0; i < SS; i += 32) {
    __m256i v = _mm256_loadu_si256((const __m256i*)(y + i));
    __m256i p = _mm256_xor_si256(_mm256_shuffle_epi8(lo, _mm256_and_si256(v, m)),
                                 _mm256_shuffle_epi8(hi, _mm256_and_si256(_mm256_srli_epi16(v, 4), m)));
    _mm256_storeu_si256((__m256i*)(x + i), _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)(x + i)), p));
  }
}
__attribute__((target("avx2"))) static void xor_256(uint8_t* d, const uint8_t* s) {
  for (int i = 0; i < SS; i += 32)
    _mm256_storeu_si256((__m256i*)(d + i), _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)(d + i)),
                                                            _mm256_loadu_si256((const __m256i*)(s + i))));
}

static inline void muladd(uint8_t* x, const uint8_t* y, unsigned lm) {
  if (g_isa == 2) muladd_gfni(x, y, lm);
  else muladd_avx2(x, y, lm);
}
static inline void xorv(uint8_t* d, const uint8_t* s) {
  if (g_isa == 2) xor_512(d, s);
  else xor_256(d, s);
}

/* ifftDIT2 / fftDIT2 (leopard8.go), log_m == 255 means xor only */
static inline void ifft2(uint8_t* x, uint8_t* y, unsigned lm) {
  xorv(y, x);
  if (lm != 255) muladd(x, y, lm);
}
static inline void fft2(uint8_t* x, uint8_t* y, unsigned lm) {
  if (lm != 255) muladd(x, y, lm);
  xorv(y, x);
}

/* One Leopard GF(2^8) encode (m = k, data -> parity), da_oracle.c orc_encode.
 * work: k pointers to 512-B slices holding the data, overwritten by parity. */
static void encode_vec(int k, uint8_t** work) {
  const uint8_t* skew = orc_gf8_skew();
  const int m = k, base = m - 1;
  int dist = 1, dist4 = 4;
  while (dist4 <= m) { /* ifftDITEncoder, skewLUT = fftSkew[m-1:] */
    for (int r = 0; r < m; r += dist4) {
      const int iend = r + dist;
      const unsigned l01 = skew[base + iend], l02 = skew[base + iend + dist],
                     l23 = skew[base + iend + 2 * dist];
      for (int i = r; i < iend; i++) {
        ifft2(work[i], work[i + dist], l01);
        ifft2(work[i + 2 * dist], work[i + 3 * dist], l23);
        ifft2(work[i], work[i + 2 * dist], l02);
        ifft2(work[i + dist], work[i + 3 * dist], l02);
      }
    }
    dist = dist4;
    dist4 <<= 2;
  }
  if (dist < m) {
    const unsigned lm = skew[base + dist];
    for (int i = 0; i < dist; i++) ifft2(work[i], work[i + dist], lm);
  }
  dist4 = m; /* fftDIT */
  dist = m >> 2;
  while (dist != 0) {
    for (int r = 0; r < k; r += dist4) {
      const int iend = r + dist;
      const unsigned l01 = skew[iend - 1], l02 = skew[iend + dist - 1], l23 = skew[iend + 2 * dist - 1];
      for (int i = r; i < iend; i++) {
        fft2(work[i], work[i + 2 * dist], l02);
        fft2(work[i + dist], work[i + 3 * dist], l02);
        fft2(work[i], work[i + dist], l01);
        fft2(work[i + 2 * dist], work[i + 3 * dist], l23);
      }
    }
    dist4 = dist;
    dist >>= 2;
  }
  if (dist4 == 2)
    for (int r = 0; r < k; r += 2) fft2(work[r], work[r + 1], skew[r]);
}

/* ---- SHA-256 -------------------------------------------------------------
 * Go's crypto/sha256 runs the x86 SHA extensions directly (sha256block_amd64);
 * so does this (sha256rnds2 / sha256msg1 / sha256msg2), with OpenSSL's
 * low-level SHA256_* as the fallback on CPUs without them.  (OpenSSL 3's
 * one-shot SHA256() fetches the algorithm per call under a lock and does not
 * scale across threads.) */
__attribute__((target("sha,sse4.1,ssse3"))) static void sha256_ni(uint32_t st[8], const uint8_t* p, size_t nb) {
  static const uint32_t K[64] = {
      0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
      0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
      0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
      0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
      0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
      0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
      0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
      0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
  const __m128i BSWAP = _mm_set_epi64x(0x0c0d0e0f08090a0bLL, 0x0405060700010203LL);
  __m128i t = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)st), 0xB1);  /* CDAB */
  __m128i s1 = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)(st + 4)), 0x1B); /* EFGH */
  __m128i s0 = _mm_alignr_epi8(t, s1, 8);                                      /* ABEF */
  s1 = _mm_blend_epi16(s1, t, 0xF0);                                           /* CDGH */
  for (; nb; nb--, p += 64) {
    const __m128i a0 = s0, c0 = s1;
    __m128i x[16];
#pragma GCC unroll 16
    for (int g = 0; g < 16; g++) {
      if (g < 4) {
        x[g] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 16 * g)), BSWAP);
      } else {
        __m128i u = _mm_add_epi32(_mm_sha256msg1_epu32(x[g - 4], x[g - 3]), _mm_alignr_epi8(x[g - 1], x[g - 2], 4));
        x[g] = _mm_sha256msg2_epu32(u, x[g - 1]);
      }
      __m128i m = _mm_add_epi32(x[g], _mm_loadu_si128((const __m128i*)(K + 4 * g)));
      s1 = _mm_sha256rnds2_epu32(s1, s0, m);
      s0 = _mm_sha256rnds2_epu32(s0, s1, _mm_shuffle_epi32(m, 0x0E));
    }
    s0 = _mm_add_epi32(s0, a0);
    s1 = _mm_add_epi32(s1, c0);
  }
  t = _mm_shuffle_epi32(s0, 0x1B);    /* FEBA */
  s1 = _mm_shuffle_epi32(s1, 0xB1);   /* DCHG */
  s0 = _mm_blend_epi16(t, s1, 0xF0);  /* DCBA */
  s1 = _mm_alignr_epi8(s1, t, 8);     /* HGFE */
  _mm_storeu_si128((__m128i*)st, s0);
  _mm_storeu_si128((__m128i*)(st + 4), s1);
}

/* SHA-256 of a message already placed in buf (capacity >= len + 72, padding
 * is written in place). */
static void sha256_buf(uint8_t* buf, size_t len, uint8_t out[32]) {
  if (!g_shani) {
    SHA256_CTX c;
    SHA256_Init(&c);
    SHA256_Update(&c, buf, len);
    SHA256_Final(out, &c);
    return;
  }
  size_t padded = (len + 9 + 63) & ~(size_t)63;
  buf[len] = 0x80;
  memset(buf + len + 1, 0, padded - len - 9);
  const uint64_t bits = (uint64_t)len * 8;
  for (int b = 0; b < 8; b++) buf[padded - 1 - b] = (uint8_t)(bits >> (8 * b));
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                    0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  sha256_ni(st, buf, padded / 64);
  for (int j = 0; j < 8; j++) {
    out[4 * j] = (uint8_t)(st[j] >> 24); out[4 * j + 1] = (uint8_t)(st[j] >> 16);
    out[4 * j + 2] = (uint8_t)(st[j] >> 8); out[4 * j + 3] = (uint8_t)st[j];
  }
}

/* ---- NMT (nmt v0.20.0 via pkg/wrapper, as in da_oracle.c) ---------------- */
static const uint8_t PARITY_NS[NS] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                      0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                      0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF};

static void leaf_hash(const uint8_t* ns, const uint8_t* share, uint8_t out[NODE]) {
  uint8_t buf[1 + NS + SS + 72];
  buf[0] = 0x00;
  memcpy(buf + 1, ns, NS);
  memcpy(buf + 1 + NS, share, SS);
  memcpy(out, ns, NS);
  memcpy(out + NS, ns, NS);
  sha256_buf(buf, 1 + NS + SS, out + 2 * NS);
}

static void node_hash(const uint8_t* l, const uint8_t* r, uint8_t out[NODE]) {
  uint8_t buf[1 + 2 * NODE + 72];
  buf[0] = 0x01;
  memcpy(buf + 1, l, NODE);
  memcpy(buf + 1 + NODE, r, NODE);
  memcpy(out, l, NS);
  memcpy(out + NS, memcmp(r, PARITY_NS, NS) == 0 ? l + NS : r + NS, NS); /* ignoreMaxNamespace */
  sha256_buf(buf, 1 + 2 * NODE, out + 2 * NS);
}

/* wrapper tree over one EDS axis: Push every cell (leaf hashed here, as nmt
 * Push does), then Root (w a power of two: a balanced RFC-6962 tree). */
static int axis_root(int k, const uint8_t* eds, int axis, int index, uint8_t* nodes, uint8_t out[NODE]) {
  const int w = 2 * k;
  const uint8_t* prev = NULL;
  int rc = ORC_OK;
  for (int j = 0; j < w; j++) {
    const int r = axis == 0 ? index : j, c = axis == 0 ? j : index;
    const uint8_t* share = eds + ((size_t)r * w + c) * SS;
    const uint8_t* ns = (j < k && index < k) ? share : PARITY_NS;
    if (prev && memcmp(ns, prev, NS) < 0) rc = ORC_ERR_PUSH_ORDER;
    prev = ns;
    leaf_hash(ns, share, nodes + (size_t)j * NODE);
  }
  if (rc) return rc;
  for (int n = w; n > 1; n >>= 1)
    for (int i = 0; i < n / 2; i++)
      node_hash(nodes + (size_t)(2 * i) * NODE, nodes + (size_t)(2 * i + 1) * NODE, nodes + (size_t)i * NODE);
  memcpy(out, nodes, NODE);
  return ORC_OK;
}

const char* simd_isa(void) {
  simd_init();
  static char buf[160];
  snprintf(buf, sizeof buf, "GF(2^8): %s; SHA-256: %s",
           g_isa == 2 ? "avx512bw+gfni (vgf2p8affineqb)" : "avx2 (pshufb split nibble)",
           g_shani ? "x86 SHA extensions (sha256rnds2)" : "OpenSSL SHA256_*");
  return buf;
}

/* da.ExtendShares + NewDataAvailabilityHeader for one k x k square (k a power
 * of two <= 128).  eds: (2k)^2*512 bytes of caller memory (the EDS the Go path
 * allocates and returns).  Returns ORC_OK / ORC_ERR_*. */
int simd_extend_and_dah(int k, const uint8_t* ods, uint8_t* eds, uint8_t* row_roots, uint8_t* col_roots,
                        uint8_t dah[32], int nthreads) {
  simd_init();
  if (k < 1 || k > 128 || (k & (k - 1))) return ORC_ERR_ARG;
  const int w = 2 * k;
  if (nthreads < 1) nthreads = 1;
  int rc = ORC_OK;
#pragma omp parallel num_threads(nthreads)
  {
    uint8_t** work = (uint8_t**)malloc(sizeof(uint8_t*) * k);
    uint8_t* colbuf = (uint8_t*)aligned_alloc(64, (size_t)k * SS);
    uint8_t* nodes = (uint8_t*)malloc((size_t)w * NODE);
    /* Q0 rows -> Q1 (rsmt2d erasureExtendRow: parity written next to the data) */
#pragma omp for schedule(dynamic, 1)
    for (int r = 0; r < k; r++) {
      uint8_t* row = eds + (size_t)r * w * SS;
      memcpy(row, ods + (size_t)r * k * SS, (size_t)k * SS);
      memcpy(row + (size_t)k * SS, row, (size_t)k * SS);
      for (int i = 0; i < k; i++) work[i] = row + (size_t)(k + i) * SS;
      encode_vec(k, work);
    }
    /* Q0 columns -> Q2 (a column's shards are strided: gathered, encoded, scattered) */
#pragma omp for schedule(dynamic, 1)
    for (int c = 0; c < k; c++) {
      for (int r = 0; r < k; r++) {
        memcpy(colbuf + (size_t)r * SS, eds + ((size_t)r * w + c) * SS, SS);
        work[r] = colbuf + (size_t)r * SS;
      }
      encode_vec(k, work);
      for (int r = 0; r < k; r++) memcpy(eds + ((size_t)(k + r) * w + c) * SS, colbuf + (size_t)r * SS, SS);
    }
    /* Q2 rows -> Q3 */
#pragma omp for schedule(dynamic, 1)
    for (int r = k; r < w; r++) {
      uint8_t* row = eds + (size_t)r * w * SS;
      memcpy(row + (size_t)k * SS, row, (size_t)k * SS);
      for (int i = 0; i < k; i++) work[i] = row + (size_t)(k + i) * SS;
      encode_vec(k, work);
    }
    /* RowRoots + ColRoots: 4k wrapper trees */
#pragma omp for schedule(dynamic, 1)
    for (int t = 0; t < 2 * w; t++) {
      const int axis = t & 1, idx = t >> 1;
      int e = axis_root(k, eds, axis, idx, nodes, (axis == 0 ? row_roots : col_roots) + (size_t)idx * NODE);
      if (e) {
#pragma omp critical
        rc = e;
      }
    }
    free(nodes);
    free(colbuf);
    free(work);
  }
  if (rc == ORC_OK) orc_dah_hash(row_roots, col_roots, (size_t)w, dah);
  return rc;
}
