/*
 * da_oracle.c -- CPU restatement of the celestia-app DA hot path.
 * TEST INFRASTRUCTURE ONLY (see da_oracle.h).  Never linked by the product.
 *
 * Leopard RS follows klauspost/reedsolomon v1.11.8 (leopard8.go / leopard.go),
 * the codec rsmt2d v0.11.0 LeoRSCodec builds via reedsolomon.New(k, k,
 * WithLeopardGF(true)) -- pkg/appconsts/global_consts.go:92.  The module is not
 * vendored in /root/reference; the algorithm is restated from its published
 * source and pinned by the reference's golden DAH hashes
 * (pkg/da/data_availability_header_test.go:27-54).
 */
#include "da_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#ifdef ORC_USE_OPENSSL
#include <openssl/sha.h>
#endif

/* ------------------------------------------------------------------------- */
/* SHA-256 (FIPS 180-4).  Go crypto/sha256 is what nmt/merkle use.            */
/* ------------------------------------------------------------------------- */
#ifndef ORC_USE_OPENSSL
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
    0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
    0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
    0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
    0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
    0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
    0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
    0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_block(uint32_t st[8], const uint8_t* p) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) |
           ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
           h = st[7];
  for (int i = 0; i < 64; i++) {
    uint32_t S1 = ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + K256[i] + w[i];
    uint32_t S0 = ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
#endif

void orc_sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
#ifdef ORC_USE_OPENSSL
  SHA256(msg, len, out);
#else
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                    0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t i = 0;
  for (; i + 64 <= len; i += 64) sha256_block(st, msg + i);
  uint8_t tail[128];
  size_t rem = len - i;
  memset(tail, 0, sizeof tail);
  if (rem) memcpy(tail, msg + i, rem);  /* msg may be NULL when len == 0 */
  tail[rem] = 0x80;
  size_t tl = (rem + 9 <= 64) ? 64 : 128;
  uint64_t bits = (uint64_t)len * 8;
  for (int b = 0; b < 8; b++) tail[tl - 1 - b] = (uint8_t)(bits >> (8 * b));
  sha256_block(st, tail);
  if (tl == 128) sha256_block(st, tail + 64);
  for (int j = 0; j < 8; j++) {
    out[4 * j] = st[j] >> 24; out[4 * j + 1] = st[j] >> 16;
    out[4 * j + 2] = st[j] >> 8; out[4 * j + 3] = st[j];
  }
#endif
}

/* ------------------------------------------------------------------------- */
/* GF(2^8) Leopard tables -- klauspost leopard8.go initLUTs8/initFFTSkew8.     */
/* ------------------------------------------------------------------------- */
#define GF8_BITS 8
#define GF8_ORDER 256
#define GF8_MOD 255
static uint8_t LOG8[256], EXP8[256], SKEW8[255], WALSH8[256];

static inline uint8_t add_mod8(unsigned a, unsigned b) {
  unsigned s = a + b;
  return (uint8_t)(s + (s >> GF8_BITS));
}
static inline uint8_t sub_mod8(unsigned a, unsigned b) {
  uint64_t d = (uint64_t)a - (uint64_t)b;
  return (uint8_t)(d + (d >> GF8_BITS));
}
uint8_t orc_gf8_mullog(uint8_t a, uint8_t log_b) {
  if (a == 0) return 0;
  return EXP8[add_mod8(LOG8[a], log_b)];
}

static void fwht8(uint8_t* data, int m, int mtrunc) {
  int dist = 1, dist4 = 4;
  while (dist4 <= m) {
    for (int r = 0; r < mtrunc; r += dist4) {
      for (int i = r; i < r + dist; i++) {
        uint8_t t0 = data[i], t1 = data[i + dist], t2 = data[i + 2 * dist],
                t3 = data[i + 3 * dist];
        uint8_t a0 = add_mod8(t0, t1), a1 = sub_mod8(t0, t1);
        uint8_t a2 = add_mod8(t2, t3), a3 = sub_mod8(t2, t3);
        t0 = add_mod8(a0, a2); t2 = sub_mod8(a0, a2);
        t1 = add_mod8(a1, a3); t3 = sub_mod8(a1, a3);
        data[i] = t0; data[i + dist] = t1; data[i + 2 * dist] = t2; data[i + 3 * dist] = t3;
      }
    }
    dist = dist4;
    dist4 <<= 2;
  }
  if (dist < m) {
    for (int i = 0; i < dist; i++) {
      uint8_t a = data[i], b = data[i + dist];
      data[i] = add_mod8(a, b);
      data[i + dist] = sub_mod8(a, b);
    }
  }
}

static void init_gf8(void) {
  static const uint8_t cantor[8] = {1, 214, 152, 146, 86, 200, 88, 230};
  unsigned state = 1;
  for (unsigned i = 0; i < GF8_MOD; i++) {
    EXP8[state] = (uint8_t)i;
    state <<= 1;
    if (state >= GF8_ORDER) state ^= 0x11D;
  }
  EXP8[0] = GF8_MOD;
  LOG8[0] = 0;
  for (int i = 0; i < 8; i++) {
    int width = 1 << i;
    for (int j = 0; j < width; j++) LOG8[j + width] = LOG8[j] ^ cantor[i];
  }
  for (int i = 0; i < 256; i++) LOG8[i] = EXP8[LOG8[i]];
  for (int i = 0; i < 256; i++) EXP8[LOG8[i]] = (uint8_t)i;
  EXP8[GF8_MOD] = EXP8[0];

  uint8_t temp[7];
  for (int i = 1; i < 8; i++) temp[i - 1] = (uint8_t)(1 << i);
  memset(SKEW8, 0, sizeof SKEW8);
  for (int m = 0; m < 7; m++) {
    int step = 1 << (m + 1);
    SKEW8[(1 << m) - 1] = 0;
    for (int i = m; i < 7; i++) {
      int s = 1 << (i + 1);
      for (int j = (1 << m) - 1; j < s; j += step) SKEW8[j + s] = SKEW8[j] ^ temp[i];
    }
    temp[m] = (uint8_t)(GF8_MOD - LOG8[orc_gf8_mullog(temp[m], LOG8[temp[m] ^ 1])]);
    for (int i = m + 1; i < 7; i++) {
      uint8_t sum = add_mod8(LOG8[temp[i] ^ 1], temp[m]);
      temp[i] = orc_gf8_mullog(temp[i], sum);
    }
  }
  for (int i = 0; i < GF8_MOD; i++) SKEW8[i] = LOG8[SKEW8[i]];
  for (int i = 0; i < 256; i++) WALSH8[i] = LOG8[i];
  WALSH8[0] = 0;
  fwht8(WALSH8, GF8_ORDER, GF8_ORDER);
}

const uint8_t* orc_gf8_log(void) { return LOG8; }
const uint8_t* orc_gf8_exp(void) { return EXP8; }
const uint8_t* orc_gf8_skew(void) { return SKEW8; }
const uint8_t* orc_gf8_logwalsh(void) { return WALSH8; }

/* ------------------------------------------------------------------------- */
/* GF(2^16) Leopard tables -- klauspost leopard.go initLUTs/initFFTSkew.       */
/* ------------------------------------------------------------------------- */
#define GF16_BITS 16
#define GF16_ORDER 65536
#define GF16_MOD 65535
static uint16_t* LOG16;
static uint16_t* EXP16;
static uint16_t* SKEW16;
static uint16_t* WALSH16;

static inline uint16_t add_mod16(unsigned a, unsigned b) {
  unsigned s = a + b;
  return (uint16_t)(s + (s >> GF16_BITS));
}
static inline uint16_t sub_mod16(unsigned a, unsigned b) {
  uint64_t d = (uint64_t)a - (uint64_t)b;
  return (uint16_t)(d + (d >> GF16_BITS));
}
static inline uint16_t mullog16(uint16_t a, uint16_t log_b) {
  if (a == 0) return 0;
  return EXP16[add_mod16(LOG16[a], log_b)];
}

static void fwht16(uint16_t* data, int m, int mtrunc) {
  int dist = 1, dist4 = 4;
  while (dist4 <= m) {
    for (int r = 0; r < mtrunc; r += dist4) {
      for (int i = r; i < r + dist; i++) {
        uint16_t t0 = data[i], t1 = data[i + dist], t2 = data[i + 2 * dist],
                 t3 = data[i + 3 * dist];
        uint16_t a0 = add_mod16(t0, t1), a1 = sub_mod16(t0, t1);
        uint16_t a2 = add_mod16(t2, t3), a3 = sub_mod16(t2, t3);
        t0 = add_mod16(a0, a2); t2 = sub_mod16(a0, a2);
        t1 = add_mod16(a1, a3); t3 = sub_mod16(a1, a3);
        data[i] = t0; data[i + dist] = t1; data[i + 2 * dist] = t2; data[i + 3 * dist] = t3;
      }
    }
    dist = dist4;
    dist4 <<= 2;
  }
  if (dist < m) {
    for (int i = 0; i < dist; i++) {
      uint16_t a = data[i], b = data[i + dist];
      data[i] = add_mod16(a, b);
      data[i + dist] = sub_mod16(a, b);
    }
  }
}

static void init_gf16(void) {
  static const uint16_t cantor[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E,
                                      0x914C, 0x4012, 0x6C98, 0x10D8, 0x6A72, 0xB900,
                                      0xFDB8, 0xFB34, 0xFF38, 0x991E};
  LOG16 = (uint16_t*)calloc(GF16_ORDER, 2);
  EXP16 = (uint16_t*)calloc(GF16_ORDER, 2);
  SKEW16 = (uint16_t*)calloc(GF16_MOD, 2);
  WALSH16 = (uint16_t*)calloc(GF16_ORDER, 2);
  unsigned state = 1;
  for (unsigned i = 0; i < GF16_MOD; i++) {
    EXP16[state] = (uint16_t)i;
    state <<= 1;
    if (state >= GF16_ORDER) state ^= 0x1002D;
  }
  EXP16[0] = GF16_MOD;
  LOG16[0] = 0;
  for (int i = 0; i < 16; i++) {
    int width = 1 << i;
    for (int j = 0; j < width; j++) LOG16[j + width] = LOG16[j] ^ cantor[i];
  }
  for (int i = 0; i < GF16_ORDER; i++) LOG16[i] = EXP16[LOG16[i]];
  for (int i = 0; i < GF16_ORDER; i++) EXP16[LOG16[i]] = (uint16_t)i;
  EXP16[GF16_MOD] = EXP16[0];

  uint16_t temp[15];
  for (int i = 1; i < 16; i++) temp[i - 1] = (uint16_t)(1 << i);
  for (int m = 0; m < 15; m++) {
    int step = 1 << (m + 1);
    SKEW16[(1 << m) - 1] = 0;
    for (int i = m; i < 15; i++) {
      int s = 1 << (i + 1);
      for (int j = (1 << m) - 1; j < s; j += step) SKEW16[j + s] = SKEW16[j] ^ temp[i];
    }
    temp[m] = (uint16_t)(GF16_MOD - LOG16[mullog16(temp[m], LOG16[temp[m] ^ 1])]);
    for (int i = m + 1; i < 15; i++) {
      uint16_t sum = add_mod16(LOG16[temp[i] ^ 1], temp[m]);
      temp[i] = mullog16(temp[i], sum);
    }
  }
  for (int i = 0; i < GF16_MOD; i++) SKEW16[i] = LOG16[SKEW16[i]];
  for (int i = 0; i < GF16_ORDER; i++) WALSH16[i] = LOG16[i];
  WALSH16[0] = 0;
  fwht16(WALSH16, GF16_ORDER, GF16_ORDER);
}

const uint16_t* orc_gf16_log(void) { return LOG16; }
const uint16_t* orc_gf16_exp(void) { return EXP16; }
const uint16_t* orc_gf16_skew(void) { return SKEW16; }

static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void init_all(void) {
  init_gf8();
  init_gf16();
}
void orc_init(void) { pthread_once(&g_once, init_all); }

/* ------------------------------------------------------------------------- */
/* Slice ops.  A "slice" is one shard; GF8 symbols are bytes, GF16 symbols are */
/* (lo = b[i], hi = b[i+32]) pairs inside each 64-byte block (leopard.go       */
/* refMulAdd).                                                                */
/* ------------------------------------------------------------------------- */
static void xor_slice(uint8_t* dst, const uint8_t* src, size_t n) {
  for (size_t i = 0; i < n; i++) dst[i] ^= src[i];
}

/* x ^= y * exp(log_m) */
static void muladd8(uint8_t* x, const uint8_t* y, uint8_t log_m, size_t n) {
  uint8_t lut[256];
  for (int v = 0; v < 256; v++) lut[v] = orc_gf8_mullog((uint8_t)v, log_m);
  for (size_t i = 0; i < n; i++) x[i] ^= lut[y[i]];
}
/* x = y * exp(log_m) */
static void mul8(uint8_t* x, const uint8_t* y, uint8_t log_m, size_t n) {
  uint8_t lut[256];
  for (int v = 0; v < 256; v++) lut[v] = orc_gf8_mullog((uint8_t)v, log_m);
  for (size_t i = 0; i < n; i++) x[i] = lut[y[i]];
}
static void muladd16(uint8_t* x, const uint8_t* y, uint16_t log_m, size_t n) {
  for (size_t b = 0; b < n; b += 64) {
    for (int i = 0; i < 32; i++) {
      uint16_t v = (uint16_t)(y[b + i] | (y[b + i + 32] << 8));
      uint16_t p = mullog16(v, log_m);
      x[b + i] ^= (uint8_t)p;
      x[b + i + 32] ^= (uint8_t)(p >> 8);
    }
  }
}
static void mul16(uint8_t* x, const uint8_t* y, uint16_t log_m, size_t n) {
  for (size_t b = 0; b < n; b += 64) {
    for (int i = 0; i < 32; i++) {
      uint16_t v = (uint16_t)(y[b + i] | (y[b + i + 32] << 8));
      uint16_t p = mullog16(v, log_m);
      x[b + i] = (uint8_t)p;
      x[b + i + 32] = (uint8_t)(p >> 8);
    }
  }
}

typedef struct {
  int gf16;
  size_t n;        /* shard bytes */
  unsigned modulus;
} field_t;

static void f_muladd(const field_t* F, uint8_t* x, const uint8_t* y, unsigned log_m) {
  if (F->gf16) muladd16(x, y, (uint16_t)log_m, F->n);
  else muladd8(x, y, (uint8_t)log_m, F->n);
}
static void f_mul(const field_t* F, uint8_t* x, const uint8_t* y, unsigned log_m) {
  if (F->gf16) mul16(x, y, (uint16_t)log_m, F->n);
  else mul8(x, y, (uint8_t)log_m, F->n);
}
static unsigned f_skew(const field_t* F, int i) {
  return F->gf16 ? SKEW16[i] : SKEW8[i];
}

/* ifftDIT2: y ^= x; x ^= y*log_m   (leopard8.go ifftDIT28) */
static void ifft2(const field_t* F, uint8_t* x, uint8_t* y, unsigned log_m) {
  xor_slice(y, x, F->n);
  if (log_m != F->modulus) f_muladd(F, x, y, log_m);
}
/* fftDIT2: x ^= y*log_m; y ^= x    (leopard8.go fftDIT28) */
static void fft2(const field_t* F, uint8_t* x, uint8_t* y, unsigned log_m) {
  if (log_m != F->modulus) f_muladd(F, x, y, log_m);
  xor_slice(y, x, F->n);
}

#define W(i) (work + (size_t)(i) * F->n)

/* ifftDITEncoder / ifftDITDecoder body.  skew(i) = skewLUT[i + off]. */
static void ifft_dit(const field_t* F, uint8_t* work, int mtrunc, int m, int skew_base) {
  int dist = 1, dist4 = 4;
  while (dist4 <= m) {
    for (int r = 0; r < mtrunc; r += dist4) {
      int iend = r + dist;
      unsigned l01 = f_skew(F, skew_base + iend);
      unsigned l02 = f_skew(F, skew_base + iend + dist);
      unsigned l23 = f_skew(F, skew_base + iend + 2 * dist);
      for (int i = r; i < iend; i++) {
        ifft2(F, W(i), W(i + dist), l01);
        ifft2(F, W(i + 2 * dist), W(i + 3 * dist), l23);
        ifft2(F, W(i), W(i + 2 * dist), l02);
        ifft2(F, W(i + dist), W(i + 3 * dist), l02);
      }
    }
    dist = dist4;
    dist4 <<= 2;
  }
  if (dist < m) {
    unsigned lm = f_skew(F, skew_base + dist);
    for (int i = 0; i < dist; i++) ifft2(F, W(i), W(i + dist), lm);
  }
}

/* fftDIT: skewLUT = fftSkew[:], index iend-1 */
static void fft_dit(const field_t* F, uint8_t* work, int mtrunc, int m) {
  int dist4 = m, dist = m >> 2;
  while (dist != 0) {
    for (int r = 0; r < mtrunc; r += dist4) {
      int iend = r + dist;
      unsigned l01 = f_skew(F, iend - 1);
      unsigned l02 = f_skew(F, iend + dist - 1);
      unsigned l23 = f_skew(F, iend + 2 * dist - 1);
      for (int i = r; i < iend; i++) {
        fft2(F, W(i), W(i + 2 * dist), l02);
        fft2(F, W(i + dist), W(i + 3 * dist), l02);
        fft2(F, W(i), W(i + dist), l01);
        fft2(F, W(i + 2 * dist), W(i + 3 * dist), l23);
      }
    }
    dist4 = dist;
    dist >>= 2;
  }
  if (dist4 == 2) {
    for (int r = 0; r < mtrunc; r += 2) fft2(F, W(r), W(r + 1), f_skew(F, r));
  }
}

static int is_pow2(long v) { return v > 0 && (v & (v - 1)) == 0; }

int orc_encode(int k, size_t shard, const uint8_t* data, uint8_t* parity) {
  orc_init();
  if (!is_pow2(k) || shard == 0 || shard % 64) return ORC_ERR_ARG;
  field_t Fs = {2 * k > 256, shard, 2 * k > 256 ? GF16_MOD : GF8_MOD};
  const field_t* F = &Fs;
  int m = k;
  /* work == parity buffer: parity = FFT(IFFT(data)) truncated to k. */
  uint8_t* work = parity;
  memcpy(work, data, (size_t)k * shard);
  /* ifftDITEncoder with skewLUT = fftSkew[m-1:] */
  ifft_dit(F, work, m, m, m - 1);
  fft_dit(F, work, k, m);
  return ORC_OK;
}

int orc_decode(int k, size_t shard, uint8_t* shards, const uint8_t* present) {
  orc_init();
  if (!is_pow2(k) || shard == 0 || shard % 64) return ORC_ERR_ARG;
  int total = 2 * k, npresent = 0;
  for (int i = 0; i < total; i++) npresent += present[i] != 0;
  if (npresent == total) return ORC_OK;
  if (npresent < k) return ORC_ERR_TOO_FEW;
  int gf16 = total > 256;
  field_t Fs = {gf16, shard, gf16 ? GF16_MOD : GF8_MOD};
  const field_t* F = &Fs;
  int order = gf16 ? GF16_ORDER : GF8_ORDER;
  int m = k, n = 2 * k; /* ceilPow2(parity), ceilPow2(m + data) */
  int dataShards = k;
  uint16_t* err = (uint16_t*)calloc(order, sizeof(uint16_t));
  /* error locations: [parity (m)] [data (k)] */
  for (int i = 0; i < k; i++)
    if (!present[dataShards + i]) err[i] = 1;
  for (int i = 0; i < k; i++)
    if (!present[i]) err[i + m] = 1;
  if (gf16) {
    fwht16(err, order, m + dataShards);
    for (int i = 0; i < order; i++) err[i] = (uint16_t)(((unsigned)err[i] * WALSH16[i]) % GF16_MOD);
    fwht16(err, order, order);
  } else {
    uint8_t e8[256];
    for (int i = 0; i < 256; i++) e8[i] = (uint8_t)err[i];
    fwht8(e8, order, m + dataShards);
    for (int i = 0; i < 256; i++) e8[i] = (uint8_t)(((unsigned)e8[i] * WALSH8[i]) % GF8_MOD);
    fwht8(e8, order, order);
    for (int i = 0; i < 256; i++) err[i] = e8[i];
  }
  uint8_t* work = (uint8_t*)calloc((size_t)n, shard);
  for (int i = 0; i < k; i++) {
    if (present[dataShards + i]) f_mul(F, W(i), shards + (size_t)(dataShards + i) * shard, err[i]);
  }
  for (int i = 0; i < k; i++) {
    if (present[i]) f_mul(F, W(m + i), shards + (size_t)i * shard, err[m + i]);
  }
  /* IFFT(work, n) with decoder skew: skewLUT[iend-1] == fftSkew[iend-1] */
  ifft_dit(F, work, m + dataShards, n, -1);
  /* formal derivative */
  for (int i = 1; i < n; i++) {
    int width = ((i ^ (i - 1)) + 1) >> 1;
    for (int j = 0; j < width; j++) xor_slice(W(i - width + j), W(i + j), shard);
  }
  fft_dit(F, work, m + dataShards, n);
  for (int i = 0; i < total; i++) {
    if (present[i]) continue;
    uint8_t* out = shards + (size_t)i * shard;
    if (i >= dataShards) {
      f_mul(F, out, W(i - dataShards), F->modulus - err[i - dataShards]);
    } else {
      f_mul(F, out, W(i + m), F->modulus - err[i + m]);
    }
  }
  free(work);
  free(err);
  return ORC_OK;
}
#undef W

/* ------------------------------------------------------------------------- */
/* rsmt2d ComputeExtendedDataSquare (erasureExtendSquare): Q0 rows -> Q1,      */
/* Q0 cols -> Q2, Q2 rows -> Q3 (specs data_structures.md:305-313).            */
/* ------------------------------------------------------------------------- */
#define SS ORC_SHARE_SIZE
int orc_extend_square(int k, const uint8_t* ods, uint8_t* eds) {
  orc_init();
  if (!is_pow2(k)) return ORC_ERR_ARG;
  size_t w = 2 * (size_t)k;
  uint8_t* in = (uint8_t*)malloc((size_t)k * SS);
  uint8_t* out = (uint8_t*)malloc((size_t)k * SS);
  for (int r = 0; r < k; r++)
    memcpy(eds + (r * w) * SS, ods + ((size_t)r * k) * SS, (size_t)k * SS);
  /* Q0 rows -> Q1 */
  for (int r = 0; r < k; r++) {
    orc_encode(k, SS, eds + (r * w) * SS, eds + (r * w + k) * SS);
  }
  /* Q0 cols -> Q2 */
  for (int c = 0; c < k; c++) {
    for (int r = 0; r < k; r++) memcpy(in + (size_t)r * SS, eds + (r * w + c) * SS, SS);
    orc_encode(k, SS, in, out);
    for (int r = 0; r < k; r++) memcpy(eds + ((k + r) * w + c) * SS, out + (size_t)r * SS, SS);
  }
  /* Q2 rows -> Q3 */
  for (int r = k; r < 2 * k; r++) {
    orc_encode(k, SS, eds + (r * w) * SS, eds + (r * w + k) * SS);
  }
  free(in);
  free(out);
  return ORC_OK;
}

/* ------------------------------------------------------------------------- */
/* NMT (nmt v0.20.0; mirror test/util/malicious/hasher.go:186-309)            */
/* ------------------------------------------------------------------------- */
static const uint8_t PARITY_NS[ORC_NS_SIZE] = {
    0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
    0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF};

/* HashLeaf: ns || ns || SHA256(0x00 || ns || data) where ndata = ns || data. */
void orc_nmt_leaf(const uint8_t* ns, const uint8_t* data, size_t len, uint8_t out[90]) {
  uint8_t* buf = (uint8_t*)malloc(1 + ORC_NS_SIZE + len);
  buf[0] = 0x00;
  memcpy(buf + 1, ns, ORC_NS_SIZE);
  memcpy(buf + 1 + ORC_NS_SIZE, data, len);
  memcpy(out, ns, ORC_NS_SIZE);
  memcpy(out + ORC_NS_SIZE, ns, ORC_NS_SIZE);
  orc_sha256(buf, 1 + ORC_NS_SIZE + len, out + 2 * ORC_NS_SIZE);
  free(buf);
}

/* HashNode with ignoreMaxNs = true (hasher.go:271-309). */
void orc_nmt_node(const uint8_t left[90], const uint8_t right[90], uint8_t out[90]) {
  uint8_t buf[1 + 2 * ORC_NODE_SIZE];
  buf[0] = 0x01;
  memcpy(buf + 1, left, ORC_NODE_SIZE);
  memcpy(buf + 1 + ORC_NODE_SIZE, right, ORC_NODE_SIZE);
  uint8_t res[90];
  memcpy(res, left, ORC_NS_SIZE); /* minNs = left.min */
  if (memcmp(right, PARITY_NS, ORC_NS_SIZE) == 0)
    memcpy(res + ORC_NS_SIZE, left + ORC_NS_SIZE, ORC_NS_SIZE); /* left.max */
  else
    memcpy(res + ORC_NS_SIZE, right + ORC_NS_SIZE, ORC_NS_SIZE); /* right.max */
  orc_sha256(buf, sizeof buf, res + 2 * ORC_NS_SIZE);
  memcpy(out, res, 90);
}

static void nmt_root_rec(const uint8_t* leaves, size_t lo, size_t hi, uint8_t out[90]) {
  size_t n = hi - lo;
  if (n == 1) {
    memcpy(out, leaves + lo * ORC_NODE_SIZE, ORC_NODE_SIZE);
    return;
  }
  size_t split = 1;
  while (split * 2 < n) split *= 2; /* largest power of two < n */
  uint8_t l[90], r[90];
  nmt_root_rec(leaves, lo, lo + split, l);
  nmt_root_rec(leaves, lo + split, hi, r);
  orc_nmt_node(l, r, out);
}

void orc_nmt_root_from_leaves(const uint8_t* leaves, size_t n, uint8_t out[90]) {
  if (n == 0) {
    memset(out, 0, 2 * ORC_NS_SIZE); /* EmptyRoot: 0^29 || 0^29 || sha256("") */
    orc_sha256(NULL, 0, out + 2 * ORC_NS_SIZE);
    return;
  }
  nmt_root_rec(leaves, 0, n, out);
}

/* Wrapper tree over EDS axis: Push(share) for j in [0,2k) (nmt_wrapper.go:93-114). */
int orc_axis_root(int k, const uint8_t* eds, int axis, int index, uint8_t out[90]) {
  size_t w = 2 * (size_t)k;
  uint8_t* leaves = (uint8_t*)malloc(w * ORC_NODE_SIZE);
  const uint8_t* prev_ns = NULL;
  int rc = ORC_OK;
  for (size_t j = 0; j < w; j++) {
    size_t r = axis == 0 ? (size_t)index : j;
    size_t c = axis == 0 ? j : (size_t)index;
    const uint8_t* share = eds + (r * w + c) * SS;
    /* isQuadrantZero: shareIndex < squareSize && axisIndex < squareSize */
    int q0 = (j < (size_t)k) && ((size_t)index < (size_t)k);
    const uint8_t* ns = q0 ? share : PARITY_NS;
    /* nmt Push: ErrInvalidPushOrder if ns < previous ns */
    if (prev_ns && memcmp(ns, prev_ns, ORC_NS_SIZE) < 0) rc = ORC_ERR_PUSH_ORDER;
    prev_ns = ns;
    orc_nmt_leaf(ns, share, SS, leaves + j * ORC_NODE_SIZE);
  }
  if (rc == ORC_OK) orc_nmt_root_from_leaves(leaves, w, out);
  free(leaves);
  return rc;
}

typedef struct {
  int k;
  const uint8_t* eds;
  uint8_t* rr;
  uint8_t* cr;
  int next;        /* shared counter */
  int rc;
  pthread_mutex_t mu;
} roots_job_t;

static void* roots_worker(void* arg) {
  roots_job_t* J = (roots_job_t*)arg;
  int w = 2 * J->k;
  for (;;) {
    pthread_mutex_lock(&J->mu);
    int t = J->next++;
    pthread_mutex_unlock(&J->mu);
    if (t >= 2 * w) break;
    int axis = t & 1, idx = t >> 1;
    int rc = orc_axis_root(J->k, J->eds, axis, idx,
                           (axis == 0 ? J->rr : J->cr) + (size_t)idx * ORC_NODE_SIZE);
    if (rc != ORC_OK) {
      pthread_mutex_lock(&J->mu);
      if (J->rc == ORC_OK) J->rc = rc;
      pthread_mutex_unlock(&J->mu);
    }
  }
  return NULL;
}

int orc_compute_roots(int k, const uint8_t* eds, uint8_t* row_roots, uint8_t* col_roots,
                      int nthreads) {
  orc_init();
  roots_job_t J;
  J.k = k; J.eds = eds; J.rr = row_roots; J.cr = col_roots; J.next = 0; J.rc = ORC_OK;
  pthread_mutex_init(&J.mu, NULL);
  if (nthreads <= 1) {
    roots_worker(&J);
  } else {
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, roots_worker, &J);
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    free(th);
  }
  pthread_mutex_destroy(&J.mu);
  return J.rc;
}

/* RFC-6962 (celestia-core crypto/merkle/tree.go HashFromByteSlices). */
static void rfc_rec(const uint8_t* items, size_t lo, size_t hi, size_t len, uint8_t out[32]) {
  size_t n = hi - lo;
  if (n == 1) {
    uint8_t* buf = (uint8_t*)malloc(len + 1);
    buf[0] = 0x00;
    memcpy(buf + 1, items + lo * len, len);
    orc_sha256(buf, len + 1, out);
    free(buf);
    return;
  }
  size_t split = 1;
  while (split * 2 < n) split *= 2;
  uint8_t buf[65];
  buf[0] = 0x01;
  rfc_rec(items, lo, lo + split, len, buf + 1);
  rfc_rec(items, lo + split, hi, len, buf + 33);
  orc_sha256(buf, 65, out);
}

void orc_rfc6962_root(const uint8_t* items, size_t n, size_t item_len, uint8_t out[32]) {
  if (n == 0) {
    orc_sha256(NULL, 0, out);
    return;
  }
  rfc_rec(items, 0, n, item_len, out);
}

void orc_dah_hash(const uint8_t* row_roots, const uint8_t* col_roots, size_t w, uint8_t out[32]) {
  uint8_t* all = (uint8_t*)malloc(2 * w * ORC_NODE_SIZE + 1);
  memcpy(all, row_roots, w * ORC_NODE_SIZE);
  memcpy(all + w * ORC_NODE_SIZE, col_roots, w * ORC_NODE_SIZE);
  orc_rfc6962_root(all, 2 * w, ORC_NODE_SIZE, out);
  free(all);
}

/* ------------------------------------------------------------------------- */
/* Threaded extension (rsmt2d runs rows/cols in errgroup goroutines).          */
/* ------------------------------------------------------------------------- */
typedef struct {
  int k;
  uint8_t* eds;
  int phase;  /* 0: Q0 rows + Q0 cols, 1: Q2 rows */
  int next;
  pthread_mutex_t mu;
} ext_job_t;

static void* ext_worker(void* arg) {
  ext_job_t* J = (ext_job_t*)arg;
  int k = J->k;
  size_t w = 2 * (size_t)k;
  uint8_t* in = (uint8_t*)malloc((size_t)k * SS);
  uint8_t* out = (uint8_t*)malloc((size_t)k * SS);
  for (;;) {
    pthread_mutex_lock(&J->mu);
    int t = J->next++;
    pthread_mutex_unlock(&J->mu);
    if (J->phase == 0) {
      if (t >= 2 * k) break;
      if (t < k) {
        orc_encode(k, SS, J->eds + (t * w) * SS, J->eds + (t * w + k) * SS);
      } else {
        int c = t - k;
        for (int r = 0; r < k; r++) memcpy(in + (size_t)r * SS, J->eds + (r * w + c) * SS, SS);
        orc_encode(k, SS, in, out);
        for (int r = 0; r < k; r++)
          memcpy(J->eds + ((k + r) * w + c) * SS, out + (size_t)r * SS, SS);
      }
    } else {
      if (t >= k) break;
      size_t r = (size_t)k + t;
      orc_encode(k, SS, J->eds + (r * w) * SS, J->eds + (r * w + k) * SS);
    }
  }
  free(in);
  free(out);
  return NULL;
}

static void run_ext_phase(ext_job_t* J, int nthreads) {
  J->next = 0;
  if (nthreads <= 1) {
    ext_worker(J);
    return;
  }
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, ext_worker, J);
  for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
  free(th);
}

int orc_extend_and_dah(int k, const uint8_t* ods, uint8_t* eds, uint8_t* row_roots,
                       uint8_t* col_roots, uint8_t dah[32], int nthreads) {
  orc_init();
  if (!is_pow2(k)) return ORC_ERR_ARG;
  size_t w = 2 * (size_t)k;
  uint8_t* buf = eds ? eds : (uint8_t*)malloc(w * w * SS);
  for (int r = 0; r < k; r++)
    memcpy(buf + (r * w) * SS, ods + ((size_t)r * k) * SS, (size_t)k * SS);
  ext_job_t J;
  J.k = k; J.eds = buf;
  pthread_mutex_init(&J.mu, NULL);
  J.phase = 0;
  run_ext_phase(&J, nthreads);
  J.phase = 1;
  run_ext_phase(&J, nthreads);
  pthread_mutex_destroy(&J.mu);
  int rc = orc_compute_roots(k, buf, row_roots, col_roots, nthreads);
  if (rc == ORC_OK) orc_dah_hash(row_roots, col_roots, w, dah);
  if (!eds) free(buf);
  return rc;
}

/* ------------------------------------------------------------------------- */
/* rsmt2d Repair (prerepairSanityCheck + solveCrossword), v0.11.0 semantics.   */
/* ------------------------------------------------------------------------- */
static int axis_complete(int k, const uint8_t* present, int axis, int i) {
  int w = 2 * k;
  for (int j = 0; j < w; j++) {
    int r = axis == 0 ? i : j, c = axis == 0 ? j : i;
    if (!present[r * w + c]) return 0;
  }
  return 1;
}

static void gather_axis(int k, const uint8_t* eds, int axis, int i, uint8_t* out) {
  size_t w = 2 * (size_t)k;
  for (size_t j = 0; j < w; j++) {
    size_t r = axis == 0 ? (size_t)i : j, c = axis == 0 ? j : (size_t)i;
    memcpy(out + j * SS, eds + (r * w + c) * SS, SS);
  }
}

/* Root of an axis given as a contiguous 2k-share vector. */
static int vector_root(int k, int axis_index, const uint8_t* vec, uint8_t out[90]) {
  size_t w = 2 * (size_t)k;
  uint8_t* leaves = (uint8_t*)malloc(w * ORC_NODE_SIZE);
  const uint8_t* prev = NULL;
  int rc = ORC_OK;
  for (size_t j = 0; j < w; j++) {
    const uint8_t* s = vec + j * SS;
    int q0 = j < (size_t)k && axis_index < k;
    const uint8_t* ns = q0 ? s : PARITY_NS;
    if (prev && memcmp(ns, prev, ORC_NS_SIZE) < 0) rc = ORC_ERR_PUSH_ORDER;
    prev = ns;
    orc_nmt_leaf(ns, s, SS, leaves + j * ORC_NODE_SIZE);
  }
  if (rc == ORC_OK) orc_nmt_root_from_leaves(leaves, w, out);
  free(leaves);
  return rc;
}

/* byz (optional, 4 ints): {axis, index, rebuilt axis, rebuilt index}, -1 when
 * none.  ORC_ERR_BAD_ROOTS: the axis/index of the "bad root input" message;
 * ORC_ERR_BYZANTINE: ErrByzantineData{Axis, Index} plus the vector whose
 * repair failed (for an orthogonal-root failure the rebuilt row/column whose
 * shares rsmt2d attaches).  On a failure eds/present are left as before the
 * failing attempt, as rsmt2d leaves them.
 * prerepairSanityCheck: upstream runs the four checks of each i concurrently
 * (errgroup) and returns whichever fails first in time; this restatement takes
 * them in launch order: row i root, col i root, row i parity, col i parity. */
int orc_repair_ex(int k, uint8_t* eds, uint8_t* present, const uint8_t* row_roots,
                  const uint8_t* col_roots, int32_t* byz) {
  orc_init();
  if (byz) byz[0] = byz[1] = byz[2] = byz[3] = -1;
  if (!is_pow2(k)) return ORC_ERR_ARG;
  int w = 2 * k;
  uint8_t* vec = (uint8_t*)malloc((size_t)w * SS);
  uint8_t* pv = (uint8_t*)malloc((size_t)w);
  uint8_t root[90];
  uint8_t* par = (uint8_t*)malloc((size_t)k * SS);
  int rc = ORC_OK, fa = -1, fi = -1, ra = -1, ri = -1;
  /* prerepairSanityCheck */
  for (int i = 0; i < w && rc == ORC_OK; i++) {
    int complete[2] = {axis_complete(k, present, 0, i), axis_complete(k, present, 1, i)};
    for (int axis = 0; axis < 2 && rc == ORC_OK; axis++) {  /* roots */
      if (!complete[axis]) continue;
      gather_axis(k, eds, axis, i, vec);
      int r2 = vector_root(k, i, vec, root);
      if (r2 != ORC_OK) { rc = r2; break; }
      if (memcmp(root, (axis == 0 ? row_roots : col_roots) + (size_t)i * 90, 90) != 0) {
        rc = ORC_ERR_BAD_ROOTS;
        fa = ra = axis; fi = ri = i;
      }
    }
    for (int axis = 0; axis < 2 && rc == ORC_OK; axis++) {  /* parity == Encode(data) */
      if (!complete[axis]) continue;
      gather_axis(k, eds, axis, i, vec);
      orc_encode(k, SS, vec, par);
      if (memcmp(par, vec + (size_t)k * SS, (size_t)k * SS) != 0) {
        rc = ORC_ERR_BYZANTINE;
        fa = ra = axis; fi = ri = i;
      }
    }
  }
  /* solveCrossword */
  while (rc == ORC_OK) {
    int solved = 1, progress = 0;
    for (int i = 0; i < w && rc == ORC_OK; i++) {
      for (int axis = 0; axis < 2 && rc == ORC_OK; axis++) {
        if (axis_complete(k, present, axis, i)) continue;
        int cnt = 0;
        for (int j = 0; j < w; j++) {
          int r = axis == 0 ? i : j, c = axis == 0 ? j : i;
          pv[j] = present[r * w + c];
          cnt += pv[j] != 0;
        }
        if (cnt < k) { solved = 0; continue; }
        gather_axis(k, eds, axis, i, vec);
        for (int j = 0; j < w; j++)
          if (!pv[j]) memset(vec + (size_t)j * SS, 0, SS);
        orc_decode(k, SS, vec, pv);
        int r2 = vector_root(k, i, vec, root);
        if (r2 != ORC_OK || memcmp(root, (axis == 0 ? row_roots : col_roots) + (size_t)i * 90, 90)) {
          rc = ORC_ERR_BYZANTINE;
          fa = ra = axis; fi = ri = i;
          break;
        }
        /* newly completed orthogonal axes */
        for (int j = 0; j < w && rc == ORC_OK; j++) {
          if (pv[j]) continue;
          int r = axis == 0 ? i : j, c = axis == 0 ? j : i;
          int oi = axis == 0 ? c : r;  /* orthogonal index */
          int full = 1;
          for (int t = 0; t < w; t++) {
            int rr = axis == 0 ? t : oi, cc = axis == 0 ? oi : t;
            if (rr == r && cc == c) continue;
            if (!present[rr * w + cc]) { full = 0; break; }
          }
          if (!full) continue;
          uint8_t* ov = (uint8_t*)malloc((size_t)w * SS);
          gather_axis(k, eds, 1 - axis, oi, ov);
          int pos = axis == 0 ? r : c;
          memcpy(ov + (size_t)pos * SS, vec + (size_t)j * SS, SS);
          int r3 = vector_root(k, oi, ov, root);
          if (r3 != ORC_OK ||
              memcmp(root, (axis == 0 ? col_roots : row_roots) + (size_t)oi * 90, 90)) {
            rc = ORC_ERR_BYZANTINE;
            fa = 1 - axis; fi = oi; ra = axis; ri = i;
          }
          free(ov);
        }
        if (rc != ORC_OK) break;
        for (int j = 0; j < w; j++) {
          int r = axis == 0 ? i : j, c = axis == 0 ? j : i;
          if (!present[r * w + c]) {
            memcpy(eds + ((size_t)r * w + c) * SS, vec + (size_t)j * SS, SS);
            present[r * w + c] = 1;
          }
        }
        progress = 1;
      }
    }
    if (rc != ORC_OK) break;
    int all = 1;
    for (int i = 0; i < w * w; i++)
      if (!present[i]) { all = 0; break; }
    if (all) break;
    (void)solved;
    if (!progress) { rc = ORC_ERR_UNREPAIRABLE; break; }
  }
  if (byz && (rc == ORC_ERR_BYZANTINE || rc == ORC_ERR_BAD_ROOTS)) {
    byz[0] = fa; byz[1] = fi; byz[2] = ra; byz[3] = ri;
  }
  free(vec);
  free(pv);
  free(par);
  return rc;
}

int orc_repair(int k, uint8_t* eds, uint8_t* present, const uint8_t* row_roots,
               const uint8_t* col_roots) {
  return orc_repair_ex(k, eds, present, row_roots, col_roots, NULL);
}
