/* asan_check.c -- drives the oracle (test infrastructure) under
 * AddressSanitizer + UndefinedBehaviorSanitizer (sanitizers on
 * the host layer).  Exercises every entry point of da_oracle.h on small
 * inputs, including ragged/odd sizes and erasure patterns, and checks the
 * round-trip identities (decode(encode) == data, repair(erased EDS) == EDS).
 * Built and run by `make -C oracle asan` (tests/test_oracle_asan.py). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "da_oracle.h"

static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {
  g_rng ^= g_rng << 13;
  g_rng ^= g_rng >> 7;
  g_rng ^= g_rng << 17;
  return (uint32_t)(g_rng >> 11);
}

static void fill(uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; i++) p[i] = (uint8_t)rnd();
}

/* sorted random-namespace square: namespace = version 0, 18 zeros, then the
 * share index big-endian in the last bytes (row-major order is sorted) */
static void square(int k, uint8_t* ods) {
  fill(ods, (size_t)k * k * 512);
  for (int i = 0; i < k * k; i++) {
    uint8_t* s = ods + (size_t)i * 512;
    memset(s, 0, 25);
    s[25] = (uint8_t)(i >> 24);
    s[26] = (uint8_t)(i >> 16);
    s[27] = (uint8_t)(i >> 8);
    s[28] = (uint8_t)i;
  }
}

static int fails = 0;
#define CHECK(c, ...)                  \
  do {                                 \
    if (!(c)) {                        \
      fprintf(stderr, __VA_ARGS__);    \
      fprintf(stderr, "\n");           \
      fails++;                         \
    }                                  \
  } while (0)

int main(void) {
  orc_init();
  uint8_t h[32];
  for (size_t len = 0; len < 300; len += 7) {  /* every padding case */
    uint8_t* m = malloc(len + 1);
    fill(m, len);
    orc_sha256(m, len, h);
    free(m);
  }
  /* codec round trips, GF(2^8) and GF(2^16) */
  const int ks[] = {1, 2, 4, 8, 16, 64, 128, 256, 512};
  for (size_t t = 0; t < sizeof ks / sizeof ks[0]; t++) {
    const int k = ks[t];
    const size_t shard = k > 128 ? 64 : 128;  /* orc_encode: k a power of two */
    uint8_t* sh = malloc(2 * k * shard);
    uint8_t* ref = malloc(2 * k * shard);
    uint8_t* pres = malloc(2 * k);
    fill(sh, k * shard);
    CHECK(orc_encode(k, shard, sh, sh + k * shard) == 0, "encode k=%d", k);
    memcpy(ref, sh, 2 * k * shard);
    for (int i = 0; i < 2 * k; i++) pres[i] = 1;
    int erased = 0;
    for (int i = 0; i < 2 * k && erased < k; i++)
      if (rnd() & 1) {
        pres[i] = 0;
        memset(sh + i * shard, 0, shard);
        erased++;
      }
    CHECK(orc_decode(k, shard, sh, pres) == 0, "decode k=%d", k);
    CHECK(memcmp(sh, ref, 2 * k * shard) == 0, "decode mismatch k=%d", k);
    for (int i = 0; i < 2 * k; i++) pres[i] = i < k - 1;  /* one too few */
    if (k > 1) CHECK(orc_decode(k, shard, sh, pres) != 0, "too few shards accepted k=%d", k);
    free(sh);
    free(ref);
    free(pres);
  }
  /* extend + roots + DAH + repair */
  for (int k = 1; k <= 16; k *= 2) {
    const int w = 2 * k;
    uint8_t* ods = malloc((size_t)k * k * 512);
    uint8_t* eds = malloc((size_t)w * w * 512);
    uint8_t* ref = malloc((size_t)w * w * 512);
    uint8_t* rr = malloc((size_t)w * 90);
    uint8_t* cr = malloc((size_t)w * 90);
    uint8_t* pres = malloc((size_t)w * w);
    uint8_t dah[32], dah2[32];
    square(k, ods);
    CHECK(orc_extend_and_dah(k, ods, eds, rr, cr, dah, 1) == 0, "extend k=%d", k);
    CHECK(orc_extend_and_dah(k, ods, NULL, rr, cr, dah2, 2) == 0 && !memcmp(dah, dah2, 32),
          "extend (no eds, 2 threads) k=%d", k);
    memcpy(ref, eds, (size_t)w * w * 512);
    uint8_t node[90];
    CHECK(orc_axis_root(k, eds, 1, w - 1, node) == 0 && !memcmp(node, cr + (w - 1) * 90, 90), "axis root k=%d", k);
    /* keep a random k x k sub-grid (the maximal recoverable erasure) */
    memset(pres, 0, (size_t)w * w);
    int rows[32], cols[32];
    for (int i = 0; i < w; i++) rows[i] = cols[i] = i;
    for (int i = w - 1; i > 0; i--) {
      int j = rnd() % (i + 1), t = rows[i];
      rows[i] = rows[j]; rows[j] = t;
      j = rnd() % (i + 1); t = cols[i]; cols[i] = cols[j]; cols[j] = t;
    }
    for (int a = 0; a < k; a++)
      for (int b = 0; b < k; b++) pres[rows[a] * w + cols[b]] = 1;
    for (int c = 0; c < w * w; c++)
      if (!pres[c]) memset(eds + (size_t)c * 512, 0, 512);
    CHECK(orc_repair(k, eds, pres, rr, cr) == 0, "repair k=%d", k);
    CHECK(memcmp(eds, ref, (size_t)w * w * 512) == 0, "repair mismatch k=%d", k);
    /* unsorted square -> push-order error, no memory error */
    if (k > 1) {
      memcpy(ods, ods + 512, 29);
      ods[28] = 0xFF;
      CHECK(orc_extend_and_dah(k, ods, eds, rr, cr, dah, 1) != 0, "push order k=%d", k);
    }
    free(ods); free(eds); free(ref); free(rr); free(cr); free(pres);
  }
  /* RFC-6962 over ragged item counts */
  for (size_t n = 0; n < 40; n++) {
    uint8_t items[40 * 90];
    fill(items, sizeof items);
    orc_rfc6962_root(items, n, 90, h);
  }
  printf("asan_check %s (%d failures)\n", fails ? "FAILED" : "ok", fails);
  return fails != 0;
}
