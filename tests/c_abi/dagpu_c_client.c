/* dagpu_c_client.c -- a plain C consumer of include/dagpu.h, calling the
 * library the way the cgo binding in INTEGRATION.md would (flat buffers, int
 * status codes, no Python, no torch).  Prints one "name value" line per check;
 * tests/test_gpu_c_client.py runs it on the GPU box and compares against the
 * reference's golden DAH hashes (pkg/da/data_availability_header_test.go).
 * Built by __graft_entry__.build() / `make -C celestia-app_amd c_client`. */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "../../include/dagpu.h"

#define SHARE 512

static void hex(const char* name, const uint8_t* h, int n) {
  printf("%s ", name);
  for (int i = 0; i < n; i++) printf("%02x", h[i]);
  printf("\n");
}

/* pkg/shares/padding.go TailPaddingShare: ns 0xFF*28|0xFE, info 0x01, seq len 0 */
static void tail_padding_share(uint8_t* s) {
  memset(s, 0, SHARE);
  memset(s, 0xFF, 28);
  s[28] = 0xFE;
  s[29] = 0x01;
}

/* the reference test's constant share: ns v0 with sub-ID 0x01*10, rest 0xFF */
static void constant_share(uint8_t* s) {
  memset(s, 0xFF, SHARE);
  memset(s, 0, 19);
  memset(s + 19, 0x01, 10);
}

static uint8_t* constant_square(int k, uint8_t* dst) {
  for (int i = 0; i < k * k; i++) constant_share(dst + (size_t)i * SHARE);
  return dst;
}

struct worker {
  int device, iters, k, ok;
  uint8_t want[32];
};

static void* run_worker(void* p) {
  struct worker* w = (struct worker*)p;
  dagpu_ctx* ctx = NULL;
  if (dagpu_init(w->device, &ctx) != DAGPU_OK) return NULL;
  const int k = w->k, wid = 2 * k;
  uint8_t* sq = (uint8_t*)malloc((size_t)k * k * SHARE);
  uint8_t* rr = (uint8_t*)malloc((size_t)wid * 90);
  uint8_t* cr = (uint8_t*)malloc((size_t)wid * 90);
  uint8_t dah[32];
  constant_square(k, sq);
  w->ok = 1;
  for (int i = 0; i < w->iters; i++) {
    if (dagpu_extend_shares(ctx, sq, (size_t)k * k, SHARE, NULL, rr, cr, dah) != DAGPU_OK ||
        memcmp(dah, w->want, 32) != 0)
      w->ok = 0;
  }
  free(sq);
  free(rr);
  free(cr);
  dagpu_destroy(ctx);
  return NULL;
}

int main(void) {
  setvbuf(stdout, NULL, _IOLBF, 0);
  dagpu_ctx* ctx = NULL;
  int rc = dagpu_init(0, &ctx);
  printf("init %d\n", rc);
  if (rc != DAGPU_OK) return 1;
  printf("version %d\n", dagpu_version());

  uint8_t rr[256 * 90], cr[256 * 90], dah[32];
  /* MinDataAvailabilityHeader: one tail padding share */
  uint8_t share[SHARE];
  tail_padding_share(share);
  rc = dagpu_extend_shares(ctx, share, 1, SHARE, NULL, rr, cr, dah);
  printf("min_rc %d\n", rc);
  hex("min_dah", dah, 32);

  /* typical 2x2 of constant shares, with the EDS returned */
  uint8_t sq2[4 * SHARE], eds2[16 * SHARE];
  rc = dagpu_extend_shares(ctx, constant_square(2, sq2), 4, SHARE, eds2, rr, cr, dah);
  printf("typical_rc %d\n", rc);
  hex("typical_dah", dah, 32);
  printf("typical_q0_kept %d\n", memcmp(eds2, sq2, SHARE) == 0 && memcmp(eds2 + 4 * SHARE, sq2 + 2 * SHARE, SHARE) == 0);

  /* max 128x128 constant squares through the batched API on page-locked memory */
  const int k = 128, n = 3;
  const size_t ods_b = (size_t)k * k * SHARE;
  uint8_t* ods = (uint8_t*)dagpu_host_alloc(ods_b * n);
  printf("host_alloc %d\n", ods != NULL);
  if (!ods) return 1;
  for (int i = 0; i < n; i++) constant_square(k, ods + i * ods_b);
  uint32_t ks[3] = {128, 128, 128};
  uint8_t* brr = (uint8_t*)malloc((size_t)n * 2 * k * 90);
  uint8_t* bcr = (uint8_t*)malloc((size_t)n * 2 * k * 90);
  uint8_t bdah[3 * 32];
  int32_t st[3] = {-1, -1, -1};
  rc = dagpu_extend_batch(ctx, ods, ks, n, NULL, brr, bcr, bdah, st);
  printf("max_rc %d %d %d %d\n", rc, st[0], st[1], st[2]);
  hex("max_dah", bdah, 32);
  printf("max_all_equal %d\n", memcmp(bdah, bdah + 32, 32) == 0 && memcmp(bdah, bdah + 64, 32) == 0);
  dagpu_host_free(ods);
  free(brr);
  free(bcr);

  /* pipelined host batches: 37 squares of k = 8 in chunks of 5 (copy stream +
   * compute stream + page-locked staging), one unsorted square in chunk 4 */
  {
    const int pk = 8, pn = 37;
    const size_t pb = (size_t)pk * pk * SHARE;
    uint8_t* p_ods = (uint8_t*)malloc(pb * pn);
    uint32_t pks[37];
    for (int i = 0; i < pn; i++) {
      constant_square(pk, p_ods + i * pb);
      pks[i] = pk;
    }
    p_ods[21 * pb + 28] = 0x09;
    uint8_t* prr = (uint8_t*)malloc((size_t)pn * 2 * pk * 90);
    uint8_t* pcr = (uint8_t*)malloc((size_t)pn * 2 * pk * 90);
    uint8_t pdah[37 * 32], sdah[37 * 32];
    int32_t pst[37], sst[37];
    setenv("DAGPU_PIPELINE_CHUNK", "5", 1);
    int prc = dagpu_extend_batch(ctx, p_ods, pks, pn, NULL, prr, pcr, pdah, pst);
    setenv("DAGPU_PIPELINE_CHUNK", "100000", 1);
    int src = dagpu_extend_batch(ctx, p_ods, pks, pn, NULL, prr, pcr, sdah, sst);
    unsetenv("DAGPU_PIPELINE_CHUNK");
    int same = memcmp(pdah, sdah, sizeof pdah) == 0 && memcmp(pst, sst, sizeof pst) == 0;
    int bad = 0;
    for (int i = 0; i < pn; i++) bad += pst[i] != 0;
    printf("pipelined %d %d %d %d %d\n", prc, src, same, bad, pst[21]);
    free(p_ods);
    free(prr);
    free(pcr);
  }

  /* ExtendShares errors: not a power of two; not a square */
  uint8_t three[3 * SHARE];
  memset(three, 0, sizeof three);
  rc = dagpu_extend_shares(ctx, three, 3, SHARE, NULL, rr, cr, dah);
  printf("err_not_pow2 %d %s\n", rc, dagpu_last_error(ctx));
  uint8_t two[2 * SHARE];
  memset(two, 0, sizeof two);
  rc = dagpu_extend_shares(ctx, two, 2, SHARE, NULL, rr, cr, dah);
  printf("err_not_square %d\n", rc);
  /* unsorted namespaces -> push-order error, still a DAGPU status (not a crash) */
  uint8_t unsorted[4 * SHARE];
  constant_square(2, unsorted);
  unsorted[28] = 0x09; /* share 0 namespace > share 1 namespace */
  rc = dagpu_extend_shares(ctx, unsorted, 4, SHARE, NULL, rr, cr, dah);
  printf("err_push_order %d\n", rc);

  /* rsmt2d.Codec: encode of all-zero data is all-zero parity */
  uint8_t data[4 * 64], parity[4 * 64];
  memset(data, 0, sizeof data);
  memset(parity, 0xAA, sizeof parity);
  rc = dagpu_encode(ctx, 4, 1, 64, data, parity);
  int zero = 1;
  for (size_t i = 0; i < sizeof parity; i++) zero &= parity[i] == 0;
  printf("codec_zero %d %d\n", rc, zero);

  /* concurrent callers, one context per host thread (the cgo threading model) */
  struct worker ws[4];
  pthread_t th[4];
  uint8_t want[32];
  dagpu_extend_shares(ctx, constant_square(2, sq2), 4, SHARE, NULL, rr, cr, want);
  for (int i = 0; i < 4; i++) {
    ws[i].device = 0;
    ws[i].iters = 25;
    ws[i].k = 2;
    ws[i].ok = 0;
    memcpy(ws[i].want, want, 32);
    pthread_create(&th[i], NULL, run_worker, &ws[i]);
  }
  int all = 1;
  for (int i = 0; i < 4; i++) {
    pthread_join(th[i], NULL);
    all &= ws[i].ok;
  }
  printf("threads_ok %d\n", all);
  dagpu_destroy(ctx);
  printf("done\n");
  fflush(stdout);
  /* Under the host-ASan build the sanitizer's device-allocator hooks trip
   * during the HIP runtime's own atexit teardown; skip static destructors. */
  if (getenv("DAGPU_CLIENT_QUICK_EXIT")) _exit(0);
  return 0;
}
