/*
 * da_oracle.h -- CPU restatement of celestia-app's data-availability hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * product path (celestia-app_amd/) and the "port" CPU baseline in bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it.  The product path never links or calls it.
 *
 * What it restates (reference = /root/reference, module celestia-app; the
 * arithmetic lives in pinned, un-vendored Go modules -- see SURVEY.md §0):
 *   - klauspost/reedsolomon v1.11.8 leopard8.go (GF(2^8) Leopard RS; reached via
 *     pkg/appconsts/global_consts.go:92 DefaultCodec = rsmt2d.NewLeoRSCodec)
 *   - klauspost/reedsolomon v1.11.8 leopard.go (GF(2^16), used when 2k > 256)
 *   - celestiaorg/rsmt2d v0.11.0 ComputeExtendedDataSquare / Repair
 *     (called at pkg/da/data_availability_header.go:74)
 *   - celestiaorg/nmt v0.20.0 hasher (in-tree copy: test/util/malicious/hasher.go:161-309)
 *   - pkg/wrapper/nmt_wrapper.go:93-140 (parity-namespace rule)
 *   - celestia-core crypto/merkle HashFromByteSlices (RFC-6962), called at
 *     pkg/da/data_availability_header.go:92-108
 * Pinned by: pkg/da/data_availability_header_test.go:15-54 golden hashes
 * (nil DAH, MinDAH, 2x2, 128x128) -- see tests/test_oracle_golden.py.
 * GF(2^16) has no reference golden vector: parity unpinned for k > 128.
 */
#ifndef DA_ORACLE_H
#define DA_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_SHARE_SIZE 512
#define ORC_NS_SIZE 29
#define ORC_NODE_SIZE 90 /* minNs(29) | maxNs(29) | sha256(32) */

enum {
  ORC_OK = 0,
  ORC_ERR_NOT_POW2 = -1,       /* "number of shares is not a power of 2" */
  ORC_ERR_NOT_SQUARE = -2,     /* rsmt2d: "number of chunks must be a square number" */
  ORC_ERR_SHARE_SIZE = -3,     /* shard size not a multiple of 64 / unequal chunks */
  ORC_ERR_PUSH_ORDER = -4,     /* nmt ErrInvalidPushOrder */
  ORC_ERR_TOO_FEW = -5,        /* reedsolomon ErrTooFewShards */
  ORC_ERR_UNREPAIRABLE = -6,   /* rsmt2d ErrUnrepairableDataSquare */
  ORC_ERR_BYZANTINE = -7,      /* rsmt2d ErrByzantineData */
  ORC_ERR_BAD_ROOTS = -8,      /* rsmt2d "bad root input" */
  ORC_ERR_ARG = -9
};

void orc_init(void);

/* SHA-256 of a byte string. */
void orc_sha256(const uint8_t* msg, size_t len, uint8_t out[32]);

/* GF(2^8) Leopard tables (klauspost leopard8.go initLUTs8 / initFFTSkew8). */
const uint8_t* orc_gf8_log(void);   /* 256 */
const uint8_t* orc_gf8_exp(void);   /* 256 */
const uint8_t* orc_gf8_skew(void);  /* 255 */
const uint8_t* orc_gf8_logwalsh(void); /* 256 */
uint8_t orc_gf8_mullog(uint8_t a, uint8_t log_b);

/* GF(2^16) Leopard tables (klauspost leopard.go). */
const uint16_t* orc_gf16_log(void);  /* 65536 */
const uint16_t* orc_gf16_exp(void);  /* 65536 */
const uint16_t* orc_gf16_skew(void); /* 65535 */

/* Systematic Leopard encode: k data shards (contiguous, k*shard bytes) ->
 * k parity shards.  GF(2^8) when 2k <= 256 else GF(2^16) (reedsolomon.New(k,k,
 * WithLeopardGF(true))).  k a power of two (the widths rsmt2d uses); shard
 * must be a multiple of 64. */
int orc_encode(int k, size_t shard, const uint8_t* data, uint8_t* parity);

/* Leopard reconstruct (reedsolomon Reconstruct): shards is 2k*shard bytes,
 * present[i] != 0 marks shard i as present; missing shards are filled in. */
int orc_decode(int k, size_t shard, uint8_t* shards, const uint8_t* present);

/* rsmt2d ComputeExtendedDataSquare with 512-B shares: ods = k*k*512 row-major,
 * eds = (2k)*(2k)*512 row-major. */
int orc_extend_square(int k, const uint8_t* ods, uint8_t* eds);

/* NMT primitives (nmt v0.20.0 hasher, IgnoreMaxNamespace=true, 29-B ns). */
void orc_nmt_leaf(const uint8_t* ns, const uint8_t* data, size_t len, uint8_t out[90]);
void orc_nmt_node(const uint8_t left[90], const uint8_t right[90], uint8_t out[90]);
/* Root over n 90-B leaf nodes (RFC-6962 split). */
void orc_nmt_root_from_leaves(const uint8_t* leaves, size_t n, uint8_t out[90]);

/* Wrapper tree root of one EDS axis (pkg/wrapper/nmt_wrapper.go).
 * axis 0 = row, 1 = column.  Returns ORC_ERR_PUSH_ORDER on an unsorted axis. */
int orc_axis_root(int k, const uint8_t* eds, int axis, int index, uint8_t out[90]);

/* All 2w row roots and 2w col roots.  nthreads <= 1 -> single thread. */
int orc_compute_roots(int k, const uint8_t* eds, uint8_t* row_roots, uint8_t* col_roots,
                      int nthreads);

/* RFC-6962 root over n items of item_len bytes (crypto/merkle HashFromByteSlices). */
void orc_rfc6962_root(const uint8_t* items, size_t n, size_t item_len, uint8_t out[32]);

/* DAH hash = RFC-6962(rowRoots || colRoots), w = 2k roots each. */
void orc_dah_hash(const uint8_t* row_roots, const uint8_t* col_roots, size_t w, uint8_t out[32]);

/* Full hot path: ExtendShares + NewDataAvailabilityHeader + Hash.
 * eds may be NULL (a scratch buffer is used). */
int orc_extend_and_dah(int k, const uint8_t* ods, uint8_t* eds, uint8_t* row_roots,
                       uint8_t* col_roots, uint8_t dah[32], int nthreads);

/* rsmt2d Repair: eds (2k)^2*512 with present[(2k)^2] flags; missing cells are
 * filled in place.  Verifies rebuilt axes against the given roots. */
int orc_repair(int k, uint8_t* eds, uint8_t* present, const uint8_t* row_roots,
               const uint8_t* col_roots);
int orc_repair_ex(int k, uint8_t* eds, uint8_t* present, const uint8_t* row_roots,
                  const uint8_t* col_roots, int32_t* byz);

#ifdef __cplusplus
}
#endif
#endif
