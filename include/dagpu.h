/*
 * dagpu.h -- C ABI of the MI355X-native celestia-app data-availability hot path.
 *
 * Library: celestia-app_amd/libdagpu.so (hipcc --offload-arch=gfx950).
 * Plain pointers and sizes only; the caller owns every buffer and nothing is
 * retained after a call returns.  Each entry point names the reference
 * interface it replaces (paths relative to the reference repo root).  The Go
 * (cgo) binding a maintainer would add on the reference side is in
 * INTEGRATION.md.
 *
 * Layouts
 *   share      512 bytes (appconsts.ShareSize, pkg/appconsts/global_consts.go:29)
 *   ODS        k*k shares, row-major                     (k*k*512 B)
 *   EDS        (2k)*(2k) shares, row-major, Q0|Q1 / Q2|Q3 ((2k)^2*512 B)
 *   root       90 bytes = minNs(29) | maxNs(29) | sha256(32)
 *   row_roots  2k roots, col_roots 2k roots, dah 32 bytes
 *   batches    squares packed back to back in each array (mixed-k batches:
 *              square i starts after the bytes of squares 0..i-1)
 *
 * Errors: functions return 0 or a negative dagpu_status; batch calls also
 * fill a per-square status array.  dagpu_last_error() gives the message of the
 * calling thread's last failure on that context (errno-like; a thread that has
 * not failed on it gets the context's most recent message), same wording as
 * the reference where one exists.
 * Threading: a context is thread-safe.  Host-memory calls are serialised on
 * it; device-resident (*_device) calls take no lock and may be issued from
 * several threads at once, each on its own stream with its own buffers.
 */
#ifndef DAGPU_H
#define DAGPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DAGPU_SHARE_SIZE 512
#define DAGPU_NAMESPACE_SIZE 29
#define DAGPU_ROOT_SIZE 90
#define DAGPU_HASH_SIZE 32

typedef enum dagpu_status {
  DAGPU_OK = 0,
  DAGPU_ERR_NOT_POW2 = -1,       /* pkg/da/data_availability_header.go:67-69 */
  DAGPU_ERR_NOT_SQUARE = -2,     /* rsmt2d newDataSquare: "number of chunks must be a square number" */
  DAGPU_ERR_SHARE_SIZE = -3,     /* shares not all 512 B / shard not a multiple of 64 */
  DAGPU_ERR_PUSH_ORDER = -4,     /* nmt ErrInvalidPushOrder (Q0 namespaces unsorted) */
  DAGPU_ERR_TOO_FEW_SHARDS = -5, /* reedsolomon ErrTooFewShards */
  DAGPU_ERR_UNREPAIRABLE = -6,   /* rsmt2d ErrUnrepairableDataSquare */
  DAGPU_ERR_BYZANTINE = -7,      /* rsmt2d ErrByzantineData */
  DAGPU_ERR_BAD_ROOTS = -8,      /* rsmt2d "bad root input" */
  DAGPU_ERR_ARG = -9,
  DAGPU_ERR_DEVICE = -10,        /* HIP runtime failure */
  DAGPU_ERR_UNSUPPORTED = -11,   /* e.g. k above what this build implements */
  DAGPU_ERR_PROOF = -12,         /* a proof does not verify against the given root */
  DAGPU_ERR_SQUARE = -13         /* square construction rejected the txs (pkg/square errors) */
} dagpu_status;

typedef struct dagpu_ctx dagpu_ctx;

/* Library version (major*10000 + minor*100 + patch). */
int dagpu_version(void);

/* Widest square one GPU serves: DAGPU_MAX_SQUARE_WIDTH (the split square
 * goes to DAGPU_MAX_SPLIT_WIDTH over >= 8 GPUs, codec vectors to
 * DAGPU_MAX_CODEC_WIDTH).  pkg/da ExtendShares (data_availability_header.go:65-75)
 * checks only that the share count is a power of two, and rsmt2d's LeoRSCodec
 * reports MaxChunks() = 32768 * 32768 (Leopard GF(2^16): 65536 shards); the EDS
 * of k = 8192 is 128 GiB, which fits one MI355X's 288 GB of HBM, and k = 16384
 * (512 GiB) does not, so every square entry point returns DAGPU_ERR_UNSUPPORTED
 * above it. */
#define DAGPU_MAX_SQUARE_WIDTH 8192
uint32_t dagpu_max_square_width(void);

/* Widest codec vector (k data shards) dagpu_encode / dagpu_decode serve:
 * Leopard GF(2^16)'s limit, k + k = 65536 shards (klauspost/reedsolomon
 * leopardFF16 New: dataShards + parityShards <= 65536).  A cgo
 * LeoRSCodec.MaxChunks() over this library returns the square of it, as
 * rsmt2d's own (32768 * 32768).  DAGPU_ERR_UNSUPPORTED above it. */
#define DAGPU_MAX_CODEC_WIDTH 32768
uint32_t dagpu_max_codec_width(void);

/* Open a context on HIP device `device` (one context per GPU per process). */
int dagpu_init(int device, dagpu_ctx** out);
void dagpu_destroy(dagpu_ctx* ctx);
const char* dagpu_last_error(dagpu_ctx* ctx);  /* NULL: this thread's last context-free call */

/* Replaces da.ExtendShares + da.NewDataAvailabilityHeader + dah.Hash()
 * (pkg/da/data_availability_header.go:65-75, :44-63, :92-108) for one square.
 * shares: n_shares * share_size bytes (host).  eds_out may be NULL (roots/DAH
 * only, the device-resident default).  Errors as ExtendShares: n_shares not a
 * power of two -> DAGPU_ERR_NOT_POW2; not a square -> DAGPU_ERR_NOT_SQUARE;
 * unsorted Q0 namespaces -> DAGPU_ERR_PUSH_ORDER (NewDataAvailabilityHeader). */
int dagpu_extend_shares(dagpu_ctx* ctx, const uint8_t* shares, size_t n_shares,
                        size_t share_size, uint8_t* eds_out, uint8_t* row_roots,
                        uint8_t* col_roots, uint8_t* dah);

/* Batched host-memory form (app/extend_block.go:14-22 block replay; mixed k).
 * k[i] = original square width of square i.  status[i] gets a dagpu_status.
 * Returns DAGPU_OK if every square succeeded, else the first failing status.
 * A run of equal k larger than ~128 MiB of ODS is pipelined: chunk c goes up
 * on a copy stream while chunk c-1 is extended.  Host->device copies run at
 * PCIe speed only from page-locked memory: allocate `ods` with
 * dagpu_host_alloc or pin it with dagpu_host_register. */
int dagpu_extend_batch(dagpu_ctx* ctx, const uint8_t* ods, const uint32_t* k, size_t n,
                       uint8_t* eds_or_null, uint8_t* row_roots, uint8_t* col_roots,
                       uint8_t* dah, int32_t* status);

/* Page-locked host memory for dagpu_extend_batch inputs (hipHostMalloc /
 * hipHostRegister).  dagpu_host_alloc returns NULL on failure. */
void* dagpu_host_alloc(size_t bytes);
void dagpu_host_free(void* p);
int dagpu_host_register(void* p, size_t bytes);
int dagpu_host_unregister(void* p);

/* Device-resident batch, one k for all n squares; every pointer is device
 * memory; work is enqueued on `stream` (hipStream_t, NULL = default stream) and
 * the call returns without synchronising.  d_ods may be NULL when Q0 is already
 * in place inside d_eds.  d_status: n int32 bitmasks (0 = OK, 1 = push order).
 * d_workspace: dagpu_workspace_size(k, n) bytes. */
size_t dagpu_workspace_size(uint32_t k, size_t n);
int dagpu_extend_batch_device(dagpu_ctx* ctx, uint32_t k, size_t n, const uint8_t* d_ods,
                              uint8_t* d_eds, uint8_t* d_row_roots, uint8_t* d_col_roots,
                              uint8_t* d_dah, int32_t* d_status, void* d_workspace,
                              void* stream);

/* Device-resident stages (for profiling and for callers that already hold an
 * EDS on the device): RS extension only, and NMT roots + DAH only. */
int dagpu_extend_rs_device(dagpu_ctx* ctx, uint32_t k, size_t n, const uint8_t* d_ods,
                           uint8_t* d_eds, void* stream);
int dagpu_roots_device(dagpu_ctx* ctx, uint32_t k, size_t n, const uint8_t* d_eds,
                       uint8_t* d_row_roots, uint8_t* d_col_roots, uint8_t* d_dah,
                       int32_t* d_status, void* d_workspace, void* stream);

/* Replaces NewDataAvailabilityHeader(eds) for an EDS already in host memory
 * (rsmt2d RowRoots/ColRoots + Hash). */
int dagpu_roots(dagpu_ctx* ctx, uint32_t k, const uint8_t* eds, uint8_t* row_roots,
                uint8_t* col_roots, uint8_t* dah);

/* rsmt2d.Codec (LeoRSCodec, pkg/appconsts/global_consts.go:92) Encode over many
 * vectors: data = nvec * k shards of shard_size bytes (contiguous per vector),
 * parity = nvec * k shards.  shard_size must be a multiple of 64. */
int dagpu_encode(dagpu_ctx* ctx, uint32_t k, size_t nvec, size_t shard_size,
                 const uint8_t* data, uint8_t* parity);

/* rsmt2d.Codec Decode (klauspost Reconstruct via Leopard GF(2^8)): shards =
 * nvec * 2k shards of shard_size bytes, present = nvec * 2k flags (non-zero =
 * shard present).  Missing shards are rebuilt in place.  Needs >= k present
 * per vector (DAGPU_ERR_TOO_FEW_SHARDS otherwise). */
int dagpu_decode(dagpu_ctx* ctx, uint32_t k, size_t nvec, size_t shard_size,
                 uint8_t* shards, const uint8_t* present);

/* rsmt2d ExtendedDataSquare.Repair for one square in host memory: eds is
 * (2k)^2 * 512 bytes with present[(2k)^2] flags; missing cells are filled in
 * place and every row/column root is re-verified against row_roots/col_roots
 * (DAGPU_ERR_BYZANTINE on mismatch, DAGPU_ERR_UNREPAIRABLE if the crossword
 * cannot be solved, DAGPU_ERR_BAD_ROOTS if a complete axis disagrees up front). */
int dagpu_repair(dagpu_ctx* ctx, uint32_t k, uint8_t* eds, uint8_t* present,
                 const uint8_t* row_roots, const uint8_t* col_roots);

/* dagpu_repair plus the failing axis, for rsmt2d's ErrByzantineData{Axis,
 * Index, Shares} (the input of celestia-node's bad-encoding fraud proof) and
 * its "bad root input: <axis> <i> ..." error.  byz (4 int32, may be NULL) =
 * {axis (0 row, 1 col), index, rebuilt axis, rebuilt index}, all -1 when the
 * status is neither DAGPU_ERR_BYZANTINE nor DAGPU_ERR_BAD_ROOTS.
 *   - prerepairSanityCheck failures: the first in the order i = 0..2k-1 x
 *     {row root, col root, row parity, col parity} (upstream runs these checks
 *     concurrently and returns whichever fails first in time); rebuilt = axis.
 *   - solveCrossword failures: the first failing attempt in rsmt2d's
 *     sequential order (each pass: row i, then column i).  Either the rebuilt
 *     axis' own root differs (axis = rebuilt axis) or an orthogonal axis it
 *     completed does (axis = that orthogonal axis; rebuilt = the row/column
 *     whose rebuild completed it, whose shares rsmt2d v0.11.0 attaches).
 * On DAGPU_ERR_BYZANTINE, present[] is left as rsmt2d leaves the square: the
 * cells filled by the attempts before the failing one (their bytes in eds are
 * the committed ones); ErrByzantineData.Shares = the cells of the rebuilt axis
 * with present[] set.  A prerepairSanityCheck failure (DAGPU_ERR_BAD_ROOTS, or
 * DAGPU_ERR_BYZANTINE from the check) returns before rsmt2d's crossword:
 * present[] is the input's.  The bytes of cells whose present[] flag is 0 are
 * unspecified (rsmt2d holds nil there).  Replaces ExtendedDataSquare.Repair
 * (rsmt2d v0.11.0). */
int dagpu_repair_ex(dagpu_ctx* ctx, uint32_t k, uint8_t* eds, uint8_t* present,
                    const uint8_t* row_roots, const uint8_t* col_roots, int32_t* byz);

/* Device-resident batched Repair: n squares of width k (device pointers),
 * d_present = n * (2k)^2 flags (updated in place), expected roots as produced by
 * dagpu_extend_batch_device.  d_status gets one dagpu_status per square.
 * d_workspace: dagpu_repair_workspace_size(k, n) bytes.  Enqueued on `stream`;
 * the call reads the round counters on the host once per crossword round (and
 * once more when deferred axes need their codeword check), so it returns when
 * its last command is queued.  Axes whose data
 * half is complete are re-encoded instead of decoded, and axes whose parity
 * half is complete are rebuilt by the inverse transform (same bytes);
 * DAGPU_REPAIR_FILL=0 in the environment selects the plain decoder schedule.
 * The _ex form also writes d_byz (n * 4 int32, device memory, as byz of
 * dagpu_repair_ex); a square whose crossword fails is then re-run in rsmt2d's
 * sequential order on the device to name its axis (synchronises `stream`).
 * Without d_byz the crossword's failing axis is not resolved and the cells of
 * a square with a failure are left as the batched crossword filled them. */
size_t dagpu_repair_workspace_size(uint32_t k, size_t n);
int dagpu_repair_batch_device(dagpu_ctx* ctx, uint32_t k, size_t n, uint8_t* d_eds,
                              uint8_t* d_present, const uint8_t* d_row_roots,
                              const uint8_t* d_col_roots, int32_t* d_status,
                              void* d_workspace, void* stream);
int dagpu_repair_batch_device_ex(dagpu_ctx* ctx, uint32_t k, size_t n, uint8_t* d_eds,
                                 uint8_t* d_present, const uint8_t* d_row_roots,
                                 const uint8_t* d_col_roots, int32_t* d_status, int32_t* d_byz,
                                 void* d_workspace, void* stream);

/* dagpu_repair_batch_device split in two: dagpu_repair_start returns at once
 * (*handle names the repair); a library worker thread makes the crossword's
 * host decisions and queues its kernels on a stream of its own, forked from
 * `stream` at the call (work already queued there runs first).
 * dagpu_repair_join(ctx, handle, stream2) waits until the worker has queued
 * its last command and makes stream2 wait for the repair; it returns the
 * repair's call status (per-square results in d_status).  Repairs started back
 * to back (slices of a batch, squares of several blocks) run side by side; a
 * context serves 64 started, not yet joined repairs.  Buffer lifetime: d_eds,
 * d_present, d_status and d_workspace (and the roots) must stay valid until
 * stream2 -- the stream passed to dagpu_repair_join -- has passed the repair.
 * Free or reuse them only in stream2's order (work queued on stream2 after the
 * join, or after hipStreamSynchronize(stream2)); an allocator that frees in
 * another stream's order must first make that stream wait for stream2 (the
 * Python wrapper calls record_stream(stream2) on each buffer).  Joins from several
 * host threads wait side by side (the slot table is locked only to claim a
 * slot); a failed repair's message is re-raised on the joining thread
 * (dagpu_last_error), and a worker that cannot be started returns
 * DAGPU_ERR_DEVICE with no slot taken. */
int dagpu_repair_start(dagpu_ctx* ctx, uint32_t k, size_t n, uint8_t* d_eds, uint8_t* d_present,
                       const uint8_t* d_row_roots, const uint8_t* d_col_roots, int32_t* d_status,
                       void* d_workspace, void* stream, uint64_t* handle);
int dagpu_repair_join(dagpu_ctx* ctx, uint64_t handle, void* stream);

/* Per-kernel timing with HIP events recorded on the launch stream around each
 * kernel the pipeline enqueues (for bench.py's roofline; off by default).
 * Kernel ids: 0 RS row pass, 1 RS column pass, 2 NMT leaves, 3 NMT trees,
 * 4 DAH, 5 decode, 6 Repair fill encode.  dagpu_profile_read synchronises the recorded events and
 * returns, per kernel id, the summed milliseconds and launch count since the
 * last reset (arrays of DAGPU_PROFILE_KERNELS entries). */
#define DAGPU_PROFILE_KERNELS 7
int dagpu_profile_enable(dagpu_ctx* ctx, int on);
int dagpu_profile_read(dagpu_ctx* ctx, double* total_ms, uint64_t* launches, int reset);

/* Stage timeline of the last host-path extend call (dagpu_extend_shares /
 * one-chunk dagpu_extend_batch) when dagpu_profile_enable(ctx, 2) is on:
 * ms[i] = milliseconds from the call's first enqueue to stage i (HIP events on
 * the compute stream, and on the copy stream for the EDS halves), -1 when the
 * stage did not run.  For diagnosing single-call latency. */
#define DAGPU_STAGES 10
#define DAGPU_STAGE_START 0      /* before the ODS upload */
#define DAGPU_STAGE_UPLOADED 1
#define DAGPU_STAGE_ROWS 2       /* RS row pass done */
#define DAGPU_STAGE_COLS 3       /* RS column pass done */
#define DAGPU_STAGE_LEAVES 4
#define DAGPU_STAGE_TREES 5
#define DAGPU_STAGE_DAH 6
#define DAGPU_STAGE_RESULTS 7    /* roots + DAH + status downloaded */
#define DAGPU_STAGE_EDS_TOP 8    /* [Q0|Q1] halves downloaded (copy stream) */
#define DAGPU_STAGE_EDS_BOTTOM 9 /* [Q2|Q3] halves downloaded (copy stream) */
int dagpu_profile_stages(dagpu_ctx* ctx, float* ms);

/* Schedule of the last Repair on this context (diagnostics; a started repair's
 * schedule becomes "the last" at its join, so started repairs in flight never
 * mix their counters): out[0] crossword
 * rounds that rebuilt something, out[1] vectors re-encoded from a complete data
 * half (fill), out[2] vectors rebuilt from a complete parity half (reverse
 * fill), out[3] vectors planned for the decoder, out[4] decodes deferred to the
 * other axis.  All zero with DAGPU_REPAIR_FILL=0 except out[0]. */
#define DAGPU_REPAIR_STATS 5
int dagpu_repair_stats(dagpu_ctx* ctx, int64_t* out);

/* RFC-6962 root of rowRoots || colRoots (DataAvailabilityHeader.Hash,
 * pkg/da/data_availability_header.go:92-108), computed on the host side of the
 * boundary for small inputs (w = number of row roots; w == 0 gives the
 * empty-tree hash SHA256("")). */
int dagpu_dah_hash(const uint8_t* row_roots, const uint8_t* col_roots, size_t w,
                   uint8_t* out32);

/* ---- Generic trees (batched; host buffers in, host buffers out) ---------- */

/* Leaf prefix modes of dagpu_nmt_roots (what is hashed for a push of `d`):
 *   NONE   0x00 | d            d is nmt namespaced data (ns = d[0:29])
 *   SELF   0x00 | d[0:29] | d  (wrapper Q0 cell; blob commitment leaf)
 *   PARITY 0x00 | 0xFF*29 | d  (wrapper cell outside Q0)
 *   FLAGS  per-push SELF / PARITY byte in prefix_flags */
#define DAGPU_PREFIX_NONE 0
#define DAGPU_PREFIX_SELF 1
#define DAGPU_PREFIX_PARITY 2
#define DAGPU_PREFIX_FLAGS 3

/* Roots of many namespaced Merkle trees: nmt.New(sha256.New(),
 * NamespaceIDSize(29), IgnoreMaxNamespace(ignore_max_ns)) followed by Push of
 * every leaf and Root() (nmt v0.20.0; hasher mirror
 * test/util/malicious/hasher.go:161-309).  Tree t has leaf_counts[t] pushes,
 * packed tree after tree in `leaves`, leaf_len bytes each.  roots: ntrees * 90
 * B (an empty tree gives 0^29 | 0^29 | SHA256("")).  status[t] (optional):
 * DAGPU_ERR_PUSH_ORDER when a pushed namespace is below its predecessor's
 * (ErrInvalidPushOrder); the call then returns that status. */
int dagpu_nmt_roots(dagpu_ctx* ctx, size_t ntrees, const uint32_t* leaf_counts,
                    const uint8_t* leaves, size_t leaf_len, int prefix_mode,
                    const uint8_t* prefix_flags, int ignore_max_ns, uint8_t* roots,
                    int32_t* status);

/* rsmt2d.Tree drop-in for wrapper.NewConstructor(squareSize)
 * (pkg/wrapper/nmt_wrapper.go:73-124): tree t is the
 * ErasuredNamespacedMerkleTree of axis index axis_index[t] after
 * leaf_counts[t] Push calls of share_len-byte shares (packed in `shares`);
 * returns every Root().  Same errors: square_size 0, pushes past 2*squareSize,
 * shares shorter than 29 B, namespace push order. */
int dagpu_wrapper_roots(dagpu_ctx* ctx, uint64_t square_size, size_t ntrees,
                        const uint32_t* axis_index, const uint32_t* leaf_counts,
                        const uint8_t* shares, size_t share_len, uint8_t* roots,
                        int32_t* status);

/* merkle.HashFromByteSlices (celestia-core v0.34 crypto/merkle, RFC-6962) for
 * many lists: list t has counts[t] items of item_len bytes (packed); out32 gets
 * ntrees 32-B roots (an empty list gives SHA256("")). */
int dagpu_merkle_roots(dagpu_ctx* ctx, size_t ntrees, const uint32_t* counts,
                       const uint8_t* items, size_t item_len, uint8_t* out32);

/* Every node of ONE RFC-6962 tree (merkle.ProofsFromByteSlices, celestia-core
 * crypto/merkle; pkg/proof/proof.go:87): the n leaf hashes, then each level
 * (ceil-halving, an odd last node promoted unchanged) up to the root, 32 B each.
 * *n_nodes: in = capacity of out32 in nodes, out = nodes written (or needed). */
int dagpu_merkle_levels(dagpu_ctx* ctx, size_t n, const uint8_t* items, size_t item_len,
                        uint8_t* out32, size_t* n_nodes);

/* Proof verification on the host (light-client side of pkg/proof):
 * nmt Proof.VerifyInclusion (nmt v0.20.0, IgnoreMaxNamespace, used by
 * celestia-core ShareProof.VerifyProof): n leaves of leaf_len bytes each, given
 * WITHOUT the namespace the tree prepends, proven at [start, end) by nnodes
 * 90-B nodes against a 90-B root.  crypto/merkle Proof.Verify: leaf bytes,
 * index/total and naunts 32-B aunts (leaf to root) against a 32-B root.
 * DAGPU_OK = valid, DAGPU_ERR_PROOF = does not verify, DAGPU_ERR_ARG = malformed. */
int dagpu_nmt_verify_inclusion(const uint8_t* ns29, const uint8_t* leaves, size_t n, size_t leaf_len,
                               int64_t start, int64_t end, const uint8_t* nodes, size_t nnodes,
                               const uint8_t* root90);
int dagpu_merkle_verify(const uint8_t* root32, const uint8_t* leaf, size_t leaf_len, int64_t index,
                        int64_t total, const uint8_t* aunts, size_t naunts);

/* inclusion.SubTreeWidth (pkg/inclusion/blob_share_commitment_rules.go:85-101). */
int dagpu_subtree_width(uint64_t share_count, uint32_t subtree_root_threshold);

/* inclusion.CreateCommitment (pkg/inclusion/commitment.go:19-75) for blobs
 * already split into shares (shares.SplitBlobs): blob b has namespace
 * namespaces[b*29..] and share_counts[b] 512-B shares (packed in `shares`).
 * Subtree widths from subtree_root_threshold (appconsts
 * DefaultSubtreeRootThreshold = 64); commitments: nblobs * 32 B. */
int dagpu_blob_commitments(dagpu_ctx* ctx, size_t nblobs, const uint8_t* namespaces,
                           const uint32_t* share_counts, const uint8_t* shares,
                           uint32_t subtree_root_threshold, uint8_t* commitments);

/* ---- One oversized square split over P GPUs (configs[4] stress) ---------
 * Same result as dagpu_extend_batch_device on the whole square; rank g of P
 * (P a power of two <= k) owns Q0 rows [g*k/P, (g+1)*k/P) and EDS columns
 * [g*2k/P, (g+1)*2k/P).  The caller runs the collectives (RCCL over xGMI)
 * between the steps; all pointers are device memory on `stream`:
 *   1 dagpu_split_rows_device   d_ods_rows (k/P rows of k shares) -> d_send:
 *                               P blocks of (k/P) x (2k/P) shares, block h for
 *                               rank h; zeroes then sets *d_status (push order)
 *   2 all-to-all of d_send      rank h receives the P blocks in rank order =
 *                               rows 0..k-1 of its slab (2k rows x 2k/P shares)
 *   3 dagpu_split_cols_device   fills slab rows k..2k-1, writes the slab's
 *                               2k/P column roots (90 B) and 2k row-subtree
 *                               records (96 B: minNs[32] maxNs[32] digest[32])
 *   4 all-gather row-subtree records (P x 2k x 96 B, rank order) and column
 *     roots (2k x 90 B, column order); max-reduce the status words
 *   5 dagpu_split_finish_device row roots (2k x 90 B) and the DAH (32 B)
 * Every step only enqueues on `stream` (nothing is read from host memory):
 * synchronise it before reading the results.  With P = 1 the one
 * send block is rows 0..k-1 of the slab: pass the slab itself as d_send and
 * skip step 2 (the encoder then writes [Q0 | Q1] in place).
 * d_workspace: dagpu_split_workspace_size(k, P) bytes (0 = invalid k / P).
 * Widths: every k up to DAGPU_MAX_SQUARE_WIDTH, and k = DAGPU_MAX_SPLIT_WIDTH
 * (16384: a 512 GiB EDS, beyond one GPU) over P >= 8 parts -- per rank a 64 GiB
 * column slab plus ~70 GiB of staging and forest records at P = 8;
 * DAGPU_ERR_UNSUPPORTED (workspace size 0) for fewer parts or wider squares. */
#define DAGPU_MAX_SPLIT_WIDTH 16384
size_t dagpu_split_workspace_size(uint32_t k, uint32_t parts);
int dagpu_split_rows_device(dagpu_ctx* ctx, uint32_t k, uint32_t parts, uint32_t part,
                            const uint8_t* d_ods_rows, uint8_t* d_send, int32_t* d_status,
                            void* d_workspace, void* stream);
int dagpu_split_cols_device(dagpu_ctx* ctx, uint32_t k, uint32_t parts, uint32_t part,
                            uint8_t* d_slab, uint8_t* d_col_roots, uint8_t* d_row_sub,
                            int32_t* d_status, void* d_workspace, void* stream);
int dagpu_split_finish_device(dagpu_ctx* ctx, uint32_t k, uint32_t parts,
                              const uint8_t* d_row_sub_all, const uint8_t* d_col_roots_all,
                              uint8_t* d_row_roots, uint8_t* d_dah, void* d_workspace,
                              void* stream);

/* ---- Row-tree inner nodes (nmt.NodeVisitor / inclusion.EDSSubTreeRootCacher,
 * pkg/inclusion/nmt_caching.go:81-128; share commitments from the EDS,
 * get_commit.go:12-30) ------------------------------------------------------
 * dagpu_row_nodes_device hashes every node of every row NMT of one EDS (device
 * memory) into d_nodes (dagpu_row_nodes_size(k) bytes): 96-B records minNs[32]
 * maxNs[32] digest[32]; level L (0 = leaves, log2(2k) = root) is packed after
 * level L-1, row-major, so node (row, L, p) is record
 * sum_{l<L} 2k*(2k>>l) + row*(2k>>L) + p.  Synchronises `stream`.
 * dagpu_row_nodes_gather_device reads n (row, depth, position) uint32 triples
 * (depth 0 = root) and writes n packed 90-B nodes. */
size_t dagpu_row_nodes_size(uint32_t k);
size_t dagpu_row_nodes_workspace_size(uint32_t k);
int dagpu_row_nodes_device(dagpu_ctx* ctx, uint32_t k, const uint8_t* d_eds, uint8_t* d_nodes,
                           void* d_workspace, void* stream);
int dagpu_row_nodes_gather_device(dagpu_ctx* ctx, uint32_t k, const uint8_t* d_nodes, size_t n,
                                  const uint32_t* d_requests, uint8_t* d_out, void* stream);

/* ---- Square construction (host; pkg/square, app version 1) ---------------
 * square.Construct (pkg/square/square.go:22-63, builder.go): ntx txs packed
 * back to back in `txs` (tx_lens[i] bytes each; blob txs in the BlobTx proto
 * wire format, pkg/blob/blob.go:56-90) -> the original data square, k*k
 * 512-B shares row-major, in ods_out (ods_cap bytes; k*k*512 needed, k <=
 * max_square_size; *square_size = k is set even when ods_out is too small,
 * which returns DAGPU_ERR_ARG).  Every tx must fit and normal txs must come
 * before blob txs, else DAGPU_ERR_SQUARE with the reference's message
 * ("not enough space to append tx at index 3", ...).  max_square_size =
 * SquareSizeUpperBound (128) and subtree_root_threshold = 64 for app v1.
 * The ODS goes straight into dagpu_extend_shares / the device batch API.
 * ctx may be NULL (then no message is kept).  No device work. */
int dagpu_square_construct(dagpu_ctx* ctx, const uint8_t* txs, const uint64_t* tx_lens, size_t ntx,
                           uint32_t max_square_size, uint32_t subtree_root_threshold, uint8_t* ods_out,
                           size_t ods_cap, uint32_t* square_size);
/* square.Build: txs that do not fit are skipped (kept[i] = 0), normal txs may
 * follow blob txs; the reference returns the kept normal txs, then the kept
 * blob txs, in input order within each group. */
int dagpu_square_build(dagpu_ctx* ctx, const uint8_t* txs, const uint64_t* tx_lens, size_t ntx,
                       uint32_t max_square_size, uint32_t subtree_root_threshold, uint8_t* ods_out,
                       size_t ods_cap, uint32_t* square_size, uint8_t* kept);

#ifdef __cplusplus
}
#endif
#endif
