// kernels.hpp -- device kernel launchers shared by the C-ABI layer (dagpu.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "switches.hpp"

namespace dagpu {

constexpr int kShareSize = 512;
constexpr int kNsSize = 29;
constexpr int kNodeSize = 90;  // minNs(29) | maxNs(29) | sha256(32)
constexpr int kDigest = 32;
// Widest square: (2k)^2 x 512 B of EDS = 128 GiB at k = 8192 fits the 288 GB of
// HBM, k = 16384 (512 GiB) does not.  GF(2^16) above k = 128; register-resident
// kernels at k = 256 / 512, LDS-slice kernels (rs_gf16_wide.hip) above.
constexpr int kMaxK = 8192;
// Widest codec vector (rsmt2d.Codec Encode / Decode, dagpu_encode / dagpu_decode):
// Leopard GF(2^16)'s whole field, k data + k parity = 65536 shards (klauspost
// leopardFF16 rejects more; rsmt2d LeoRSCodec.MaxChunks = 32768 * 32768).  A
// vector is k x shard bytes, so these widths fit one GPU even where the square
// of the same width does not; the wide kernels serve k = 16384 / 32768 with
// 2- / 1-symbol LDS slices (rs_gf16_wide.hip).
constexpr int kMaxCodecK = 32768;
// Widest split square (split.cpp, one oversized square over P GPUs): k = 16384,
// whose 512 GiB EDS one GPU cannot hold, over P >= kMinWideSplitParts ranks
// (P = 8: per rank a 64 GiB column slab, 32 GiB of row staging and send
// block, ~38 GiB of forest records -- under 288 GB; P = 4 would not fit).
constexpr int kMaxSplitK = 2 * kMaxK;
constexpr int kMinWideSplitParts = 8;

// Bytes of error-locator workspace per decoded vector.
// Error-locator workspace per vector: GF(2^8) 256 B; GF(2^16) the n = 2k uint16
// locators (4k B) and after them, at rs_err_tab_off(k), what the decoders'
// per-element multiplies need, built once per erasure pattern by the locator
// kernel (round 6) instead of in every decoder workgroup: at k = 256 / 512 the
// n x 80-B image of the product tables (exp(errLoc) for a present element,
// exp(-errLoc) for a missing one) that a half-lane decoder copies into LDS;
// at k >= 1024 the n x 32-B basis products (1 << b) * that factor, b < 16, from
// which a wide decoder workgroup builds an element's table without gathers.
constexpr long rs_err_tab_off(int k) { return 4L * k; }
constexpr long rs_err_elem_bytes(int k) { return k <= 1024 ? 80 : 32; }
constexpr long rs_err_bytes(int k) { return k <= 128 ? 256 : 4L * k + 2L * k * rs_err_elem_bytes(k); }

// Per-square status bits written by the kernels (0 = OK).
constexpr int kStatusPushOrder = 1;

// Generic strided "vector" addressing for the encoder.  For square s, vector v
// and shard i, the input dword column at byte offset `col` lives at
//   in + s*in_sq_stride + v*in_vec_stride + i*in_shard_stride + col.
struct EncodeArgs {
  const uint8_t* in;
  uint8_t* out;
  uint8_t* copy;  // optional: also store the data shards here (Q0 placement)
  long in_sq_stride, in_vec_stride, in_shard_stride;
  long out_sq_stride, out_vec_stride, out_shard_stride;
  long copy_sq_stride, copy_vec_stride, copy_shard_stride;
  long nsq, nvec, nchunk;  // nchunk = ceil(shard_bytes / 512)
  long shard_bytes;
  // Compare mode (rsmt2d prerepairSanityCheck): when `mismatch` is set the
  // kernel compares the computed parity with the bytes already at `out` and
  // ORs `mismatch_bit` into mismatch[square] on any difference; vectors whose
  // vec_flags entry is 0 are skipped.
  const int32_t* vec_flags;
  int32_t* mismatch;
  int mismatch_bit;
  int32_t* mismatch_vec;  // optional: mismatch_vec[square * nvec + vec] = 1 on a difference
  // Fill mode (Repair, dagpu.cpp repair_device): a vector whose data half is
  // complete is rebuilt by encoding that half.  A parity shard is stored only
  // where out_present[sq * op_sq_stride + vec * op_vec_stride + j * op_shard_stride]
  // is 0; a given (present) one that differs from the encoding sets
  // redo[sq * nvec + vec] = 1, and that vector goes to the decoder instead.
  // vec_flags selects the vectors; the k = 128 bit-sliced encoder instead takes
  // pair_list (pairs of same-square vectors, flattened sq * nvec + vec, -1 =
  // none) with *pair_count pairs.
  const uint8_t* out_present;
  long op_sq_stride, op_vec_stride, op_shard_stride;
  int32_t* redo;
  const int32_t* pair_list;
  const int32_t* pair_count;
  // Reverse transform (Repair reverse fill): `in` holds the parity half of each
  // vector and `out` receives its data half.  Leopard's encode is
  // parity = FFT(skew offset 0) of IFFT(skew offset k) of the data, both over
  // the same polynomial of degree < k (k = m, a power of two), so
  // data = FFT(offset k) of IFFT(offset 0) of the parity.  Fill mode only.
  int reverse;
  // With vec_flags: 0 = every nonzero entry selects its vector; otherwise only
  // entries equal to vec_flag_match do (Repair fill: 1 forward, 2 reverse).
  int vec_flag_match;
};

__device__ __forceinline__ bool fill_given(const EncodeArgs& a, long sq, long vec, long j) {
  return a.out_present[sq * a.op_sq_stride + vec * a.op_vec_stride + j * a.op_shard_stride] != 0;
}

// vector v (flattened sq * nvec + vec) not selected by vec_flags (wave-uniform)
__device__ __forceinline__ bool vec_skipped(const EncodeArgs& a, long v) {
  if (!a.vec_flags) return false;
  const int32_t f = a.vec_flags[v];
  return a.vec_flag_match ? f != a.vec_flag_match : f == 0;
}

hipError_t launch_leo8_encode(int k, const EncodeArgs& a, hipStream_t s);
// bit-sliced GF(2^8) encode (rs_gf8_sliced.hip); launch_leo8_encode uses it
// whenever leo8_sliced_applicable() holds
bool leo8_sliced_applicable(int k, const EncodeArgs& a);
hipError_t launch_leo8_encode_sliced(int k, const EncodeArgs& a, hipStream_t s);
// k = 128 Repair fill over EncodeArgs.pair_list (up to max_pairs pairs)
bool leo8_fill_sliced_applicable(const EncodeArgs& a);
hipError_t launch_leo8_fill_sliced(const EncodeArgs& a, long max_pairs, hipStream_t s);

// Decode addressing: shard i of vector (s, v) at
//   data + s*sq_stride + v*vec_stride + i*shard_stride   (2k shards)
// and its presence flag at present + s*p_sq_stride + v*p_vec_stride + i*p_shard_stride.
struct DecodeArgs {
  uint8_t* data;
  long sq_stride, vec_stride, shard_stride;
  uint8_t* present;
  long p_sq_stride, p_vec_stride, p_shard_stride;
  uint8_t* err;        // workspace: nsq*nvec*rs_err_bytes(k) error locators
  int32_t* flags;      // workspace: nsq*nvec (1 = vector decoded this pass)
  int32_t* too_few;    // optional: set to 1 if any vector has < k shards
  int32_t* progress;   // optional: += number of vectors rebuilt (mark pass)
  int32_t* ndecodable; // optional: += number of decodable vectors (errlocs pass)
  int32_t* nfill;      // optional (vec_count): += decodable vectors with a complete data or parity half
  // Optional error-locator sharing: the locators depend only on the erasure
  // pattern, and many vectors of a repair pass share it (every row of a square
  // kept by the same column set).  err_key[v] = 32-bit hash of v's pattern;
  // err_head[v] = the first vector of v's square with the same pattern
  // (checked flag by flag), whose locators v uses.  Both nsq * nvec int32 of
  // workspace; NULL = one computation per vector.
  int32_t* err_key;
  int32_t* err_head;
  // Test builds only (DAGPU_TEST_HOOKS; the product library never sets it):
  // every key equal, so the candidate-head checks decide every vector's head.
  int key_collide;
  // Locators only (Repair, after the fill/deferral plan): compute the error
  // locators of the vectors whose flags[] are already set, leaving flags and
  // counts alone; a flagged vector whose head is not flagged computes the
  // head's locators itself (same pattern, same values).
  int locators_only;
  // Optional (launch_vec_count): vec_counts[v] = present data shards | present
  // shards << 16 (Repair plan).
  int32_t* vec_counts;
  // Optional vector selection (exact-order Repair, dagpu.cpp): only vectors v
  // with sel_level[v] == sel_value are decodable in this pass.  Requires
  // err_key/err_head = NULL (an unselected head computes no locators).
  const int32_t* sel_level;
  int sel_value;
  long nsq, nvec, nchunk, shard_bytes;
  int k;
};

__device__ __forceinline__ bool vec_selected(const DecodeArgs& a, long v) {
  return !a.sel_level || a.sel_level[v] == a.sel_value;
}

// vector whose error locators vector v uses
__device__ __forceinline__ long err_vec(const DecodeArgs& a, long v) { return a.err_head ? a.err_head[v] : v; }
// Round 6: the flag-by-flag check of a candidate head (errloc_heads_kernel:
// the first vector of the square with an equal key) runs inside the locator
// kernels.  Returns v's head: the candidate when the two vectors' presence
// flags agree one by one, else v itself (a key collision; err_head[v] is
// rewritten, and no other vector has v as its candidate).  Block-wide: every
// thread of the block calls it for the same v.
__device__ __forceinline__ bool err_flags_differ(const DecodeArgs& a, long v, long hv, int first, int step) {
  const long sq = v / a.nvec;
  const uint8_t* pv = a.present + sq * a.p_sq_stride + (v - sq * a.nvec) * a.p_vec_stride;
  const uint8_t* pu = a.present + sq * a.p_sq_stride + (hv - sq * a.nvec) * a.p_vec_stride;
  bool diff = false;
  for (int i = first; i < 2 * a.k; i += step)
    diff |= (pv[(long)i * a.p_shard_stride] != 0) != (pu[(long)i * a.p_shard_stride] != 0);
  return diff;
}
__device__ __forceinline__ long err_head_checked_block(const DecodeArgs& a, long v) {
  if (!a.err_head) return v;
  const long hv = a.err_head[v];
  if (hv == v) return v;  // uniform
  const bool diff = err_flags_differ(a, v, hv, threadIdx.x, blockDim.x);
  if (!__syncthreads_or(diff)) return hv;
  if (threadIdx.x == 0) a.err_head[v] = (int32_t)v;
  return v;
}
// the same for one wave per vector
__device__ __forceinline__ long err_head_checked_wave(const DecodeArgs& a, long v, int lane) {
  if (!a.err_head) return v;
  const long hv = a.err_head[v];
  if (hv == v) return v;  // uniform per wave
  if (!__any(err_flags_differ(a, v, hv, lane, 64))) return hv;
  if (lane == 0) a.err_head[v] = (int32_t)v;
  return v;
}
// does vector v (decodable) compute the locators of its head hv?
__device__ __forceinline__ bool err_computes(const DecodeArgs& a, long v, long hv) {
  return hv == v || (a.locators_only && a.flags[hv] == 0);
}

hipError_t launch_leo8_decode(const DecodeArgs& a, hipStream_t s, bool mark_present);
hipError_t launch_leo8_errlocs(const DecodeArgs& a, hipStream_t s);
hipError_t launch_leo8_decode_only(const DecodeArgs& a, hipStream_t s, bool mark_present);
// bit-sliced k = 128 decode (rs_decode_sliced.hip); launch_leo8_decode_only
// uses it whenever leo8_decode_sliced_applicable() holds
bool leo8_decode_sliced_applicable(const DecodeArgs& a);
hipError_t launch_leo8_decode128_sliced(const DecodeArgs& a, hipStream_t s);

// GF(2^16) (rs_gf16.hip) and the field dispatch the host runtime uses:
// GF(2^8) for k <= 128, GF(2^16) for 256 <= k <= kMaxK.  DecodeArgs.err then
// holds rs_err_bytes(k) bytes per vector.
hipError_t launch_leo16_encode(int k, const EncodeArgs& a, hipStream_t s);
hipError_t launch_leo16_errlocs(const DecodeArgs& a, hipStream_t s);
hipError_t launch_leo16_decode_only(const DecodeArgs& a, hipStream_t s, bool mark_present);
// wide GF(2^16) (rs_gf16_wide.hip): k = 1024 .. kMaxK (also 256 / 512 for A/B)
hipError_t launch_leo16w_encode(int k, const EncodeArgs& a, hipStream_t s);
hipError_t launch_leo16w_errlocs(const DecodeArgs& a, hipStream_t s);
hipError_t launch_leo16w_decode_only(const DecodeArgs& a, hipStream_t s, bool mark_present);
// one-time per-device setup (tables, LDS attributes) of the codec of width k,
// so that later launches allocate and upload nothing
hipError_t launch_rs_prepare(int k);
hipError_t leo16w_prepare();
hipError_t launch_rs_encode(int k, const EncodeArgs& a, hipStream_t s);
hipError_t launch_rs_errlocs(const DecodeArgs& a, hipStream_t s);
// the two halves of launch_rs_errlocs: candidate heads (of a, and of a1 when
// given, in the same launches) and the locators (whose kernels check the
// candidates flag by flag)
hipError_t launch_errloc_heads2(const DecodeArgs& a, const DecodeArgs* a1, hipStream_t s);
hipError_t launch_rs_errlocs_only(const DecodeArgs& a, hipStream_t s);
hipError_t launch_rs_decode_only(const DecodeArgs& a, hipStream_t s, bool mark_present);
hipError_t launch_rs_decode(const DecodeArgs& a, hipStream_t s, bool mark_present);

// Repair helpers (repair.hip).  Status bits per square:
constexpr int kRepByz = 4;         // rebuilt axis, root mismatch
constexpr int kRepIncomplete = 8;  // crossword could not finish
// Axis arrays (complete, root_bad, parity_bad) are [axis][square][idx].
// complete[axis*nsq*w + sq*w + idx] = axis fully present
// (optional) *ncomplete += number of complete axes
hipError_t launch_axis_complete(const uint8_t* present, int k, long nsq, int32_t* complete, hipStream_t s,
                                int32_t* ncomplete = nullptr);
// root_bad[a] = 1 for an axis complete before the repair whose root differs
// (pre-repair "bad root input"); a rebuilt axis whose root differs ORs kRepByz
// into bits[sq]; an incomplete axis ORs kRepIncomplete
hipError_t launch_verify_roots(const uint8_t* exp_rr, const uint8_t* exp_cr, const uint8_t* got_rr,
                               const uint8_t* got_cr, const int32_t* complete_now,
                               const int32_t* complete_before, int k, long nsq, int32_t* bits,
                               int32_t* root_bad, hipStream_t s);
// status[sq] and (optional) byz[sq*4 .. +3] = {axis, index, rebuilt axis,
// rebuilt index} (-1 = none / not known): the first pre-repair failure in the
// order i = 0..2k-1 x {row root, col root, row parity, col parity}, else a
// crossword failure (kRepByz, axis resolved by the host), else unrepairable
// Repair shortcut plan for one round on one axis (see repair_device): every
// decodable vector of the axis whose data half is complete moves from the
// decoder (flags) to the fill encoder (fill[v] = 1, forward), and one whose
// parity half is complete to the reverse fill (fill[v] = 2); pair_list /
// pair_list_rev (when set) pair each square's forward / reverse fills; when every
// vector i < k of a square is decodable or complete (and nodefer[sq] is 0), the
// decodes of its vectors i >= k are deferred: the other axis then has complete
// data halves everywhere and is filled in the next round.  known[axis][sq][i]
// records axes that are codewords by construction (rebuilt from exactly k
// shares, or filled); deferred[axis][sq][i] the deferred ones; *ndeferred counts them.
struct PlanArgs {
  const int32_t* counts;  // vec_counts of the axis (launch_vec_count)
  int32_t* flags;
  int32_t* fill;
  int32_t* pair_list;
  int32_t* pair_count;
  int32_t* pair_list_rev;
  int32_t* pair_count_rev;
  int32_t* known;
  int32_t* deferred;
  const int32_t* nodefer;
  int32_t* ndeferred;
  int32_t* nplan;  // optional: += [forward fills, reverse fills, decodes] of the round (diagnostics)
  int k;
  long nsq;
  int axis;
};
hipError_t launch_repair_plan(const PlanArgs& p, hipStream_t s);
// After the crossword: squares with deferred axes whose codeword property does
// not follow from the known ones (all rows and the columns < k, or all columns
// and the rows < k) keep their deferred[] marks for a compare-mode encode;
// the others' marks are cleared.  check[sq] = 0; (optional) *nleft += squares
// whose marks stay.
hipError_t launch_repair_defer_check(int32_t* deferred, const int32_t* known, int k, long nsq, int32_t* check,
                                     hipStream_t s, int32_t* nleft = nullptr);
// Decodable vectors and counts without locators (Repair rounds): one lane per
// vector; flags[v], vec_counts[v] (when set) and *ndecodable as the locator pass
// would leave them.
hipError_t launch_vec_count(const DecodeArgs& a, hipStream_t s);
// Repair round counters (int32 slots of the 64-slot counters array):
// decodable rows / columns of the round and, of those, the fill candidates
// (a complete data or parity half) per axis (vec_count; the round's last
// launch clears these four), deferrals of the round's plan, its fill pair
// counts, complete axes before the repair, squares left for the deferral
// check, the previous round's deferrals (moved there by the next round's count
// launch, so the host reads it with the round's counts), the plan's totals (3
// slots), the count launch's last-block ticket.  The host reads [0, kCtrRead).
constexpr int kCtrRowsDec = 0, kCtrColsDec = 1, kCtrFillRows = 2, kCtrFillCols = 3, kCtrDeferred = 4,
              kCtrPairs = 5, kCtrPairsRev = 6, kCtrComplete = 7, kCtrDeferSquares = 8, kCtrDeferredPrev = 9,
              kCtrPlan = 10, kCtrRead = 13, kCtrTicket = 14, kCtrSlots = 64;
struct RoundCounters {
  int32_t* ctr;   // device counters (kCtrSlots)
  int32_t* host;  // optional: page-locked host copy of slots [0, kCtrRead), written by the last block,
                  // then host[kCtrRead] = seq (the host spins on it, not on the stream)
  int32_t seq;
};
// Both axes' vec_count of a Repair round in one launch plus the counter
// bookkeeping above.  Slots kCtrRowsDec .. kCtrFillCols must be 0 on entry
// (the previous round's launch_rs_mark_round clears them).
hipError_t launch_vec_count_round(const DecodeArgs& a0, const DecodeArgs& a1, const RoundCounters& rc,
                                  hipStream_t s);
// presence += vectors with flags[v] != 0 (axis given by the args); with
// `known` ([sq][idx] of that axis), known[v] = 0 where a.flags[v] is set too
hipError_t launch_rs_mark_present(const DecodeArgs& a, const int32_t* flags, hipStream_t s,
                                  int32_t* known = nullptr);
// The end of a Repair round in one launch: presence += vectors flagged in
// a.flags (decoded) or fill (optional, filled); known[v] = 0 where both are
// set; zero4[0..3] (optional) := 0 for the next round's counts.
hipError_t launch_rs_mark_round(const DecodeArgs& a, const int32_t* fill, int32_t* known, int32_t* zero4,
                                hipStream_t s);
// (optional) pre_fail[sq] = 1 where the pre-repair check failed
hipError_t launch_finalize_repair(const int32_t* bits, const int32_t* complete_before, const int32_t* root_bad,
                                  const int32_t* parity_bad, int k, long nsq, int32_t* status, int32_t* byz,
                                  hipStream_t s, int32_t* pre_fail = nullptr);
// present of the squares with pre_fail[sq] set := p0 (their input presence)
hipError_t launch_restore_presence(uint8_t* present, const uint8_t* p0, const int32_t* pre_fail, int k, long nsq,
                                   hipStream_t s);

struct SquareArgs {
  const uint8_t* eds;   // nsq squares, each (2k)^2 * 512 B, row-major
  long eds_sq_stride;
  uint8_t* digests;     // leaf digests: nsq * (2k)^2 * 32 B
  uint8_t* ns_table;    // Q0 namespaces: nsq * k^2 * 32 B
  uint8_t* rec_a;       // tree node records (48 B): nsq * 2w * w/2
  uint8_t* rec_b;       // nsq * 2w * w/4
  uint8_t* row_roots;   // nsq * 2k * 90 B
  uint8_t* col_roots;   // nsq * 2k * 90 B
  uint8_t* dah;         // nsq * 32 B
  int32_t* status;      // nsq status words (kernels OR bits into them)
  int k;
  long nsq;
};

hipError_t launch_nmt_leaves(const SquareArgs& a, hipStream_t s);
// workspace layout for SquareArgs (digests | ns_table | rec_a | rec_b)
size_t nmt_workspace_bytes(int k, long nsq);
void nmt_workspace_carve(SquareArgs& a, void* ws);
hipError_t launch_nmt_trees(const SquareArgs& a, hipStream_t s);
hipError_t launch_dah(const SquareArgs& a, hipStream_t s);

}  // namespace dagpu
