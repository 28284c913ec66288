// split.cpp -- one oversized square split over `parts` GPUs (BASELINE configs[4]
// stress square).  The square is the same rsmt2d extension +
// wrapper NMT roots + DAH as the single-GPU path (pkg/da/data_availability_header.go:44-108);
// only the placement differs.  Rank g owns Q0 rows R_g = [g*k/P, (g+1)*k/P)
// and, after one all-to-all, EDS columns C_g = [g*2k/P, (g+1)*2k/P):
//
//   1 rows    row-encode R_g -> [Q0|Q1] rows, check their namespace order, pack P
//             send blocks (block h = rows R_g x columns C_h)
//   2 caller  all-to-all (RCCL over xGMI): block h -> rank h.  Rank h's receive
//             buffer is then rows 0..k-1 of its column slab, in row order.
//   3 cols    column-encode the slab (rows k..2k-1 = Q2|Q3 columns of C_h; Q3
//             by columns of Q1 equals Q3 by rows of Q2), hash every cell once,
//             full column roots of C_h, and NMT subtree roots of every row over
//             C_h (2k/P leaves: a power of two, so each is a node of the row tree)
//   4 caller  all-gather subtree records and column roots, max-reduce status
//   5 finish  top log2(P) levels of every row tree -> row roots; DAH
//
// Q2/Q3 never move back; the only data-path exchange is step 2.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "../../include/dagpu.h"
#include "forest.hpp"
#include "kernels.hpp"
#include "runtime.hpp"

namespace {

size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

// k <= kMaxK as every square entry point; k = kMaxSplitK only over at least
// kMinWideSplitParts ranks (its EDS fits 8 GPUs, not fewer)
bool wide_split(uint32_t k) { return k > (uint32_t)kMaxK && k <= (uint32_t)kMaxSplitK && is_pow2(k); }

int check_split(dagpu_ctx* ctx, uint32_t k, uint32_t parts, uint32_t part) {
  if (wide_split(k)) {
    if (parts < (uint32_t)kMinWideSplitParts)
      return set_err(ctx, DAGPU_ERR_UNSUPPORTED,
                     "split square k = " + std::to_string(k) + " needs >= " + std::to_string(kMinWideSplitParts) +
                         " parts (its EDS is 512 GiB)");
  } else {
    int rc = check_k(ctx, k);
    if (rc) return rc;
  }
  if (!is_pow2(parts) || parts > k) return set_err(ctx, DAGPU_ERR_ARG, "parts must be a power of two <= k");
  if (part >= parts) return set_err(ctx, DAGPU_ERR_ARG, "part out of range");
  return DAGPU_OK;
}

// workspace pieces (bytes) for one rank
struct SplitWs {
  uint8_t* rows_tmp;    // (k/P) x 2k shares
  uint8_t* leaves;      // 2k x W NMT leaf records
  uint8_t* col_inner;   // column forest inner levels
  uint8_t* row_inner;   // row subtree inner levels
  uint8_t* top_inner;   // finishing forest inner levels
  int64_t* meta;        // forest metadata (three plans)
};

struct SplitPlans {
  dagpu::ForestPlan cols, rows, top;
};

SplitPlans make_plans(uint32_t k, uint32_t parts) {
  const long w = 2L * k, W = w / parts;
  SplitPlans p;
  p.cols = dagpu::ForestPlan::uniform_plan(W, w, 1, W);   // tree c: leaf r at r*W + c
  p.rows = dagpu::ForestPlan::uniform_plan(w, W, W, 1);   // tree r: leaf c at r*W + c
  p.top = dagpu::ForestPlan::uniform_plan(w, parts, 1, w);  // tree r: leaf g at g*w + r
  return p;
}

size_t split_ws_bytes(uint32_t k, uint32_t parts, SplitWs* out, void* base) {
  const size_t w = 2 * (size_t)k, W = w / parts, rows = k / parts;
  SplitPlans p = make_plans(k, parts);
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off += al256(bytes > 0 ? bytes : 1); return o; };
  // rows_tmp also holds the square roots workspace at one part (cols step)
  const size_t sq_ws = parts == 1 ? dagpu::nmt_workspace_bytes((int)k, 1) : 0;
  const size_t o_tmp = take(rows * w * kSS > sq_ws ? rows * w * kSS : sq_ws);
  const size_t o_leaves = take(w * W * dagpu::kRecNmt);
  const size_t o_ci = take((size_t)p.cols.inner_records * dagpu::kRecNmt);
  const size_t o_ri = take((size_t)p.rows.inner_records * dagpu::kRecNmt);
  const size_t o_ti = take((size_t)p.top.inner_records * dagpu::kRecNmt);
  const size_t o_meta = take((p.cols.meta.size() + p.rows.meta.size() + p.top.meta.size()) * sizeof(int64_t));
  if (out) {
    uint8_t* b = (uint8_t*)base;
    out->rows_tmp = b + o_tmp;
    out->leaves = b + o_leaves;
    out->col_inner = b + o_ci;
    out->row_inner = b + o_ri;
    out->top_inner = b + o_ti;
    out->meta = (int64_t*)(b + o_meta);
  }
  return off;
}

}  // namespace

extern "C" {

size_t dagpu_split_workspace_size(uint32_t k, uint32_t parts) {
  if (k == 0 || parts == 0 || !is_pow2(k) || !is_pow2(parts) || parts > k) return 0;
  if (k > (uint32_t)kMaxK && (!wide_split(k) || parts < (uint32_t)kMinWideSplitParts)) return 0;
  return split_ws_bytes(k, parts, nullptr, nullptr) + 256;
}

int dagpu_split_rows_device(dagpu_ctx* ctx, uint32_t k, uint32_t parts, uint32_t part,
                            const uint8_t* d_ods_rows, uint8_t* d_send, int32_t* d_status,
                            void* d_workspace, void* stream) {
  if (!ctx || !d_ods_rows || !d_send || !d_status || !d_workspace) return DAGPU_ERR_ARG;
  int rc = check_split(ctx, k, parts, part);
  if (rc) return rc;
  (void)part;  // every rank runs the same code on its own rows
  hipStream_t s = (hipStream_t)stream;
  const long w = 2L * k, W = w / parts, rows = k / parts;
  SplitWs ws;
  split_ws_bytes(k, parts, &ws, d_workspace);
  HIP_TRY(ctx, hipMemsetAsync(d_status, 0, sizeof(int32_t), s));
  // nmt push order over whole Q0 rows (a row's Q0 part spans several slabs)
  HIP_TRY(ctx, dagpu::launch_ns_order_check(d_ods_rows, rows, k, (long)k * kSS, kSS, d_status,
                                            dagpu::kStatusPushOrder, s));
  // one part: the send block is the whole row-major [Q0 | Q1] of the rows, so
  // the encoder writes it in place (no staging copy)
  uint8_t* rows_out = parts == 1 ? d_send : ws.rows_tmp;
  EncodeArgs ea{};
  ea.in = d_ods_rows;
  ea.in_vec_stride = (long)k * kSS;
  ea.in_shard_stride = kSS;
  ea.copy = rows_out;
  ea.copy_vec_stride = w * kSS;
  ea.copy_shard_stride = kSS;
  ea.out = rows_out + (long)k * kSS;
  ea.out_vec_stride = w * kSS;
  ea.out_shard_stride = kSS;
  ea.nsq = 1;
  ea.nvec = rows;
  ea.nchunk = 1;
  ea.shard_bytes = kSS;
  {
    ProfScope p(ctx, 0, s);
    HIP_TRY(ctx, launch_rs_encode((int)k, ea, s));
  }
  // send block h = rows x columns [h*W, (h+1)*W), row-major
  for (uint32_t h = 0; parts > 1 && h < parts; h++) {
    HIP_TRY(ctx, hipMemcpy2DAsync(d_send + (size_t)h * rows * W * kSS, (size_t)W * kSS,
                                  ws.rows_tmp + (size_t)h * W * kSS, (size_t)w * kSS, (size_t)W * kSS,
                                  (size_t)rows, hipMemcpyDeviceToDevice, s));
  }
  return DAGPU_OK;
}

int dagpu_split_cols_device(dagpu_ctx* ctx, uint32_t k, uint32_t parts, uint32_t part, uint8_t* d_slab,
                            uint8_t* d_col_roots, uint8_t* d_row_sub, int32_t* d_status,
                            void* d_workspace, void* stream) {
  if (!ctx || !d_slab || !d_col_roots || !d_row_sub || !d_status || !d_workspace) return DAGPU_ERR_ARG;
  int rc = check_split(ctx, k, parts, part);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const long w = 2L * k, W = w / parts;
  SplitWs ws;
  split_ws_bytes(k, parts, &ws, d_workspace);
  SplitPlans pl = make_plans(k, parts);
  // column encode: vector c = column c of the slab (k data shards) -> rows k..2k-1
  EncodeArgs ea{};
  ea.in = d_slab;
  ea.in_vec_stride = kSS;
  ea.in_shard_stride = W * kSS;
  ea.out = d_slab + (long)k * W * kSS;
  ea.out_vec_stride = kSS;
  ea.out_shard_stride = W * kSS;
  ea.copy = nullptr;
  ea.nsq = 1;
  ea.nvec = W;
  ea.nchunk = 1;
  ea.shard_bytes = kSS;
  // every cell of the slab hashed once (wrapper namespace rule by global
  // coordinates).  Rows 0..k-1 are here already, so their leaves can overlap
  // the column encode on a side stream forked from `stream` (DAGPU_SPLIT_OVERLAP:
  // 1 = encode at the greatest stream priority, 2 = normal priority, 0 = off).
  // Default 1 for k >= 1024, where the LDS-slice encoders leave issue slots
  // free (k = 1024: 6.38 vs 6.49 ms); at k = 512 both kernels are issue-bound
  // and it measured 1.315-1.325 vs 1.298-1.325 ms (profiles/split_overlap_r05.log).
  // Off while profiling, so that each bracket times one kernel.
  dagpu::ForestLeafArgs la{};
  la.data = d_slab;
  la.data_stride = kSS;
  la.dlen = kSS;
  la.nleaves = w * W;
  la.pmode = dagpu::kPfxGrid;
  la.grid_k = (int)k;
  la.grid_w = W;
  la.grid_r0 = 0;
  la.grid_c0 = (long)part * W;
  la.rfc = 0;
  la.out = ws.leaves;
  // One part (below k = 1024, DAGPU_SPLIT_SQUARE != 0): the slab is the whole
  // EDS, so the square pipeline's roots kernels apply as they are (48-B node
  // records with namespace references, both axes' push order at level 1): its
  // column roots go out directly, its row roots as the 96-B records the finish
  // step reads.  (At k >= 1024 the forest path overlaps the top half's leaves
  // with the column encode, which measured faster.)
  const char* sq_env = sw(SW_SPLIT_SQUARE);
  if (parts == 1 && k < 1024 && !(sq_env && sq_env[0] == '0')) {
    {
      ProfScope p(ctx, 1, s);
      HIP_TRY(ctx, launch_rs_encode((int)k, ea, s));
    }
    SquareArgs sa{};
    sa.eds = d_slab;
    sa.eds_sq_stride = w * w * (long)kSS;
    sa.k = (int)k;
    sa.nsq = 1;
    nmt_workspace_carve(sa, ws.rows_tmp);  // rows_tmp is unused at one part (rows are encoded in place)
    sa.row_roots = ws.leaves;              // 2k packed row roots, then expanded into d_row_sub
    sa.col_roots = d_col_roots;
    sa.status = d_status;
    {
      ProfScope p(ctx, 2, s);
      HIP_TRY(ctx, launch_nmt_leaves(sa, s));
    }
    ProfScope p(ctx, 3, s);
    HIP_TRY(ctx, launch_nmt_trees(sa, s));
    HIP_TRY(ctx, dagpu::launch_node_to_rec(ws.leaves, w, d_row_sub, s));
    return DAGPU_OK;
  }
  const char* ov_env = sw(SW_SPLIT_OVERLAP);
  const int overlap = ctx->prof ? 0 : ov_env ? atoi(ov_env) : k >= 1024 ? 1 : 0;
  hipStream_t es = overlap ? side_stream(ctx, s, overlap == 1 ? 1 : 0) : nullptr;
  hipEvent_t fork = es ? ev_take(ctx) : nullptr, joined = es ? ev_take(ctx) : nullptr;
  if (es && fork && joined && hipEventRecord(fork, s) == hipSuccess && hipStreamWaitEvent(es, fork, 0) == hipSuccess) {
    hipError_t e = launch_rs_encode((int)k, ea, es);
    const bool encoding = e == hipSuccess && (e = hipEventRecord(joined, es)) == hipSuccess;
    dagpu::ForestLeafArgs top = la, bottom = la;
    top.nleaves = (long)k * W;
    bottom.data = d_slab + (size_t)k * W * kSS;
    bottom.nleaves = (long)k * W;
    bottom.grid_r0 = k;
    bottom.out = ws.leaves + (size_t)k * W * dagpu::kRecNmt;
    if (e == hipSuccess) e = dagpu::launch_forest_leaves(top, s);
    // the caller's stream waits for the side stream's encode whatever failed
    // after it, so nothing of this call writes the slab out of stream order
    if (encoding) {
      const hipError_t we = hipStreamWaitEvent(s, joined, 0);
      if (e == hipSuccess) e = we;
    }
    if (e == hipSuccess) e = dagpu::launch_forest_leaves(bottom, s);
    ev_give(ctx, fork);
    ev_give(ctx, joined);
    if (e != hipSuccess) return hip_fail(ctx, e, "split column encode / leaves");
  } else {
    ev_give(ctx, fork);
    ev_give(ctx, joined);
    {
      ProfScope p(ctx, 1, s);
      HIP_TRY(ctx, launch_rs_encode((int)k, ea, s));
    }
    ProfScope p(ctx, 2, s);
    HIP_TRY(ctx, dagpu::launch_forest_leaves(la, s));
  }
  {
    ProfScope p(ctx, 3, s);
    // full column trees (push order of the Q0 column parts checked at level 1,
    // into the step's one status word) and the row subtrees over this slab (row
    // order was checked on the row owners), each level of both in one launch
    const dagpu::ForestJob cols{&pl.cols, ws.leaves, ws.col_inner, ws.meta, 1, 1, 0, d_status, d_col_roots, 0, 0, 1};
    const dagpu::ForestJob rows{&pl.rows, ws.leaves, ws.row_inner, ws.meta + pl.cols.meta.size(), 1, 0, 0,
                                nullptr, d_row_sub, 1, 0};
    HIP_TRY(ctx, dagpu::forest_enqueue_pair(cols, rows, s));
  }
  // uniform plans: nothing uploaded, so nothing to wait for here
  return DAGPU_OK;
}

int dagpu_split_finish_device(dagpu_ctx* ctx, uint32_t k, uint32_t parts, const uint8_t* d_row_sub_all,
                              const uint8_t* d_col_roots_all, uint8_t* d_row_roots, uint8_t* d_dah,
                              void* d_workspace, void* stream) {
  if (!ctx || !d_row_sub_all || !d_col_roots_all || !d_row_roots || !d_dah || !d_workspace)
    return DAGPU_ERR_ARG;
  int rc = check_split(ctx, k, parts, 0);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  SplitWs ws;
  split_ws_bytes(k, parts, &ws, d_workspace);
  SplitPlans pl = make_plans(k, parts);
  {
    ProfScope p(ctx, 3, s);
    HIP_TRY(ctx, dagpu::forest_enqueue(pl.top, d_row_sub_all, ws.top_inner,
                                       ws.meta + pl.cols.meta.size() + pl.rows.meta.size(), 1, 0, 0, nullptr,
                                       d_row_roots, 0, 0, s));
  }
  SquareArgs sa{};
  sa.row_roots = d_row_roots;
  sa.col_roots = (uint8_t*)d_col_roots_all;
  sa.dah = d_dah;
  sa.digests = ws.leaves;  // slab leaf records, consumed by now: scratch for the DAH's subtree roots
  sa.k = (int)k;
  sa.nsq = 1;
  {
    ProfScope p(ctx, 4, s);
    HIP_TRY(ctx, launch_dah(sa, s));
  }
  return DAGPU_OK;
}

}  // extern "C"
