// forest.hpp -- generic batched Merkle forests (nmt_forest.hip) and the host
// planner that lays out their levels.  See nmt_forest.hip for the semantics.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "kernels.hpp"

namespace dagpu {

// leaf prefix modes
constexpr int kPfxNone = 0;    // message 0x00 | data (plain nmt Push / RFC-6962 item)
constexpr int kPfxSelf = 1;    // 0x00 | data[0:29] | data   (wrapper Q0, blob commitment)
constexpr int kPfxParity = 2;  // 0x00 | 0xFF*29 | data      (wrapper Q1..Q3)
constexpr int kPfxFlags = 3;   // per-leaf kPfxSelf / kPfxParity byte
constexpr int kPfxGrid = 4;    // wrapper rule by cell coordinates (row<k && col<k -> self)

constexpr int kRecNmt = 96;    // minNs[32] | maxNs[32] | digest[32]
constexpr int kRecRfc = 32;    // digest

// Per-tree status bit (nmt ErrInvalidPushOrder).
constexpr int kForestPushOrder = 1;

struct ForestLeafArgs {
  const uint8_t* data;
  long data_stride;  // bytes between consecutive leaves (multiple of 4)
  long dlen;         // data bytes per leaf
  long nleaves;
  int pmode;
  const uint8_t* pflags;          // kPfxFlags
  int grid_k;                     // kPfxGrid: original square width
  long grid_w, grid_r0, grid_c0;  // leaf i = cell (r0 + i / w, c0 + i % w)
  int rfc;                        // 1: RFC-6962 leaf digest, 0: NMT leaf record
  uint8_t* out;                   // nleaves records
};

struct ForestLevelArgs {
  const uint8_t* in;
  uint8_t* out;
  // input node j of tree t: in + (base(t) + j * in_lstride) * rec, where
  // base(t) = in_off ? in_off[t] : t * in_tstride and count(t) = in_off ?
  // in_off[t+1] - in_off[t] : in_per.
  const int64_t* in_off;
  long in_tstride, in_lstride, in_per;
  // output node j of tree t: out + (obase(t) + j) * rec, obase(t) = out_off ?
  // out_off[t] : t * out_per
  const int64_t* out_off;
  long out_per;
  long ntrees, total_out;
  int ignore_max, check_order, rfc;
  int32_t* status;  // per tree, OR kForestPushOrder (check_order only)
  int status_shared;  // 1: every tree ORs into status[0] (one flag for the batch)
};

hipError_t launch_forest_leaves(const ForestLeafArgs& a, hipStream_t s);
hipError_t launch_forest_level(const ForestLevelArgs& a, hipStream_t s);
// roots: root_idx[t] >= 0 is a record index into `inner`; -1 = empty tree
// (root = zero namespaces | SHA256("") for NMT, SHA256("") for RFC-6962);
// <= -2 is record -(idx + 2) of the leaf array `leaves`.  NMT roots are written
// as packed 90-B nodes (or 96-B records when records != 0); RFC-6962 roots as
// 32-B digests.
// out_stride: bytes between consecutive roots (0 = 90 / 96 / 32).
hipError_t launch_forest_roots(const uint8_t* leaves, const uint8_t* inner, const int64_t* root_idx,
                               long ntrees, int rfc, int records, uint8_t* out, long out_stride,
                               hipStream_t s);

// Push-order check over share vectors (ns = first 29 bytes of each share).
hipError_t launch_ns_order_check(const uint8_t* base, long nvec, long nper, long vec_stride, long elem_stride,
                                 int32_t* status, int bit, hipStream_t s);

// Packed 90-B nodes -> 96-B NMT records (the forest's record format).
hipError_t launch_node_to_rec(const uint8_t* nodes, long n, uint8_t* recs, hipStream_t s);

// Gather (row, depth, position) nodes of exported row trees as packed 90-B nodes.
hipError_t launch_node_gather(const uint8_t* nodes, int w, const uint32_t* req, long n, uint8_t* out,
                              hipStream_t s);

// Host-side level plan of one forest.  Leaves (level 0) are either packed tree
// after tree (ragged: counts[t] leaves each) or uniform with (tstride,
// lstride) addressing inside a caller-owned leaf array.  Levels >= 1 are packed
// tree-major, one after another, in a single record buffer.
struct ForestPlan {
  long ntrees = 0;
  bool uniform = true;
  long per0 = 0;                 // uniform leaf count
  long tstride0 = 0, lstride0 = 1;
  std::vector<long> counts0;     // ragged leaf counts
  int nlevels = 0;               // inner levels (level 1..nlevels)
  std::vector<long> total;       // total[L] nodes at level L (L >= 1)
  std::vector<long> base;        // base[L] record offset of level L in the inner buffer
  std::vector<long> per;         // uniform: nodes per tree at level L
  std::vector<std::vector<int64_t>> off;  // ragged: off[L] (ntrees + 1 prefix sums), L >= 0
  // root_idx per tree in the launch_forest_roots encoding
  std::vector<int64_t> root_idx;
  long inner_records = 0;        // records needed for levels >= 1
  // device metadata image: ragged offset arrays then root_idx (int64)
  std::vector<int64_t> meta;
  std::vector<long> meta_off;    // meta_off[L]: start of off[L] in meta (ragged)
  long meta_root = 0;            // start of root_idx in meta
  void finalize();

  static ForestPlan uniform_plan(long ntrees, long leaves, long tstride, long lstride);
  static ForestPlan ragged_plan(const std::vector<long>& counts);
};

// Enqueue every inner level and the roots of plan `p` on stream s.
//   d_leaves  level-0 records (rec = 96 B NMT / 32 B RFC-6962)
//   d_inner   p.inner_records records
//   d_meta    p.meta.size() int64 (ragged plans: uploaded here, keep `p` alive
//             until the stream has passed this point; uniform plans upload
//             nothing and need neither)
//   d_status  per-tree status (check_order), may be null otherwise
//   d_roots   ntrees roots (90 B packed / 96 B records / 32 B digests)
hipError_t forest_enqueue(const ForestPlan& p, const uint8_t* d_leaves, uint8_t* d_inner, int64_t* d_meta,
                          int ignore_max, int check_order, int rfc, int32_t* d_status, uint8_t* d_roots,
                          int records, long roots_stride, hipStream_t s);

// Two forests hashed level by level in shared launches (level L of both in
// one grid): the column trees and the row subtrees of a split slab.
struct ForestJob {
  const ForestPlan* p;
  const uint8_t* d_leaves;
  uint8_t* d_inner;
  int64_t* d_meta;
  int ignore_max, check_order, rfc;
  int32_t* d_status;
  uint8_t* d_roots;
  int records;
  long roots_stride;
  int status_shared = 0;  // ForestLevelArgs::status_shared
};
hipError_t forest_enqueue_pair(const ForestJob& x, const ForestJob& y, hipStream_t s);

}  // namespace dagpu
