// trees.cpp -- C ABI for batched generic trees on the GPU (include/dagpu.h):
//   dagpu_nmt_roots        nmt.New(sha256, NamespaceIDSize(29), IgnoreMaxNamespace)
//                          Push*/Root (nmt v0.20.0; hasher mirror
//                          test/util/malicious/hasher.go:161-309)
//   dagpu_wrapper_roots    wrapper.ErasuredNamespacedMerkleTree Push/Root as the
//                          rsmt2d.Tree of wrapper.NewConstructor
//                          (pkg/wrapper/nmt_wrapper.go:55-124)
//   dagpu_merkle_roots     merkle.HashFromByteSlices (celestia-core crypto/merkle)
//   dagpu_blob_commitments inclusion.CreateCommitment over already-split blob
//                          shares (pkg/inclusion/commitment.go:19-75,
//                          blob_share_commitment_rules.go:76-101)
// Each call uploads the pushes once, hashes every leaf and level of every
// tree in a handful of launches (nmt_forest.hip) and returns the roots.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <cmath>
#include <string>
#include <functional>
#include <vector>

#include "../../include/dagpu.h"
#include "forest.hpp"
#include "kernels.hpp"
#include "host_sha256.hpp"
#include "runtime.hpp"

namespace {

long round4(long v) { return (v + 3) & ~3L; }

// Upload `n` leaves of `len` bytes (packed on the host) into a 4-B aligned
// device array with stride round4(len).
int upload_leaves(dagpu_ctx* ctx, const uint8_t* host, long n, long len, long* stride_out,
                  hipStream_t s) {
  const long stride = round4(len < 1 ? 1 : len);
  *stride_out = stride;
  HIP_TRY(ctx, ctx->t_leaf_data.ensure((size_t)(stride * (n > 0 ? n : 1))));
  if (n == 0 || len == 0) return DAGPU_OK;
  if (stride == len) {
    HIP_TRY(ctx, hipMemcpyAsync(ctx->t_leaf_data.p, host, (size_t)(n * len), hipMemcpyHostToDevice, s));
  } else {
    HIP_TRY(ctx, hipMemcpy2DAsync(ctx->t_leaf_data.p, (size_t)stride, host, (size_t)len, (size_t)len,
                                  (size_t)n, hipMemcpyHostToDevice, s));
  }
  return DAGPU_OK;
}

// One NMT forest over leaves already in ctx->t_leaf_data; roots to host.
int nmt_forest_host(dagpu_ctx* ctx, const std::vector<long>& counts, long dlen, long stride, int pmode,
                    const uint8_t* flags_host, int ignore_max, uint8_t* roots, int32_t* status,
                    hipStream_t s) {
  const long T = (long)counts.size();
  long nleaves = 0;
  for (long c : counts) nleaves += c;
  ForestPlan plan = ForestPlan::ragged_plan(counts);
  HIP_TRY(ctx, ctx->t_leaves.ensure((size_t)(kRecNmt * (nleaves > 0 ? nleaves : 1))));
  HIP_TRY(ctx, ctx->t_inner.ensure((size_t)(kRecNmt * (plan.inner_records > 0 ? plan.inner_records : 1))));
  HIP_TRY(ctx, ctx->t_meta.ensure(plan.meta.size() * sizeof(int64_t) + 8));
  HIP_TRY(ctx, ctx->t_out.ensure((size_t)(kNodeSize * T + 16)));
  HIP_TRY(ctx, ctx->t_status.ensure((size_t)(4 * T + 4)));
  HIP_TRY(ctx, hipMemsetAsync(ctx->t_status.p, 0, (size_t)(4 * T + 4), s));
  if (pmode == kPfxFlags) {
    HIP_TRY(ctx, ctx->t_flags.ensure((size_t)(nleaves + 1)));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->t_flags.p, flags_host, (size_t)nleaves, hipMemcpyHostToDevice, s));
  }
  ForestLeafArgs la{};
  la.data = (const uint8_t*)ctx->t_leaf_data.p;
  la.data_stride = stride;
  la.dlen = dlen;
  la.nleaves = nleaves;
  la.pmode = pmode;
  la.pflags = (const uint8_t*)ctx->t_flags.p;
  la.rfc = 0;
  la.out = (uint8_t*)ctx->t_leaves.p;
  HIP_TRY(ctx, launch_forest_leaves(la, s));
  HIP_TRY(ctx, forest_enqueue(plan, (const uint8_t*)ctx->t_leaves.p, (uint8_t*)ctx->t_inner.p,
                              (int64_t*)ctx->t_meta.p, ignore_max, 1, 0, (int32_t*)ctx->t_status.p,
                              (uint8_t*)ctx->t_out.p, 0, 0, s));
  std::vector<int32_t> st(T);
  if (T) {
    HIP_TRY(ctx, hipMemcpyAsync(roots, ctx->t_out.p, (size_t)(kNodeSize * T), hipMemcpyDeviceToHost, s));
    HIP_TRY(ctx, hipMemcpyAsync(st.data(), ctx->t_status.p, (size_t)(4 * T), hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(ctx, hipStreamSynchronize(s));  // also keeps `plan` alive past its upload
  int first = DAGPU_OK;
  for (long t = 0; t < T; t++) {
    const int v = (st[t] & kForestPushOrder) ? DAGPU_ERR_PUSH_ORDER : DAGPU_OK;
    if (status) status[t] = v;
    if (v && !first) first = v;
  }
  if (first) set_err(ctx, first, "invalid push order: pushed namespace is smaller than the last one");
  return first;
}

// RoundUpPowerOfTwo (pkg/shares/powers_of_two.go:10-16)
uint64_t round_up_pow2(uint64_t v) {
  uint64_t r = 1;
  while (r < v) r <<= 1;
  return r;
}

// inclusion.SubTreeWidth (pkg/inclusion/blob_share_commitment_rules.go:85-101)
uint64_t subtree_width(uint64_t share_count, uint64_t threshold) {
  uint64_t s = share_count / threshold;
  if (share_count % threshold != 0) s++;
  s = round_up_pow2(s);
  const uint64_t min_sq = round_up_pow2((uint64_t)std::ceil(std::sqrt((double)share_count)));
  return s < min_sq ? s : min_sq;
}

// inclusion.MerkleMountainRangeSizes (pkg/inclusion/commitment.go:85-107)
std::vector<long> mmr_sizes(uint64_t total, uint64_t max_tree) {
  std::vector<long> out;
  while (total != 0) {
    if (total >= max_tree) {
      out.push_back((long)max_tree);
      total -= max_tree;
    } else {
      const uint64_t up = round_up_pow2(total);
      const uint64_t t = up == total ? up : up / 2;
      out.push_back((long)t);
      total -= t;
    }
  }
  return out;
}

}  // namespace

extern "C" {

int dagpu_nmt_roots(dagpu_ctx* ctx, size_t ntrees, const uint32_t* leaf_counts, const uint8_t* leaves,
                    size_t leaf_len, int prefix_mode, const uint8_t* prefix_flags, int ignore_max_ns,
                    uint8_t* roots, int32_t* status) {
  if (!ctx || (ntrees && (!leaf_counts || !roots))) return DAGPU_ERR_ARG;
  if (prefix_mode < DAGPU_PREFIX_NONE || prefix_mode > DAGPU_PREFIX_FLAGS) return DAGPU_ERR_ARG;
  std::lock_guard<std::mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  std::vector<long> counts(ntrees);
  long n = 0;
  for (size_t t = 0; t < ntrees; t++) n += (counts[t] = leaf_counts[t]);
  if (n && !leaves) return DAGPU_ERR_ARG;
  if (prefix_mode == DAGPU_PREFIX_FLAGS && n && !prefix_flags) return DAGPU_ERR_ARG;
  // nmt HashLeaf / Push: namespaced data shorter than the namespace is rejected
  // (ErrInvalidLeafLen / ErrMismatchedNamespaceSize); prepending modes need the
  // namespace inside the data only for DAGPU_PREFIX_SELF.
  const bool need_ns = prefix_mode == DAGPU_PREFIX_NONE || prefix_mode == DAGPU_PREFIX_SELF ||
                       prefix_mode == DAGPU_PREFIX_FLAGS;
  if (n && need_ns && leaf_len < (size_t)kNsSize)
    return set_err(ctx, DAGPU_ERR_SHARE_SIZE, "invalid leaf length: shorter than the namespace size");
  if (prefix_mode == DAGPU_PREFIX_FLAGS)
    for (long i = 0; i < n; i++)
      if (prefix_flags[i] != DAGPU_PREFIX_SELF && prefix_flags[i] != DAGPU_PREFIX_PARITY) return DAGPU_ERR_ARG;
  hipStream_t s = ctx->stream;
  long stride = 0;
  int rc = upload_leaves(ctx, leaves, n, (long)leaf_len, &stride, s);
  if (rc) return rc;
  return nmt_forest_host(ctx, counts, (long)leaf_len, stride, prefix_mode, prefix_flags, ignore_max_ns != 0,
                         roots, status, s);
}

int dagpu_wrapper_roots(dagpu_ctx* ctx, uint64_t square_size, size_t ntrees, const uint32_t* axis_index,
                        const uint32_t* leaf_counts, const uint8_t* shares, size_t share_len,
                        uint8_t* roots, int32_t* status) {
  if (!ctx || (ntrees && (!axis_index || !leaf_counts || !roots))) return DAGPU_ERR_ARG;
  // NewErasuredNamespacedMerkleTree panics on squareSize == 0 (nmt_wrapper.go:56-58)
  if (square_size == 0) return set_err(ctx, DAGPU_ERR_ARG, "cannot create a ErasuredNamespacedMerkleTree of squareSize == 0");
  long n = 0;
  for (size_t t = 0; t < ntrees; t++) {
    // Push bounds check (nmt_wrapper.go:94-96)
    if ((uint64_t)axis_index[t] + 1 > 2 * square_size || (uint64_t)leaf_counts[t] > 2 * square_size) {
      if (status) status[t] = DAGPU_ERR_ARG;
      char buf[160];
      snprintf(buf, sizeof buf, "pushed past predetermined square size: boundary at %llu index at %u %u",
               (unsigned long long)(2 * square_size), axis_index[t],
               leaf_counts[t] ? leaf_counts[t] - 1 : 0);
      return set_err(ctx, DAGPU_ERR_ARG, buf);
    }
    n += leaf_counts[t];
  }
  if (n && !shares) return DAGPU_ERR_ARG;
  // nmt_wrapper.go:97-99
  if (n && share_len < (size_t)kNsSize)
    return set_err(ctx, DAGPU_ERR_SHARE_SIZE, "data is too short to contain namespace ID");
  // isQuadrantZero (nmt_wrapper.go:138-140): shareIndex < k && axisIndex < k
  std::vector<uint8_t> flags((size_t)n);
  long i = 0;
  for (size_t t = 0; t < ntrees; t++)
    for (uint32_t j = 0; j < leaf_counts[t]; j++, i++)
      flags[i] = (j < square_size && axis_index[t] < square_size) ? DAGPU_PREFIX_SELF : DAGPU_PREFIX_PARITY;
  return dagpu_nmt_roots(ctx, ntrees, leaf_counts, shares, share_len, DAGPU_PREFIX_FLAGS, flags.data(), 1,
                         roots, status);
}

int dagpu_merkle_roots(dagpu_ctx* ctx, size_t ntrees, const uint32_t* counts, const uint8_t* items,
                       size_t item_len, uint8_t* out32) {
  if (!ctx || (ntrees && (!counts || !out32))) return DAGPU_ERR_ARG;
  std::lock_guard<std::mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  std::vector<long> cnt(ntrees);
  long n = 0;
  for (size_t t = 0; t < ntrees; t++) n += (cnt[t] = counts[t]);
  if (n && !items) return DAGPU_ERR_ARG;
  hipStream_t s = ctx->stream;
  long stride = 0;
  int rc = upload_leaves(ctx, items, n, (long)item_len, &stride, s);
  if (rc) return rc;
  ForestPlan plan = ForestPlan::ragged_plan(cnt);
  HIP_TRY(ctx, ctx->t_leaves.ensure((size_t)(kRecRfc * (n > 0 ? n : 1))));
  HIP_TRY(ctx, ctx->t_inner.ensure((size_t)(kRecRfc * (plan.inner_records > 0 ? plan.inner_records : 1))));
  HIP_TRY(ctx, ctx->t_meta.ensure(plan.meta.size() * sizeof(int64_t) + 8));
  HIP_TRY(ctx, ctx->t_out.ensure((size_t)(32 * ntrees + 16)));
  ForestLeafArgs la{};
  la.data = (const uint8_t*)ctx->t_leaf_data.p;
  la.data_stride = stride;
  la.dlen = (long)item_len;
  la.nleaves = n;
  la.pmode = kPfxNone;
  la.rfc = 1;
  la.out = (uint8_t*)ctx->t_leaves.p;
  HIP_TRY(ctx, launch_forest_leaves(la, s));
  HIP_TRY(ctx, forest_enqueue(plan, (const uint8_t*)ctx->t_leaves.p, (uint8_t*)ctx->t_inner.p,
                              (int64_t*)ctx->t_meta.p, 0, 0, 1, nullptr, (uint8_t*)ctx->t_out.p, 0, 0, s));
  if (ntrees) HIP_TRY(ctx, hipMemcpyAsync(out32, ctx->t_out.p, 32 * ntrees, hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  return DAGPU_OK;
}

size_t dagpu_row_nodes_size(uint32_t k) {
  if (k == 0 || !is_pow2(k) || k > (uint32_t)kMaxK) return 0;
  const long w = 2L * k;
  long recs = 0;
  for (long per = w; per >= 1; per >>= 1) recs += w * per;
  return (size_t)recs * kRecNmt;
}

size_t dagpu_row_nodes_workspace_size(uint32_t k) {
  if (k == 0 || !is_pow2(k) || k > (uint32_t)kMaxK) return 0;
  const long w = 2L * k;
  return (size_t)w * sizeof(int64_t) + 256;  // plan metadata (root indices)
}

int dagpu_row_nodes_device(dagpu_ctx* ctx, uint32_t k, const uint8_t* d_eds, uint8_t* d_nodes, void* d_workspace,
                           void* stream) {
  if (!ctx || !d_eds || !d_nodes || !d_workspace) return DAGPU_ERR_ARG;
  int rc = check_k(ctx, k);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const long w = 2L * k;
  // leaves (level 0): every cell with the wrapper namespace rule, row-major
  ForestLeafArgs la{};
  la.data = d_eds;
  la.data_stride = kShareSize;
  la.dlen = kShareSize;
  la.nleaves = w * w;
  la.pmode = kPfxGrid;
  la.grid_k = (int)k;
  la.grid_w = w;
  la.out = d_nodes;
  HIP_TRY(ctx, launch_forest_leaves(la, s));
  // every row tree, all levels kept: level L packed right after level L-1
  ForestPlan plan = ForestPlan::uniform_plan(w, w, w, 1);
  HIP_TRY(ctx, forest_enqueue(plan, d_nodes, d_nodes + (size_t)w * w * kRecNmt, (int64_t*)d_workspace, 1, 0, 0,
                              nullptr, d_nodes + (size_t)w * w * kRecNmt + (size_t)plan.base[plan.nlevels] * kRecNmt,
                              1, 0, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));  // plan metadata upload complete
  return DAGPU_OK;
}

int dagpu_row_nodes_gather_device(dagpu_ctx* ctx, uint32_t k, const uint8_t* d_nodes, size_t n,
                                  const uint32_t* d_requests, uint8_t* d_out, void* stream) {
  if (!ctx || !d_nodes || (n && (!d_requests || !d_out))) return DAGPU_ERR_ARG;
  int rc = check_k(ctx, k);
  if (rc) return rc;
  HIP_TRY(ctx, launch_node_gather(d_nodes, 2 * (int)k, d_requests, (long)n, d_out, (hipStream_t)stream));
  return DAGPU_OK;
}

int dagpu_merkle_levels(dagpu_ctx* ctx, size_t n, const uint8_t* items, size_t item_len, uint8_t* out32,
                        size_t* n_nodes) {
  if (!ctx || !n_nodes || (n && (!items || !out32))) return DAGPU_ERR_ARG;
  std::lock_guard<std::mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  std::vector<long> cnt{(long)n};
  ForestPlan plan = ForestPlan::ragged_plan(cnt);
  const size_t total = n + (size_t)plan.inner_records;
  if (*n_nodes < total) {
    *n_nodes = total;
    return set_err(ctx, DAGPU_ERR_ARG, "output too small for every tree level");
  }
  *n_nodes = total;
  if (n == 0) return DAGPU_OK;
  hipStream_t s = ctx->stream;
  long stride = 0;
  int rc = upload_leaves(ctx, items, (long)n, (long)item_len, &stride, s);
  if (rc) return rc;
  HIP_TRY(ctx, ctx->t_leaves.ensure(total * kRecRfc + 64));
  HIP_TRY(ctx, ctx->t_meta.ensure(plan.meta.size() * sizeof(int64_t) + 8));
  HIP_TRY(ctx, ctx->t_out.ensure(64));
  ForestLeafArgs la{};
  la.data = (const uint8_t*)ctx->t_leaf_data.p;
  la.data_stride = stride;
  la.dlen = (long)item_len;
  la.nleaves = (long)n;
  la.pmode = kPfxNone;
  la.rfc = 1;
  la.out = (uint8_t*)ctx->t_leaves.p;
  HIP_TRY(ctx, launch_forest_leaves(la, s));
  uint8_t* inner = (uint8_t*)ctx->t_leaves.p + n * kRecRfc;  // levels right after the leaves
  HIP_TRY(ctx, forest_enqueue(plan, (const uint8_t*)ctx->t_leaves.p, inner, (int64_t*)ctx->t_meta.p, 0, 0, 1,
                              nullptr, (uint8_t*)ctx->t_out.p, 0, 0, s));
  HIP_TRY(ctx, hipMemcpyAsync(out32, ctx->t_leaves.p, total * kRecRfc, hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  return DAGPU_OK;
}

int dagpu_nmt_verify_inclusion(const uint8_t* ns29, const uint8_t* leaves, size_t n, size_t leaf_len,
                               int64_t start, int64_t end, const uint8_t* nodes, size_t nnodes,
                               const uint8_t* root90) {
  using namespace dagpu::host;
  if (!ns29 || !root90 || (n && !leaves) || (nnodes && !nodes)) return DAGPU_ERR_ARG;
  // Proof.VerifyInclusion: valid range, one leaf per proven index
  if (start < 0 || start >= end || (int64_t)n != end - start) return DAGPU_ERR_PROOF;
  std::vector<uint8_t> lh(n * kNodeLen);
  for (size_t i = 0; i < n; i++) nmt_hash_leaf(ns29, leaves + i * leaf_len, leaf_len, &lh[i * kNodeLen]);
  size_t next_leaf = 0, next_node = 0;
  bool ok = true;
  // nmt getSplitPoint: largest power of two strictly below length (length >= 2)
  auto split = [](int64_t len) {
    int64_t k = 1;
    while (k * 2 < len) k *= 2;
    return k;
  };
  // verifyLeafHashes.computeRoot: proof nodes fill the subtrees disjoint from
  // [start, end), popped left to right; an absent right subtree is skipped.
  std::function<bool(int64_t, int64_t, uint8_t*)> root_of = [&](int64_t lo, int64_t hi, uint8_t* out) -> bool {
    if (hi - lo == 1 && start <= lo && lo < end) {
      memcpy(out, &lh[next_leaf++ * kNodeLen], kNodeLen);
      return true;
    }
    if (hi - lo == 1 || hi <= start || lo >= end) {
      if (next_node >= nnodes) return false;
      memcpy(out, nodes + next_node++ * kNodeLen, kNodeLen);
      return true;
    }
    const int64_t k = split(hi - lo);
    uint8_t l[kNodeLen], r[kNodeLen];
    if (!root_of(lo, lo + k, l)) return false;  // a missing left subtree cannot verify
    if (!root_of(lo + k, hi, r)) {
      memcpy(out, l, kNodeLen);
      return true;
    }
    if (!nmt_hash_node(l, r, out)) ok = false;
    return true;
  };
  int64_t est = 1;
  while (est < end) est *= 2;  // getSplitPoint(end) * 2: the subtree holding the range
  uint8_t root[kNodeLen];
  if (!root_of(0, est, root)) return DAGPU_ERR_PROOF;
  for (; next_node < nnodes; next_node++) {  // remaining right-hand nodes
    uint8_t t[kNodeLen];
    if (!nmt_hash_node(root, nodes + next_node * kNodeLen, t)) ok = false;
    memcpy(root, t, kNodeLen);
  }
  if (!ok || next_leaf != n) return DAGPU_ERR_PROOF;
  return memcmp(root, root90, kNodeLen) == 0 ? DAGPU_OK : DAGPU_ERR_PROOF;
}

int dagpu_merkle_verify(const uint8_t* root32, const uint8_t* leaf, size_t leaf_len, int64_t index,
                        int64_t total, const uint8_t* aunts, size_t naunts) {
  using namespace dagpu::host;
  if (!root32 || (leaf_len && !leaf) || (naunts && !aunts)) return DAGPU_ERR_ARG;
  if (total < 0 || index < 0) return DAGPU_ERR_PROOF;
  uint8_t h[32];
  merkle_leaf_hash(leaf, leaf_len, h);
  // crypto/merkle computeHashFromAunts, aunts ordered leaf to root
  std::function<bool(int64_t, int64_t, size_t, uint8_t*)> up = [&](int64_t idx, int64_t tot, size_t na,
                                                                     uint8_t* out) -> bool {
    if (idx >= tot || idx < 0 || tot <= 0) return false;
    if (tot == 1) {
      if (na != 0) return false;
      memcpy(out, h, 32);
      return true;
    }
    if (na == 0) return false;
    int64_t left = 1;
    while (left * 2 < tot) left *= 2;
    uint8_t sub[32];
    const uint8_t* aunt = aunts + (na - 1) * 32;
    if (idx < left) {
      if (!up(idx, left, na - 1, sub)) return false;
      merkle_inner_hash(sub, aunt, out);
    } else {
      if (!up(idx - left, tot - left, na - 1, sub)) return false;
      merkle_inner_hash(aunt, sub, out);
    }
    return true;
  };
  uint8_t root[32];
  if (!up(index, total, naunts, root)) return DAGPU_ERR_PROOF;
  return memcmp(root, root32, 32) == 0 ? DAGPU_OK : DAGPU_ERR_PROOF;
}

int dagpu_subtree_width(uint64_t share_count, uint32_t subtree_root_threshold) {
  if (subtree_root_threshold == 0) return DAGPU_ERR_ARG;
  return (int)subtree_width(share_count, subtree_root_threshold);
}

int dagpu_blob_commitments(dagpu_ctx* ctx, size_t nblobs, const uint8_t* namespaces,
                           const uint32_t* share_counts, const uint8_t* shares,
                           uint32_t subtree_root_threshold, uint8_t* commitments) {
  if (!ctx || (nblobs && (!namespaces || !share_counts || !commitments))) return DAGPU_ERR_ARG;
  if (subtree_root_threshold == 0) return set_err(ctx, DAGPU_ERR_ARG, "subtree root threshold must be positive");
  std::lock_guard<std::mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  // Plan: one NMT per MMR tree (leaf = namespace | share, commitment.go:53-63),
  // then one RFC-6962 tree per blob over its subtree roots (commitment.go:73).
  std::vector<long> tree_sizes, trees_per_blob(nblobs);
  long nshares = 0;
  for (size_t b = 0; b < nblobs; b++) {
    const uint64_t c = share_counts[b];
    if (c == 0) return set_err(ctx, DAGPU_ERR_ARG, "blob has no shares");
    const auto sz = mmr_sizes(c, subtree_width(c, subtree_root_threshold));
    trees_per_blob[b] = (long)sz.size();
    tree_sizes.insert(tree_sizes.end(), sz.begin(), sz.end());
    nshares += (long)c;
  }
  if (nshares && !shares) return DAGPU_ERR_ARG;
  hipStream_t s = ctx->stream;
  // leaves: namespace(29) | share(512) = 541 B, stride 544
  const long llen = kNsSize + kShareSize, stride = round4(llen);
  std::vector<uint8_t> host((size_t)(stride * (nshares > 0 ? nshares : 1)), 0);
  {
    long i = 0;
    for (size_t b = 0; b < nblobs; b++)
      for (uint32_t j = 0; j < share_counts[b]; j++, i++) {
        memcpy(&host[(size_t)(i * stride)], namespaces + b * kNsSize, kNsSize);
        memcpy(&host[(size_t)(i * stride + kNsSize)], shares + (size_t)i * kShareSize, kShareSize);
      }
  }
  HIP_TRY(ctx, ctx->t_leaf_data.ensure(host.size()));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->t_leaf_data.p, host.data(), host.size(), hipMemcpyHostToDevice, s));
  ForestPlan nplan = ForestPlan::ragged_plan(tree_sizes);
  ForestPlan rplan = ForestPlan::ragged_plan(trees_per_blob);
  const long ntrees = (long)tree_sizes.size();
  const long item_stride = 92;  // 90-B subtree roots, 4-B aligned
  const size_t meta_n = nplan.meta.size() + rplan.meta.size();
  HIP_TRY(ctx, ctx->t_leaves.ensure((size_t)(kRecNmt * (nshares + 1))));
  HIP_TRY(ctx, ctx->t_inner.ensure((size_t)(kRecNmt * (nplan.inner_records + 1))));
  HIP_TRY(ctx, ctx->t_meta.ensure(meta_n * sizeof(int64_t) + 16));
  HIP_TRY(ctx, ctx->t_out.ensure((size_t)(item_stride * ntrees + kRecRfc * (ntrees + rplan.inner_records) +
                                          32 * nblobs + 64)));
  HIP_TRY(ctx, ctx->t_status.ensure((size_t)(4 * ntrees + 4)));
  HIP_TRY(ctx, hipMemsetAsync(ctx->t_status.p, 0, (size_t)(4 * ntrees + 4), s));
  ForestLeafArgs la{};
  la.data = (const uint8_t*)ctx->t_leaf_data.p;
  la.data_stride = stride;
  la.dlen = llen;
  la.nleaves = nshares;
  la.pmode = kPfxNone;
  la.rfc = 0;
  la.out = (uint8_t*)ctx->t_leaves.p;
  HIP_TRY(ctx, launch_forest_leaves(la, s));
  uint8_t* items = (uint8_t*)ctx->t_out.p;
  uint8_t* rleaves = items + item_stride * ntrees;
  uint8_t* rinner = rleaves + kRecRfc * ntrees;
  uint8_t* out = rinner + kRecRfc * (rplan.inner_records + 1);
  int64_t* meta = (int64_t*)ctx->t_meta.p;
  HIP_TRY(ctx, forest_enqueue(nplan, (const uint8_t*)ctx->t_leaves.p, (uint8_t*)ctx->t_inner.p, meta, 1, 1, 0,
                              (int32_t*)ctx->t_status.p, items, 0, item_stride, s));
  ForestLeafArgs ra{};
  ra.data = items;
  ra.data_stride = item_stride;
  ra.dlen = kNodeSize;
  ra.nleaves = ntrees;
  ra.pmode = kPfxNone;
  ra.rfc = 1;
  ra.out = rleaves;
  HIP_TRY(ctx, launch_forest_leaves(ra, s));
  HIP_TRY(ctx, forest_enqueue(rplan, rleaves, rinner, meta + nplan.meta.size(), 0, 0, 1, nullptr, out, 0, 0, s));
  std::vector<int32_t> st(ntrees);
  if (nblobs) HIP_TRY(ctx, hipMemcpyAsync(commitments, out, 32 * nblobs, hipMemcpyDeviceToHost, s));
  if (ntrees) HIP_TRY(ctx, hipMemcpyAsync(st.data(), ctx->t_status.p, 4 * ntrees, hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  for (long t = 0; t < ntrees; t++)
    if (st[t]) return set_err(ctx, DAGPU_ERR_PUSH_ORDER, "invalid push order");
  return DAGPU_OK;
}

}  // extern "C"
