// runtime.hpp -- internal host runtime shared by the C-ABI translation units
// (dagpu.cpp, trees.cpp, split.cpp): the context, device buffers, error
// helpers and the per-kernel profiling bracket.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/dagpu.h"
#include "kernels.hpp"

using namespace dagpu;

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= n) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) n = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

// Page-locked host staging (hipHostMalloc), grown on demand.
struct HostBuf {
  void* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= n) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e == hipSuccess) n = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
  }
};

struct ProfRec {
  int id;
  hipEvent_t a, b;
};

struct dagpu_ctx {
  int device = 0;
  // unique per context ever opened in this process: a thread's saved error is
  // tied to (pointer, generation), so a later context at the same address
  // never reports a destroyed one's message (see dagpu_last_error)
  uint64_t gen = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  // Last error message.  Device-resident entry points run without `mu`
  // (several host threads may enqueue on one context, each on its own
  // stream), so the message has its own lock; see set_err / dagpu_last_error.
  std::mutex err_mu;
  std::string err;
  DevBuf ods, eds, rr, cr, dah, status, ws;
  DevBuf res;  // host path: roots | roots | DAHs | status, one device->host copy
  // host-mode pipeline (dagpu.cpp run_group_pipelined): H2D on copy_stream,
  // kernels + D2H on stream, two slots handed over with events
  hipStream_t copy_stream = nullptr;
  // device-resident pipeline (dagpu.cpp dagpu_extend_batch_device): RS of later
  // slices on a side stream beside the NMT work of earlier slices on the caller's
  // stream.  One side stream per caller stream (up to kMaxSideStreams, then
  // callers share them round-robin), so concurrent callers on different streams
  // do not queue their RS slices behind each other.
  // Each caller stream also gets a second NMT stream (slices alternate between
  // it and the caller's stream, so the tree levels and DAH of slice i, which
  // fill few CUs, overlap the leaves of slice i+1) and a high-priority RS stream.
  static constexpr size_t kMaxSideStreams = 16;
  struct Side {
    hipStream_t caller = nullptr, rs = nullptr, rs_hi = nullptr;
  };
  std::mutex side_mu;
  std::vector<Side> side;
  std::mutex ev_mu;
  std::vector<hipEvent_t> ev_pool;  // timing-disabled events, recycled per call
  // page-locked 4 KiB mailboxes for the small device->host reads of Repair's
  // rounds (counters, check flags), one per concurrent call, recycled
  static constexpr size_t kMailbox = 4096;
  std::mutex mb_mu;
  std::vector<void*> mailboxes;
  hipEvent_t ev_loaded[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr};
  HostBuf h_out;
  // generic forests / commitments / split square (trees.cpp, split.cpp)
  DevBuf t_leaf_data, t_leaves, t_inner, t_meta, t_out, t_status, t_flags;
  // profiling: per-kernel brackets (prof) and, for host-path calls, a stage
  // timeline of the last call (stages_on; dagpu_profile_stages)
  bool prof = false;
  bool stages_on = false;
  static constexpr int kStages = DAGPU_STAGES;
  hipEvent_t stage_ev[kStages] = {};
  uint32_t stage_mask = 0;  // stages recorded by the last host-path call
  std::mutex prof_mu;
  std::vector<ProfRec> pending;
  std::vector<hipEvent_t> pool;
  double prof_ms[DAGPU_PROFILE_KERNELS] = {};
  // the last Repair call's schedule (dagpu_repair_stats), under prof_mu; a
  // started Repair keeps its own in its slot and publishes them at its join
  int64_t rep_stats[DAGPU_REPAIR_STATS] = {};
  uint64_t prof_n[DAGPU_PROFILE_KERNELS] = {};
  // Started Repairs (dagpu_repair_start / dagpu_repair_join): each runs its
  // host-driven crossword on a worker thread and a stream of its slot, forked
  // from the caller's stream; the join waits for the worker (all commands
  // queued) and makes a stream wait for the slot's `finished` event.
  static constexpr int kAsyncSlots = 64;
  // async_mu guards the slot table only: a join marks its slot `joining` under
  // the lock and waits for the worker without it, so starts and joins from
  // other host threads never queue behind one repair's crossword.
  struct AsyncSlot {
    bool busy = false;
    bool joining = false;
    uint32_t gen = 0;
    // written by the worker, read by the join after std::thread::join
    int rc = 0;
    std::string err;  // the worker's failure message (set_err on its own thread)
    int64_t stats[DAGPU_REPAIR_STATS] = {};
    hipStream_t stream = nullptr;
    hipEvent_t fork = nullptr, finished = nullptr;
    std::thread worker;
  };
  std::mutex async_mu;
  uint32_t async_gen = 0;
  AsyncSlot async_slot[kAsyncSlots];
};

constexpr size_t kSS = dagpu::kShareSize;

inline bool is_pow2(uint64_t v) { return v != 0 && (v & (v - 1)) == 0; }

// The calling thread's own last failure (errno-like), so that a thread that
// just failed reads its own message even while another thread fails on the
// same context.
struct ThreadErr {
  const dagpu_ctx* ctx = nullptr;
  uint64_t gen = 0;
  bool own = false;  // msg is this thread's own failure (not a snapshot)
  std::string msg;
};
inline ThreadErr& thread_err() {
  static thread_local ThreadErr t;
  return t;
}

inline int set_err(dagpu_ctx* c, int code, const std::string& msg) {
  if (!c) {  // context-free host calls (square construction): dagpu_last_error(NULL)
    ThreadErr& t = thread_err();
    t.ctx = nullptr;
    t.gen = 0;
    t.own = true;
    t.msg = msg;
    return code;
  }
  {
    std::lock_guard<std::mutex> g(c->err_mu);
    c->err = msg;
  }
  ThreadErr& t = thread_err();
  t.ctx = c;
  t.gen = c->gen;
  t.own = true;
  t.msg = msg;
  return code;
}

inline int hip_fail(dagpu_ctx* c, hipError_t e, const char* what) {
  char buf[256];
  snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
  return set_err(c, DAGPU_ERR_DEVICE, buf);
}

#define HIP_TRY(ctx, expr)                                   \
  do {                                                       \
    hipError_t e_ = (expr);                                  \
    if (e_ != hipSuccess) return hip_fail((ctx), e_, #expr); \
  } while (0)

inline uint64_t next_ctx_gen() {
  static std::atomic<uint64_t> g{0};
  return ++g;
}

// True on a started Repair's worker thread: it runs without the caller's
// ctx->mu, so it records no stage marks or profile brackets (their event
// state belongs to host-path calls under ctx->mu).
inline bool& on_repair_worker() {
  static thread_local bool w = false;
  return w;
}

// dagpu.cpp: timing-disabled events recycled per call, and the side streams
// paired with a caller stream (which: 0 normal, 1 the greatest priority).
namespace dagpu {
hipEvent_t ev_take(dagpu_ctx* c);
void ev_give(dagpu_ctx* c, hipEvent_t e);
hipStream_t side_stream(dagpu_ctx* ctx, hipStream_t s, int which = 0);
size_t pipe_slices(dagpu_ctx* ctx, uint32_t k, size_t n);
}  // namespace dagpu

inline hipEvent_t pool_get(dagpu_ctx* c) {
  if (!c->pool.empty()) {
    hipEvent_t e = c->pool.back();
    c->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

// Stage mark of a host-path call (see DAGPU_STAGE_* in dagpu.h).
inline void stage_mark(dagpu_ctx* c, int i, hipStream_t s) {
  if (!c->stages_on || !c->stage_ev[i] || on_repair_worker()) return;
  if (hipEventRecord(c->stage_ev[i], s) == hipSuccess) c->stage_mask |= 1u << i;
}

// RAII bracket: records events around one kernel launch when profiling is on.
struct ProfScope {
  dagpu_ctx* c;
  int id;
  hipStream_t s;
  hipEvent_t a = nullptr, b = nullptr;
  ProfScope(dagpu_ctx* c_, int id_, hipStream_t s_) : c(c_), id(id_), s(s_) {
    if (!c->prof || on_repair_worker()) return;
    std::lock_guard<std::mutex> g(c->prof_mu);
    a = pool_get(c);
    b = pool_get(c);
    (void)hipEventRecord(a, s);
  }
  ~ProfScope() {
    if (!a) return;
    (void)hipEventRecord(b, s);
    std::lock_guard<std::mutex> g(c->prof_mu);
    c->pending.push_back({id, a, b});
  }
};

inline int check_k(dagpu_ctx* ctx, uint64_t k) {
  if (!is_pow2(k)) return set_err(ctx, DAGPU_ERR_ARG, "square width must be a power of two");
  if (k > (uint64_t)kMaxK) {
    return set_err(ctx, DAGPU_ERR_UNSUPPORTED,
                   "square width k > " + std::to_string(kMaxK) + " is not supported on one GPU" +
                       (k <= (uint64_t)kMaxSplitK ? " (k = " + std::to_string(kMaxSplitK) +
                                                        ": the split square over >= 8 GPUs, dagpu_split_*)"
                                                  : ""));
  }
  return DAGPU_OK;
}

// codec width (dagpu_encode / dagpu_decode): one vector, not a square
inline int check_codec_k(dagpu_ctx* ctx, uint64_t k) {
  if (!is_pow2(k)) return set_err(ctx, DAGPU_ERR_ARG, "codec width must be a power of two");
  if (k > (uint64_t)kMaxCodecK) {
    return set_err(ctx, DAGPU_ERR_UNSUPPORTED,
                   "codec width k > " + std::to_string(kMaxCodecK) + " is not supported (Leopard: 65536 shards)");
  }
  return DAGPU_OK;
}
