// dagpu.cpp -- C-ABI host runtime for the MI355X DA hot path (include/dagpu.h).
//
// Mirrors the reference entry points:
//   da.ExtendShares            pkg/da/data_availability_header.go:65-75
//   da.NewDataAvailabilityHeader / Hash   :44-63, :92-108
//   rsmt2d.ComputeExtendedDataSquare (3k Encode calls) via the Leopard codec
//   appconsts.DefaultCodec     pkg/appconsts/global_consts.go:92
// The pipeline per batch of same-k squares (all on one HIP stream):
//   row encode Q0 -> Q1 (+ Q0 placement)  |  column encode [Q0|Q1] -> [Q2|Q3]
//   leaf digests (each cell once)  |  row+col NMT trees  |  DAH
// The EDS never leaves HBM unless the caller asks for it.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/dagpu.h"
#include "host_sha256.hpp"
#include "kernels.hpp"
#include "runtime.hpp"

using namespace dagpu;

namespace {

size_t eds_bytes(uint64_t k) { return 4ull * k * k * kSS; }
size_t ods_bytes(uint64_t k) { return 1ull * k * k * kSS; }

// RS extension of n squares (uniform k), device pointers.
// ev_rows (optional) is recorded between the row and the column pass: rows
// 0..k-1 of every EDS ([Q0|Q1]) are final from that point on.
int enqueue_rs(dagpu_ctx* ctx, uint32_t k, size_t n, const uint8_t* d_ods, uint8_t* d_eds,
               hipStream_t s, hipEvent_t ev_rows = nullptr) {
  const long w = 2L * k;
  const long esq = (long)eds_bytes(k);
  EncodeArgs ra{};
  // Row pass: vector r = row r of Q0 -> Q1 (and copy Q0 into place).
  if (d_ods) {
    ra.in = d_ods;
    ra.in_sq_stride = (long)ods_bytes(k);
    ra.in_vec_stride = (long)k * kSS;
    ra.in_shard_stride = kSS;
    ra.copy = d_eds;
    ra.copy_sq_stride = esq;
    ra.copy_vec_stride = w * kSS;
    ra.copy_shard_stride = kSS;
  } else {
    ra.in = d_eds;
    ra.in_sq_stride = esq;
    ra.in_vec_stride = w * kSS;
    ra.in_shard_stride = kSS;
    ra.copy = nullptr;
  }
  ra.out = d_eds + (long)k * kSS;
  ra.out_sq_stride = esq;
  ra.out_vec_stride = w * kSS;
  ra.out_shard_stride = kSS;
  ra.nsq = (long)n;
  ra.nvec = k;
  ra.nchunk = 1;
  ra.shard_bytes = kSS;
  {
    ProfScope p(ctx, 0, s);
    HIP_TRY(ctx, launch_rs_encode((int)k, ra, s));
  }
  stage_mark(ctx, DAGPU_STAGE_ROWS, s);
  if (ev_rows) HIP_TRY(ctx, hipEventRecord(ev_rows, s));
  // Column pass: vector c = column c of [Q0|Q1] -> [Q2|Q3].
  EncodeArgs ca{};
  ca.in = d_eds;
  ca.in_sq_stride = esq;
  ca.in_vec_stride = kSS;
  ca.in_shard_stride = w * kSS;
  ca.out = d_eds + (long)k * w * kSS;
  ca.out_sq_stride = esq;
  ca.out_vec_stride = kSS;
  ca.out_shard_stride = w * kSS;
  ca.copy = nullptr;
  ca.nsq = (long)n;
  ca.nvec = w;
  ca.nchunk = 1;
  ca.shard_bytes = kSS;
  {
    ProfScope p(ctx, 1, s);
    HIP_TRY(ctx, launch_rs_encode((int)k, ca, s));
  }
  stage_mark(ctx, DAGPU_STAGE_COLS, s);
  return DAGPU_OK;
}

// d_dah = NULL: roots only (Repair's verification needs no DAH)
int enqueue_roots(dagpu_ctx* ctx, uint32_t k, size_t n, const uint8_t* d_eds, uint8_t* d_rr,
                  uint8_t* d_cr, uint8_t* d_dah, int32_t* d_status, void* d_ws, hipStream_t s) {
  SquareArgs sa{};
  sa.eds = d_eds;
  sa.eds_sq_stride = (long)eds_bytes(k);
  sa.k = (int)k;
  sa.nsq = (long)n;
  nmt_workspace_carve(sa, d_ws);
  sa.row_roots = d_rr;
  sa.col_roots = d_cr;
  sa.dah = d_dah;
  sa.status = d_status;
  sa.k = (int)k;
  sa.nsq = (long)n;
  HIP_TRY(ctx, hipMemsetAsync(d_status, 0, n * sizeof(int32_t), s));
  {
    ProfScope p(ctx, 2, s);
    HIP_TRY(ctx, launch_nmt_leaves(sa, s));
  }
  stage_mark(ctx, DAGPU_STAGE_LEAVES, s);
  {
    ProfScope p(ctx, 3, s);
    HIP_TRY(ctx, launch_nmt_trees(sa, s));
  }
  stage_mark(ctx, DAGPU_STAGE_TREES, s);
  if (d_dah) {
    ProfScope p(ctx, 4, s);
    HIP_TRY(ctx, launch_dah(sa, s));
  }
  stage_mark(ctx, DAGPU_STAGE_DAH, s);
  return DAGPU_OK;
}

// Squares per pipeline chunk: about 128 MiB of ODS per host->device copy.
// DAGPU_PIPELINE_CHUNK (squares) overrides it, e.g. to exercise many chunks in tests.
size_t pipeline_chunk(uint32_t k, size_t n) {
  size_t m = (size_t(128) << 20) / ods_bytes(k);
  const long v = sw_long(SW_PIPELINE_CHUNK);
  if (v > 0) m = (size_t)v;
  return m < 1 ? 1 : (m > n ? n : m);
}

int finish_status(dagpu_ctx* ctx, const int32_t* st, size_t n, int32_t* status) {
  int first = DAGPU_OK;
  for (size_t i = 0; i < n; i++) {
    int v = (st[i] & kStatusPushOrder) ? DAGPU_ERR_PUSH_ORDER : DAGPU_OK;
    if (status) status[i] = v;
    if (v && !first) first = v;
  }
  if (first) set_err(ctx, first, "invalid push order: namespaces of original data square are not sorted");
  return first;
}

// Host-mode batch of >= 2 chunks: chunk c's ODS goes up on copy_stream while
// chunk c-1 is extended on ctx->stream; roots, DAHs and status come back into
// page-locked staging per slot and are copied to the caller's arrays once the
// slot's event fires (the caller's buffers may be pageable Go memory, whose
// device->host copies would otherwise block this thread and the pipeline).
// An EDS requested back is copied straight into eds_out.  Caller holds ctx->mu.
int run_group_pipelined(dagpu_ctx* ctx, uint32_t k, size_t n, size_t m, const uint8_t* ods,
                        uint8_t* eds_out, uint8_t* rr, uint8_t* cr, uint8_t* dah, int32_t* status) {
  const size_t w = 2 * (size_t)k;
  const size_t rb = w * kNodeSize, ob = ods_bytes(k), eb = eds_bytes(k);
  const size_t wsb = dagpu_workspace_size(k, m);
  hipStream_t s = ctx->stream, cs = ctx->copy_stream;
  HIP_TRY(ctx, ctx->ods.ensure(2 * m * ob));
  HIP_TRY(ctx, ctx->eds.ensure(2 * m * eb));
  HIP_TRY(ctx, ctx->rr.ensure(2 * m * rb));
  HIP_TRY(ctx, ctx->cr.ensure(2 * m * rb));
  HIP_TRY(ctx, ctx->dah.ensure(2 * m * 32));
  HIP_TRY(ctx, ctx->status.ensure(2 * m * sizeof(int32_t)));
  HIP_TRY(ctx, ctx->ws.ensure(2 * wsb));
  const size_t hslot = m * (2 * rb + 32 + sizeof(int32_t));
  HIP_TRY(ctx, ctx->h_out.ensure(2 * hslot));
  std::vector<int32_t> st(n);
  const size_t nchunks = (n + m - 1) / m;
  auto slot_dev = [&](DevBuf& b, size_t per, int slot) { return (uint8_t*)b.p + slot * m * per; };
  auto slot_host = [&](int slot) { return (uint8_t*)ctx->h_out.p + slot * hslot; };
  // copy chunk c's outputs from its slot's staging to the caller (slot's event done)
  auto drain = [&](size_t c) -> int {
    const int slot = (int)(c & 1);
    const size_t off = c * m, cnt = (n - off < m) ? n - off : m;
    HIP_TRY(ctx, hipEventSynchronize(ctx->ev_done[slot]));
    const uint8_t* h = slot_host(slot);
    memcpy(rr + off * rb, h, cnt * rb);
    memcpy(cr + off * rb, h + m * rb, cnt * rb);
    memcpy(dah + off * 32, h + 2 * m * rb, cnt * 32);
    memcpy(st.data() + off, h + 2 * m * rb + m * 32, cnt * sizeof(int32_t));
    return DAGPU_OK;
  };
  for (size_t c = 0; c < nchunks; c++) {
    const int slot = (int)(c & 1);
    const size_t off = c * m, cnt = (n - off < m) ? n - off : m;
    if (c >= 2) {  // the slot's previous chunk must be drained before reuse
      int rc = drain(c - 2);
      if (rc) return rc;
      HIP_TRY(ctx, hipStreamWaitEvent(cs, ctx->ev_done[slot], 0));
    }
    uint8_t* d_ods = slot_dev(ctx->ods, ob, slot);
    uint8_t* d_eds = slot_dev(ctx->eds, eb, slot);
    uint8_t* d_rr = slot_dev(ctx->rr, rb, slot);
    uint8_t* d_cr = slot_dev(ctx->cr, rb, slot);
    uint8_t* d_dah = slot_dev(ctx->dah, 32, slot);
    int32_t* d_st = (int32_t*)slot_dev(ctx->status, sizeof(int32_t), slot);
    HIP_TRY(ctx, hipMemcpyAsync(d_ods, ods + off * ob, cnt * ob, hipMemcpyHostToDevice, cs));
    HIP_TRY(ctx, hipEventRecord(ctx->ev_loaded[slot], cs));
    HIP_TRY(ctx, hipStreamWaitEvent(s, ctx->ev_loaded[slot], 0));
    int rc = enqueue_rs(ctx, k, cnt, d_ods, d_eds, s);
    if (rc) return rc;
    rc = enqueue_roots(ctx, k, cnt, d_eds, d_rr, d_cr, d_dah, d_st, (uint8_t*)ctx->ws.p + slot * wsb, s);
    if (rc) return rc;
    if (eds_out)
      HIP_TRY(ctx, hipMemcpyAsync(eds_out + off * eb, d_eds, cnt * eb, hipMemcpyDeviceToHost, s));
    uint8_t* h = slot_host(slot);
    HIP_TRY(ctx, hipMemcpyAsync(h, d_rr, cnt * rb, hipMemcpyDeviceToHost, s));
    HIP_TRY(ctx, hipMemcpyAsync(h + m * rb, d_cr, cnt * rb, hipMemcpyDeviceToHost, s));
    HIP_TRY(ctx, hipMemcpyAsync(h + 2 * m * rb, d_dah, cnt * 32, hipMemcpyDeviceToHost, s));
    HIP_TRY(ctx, hipMemcpyAsync(h + 2 * m * rb + m * 32, d_st, cnt * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(ctx, hipEventRecord(ctx->ev_done[slot], s));
  }
  for (size_t c = nchunks >= 2 ? nchunks - 2 : 0; c < nchunks; c++) {
    int rc = drain(c);
    if (rc) return rc;
  }
  return finish_status(ctx, st.data(), n, status);
}

// Roots, DAHs and status of a host-path call share one device buffer
// (ctx->res: rr | cr | dah | status) and come back in ONE copy to page-locked
// staging, then go to the caller's (possibly pageable) arrays by memcpy: four
// small device->host copies cost ~20 us each on the single-square latency path
// (profiles/single_square_r02.log).  Caller holds ctx->mu.
struct HostResults {
  size_t n = 0, rb = 0, bytes = 0;
  uint8_t *rr = nullptr, *cr = nullptr, *dah = nullptr;
  int32_t* st = nullptr;
  hipError_t alloc(dagpu_ctx* ctx, uint32_t k, size_t cnt) {
    n = cnt;
    rb = 2 * (size_t)k * kNodeSize * n;
    bytes = 2 * rb + 32 * n + sizeof(int32_t) * n;
    hipError_t e = ctx->res.ensure(bytes);
    if (e == hipSuccess) e = ctx->h_out.ensure(bytes);
    if (e != hipSuccess) return e;
    rr = (uint8_t*)ctx->res.p;
    cr = rr + rb;
    dah = cr + rb;
    st = (int32_t*)(dah + 32 * n);  // rb = 180 k n: 4-byte aligned
    return hipSuccess;
  }
  hipError_t download(dagpu_ctx* ctx, hipStream_t s) const {
    return hipMemcpyAsync(ctx->h_out.p, ctx->res.p, bytes, hipMemcpyDeviceToHost, s);
  }
  // after the stream has synchronised
  void deliver(const dagpu_ctx* ctx, uint8_t* o_rr, uint8_t* o_cr, uint8_t* o_dah, int32_t* o_st) const {
    const uint8_t* h = (const uint8_t*)ctx->h_out.p;
    memcpy(o_rr, h, rb);
    memcpy(o_cr, h + rb, rb);
    memcpy(o_dah, h + 2 * rb, 32 * n);
    memcpy(o_st, h + 2 * rb + 32 * n, sizeof(int32_t) * n);
  }
};

// hipHostMalloc / hipHostRegister memory: device->host copies into it are
// asynchronous DMA.  Into pageable memory they run synchronously on this thread.
bool host_pinned(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// Completion wait of a host-path call.  Calls that finish in about a
// millisecond (single squares, the production callers' shape) spin on the
// stream: the blocking wait's wake-up added up to 0.25 ms to single-square
// calls (bench.py single_square stages, r03).
hipError_t wait_stream(hipStream_t s, bool spin) {
  if (!spin) return hipStreamSynchronize(s);
  hipError_t e;
  while ((e = hipStreamQuery(s)) == hipErrorNotReady) __builtin_ia32_pause();
  return e;
}

// Runs one uniform-k group from host memory.  Caller holds ctx->mu.
int run_group_host(dagpu_ctx* ctx, uint32_t k, size_t n, const uint8_t* ods, uint8_t* eds_out,
                   uint8_t* rr, uint8_t* cr, uint8_t* dah, int32_t* status) {
  int rc = check_k(ctx, k);
  if (rc) return rc;
  const size_t m = pipeline_chunk(k, n);
  if (n > m) return run_group_pipelined(ctx, k, n, m, ods, eds_out, rr, cr, dah, status);
  hipStream_t s = ctx->stream, cs = ctx->copy_stream;
  const bool spin = eds_bytes(k) * n <= (size_t(64) << 20);
  HostResults res;
  HIP_TRY(ctx, ctx->ods.ensure(ods_bytes(k) * n));
  HIP_TRY(ctx, ctx->eds.ensure(eds_bytes(k) * n));
  HIP_TRY(ctx, res.alloc(ctx, k, n));
  HIP_TRY(ctx, ctx->ws.ensure(dagpu_workspace_size(k, n)));
  ctx->stage_mask = 0;
  stage_mark(ctx, DAGPU_STAGE_START, s);
  HIP_TRY(ctx, hipMemcpyAsync(ctx->ods.p, ods, ods_bytes(k) * n, hipMemcpyHostToDevice, s));
  stage_mark(ctx, DAGPU_STAGE_UPLOADED, s);
  // An EDS requested back goes down on the copy stream while the kernels run:
  // the top halves ([Q0|Q1], final after the row pass) during the column pass
  // and the NMT kernels, the bottom halves ([Q2|Q3]) during the NMT kernels.
  // Into page-locked memory the copies are queued right after the RS passes,
  // so the DMA starts as soon as the rows are final.  Into pageable memory a
  // device->host copy runs synchronously on this thread, so there the whole
  // kernel chain and the results download are queued first.
  rc = enqueue_rs(ctx, k, n, (const uint8_t*)ctx->ods.p, (uint8_t*)ctx->eds.p, s,
                  eds_out ? ctx->ev_loaded[0] : nullptr);
  if (rc) return rc;
  if (eds_out) HIP_TRY(ctx, hipEventRecord(ctx->ev_loaded[1], s));
  // from the first EDS copy on, DMA may be writing into eds_out: every return
  // path waits for the copy stream
  struct CopyJoin {
    hipStream_t cs;
    bool armed = false;
    ~CopyJoin() {
      if (armed) (void)hipStreamSynchronize(cs);
    }
  } join{cs};
  auto eds_copies = [&]() -> int {
    join.armed = true;
    const size_t eb = eds_bytes(k), half = eb / 2;
    HIP_TRY(ctx, hipStreamWaitEvent(cs, ctx->ev_loaded[0], 0));
    const uint8_t* d = (const uint8_t*)ctx->eds.p;
    for (size_t i = 0; i < n; i++)  // plain 1D copies: the DMA engines' fast path
      HIP_TRY(ctx, hipMemcpyAsync(eds_out + i * eb, d + i * eb, half, hipMemcpyDeviceToHost, cs));
    stage_mark(ctx, DAGPU_STAGE_EDS_TOP, cs);
    HIP_TRY(ctx, hipStreamWaitEvent(cs, ctx->ev_loaded[1], 0));
    for (size_t i = 0; i < n; i++)
      HIP_TRY(ctx, hipMemcpyAsync(eds_out + i * eb + half, d + i * eb + half, half,
                                  hipMemcpyDeviceToHost, cs));
    stage_mark(ctx, DAGPU_STAGE_EDS_BOTTOM, cs);
    return DAGPU_OK;
  };
  const bool early = eds_out && host_pinned(eds_out);
  if (early && (rc = eds_copies())) return rc;
  rc = enqueue_roots(ctx, k, n, (const uint8_t*)ctx->eds.p, res.rr, res.cr, res.dah, res.st, ctx->ws.p, s);
  if (rc) return rc;
  HIP_TRY(ctx, res.download(ctx, s));
  stage_mark(ctx, DAGPU_STAGE_RESULTS, s);
  if (eds_out && !early && (rc = eds_copies())) return rc;
  if (eds_out) {
    HIP_TRY(ctx, wait_stream(cs, spin));
    join.armed = false;
  }
  HIP_TRY(ctx, wait_stream(s, spin));
  std::vector<int32_t> st(n);
  res.deliver(ctx, rr, cr, dah, st.data());
  return finish_status(ctx, st.data(), n, status);
}

}  // namespace

extern "C" {

int dagpu_version(void) { return 100; }

uint32_t dagpu_max_square_width(void) {
  static_assert(DAGPU_MAX_SQUARE_WIDTH == kMaxK, "header and kernels disagree on the widest square");
  return (uint32_t)kMaxK;
}

uint32_t dagpu_max_codec_width(void) {
  static_assert(DAGPU_MAX_CODEC_WIDTH == kMaxCodecK, "header and kernels disagree on the widest codec vector");
  return (uint32_t)kMaxCodecK;
}

int dagpu_init(int device, dagpu_ctx** out) {
  if (!out) return DAGPU_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return DAGPU_ERR_DEVICE;
  if (device < 0 || device >= ndev) return DAGPU_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return DAGPU_ERR_DEVICE;
  dagpu_ctx* c = new dagpu_ctx();
  c->device = device;
  c->gen = next_ctx_gen();
  bool ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) == hipSuccess;
  for (int i = 0; ok && i < 2; i++)
    ok = hipEventCreateWithFlags(&c->ev_loaded[i], hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&c->ev_done[i], hipEventDisableTiming) == hipSuccess;
  for (int i = 0; ok && i < dagpu_ctx::kStages; i++) ok = hipEventCreate(&c->stage_ev[i]) == hipSuccess;
  if (!ok) {
    dagpu_destroy(c);
    return DAGPU_ERR_DEVICE;
  }
  *out = c;
  return DAGPU_OK;
}

void dagpu_destroy(dagpu_ctx* c) {
  if (!c) return;
  if (thread_err().ctx == c && thread_err().gen == c->gen) thread_err() = ThreadErr{};
  (void)hipSetDevice(c->device);
  for (auto& sl : c->async_slot) {  // started Repairs finish first
    if (sl.worker.joinable()) sl.worker.join();
    if (sl.stream) (void)hipStreamSynchronize(sl.stream);
  }
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
  c->h_out.release();
  c->res.release();
  c->ods.release(); c->eds.release(); c->rr.release(); c->cr.release();
  c->dah.release(); c->status.release(); c->ws.release();
  for (DevBuf* b : {&c->t_leaf_data, &c->t_leaves, &c->t_inner, &c->t_meta, &c->t_out, &c->t_status, &c->t_flags})
    b->release();
  for (auto& r : c->pending) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
  for (auto e : c->pool) (void)hipEventDestroy(e);
  for (int i = 0; i < 2; i++) {
    if (c->ev_loaded[i]) (void)hipEventDestroy(c->ev_loaded[i]);
    if (c->ev_done[i]) (void)hipEventDestroy(c->ev_done[i]);
  }
  for (auto e : c->stage_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& cs : c->side)
    for (hipStream_t x : {cs.rs, cs.rs_hi})
      if (x) (void)hipStreamSynchronize(x);
  for (auto e : c->ev_pool) (void)hipEventDestroy(e);
  for (void* m : c->mailboxes) (void)hipHostFree(m);
  for (auto& cs : c->side)
    for (hipStream_t x : {cs.rs, cs.rs_hi})
      if (x) (void)hipStreamDestroy(x);
  for (auto& sl : c->async_slot) {
    if (sl.fork) (void)hipEventDestroy(sl.fork);
    if (sl.finished) (void)hipEventDestroy(sl.finished);
    if (sl.stream) (void)hipStreamDestroy(sl.stream);
  }
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

void* dagpu_host_alloc(size_t bytes) {
  void* p = nullptr;
  return hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) == hipSuccess ? p : nullptr;
}

void dagpu_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

int dagpu_host_register(void* p, size_t bytes) {
  if (!p || !bytes) return DAGPU_ERR_ARG;
  return hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess ? DAGPU_OK : DAGPU_ERR_DEVICE;
}

int dagpu_host_unregister(void* p) {
  if (!p) return DAGPU_ERR_ARG;
  return hipHostUnregister(p) == hipSuccess ? DAGPU_OK : DAGPU_ERR_DEVICE;
}

// The message of this thread's last failure on `c`; if this thread has not
// failed on `c`, a snapshot of the context's most recent message.  The pointer
// stays valid until this thread's next call into the library.
const char* dagpu_last_error(dagpu_ctx* c) {
  ThreadErr& t = thread_err();
  if (!c) return t.ctx == nullptr && t.own ? t.msg.c_str() : "null context";
  if (t.ctx == c && t.gen == c->gen && t.own) return t.msg.c_str();
  std::lock_guard<std::mutex> g(c->err_mu);
  t.ctx = c;
  t.gen = c->gen;
  t.own = false;
  t.msg = c->err;
  return t.msg.c_str();
}

size_t dagpu_workspace_size(uint32_t k, size_t n) {
  if (k == 0 || n == 0) return 256;
  return nmt_workspace_bytes((int)k, (long)n) + 256;
}

int dagpu_extend_shares(dagpu_ctx* ctx, const uint8_t* shares, size_t n_shares,
                        size_t share_size, uint8_t* eds_out, uint8_t* row_roots,
                        uint8_t* col_roots, uint8_t* dah) {
  if (!ctx || !row_roots || !col_roots || !dah) return DAGPU_ERR_ARG;
  std::lock_guard<std::mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  // pkg/da/data_availability_header.go:67-69
  if (!is_pow2(n_shares)) {
    return set_err(ctx, DAGPU_ERR_NOT_POW2,
                   "number of shares is not a power of 2: got " + std::to_string(n_shares));
  }
  // SquareSize (:205-207) then rsmt2d newDataSquare's square check
  const uint64_t k = (uint64_t)std::llround(std::ceil(std::sqrt((double)n_shares)));
  if (k * k != n_shares) return set_err(ctx, DAGPU_ERR_NOT_SQUARE, "number of chunks must be a square number");
  if (share_size != kSS) {
    return set_err(ctx, DAGPU_ERR_SHARE_SIZE,
                   "share size must be " + std::to_string(kSS) + " bytes (appconsts.ShareSize)");
  }
  if (!shares) return DAGPU_ERR_ARG;
  int32_t st = 0;
  return run_group_host(ctx, (uint32_t)k, 1, shares, eds_out, row_roots, col_roots, dah, &st);
}

int dagpu_extend_batch(dagpu_ctx* ctx, const uint8_t* ods, const uint32_t* k, size_t n,
                       uint8_t* eds_or_null, uint8_t* row_roots, uint8_t* col_roots,
                       uint8_t* dah, int32_t* status) {
  if (!ctx || (n && (!ods || !k || !row_roots || !col_roots || !dah))) return DAGPU_ERR_ARG;
  std::lock_guard<std::mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  // per-square offsets in the packed arrays
  std::vector<size_t> o_ods(n), o_eds(n), o_root(n);
  size_t a = 0, b = 0, c = 0;
  for (size_t i = 0; i < n; i++) {
    int rc = check_k(ctx, k[i]);
    if (rc) {
      if (status) status[i] = rc;
      return rc;
    }
    o_ods[i] = a; o_eds[i] = b; o_root[i] = c;
    a += ods_bytes(k[i]); b += eds_bytes(k[i]); c += 2ull * k[i] * kNodeSize;
  }
  // group consecutive runs of equal k (block replay batches are mostly uniform)
  int first = DAGPU_OK;
  size_t i = 0;
  std::vector<int32_t> st;
  while (i < n) {
    size_t j = i;
    while (j < n && k[j] == k[i]) j++;
    st.assign(j - i, 0);
    int rc = run_group_host(ctx, k[i], j - i, ods + o_ods[i],
                            eds_or_null ? eds_or_null + o_eds[i] : nullptr,
                            row_roots + o_root[i], col_roots + o_root[i], dah + 32 * i, st.data());
    if (rc && rc != DAGPU_ERR_PUSH_ORDER) return rc;
    for (size_t t = i; t < j; t++) {
      if (status) status[t] = st[t - i];
      if (st[t - i] && !first) first = st[t - i];
    }
    i = j;
  }
  return first;
}

int dagpu_extend_rs_device(dagpu_ctx* ctx, uint32_t k, size_t n, const uint8_t* d_ods,
                           uint8_t* d_eds, void* stream) {
  if (!ctx || !d_eds) return DAGPU_ERR_ARG;
  int rc = check_k(ctx, k);
  if (rc) return rc;
  return enqueue_rs(ctx, k, n, d_ods, d_eds, (hipStream_t)stream);
}

int dagpu_roots_device(dagpu_ctx* ctx, uint32_t k, size_t n, const uint8_t* d_eds,
                       uint8_t* d_row_roots, uint8_t* d_col_roots, uint8_t* d_dah,
                       int32_t* d_status, void* d_workspace, void* stream) {
  if (!ctx || !d_eds || !d_row_roots || !d_col_roots || !d_dah || !d_status || !d_workspace)
    return DAGPU_ERR_ARG;
  int rc = check_k(ctx, k);
  if (rc) return rc;
  return enqueue_roots(ctx, k, n, d_eds, d_row_roots, d_col_roots, d_dah, d_status, d_workspace,
                       (hipStream_t)stream);
}

extern "C++" {  // external C++ helpers (runtime.hpp): split.cpp forks onto the side streams too
namespace dagpu {

// ---- switches (switches.hpp) ----
namespace {
const char* const kSwNames[SW_COUNT] = {
    "DAGPU_PIPELINE_CHUNK", "DAGPU_PIPE_SLICES", "DAGPU_REPAIR_FILL", "DAGPU_SPLIT_SQUARE", "DAGPU_SPLIT_OVERLAP",
    "DAGPU_DAH_SPLIT",      "DAGPU_DEC_SLICED",  "DAGPU_ENC_SLICED",  "DAGPU_ENC_SLICED2",  "DAGPU_GF16_WIDE"};
thread_local const SwSnapshot* tl_sw = nullptr;
}  // namespace

const char* sw(Switch s) {
  if (s < 0 || s >= SW_COUNT) return nullptr;
  if (tl_sw) return tl_sw->set[s] ? tl_sw->v[s] : nullptr;
  return getenv(kSwNames[s]);
}

long sw_long(Switch s, long dflt) {
  const char* e = sw(s);
  return e ? atol(e) : dflt;
}

void sw_snapshot(SwSnapshot* out) {
  for (int i = 0; i < SW_COUNT; i++) {
    const char* e = getenv(kSwNames[i]);
    out->set[i] = e != nullptr;
    out->v[i][0] = 0;
    if (e) snprintf(out->v[i], sizeof out->v[i], "%s", e);
  }
}

void sw_bind(const SwSnapshot* snap) { tl_sw = snap; }

hipEvent_t ev_take(dagpu_ctx* c) {
  std::lock_guard<std::mutex> g(c->ev_mu);
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  return e;
}

void ev_give(dagpu_ctx* c, hipEvent_t e) {
  if (!e) return;
  std::lock_guard<std::mutex> g(c->ev_mu);
  c->ev_pool.push_back(e);
}

// Slices of a device batch for the RS/NMT pipeline: RS of slice i+1.. runs on
// a side stream while the NMT kernels of slice i run on the caller's stream
// (bench: 256 squares at k = 128, 4 slices 11.98 -> 11.63 ms; tools/pipe_exp.py).
// DAGPU_PIPE_SLICES overrides (1 = off; read per call, so tests can vary it).
// Off while profiling, so that every kernel's event bracket times that kernel alone.
size_t pipe_slices(dagpu_ctx* ctx, uint32_t k, size_t n) {
  const long env = sw_long(SW_PIPE_SLICES);
  if (ctx->prof) return 1;
  size_t s = env > 0 ? (size_t)env : (k >= 128 && n >= 64 ? 4 : 1);
  while (s > 1 && n / s < 8) s >>= 1;
  return s < 1 ? 1 : s;
}

// The side streams paired with caller stream `s` (created on first use).
// which: 0 = normal priority, 1 = the device's greatest stream priority.
hipStream_t side_stream(dagpu_ctx* ctx, hipStream_t s, int which) {
  std::lock_guard<std::mutex> g(ctx->side_mu);
  dagpu_ctx::Side* sd = nullptr;
  for (auto& p : ctx->side)
    if (p.caller == s) sd = &p;
  if (!sd) {
    if (ctx->side.size() >= dagpu_ctx::kMaxSideStreams) {
      // more caller streams than side streams: share them round-robin (the
      // callers then serialise their side work, results are unaffected)
      const size_t i = (size_t)((((uint64_t)(uintptr_t)s) * 0x9E3779B97F4A7C15ull) >> 32) % ctx->side.size();
      sd = &ctx->side[i];
    } else {
      ctx->side.emplace_back();
      sd = &ctx->side.back();
      sd->caller = s;
    }
  }
  hipStream_t* slot = which == 1 ? &sd->rs_hi : &sd->rs;
  if (!*slot) {
    hipError_t e;
    if (which == 1) {
      int lo = 0, hi = 0;
      (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
      e = hipStreamCreateWithPriority(slot, hipStreamNonBlocking, hi);
    } else {
      e = hipStreamCreateWithFlags(slot, hipStreamNonBlocking);
    }
    if (e != hipSuccess) {
      *slot = nullptr;
      return nullptr;
    }
  }
  return *slot;
}

}  // namespace dagpu
}  // extern "C++"

int dagpu_extend_batch_device(dagpu_ctx* ctx, uint32_t k, size_t n, const uint8_t* d_ods,
                              uint8_t* d_eds, uint8_t* d_row_roots, uint8_t* d_col_roots,
                              uint8_t* d_dah, int32_t* d_status, void* d_workspace,
                              void* stream) {
  if (!ctx || !d_eds || !d_row_roots || !d_col_roots || !d_dah || !d_status || !d_workspace)
    return DAGPU_ERR_ARG;
  int rc = check_k(ctx, k);
  if (rc) return rc;
  const size_t S = pipe_slices(ctx, k, n);
  hipStream_t s = (hipStream_t)stream;
  if (S <= 1) {
    rc = enqueue_rs(ctx, k, n, d_ods, d_eds, s);
    if (rc) return rc;
    return enqueue_roots(ctx, k, n, d_eds, d_row_roots, d_col_roots, d_dah, d_status, d_workspace, s);
  }
  // fork: the side stream starts after the work already queued on the caller's stream
  std::vector<hipEvent_t> ev(S + 1, nullptr);
  for (auto& e : ev)
    if (!(e = ev_take(ctx))) {
      for (auto x : ev) ev_give(ctx, x);
      return set_err(ctx, DAGPU_ERR_DEVICE, "hipEventCreate failed");
    }
  auto done = [&](int r) {
    for (auto x : ev) ev_give(ctx, x);
    return r;
  };
  hipStream_t rs = side_stream(ctx, s, 0);
  if (!rs) return done(set_err(ctx, DAGPU_ERR_DEVICE, "hipStreamCreate failed"));
  const size_t w = 2 * (size_t)k;
  if (hipEventRecord(ev[S], s) != hipSuccess || hipStreamWaitEvent(rs, ev[S], 0) != hipSuccess)
    return done(set_err(ctx, DAGPU_ERR_DEVICE, "pipeline fork failed"));
  // equal slices (tried and dropped, profiles/pipeline_r02.log, pipe_streams_r03.log:
  // a smaller first slice, a high-priority RS stream, a second NMT stream)
  std::vector<size_t> cut(S + 1);
  for (size_t i = 0; i <= S; i++) cut[i] = n * i / S;
  for (size_t i = 0; i < S; i++) {
    const size_t a = cut[i], b = cut[i + 1];
    rc = enqueue_rs(ctx, k, b - a, d_ods ? d_ods + a * ods_bytes(k) : nullptr, d_eds + a * eds_bytes(k), rs);
    if (rc) return done(rc);
    if (hipEventRecord(ev[i], rs) != hipSuccess) return done(set_err(ctx, DAGPU_ERR_DEVICE, "hipEventRecord failed"));
  }
  // NMT work of the slices: in order on the caller's stream, sharing the front
  // of the workspace; waiting on the last slice's event joins the RS stream
  for (size_t i = 0; i < S; i++) {
    const size_t a = cut[i], b = cut[i + 1];
    if (hipStreamWaitEvent(s, ev[i], 0) != hipSuccess)
      return done(set_err(ctx, DAGPU_ERR_DEVICE, "hipStreamWaitEvent failed"));
    rc = enqueue_roots(ctx, k, b - a, d_eds + a * eds_bytes(k), d_row_roots + a * w * kNodeSize,
                       d_col_roots + a * w * kNodeSize, d_dah + a * 32, d_status + a, (uint8_t*)d_workspace, s);
    if (rc) return done(rc);
  }
  return done(DAGPU_OK);
}

int dagpu_roots(dagpu_ctx* ctx, uint32_t k, const uint8_t* eds, uint8_t* row_roots,
                uint8_t* col_roots, uint8_t* dah) {
  if (!ctx || !eds || !row_roots || !col_roots || !dah) return DAGPU_ERR_ARG;
  std::lock_guard<std::mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  int rc = check_k(ctx, k);
  if (rc) return rc;
  hipStream_t s = ctx->stream;
  HostResults res;
  HIP_TRY(ctx, ctx->eds.ensure(eds_bytes(k)));
  HIP_TRY(ctx, res.alloc(ctx, k, 1));
  HIP_TRY(ctx, ctx->ws.ensure(dagpu_workspace_size(k, 1)));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->eds.p, eds, eds_bytes(k), hipMemcpyHostToDevice, s));
  rc = enqueue_roots(ctx, k, 1, (const uint8_t*)ctx->eds.p, res.rr, res.cr, res.dah, res.st, ctx->ws.p, s);
  if (rc) return rc;
  HIP_TRY(ctx, res.download(ctx, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  int32_t st = 0;
  res.deliver(ctx, row_roots, col_roots, dah, &st);
  if (st & kStatusPushOrder)
    return set_err(ctx, DAGPU_ERR_PUSH_ORDER, "invalid push order: namespaces of original data square are not sorted");
  return DAGPU_OK;
}

int dagpu_encode(dagpu_ctx* ctx, uint32_t k, size_t nvec, size_t shard_size,
                 const uint8_t* data, uint8_t* parity) {
  if (!ctx || (nvec && (!data || !parity))) return DAGPU_ERR_ARG;
  if (shard_size == 0 || shard_size % 64)
    return set_err(ctx, DAGPU_ERR_SHARE_SIZE, "shard size must be a multiple of 64");
  std::lock_guard<std::mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  int rc = check_codec_k(ctx, k);
  if (rc) return rc;
  if (nvec == 0) return DAGPU_OK;
  const size_t bytes = (size_t)k * shard_size * nvec;
  hipStream_t s = ctx->stream;
  HIP_TRY(ctx, ctx->ods.ensure(bytes));
  HIP_TRY(ctx, ctx->eds.ensure(bytes));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->ods.p, data, bytes, hipMemcpyHostToDevice, s));
  EncodeArgs ea{};
  ea.in = (const uint8_t*)ctx->ods.p;
  ea.out = (uint8_t*)ctx->eds.p;
  ea.copy = nullptr;
  ea.in_sq_stride = 0;
  ea.out_sq_stride = 0;
  ea.in_vec_stride = (long)k * (long)shard_size;
  ea.out_vec_stride = (long)k * (long)shard_size;
  ea.in_shard_stride = (long)shard_size;
  ea.out_shard_stride = (long)shard_size;
  ea.nsq = 1;
  ea.nvec = (long)nvec;
  ea.nchunk = (long)((shard_size + 511) / 512);
  ea.shard_bytes = (long)shard_size;
  HIP_TRY(ctx, launch_rs_encode((int)k, ea, s));
  HIP_TRY(ctx, hipMemcpyAsync(parity, ctx->eds.p, bytes, hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  return DAGPU_OK;
}

int dagpu_decode(dagpu_ctx* ctx, uint32_t k, size_t nvec, size_t shard_size, uint8_t* shards,
                 const uint8_t* present) {
  if (!ctx || (nvec && (!shards || !present))) return DAGPU_ERR_ARG;
  if (shard_size == 0 || shard_size % 64)
    return set_err(ctx, DAGPU_ERR_SHARE_SIZE, "shard size must be a multiple of 64");
  std::lock_guard<std::mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  int rc = check_codec_k(ctx, k);
  if (rc) return rc;
  if (nvec == 0) return DAGPU_OK;
  const size_t n = 2 * (size_t)k;
  const size_t bytes = n * shard_size * nvec;
  hipStream_t s = ctx->stream;
  HIP_TRY(ctx, ctx->eds.ensure(bytes));
  HIP_TRY(ctx, ctx->ods.ensure(n * nvec));
  const size_t errb = (size_t)rs_err_bytes((int)k) * nvec;
  HIP_TRY(ctx, ctx->ws.ensure(errb + 3 * nvec * sizeof(int32_t) + 256));
  HIP_TRY(ctx, ctx->status.ensure(sizeof(int32_t)));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->eds.p, shards, bytes, hipMemcpyHostToDevice, s));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->ods.p, present, n * nvec, hipMemcpyHostToDevice, s));
  HIP_TRY(ctx, hipMemsetAsync(ctx->status.p, 0, sizeof(int32_t), s));
  DecodeArgs da{};
  da.data = (uint8_t*)ctx->eds.p;
  da.sq_stride = 0;
  da.vec_stride = (long)(n * shard_size);
  da.shard_stride = (long)shard_size;
  da.present = (uint8_t*)ctx->ods.p;
  da.p_sq_stride = 0;
  da.p_vec_stride = (long)n;
  da.p_shard_stride = 1;
  da.err = (uint8_t*)ctx->ws.p;
  da.flags = (int32_t*)((uint8_t*)ctx->ws.p + errb);
  // locator sharing runs one workgroup over all vectors of a "square" (<= 2 kMaxK)
  da.err_key = nvec <= 2 * (size_t)kMaxK ? da.flags + nvec : nullptr;
  da.err_head = nvec <= 2 * (size_t)kMaxK ? da.flags + 2 * nvec : nullptr;
  da.too_few = (int32_t*)ctx->status.p;
  da.nsq = 1;
  da.nvec = (long)nvec;
  da.nchunk = (long)((shard_size + 511) / 512);
  da.shard_bytes = (long)shard_size;
  da.k = (int)k;
  {
    ProfScope p(ctx, 5, s);
    HIP_TRY(ctx, launch_rs_decode(da, s, false));
  }
  int32_t too_few = 0;
  HIP_TRY(ctx, hipMemcpyAsync(&too_few, ctx->status.p, sizeof too_few, hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipMemcpyAsync(shards, ctx->eds.p, bytes, hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  if (too_few) return set_err(ctx, DAGPU_ERR_TOO_FEW_SHARDS, "too few shards given");
  return DAGPU_OK;
}

namespace {

struct RepairWs {
  SquareArgs sa;        // NMT verification (roots of the repaired square)
  uint8_t* p0;          // presence before repair
  int32_t* complete_before;
  int32_t* complete_now;
  int32_t* root_bad;    // [axis][sq][idx]: complete-before axis whose root differs
  int32_t* parity_bad;  // [axis][sq][idx]: complete-before axis whose parity != Encode(data)
  uint8_t* err_rows;
  uint8_t* err_cols;
  int32_t* flags_rows;
  int32_t* flags_cols;
  int32_t* err_share[2][2];  // [axis][same, head]
  int32_t* sel;         // exact-order repair: level of each axis' attempt, [2][w]
  int32_t* bits;
  int32_t* counters;    // kCtrSlots round counters (kernels.hpp kCtr*)
  // fill route / deferral (repair.hip PlanArgs)
  int32_t* fill;        // [sq][idx] of the round's axis
  int32_t* pair_list;   // k = 128 fill pairs, n * w entries
  int32_t* pair_list_rev;  // k = 128 reverse fill pairs, n * w entries
  int32_t* known;       // [axis][sq][idx]
  int32_t* deferred;    // [axis][sq][idx]
  int32_t* nodefer;     // [sq]
  int32_t* check;       // [sq]: a deferred axis is not a codeword
  int32_t* counts[2];   // [axis] vec_counts: present data shards | present shards << 16
};

size_t a256(size_t v) { return (v + 255) & ~(size_t)255; }

size_t repair_ws_bytes(uint32_t k, size_t n) {
  const size_t w = 2 * (size_t)k;
  size_t t = a256(nmt_workspace_bytes((int)k, (long)n));
  t += 2 * a256(n * w * kNodeSize) + a256(n * 32) + a256(n * 4);  // got roots, dah, nmt status
  t += a256(n * w * w);                                           // p0
  t += 4 * a256(n * 2 * w * 4);                                   // complete before/now, root/parity bad
  t += 2 * a256(n * w * rs_err_bytes((int)k)) + 2 * a256(n * w * 4);  // err, flags
  t += 4 * a256(n * w * 4);                                             // err_key, err_head per axis
  t += a256(2 * w * 4);                                                 // sel
  t += a256(n * 4) + 256;                                         // bits, counters
  t += 3 * a256(n * w * 4);                                                 // fill, pairs, reverse pairs
  t += 2 * a256(n * 2 * w * 4) + 2 * a256(n * 4);                           // known, deferred, nodefer, check
  t += 2 * a256(n * w * 4);                                                 // counts
  return t;
}

RepairWs carve_repair(uint32_t k, size_t n, void* base) {
  const size_t w = 2 * (size_t)k;
  uint8_t* p = (uint8_t*)base;
  RepairWs r{};
  r.sa.k = (int)k;
  r.sa.nsq = (long)n;
  nmt_workspace_carve(r.sa, p);
  p += a256(nmt_workspace_bytes((int)k, (long)n));
  r.sa.row_roots = p; p += a256(n * w * kNodeSize);
  r.sa.col_roots = p; p += a256(n * w * kNodeSize);
  r.sa.dah = p; p += a256(n * 32);
  r.sa.status = (int32_t*)p; p += a256(n * 4);
  r.p0 = p; p += a256(n * w * w);
  r.complete_before = (int32_t*)p; p += a256(n * 2 * w * 4);
  r.complete_now = (int32_t*)p; p += a256(n * 2 * w * 4);
  r.root_bad = (int32_t*)p; p += a256(n * 2 * w * 4);
  r.parity_bad = (int32_t*)p; p += a256(n * 2 * w * 4);
  r.err_rows = p; p += a256(n * w * rs_err_bytes((int)k));
  r.err_cols = p; p += a256(n * w * rs_err_bytes((int)k));
  r.flags_rows = (int32_t*)p; p += a256(n * w * 4);
  r.flags_cols = (int32_t*)p; p += a256(n * w * 4);
  for (int ax = 0; ax < 2; ax++)
    for (int j = 0; j < 2; j++) {
      r.err_share[ax][j] = (int32_t*)p;
      p += a256(n * w * 4);
    }
  r.sel = (int32_t*)p; p += a256(2 * w * 4);
  r.bits = (int32_t*)p; p += a256(n * 4);
  r.counters = (int32_t*)p; p += 256;
  r.fill = (int32_t*)p; p += a256(n * w * 4);
  r.pair_list = (int32_t*)p; p += a256(n * w * 4);
  r.pair_list_rev = (int32_t*)p; p += a256(n * w * 4);
  r.known = (int32_t*)p; p += a256(n * 2 * w * 4);
  r.deferred = (int32_t*)p; p += a256(n * 2 * w * 4);
  r.nodefer = (int32_t*)p; p += a256(n * 4);
  r.check = (int32_t*)p; p += a256(n * 4);
  r.counts[0] = (int32_t*)p; p += a256(n * w * 4);
  r.counts[1] = (int32_t*)p;
  return r;
}

DecodeArgs axis_decode_args(uint32_t k, size_t n, uint8_t* eds, uint8_t* present, int axis,
                            const RepairWs& r) {
  const long w = 2L * k;
  DecodeArgs d{};
  d.data = eds;
  d.sq_stride = (long)eds_bytes(k);
  d.present = present;
  d.p_sq_stride = w * w;
  if (axis == 0) {
    d.vec_stride = w * (long)kSS; d.shard_stride = kSS;
    d.p_vec_stride = w; d.p_shard_stride = 1;
    d.err = r.err_rows; d.flags = r.flags_rows; d.ndecodable = r.counters + kCtrRowsDec;
    d.nfill = r.counters + kCtrFillRows;
  } else {
    d.vec_stride = kSS; d.shard_stride = w * (long)kSS;
    d.p_vec_stride = 1; d.p_shard_stride = w;
    d.err = r.err_cols; d.flags = r.flags_cols; d.ndecodable = r.counters + kCtrColsDec;
    d.nfill = r.counters + kCtrFillCols;
  }
  d.err_key = r.err_share[axis][0];
  d.err_head = r.err_share[axis][1];
#ifdef DAGPU_TEST_HOOKS
  static const bool collide = getenv("DAGPU_TEST_KEY_COLLIDE") != nullptr;  // read once
  d.key_collide = collide ? 1 : 0;
#endif
  d.nsq = (long)n;
  d.nvec = w;
  d.nchunk = 1;
  d.shard_bytes = kSS;
  d.k = (int)k;
  return d;
}

extern "C++" {  // (this file's helpers sit inside the extern "C" block)
// rsmt2d solveCrossword (v0.11.0) replayed on presence bitmaps alone: the
// attempts in its sequential order (for each pass, i = 0..2k-1: row i, then
// column i; an incomplete axis with >= k shares is rebuilt), each with the
// orthogonal axes it completes (verified by rsmt2d right after the rebuild, in
// ascending index), and a dependency level: an attempt reads the cells of its
// own axis and of those orthogonal axes, so it must run after every earlier
// attempt that filled one of them.  Attempts of one level touch disjoint
// missing cells and run as one batched decode per orientation.
struct CrossPlan {
  std::vector<int> axis, idx, level;
  std::vector<int> ortho_off, ortho;  // CSR: orthogonal axes completed by attempt j
  std::vector<int32_t> att_level;     // [axis][w]: level of the axis' attempt, -1 = none
  int nlevels = 0;
  bool complete = false;              // the crossword fills the square
};

CrossPlan plan_crossword(int k, const uint8_t* p0) {
  const int w = 2 * k;
  CrossPlan pl;
  pl.att_level.assign(2 * (size_t)w, -1);
  std::vector<uint8_t> pres(p0, p0 + (size_t)w * w);
  std::vector<int> miss[2] = {std::vector<int>(w, 0), std::vector<int>(w, 0)};
  std::vector<int> lvl[2] = {std::vector<int>(w, -1), std::vector<int>(w, -1)};
  long missing = 0;
  for (int r = 0; r < w; r++)
    for (int c = 0; c < w; c++)
      if (!pres[(size_t)r * w + c]) { miss[0][r]++; miss[1][c]++; missing++; }
  pl.ortho_off.push_back(0);
  while (missing > 0) {
    bool progress = false;
    for (int i = 0; i < w; i++) {
      for (int ax = 0; ax < 2; ax++) {
        if (miss[ax][i] == 0 || w - miss[ax][i] < k) continue;
        int L = lvl[ax][i];
        const size_t o0 = pl.ortho.size();
        for (int j = 0; j < w; j++) {
          const size_t cell = ax == 0 ? (size_t)i * w + j : (size_t)j * w + i;
          if (pres[cell]) continue;
          if (miss[1 - ax][j] == 1) {  // this cell is the orthogonal axis' last gap
            pl.ortho.push_back(j);
            L = std::max(L, lvl[1 - ax][j]);
          }
        }
        L += 1;
        for (int j = 0; j < w; j++) {
          const size_t cell = ax == 0 ? (size_t)i * w + j : (size_t)j * w + i;
          if (pres[cell]) continue;
          pres[cell] = 1;
          miss[ax][i]--;
          miss[1 - ax][j]--;
          lvl[1 - ax][j] = std::max(lvl[1 - ax][j], L);
          missing--;
        }
        lvl[ax][i] = std::max(lvl[ax][i], L);
        (void)o0;
        pl.axis.push_back(ax);
        pl.idx.push_back(i);
        pl.level.push_back(L);
        pl.ortho_off.push_back((int)pl.ortho.size());
        pl.att_level[(size_t)ax * w + i] = L;
        pl.nlevels = std::max(pl.nlevels, L + 1);
        progress = true;
      }
    }
    if (!progress) break;
  }
  pl.complete = missing == 0;
  return pl;
}

std::string go_bytes(const uint8_t* p, size_t n) {  // fmt %v of a []byte
  std::string s = "[";
  for (size_t i = 0; i < n; i++) {
    if (i) s += ' ';
    s += std::to_string(p[i]);
  }
  return s + "]";
}

}  // extern "C++"

// Square `sq` of a batch whose parallel crossword found a rebuilt axis with the
// wrong root: rerun it in rsmt2d's sequential order to name the axis rsmt2d
// reports.  Every rebuild that verifies restores committed bytes, so up to the
// first failing attempt the batched level order fills exactly the cells
// rsmt2d's order fills, with the same bytes; an attempt's result is final once
// its axis (and the orthogonal axes it completes) are full, so one root pass at
// the end decides every attempt.  Leaves present[] as rsmt2d leaves it (cells
// of the attempts before the failing one) and byz[4] = {axis, index, rebuilt
// axis, rebuilt index}.  Synchronises `s`.
int exact_repair(dagpu_ctx* ctx, uint32_t k, size_t n, size_t sq, uint8_t* d_eds, uint8_t* d_present,
                 const uint8_t* d_rr, const uint8_t* d_cr, int32_t* d_byz, const RepairWs& r,
                 hipStream_t s) {
  const size_t w = 2 * (size_t)k;
  uint8_t* eds = d_eds + sq * eds_bytes(k);
  uint8_t* pres = d_present + sq * w * w;
  std::vector<uint8_t> p0(w * w);
  HIP_TRY(ctx, hipMemcpyAsync(p0.data(), r.p0 + sq * w * w, w * w, hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  const CrossPlan pl = plan_crossword((int)k, p0.data());
  HIP_TRY(ctx, hipMemcpyAsync(pres, r.p0 + sq * w * w, w * w, hipMemcpyDeviceToDevice, s));
  HIP_TRY(ctx, hipMemcpyAsync(r.sel, pl.att_level.data(), 2 * w * 4, hipMemcpyHostToDevice, s));
  std::vector<uint8_t> has(2 * (size_t)pl.nlevels, 0);
  for (size_t j = 0; j < pl.axis.size(); j++) has[2 * (size_t)pl.level[j] + pl.axis[j]] = 1;
  for (int L = 0; L < pl.nlevels; L++) {
    for (int ax = 0; ax < 2; ax++) {
      if (!has[2 * (size_t)L + ax]) continue;
      DecodeArgs d = axis_decode_args(k, 1, eds, pres, ax, r);
      d.err_key = d.err_head = nullptr;
      d.ndecodable = nullptr;
      d.sel_level = r.sel + (size_t)ax * w;
      d.sel_value = L;
      HIP_TRY(ctx, launch_rs_errlocs(d, s));
      HIP_TRY(ctx, launch_rs_decode_only(d, s, true));
    }
  }
  int rc = enqueue_roots(ctx, k, 1, eds, r.sa.row_roots, r.sa.col_roots, nullptr, r.sa.status, r.sa.digests, s);
  if (rc) return rc;
  std::vector<uint8_t> got(2 * w * kNodeSize), want(2 * w * kNodeSize);
  HIP_TRY(ctx, hipMemcpyAsync(got.data(), r.sa.row_roots, w * kNodeSize, hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipMemcpyAsync(got.data() + w * kNodeSize, r.sa.col_roots, w * kNodeSize, hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipMemcpyAsync(want.data(), d_rr + sq * w * kNodeSize, w * kNodeSize, hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipMemcpyAsync(want.data() + w * kNodeSize, d_cr + sq * w * kNodeSize, w * kNodeSize,
                              hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  auto bad = [&](int ax, int i) {
    const size_t off = ((size_t)ax * w + i) * kNodeSize;
    return memcmp(got.data() + off, want.data() + off, kNodeSize) != 0;
  };
  int32_t byz[4] = {-1, -1, -1, -1};
  size_t fail = pl.axis.size();
  for (size_t j = 0; j < pl.axis.size() && fail == pl.axis.size(); j++) {
    const int ax = pl.axis[j], i = pl.idx[j];
    if (bad(ax, i)) {
      byz[0] = byz[2] = ax;
      byz[1] = byz[3] = i;
      fail = j;
      break;
    }
    for (int o = pl.ortho_off[j]; o < pl.ortho_off[j + 1]; o++)
      if (bad(1 - ax, pl.ortho[o])) {
        byz[0] = 1 - ax;
        byz[1] = pl.ortho[o];
        byz[2] = ax;
        byz[3] = i;
        fail = j;
        break;
      }
  }
  if (fail < pl.axis.size()) {  // presence as rsmt2d leaves it: attempts before the failing one
    std::vector<uint8_t> p = p0;
    for (size_t j = 0; j < fail; j++)
      for (size_t t = 0; t < w; t++) {
        const size_t cell = pl.axis[j] == 0 ? (size_t)pl.idx[j] * w + t : t * w + pl.idx[j];
        p[cell] = 1;
      }
    HIP_TRY(ctx, hipMemcpyAsync(pres, p.data(), w * w, hipMemcpyHostToDevice, s));
  }
  HIP_TRY(ctx, hipMemcpyAsync(d_byz + 4 * sq, byz, sizeof byz, hipMemcpyHostToDevice, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  (void)n;
  return DAGPU_OK;
}

// A page-locked mailbox for the round counters (RAII; back to the context's pool).
struct Mailbox {
  dagpu_ctx* c;
  void* p = nullptr;
  Mailbox(const Mailbox&) = delete;
  Mailbox(Mailbox&& o) noexcept : c(o.c), p(o.p) { o.p = nullptr; }
  explicit Mailbox(dagpu_ctx* c_) : c(c_) {
    if (!c) return;  // (an empty mailbox: read_small then copies straight to the destination)
    {
      std::lock_guard<std::mutex> g(c->mb_mu);
      if (!c->mailboxes.empty()) {
        p = c->mailboxes.back();
        c->mailboxes.pop_back();
        return;
      }
    }
    if (hipHostMalloc(&p, dagpu_ctx::kMailbox, hipHostMallocDefault) != hipSuccess) p = nullptr;
  }
  ~Mailbox() {
    if (!p) return;
    std::lock_guard<std::mutex> g(c->mb_mu);
    c->mailboxes.push_back(p);
  }
};

// Small device->host read that the next host decision waits for: into the
// mailbox when there is one (a direct DMA), then a spin on the stream (the
// blocking wait's wake-up cost 50-200 us per Repair round, profiles/
// repair_timeline_r03.txt).
hipError_t read_small(void* dst, const void* src, size_t bytes, Mailbox& mb, hipStream_t s) {
  void* via = (mb.p && bytes <= dagpu_ctx::kMailbox) ? mb.p : dst;
  hipError_t e = hipMemcpyAsync(via, src, bytes, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = wait_stream(s, true);
  if (e == hipSuccess && via != dst) memcpy(dst, via, bytes);
  return e;
}

// The round counters a vec_count_round launch left in the mailbox: spin on its
// sequence word (kernels queued behind that launch keep the stream busy, so
// the stream itself is not waited for); the stream is polled now and then, for
// errors and for a word that never arrives (then the counters are copied).
hipError_t wait_round_counters(int32_t* cnt, const RoundCounters& rc, Mailbox& mb, hipStream_t s) {
  const volatile int32_t* word = rc.host + kCtrRead;
  for (unsigned spin = 0;; spin++) {
    if (*word == rc.seq) {
      __atomic_thread_fence(__ATOMIC_ACQUIRE);
      memcpy(cnt, (const void*)rc.host, kCtrRead * sizeof(int32_t));
      return hipSuccess;
    }
    if ((spin & 1023) == 1023) {
      const hipError_t e = hipStreamQuery(s);
      if (e == hipSuccess && *word != rc.seq) return read_small(cnt, rc.ctr, kCtrRead * sizeof(int32_t), mb, s);
      if (e != hipSuccess && e != hipErrorNotReady) return e;
    }
    __builtin_ia32_pause();
  }
}

std::atomic<int32_t> g_round_seq{1};

// rsmt2d Repair for n same-k squares resident on the device (see repair.hip).
// d_byz (optional, n * 4 int32): failing axis per square; asking for it makes
// the call resolve crossword failures in rsmt2d's order (exact_repair).
// mb_in (optional): a mailbox the caller took already (the asynchronous path
// allocates nothing on its worker thread: an allocation there could wait for
// a stream that is itself waiting for the worker).
int repair_device(dagpu_ctx* ctx, uint32_t k, size_t n, uint8_t* d_eds, uint8_t* d_present,
                  const uint8_t* d_rr, const uint8_t* d_cr, int32_t* d_status, int32_t* d_byz, void* d_ws,
                  hipStream_t s, Mailbox* mb_in = nullptr, int64_t* stats_out = nullptr) {
  const long w = 2L * k;
  RepairWs r = carve_repair(k, n, d_ws);
  HIP_TRY(ctx, hipMemcpyAsync(r.p0, d_present, n * w * w, hipMemcpyDeviceToDevice, s));
  HIP_TRY(ctx, hipMemsetAsync(r.bits, 0, n * sizeof(int32_t), s));
  HIP_TRY(ctx, hipMemsetAsync(r.parity_bad, 0, n * 2 * w * sizeof(int32_t), s));
  HIP_TRY(ctx, hipMemsetAsync(r.counters, 0, kCtrSlots * sizeof(int32_t), s));  // kernels.hpp kCtr*
  int64_t rounds_run = 0, deferred_run = 0;
  HIP_TRY(ctx, launch_axis_complete(d_present, (int)k, (long)n, r.complete_before, s, r.counters + kCtrComplete));
  // prerepairSanityCheck: complete axes must satisfy parity == Encode(data).
  // Queued after the first round's counter read, and only when some axis is
  // complete (a complete axis is never written by the crossword, so the order
  // does not matter; the maximal erasure patterns have none).
  auto prerepair = [&]() -> int {
    for (int axis = 0; axis < 2; axis++) {
      EncodeArgs e{};
      e.in = d_eds;
      e.in_sq_stride = (long)eds_bytes(k);
      e.out_sq_stride = (long)eds_bytes(k);
      if (axis == 0) {
        e.in_vec_stride = w * kSS; e.in_shard_stride = kSS;
        e.out = d_eds + (long)k * kSS; e.out_vec_stride = w * kSS; e.out_shard_stride = kSS;
      } else {
        e.in_vec_stride = kSS; e.in_shard_stride = w * kSS;
        e.out = d_eds + (long)k * w * kSS; e.out_vec_stride = kSS; e.out_shard_stride = w * kSS;
      }
      e.nsq = (long)n; e.nvec = w; e.nchunk = 1; e.shard_bytes = kSS;
      e.vec_flags = r.complete_before + (long)axis * n * w;
      e.mismatch = r.bits;
      e.mismatch_bit = 0;
      e.mismatch_vec = r.parity_bad + (long)axis * n * w;
      HIP_TRY(ctx, launch_rs_encode((int)k, e, s));
    }
    return DAGPU_OK;
  };
  // solveCrossword: each round rebuilds every decodable row or every decodable
  // column (whichever set is larger) until no axis can make progress.
  // Fill route and deferral (repair.hip PlanArgs; DAGPU_REPAIR_FILL=0 turns
  // them off): a decodable vector whose data half is complete is re-encoded
  // instead of decoded, and one whose parity half is complete is rebuilt by the
  // reverse transform (EncodeArgs.reverse); both give the decoder's bytes
  // whenever the vector's given shards agree with them, and a vector whose
  // given shards disagree goes to the decoder; when every vector i < k of an axis is decodable or
  // complete, the decodes of i >= k wait and the next round (the other axis)
  // fills everything.  For the maximal erasure pattern (Q3 given) that is k
  // reverse row fills, k reverse column fills and k row fills instead of
  // k + 2k decodes.  A deferred
  // vector the decoder would have rebuilt is the same codeword whenever the
  // square ends up a codeword square, which the known[] bookkeeping proves for
  // that pattern; otherwise a compare-mode encode checks every deferred vector,
  // and a square that fails is re-run from its original presence without
  // deferral (the decoders read present shards only).
  const char* fill_env = sw(SW_REPAIR_FILL);  // read per call (tests compare both)
  const bool shortcut = !(fill_env && fill_env[0] == '0');
  const bool fill_list = k == 128;
  if (shortcut) {
    HIP_TRY(ctx, hipMemcpyAsync(r.known, r.complete_before, n * 2 * w * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
    HIP_TRY(ctx, hipMemsetAsync(r.deferred, 0, n * 2 * w * sizeof(int32_t), s));
    HIP_TRY(ctx, hipMemsetAsync(r.nodefer, 0, n * sizeof(int32_t), s));
  }
  const int max_rounds = 4 * (int)w + 4;
  Mailbox mb_own(mb_in ? nullptr : ctx);
  Mailbox& mb = mb_in ? *mb_in : mb_own;
  // Per round: one launch counts both axes and leaves the counters in the
  // mailbox (RoundCounters), the host picks the axis, and the round's last
  // launch (launch_rs_mark_round) clears the next round's counts: no memsets
  // or copies between the kernels of a round.
  RoundCounters rcnt{r.counters, mb.p ? (int32_t*)mb.p : nullptr, 0};
  for (int pass = 0; pass < 2; pass++) {
    long deferred_total = 0;
    int last_ax = -1;
    if (pass > 0) {  // (the repair's first memset covers pass 0)
      HIP_TRY(ctx, hipMemsetAsync(r.counters, 0, (kCtrPairsRev + 1) * sizeof(int32_t), s));
      HIP_TRY(ctx, hipMemsetAsync(r.counters + kCtrDeferSquares, 0, 2 * sizeof(int32_t), s));  // and DeferredPrev
    }
    for (int round = 0; round < max_rounds; round++) {
      DecodeArgs dr = axis_decode_args(k, n, d_eds, d_present, 0, r);
      DecodeArgs dc = axis_decode_args(k, n, d_eds, d_present, 1, r);
      // decodable vectors and counts of both axes (no locators yet)
      dr.vec_counts = r.counts[0];
      dc.vec_counts = r.counts[1];
      rcnt.seq = g_round_seq.fetch_add(1) & 0x7fffffff;
      HIP_TRY(ctx, launch_vec_count_round(dr, dc, rcnt, s));
      // Few vectors (a launch is mostly latency): both axes' candidate locator
      // heads while the host reads the counts; else the chosen axis' after it.
      const bool early_heads = (long)n * w <= 8192;
      if (early_heads) HIP_TRY(ctx, launch_errloc_heads2(dr, &dc, s));
      int32_t cnt[kCtrRead] = {};
      if (rcnt.host) {
        HIP_TRY(ctx, wait_round_counters(cnt, rcnt, mb, s));
      } else {
        HIP_TRY(ctx, read_small(cnt, r.counters, sizeof cnt, mb, s));
      }
      cnt[kCtrDeferred] = cnt[kCtrDeferredPrev];  // the previous round's plan
      {  // schedule totals so far (diagnostics): plans of the earlier rounds are complete;
         // a started Repair writes its slot's copy (published at its join)
        std::unique_lock<std::mutex> g(ctx->prof_mu, std::defer_lock);
        if (!stats_out) g.lock();
        int64_t* st = stats_out ? stats_out : ctx->rep_stats;
        st[0] = rounds_run;
        st[1] = cnt[kCtrPlan];
        st[2] = cnt[kCtrPlan + 1];
        st[3] = cnt[kCtrPlan + 2];
        st[4] = deferred_run + cnt[kCtrDeferred];
      }
      if (pass == 0 && round == 0 && cnt[kCtrComplete] > 0) {
        const int prc = prerepair();
        if (prc) return prc;
      }
      deferred_total += cnt[kCtrDeferred];
      deferred_run += cnt[kCtrDeferred];
      if (cnt[kCtrRowsDec] == 0 && cnt[kCtrColsDec] == 0) break;
      rounds_run++;
      int ax = cnt[kCtrRowsDec] >= cnt[kCtrColsDec] ? 0 : 1;
      // after a deferral the other axis is the one with complete data halves
      if (cnt[kCtrDeferred] > 0 && last_ax >= 0 && cnt[kCtrRowsDec + 1 - last_ax] > 0) ax = 1 - last_ax;
      last_ax = ax;
      DecodeArgs& d = ax == 0 ? dr : dc;
      if (shortcut) {
        const long w_ = w;
        EncodeArgs e{};
        e.in = d_eds;
        e.in_sq_stride = e.out_sq_stride = (long)eds_bytes(k);
        e.op_sq_stride = w_ * w_;
        if (ax == 0) {
          e.in_vec_stride = w_ * kSS; e.in_shard_stride = kSS;
          e.out = d_eds + (long)k * kSS; e.out_vec_stride = w_ * kSS; e.out_shard_stride = kSS;
          e.out_present = d_present + k; e.op_vec_stride = w_; e.op_shard_stride = 1;
        } else {
          e.in_vec_stride = kSS; e.in_shard_stride = w_ * kSS;
          e.out = d_eds + (long)k * w_ * kSS; e.out_vec_stride = kSS; e.out_shard_stride = w_ * kSS;
          e.out_present = d_present + (long)k * w_; e.op_vec_stride = 1; e.op_shard_stride = w_;
        }
        e.nsq = (long)n; e.nvec = w_; e.nchunk = 1; e.shard_bytes = kSS;
        e.redo = d.flags;
        const bool listed = fill_list && leo8_fill_sliced_applicable(e);
        PlanArgs pa{};
        pa.counts = d.vec_counts;
        pa.flags = d.flags;
        pa.fill = r.fill;
        pa.pair_list = listed ? r.pair_list : nullptr;
        pa.pair_count = r.counters + kCtrPairs;
        pa.pair_list_rev = listed ? r.pair_list_rev : nullptr;
        pa.pair_count_rev = r.counters + kCtrPairsRev;
        pa.known = r.known;
        pa.deferred = r.deferred;
        pa.nodefer = r.nodefer;
        pa.ndeferred = r.counters + kCtrDeferred;
        pa.nplan = r.counters + kCtrPlan;
        pa.k = (int)k;
        pa.nsq = (long)n;
        pa.axis = ax;
        HIP_TRY(ctx, launch_repair_plan(pa, s));
        // no fill candidates on this axis (the count launch's tally of the
        // plan's f / r vectors): the two fill launches would find nothing
        if (cnt[ax == 0 ? kCtrFillRows : kCtrFillCols] > 0) {
          ProfScope p(ctx, 6, s);
          // reverse fills: parity half in, data half out (its presence k shards before)
          EncodeArgs er = e;
          er.in = e.out;
          er.out = (uint8_t*)e.in;
          er.out_present = e.out_present - (long)k * e.op_shard_stride;
          er.reverse = 1;
          if (listed) {
            e.pair_list = r.pair_list;
            e.pair_count = r.counters + kCtrPairs;
            HIP_TRY(ctx, launch_leo8_fill_sliced(e, (long)n * w_ / 2, s));
            er.pair_list = r.pair_list_rev;
            er.pair_count = r.counters + kCtrPairsRev;
            HIP_TRY(ctx, launch_leo8_fill_sliced(er, (long)n * w_ / 2, s));
          } else {
            e.vec_flags = er.vec_flags = r.fill;
            e.vec_flag_match = 1;
            er.vec_flag_match = 2;
            HIP_TRY(ctx, launch_rs_encode((int)k, e, s));
            HIP_TRY(ctx, launch_rs_encode((int)k, er, s));
          }
        }
      }
      // locators of the vectors left to the decoder (fill redos included)
      d.locators_only = 1;
      if (!early_heads) HIP_TRY(ctx, launch_errloc_heads2(d, nullptr, s));
      HIP_TRY(ctx, launch_rs_errlocs_only(d, s));
      {
        ProfScope p(ctx, 5, s);
        HIP_TRY(ctx, launch_rs_decode_only(d, s, false));
      }
      HIP_TRY(ctx, launch_rs_mark_round(d, shortcut ? r.fill : nullptr,
                                        shortcut ? r.known + (long)ax * n * w : nullptr, r.counters, s));
    }
    if (!shortcut || deferred_total == 0) break;
    // deferred vectors whose codeword property is not implied: compare-mode encodes
    HIP_TRY(ctx, launch_repair_defer_check(r.deferred, r.known, (int)k, (long)n, r.check, s,
                                           r.counters + kCtrDeferSquares));
    int32_t left = 0;  // squares whose deferred axes are not proven codewords
    HIP_TRY(ctx, read_small(&left, r.counters + kCtrDeferSquares, sizeof left, mb, s));
    if (left == 0) break;
    for (int axis = 0; axis < 2; axis++) {
      EncodeArgs e{};
      e.in = d_eds;
      e.in_sq_stride = e.out_sq_stride = (long)eds_bytes(k);
      if (axis == 0) {
        e.in_vec_stride = w * kSS; e.in_shard_stride = kSS;
        e.out = d_eds + (long)k * kSS; e.out_vec_stride = w * kSS; e.out_shard_stride = kSS;
      } else {
        e.in_vec_stride = kSS; e.in_shard_stride = w * kSS;
        e.out = d_eds + (long)k * w * kSS; e.out_vec_stride = kSS; e.out_shard_stride = w * kSS;
      }
      e.nsq = (long)n; e.nvec = w; e.nchunk = 1; e.shard_bytes = kSS;
      e.vec_flags = r.deferred + (long)axis * n * w;
      e.mismatch = r.check;
      e.mismatch_bit = 1;
      HIP_TRY(ctx, launch_rs_encode((int)k, e, s));
    }
    std::vector<int32_t> chk(n);
    HIP_TRY(ctx, read_small(chk.data(), r.check, n * sizeof(int32_t), mb, s));
    bool rerun = false;
    for (size_t i = 0; i < n; i++) {
      if (!chk[i]) continue;
      rerun = true;
      HIP_TRY(ctx, hipMemcpyAsync(d_present + i * w * w, r.p0 + i * w * w, w * w, hipMemcpyDeviceToDevice, s));
      HIP_TRY(ctx, hipMemsetD32Async((hipDeviceptr_t)(r.nodefer + i), 1, 1, s));
    }
    if (!rerun) break;
  }
  // verify every complete axis against the given roots
  HIP_TRY(ctx, launch_axis_complete(d_present, (int)k, (long)n, r.complete_now, s));
  r.sa.eds = d_eds;
  r.sa.eds_sq_stride = (long)eds_bytes(k);
  int rc = enqueue_roots(ctx, k, n, d_eds, r.sa.row_roots, r.sa.col_roots, nullptr, r.sa.status,
                         r.sa.digests, s);
  if (rc) return rc;
  HIP_TRY(ctx, launch_verify_roots(d_rr, d_cr, r.sa.row_roots, r.sa.col_roots, r.complete_now,
                                   r.complete_before, (int)k, (long)n, r.bits, r.root_bad, s));
  HIP_TRY(ctx, launch_finalize_repair(r.bits, r.complete_before, r.root_bad, r.parity_bad, (int)k, (long)n,
                                      d_status, d_byz, s, r.check));
  // a square failing prerepairSanityCheck is left as its input (rsmt2d never
  // reaches solveCrossword for it): presence back to p0; the bytes of cells
  // not present are unspecified, as they are for any missing cell
  HIP_TRY(ctx, launch_restore_presence(d_present, r.p0, r.check, (int)k, (long)n, s));
  if (!d_byz) return DAGPU_OK;
  // crossword failures: name the axis in rsmt2d's order (rare; synchronises)
  std::vector<int32_t> st(n), bz(4 * n);
  HIP_TRY(ctx, hipMemcpyAsync(st.data(), d_status, n * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipMemcpyAsync(bz.data(), d_byz, 4 * n * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  for (size_t i = 0; i < n; i++) {
    if (st[i] != DAGPU_ERR_BYZANTINE || bz[4 * i] >= 0) continue;
    rc = exact_repair(ctx, k, n, i, d_eds, d_present, d_rr, d_cr, d_byz, r, s);
    if (rc) return rc;
  }
  return DAGPU_OK;
}

}  // namespace

size_t dagpu_repair_workspace_size(uint32_t k, size_t n) {
  if (k == 0 || n == 0) return 256;
  return repair_ws_bytes(k, n) + 256;
}

int dagpu_repair_batch_device_ex(dagpu_ctx* ctx, uint32_t k, size_t n, uint8_t* d_eds,
                                 uint8_t* d_present, const uint8_t* d_row_roots,
                                 const uint8_t* d_col_roots, int32_t* d_status, int32_t* d_byz,
                                 void* d_workspace, void* stream) {
  if (!ctx || !d_eds || !d_present || !d_row_roots || !d_col_roots || !d_status || !d_workspace)
    return DAGPU_ERR_ARG;
  int rc = check_k(ctx, k);
  if (rc) return rc;
  if (n == 0) return DAGPU_OK;
  return repair_device(ctx, k, n, d_eds, d_present, d_row_roots, d_col_roots, d_status, d_byz, d_workspace,
                       (hipStream_t)stream);
}

}  // extern "C"

namespace {

hipError_t async_init_slot(dagpu_ctx::AsyncSlot& sl) {
  hipError_t e = hipSuccess;
  if (!sl.stream && (e = hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking)) != hipSuccess) return e;
  if (!sl.fork && (e = hipEventCreateWithFlags(&sl.fork, hipEventDisableTiming)) != hipSuccess) return e;
  if (!sl.finished && (e = hipEventCreateWithFlags(&sl.finished, hipEventDisableTiming)) != hipSuccess) return e;
  return e;
}

}  // namespace

extern "C" {

// Asynchronous Repair: the crossword's host decisions (one counter read per
// round) run on a library worker thread that queues the kernels on a stream
// of its own, forked from `stream` at the call; dagpu_repair_join then makes a
// stream wait for the finished repair.  Nothing on the device ever waits for
// work queued later: a first design whose caller stream waited on a signal
// word the worker would write later (hipStreamWaitValue32) hung inside the
// test suite although the primitives pass alone (tools/waitvalue_probe.hip) --
// with GPU_MAX_HW_QUEUES = 4 two streams can share one hardware queue, and a
// wait ahead of its own release in that queue never passes.  So a join blocks
// the calling thread until the worker has queued its last command, and calls
// started back to back (e.g. slices of a batch) run side by side
// (profiles/repair_async_r04.log).
int dagpu_repair_start(dagpu_ctx* ctx, uint32_t k, size_t n, uint8_t* d_eds, uint8_t* d_present,
                       const uint8_t* d_row_roots, const uint8_t* d_col_roots, int32_t* d_status,
                       void* d_workspace, void* stream, uint64_t* handle) {
  if (!ctx || !handle || !d_eds || !d_present || !d_row_roots || !d_col_roots || !d_status || !d_workspace)
    return DAGPU_ERR_ARG;
  *handle = 0;
  int rc = check_k(ctx, k);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  std::lock_guard<std::mutex> g(ctx->async_mu);
  int si = -1;
  for (int i = 0; i < dagpu_ctx::kAsyncSlots && si < 0; i++)
    if (!ctx->async_slot[i].busy) si = i;
  if (si < 0) return set_err(ctx, DAGPU_ERR_ARG, "too many repairs started and not joined");
  dagpu_ctx::AsyncSlot& sl = ctx->async_slot[si];
  HIP_TRY(ctx, async_init_slot(sl));
  HIP_TRY(ctx, launch_rs_prepare((int)k));  // first-use table uploads here, not on the worker
  HIP_TRY(ctx, hipEventRecord(sl.fork, s));
  sl.rc = DAGPU_OK;
  sl.err.clear();
  for (auto& x : sl.stats) x = 0;
  hipStream_t ws = sl.stream;
  hipEvent_t fork = sl.fork, fin = sl.finished;
  dagpu_ctx::AsyncSlot* slp = &sl;
  const int dev = ctx->device;
  // std::thread / make_shared may throw (no threads or memory left): nothing
  // may escape an extern "C" entry point, and the slot stays free
  try {
    auto mb = std::make_shared<Mailbox>(ctx);
    auto snap = std::make_shared<SwSnapshot>();
    sw_snapshot(snap.get());  // on the caller's thread (getenv is not thread-safe against setenv)
#ifdef DAGPU_TEST_HOOKS
    const char* inj = getenv("DAGPU_TEST_WORKER_FAIL");
    const bool inject_fail = inj && inj[0] == '1';
#endif
    sl.worker = std::thread([=]() {
      on_repair_worker() = true;
      sw_bind(snap.get());  // the switches as the start call saw them
      (void)hipSetDevice(dev);
      int r = hipStreamWaitEvent(ws, fork, 0) == hipSuccess ? DAGPU_OK : DAGPU_ERR_DEVICE;
#ifdef DAGPU_TEST_HOOKS
      // test build only (libdagpu_test.so, tests/test_gpu_repair_async.py): the
      // worker fails before its first kernel, so the join's error path is exercised
      if (r == DAGPU_OK && inject_fail) r = set_err(ctx, DAGPU_ERR_DEVICE, "injected worker failure");
#endif
      if (r == DAGPU_OK && n)
        r = repair_device(ctx, k, n, d_eds, d_present, d_row_roots, d_col_roots, d_status, nullptr, d_workspace, ws,
                          mb.get(), slp->stats);
      if (r != DAGPU_OK) {
        // the worker's own message (set_err wrote it to this thread's state);
        // the join re-raises it on the caller's thread
        const ThreadErr& te = thread_err();
        slp->err = te.own && !te.msg.empty() ? te.msg : "started repair failed on the device";
        (void)hipMemsetD32Async((hipDeviceptr_t)d_status, (int)DAGPU_ERR_DEVICE, n, ws);
      }
      (void)hipEventRecord(fin, ws);
      slp->rc = r;
    });
  } catch (...) {
    return set_err(ctx, DAGPU_ERR_DEVICE, "could not start the repair worker thread");
  }
  if (++ctx->async_gen == 0) ++ctx->async_gen;
  sl.busy = true;
  sl.joining = false;
  sl.gen = ctx->async_gen;
  *handle = ((uint64_t)sl.gen << 8) | (uint64_t)si;
  return DAGPU_OK;
}

int dagpu_repair_join(dagpu_ctx* ctx, uint64_t handle, void* stream) {
  if (!ctx) return DAGPU_ERR_ARG;
  const int si = (int)(handle & 0xFF);
  std::thread worker;
  {  // claim the slot under the lock, wait for its worker without it
    std::lock_guard<std::mutex> g(ctx->async_mu);
    if (si >= dagpu_ctx::kAsyncSlots || !ctx->async_slot[si].busy || ctx->async_slot[si].joining ||
        ctx->async_slot[si].gen != (uint32_t)(handle >> 8))
      return set_err(ctx, DAGPU_ERR_ARG, "unknown or already joined repair handle");
    ctx->async_slot[si].joining = true;
    worker = std::move(ctx->async_slot[si].worker);
  }
  if (worker.joinable()) worker.join();  // its last command is queued
  std::lock_guard<std::mutex> g(ctx->async_mu);
  dagpu_ctx::AsyncSlot& sl = ctx->async_slot[si];
  const int rc = sl.rc;
  {
    std::lock_guard<std::mutex> gp(ctx->prof_mu);
    for (int i = 0; i < DAGPU_REPAIR_STATS; i++) ctx->rep_stats[i] = sl.stats[i];
  }
  const hipError_t e = hipStreamWaitEvent((hipStream_t)stream, sl.finished, 0);
  sl.busy = false;
  sl.joining = false;
  if (e != hipSuccess) return hip_fail(ctx, e, "hipStreamWaitEvent(stream, finished)");
  if (rc != DAGPU_OK) return set_err(ctx, rc, sl.err);
  return DAGPU_OK;
}

// Start + join on the same stream: returns once every kernel of the repair is
// queued (the caller's stream then runs them in order with its later work).
int dagpu_repair_batch_device(dagpu_ctx* ctx, uint32_t k, size_t n, uint8_t* d_eds,
                              uint8_t* d_present, const uint8_t* d_row_roots,
                              const uint8_t* d_col_roots, int32_t* d_status, void* d_workspace,
                              void* stream) {
  if (!ctx || !d_eds || !d_present || !d_row_roots || !d_col_roots || !d_status || !d_workspace)
    return DAGPU_ERR_ARG;
  int rc = check_k(ctx, k);
  if (rc) return rc;
  if (n == 0) return DAGPU_OK;
  return repair_device(ctx, k, n, d_eds, d_present, d_row_roots, d_col_roots, d_status, nullptr, d_workspace,
                       (hipStream_t)stream);
}

int dagpu_repair_ex(dagpu_ctx* ctx, uint32_t k, uint8_t* eds, uint8_t* present,
                    const uint8_t* row_roots, const uint8_t* col_roots, int32_t* byz) {
  if (!ctx || !eds || !present || !row_roots || !col_roots) return DAGPU_ERR_ARG;
  std::lock_guard<std::mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  if (byz) byz[0] = byz[1] = byz[2] = byz[3] = -1;
  int rc = check_k(ctx, k);
  if (rc) return rc;
  const size_t w = 2 * (size_t)k;
  hipStream_t s = ctx->stream;
  HIP_TRY(ctx, ctx->eds.ensure(eds_bytes(k)));
  HIP_TRY(ctx, ctx->ods.ensure(w * w));
  HIP_TRY(ctx, ctx->rr.ensure(w * kNodeSize));
  HIP_TRY(ctx, ctx->cr.ensure(w * kNodeSize));
  HIP_TRY(ctx, ctx->status.ensure(5 * sizeof(int32_t)));
  HIP_TRY(ctx, ctx->ws.ensure(dagpu_repair_workspace_size(k, 1)));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->eds.p, eds, eds_bytes(k), hipMemcpyHostToDevice, s));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->ods.p, present, w * w, hipMemcpyHostToDevice, s));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->rr.p, row_roots, w * kNodeSize, hipMemcpyHostToDevice, s));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->cr.p, col_roots, w * kNodeSize, hipMemcpyHostToDevice, s));
  int32_t* d_st = (int32_t*)ctx->status.p;
  rc = repair_device(ctx, k, 1, (uint8_t*)ctx->eds.p, (uint8_t*)ctx->ods.p, (const uint8_t*)ctx->rr.p,
                     (const uint8_t*)ctx->cr.p, d_st, d_st + 1, ctx->ws.p, s);
  if (rc) return rc;
  int32_t st[5] = {0, -1, -1, -1, -1};
  HIP_TRY(ctx, hipMemcpyAsync(st, d_st, sizeof st, hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipMemcpyAsync(eds, ctx->eds.p, eds_bytes(k), hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipMemcpyAsync(present, ctx->ods.p, w * w, hipMemcpyDeviceToHost, s));
  HIP_TRY(ctx, hipStreamSynchronize(s));
  if (byz) memcpy(byz, st + 1, 4 * sizeof(int32_t));
  const char* axn = st[1] == 1 ? "col" : "row";
  switch (st[0]) {
    case DAGPU_OK: return DAGPU_OK;
    case DAGPU_ERR_BAD_ROOTS: {
      // "bad root input: row %d expected %v got %v" (prerepairSanityCheck)
      const RepairWs r = carve_repair(k, 1, ctx->ws.p);
      std::vector<uint8_t> got(kNodeSize);
      const uint8_t* src = (st[1] == 1 ? r.sa.col_roots : r.sa.row_roots) + (size_t)st[2] * kNodeSize;
      HIP_TRY(ctx, hipMemcpy(got.data(), src, kNodeSize, hipMemcpyDeviceToHost));
      const uint8_t* want = (st[1] == 1 ? col_roots : row_roots) + (size_t)st[2] * kNodeSize;
      return set_err(ctx, st[0], std::string("bad root input: ") + axn + " " + std::to_string(st[2]) +
                                     " expected " + go_bytes(want, kNodeSize) + " got " +
                                     go_bytes(got.data(), kNodeSize));
    }
    case DAGPU_ERR_BYZANTINE:  // ErrByzantineData.Error(): "byzantine %s: %d"
      return set_err(ctx, st[0], st[1] >= 0 ? std::string("byzantine ") + axn + ": " + std::to_string(st[2])
                                            : std::string("byzantine data"));
    case DAGPU_ERR_UNREPAIRABLE: return set_err(ctx, st[0], "failed to solve data square");
    default: return set_err(ctx, st[0], "repair failed");
  }
}

int dagpu_repair(dagpu_ctx* ctx, uint32_t k, uint8_t* eds, uint8_t* present,
                 const uint8_t* row_roots, const uint8_t* col_roots) {
  return dagpu_repair_ex(ctx, k, eds, present, row_roots, col_roots, nullptr);
}

int dagpu_profile_enable(dagpu_ctx* ctx, int on) {
  if (!ctx) return DAGPU_ERR_ARG;
  ctx->prof = (on & 1) != 0;
  ctx->stages_on = (on & 2) != 0;
  return DAGPU_OK;
}

int dagpu_repair_stats(dagpu_ctx* ctx, int64_t* out) {
  if (!ctx || !out) return DAGPU_ERR_ARG;
  std::lock_guard<std::mutex> g(ctx->prof_mu);
  for (int i = 0; i < DAGPU_REPAIR_STATS; i++) out[i] = ctx->rep_stats[i];
  return DAGPU_OK;
}

int dagpu_profile_stages(dagpu_ctx* ctx, float* ms) {
  if (!ctx || !ms) return DAGPU_ERR_ARG;
  std::lock_guard<std::mutex> g(ctx->mu);
  for (int i = 0; i < dagpu_ctx::kStages; i++) ms[i] = -1.0f;
  if (!(ctx->stage_mask & 1u)) return DAGPU_OK;
  for (int i = 0; i < dagpu_ctx::kStages; i++) {
    if (!(ctx->stage_mask & (1u << i))) continue;
    HIP_TRY(ctx, hipEventSynchronize(ctx->stage_ev[i]));
    HIP_TRY(ctx, hipEventElapsedTime(&ms[i], ctx->stage_ev[0], ctx->stage_ev[i]));
  }
  return DAGPU_OK;
}

int dagpu_profile_read(dagpu_ctx* ctx, double* total_ms, uint64_t* launches, int reset) {
  if (!ctx) return DAGPU_ERR_ARG;
  std::lock_guard<std::mutex> g(ctx->prof_mu);
  for (auto& r : ctx->pending) {
    HIP_TRY(ctx, hipEventSynchronize(r.b));
    float ms = 0;
    HIP_TRY(ctx, hipEventElapsedTime(&ms, r.a, r.b));
    ctx->prof_ms[r.id] += ms;
    ctx->prof_n[r.id] += 1;
    ctx->pool.push_back(r.a);
    ctx->pool.push_back(r.b);
  }
  ctx->pending.clear();
  for (int i = 0; i < DAGPU_PROFILE_KERNELS; i++) {
    if (total_ms) total_ms[i] = ctx->prof_ms[i];
    if (launches) launches[i] = ctx->prof_n[i];
    if (reset) { ctx->prof_ms[i] = 0; ctx->prof_n[i] = 0; }
  }
  return DAGPU_OK;
}

int dagpu_dah_hash(const uint8_t* row_roots, const uint8_t* col_roots, size_t w,
                   uint8_t* out32) {
  if (!out32 || (w && (!row_roots || !col_roots))) return DAGPU_ERR_ARG;
  std::vector<const uint8_t*> items;
  items.reserve(2 * w);
  for (size_t i = 0; i < w; i++) items.push_back(row_roots + i * kNodeSize);
  for (size_t i = 0; i < w; i++) items.push_back(col_roots + i * kNodeSize);
  host::rfc6962_root(items, kNodeSize, out32);
  return DAGPU_OK;
}

}  // extern "C"
