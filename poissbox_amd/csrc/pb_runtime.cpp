// pb_runtime.cpp -- host runtime of libpoissbox_gpu: errors, context (device, stream, RCCL),
// slab grid, vectors, halo exchange and allreduce, the operator entry point and kernel timing.
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>

#include "pb_internal.hpp"

namespace pb {

// ---- field allocations (pb_internal.hpp) ----
// (r06 measured a stagger of every allocation by 4-260 KiB and the KSP vectors pooled in one
// allocation: neither controls pass B's placement-dependent rate; code in commit 8e8b21f)
hipError_t field_alloc(void** p, size_t bytes) { return hipMalloc(p, bytes); }

void field_free(void* p) {
  if (p) (void)hipFree(p);
}

// ---- tuning table (pb_tune_set; pb_internal.hpp tune()) ----
namespace {
// every name a kernel launcher consults; the defaults live at the call sites (the measured
// choices), the table only holds values a caller set
const char* const kTuneNames[] = {
    "a2a_copy_self", "cg_defer_x", "engine_kc_skew", "cg_fold", "cg_fuse", "cg_sr_fused", "comm_mark_every",
    "comm_stall_test_ms", "compact_lines", "fft_rupd", "fft_zpad", "fft_zpad_min_plane",
    "force_comm", "ksp_lazy0", "mg_agglomerate", "mg_engine_min_plane", "mg_restrict_z_min_cols",
    "mg_split_fused", "mg_sweep2", "mg_tail_max", "mg_u4_split", "pcr_lines", "sor_omega_any", "sr_ddiff",
    "stencil_kc", "stencil_kc_skew", "stencil_nt", "stencil_tall", "stencil_wgcu", "x_dot_cu"};
constexpr int kNumTune = (int)(sizeof(kTuneNames) / sizeof(kTuneNames[0]));
// lock-free table (tune() runs several times per CG iteration / V-cycle): a value and
// a set flag per name, and a count of set names so the common case (nothing set) is one load.
// Like every table update, pb_tune_set is not meant to race with running calls.
std::atomic<int> g_tune_val[kNumTune];
std::atomic<int> g_tune_set[kNumTune];
std::atomic<int> g_tune_nset{0};
int tune_index(const char* name) {
  for (int i = 0; i < kNumTune; ++i)
    if (strcmp(kTuneNames[i], name) == 0) return i;
  return -1;
}
}  // namespace

int tune(const char* name, int dflt) {
  if (g_tune_nset.load(std::memory_order_acquire) == 0) return dflt;
  const int i = tune_index(name);
  if (i < 0 || !g_tune_set[i].load(std::memory_order_acquire)) return dflt;
  return g_tune_val[i].load(std::memory_order_relaxed);
}

bool tune_is_set(const char* name) {
  const int i = tune_index(name);
  return i >= 0 && g_tune_set[i].load(std::memory_order_acquire) != 0;
}

static thread_local char g_err[1024] = "";

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  // a failed HIP call reported here is consumed: without this, HIP's per-thread last error (e.g.
  // a refused hipMalloc) would resurface at the next, unrelated kernel-launch check
  if (code == PB_ERR_ALLOC || code == PB_ERR_HIP) (void)hipGetLastError();
  return code;
}

// src/coefficients.f90:22-48: [1,-2,1]/dx^2 per direction, centre summed x then y then z
Star star_coeffs(const double h[3]) {
  double inv[3];
  for (int d = 0; d < 3; ++d) inv[d] = 1.0 / (h[d] * h[d]);
  Star s;
  s.cx = inv[0];
  s.cy = inv[1];
  s.cz = inv[2];
  double c = 0.0;
  c = c + -(2.0 * inv[0]);
  c = c + -(2.0 * inv[1]);
  c = c + -(2.0 * inv[2]);
  s.cc = c;
  return s;
}

// ---- timing ----
static hipEvent_t take_event(pb_ctx* ctx) {
  if (!ctx->event_pool.empty()) {
    hipEvent_t e = ctx->event_pool.back();
    ctx->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

bool timer_wanted(pb_ctx* ctx, const char* name) {
  bool want = ctx->timing_only.empty();
  for (const auto& n : ctx->timing_only)
    if (n == name) want = true;
  if (!want || ctx->timing_every <= 1) return want;
  return ctx->timer_calls[name]++ % ctx->timing_every == 0;  // sampled phase
}

void timer_begin(pb_ctx* ctx, const char*, hipEvent_t* ev, hipStream_t s) {
  *ev = take_event(ctx);
  (void)hipEventRecord(*ev, s ? s : ctx->stream);
}

void timer_end(pb_ctx* ctx, const char* name, hipEvent_t ev0, hipStream_t s) {
  hipEvent_t ev1 = take_event(ctx);
  (void)hipEventRecord(ev1, s ? s : ctx->stream);
  ctx->pending.push_back({std::string(name), {ev0, ev1}});
  if (ctx->pending.size() > 4096) timers_collect(ctx);
}

void timers_collect(pb_ctx* ctx) {
  for (auto& p : ctx->pending) {
    float ms = 0.f;
    (void)hipEventSynchronize(p.second.second);
    (void)hipEventElapsedTime(&ms, p.second.first, p.second.second);
    TimerSlot& t = ctx->timers[p.first];
    t.total_ms += ms;
    t.count += 1;
    if (t.samples.size() < kMaxTimerSamples) t.samples.push_back(ms);
    ctx->event_pool.push_back(p.second.first);
    ctx->event_pool.push_back(p.second.second);
  }
  ctx->pending.clear();
}

// ---- bounded waits ----
int comm_fail(pb_ctx* ctx, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  if (ctx->h_stall) __atomic_store_n(ctx->h_stall, 1, __ATOMIC_RELEASE);  // (test hook)
  if (!ctx->comm_failed) {
    ctx->comm_failed = true;
    fprintf(stderr, "[poissbox rank %d] communication failure: %s\n", ctx->rank, g_err);
    if (ctx->comm) {
      // releases RCCL kernels still waiting for a peer, so the streams can drain
      (void)ncclCommAbort(ctx->comm);
      ctx->comm = nullptr;
    }
  }
  return PB_ERR_COMM;
}

static int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

static hipEvent_t take_mark_event(pb_ctx* ctx) {
  if (!ctx->mark_pool.empty()) {
    hipEvent_t e = ctx->mark_pool.back();
    ctx->mark_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  return e;
}

// retire completed marks; returns how many completed
static int comm_marks_poll(pb_ctx* ctx) {
  int done = 0;
  for (auto it = ctx->comm_marks.begin(); it != ctx->comm_marks.end();) {
    if (hipEventQuery(*it) == hipSuccess) {
      ctx->mark_pool.push_back(*it);
      it = ctx->comm_marks.erase(it);
      ++done;
    } else {
      ++it;
    }
  }
  return done;
}

CommScope::CommScope(pb_ctx* c, hipStream_t st, bool force) : ctx(c), s(st), mark(false) {
  const int every = std::max(1, tune("comm_mark_every", 4));
  mark = force || ctx->comm_groups++ % every == every - 1;
  if (mark && ctx->comm_marks.size() > 64) (void)comm_marks_poll(ctx);
}

static bool& unmarked_flag(pb_ctx* ctx, hipStream_t s) {
  return s == ctx->comm_stream ? ctx->unmarked_comm : ctx->unmarked_main;
}

static void push_mark(pb_ctx* ctx, hipStream_t s) {
  hipEvent_t e = take_mark_event(ctx);
  (void)hipEventRecord(e, s);
  ctx->comm_marks.push_back(e);
  unmarked_flag(ctx, s) = false;
}

CommScope::~CommScope() {
  if (mark) push_mark(ctx, s);
  else unmarked_flag(ctx, s) = true;
}

// before a host wait: a mark after the groups enqueued since each stream's last mark, so every
// enqueued group is behind some pending mark until it completes
static void mark_unmarked(pb_ctx* ctx) {
  if (ctx->unmarked_main) push_mark(ctx, ctx->stream);
  if (ctx->unmarked_comm) push_mark(ctx, ctx->comm_stream);
}

// Waits for query() to report completion. On a split context the wait is bounded: it fails with
// PB_ERR_COMM when a communication mark (CommScope) is pending and none has completed for longer
// than PB_COMM_TIMEOUT_MS (a dead or stalled peer), or on an RCCL asynchronous error. Local work
// queued ahead of the wait with no communication behind it does not count, however long it runs.
template <class Query>
static int bounded_wait(pb_ctx* ctx, Query query, const char* what) {
  const int64_t t0 = now_ms();
  // after a failure, drain for a short while only (never block teardown on a dead peer)
  const int64_t limit_ms = ctx->comm_failed ? 5000 : ctx->comm_timeout_ms;
  mark_unmarked(ctx);
  (void)comm_marks_poll(ctx);
  int64_t progress_ms = t0;  // the last time communication was seen to progress (or none pending)
  for (int64_t spin = 0;; ++spin) {
    const hipError_t e = query();
    if (e == hipSuccess) return ctx->comm_failed ? set_error(PB_ERR_COMM, "%s after a "
                                                             "communication failure", what)
                                                 : PB_OK;
    if (e != hipErrorNotReady)
      return set_error(PB_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    if ((spin & 63) == 63) {
      if (ctx->comm && !ctx->comm_failed) {
        ncclResult_t ar = ncclSuccess;
        if (ncclCommGetAsyncError(ctx->comm, &ar) == ncclSuccess && ar != ncclSuccess &&
            ar != ncclInProgress)
          return comm_fail(ctx, "%s: RCCL asynchronous error: %s", what, ncclGetErrorString(ar));
      }
      if (ctx->comm_failed) {
        if (now_ms() - t0 > limit_ms)
          return set_error(PB_ERR_COMM, "%s: still pending after a communication failure", what);
      } else {
        const int64_t now = now_ms();
        if (comm_marks_poll(ctx) > 0 || ctx->comm_marks.empty()) progress_ms = now;
        if (now - progress_ms > limit_ms)
          return comm_fail(ctx, "%s: communication pending with no progress for %lld ms "
                           "(PB_COMM_TIMEOUT_MS); a peer rank is dead or stalled", what,
                           (long long)(now - progress_ms));
      }
    }
    if (spin > 4096) {  // past the first few hundred microseconds: back off
      timespec ts{0, 50000};
      nanosleep(&ts, nullptr);
    }
  }
}

int wait_stream(pb_ctx* ctx, hipStream_t s, const char* what) {
  if (!ctx->split && !ctx->comm_failed) {
    PB_HIP(hipStreamSynchronize(s));
    return PB_OK;
  }
  return bounded_wait(ctx, [s] { return hipStreamQuery(s); }, what);
}

int wait_event(pb_ctx* ctx, hipEvent_t ev, const char* what) {
  if (!ctx->split && !ctx->comm_failed) {
    PB_HIP(hipEventSynchronize(ev));
    return PB_OK;
  }
  return bounded_wait(ctx, [ev] { return hipEventQuery(ev); }, what);
}

// ---- communication ----
int halo_exchange(pb_grid* g, const double* lo, const double* hi) {
  pb_ctx* ctx = g->ctx;
  PB_COMM_OK(ctx);
  ScopedTimer tm(ctx, "halo");
  const int64_t cnt = g->plane;
  if (!ctx->split) {
    PB_HIP(hipMemcpyAsync(g->ghost_lo, hi, cnt * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
    PB_HIP(hipMemcpyAsync(g->ghost_hi, lo, cnt * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
    return PB_OK;
  }
  const int down = (ctx->rank + ctx->nranks - 1) % ctx->nranks;
  const int up = (ctx->rank + 1) % ctx->nranks;
  if (ctx->h_sendrecv) {
    double* s_lo = g->h_stage;
    double* s_hi = g->h_stage + cnt;
    double* r_lo = g->h_stage + 2 * cnt;
    double* r_hi = g->h_stage + 3 * cnt;
    PB_HIP(hipMemcpyAsync(s_lo, lo, cnt * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    PB_HIP(hipMemcpyAsync(s_hi, hi, cnt * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    PB_SYNC(ctx, "halo staging");
    if (ctx->h_sendrecv(ctx->h_user, s_lo, s_hi, r_lo, r_hi, cnt) != 0)
      return comm_fail(ctx, "host sendrecv callback failed");
    PB_HIP(hipMemcpyAsync(g->ghost_lo, r_lo, cnt * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    PB_HIP(hipMemcpyAsync(g->ghost_hi, r_hi, cnt * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    return PB_OK;
  }
  // Two phases whose issue order pairs correctly even when down == up (2 ranks):
  //   (1) send my lowest plane down, receive the plane above me from up  -> ghost_hi
  //   (2) send my highest plane up,  receive the plane below me from down -> ghost_lo
  CommScope cs(ctx, ctx->stream);
  PB_NCCL(ncclGroupStart());
  PB_NCCL(ncclSend(lo, (size_t)cnt, ncclDouble, down, ctx->comm, ctx->stream));
  PB_NCCL(ncclRecv(g->ghost_hi, (size_t)cnt, ncclDouble, up, ctx->comm, ctx->stream));
  PB_NCCL(ncclSend(hi, (size_t)cnt, ncclDouble, up, ctx->comm, ctx->stream));
  PB_NCCL(ncclRecv(g->ghost_lo, (size_t)cnt, ncclDouble, down, ctx->comm, ctx->stream));
  PB_NCCL(ncclGroupEnd());
  return PB_OK;
}

int halo_exchange_n(pb_grid* g, const double* lo, const double* hi, int np, double* rlo,
                    double* rhi) {
  pb_ctx* ctx = g->ctx;
  PB_COMM_OK(ctx);
  ScopedTimer tm(ctx, "halo");
  const int64_t cnt = (int64_t)np * g->plane;
  const size_t bytes = (size_t)cnt * sizeof(double);
  if (!ctx->split) {
    PB_HIP(hipMemcpyAsync(rlo, hi, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    PB_HIP(hipMemcpyAsync(rhi, lo, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    return PB_OK;
  }
  const int down = (ctx->rank + ctx->nranks - 1) % ctx->nranks;
  const int up = (ctx->rank + 1) % ctx->nranks;
  if (ctx->h_sendrecv) {
    if (np > 3) return set_error(PB_ERR_UNSUPPORTED, "host halo of %d planes", np);
    if (!g->h_stage2)  // up to three planes each way (the fused MG pre-pass's b ghosts)
      PB_HIP(hipHostMalloc(&g->h_stage2, 12 * (size_t)g->plane * sizeof(double),
                           hipHostMallocDefault));
    double* s_lo = g->h_stage2;
    double* s_hi = s_lo + cnt;
    double* r_lo = s_hi + cnt;
    double* r_hi = r_lo + cnt;
    PB_HIP(hipMemcpyAsync(s_lo, lo, bytes, hipMemcpyDeviceToHost, ctx->stream));
    PB_HIP(hipMemcpyAsync(s_hi, hi, bytes, hipMemcpyDeviceToHost, ctx->stream));
    PB_SYNC(ctx, "halo staging");
    if (ctx->h_sendrecv(ctx->h_user, s_lo, s_hi, r_lo, r_hi, cnt) != 0)
      return comm_fail(ctx, "host sendrecv callback failed");
    PB_HIP(hipMemcpyAsync(rlo, r_lo, bytes, hipMemcpyHostToDevice, ctx->stream));
    PB_HIP(hipMemcpyAsync(rhi, r_hi, bytes, hipMemcpyHostToDevice, ctx->stream));
    return PB_OK;
  }
  // the two-phase order of halo_exchange (pairs correctly when down == up)
  CommScope cs(ctx, ctx->stream);
  PB_NCCL(ncclGroupStart());
  PB_NCCL(ncclSend(lo, (size_t)cnt, ncclDouble, down, ctx->comm, ctx->stream));
  PB_NCCL(ncclRecv(rhi, (size_t)cnt, ncclDouble, up, ctx->comm, ctx->stream));
  PB_NCCL(ncclSend(hi, (size_t)cnt, ncclDouble, up, ctx->comm, ctx->stream));
  PB_NCCL(ncclRecv(rlo, (size_t)cnt, ncclDouble, down, ctx->comm, ctx->stream));
  PB_NCCL(ncclGroupEnd());
  return PB_OK;
}

int halo_begin(pb_grid* g, const double* lo, const double* hi) {
  pb_ctx* ctx = g->ctx;
  PB_COMM_OK(ctx);
  if (!ctx->split || !ctx->comm) return halo_exchange(g, lo, hi);
  const int64_t cnt = g->plane;
  const int down = (ctx->rank + ctx->nranks - 1) % ctx->nranks;
  const int up = (ctx->rank + 1) % ctx->nranks;
  PB_HIP(hipEventRecord(ctx->ev_ready, ctx->stream));
  PB_HIP(hipStreamWaitEvent(ctx->comm_stream, ctx->ev_ready, 0));
  // "halo_comm": the exchange itself on the comm stream (overlapped with interior planes)
  hipEvent_t tev = nullptr;
  const bool timed = ctx->timing && timer_wanted(ctx, "halo_comm");
  if (timed) timer_begin(ctx, "halo_comm", &tev, ctx->comm_stream);
  {
    CommScope cs(ctx, ctx->comm_stream);
    PB_NCCL(ncclGroupStart());
    PB_NCCL(ncclSend(lo, (size_t)cnt, ncclDouble, down, ctx->comm, ctx->comm_stream));
    PB_NCCL(ncclRecv(g->ghost_hi, (size_t)cnt, ncclDouble, up, ctx->comm, ctx->comm_stream));
    PB_NCCL(ncclSend(hi, (size_t)cnt, ncclDouble, up, ctx->comm, ctx->comm_stream));
    PB_NCCL(ncclRecv(g->ghost_lo, (size_t)cnt, ncclDouble, down, ctx->comm, ctx->comm_stream));
    PB_NCCL(ncclGroupEnd());
  }
  if (timed) timer_end(ctx, "halo_comm", tev, ctx->comm_stream);
  PB_HIP(hipEventRecord(ctx->ev_done, ctx->comm_stream));
  return PB_OK;
}

int halo_begin_after(pb_grid* g, const double* lo, const double* hi,
                     const std::function<int(hipStream_t)>& pre) {
  pb_ctx* ctx = g->ctx;
  PB_COMM_OK(ctx);
  if (!ctx->split || !ctx->comm) {
    PB_TRY(pre(ctx->stream));
    return halo_exchange(g, lo, hi);
  }
  PB_HIP(hipEventRecord(ctx->ev_ready, ctx->stream));
  PB_HIP(hipStreamWaitEvent(ctx->comm_stream, ctx->ev_ready, 0));
  PB_TRY(pre(ctx->comm_stream));
  const int64_t cnt = g->plane;
  const int down = (ctx->rank + ctx->nranks - 1) % ctx->nranks;
  const int up = (ctx->rank + 1) % ctx->nranks;
  hipEvent_t tev = nullptr;
  const bool timed = ctx->timing && timer_wanted(ctx, "halo_comm");
  if (timed) timer_begin(ctx, "halo_comm", &tev, ctx->comm_stream);
  {
    CommScope cs(ctx, ctx->comm_stream);
    PB_NCCL(ncclGroupStart());
    PB_NCCL(ncclSend(lo, (size_t)cnt, ncclDouble, down, ctx->comm, ctx->comm_stream));
    PB_NCCL(ncclRecv(g->ghost_hi, (size_t)cnt, ncclDouble, up, ctx->comm, ctx->comm_stream));
    PB_NCCL(ncclSend(hi, (size_t)cnt, ncclDouble, up, ctx->comm, ctx->comm_stream));
    PB_NCCL(ncclRecv(g->ghost_lo, (size_t)cnt, ncclDouble, down, ctx->comm, ctx->comm_stream));
    PB_NCCL(ncclGroupEnd());
  }
  if (timed) timer_end(ctx, "halo_comm", tev, ctx->comm_stream);
  PB_HIP(hipEventRecord(ctx->ev_done, ctx->comm_stream));
  return PB_OK;
}

int halo_end(pb_grid* g) {
  pb_ctx* ctx = g->ctx;
  if (!ctx->split || !ctx->comm) return PB_OK;
  PB_HIP(hipStreamWaitEvent(ctx->stream, ctx->ev_done, 0));
  return PB_OK;
}

int alltoallv_device(pb_ctx* ctx, const double* send, const int64_t* scount, double* recv,
                     const int64_t* rcount, bool skip_self) {
  PB_COMM_OK(ctx);
  ScopedTimer tm(ctx, "alltoallv");
  const int P = ctx->nranks;
  std::vector<int64_t> so(P + 1, 0), ro(P + 1, 0);
  for (int p = 0; p < P; ++p) {
    so[p + 1] = so[p] + scount[p];
    ro[p + 1] = ro[p] + rcount[p];
  }
  if (P == 1 && !ctx->comm) {
    if (scount[0])
      PB_HIP(hipMemcpyAsync(recv, send, scount[0] * sizeof(double), hipMemcpyDeviceToDevice,
                            ctx->stream));
    return PB_OK;
  }
  if (ctx->comm) {
    CommScope cs(ctx, ctx->stream);
    PB_NCCL(ncclGroupStart());
    for (int p = 0; p < P; ++p) {
      if (p == ctx->rank) continue;
      if (scount[p])
        PB_NCCL(ncclSend(send + so[p], (size_t)scount[p], ncclDouble, p, ctx->comm, ctx->stream));
      if (rcount[p])
        PB_NCCL(ncclRecv(recv + ro[p], (size_t)rcount[p], ncclDouble, p, ctx->comm, ctx->stream));
    }
    PB_NCCL(ncclGroupEnd());
    const int me = ctx->rank;
    if (scount[me] && !skip_self)
      PB_HIP(hipMemcpyAsync(recv + ro[me], send + so[me], scount[me] * sizeof(double),
                            hipMemcpyDeviceToDevice, ctx->stream));
    return PB_OK;
  }
  if (!ctx->h_alltoallv)
    return set_error(PB_ERR_COMM, "host transport without an alltoallv callback");
  const size_t need = (size_t)(so[P] + ro[P]);
  if (need > ctx->h_a2a_len) {
    if (ctx->h_a2a) PB_HIP(hipHostFree(ctx->h_a2a));
    ctx->h_a2a = nullptr;
    PB_HIP(hipHostMalloc(&ctx->h_a2a, need * sizeof(double), hipHostMallocDefault));
    ctx->h_a2a_len = need;
  }
  double* hs = ctx->h_a2a;
  double* hr = ctx->h_a2a + so[P];
  PB_HIP(hipMemcpyAsync(hs, send, so[P] * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  PB_SYNC(ctx, "all-to-all staging");
  if (ctx->h_alltoallv(ctx->h_a2a_user, hs, scount, hr, rcount) != 0)
    return comm_fail(ctx, "host alltoallv callback failed");
  if (!skip_self) {
    PB_HIP(hipMemcpyAsync(recv, hr, ro[P] * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  } else {
    // the self block is already in place (the pack wrote it there): the staged buffers carried
    // a stale copy through the callback, which is not brought back -- the same offsets
    // (YSlabPlan::self_shift) as the RCCL path, on a transport the one-GPU tests can run
    const int me = ctx->rank;
    if (ro[me])
      PB_HIP(hipMemcpyAsync(recv, hr, ro[me] * sizeof(double), hipMemcpyHostToDevice,
                            ctx->stream));
    if (ro[P] > ro[me + 1])
      PB_HIP(hipMemcpyAsync(recv + ro[me + 1], hr + ro[me + 1],
                            (ro[P] - ro[me + 1]) * sizeof(double), hipMemcpyHostToDevice,
                            ctx->stream));
  }
  PB_SYNC(ctx, "all-to-all staging");
  return PB_OK;
}

int ctx_scratch(pb_ctx* ctx, size_t n, double** out) {
  if (n > ctx->scratch_len) {
    PB_SYNC(ctx, "scratch");  // previous users of the old buffer are done
    if (ctx->scratch) PB_HIP(hipFree(ctx->scratch));
    ctx->scratch = nullptr;
    ctx->scratch_len = 0;
    if (hipMalloc(&ctx->scratch, n * sizeof(double)) != hipSuccess)
      return set_error(PB_ERR_ALLOC, "scratch of %zu doubles: out of device memory", n);
    ctx->scratch_len = n;
  }
  *out = ctx->scratch;
  return PB_OK;
}

int allreduce_device(pb_ctx* ctx, double* d_vals, int count) {
  if (!ctx->split) return PB_OK;
  PB_COMM_OK(ctx);
  ScopedTimer tm(ctx, "allreduce");
  if (ctx->h_allreduce) {
    // test hook: a peer that never answers (ms < 0: inside an unforced group, which carries a
    // progress mark only as every comm_mark_every-th group does)
    if (const int stall = tune("comm_stall_test_ms", 0)) {
      CommScope cs(ctx, ctx->stream, stall > 0);
      PB_TRY(launch_comm_stall(ctx, ctx->stream, stall > 0 ? stall : -stall));
    }
    PB_HIP(hipMemcpyAsync(ctx->h_scalars + 16, d_vals, count * sizeof(double), hipMemcpyDeviceToHost,
                          ctx->stream));
    PB_SYNC(ctx, "allreduce staging");
    if (ctx->h_allreduce(ctx->h_user, ctx->h_scalars + 16, count) != 0)
      return comm_fail(ctx, "host allreduce callback failed");
    PB_HIP(hipMemcpyAsync(d_vals, ctx->h_scalars + 16, count * sizeof(double), hipMemcpyHostToDevice,
                          ctx->stream));
    PB_SYNC(ctx, "allreduce staging");  // staging buffer is reused by the next call
    return PB_OK;
  }
  CommScope cs(ctx, ctx->stream);
  PB_NCCL(ncclAllReduce(d_vals, d_vals, (size_t)count, ncclDouble, ncclSum, ctx->comm, ctx->stream));
  return PB_OK;
}

}  // namespace pb

using namespace pb;

namespace pb {
// grid with an explicit slab [k0, k0 + nzl) (multigrid levels: the fine partition halved)
int grid_create_part(pb_ctx* ctx, const int64_t n[3], const double L[3], int64_t k0, int64_t nzl,
                     pb_grid** out) {
  PB_HIP(hipSetDevice(ctx->device));
  pb_grid* g = new pb_grid();
  g->ctx = ctx;
  for (int d = 0; d < 3; ++d) {
    g->n[d] = n[d];
    g->L[d] = L ? L[d] : 1.0;
    g->h[d] = g->L[d] / (double)n[d];  // src/example.f90:33-35
  }
  g->k0 = k0;
  g->nzl = nzl;
  g->plane = n[0] * n[1];
  g->nlocal = g->plane * g->nzl;
  const size_t pb = (size_t)g->plane * sizeof(double);
  double* ghosts = nullptr;
  if (hipMalloc(&ghosts, 4 * pb) != hipSuccess) {
    delete g;
    return set_error(PB_ERR_ALLOC, "ghost planes: out of device memory");
  }
  g->ghost_lo = ghosts;
  g->ghost_hi = ghosts + g->plane;
  g->bnd_lo = ghosts + 2 * g->plane;
  g->bnd_hi = ghosts + 3 * g->plane;
  if (ctx->h_sendrecv && hipHostMalloc(&g->h_stage, 4 * pb, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipFree(ghosts);
    delete g;
    return set_error(PB_ERR_ALLOC, "host staging planes: out of pinned memory");
  }
  *out = g;
  return PB_OK;
}
}  // namespace pb

extern "C" {

const char* pb_last_error(void) { return g_err; }

// src/coefficients.f90:22-35 (invdx2 = 1/dx**2; [invdx2, -2 invdx2, invdx2])
int pb_lapl_1d_coeffs(double dx, double c[3]) {
  PB_CHECK_ARG(c, "c is NULL");
  const double inv = 1.0 / (dx * dx);
  c[0] = inv;
  c[1] = -2.0 * inv;
  c[2] = inv;
  return PB_OK;
}

// src/coefficients.f90:38-48: the 3x3x3 box (column-major, i fastest), zero but for the three
// 1-D lines through the centre, each added onto the box in x, y, z order
int pb_lapl_star_coeffs(double dx, double dy, double dz, double c[27]) {
  PB_CHECK_ARG(c, "c is NULL");
  double l[3][3];
  pb_lapl_1d_coeffs(dx, l[0]);
  pb_lapl_1d_coeffs(dy, l[1]);
  pb_lapl_1d_coeffs(dz, l[2]);
  for (int m = 0; m < 27; ++m) c[m] = 0.0;
  for (int t = 0; t < 3; ++t) c[t + 3 * 1 + 9 * 1] = c[t + 3 * 1 + 9 * 1] + l[0][t];
  for (int t = 0; t < 3; ++t) c[1 + 3 * t + 9 * 1] = c[1 + 3 * t + 9 * 1] + l[1][t];
  for (int t = 0; t < 3; ++t) c[1 + 3 * 1 + 9 * t] = c[1 + 3 * 1 + 9 * t] + l[2][t];
  return PB_OK;
}

int pb_version(int* major, int* minor) {
  if (major) *major = PB_VERSION_MAJOR;
  if (minor) *minor = PB_VERSION_MINOR;
  return PB_OK;
}

// ---------------------------------------------------------------------------------------------
// Context
// ---------------------------------------------------------------------------------------------
int pb_comm_unique_id(unsigned char uid[128]) {
  PB_CHECK_ARG(uid, "uid is NULL");
  ncclUniqueId id;
  PB_NCCL(ncclGetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  memcpy(uid, &id, 128);
  return PB_OK;
}

namespace {
// ncclCommInitRank bounded by PB_COMM_TIMEOUT_MS. RCCL's bootstrap waits for every rank without
// a limit, so a peer that dies during start-up (or a rank that was handed a stale unique id)
// would block the caller forever. The init runs on a helper thread; this thread waits for it with
// the context's timeout and, on expiry, returns PB_ERR_COMM. There is no communicator handle to
// abort before ncclCommInitRank returns, so a timed-out helper is detached: should the init ever
// complete late, the helper destroys the communicator it made. The communicator itself is an
// ordinary blocking one, so the halo / allreduce calls of the hot path are unchanged.
struct CommInit {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false, abandoned = false;
  ncclResult_t rc = ncclSuccess;
  ncclComm_t comm = nullptr;
};

int comm_init_bounded(pb_ctx* ctx, int nranks, const ncclUniqueId& id, int rank) {
  auto st = std::make_shared<CommInit>();
  const int device = ctx->device;
  std::thread th([st, device, nranks, id, rank] {
    (void)hipSetDevice(device);
    ncclComm_t c = nullptr;
    const ncclResult_t r = ncclCommInitRank(&c, nranks, id, rank);
    std::lock_guard<std::mutex> lk(st->mu);
    st->rc = r;
    st->comm = c;
    st->done = true;
    if (st->abandoned && r == ncclSuccess && c) (void)ncclCommDestroy(c);
    st->cv.notify_all();
  });
  std::unique_lock<std::mutex> lk(st->mu);
  const bool ok = st->cv.wait_for(lk, std::chrono::milliseconds(ctx->comm_timeout_ms),
                                  [&] { return st->done; });
  if (!ok) {
    st->abandoned = true;
    lk.unlock();
    th.detach();
    fprintf(stderr, "[poissbox rank %d] RCCL communicator init: not every rank joined within "
            "%lld ms\n", rank, (long long)ctx->comm_timeout_ms);
    return set_error(PB_ERR_COMM, "RCCL communicator init (rank %d of %d): not every rank joined "
                     "within %lld ms (PB_COMM_TIMEOUT_MS); a peer died during start-up or holds "
                     "another unique id", rank, nranks, (long long)ctx->comm_timeout_ms);
  }
  lk.unlock();
  th.join();
  if (st->rc != ncclSuccess)
    return set_error(PB_ERR_COMM, "ncclCommInitRank (rank %d of %d): %s", rank, nranks,
                     ncclGetErrorString(st->rc));
  ctx->comm = st->comm;
  return PB_OK;
}
}  // namespace

int pb_ctx_create(int device, int rank, int nranks, const unsigned char* uid, pb_ctx** out) {
  PB_CHECK_ARG(out, "ctx out is NULL");
  PB_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank/nranks");
  int ndev = 0;
  PB_HIP(hipGetDeviceCount(&ndev));
  PB_CHECK_ARG(device >= 0 && device < ndev, "device index out of range");
  PB_HIP(hipSetDevice(device));
  pb_ctx* ctx = new pb_ctx();
  ctx->device = device;
  ctx->rank = rank;
  ctx->nranks = nranks;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
      cus > 0)
    ctx->num_cus = cus;
  ctx->roctx = env_int("PB_ROCTX", 0) != 0;
  ctx->comm_timeout_ms = std::max(1, env_int("PB_COMM_TIMEOUT_MS", 180000));
  ctx->partials_cap = (int64_t)1 << 20;  // doubles: room for 131072 blocks x 8 sums
  // streams, events and the scalar buffers; a failure tears the partial context down below
  auto resources = [&]() -> int {
    PB_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    PB_HIP(hipStreamCreateWithFlags(&ctx->comm_stream, hipStreamNonBlocking));
    PB_HIP(hipEventCreateWithFlags(&ctx->ev_ready, hipEventDisableTiming));
    PB_HIP(hipEventCreateWithFlags(&ctx->ev_done, hipEventDisableTiming));
    PB_HIP(hipMalloc(&ctx->d_partials, ctx->partials_cap * sizeof(double)));
    PB_HIP(hipMalloc(&ctx->d_scalars, 64 * sizeof(double)));
    PB_HIP(hipMemsetAsync(ctx->d_scalars, 0, 64 * sizeof(double), ctx->stream));
    PB_HIP(hipHostMalloc(&ctx->h_scalars, 64 * sizeof(double), hipHostMallocDefault));
    return PB_OK;
  };
  int rc = resources();
  if (rc == PB_OK && nranks > 1 && uid) {
    ncclUniqueId id;
    memcpy(&id, uid, 128);
    rc = comm_init_bounded(ctx, nranks, id, rank);
  }
  ctx->split = nranks > 1;
  if (rc == PB_OK && nranks == 1 && tune("force_comm", 0)) {
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    rc = r == ncclSuccess ? comm_init_bounded(ctx, 1, id, 0)
                          : set_error(PB_ERR_COMM, "ncclGetUniqueId: %s", ncclGetErrorString(r));
    ctx->split = true;
  }
  if (rc != PB_OK) {
    std::string msg = g_err;
    ctx->split = false;  // nothing communicating is queued: plain teardown
    pb_ctx_destroy(ctx);
    return set_error(rc, "%s", msg.c_str());
  }
  *out = ctx;
  return PB_OK;
}

int pb_ctx_comm_info(const pb_ctx* ctx, int* transport, int* comm_nranks, int* comm_rank) {
  PB_CHECK_ARG(ctx, "ctx is NULL");
  int t = PB_TRANSPORT_NONE, n = 1, r = 0;
  if (ctx->comm) {
    t = PB_TRANSPORT_RCCL;
    PB_NCCL(ncclCommCount(ctx->comm, &n));
    PB_NCCL(ncclCommUserRank(ctx->comm, &r));
  } else if (ctx->h_sendrecv) {
    t = PB_TRANSPORT_HOST;
    n = ctx->nranks;
    r = ctx->rank;
  }
  if (transport) *transport = t;
  if (comm_nranks) *comm_nranks = n;
  if (comm_rank) *comm_rank = r;
  return PB_OK;
}

int pb_ctx_set_host_transport(pb_ctx* ctx, pb_sendrecv_fn sr, pb_allreduce_fn ar, void* user) {
  PB_CHECK_ARG(ctx && sr && ar, "bad host transport");
  ctx->h_sendrecv = sr;
  ctx->h_allreduce = ar;
  ctx->h_user = user;
  return PB_OK;
}

int pb_ctx_set_host_alltoallv(pb_ctx* ctx, pb_alltoallv_fn fn, void* user) {
  PB_CHECK_ARG(ctx && fn, "bad host alltoallv");
  ctx->h_alltoallv = fn;
  ctx->h_a2a_user = user;
  return PB_OK;
}

int pb_ctx_get_rank(const pb_ctx* ctx, int* rank, int* nranks) {
  PB_CHECK_ARG(ctx, "ctx is NULL");
  if (rank) *rank = ctx->rank;
  if (nranks) *nranks = ctx->nranks;
  return PB_OK;
}

int pb_ctx_sync(pb_ctx* ctx) {
  PB_CHECK_ARG(ctx, "ctx is NULL");
  PB_SYNC(ctx, "pb_ctx_sync");
  return PB_OK;
}

int pb_ctx_barrier(pb_ctx* ctx) {
  PB_CHECK_ARG(ctx, "ctx is NULL");
  PB_SYNC(ctx, "pb_ctx_barrier");
  if (ctx->split) {
    PB_TRY(allreduce_device(ctx, ctx->d_scalars + 32, 1));
    PB_SYNC(ctx, "pb_ctx_barrier");
  }
  return PB_OK;
}

int pb_ctx_comm_status(const pb_ctx* ctx, int* failed) {
  PB_CHECK_ARG(ctx && failed, "bad args");
  *failed = ctx->comm_failed ? 1 : 0;
  return PB_OK;
}

int pb_ctx_destroy(pb_ctx* ctx) {
  if (!ctx) return PB_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)wait_stream(ctx, ctx->stream, "pb_ctx_destroy");
  if (ctx->comm_stream) (void)wait_stream(ctx, ctx->comm_stream, "pb_ctx_destroy");
  if (!ctx->comm_failed) timers_collect(ctx);
  for (hipEvent_t e : ctx->event_pool) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->comm_marks) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->mark_pool) (void)hipEventDestroy(e);
  if (ctx->h_stall) (void)hipHostFree(ctx->h_stall);
  if (ctx->comm) ncclCommDestroy(ctx->comm);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->h_a2a) (void)hipHostFree(ctx->h_a2a);
  transport_destroy(ctx);
  (void)hipFree(ctx->d_partials);
  (void)hipFree(ctx->d_scalars);
  if (ctx->h_scalars) (void)hipHostFree(ctx->h_scalars);
  if (ctx->ev_ready) (void)hipEventDestroy(ctx->ev_ready);
  if (ctx->ev_done) (void)hipEventDestroy(ctx->ev_done);
  if (ctx->comm_stream) (void)hipStreamDestroy(ctx->comm_stream);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  (void)hipGetLastError();  // a teardown error is not the next launch's error
  return PB_OK;
}

int pb_tune_set(const char* name, int value) {
  PB_CHECK_ARG(name, "tuning name is NULL");
  const int i = tune_index(name);
  if (i < 0) return set_error(PB_ERR_ARG, "unknown tuning parameter '%s'", name);
  g_tune_val[i].store(value, std::memory_order_relaxed);
  if (g_tune_set[i].exchange(1, std::memory_order_acq_rel) == 0)
    g_tune_nset.fetch_add(1, std::memory_order_acq_rel);
  return PB_OK;
}

int pb_tune_get(const char* name, int* value, int* is_set) {
  PB_CHECK_ARG(name && value, "bad tuning args");
  const int i = tune_index(name);
  if (i < 0) return set_error(PB_ERR_ARG, "unknown tuning parameter '%s'", name);
  const bool set = g_tune_set[i].load(std::memory_order_acquire) != 0;
  if (is_set) *is_set = set;
  if (set) *value = g_tune_val[i].load(std::memory_order_relaxed);
  return PB_OK;
}

int pb_tune_reset(void) {
  for (int i = 0; i < kNumTune; ++i) g_tune_set[i].store(0, std::memory_order_release);
  g_tune_nset.store(0, std::memory_order_release);
  return PB_OK;
}

int pb_ctx_set_timing(pb_ctx* ctx, int enable) {
  return pb_ctx_set_timing_filter(ctx, enable, nullptr, 1);
}

int pb_ctx_set_timing_filter(pb_ctx* ctx, int enable, const char* only, int every) {
  PB_CHECK_ARG(ctx, "ctx is NULL");
  ctx->timing = enable != 0;
  // only (comma-separated phase names, or NULL / ""): record events around those phases only, and
  // of each such phase around one launch in `every`, so a timed region is not perturbed by event
  // records around every kernel
  ctx->timing_only.clear();
  ctx->timer_calls.clear();
  ctx->timing_every = std::max(1, every);
  if (enable && only && *only) {
    std::string cur;
    for (const char* c = only;; ++c) {
      if (*c == ',' || *c == '\0') {
        if (!cur.empty()) ctx->timing_only.push_back(cur);
        cur.clear();
        if (!*c) break;
      } else {
        cur += *c;
      }
    }
  }
  return PB_OK;
}

int pb_ctx_get_timing(pb_ctx* ctx, const char* name, double* total_ms, int64_t* count) {
  PB_CHECK_ARG(ctx && name, "bad args");
  timers_collect(ctx);
  auto it = ctx->timers.find(name);
  if (total_ms) *total_ms = it == ctx->timers.end() ? 0.0 : it->second.total_ms;
  if (count) *count = it == ctx->timers.end() ? 0 : it->second.count;
  return PB_OK;
}

int pb_ctx_get_timing_samples(pb_ctx* ctx, const char* name, float* ms, int64_t cap,
                               int64_t* count) {
  PB_CHECK_ARG(ctx && name && count && (ms || cap == 0) && cap >= 0, "bad args");
  timers_collect(ctx);
  auto it = ctx->timers.find(name);
  const int64_t n = it == ctx->timers.end() ? 0 : (int64_t)it->second.samples.size();
  for (int64_t i = 0; i < std::min(n, cap); ++i) ms[i] = it->second.samples[(size_t)i];
  *count = n;
  return PB_OK;
}

int pb_ctx_reset_timing(pb_ctx* ctx) {
  PB_CHECK_ARG(ctx, "ctx is NULL");
  timers_collect(ctx);
  ctx->timers.clear();
  return PB_OK;
}

int pb_ctx_copy_probe(pb_ctx* ctx, int64_t n, int reps, double* best_gbps, double* median_gbps) {
  PB_CHECK_ARG(ctx && n >= 2 && reps >= 1 && best_gbps && median_gbps, "bad copy probe args");
  PB_HIP(hipSetDevice(ctx->device));
  std::vector<float> ms;
  PB_TRY(copy_probe(ctx, n, reps, ms));
  std::sort(ms.begin(), ms.end());
  const double bytes = 16.0 * (double)(n / 2 * 2);
  *best_gbps = bytes / (ms.front() * 1e-3) / 1e9;
  *median_gbps = bytes / (ms[ms.size() / 2] * 1e-3) / 1e9;
  return PB_OK;
}

int pb_vec_copy_probe(const pb_vec* x, pb_vec* y, int reps, double* best_gbps,
                      double* median_gbps) {
  PB_CHECK_ARG(x && y && x != y && reps >= 1 && best_gbps && median_gbps,
               "bad copy probe args");
  PB_CHECK_ARG(x->grid == y->grid && x->nlocal == y->nlocal, "vectors of different grids");
  pb_ctx* ctx = x->grid->ctx;
  PB_HIP(hipSetDevice(ctx->device));
  const int64_t n = x->nlocal / 2 * 2;
  PB_CHECK_ARG(n >= 2, "vector too short for the copy probe");
  std::vector<float> ms;
  PB_TRY(copy_probe(ctx, n, reps, ms, x->d, y->d));
  std::sort(ms.begin(), ms.end());
  const double bytes = 16.0 * (double)n;
  *best_gbps = bytes / (ms.front() * 1e-3) / 1e9;
  *median_gbps = bytes / (ms[ms.size() / 2] * 1e-3) / 1e9;
  return PB_OK;
}

// ---------------------------------------------------------------------------------------------
// Grid
// ---------------------------------------------------------------------------------------------
int pb_slab_partition(int64_t nz, int nranks, int rank, int64_t* kstart, int64_t* nk) {
  PB_CHECK_ARG(nz >= 1 && nranks >= 1 && rank >= 0 && rank < nranks, "bad partition args");
  const int64_t q = nz / nranks, r = nz % nranks;
  const int64_t mine = q + (rank < r ? 1 : 0);
  const int64_t start = rank * q + (rank < r ? rank : r);
  if (kstart) *kstart = start;
  if (nk) *nk = mine;
  return PB_OK;
}

int pb_grid_create(pb_ctx* ctx, const int64_t n[3], const double L[3], pb_grid** out) {
  PB_CHECK_ARG(ctx && n && out, "bad grid args");
  for (int d = 0; d < 3; ++d) PB_CHECK_ARG(n[d] >= 3, "grid needs n >= 3 in every direction");
  PB_CHECK_ARG(n[0] < (1 << 30) && n[1] < (1 << 30), "nx, ny must fit in int32");
  PB_CHECK_ARG(n[2] >= ctx->nranks, "fewer z-planes than ranks");
  PB_CHECK_ARG(ctx->nranks == 1 || ctx->comm || ctx->h_sendrecv,
               "multi-rank context has neither RCCL nor a host transport");
  int64_t k0 = 0, nzl = 0;
  PB_TRY(pb_slab_partition(n[2], ctx->nranks, ctx->rank, &k0, &nzl));
  return pb::grid_create_part(ctx, n, L, k0, nzl, out);
}

int pb_grid_get_corners(const pb_grid* g, int64_t start[3], int64_t size[3]) {
  PB_CHECK_ARG(g, "grid is NULL");
  if (start) {
    start[0] = 0;
    start[1] = 0;
    start[2] = g->k0;
  }
  if (size) {
    size[0] = g->n[0];
    size[1] = g->n[1];
    size[2] = g->nzl;
  }
  return PB_OK;
}

int pb_grid_get_info(const pb_grid* g, int64_t n[3], double h[3], int64_t* nlocal) {
  PB_CHECK_ARG(g, "grid is NULL");
  for (int d = 0; d < 3; ++d) {
    if (n) n[d] = g->n[d];
    if (h) h[d] = g->h[d];
  }
  if (nlocal) *nlocal = g->nlocal;
  return PB_OK;
}

int pb_grid_destroy(pb_grid* g) {
  if (!g) return PB_OK;
  (void)wait_stream(g->ctx, g->ctx->stream, "pb_grid_destroy");
  (void)hipFree(g->ghost_lo);
  if (g->ghost2) (void)hipFree(g->ghost2);
  if (g->yslab_tab) (void)hipFree(g->yslab_tab);
  if (g->h_stage) (void)hipHostFree(g->h_stage);
  if (g->h_stage2) (void)hipHostFree(g->h_stage2);
  delete g;
  return PB_OK;
}

// ---------------------------------------------------------------------------------------------
// Vectors
// ---------------------------------------------------------------------------------------------
int pb_vec_create(pb_grid* g, pb_vec** out) {
  PB_CHECK_ARG(g && out, "bad vec args");
  pb_vec* v = new pb_vec();
  v->grid = g;
  v->nlocal = g->nlocal;
  if (field_alloc(&v->d, (size_t)v->nlocal * sizeof(double)) != hipSuccess) {
    delete v;
    return set_error(PB_ERR_ALLOC, "vector of %lld doubles: out of device memory",
                     (long long)g->nlocal);
  }
  const int rc = vec_fill(g->ctx, v->d, v->nlocal, 0.0);  // PETSc vectors start zeroed
  if (rc) {
    const std::string msg = pb_last_error();
    (void)pb_vec_destroy(v);
    return set_error(rc, "%s", msg.c_str());
  }
  *out = v;
  return PB_OK;
}

int pb_vec_duplicate(const pb_vec* v, pb_vec** out) {
  PB_CHECK_ARG(v, "vec is NULL");
  return pb_vec_create(v->grid, out);
}

int pb_vec_destroy(pb_vec* v) {
  if (!v) return PB_OK;
  (void)wait_stream(v->grid->ctx, v->grid->ctx->stream, "pb_vec_destroy");
  field_free(v->d);
  delete v;
  return PB_OK;
}

int pb_vec_set(pb_vec* v, double a) {
  PB_CHECK_ARG(v, "vec is NULL");
  return vec_fill(v->grid->ctx, v->d, v->nlocal, a);
}

static int same_layout(const pb_vec* a, const pb_vec* b) {
  return a && b && a->grid == b->grid;
}

int pb_vec_copy(const pb_vec* src, pb_vec* dst) {
  PB_CHECK_ARG(same_layout(src, dst), "vectors of different grids");
  if (src == dst) return PB_OK;
  PB_HIP(hipMemcpyAsync(dst->d, src->d, (size_t)src->nlocal * sizeof(double),
                        hipMemcpyDeviceToDevice, src->grid->ctx->stream));
  return PB_OK;
}

int pb_vec_axpy(pb_vec* y, double a, const pb_vec* x) {
  PB_CHECK_ARG(same_layout(x, y), "vectors of different grids");
  return vec_update(y->grid->ctx, 0, y->d, x->d, y->nlocal, a);
}

int pb_vec_aypx(pb_vec* y, double b, const pb_vec* x) {
  PB_CHECK_ARG(same_layout(x, y), "vectors of different grids");
  return vec_update(y->grid->ctx, 1, y->d, x->d, y->nlocal, b);
}

int pb_vec_scale(pb_vec* v, double a) {
  PB_CHECK_ARG(v, "vec is NULL");
  return vec_update(v->grid->ctx, 2, v->d, nullptr, v->nlocal, a);
}

int pb_vec_dot(const pb_vec* x, const pb_vec* y, double* out) {
  PB_CHECK_ARG(same_layout(x, y) && out, "bad dot args");
  return vec_reduce(x->grid->ctx, 1, x->d, y->d, x->nlocal, out);
}

int pb_vec_norm2(const pb_vec* v, double* out) {
  PB_CHECK_ARG(v && out, "bad norm args");
  double s = 0.0;
  PB_TRY(vec_reduce(v->grid->ctx, 1, v->d, v->d, v->nlocal, &s));
  *out = sqrt(s);
  return PB_OK;
}

int pb_vec_sum(const pb_vec* v, double* out) {
  PB_CHECK_ARG(v && out, "bad sum args");
  return vec_reduce(v->grid->ctx, 0, v->d, nullptr, v->nlocal, out);
}

int pb_vec_set_values_host(pb_vec* v, const double* owned) {
  PB_CHECK_ARG(v && owned, "bad set_values args");
  // stream-ordered after any pending work on the vector (e.g. the zero fill at creation)
  hipStream_t s = v->grid->ctx->stream;
  PB_HIP(hipMemcpyAsync(v->d, owned, (size_t)v->nlocal * sizeof(double), hipMemcpyHostToDevice, s));
  PB_TRY(wait_stream(v->grid->ctx, s, "pb_vec_set_values_host"));
  return PB_OK;
}

int pb_vec_get_values_host(const pb_vec* v, double* owned) {
  PB_CHECK_ARG(v && owned, "bad get_values args");
  hipStream_t s = v->grid->ctx->stream;
  PB_HIP(hipMemcpyAsync(owned, v->d, (size_t)v->nlocal * sizeof(double), hipMemcpyDeviceToHost, s));
  PB_TRY(wait_stream(v->grid->ctx, s, "pb_vec_get_values_host"));
  return PB_OK;
}

int pb_vec_set_random(pb_vec* v, uint64_t seed) {
  PB_CHECK_ARG(v, "vec is NULL");
  return vec_random(v->grid->ctx, v->d, v->nlocal, seed, v->grid->k0 * v->grid->plane);
}

int pb_vec_device_ptr(pb_vec* v, double** dptr, int64_t* nlocal) {
  PB_CHECK_ARG(v, "vec is NULL");
  if (dptr) *dptr = v->d;
  if (nlocal) *nlocal = v->nlocal;
  return PB_OK;
}

}  // extern "C"
