// pb_internal.hpp -- shared internals of libpoissbox_gpu (host runtime + HIP kernels, gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstdint>
#include <cstdio>
#include <deque>
#include <map>
#include <string>
#include <functional>
#include <vector>

#include "poissbox_gpu.h"

namespace pb {

// ---------------------------------------------------------------------------------------------
// Errors
// ---------------------------------------------------------------------------------------------
int set_error(int code, const char* fmt, ...);

#define PB_HIP(call)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess)                                                               \
      return ::pb::set_error(PB_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #call,     \
                             hipGetErrorString(e_));                                    \
  } while (0)

#define PB_NCCL(call)                                                                   \
  do {                                                                                  \
    ncclResult_t r_ = (call);                                                           \
    if (r_ != ncclSuccess)                                                              \
      return ::pb::set_error(PB_ERR_COMM, "%s:%d %s: %s", __FILE__, __LINE__, #call,    \
                             ncclGetErrorString(r_));                                   \
  } while (0)

#define PB_TRY(call)            \
  do {                          \
    int rc_ = (call);           \
    if (rc_ != PB_OK) return rc_; \
  } while (0)

#define PB_CHECK_ARG(cond, msg)                                  \
  do {                                                           \
    if (!(cond)) return ::pb::set_error(PB_ERR_ARG, "%s", msg);  \
  } while (0)

// ---------------------------------------------------------------------------------------------
// Kernel timing (HIP events on the context stream)
// ---------------------------------------------------------------------------------------------
struct TimerSlot {
  double total_ms = 0.0;
  int64_t count = 0;
  std::vector<float> samples;  // per-launch ms, the first kMaxTimerSamples since the last reset
};
constexpr size_t kMaxTimerSamples = 1 << 16;

struct CgFuse;
}  // namespace pb

struct pb_ctx {
  // device "done" flag of the KSP whose iteration is being enqueued (OpApplySkip): operator
  // kernels launched meanwhile exit at entry once it is set -- the host enqueues iterations
  // ahead of its lagged convergence poll, and an operator apply is the costly part of them
  const int* op_skip = nullptr;
  // CG fusions for the compact operator inside a stored-z CG iteration (CgFuse), set around one
  // operator apply like op_skip
  pb::CgFuse* cg_fuse = nullptr;
  int device = 0;
  int rank = 0;
  int nranks = 1;
  // decomposed code paths (halo exchange, allreduce, transposes): nranks > 1, or one rank with
  // PB_FORCE_COMM=1 (a 1-rank RCCL communicator: exercises the RCCL paths on a single GPU)
  bool split = false;
  hipStream_t stream = nullptr;
  hipStream_t comm_stream = nullptr;  // RCCL halo exchange, overlapped with interior planes
  hipStream_t engine_stream = nullptr;  // stencil-engine launches go here when set (EngineOn)
  hipEvent_t ev_ready = nullptr, ev_done = nullptr;
  ncclComm_t comm = nullptr;
  // bounded waits on split contexts (a dead or stalled peer must surface as PB_ERR_COMM, not a
  // hang): PB_COMM_TIMEOUT_MS per wait; after a failure the communicator is aborted and every
  // later collective call returns PB_ERR_COMM at once
  int64_t comm_timeout_ms = 180000;
  bool comm_failed = false;
  // device-side communication progress: an event after every 4th group of RCCL operations
  // (pb::CommScope). A wait times out only while such a mark is pending and no mark has completed
  // for longer than comm_timeout_ms -- local queued work with no communication behind it never
  // counts, however long it runs
  std::deque<hipEvent_t> comm_marks;
  std::vector<hipEvent_t> mark_pool;
  int64_t comm_groups = 0;
  // groups enqueued after the last mark of ctx->stream / ctx->comm_stream: a bounded wait marks
  // them first, so a stuck unmarked group counts as pending
  bool unmarked_main = false, unmarked_comm = false;
  int* h_stall = nullptr;  // test hook (tuning "comm_stall_test_ms"): released by comm_fail
  void* shm = nullptr;  // built-in shared-memory host transport (pb_transport.cpp), if attached
  // host transport (tests)
  pb_sendrecv_fn h_sendrecv = nullptr;
  pb_allreduce_fn h_allreduce = nullptr;
  void* h_user = nullptr;
  pb_alltoallv_fn h_alltoallv = nullptr;
  void* h_a2a_user = nullptr;
  double* h_a2a = nullptr;  // pinned staging for the host all-to-all (send | recv)
  size_t h_a2a_len = 0;
  // reduction scratch
  double* d_partials = nullptr;   // [max_blocks * 8]
  int64_t partials_cap = 0;
  double* d_scalars = nullptr;    // small device scalars for vector reductions
  double* h_scalars = nullptr;    // pinned mirror
  int num_cus = 256;
  // z-march direction of the next standalone stencil apply (alternates: each apply starts on
  // the planes the previous one touched last, which are still in the Infinity Cache)
  int zflip = 0;
  // context-owned scratch for the one-shot compact / tridiagonal entry points (grown on demand;
  // every use is ordered on `stream`, so one buffer serves all of them)
  double* scratch = nullptr;
  size_t scratch_len = 0;
  // timing
  bool timing = false;
  std::vector<std::string> timing_only;  // PB_TIMING_ONLY="a,b": time only these phases
  int timing_every = 1;  // PB_TIMING_EVERY=n: events around every n-th call of a phase only
  std::map<std::string, int64_t> timer_calls;
  bool roctx = false;  // PB_ROCTX=1: roctx ranges around every timed phase (rocprofv3 --marker-trace)
  std::map<std::string, pb::TimerSlot> timers;
  std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> pending;
  std::vector<hipEvent_t> event_pool;
};

struct pb_grid {
  pb_ctx* ctx = nullptr;
  int64_t n[3] = {0, 0, 0};
  double L[3] = {1, 1, 1};
  double h[3] = {1, 1, 1};
  int64_t k0 = 0, nzl = 0;   // owned planes [k0, k0 + nzl)
  int64_t plane = 0;         // n[0] * n[1]
  int64_t nlocal = 0;        // plane * nzl
  // ghost planes (received halos) and send staging (CG boundary p planes)
  double* ghost_lo = nullptr;
  double* ghost_hi = nullptr;
  double* bnd_lo = nullptr;
  double* bnd_hi = nullptr;
  double* h_stage = nullptr;  // pinned host staging for the host transport (4 planes)
  // deep ghosts for the fused multigrid sweeps on N ranks (allocated on first use, six planes):
  // two deep = [planes -2, -1 | nzl, nzl+1], three deep = [-3 .. -1 | nzl .. nzl+2];
  // h_stage2 = host staging (12 planes)
  double* ghost2 = nullptr;
  double* h_stage2 = nullptr;
  // z-slab <-> y-slab rank tables (j -> rank, j0, nyl; pb_compact_dist.hip), uploaded once on
  // first use, so the transposes inside CG iterations never wait on the host
  int* yslab_tab = nullptr;
  // the whole domain on this rank even on a multi-rank context (host-array compact entry points:
  // the reference's module procedures work on process-local arrays)
  bool whole = false;
};
inline bool grid_split(const pb_grid* g) { return g->ctx->split && !g->whole; }

struct pb_vec {
  pb_grid* grid = nullptr;
  double* d = nullptr;
  int64_t nlocal = 0;
};

struct pb_op {
  pb_grid* grid = nullptr;
  int kind = PB_OP_STAR7;
  double deltas[3] = {1, 1, 1};
  double cx = 0, cy = 0, cz = 0, cc = 0;  // star coefficients
  // compact scratch
  double* work = nullptr;
  int64_t work_len = 0;
};

namespace pb {

// ---- coefficient helpers (src/coefficients.f90:22-48) ----
struct Star {
  double cx, cy, cz, cc;
};
Star star_coeffs(const double h[3]);

// ---- timing ----
// events on `s` (default: the context stream)
void timer_begin(pb_ctx* ctx, const char* name, hipEvent_t* ev, hipStream_t s = nullptr);
void timer_end(pb_ctx* ctx, const char* name, hipEvent_t ev0, hipStream_t s = nullptr);
void timers_collect(pb_ctx* ctx);

bool timer_wanted(pb_ctx* ctx, const char* name);

// stencil-engine launches of this scope go to stream s instead of the context stream
struct EngineOn {
  pb_ctx* ctx;
  EngineOn(pb_ctx* c, hipStream_t s) : ctx(c) { ctx->engine_stream = s; }
  ~EngineOn() { ctx->engine_stream = nullptr; }
};

struct ScopedTimer {
  pb_ctx* ctx;
  const char* name;
  hipEvent_t ev0 = nullptr;
  bool on = false;
  ScopedTimer(pb_ctx* c, const char* n) : ctx(c), name(n) {
    if (ctx->roctx) roctxRangePushA(name);
    on = ctx->timing && timer_wanted(ctx, name);
    if (on) timer_begin(ctx, name, &ev0);
  }
  ~ScopedTimer() {
    if (on) timer_end(ctx, name, ev0);
    if (ctx->roctx) roctxRangePop();
  }
};

// ---- communication (RCCL or host transport) ----
// Exchange z-boundary planes: send `lo` (first owned plane data) to rank-1 and `hi` to rank+1,
// receive into grid->ghost_lo (from rank-1) / grid->ghost_hi (from rank+1). Stream ordered.
int halo_exchange(pb_grid* g, const double* lo, const double* hi);
// Split form: begin (RCCL on the context's comm stream after an event on the compute stream;
// host transport: synchronous), end (compute stream waits for the exchange).
int halo_begin(pb_grid* g, const double* lo, const double* hi);
// halo_begin with the boundary planes produced on the comm stream first (RCCL split grids): pre
// enqueues their kernel on the given stream after the context stream's work so far
int halo_begin_after(pb_grid* g, const double* lo, const double* hi,
                     const std::function<int(hipStream_t)>& pre);
// np-plane exchange into explicit buffers: send the np planes at `lo` (first owned) to rank-1
// and at `hi` (last owned) to rank+1; rlo receives the np planes below the slab (from rank-1),
// rhi the np planes above it (from rank+1). Stream ordered; one rank: periodic copies.
int halo_exchange_n(pb_grid* g, const double* lo, const double* hi, int np, double* rlo,
                    double* rhi);
int halo_end(pb_grid* g);
// release the shared-memory transport of a context (pb_transport.cpp)
void transport_destroy(pb_ctx* ctx);
// In-place SUM allreduce of `count` device doubles (stream ordered).
int allreduce_device(pb_ctx* ctx, double* d_vals, int count);
// Bounded host waits. One rank without a communicator: plain hipStream/EventSynchronize. Split
// contexts poll (hipStreamQuery / hipEventQuery) and check ncclCommGetAsyncError; a peer error
// or a wait longer than ctx->comm_timeout_ms aborts the communicator (ncclCommAbort) and returns
// PB_ERR_COMM. `what` names the wait in the error message.
int wait_stream(pb_ctx* ctx, hipStream_t s, const char* what);
int wait_event(pb_ctx* ctx, hipEvent_t ev, const char* what);
// mark the context's communication as failed (aborting RCCL) and return PB_ERR_COMM
int comm_fail(pb_ctx* ctx, const char* fmt, ...);
#define PB_SYNC(ctx, what) PB_TRY(::pb::wait_stream((ctx), (ctx)->stream, (what)))
// a group of RCCL operations enqueued on `s`; every 4th (and every forced one) gets an event
// after it: the progress marks the bounded waits watch (pb_ctx::comm_marks)
struct CommScope {
  pb_ctx* ctx;
  hipStream_t s;
  bool mark;
  CommScope(pb_ctx* c, hipStream_t st, bool force = false);
  ~CommScope();
};
// test hook: a kernel on `s` that waits for ctx->h_stall (a peer that never answers), bounded by
// `ms` of device time so it always ends
int launch_comm_stall(pb_ctx* ctx, hipStream_t s, int ms);
#define PB_COMM_OK(ctx)                                                                     \
  do {                                                                                      \
    if ((ctx)->comm_failed)                                                                 \
      return ::pb::set_error(PB_ERR_COMM, "communication failed earlier on this context");  \
  } while (0)

// ---- kernels (pb_stencil.hip) ----
struct StencilPlanes {
  const double* ghost_lo;  // plane at k = -1
  const double* ghost_hi;  // plane at k = nzl
  // one rank: read the periodic wrap planes of the loader's raw arrays in place (k mod nzl)
  // instead of ghost planes (which then need not exist)
  bool wrap = false;
};
enum { PLANES_ALL = 0, PLANES_INTERIOR = 1, PLANES_BOUNDARY = 2 };
int launch_star7_apply(pb_grid* g, const Star& s, const double* x, double* y,
                       const StencilPlanes& gp, int mode);
// assembled P (pb_assembled.hip): re-sum the seam and slab-boundary rows of y = P x in PETSc AIJ
// order after the stencil engine produced y (glo / ghi: x's ghost planes, nullptr on one rank)
int launch_aij_seams(pb_grid* g, const Star& s, const double* x, const double* glo,
                     const double* ghi, double* y);
// red-black SOR half-sweep in place (first = 1: zero-start red + black fused, x written from b)
// and the multigrid residual, on the stencil engine (pb_mg.hip)
struct CgState;
int launch_mg_sor(pb_grid* g, const Star& s, double* x, const double* b, const StencilPlanes& gp,
                  double omega, int color, int first, const int* skip,
                  const CgState* sums_st = nullptr, int* nparts = nullptr);
// both red-black half-sweeps (c1 first) in one pass, out of place, one rank (pb_stencil.hip)
bool sor_sweep2_supported(const pb_grid* g);
int launch_sor_sweep2(pb_grid* g, const Star& s, const double* xin, const double* b, double* xout,
                      double omega, int c1, const int* skip, const CgState* sums_st = nullptr,
                      int* nparts = nullptr);
// pre-smoothing from zero (red + black half-sweeps) fused with the residual: x, res from b
// post-smoothing with the prolongation folded in (one rank): xout = both half-sweeps (black, red)
// of xin = xs + P xc (cg: the coarse grid of xc), optional CG residual sums
// pre-smoothing from zero + residual + restriction to the coarse b in one pass (one rank)
int launch_presmooth_restrict(pb_grid* g, const Star& s, const pb_grid* cg, const double* b,
                              double* xout, double* bc, double omega, const int* skip);
// xc_full (decomposed grids, agglomerated coarse level): the whole coarse correction on this
// rank -- its ghost planes are read in place instead of exchanged
int launch_post_sweep(pb_grid* g, const Star& s, const pb_grid* cg, const double* xs,
                      const double* xc, const double* b, double* xout, double omega,
                      const int* skip, const CgState* sums_st = nullptr, int* nparts = nullptr,
                      const double* xc_full = nullptr);
int launch_presmooth_residual(pb_grid* g, const Star& s, const double* b, double* x, double* res,
                              double omega, const int* skip);
int launch_mg_residual(pb_grid* g, const Star& s, const double* x, const double* b,
                       const StencilPlanes& gp, double* res, const int* skip);

// CG state (device resident; all scalars computed on device, host only polls `done`)
// Deferred solution update (defer_x = D in {0, 2, 4}): x += sum of alpha_m p_m over D
// iterations in the pass B of every D-th iteration; pend_* describe what is still pending
// (alphas pa[0 .. pend_count-1] of iterations pend_iter, pend_iter + 1, ...).
struct CgState {
  double beta, betaold, dpi, dpiold, alpha, alpha_prev, mu, dp, ttol, rnorm0;
  double pa[3];
  double rtol, atol, dtol, dinv, ntot;
  int64_t it, its, max_it, nhist, pend_iter, pend_count;
  int64_t nlog;  // history entries logged (PETSc KSPLogResidualHistory): its + 1, or its after a
                 // breakdown exit (beta = 0, indefinite PC / matrix) that skips the last norm
  int reason, done, pc, nullspace, defer_x;
  double bbp;  // beta / betaold of the current pass A (stage 1), for pass B re-forming p
  // single-reduction CG (-ksp_cg_single_reduction): delta = z'A z of the current z (taken with
  // z'z, z'r in the one reduction per iteration); sr = 1 selects that iteration's scalar logic
  double delta;
  int sr;
};
int launch_cg_init(pb_grid* g, const double* b, double* x, double* r, double* p, CgState* st,
                   double dinv, double* hist, int* h_done);
struct Fold {
  // 0: no fold; 1: stage 1 (pass B); 2: stage 2 (pass A); single-reduction pass P: 3: the
  // residual-sum stage of the previous iteration, then the top of this one; 4: the top only
  int stage = 0;
  int nparts = 0, width = 1;      // partials of the previous pass
  const double* parts = nullptr;
  const CgState* in = nullptr;    // state slot read
  CgState* out = nullptr;         // state slot written (block 0)
  double* hist = nullptr;         // stage 2: history / host-mapped done flags, as finalize's
  int* h_done = nullptr;
  int64_t host_iter = 0;          // stage 2: the iteration whose stage 2 this is
};
// fold.stage = 2: the previous iteration's stage 2 in the prologue (split grids, folded iteration;
// fold.out = nullptr: the state stays in registers). stream = nullptr: the context stream.
int launch_cg_boundary(pb_grid* g, const double* r, const double* p_old, CgState* st,
                       const Fold& fold, hipStream_t stream = nullptr);
int launch_cg_boundary(pb_grid* g, const double* r, const double* p_old, CgState* st);
// pass A launch (mode: PLANES_*) whose prologue runs fold (stage 2, split grids)
int launch_cg_pass_a_fold(pb_grid* g, const Star& s, const double* r, const double* p_old,
                          double* p_new, const StencilPlanes& gp, const Fold& fold, int mode,
                          int part_off, int* nblocks, bool store);
// split grids, folded iteration: a pass's partials reduced and allreduced into ctx->d_scalars
int cg_reduce_allreduce(pb_ctx* ctx, int nparts, int width, bool b_region);
int cg_reduce_allreduce(pb_ctx* ctx, const double* parts, int nparts, int width);
// stage 2 on st in place from the sums cg_reduce_allreduce left in ctx->d_scalars
int cg_stage2_from_sums(pb_ctx* ctx, int width, CgState* st, double* hist, int* h_done,
                        int64_t host_iter);
// store = false: pass A only takes p.Ap; pass B forms and stores p (PB_CG_PSTORE_B, PStore)
int launch_cg_pass_a(pb_grid* g, const Star& s, const double* r, const double* p_old,
                     double* p_new, const StencilPlanes& gp, CgState* st, int mode, int part_off,
                     int* nblocks, bool store = true);
// pass B re-forming p (PB_CG_PSTORE_B): zsrc = the array pass A combined (r), r_out = the
// residual's other buffer; r_out == nullptr: p is read as stored by pass A, r updated in place
struct PStore {
  const double* zsrc = nullptr;
  double* r_out = nullptr;
};
int cg_finalize_pass_a(pb_ctx* ctx, int nparts, CgState* st);
// p_prev[m] = p of iteration host_iter - 1 - m (m < 3; only the first defer-1 are read)
int launch_cg_pass_b(pb_grid* g, const Star& s, const double* p, const double* const* p_prev,
                     double* x, double* r, const StencilPlanes& gp, CgState* st, double* hist,
                     int* h_done, int64_t host_iter, int defer, bool finalize = true,
                     const PStore& ps = PStore{});
int launch_cg_flush(pb_grid* g, double* x, const double* p, double alpha);
// Folded single-rank Jacobi iteration (finalize in the passes' prologues, pb_stencil.hip): state
// in two slots st2[0..1]; pass A of iteration host_iter >= 1 runs stage 2 of host_iter - 1
// (st2[1] -> st2[0], history and done flag as finalize's), pass B stage 1 (st2[0] -> st2[1]);
// cg_fold_tail completes the last iteration of a batch and leaves the state in st2[0].
int launch_cg_pass_a_folded(pb_grid* g, const Star& s, const double* r, const double* p_old,
                            double* p_new, const StencilPlanes& gp, CgState* st2, int nparts_b,
                            double* hist, int* h_done, int64_t host_iter, int* nblocks,
                            bool store = true);
int launch_cg_pass_b_folded(pb_grid* g, const Star& s, const double* p,
                            const double* const* p_prev, double* x, double* r,
                            const StencilPlanes& gp, CgState* st2, int nparts_a, int64_t host_iter,
                            int defer, int* nparts_b, const PStore& ps = PStore{},
                            const double* parts_a = nullptr);
int cg_fold_tail(pb_ctx* ctx, int nparts_b, CgState* st2, double* hist, int* h_done,
                 int64_t host_iter);
// Single-reduction CG (PETSc KSPSolve_CG_SingleReduction, -ksp_cg_single_reduction), two engine
// passes per iteration and ONE reduction (pb_stencil.hip):
//   pass P: prologue = [the previous iteration's residual-sum stage (folded, one rank)] + the top
//     of the iteration (beta / betaold, p'w = delta - beta^2 dpiold / betaold^2, alpha); body:
//     p = (dinv r - mu) + b p_old on load, w = A p, r_out = r - alpha w, store p and r_out, the
//     deferred x update every defer-th iteration. Reads state slot `in`, writes slot `out`.
//   pass S: t = dinv r_out - mu on load, s = A t; per-block sums t, t^2, t.r, r, t.s (5 wide)
//     into ctx->d_partials + part_off * 5.
// fold_sums: 1 = the prologue first reduces pass S's partials (nparts_s blocks at offset 0) and
// runs their stage (history / done flag of host_iter - 1); 0 = the state in `in` is complete.
struct SrFold {
  int fold_sums = 0;
  int nparts_s = 0;
  const double* parts = nullptr;  // the partials fold_sums reduces (5 wide)
  const CgState* in = nullptr;
  CgState* out = nullptr;
  double* hist = nullptr;
  int* h_done = nullptr;
};
int launch_cg_sr_pass_p(pb_grid* g, const Star& s, const double* r, const double* const* p_prev,
                        double* p_new, double* x, double* r_out, const StencilPlanes& gp,
                        const SrFold& f, int mode, int64_t host_iter, int defer);
int launch_cg_sr_pass_s(pb_grid* g, const Star& s, const double* r, const StencilPlanes& gp,
                        const CgState* st, int mode, int part_off, int part_end,
                        int* nblocks);
// after pass S (unfolded): reduce its partials `parts` (+ allreduce on split grids) and run the
// residual-sum stage on st in place (stage_delta0: the setup's delta = z0'A z0 only)
int cg_sr_finalize(pb_ctx* ctx, const double* parts, int nparts, CgState* st, double* hist,
                   int* h_done, int64_t host_iter, bool stage_delta0 = false);
// The same iteration as ONE pass (pb_cg_sr.hip; one rank, even nx, tuning cg_sr_fused): p, r',
// and all five sums; the prologue as pass P's (sf), partials into parts_out (*nblocks blocks)
bool cg_sr1_supported(const pb_grid* g);
// x != nullptr: the iteration also carries the depth-4 deferred x update (p_m2, p_m3 = p_{i-2},
// p_{i-3}; p_{i-1} is p_old)
int launch_cg_sr1(pb_grid* g, const Star& s, const double* r, const double* p_old,
                  double* p_new, double* r_out, const SrFold& sf, const double* parts_in, double* parts_out, int64_t host_iter,
                  int* nblocks);

// ---- compact fast path + generic CG (pb_compact_fast.hip) ----
int64_t compact_fast_work_len(const pb_grid* g);
int compact_lapl_fast(pb_grid* g, const double dx[3], const double* f, double* out, double* work);
// integer user setting from the environment (the PB_* variables INTEGRATION.md lists), dflt when
// unset
inline int env_int(const char* name, int dflt) {
  const char* s = getenv(name);
  return s ? atoi(s) : dflt;
}
// Kernel-selection / launch-shape parameter: the value a caller set with pb_tune_set (tests and
// A/B runs), else dflt -- the measured default at the call site. Never read from the environment.
int tune(const char* name, int dflt);
bool tune_is_set(const char* name);
// Timing-only ablations (they skip traffic and give wrong results): compile-time only, for
// scripts/build_variant.sh builds, never in the product library
#ifndef PB_ABLATE_FFT
#define PB_ABLATE_FFT 0
#endif
#ifndef PB_ABLATE_LINES
#define PB_ABLATE_LINES 0
#endif
// Field-sized device allocations (vectors, KSP work vectors). Free with field_free.
hipError_t field_alloc(void** p, size_t bytes);
void field_free(void* p);
template <class T>
inline hipError_t field_alloc(T** p, size_t bytes) {
  return field_alloc(reinterpret_cast<void**>(p), bytes);
}

// ---- register-resident line solves (pb_compact_lines.hip) ----
bool compact_lines_supported(int64_t n);
bool compact_cg_fusable(const pb_grid* g);  // CgFuse applies to the compact operator on g
bool compact_cg_fusable_split(const pb_grid* g);  // ... on a split grid (pack + X pass)
struct YSlabPlan;
// blk_in (Y pass of a decomposed grid): in0 / in1 are the all-to-all receive buffers in their
// blocked layout (yslab_blocked), not z-slab fields
int compact_lines_pass(pb_ctx* ctx, const int64_t dims[3], int axis, double h, const double* in0,
                       const double* in1, double* out0, double* out1,
                       const YSlabPlan* blk_in = nullptr);
// batched periodic (alpha,1,alpha) solve in registers (n = 64*C); PB_ERR_UNSUPPORTED otherwise
int lines_solve_batched(pb_ctx* ctx, int64_t n, int64_t nbatch, int64_t line_stride,
                        int64_t elem_stride, double alpha, double* d);
// the three passes of the factorised compact Laplacian on a box with complete lines
int compact_pass_z(pb_ctx* ctx, const int64_t d[3], double h, const double* f, double* u, double* v);
int compact_pass_y(pb_ctx* ctx, const int64_t d[3], double h, const double* u, const double* v,
                   double* s, double* t, const YSlabPlan* blk_in = nullptr);
int compact_pass_x(pb_ctx* ctx, const int64_t d[3], double h, const double* s, const double* t,
                   double* out);
// ---- multi-rank Z pass: z-slab <-> y-slab all-to-all transposes (compact_dist.cpp) ----
int64_t compact_dist_work_len(const pb_grid* g);
// plan_out != nullptr: on equal 2^k-row y-slabs u, v are left in the all-to-all layout (the plan
// in *plan_out, *blocked = true) for a Y pass that reads them so; otherwise unpacked as z-slabs
int compact_dist_pass_z(pb_grid* g, double h, const double* f, double* u, double* v, double* work,
                        YSlabPlan* plan_out = nullptr, bool* blocked = nullptr);
// z-slab <-> y-slab transposes (rank r holds rows [j0_r, j0_r + nyl_r) of every plane: complete
// z-lines) for line operations along z on a split grid; pb_compact_dist.hip
struct YSlabPlan {
  std::vector<int64_t> k0, nzl, j0, nyl, zc, yc;
  int64_t ny_me = 0, ny_slab = 0;  // this rank's y rows; doubles of one y-slab field
  double* stage = nullptr;
  int* tab = nullptr;
  int nb = 0;
  // self block (r05): on RCCL contexts the block a rank keeps is never copied by the all-to-all;
  // its producer writes it where the consumer reads it. A z-slab-layout offset o of the self
  // block lives at ybuf + self_shift + o in a y-slab buffer (self_shift = the y-side block offset
  // minus the z-side one)
  bool self_direct = false;
  int me = 0;
  int64_t self_shift = 0;
  // the y-slab buffers holding the self block of the blocked consumers' inputs / producer's
  // output (set by the caller that owns them; + self_shift applied)
  const double* alt0 = nullptr;
  const double* alt1 = nullptr;
  double* alt_out = nullptr;
};
int64_t yslab_len(const pb_grid* g);
int64_t yslab_aux_len(const pb_grid* g);
int yslab_begin(pb_grid* g, double* aux, YSlabPlan* p);  // aux: yslab_aux_len doubles
struct CgFuse;
// cf (CG on a split grid): the pack forms CG's p from cf->z and p_old = f in place (sets
// cf->fused_z)
int yslab_to(pb_grid* g, const YSlabPlan& p, const double* f, double* fy, CgFuse* cf = nullptr);
// equal y-slabs of 2^k rows: a z-slab row (kl, j) sits in the all-to-all buffer at block j >> k,
// row kl * nyl + (j & (nyl - 1)) -- producers / consumers may address it directly
bool yslab_blocked(const YSlabPlan& p);
int yslab_from(pb_grid* g, const YSlabPlan& p, const double* fy, double* f);
// all-to-all with per-peer counts; blocks are contiguous in rank order on both sides
// skip_self: the rank's own block is already in place (YSlabPlan::self_direct), not copied
int alltoallv_device(pb_ctx* ctx, const double* send, const int64_t* scount, double* recv,
                     const int64_t* rcount, bool skip_self = false);
// Config-5 iteration fusions (compact A with a stored-z preconditioner, one rank, register line
// solves): the compact operator's Z pass forms p = (dinv z - mu) + beta/beta_old p_old from its
// tile loads and stores p (cg_gen_p_kernel's arithmetic, bit-identical), and its X pass takes the
// per-block partial sums of p . w as it writes w (cg_gen_dot_kernel's job). The caller sets
// ctx->cg_fuse around the apply; the passes report what they fused, the caller runs the
// separate kernels for anything they did not.
struct CgFuse {
  const double* z = nullptr;      // Z pass: stored z, the source of p
  const double* p_old = nullptr;  // previous direction (not used when first)
  double* p_out = nullptr;        // p as formed
  const CgState* st = nullptr;
  int first = 0;                  // KSPSolve_CG's i = 0 (p = z - mu)
  const double* dot_p = nullptr;  // X pass: p, for the p . w partial sums into ctx->d_partials
  int nparts = 0;                 // out: partial-sum blocks written by the X pass
  bool fused_z = false, fused_dot = false;  // out
};
int launch_cg_generic_p(pb_grid* g, const double* r, double* p, CgState* st, int first = 0);
int launch_cg_generic_dot(pb_grid* g, const double* p, const double* w, CgState* st, int* nparts);
int launch_cg_generic_xr(pb_grid* g, const double* p, const double* w, double* x, double* r,
                         CgState* st, int* nparts);
int cg_finalize_stage2(pb_ctx* ctx, int nparts, CgState* st, double* hist, int* h_done,
                       int64_t host_iter);

// ---- vector ops (pb_vecops.hip) ----
int vec_fill(pb_ctx* ctx, double* d, int64_t n, double a);
// form 0: VecAXPY y = y + coef*x;  1: VecAYPX y = x + coef*y;  2: VecScale y = coef*y
int vec_update(pb_ctx* ctx, int form, double* y, const double* x, int64_t n, double coef);
int vec_random(pb_ctx* ctx, double* d, int64_t n, uint64_t seed, int64_t g0);
// reduce kind: 0 = sum(x), 1 = dot(x, y); result into *out (global over ranks)
int vec_reduce(pb_ctx* ctx, int kind, const double* x, const double* y, int64_t n, double* out);
// flat fp64 copy of n doubles (HBM calibration): per-launch ms of `reps` timed launches
int copy_probe(pb_ctx* ctx, int64_t n, int reps, std::vector<float>& ms,
               const double* src = nullptr, double* dst = nullptr);

// ---- grid with an explicit slab (multigrid levels) ----
int grid_create_part(pb_ctx* ctx, const int64_t n[3], const double L[3], int64_t k0, int64_t nzl,
                     pb_grid** out);

// ---- preconditioned CG pieces (pb_cg_generic.hip) ----
int launch_cg_pc_xr(pb_grid* g, const double* p, const double* w, double* x, const double* r_in,
                    double* r, CgState* st, int first);
int launch_cg_pc_sums(pb_grid* g, const double* z, const double* r, CgState* st, int* nparts);
int cg_finalize_init(pb_ctx* ctx, int nparts, CgState* st, double* hist, int* h_done);

// ---- geometric multigrid / red-black SOR preconditioner (pb_mg.hip) ----
struct Mg;
// levels_req: 0 = automatic; pc_type PB_PC_SOR (one symmetric red-black sweep) or PB_PC_MG
int mg_create(pb_grid* g, const double deltas[3], int pc_type, int levels_req, int coarse_its,
              double omega, Mg** out);
// z = M^-1 r (zero initial guess); skip: optional device flag (CG's `done`) -- when set, the
// kernels exit at entry (halo exchanges still run, so ranks stay matched)
// sums_st: also take CG's residual sums of z (t = z - mu_old: t, t^2, t.r, r) in the last
// half-sweep when it runs on the stencil engine; *nparts = partial-sum blocks written, 0 if not
int mg_apply(Mg* mg, const double* r, double* z, const int* skip = nullptr,
             const CgState* sums_st = nullptr, int* nparts = nullptr);
int mg_levels(const Mg* mg);
void mg_destroy(Mg* mg);
// deterministic level count for a global grid split over nranks z-slabs (every rank agrees)
int mg_plan_levels(const int64_t n[3], int nranks, int levels_req);

// ---- spectral preconditioner (pb_fft.hip): z = P^+ r by separable Hartley transforms ----
struct FftPc;
// compact: invert the compact operator's symbol (else the 7-point star's); power-of-two extents
int fftpc_create(pb_grid* g, const double deltas[3], int compact, FftPc** out);
// sums_st / nparts: the last pass also takes CG's residual sums of z against r (mu from sums_st)
// into ctx->d_partials, *nparts blocks (0: the caller takes them)
// CG's x / r update on the PC's first pass (cg_pc_xr_kernel's arithmetic): r = r_in + (-alpha) w
// is formed as the pass loads it, stored to r_out and transformed; x = x + alpha p (first: alpha p)
// rides along. With CG's done flag set the pass exits, after writing x = 0 on a first iteration.
struct RUpdate {
  const double* r_in;
  const double* w;
  double* r_out;
  const double* p;
  double* x;
  int first;
  const CgState* st;
};
int fftpc_apply(FftPc* f, const double* r, double* z, const int* skip = nullptr,
                const CgState* sums_st = nullptr, int* nparts = nullptr,
                const RUpdate* ru = nullptr);
// whether fftpc_apply takes an RUpdate on this grid (X passes on the register-edge kernel)
bool fftpc_fuses_r_update(const FftPc* f);
void fftpc_destroy(FftPc* f);

// ---- context scratch: at least n doubles, valid until the next call on this context ----
int ctx_scratch(pb_ctx* ctx, size_t n, double** out);

// ---- partial-sum reduction (deterministic, fixed order) ----
int reduce_partials(pb_ctx* ctx, const double* parts, int nparts, int width, double* out);

}  // namespace pb
