// pb_solver.cpp -- operator (MatShell analogue) and KSP (KSPSolve_CG analogue) host logic.
//
// The CG iteration runs as 2 fused stencil passes + 2 one-block finalize kernels per iteration
// (plus a plane-sized boundary kernel and, on several ranks, one halo exchange and two scalar
// allreduces). All CG scalars live on the device; the host never waits inside an iteration and
// polls a per-iteration "done" flag (host-mapped) every `check_every` iterations, lagged by one
// poll interval so that every rank stops after the same number of enqueued iterations.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <strings.h>
#include <string>
#include <vector>

#include "pb_internal.hpp"

using namespace pb;

namespace pb {
int compact_lapl(pb_grid* g, const double dx[3], const double* f, double* out, double* work);
int64_t compact_work_len(const pb_grid* g);
}

// the fused CG passes evaluate A p inside the stencil engine (reference order); the assembled P
// (AIJ order at the seams) runs the unfused iteration around its own MatMult
static bool fused_kind(int kind) { return kind == PB_OP_STAR7; }

struct pb_ksp {
  pb_op* A = nullptr;
  pb_op* P = nullptr;
  pb_ksp_opts opts;
  double* r = nullptr;
  // Jacobi / none on the fused operator: pass B forms and stores p and writes the residual to
  // the other buffer -- iteration i reads rbuf(i), writes rbuf(i + 1)
  double* r2 = nullptr;
  bool pst = false;
  double* rbuf(int64_t i) const { return (pst && (i & 1)) ? r2 : r; }
  // iteration i: p_old = pb[i % ns], p_new = pb[(i + 1) % ns]; ns = 2, or 4 with the depth-4
  // deferred x update (pb[2], pb[3] allocated on first use)
  double* pb[4] = {nullptr, nullptr, nullptr, nullptr};
  double* w = nullptr;   // generic (unfused) path only
  double* z = nullptr;   // generic path only
  pb::Mg* mg = nullptr;  // SOR / multigrid preconditioner (PB_PC_SOR, PB_PC_MG)
  pb::FftPc* fft = nullptr;  // spectral preconditioner (PB_PC_FFT)
  int fold_nparts_b = 0;     // partial-sum blocks of the last folded pass B
  bool stored_z() const { return mg || fft; }  // PCs whose z = M^-1 r is stored (not Jacobi)
  bool lazy0 = false;  // r0 = b, x0 = 0, p0 = 0 left implicit by pb_ksp_begin
  CgState* d_st = nullptr;
  double* d_hist = nullptr;
  int64_t nhist = 0;
  int* h_done = nullptr;      // host-mapped, one flag per host iteration (+1)
  int* h_done_dev = nullptr;  // its device alias
  int64_t done_cap = 0;
  std::vector<hipEvent_t> ring;
  // solve state
  const pb_vec* b = nullptr;
  pb_vec* x = nullptr;
  int64_t host_iter = 0;
  bool stopped = false;
  bool begun = false;
  int defer_x = 4;  // x updated every defer_x-th iteration (PB_CG_DEFER_X = 0, 2 or 4)
  int pslots() const { return defer_x == 4 ? 4 : 2; }
  // single-reduction iteration (-ksp_cg_single_reduction on the fused operator, Jacobi / none):
  // the state alternates between the two slots d_st[0..1] within a pb_ksp_iterate batch (pass P
  // of the batch's n-th iteration reads slot n & 1 and writes the other); sr_nparts = pass S's
  // partial-sum blocks of the last iteration (folded: reduced by the next pass P's prologue)
  bool sr = false;
  int sr_nparts = 0;
};

static int sr_pass_s(pb_ksp* k, const double* r, const CgState* st, int* nparts, int64_t n);
static const double* sr_region(const pb_ctx* ctx, int64_t n);

extern "C" {

// ---------------------------------------------------------------------------------------------
// Operator (src/poissbox.f90:242-267 initialise_matrix_free; :300-322 mfmult)
// ---------------------------------------------------------------------------------------------
int pb_op_create(pb_grid* g, int kind, const double deltas[3], pb_op** out) {
  PB_CHECK_ARG(g && out, "bad op args");
  PB_CHECK_ARG(kind == PB_OP_STAR7 || kind == PB_OP_COMPACT || kind == PB_OP_ASSEMBLED27,
               "unknown operator kind");
  pb_op* op = new pb_op();
  op->grid = g;
  op->kind = kind;
  for (int d = 0; d < 3; ++d) op->deltas[d] = deltas ? deltas[d] : g->h[d];
  Star s = star_coeffs(op->deltas);
  op->cx = s.cx;
  op->cy = s.cy;
  op->cz = s.cz;
  op->cc = s.cc;
  if (kind == PB_OP_COMPACT) {
    op->work_len = compact_fast_work_len(g);
    if (hipMalloc(&op->work, (size_t)op->work_len * sizeof(double)) != hipSuccess) {
      delete op;
      return set_error(PB_ERR_ALLOC, "compact operator workspace: out of device memory");
    }
  }
  *out = op;
  return PB_OK;
}

static int star7_apply(pb_op* op, const double* x, double* y) {
  pb_grid* g = op->grid;
  Star s{op->cx, op->cy, op->cz, op->cc};
  StencilPlanes gp;
  if (!g->ctx->split) {
    gp.ghost_lo = x + (g->nzl - 1) * g->plane;  // periodic wrap: no copy
    gp.ghost_hi = x;
    return launch_star7_apply(g, s, x, y, gp, PLANES_ALL);
  }
  gp.ghost_lo = g->ghost_lo;
  gp.ghost_hi = g->ghost_hi;
  if (g->nzl < 3) {
    PB_TRY(halo_exchange(g, x, x + (g->nzl - 1) * g->plane));
    return launch_star7_apply(g, s, x, y, gp, PLANES_ALL);
  }
  // interior planes overlap the halo exchange; the two boundary planes follow it (timed as one
  // apply: interior launch, wait for the exchange, boundary launch)
  ScopedTimer tm(g->ctx, "stencil");
  PB_TRY(halo_begin(g, x, x + (g->nzl - 1) * g->plane));
  PB_TRY(launch_star7_apply(g, s, x, y, gp, PLANES_INTERIOR));
  PB_TRY(halo_end(g));
  return launch_star7_apply(g, s, x, y, gp, PLANES_BOUNDARY);
}

// KSP iterations enqueued ahead of the convergence poll: the operator kernels launched inside
// the guard's scope exit at entry once the KSP's device flag is set (pb_ctx::op_skip)
struct OpApplySkip {
  pb_ctx* ctx;
  OpApplySkip(pb_ctx* c, const int* flag) : ctx(c) { ctx->op_skip = flag; }
  ~OpApplySkip() { ctx->op_skip = nullptr; }
};

static int op_apply_raw(pb_op* op, const double* x, double* y) {
  pb_grid* g = op->grid;
  if (op->kind == PB_OP_COMPACT) return compact_lapl_fast(g, op->deltas, x, y, op->work);
  PB_TRY(star7_apply(op, x, y));
  if (op->kind != PB_OP_ASSEMBLED27) return PB_OK;
  // assembled P: same 7 non-zeros; re-sum the seam / slab-boundary rows in AIJ order (the
  // ghost planes hold x's halo after the apply on a split grid)
  Star s{op->cx, op->cy, op->cz, op->cc};
  const bool split = g->ctx->split;
  return launch_aij_seams(g, s, x, split ? g->ghost_lo : nullptr, split ? g->ghost_hi : nullptr, y);
}

int pb_op_set_deltas(pb_op* op, const double deltas[3]) {
  PB_CHECK_ARG(op && deltas, "bad args");
  for (int d = 0; d < 3; ++d) op->deltas[d] = deltas[d];
  Star s = star_coeffs(op->deltas);
  op->cx = s.cx;
  op->cy = s.cy;
  op->cz = s.cz;
  op->cc = s.cc;
  return PB_OK;
}

int pb_op_apply(pb_op* op, const pb_vec* x, pb_vec* y) {
  PB_CHECK_ARG(op && x && y, "bad apply args");
  PB_CHECK_ARG(x->grid == op->grid && y->grid == op->grid, "vector/operator grid mismatch");
  PB_CHECK_ARG(x != y, "MatMult requires distinct input and output vectors");
  return op_apply_raw(op, x->d, y->d);
}

int pb_op_get_ownership_range(const pb_op* op, int64_t* first, int64_t* next) {
  PB_CHECK_ARG(op && first && next, "bad args");
  const pb_grid* g = op->grid;
  *first = g->k0 * g->plane;
  *next = (g->k0 + g->nzl) * g->plane;
  return PB_OK;
}

int pb_vec_get_ownership_range(const pb_vec* v, int64_t* first, int64_t* next) {
  PB_CHECK_ARG(v && first && next, "bad args");
  const pb_grid* g = v->grid;
  *first = g->k0 * g->plane;
  *next = (g->k0 + g->nzl) * g->plane;
  return PB_OK;
}

int pb_op_get_diagonal(const pb_op* op, double* diag) {
  PB_CHECK_ARG(op && diag, "bad args");
  *diag = op->cc;
  return PB_OK;
}

int pb_op_destroy(pb_op* op) {
  if (!op) return PB_OK;
  if (op->work) {
    (void)wait_stream(op->grid->ctx, op->grid->ctx->stream, "pb_op_destroy");
    (void)hipFree(op->work);
  }
  delete op;
  return PB_OK;
}

// ---------------------------------------------------------------------------------------------
// Options (PETSc options database names, src/poissbox.f90:295 KSPSetFromOptions)
// ---------------------------------------------------------------------------------------------
int pb_ksp_opts_default(pb_ksp_opts* o) {
  PB_CHECK_ARG(o, "opts is NULL");
  o->rtol = 1e-5;
  o->atol = 1e-50;
  o->dtol = 1e5;
  o->max_it = 10000;
  o->ksp_type = PB_KSP_CG;
  o->pc_type = PB_PC_JACOBI;
  o->nullspace = 1;
  o->monitor = 0;
  o->converged_reason = 0;
  o->check_every = 8;
  o->mg_levels = 0;
  o->mg_coarse_its = 8;
  o->sor_omega = 1.0;
  o->cg_single_reduction = 0;
  return PB_OK;
}

int pb_ksp_opts_parse(pb_ksp_opts* o, int argc, const char* const* argv) {
  PB_CHECK_ARG(o, "opts is NULL");
  for (int i = 0; i < argc; ++i) {
    const char* a = argv[i];
    const char* v = i + 1 < argc ? argv[i + 1] : nullptr;
    if (!strcmp(a, "-ksp_type") && v) {
      if (strcmp(v, "cg")) return set_error(PB_ERR_UNSUPPORTED, "-ksp_type %s: only cg", v);
      o->ksp_type = PB_KSP_CG;
      ++i;
    } else if (!strcmp(a, "-pc_type") && v) {
      if (!strcmp(v, "none")) o->pc_type = PB_PC_NONE;
      else if (!strcmp(v, "jacobi")) o->pc_type = PB_PC_JACOBI;
      else if (!strcmp(v, "sor")) o->pc_type = PB_PC_SOR;
      else if (!strcmp(v, "mg") || !strcmp(v, "gamg")) o->pc_type = PB_PC_MG;
      else if (!strcmp(v, "fft")) o->pc_type = PB_PC_FFT;
      else return set_error(PB_ERR_UNSUPPORTED, "-pc_type %s", v);
      ++i;
    } else if (!strcmp(a, "-ksp_rtol") && v) {
      o->rtol = atof(v);
      ++i;
    } else if (!strcmp(a, "-ksp_atol") && v) {
      o->atol = atof(v);
      ++i;
    } else if (!strcmp(a, "-ksp_divtol") && v) {
      o->dtol = atof(v);
      ++i;
    } else if (!strcmp(a, "-ksp_max_it") && v) {
      o->max_it = atoll(v);
      ++i;
    } else if (!strcmp(a, "-pc_mg_levels") && v) {
      o->mg_levels = atoi(v);
      ++i;
    } else if ((!strcmp(a, "-pc_mg_coarse_its") || !strcmp(a, "-mg_coarse_ksp_max_it")) && v) {
      o->mg_coarse_its = atoi(v);
      ++i;
    } else if (!strcmp(a, "-pc_sor_omega") && v) {
      o->sor_omega = atof(v);
      ++i;
    } else if (!strcmp(a, "-ksp_cg_single_reduction")) {
      // PetscOptionsBool: a bare flag is true; an explicit value may follow
      o->cg_single_reduction = 1;
      // (PetscOptionsStringToBool: case-insensitive true/yes/on/1 and false/no/off/0)
      auto is = [&](const char* w) { return v && !strcasecmp(v, w); };
      if (is("true") || is("yes") || is("on") || is("1")) {
        ++i;
      } else if (is("false") || is("no") || is("off") || is("0")) {
        o->cg_single_reduction = 0;
        ++i;
      }
    } else if (!strcmp(a, "-ksp_monitor")) {
      o->monitor = 1;
    } else if (!strcmp(a, "-ksp_converged_reason")) {
      o->converged_reason = 1;
    }
  }
  return PB_OK;
}

// ---------------------------------------------------------------------------------------------
// KSP
// ---------------------------------------------------------------------------------------------
int pb_ksp_create(pb_op* A, pb_op* P, const pb_ksp_opts* opts, pb_ksp** out) {
  PB_CHECK_ARG(A && out, "bad ksp args");
  if (!P) P = A;
  PB_CHECK_ARG(A->grid == P->grid, "A and P on different grids");
  pb_ksp* k = new pb_ksp();
  k->A = A;
  k->P = P;
  // every failure below releases what was built so far (pb_ksp_destroy takes a partial KSP:
  // each field, the PC objects and the state are freed only if they exist)
  auto fail = [k](int rc) {
    const std::string msg = pb_last_error();
    pb_ksp_destroy(k);
    return set_error(rc, "%s", msg.c_str());
  };
  if (opts) k->opts = *opts;
  else pb_ksp_opts_default(&k->opts);
  if (k->opts.check_every < 1) k->opts.check_every = 8;
  // SOR / MG / FFT iterations are expensive and few: poll the device flag more often -- every
  // iteration with the spectral PC (1-3 iterations per solve: an iteration enqueued ahead of the
  // poll costs its skipped launches, ~0.15 ms of a 512^3 config-5 solve, more than the idle
  // stream time of waiting for each iteration)
  // (only clamped down: a caller's explicit smaller interval stands -- ADVICE r03)
  if ((k->opts.pc_type == PB_PC_SOR || k->opts.pc_type == PB_PC_MG) && k->opts.check_every > 2)
    k->opts.check_every = 2;
  if (k->opts.pc_type == PB_PC_FFT)
    k->opts.check_every = 1;
  const int pc = k->opts.pc_type;
  if (pc != PB_PC_NONE && pc != PB_PC_JACOBI && pc != PB_PC_SOR && pc != PB_PC_MG &&
      pc != PB_PC_FFT)
    return fail(set_error(PB_ERR_UNSUPPORTED, "unknown pc_type %d", pc));
  pb_grid* g = A->grid;
  const size_t vb = (size_t)g->nlocal * sizeof(double);
  if (pc == PB_PC_SOR || pc == PB_PC_MG) {
    // the smoother / coarse operators are the 7-point P (src/coefficients.f90 star)
    if (P->kind == PB_OP_COMPACT)
      return fail(set_error(PB_ERR_UNSUPPORTED, "SOR / MG preconditioning needs a 7-point P"));
    const int rc = mg_create(g, P->deltas, pc, k->opts.mg_levels, k->opts.mg_coarse_its,
                             k->opts.sor_omega, &k->mg);
    if (rc != PB_OK) return fail(rc);
  }
  if (pc == PB_PC_FFT) {
    // the symbol of P: the compact operator (config 5: A = P = compact) or the 7-point star
    const int rc = fftpc_create(g, P->deltas, P->kind == PB_OP_COMPACT, &k->fft);
    if (rc != PB_OK) return fail(rc);
  }
  if (field_alloc(&k->r, vb) != hipSuccess || field_alloc(&k->pb[0], vb) != hipSuccess ||
      field_alloc(&k->pb[1], vb) != hipSuccess)
    return fail(set_error(PB_ERR_ALLOC, "KSP work vectors: out of device memory"));
  if (!fused_kind(A->kind) || k->stored_z()) {
    if (field_alloc(&k->w, vb) != hipSuccess || field_alloc(&k->z, vb) != hipSuccess)
      return fail(set_error(PB_ERR_ALLOC, "KSP work vectors: out of device memory"));
  }
  // [1]: the folded iteration's second slot
  if (hipMalloc(&k->d_st, 2 * sizeof(CgState)) != hipSuccess)
    return fail(set_error(PB_ERR_ALLOC, "KSP state: out of device memory"));
  *out = k;
  return PB_OK;
}

static int ensure_done_cap(pb_ksp* k, int64_t need) {
  if (need <= k->done_cap) return PB_OK;
  int64_t cap = need < 1024 ? 1024 : need * 2;
  int* h = nullptr;
  PB_HIP(hipHostMalloc(&h, (size_t)cap * sizeof(int), hipHostMallocMapped));
  memset(h, 0, (size_t)cap * sizeof(int));
  if (k->h_done) {
    PB_TRY(wait_stream(k->A->grid->ctx, k->A->grid->ctx->stream, "KSP flag buffer"));
    memcpy(h, k->h_done, (size_t)k->done_cap * sizeof(int));
    (void)hipHostFree(k->h_done);
  }
  k->h_done = h;
  PB_HIP(hipHostGetDevicePointer((void**)&k->h_done_dev, h, 0));
  k->done_cap = cap;
  return PB_OK;
}

// z = M^-1 r for the stored-z preconditioners; *np = residual-sum partial blocks written by the
// PC itself (MG's last sweep), 0 if the caller must take the sums
static int pc_apply_dev(pb_ksp* k, const double* r, double* z, const int* skip, int* np) {
  *np = 0;
  if (k->fft) return fftpc_apply(k->fft, r, z, skip, k->d_st, np);
  return mg_apply(k->mg, r, z, skip, k->d_st, np);
}

int pb_ksp_begin(pb_ksp* k, const pb_vec* b, pb_vec* x) {
  PB_CHECK_ARG(k && b && x, "bad begin args");
  pb_grid* g = k->A->grid;
  PB_CHECK_ARG(b->grid == g && x->grid == g, "vector/operator grid mismatch");
  pb_ctx* ctx = g->ctx;
  // history buffer: max_it + 1 entries
  const int64_t nh = k->opts.max_it + 1;
  if (nh > k->nhist) {
    if (k->d_hist) (void)hipFree(k->d_hist);
    PB_HIP(hipMalloc(&k->d_hist, (size_t)nh * sizeof(double)));
    k->nhist = nh;
  }
  PB_TRY(ensure_done_cap(k, 1024));
  memset(k->h_done, 0, (size_t)k->done_cap * sizeof(int));
  CgState st;
  memset(&st, 0, sizeof(st));
  st.rtol = k->opts.rtol;
  st.atol = k->opts.atol;
  st.dtol = k->opts.dtol;
  st.max_it = k->opts.max_it;
  st.nhist = k->nhist;
  st.pc = k->opts.pc_type;
  st.nullspace = k->opts.nullspace;
  // PCJacobi stores the reciprocal of diag(P) (src/coefficients.f90:44-46 centre coefficient);
  // with SOR / MG the sums are taken over z = M^-1 r itself (dinv = 1)
  st.dinv = k->opts.pc_type == PB_PC_JACOBI ? 1.0 / k->P->cc : 1.0;
  st.ntot = (double)(g->n[0] * g->n[1] * g->n[2]);
  // depth 4 (default): 58 instead of 60 B/DoF per iteration, measured 3 % faster at 512^3
  // (profiles/r01/ab_defer_x.txt); the x update sums four alpha p terms instead of adding them
  // one per iteration (rounding-level difference in x only: the history is unaffected)
  const int dx = tune("cg_defer_x", 4);
  k->defer_x = dx == 0 ? 0 : (dx == 2 ? 2 : 4);
  if (!fused_kind(k->A->kind)) k->defer_x = 0;  // generic path: x every iteration
  st.defer_x = k->defer_x;
  // p stored by pass B (default): pass A read-only, 56 instead of 58 B/DoF per iteration and
  // the passes closer to their patterns' rates -- 1.29 vs 1.36 ms/iteration at 512^3 on one box
  // (profiles/r02/ab_pst_defer_512.jsonl); with a stored-z PC pass A stores p (the r01 split)
  k->pst = fused_kind(k->A->kind) && !k->stored_z();
  // single reduction: the fused operator with Jacobi / no PC (pass P forms p from r on load);
  // elsewhere the KSPSolve_CG iteration runs (equal in exact arithmetic; pb_ksp_opts)
  k->sr = k->opts.cg_single_reduction != 0 && fused_kind(k->A->kind) && !k->stored_z();
  st.sr = k->sr ? 1 : 0;
  if (k->sr) k->pst = true;  // r ping-pongs between r and r2 (pass P reads r_i, writes r_i+1)
  if (k->pst && !k->r2) {
    const size_t vb = (size_t)g->nlocal * sizeof(double);
    if (field_alloc(&k->r2, vb) != hipSuccess)
      return set_error(PB_ERR_ALLOC, "CG residual buffer: out of device memory");
  }
  if (k->defer_x == 4 && !k->pb[2]) {
    const size_t vb = (size_t)g->nlocal * sizeof(double);
    if (field_alloc(&k->pb[2], vb) != hipSuccess || field_alloc(&k->pb[3], vb) != hipSuccess)
      return set_error(PB_ERR_ALLOC, "CG direction buffers: out of device memory");
  }
  PB_HIP(hipMemcpyAsync(k->d_st, &st, sizeof(st), hipMemcpyHostToDevice, ctx->stream));
  // stored z with an operator without a stencil engine (compact A): r0 = b, x0 = 0 and p0 = 0 are
  // implicit -- the setup reads b in place of r, and the first iteration writes p = z, x = alpha p
  // and r = b - alpha w without reading them (three vector passes fewer)
  k->lazy0 = k->stored_z() && !fused_kind(k->A->kind) && tune("ksp_lazy0", 1) != 0;
  if (k->stored_z()) {
    // r = b, x = 0, p = 0; z = M^-1 r; sums of z (KSPSolve_CG setup, PC_LEFT)
    const size_t vb = (size_t)g->nlocal * sizeof(double);
    const double* r0 = k->lazy0 ? b->d : k->r;
    if (!k->lazy0) {
      PB_HIP(hipMemcpyAsync(k->r, b->d, vb, hipMemcpyDeviceToDevice, ctx->stream));
      PB_HIP(hipMemsetAsync(x->d, 0, vb, ctx->stream));
      PB_HIP(hipMemsetAsync(k->pb[0], 0, vb, ctx->stream));
    }
    int np = 0;
    PB_TRY(pc_apply_dev(k, r0, k->z, nullptr, &np));
    if (np == 0) PB_TRY(launch_cg_pc_sums(g, k->z, r0, k->d_st, &np));
    PB_TRY(cg_finalize_init(ctx, np, k->d_st, k->d_hist, k->h_done_dev));
  } else {
    PB_TRY(launch_cg_init(g, b->d, x->d, k->r, k->pb[0], k->d_st, st.dinv, k->d_hist,
                          k->h_done_dev));
    if (k->sr) {
      // KSPSolve_CG_SingleReduction's setup: S = A z, delta = z'S (pass S over r0 = b)
      int np = 0;
      PB_TRY(sr_pass_s(k, k->r, k->d_st, &np, 0));
      PB_TRY(cg_sr_finalize(ctx, sr_region(ctx, 0), np, k->d_st, k->d_hist, k->h_done_dev, -1,
                            true));
    }
  }
  PB_SYNC(ctx, "pb_ksp_begin");
  k->b = b;
  k->x = x;
  k->host_iter = 0;
  k->stopped = k->h_done[0] != 0;
  k->begun = true;
  return PB_OK;
}

// Unfused iteration for operators without a stencil engine (PB_OP_COMPACT): one vector pass
// for p, the operator, a dot pass, an x/r pass (same device scalar logic as the fused path).
static int enqueue_generic_iteration(pb_ksp* k) {
  pb_grid* g = k->A->grid;
  pb_ctx* ctx = g->ctx;
  double* p = k->pb[0];
  int np = 0;
  PB_TRY(launch_cg_generic_p(g, k->r, p, k->d_st));
  {
    OpApplySkip guard(ctx, &k->d_st->done);
    PB_TRY(op_apply_raw(k->A, p, k->w));
  }
  PB_TRY(launch_cg_generic_dot(g, p, k->w, k->d_st, &np));
  PB_TRY(cg_finalize_pass_a(ctx, np, k->d_st));
  PB_TRY(launch_cg_generic_xr(g, p, k->w, k->x->d, k->r, k->d_st, &np));
  return cg_finalize_stage2(ctx, np, k->d_st, k->d_hist, k->h_done_dev, k->host_iter);
}

// Preconditioned iteration (SOR / MG): p = (z - mu) + b/b0 p, w = A p, p.w, x/r update,
// z = M^-1 r, sums of z -- PETSc KSPSolve_CG order with PC_LEFT and the null-space shift.
static int enqueue_pc_iteration(pb_ksp* k) {
  pb_grid* g = k->A->grid;
  pb_ctx* ctx = g->ctx;
  double* p = k->pb[0];
  int np = 0;
  const int first = k->lazy0 && k->host_iter == 0;  // r0 = b, x0 = 0, p0 = 0 implicit
  if (k->A->kind == PB_OP_COMPACT && (compact_cg_fusable(g) || compact_cg_fusable_split(g))) {
    // the compact operator forms p in its Z pass (split grids: in the pack of the z -> y
    // transpose) and takes p . w in its X pass (CgFuse): two vector passes fewer (cg_gen_p,
    // cg_gen_dot), 16 B/DoF less per iteration
    CgFuse cf;
    cf.z = k->z;
    cf.p_old = p;
    cf.p_out = p;
    cf.st = k->d_st;
    cf.first = first;
    cf.dot_p = p;
    {
      OpApplySkip guard(ctx, &k->d_st->done);
      struct Set {
        pb_ctx* c;
        ~Set() { c->cg_fuse = nullptr; }
      } set{ctx};
      ctx->cg_fuse = &cf;
      PB_TRY(op_apply_raw(k->A, p, k->w));
    }
    np = cf.nparts;
    if (!cf.fused_z) {
      // a pass did not take the fusion (a launch shape the predicate cannot see): the operator
      // ran on p_old -- form p and apply again, unfused
      PB_TRY(launch_cg_generic_p(g, k->z, p, k->d_st, first));
      OpApplySkip guard(ctx, &k->d_st->done);
      PB_TRY(op_apply_raw(k->A, p, k->w));
    }
    if (!cf.fused_z || !cf.fused_dot) PB_TRY(launch_cg_generic_dot(g, p, k->w, k->d_st, &np));
  } else {
    PB_TRY(launch_cg_generic_p(g, k->z, p, k->d_st, first));  // dinv = 1: z - mu
    {
      OpApplySkip guard(ctx, &k->d_st->done);
      PB_TRY(op_apply_raw(k->A, p, k->w));
    }
    PB_TRY(launch_cg_generic_dot(g, p, k->w, k->d_st, &np));
  }
  PB_TRY(cg_finalize_pass_a(ctx, np, k->d_st));
  const double* r_in = first ? k->b->d : k->r;
  const int rupd = tune("fft_rupd", 1);
  if (k->fft && rupd && fftpc_fuses_r_update(k->fft)) {
    // r = r_in - alpha w formed by the spectral PC's first pass as it loads r, x = x + alpha p
    // beside it (8 B/DoF and one vector pass fewer)
    const RUpdate ru{r_in, k->w, k->r, p, k->x->d, first, k->d_st};
    np = 0;
    PB_TRY(fftpc_apply(k->fft, k->r, k->z, &k->d_st->done, k->d_st, &np, &ru));
  } else {
    PB_TRY(launch_cg_pc_xr(g, p, k->w, k->x->d, r_in, k->r, k->d_st, first));
    PB_TRY(pc_apply_dev(k, k->r, k->z, &k->d_st->done, &np));
  }
  if (np == 0) PB_TRY(launch_cg_pc_sums(g, k->z, k->r, k->d_st, &np));
  return cg_finalize_stage2(ctx, np, k->d_st, k->d_hist, k->h_done_dev, k->host_iter);
}

// the single-reduction iteration's two partial-sum regions (5 wide): iteration n of a batch
// writes region n & 1 and its folded prologue reduces region (n - 1) & 1, so a launch never
// overwrites the partials its own blocks may still be reading (part_off in 5-wide blocks)
static int64_t sr_region_off(const pb_ctx* ctx, int64_t n) {
  return (n & 1) * (ctx->partials_cap / 10);
}
static const double* sr_region(const pb_ctx* ctx, int64_t n) {
  return ctx->d_partials + sr_region_off(ctx, n) * 5;
}

// pass S over r (t = dinv r - mu of state st): split grids exchange r's boundary planes (raw;
// the loader transforms ghosts too) under the interior planes. Every launch is bounded by the
// end of region n & 1 (a grid that does not fit is PB_ERR_UNSUPPORTED, not a spill into the
// region the next prologue reads)
static int sr_pass_s(pb_ksp* k, const double* r, const CgState* st, int* nparts, int64_t n) {
  pb_grid* g = k->A->grid;
  pb_ctx* ctx = g->ctx;
  Star s{k->A->cx, k->A->cy, k->A->cz, k->A->cc};
  StencilPlanes gp;
  const int off = (int)sr_region_off(ctx, n);
  const int end = off + (int)(ctx->partials_cap / 10);
  if (!ctx->split) {
    gp.ghost_lo = gp.ghost_hi = nullptr;
    gp.wrap = true;
    return launch_cg_sr_pass_s(g, s, r, gp, st, PLANES_ALL, off, end, nparts);
  }
  gp.ghost_lo = g->ghost_lo;
  gp.ghost_hi = g->ghost_hi;
  const double* hi = r + (g->nzl - 1) * g->plane;
  if (g->nzl < 3) {
    PB_TRY(halo_exchange(g, r, hi));
    return launch_cg_sr_pass_s(g, s, r, gp, st, PLANES_ALL, off, end, nparts);
  }
  int nb1 = 0, nb2 = 0;
  ScopedTimer tm(ctx, "cg_sr_s");
  PB_TRY(halo_begin(g, r, hi));
  PB_TRY(launch_cg_sr_pass_s(g, s, r, gp, st, PLANES_INTERIOR, off, end, &nb1));
  PB_TRY(halo_end(g));
  PB_TRY(launch_cg_sr_pass_s(g, s, r, gp, st, PLANES_BOUNDARY, off + nb1, end, &nb2));
  *nparts = nb1 + nb2;
  return PB_OK;
}

// One single-reduction iteration (PETSc KSPSolve_CG_SingleReduction): pass P, pass S, and -- unless
// folded into the next pass P's prologue (one rank) -- the reduction + residual-sum stage.
// n = the iteration's index inside this pb_ksp_iterate batch (state slot parity).
static int enqueue_sr_iteration(pb_ksp* k, bool fold, int64_t n) {
  pb_grid* g = k->A->grid;
  pb_ctx* ctx = g->ctx;
  Star s{k->A->cx, k->A->cy, k->A->cz, k->A->cc};
  const int64_t i = k->host_iter;
  const int ns = k->pslots();
  const double* p_prev[3] = {k->pb[i % ns], k->pb[(i + ns - 1) % ns], k->pb[(i + ns - 2) % ns]};
  double* p_new = k->pb[(i + 1) % ns];
  double* r = k->rbuf(i);
  double* r_out = k->rbuf(i + 1);
  // one rank: the state alternates between the slots by the batch index's parity; split grids:
  // slot 0 holds the state after the residual-sum stage (written by the boundary-plane kernel's
  // folded prologue, or copied there unfolded), slot 1 after the top of the iteration (pass P)
  CgState* st_in = ctx->split ? k->d_st : k->d_st + (n & 1);
  CgState* st_out = ctx->split ? k->d_st + 1 : k->d_st + ((n + 1) & 1);
  SrFold f;
  f.fold_sums = fold && n > 0 && !ctx->split;
  f.nparts_s = k->sr_nparts;
  f.parts = sr_region(ctx, n - 1);
  f.in = st_in;
  f.out = st_out;
  f.hist = k->d_hist;
  f.h_done = k->h_done_dev;
  StencilPlanes gp;
  // one pass per iteration where it applies: one rank, depth-4 x deferral; the iterations that
  // carry the x update run the two passes (pass P's x-update form streams at the copy rate)
  if (cg_sr1_supported(g) && k->defer_x == 4 && i % 4 != 3) {
    PB_TRY(launch_cg_sr1(g, s, r, p_prev[0], p_new, r_out, f, f.parts, const_cast<double*>(sr_region(ctx, n)), i,
                         &k->sr_nparts));
    if (!fold)
      PB_TRY(cg_sr_finalize(ctx, sr_region(ctx, n), k->sr_nparts, st_out, k->d_hist,
                            k->h_done_dev, i));
    return PB_OK;
  }
  if (!ctx->split) {
    gp.ghost_lo = gp.ghost_hi = nullptr;
    gp.wrap = true;
    PB_TRY(launch_cg_sr_pass_p(g, s, r, p_prev, p_new, k->x->d, r_out, gp, f, PLANES_ALL, i,
                               k->defer_x));
  } else {
    // p's boundary planes -> halo, under the interior planes. Folded: the boundary-plane kernel
    // first runs the previous iteration's residual-sum stage from pass S's allreduced sums (a
    // one-block partial, slot 1 -> slot 0); pass P then runs the top (slot 0 -> slot 1)
    Fold fb;
    if (fold && n > 0) {
      fb.stage = 2;
      fb.nparts = 1;
      fb.width = 5;
      fb.parts = ctx->d_scalars;
      fb.in = k->d_st + 1;
      fb.out = k->d_st;
      fb.hist = k->d_hist;
      fb.h_done = k->h_done_dev;
      fb.host_iter = i - 1;
    }
    gp.ghost_lo = g->ghost_lo;
    gp.ghost_hi = g->ghost_hi;
    PB_TRY(launch_cg_boundary(g, r, p_prev[0], st_in, fb));
    if (g->nzl < 3) {
      PB_TRY(halo_exchange(g, g->bnd_lo, g->bnd_hi));
      PB_TRY(launch_cg_sr_pass_p(g, s, r, p_prev, p_new, k->x->d, r_out, gp, f, PLANES_ALL, i,
                                 k->defer_x));
    } else {
      ScopedTimer tm(ctx, "cg_sr_p_split");
      PB_TRY(halo_begin(g, g->bnd_lo, g->bnd_hi));
      PB_TRY(launch_cg_sr_pass_p(g, s, r, p_prev, p_new, k->x->d, r_out, gp, f, PLANES_INTERIOR,
                                 i, k->defer_x));
      PB_TRY(halo_end(g));
      PB_TRY(launch_cg_sr_pass_p(g, s, r, p_prev, p_new, k->x->d, r_out, gp, f, PLANES_BOUNDARY,
                                 i, k->defer_x));
    }
  }
  PB_TRY(sr_pass_s(k, r_out, st_out, &k->sr_nparts, n));
  if (fold && ctx->split) return cg_reduce_allreduce(ctx, sr_region(ctx, n), k->sr_nparts, 5);
  if (!fold)
    PB_TRY(cg_sr_finalize(ctx, sr_region(ctx, n), k->sr_nparts, st_out, k->d_hist,
                          k->h_done_dev, i));
  if (!fold && ctx->split)  // the next boundary-plane kernel reads slot 0
    PB_HIP(hipMemcpyAsync(k->d_st, st_out, sizeof(CgState), hipMemcpyDeviceToDevice,
                          ctx->stream));
  return PB_OK;
}

// fold: the finalize steps run in the passes' prologues (one rank, Jacobi; fold_a = pass A also
// folds, i.e. this is not the first iteration of the batch)
static int enqueue_iteration(pb_ksp* k, bool fold, bool fold_a) {
  if (!fused_kind(k->A->kind))
    return k->stored_z() ? enqueue_pc_iteration(k) : enqueue_generic_iteration(k);
  pb_grid* g = k->A->grid;
  pb_ctx* ctx = g->ctx;
  Star s{k->A->cx, k->A->cy, k->A->cz, k->A->cc};
  const int64_t i = k->host_iter;  // == device iteration index until convergence
  const int ns = k->pslots();
  double* p_old = k->pb[i % ns];
  double* p_new = k->pb[(i + 1) % ns];
  // p of iterations i-1, i-2, i-3 (depth-4 deferral reads all three at i % 4 == 3)
  const double* p_prev[3] = {p_old, k->pb[(i + ns - 1) % ns], k->pb[(i + ns - 2) % ns]};
  // Jacobi: pass A builds z = dinv*r - mu on the fly; SOR / MG: z is stored (dinv = 1)
  double* r = k->rbuf(i);
  const double* zsrc = k->stored_z() ? k->z : r;
  // Jacobi / none: pass A read-only, pass B stores p and the residual into the other buffer
  PStore ps;
  if (k->pst) {
    ps.zsrc = zsrc;
    ps.r_out = k->rbuf(i + 1);
  }
  const bool store_a = !k->pst;
  StencilPlanes gp;
  int nparts = 0;
  const bool fold_split = fold && ctx->split;
  if (fold && !ctx->split) {
    gp.ghost_lo = gp.ghost_hi = nullptr;
    gp.wrap = true;
    if (fold_a)
      PB_TRY(launch_cg_pass_a_folded(g, s, zsrc, p_old, p_new, gp, k->d_st, k->fold_nparts_b,
                                     k->d_hist, k->h_done_dev, i, &nparts, store_a));
    else
      PB_TRY(launch_cg_pass_a(g, s, zsrc, p_old, p_new, gp, k->d_st, PLANES_ALL, 0, &nparts,
                              store_a));
    return launch_cg_pass_b_folded(g, s, p_new, p_prev, k->x->d, r, gp, k->d_st, nparts, i,
                                   k->defer_x, &k->fold_nparts_b, ps);
  }
  if (fold_split) {
    // split grids, folded (r05): the previous iteration's stage 2 runs in the prologues of the
    // boundary-plane kernel and pass A (from pass B's allreduced sums, a one-block partial), stage
    // 1 in pass B's (from pass A's); only the reductions before each allreduce stay separate
    // launches (bit-identical to unfolded)
    Fold fb;
    if (fold_a) {
      fb.stage = 2;
      fb.nparts = 1;
      fb.width = 4;
      fb.parts = ctx->d_scalars;
      fb.in = k->d_st + 1;
      fb.out = k->d_st;
      fb.hist = k->d_hist;
      fb.h_done = k->h_done_dev;
      fb.host_iter = i - 1;
    }
    gp.ghost_lo = g->ghost_lo;
    gp.ghost_hi = g->ghost_hi;
    if (g->nzl >= 3) {
      // the boundary-plane kernel runs on the comm stream ahead of the exchange, beside pass A's
      // interior planes, from the stage-2 state in its registers; pass A's interior launch runs the
      // same stage 2 in its prologue and writes the state (the boundary launch reads it)
      Fold fbr = fb;
      fbr.out = nullptr;
      fbr.hist = nullptr;
      fbr.h_done = nullptr;
      int nb1 = 0, nb2 = 0;
      ScopedTimer tm(ctx, "cg_pass_a");
      PB_TRY(halo_begin_after(g, g->bnd_lo, g->bnd_hi, [&](hipStream_t sm) {
        return launch_cg_boundary(g, zsrc, p_old, k->d_st, fbr, sm);
      }));
      if (fold_a)
        PB_TRY(launch_cg_pass_a_fold(g, s, zsrc, p_old, p_new, gp, fb, PLANES_INTERIOR, 0, &nb1,
                                     store_a));
      else
        PB_TRY(launch_cg_pass_a(g, s, zsrc, p_old, p_new, gp, k->d_st, PLANES_INTERIOR, 0, &nb1,
                                store_a));
      if (ctx->comm) {
        // the two boundary planes on the comm stream right after the exchange (beside the
        // interior planes), from the stage-2 state in registers as well
        EngineOn eo(ctx, ctx->comm_stream);
        if (fold_a)
          PB_TRY(launch_cg_pass_a_fold(g, s, zsrc, p_old, p_new, gp, fbr, PLANES_BOUNDARY, nb1,
                                       &nb2, store_a));
        else
          PB_TRY(launch_cg_pass_a(g, s, zsrc, p_old, p_new, gp, k->d_st, PLANES_BOUNDARY, nb1,
                                  &nb2, store_a));
        PB_HIP(hipEventRecord(ctx->ev_done, ctx->comm_stream));
        PB_TRY(halo_end(g));
      } else {
        PB_TRY(halo_end(g));
        PB_TRY(launch_cg_pass_a(g, s, zsrc, p_old, p_new, gp, k->d_st, PLANES_BOUNDARY, nb1,
                                &nb2, store_a));
      }
      nparts = nb1 + nb2;
    } else {
      PB_TRY(launch_cg_boundary(g, zsrc, p_old, k->d_st, fb));
      PB_TRY(halo_exchange(g, g->bnd_lo, g->bnd_hi));
      PB_TRY(launch_cg_pass_a(g, s, zsrc, p_old, p_new, gp, k->d_st, PLANES_ALL, 0, &nparts,
                              store_a));
    }
    PB_TRY(cg_reduce_allreduce(ctx, nparts, 1, false));
    PB_TRY(launch_cg_pass_b_folded(g, s, p_new, p_prev, k->x->d, r, gp, k->d_st, 1, i,
                                   k->defer_x, &k->fold_nparts_b, ps, ctx->d_scalars));
    return cg_reduce_allreduce(ctx, k->fold_nparts_b, 4, true);
  }
  if (!ctx->split) {
    // periodic wrap read in place: pass A combines r, p_old of the wrap planes itself and pass B
    // reads p_new's wrap planes (no boundary-plane kernel on one rank)
    gp.ghost_lo = gp.ghost_hi = nullptr;
    gp.wrap = true;
    PB_TRY(launch_cg_pass_a(g, s, zsrc, p_old, p_new, gp, k->d_st, PLANES_ALL, 0, &nparts,
                            store_a));
  } else if (g->nzl < 3) {
    PB_TRY(launch_cg_boundary(g, zsrc, p_old, k->d_st));
    PB_TRY(halo_exchange(g, g->bnd_lo, g->bnd_hi));
    gp.ghost_lo = g->ghost_lo;
    gp.ghost_hi = g->ghost_hi;
    PB_TRY(launch_cg_pass_a(g, s, zsrc, p_old, p_new, gp, k->d_st, PLANES_ALL, 0, &nparts,
                            store_a));
  } else {
    // the p-plane halo exchange (RCCL, comm stream) overlaps pass A's interior planes
    PB_TRY(launch_cg_boundary(g, zsrc, p_old, k->d_st));
    gp.ghost_lo = g->ghost_lo;
    gp.ghost_hi = g->ghost_hi;
    int nb1 = 0, nb2 = 0;
    ScopedTimer tm(ctx, "cg_pass_a");  // the whole pass A (both launches and the wait)
    PB_TRY(halo_begin(g, g->bnd_lo, g->bnd_hi));
    PB_TRY(launch_cg_pass_a(g, s, zsrc, p_old, p_new, gp, k->d_st, PLANES_INTERIOR, 0, &nb1,
                            store_a));
    PB_TRY(halo_end(g));
    PB_TRY(launch_cg_pass_a(g, s, zsrc, p_old, p_new, gp, k->d_st, PLANES_BOUNDARY, nb1, &nb2,
                            store_a));
    nparts = nb1 + nb2;
  }
  PB_TRY(cg_finalize_pass_a(ctx, nparts, k->d_st));
  PB_TRY(launch_cg_pass_b(g, s, p_new, p_prev, k->x->d, r, gp, k->d_st, k->d_hist,
                          k->h_done_dev, i, k->defer_x, !k->stored_z(), ps));
  if (k->stored_z()) {  // z = M^-1 r, then the residual sums over z
    int np = 0;
    PB_TRY(pc_apply_dev(k, r, k->z, &k->d_st->done, &np));
    if (np == 0) PB_TRY(launch_cg_pc_sums(g, k->z, r, k->d_st, &np));
    PB_TRY(cg_finalize_stage2(ctx, np, k->d_st, k->d_hist, k->h_done_dev, i));
  }
  return PB_OK;
}

int pb_ksp_iterate(pb_ksp* k, int64_t iters) {
  PB_CHECK_ARG(k, "ksp is NULL");
  if (!k->begun) return set_error(PB_ERR_STATE, "pb_ksp_iterate before pb_ksp_begin");
  pb_ctx* ctx = k->A->grid->ctx;
  const int C = k->opts.check_every;
  const int R = 4 * C;
  if ((int)k->ring.size() < R) {
    for (int i = (int)k->ring.size(); i < R; ++i) {
      hipEvent_t e;
      PB_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      k->ring.push_back(e);
    }
  }
  PB_TRY(ensure_done_cap(k, k->host_iter + iters + 2));
  // one rank, Jacobi, fused operator: the finalize steps ride in the passes' prologues
  // (PB_CG_FOLD=0 keeps the separate finalize launches)
  const bool fold = C >= 2 && fused_kind(k->A->kind) && !k->stored_z() && tune("cg_fold", 1) != 0;
  int64_t n = 0;
  for (; n < iters && !k->stopped; ++n) {
    if (k->sr) PB_TRY(enqueue_sr_iteration(k, fold, n));
    else PB_TRY(enqueue_iteration(k, fold, fold && n > 0));
    const int64_t hi = k->host_iter++;
    // only the iterations the poll below waits for get an event (j = 0 mod C; folded j + 1): an
    // event record between two kernels costs the stream ~6 us of idle time (measured 5.9 us per
    // iteration with one record per iteration; profiles/r02/cg_gaps_*.txt)
    if (hi % C == (fold ? 1 : 0) % C)
      PB_HIP(hipEventRecord(k->ring[hi % R], ctx->stream));
    // lagged, rank-consistent poll: decide on the flag of iteration hi + 1 - C only (folded:
    // that flag is written by the next iteration's pass A, so wait for that iteration's event)
    if ((hi + 1) % C == 0 && hi + 1 >= C) {
      const int64_t j = hi + 1 - C;
      PB_TRY(wait_event(ctx, k->ring[(fold ? j + 1 : j) % R], "KSP convergence poll"));
      if (k->h_done[j + 1]) k->stopped = true;
    }
  }
  if (k->sr) {
    // the residual-sum stage of the batch's last iteration (folded runs), then the state back
    // into slot 0 for the next batch and the other entry points
    if (ctx->split) {  // (unfolded: the state is in slot 0 already)
      if (fold && n > 0) {
        PB_TRY(cg_stage2_from_sums(ctx, 5, k->d_st + 1, k->d_hist, k->h_done_dev,
                                   k->host_iter - 1));
        PB_HIP(hipMemcpyAsync(k->d_st, k->d_st + 1, sizeof(CgState), hipMemcpyDeviceToDevice,
                              ctx->stream));
      }
      return PB_OK;
    }
    if (fold && n > 0)
      PB_TRY(cg_sr_finalize(ctx, sr_region(ctx, n - 1), k->sr_nparts, k->d_st + (n & 1),
                            k->d_hist, k->h_done_dev, k->host_iter - 1));
    if (n & 1)
      PB_HIP(hipMemcpyAsync(k->d_st, k->d_st + 1, sizeof(CgState), hipMemcpyDeviceToDevice,
                            ctx->stream));
    return PB_OK;
  }
  if (fold && n > 0)
    PB_TRY(cg_fold_tail(ctx, k->fold_nparts_b, k->d_st, k->d_hist, k->h_done_dev,
                        k->host_iter - 1));
  return PB_OK;
}

static const char* reason_name(int r) {
  switch (r) {
    case PB_KSP_CONVERGED_RTOL: return "CONVERGED_RTOL";
    case PB_KSP_CONVERGED_ATOL: return "CONVERGED_ATOL";
    case PB_KSP_CONVERGED_ITS: return "CONVERGED_ITS";
    case PB_KSP_DIVERGED_ITS: return "DIVERGED_ITS";
    case PB_KSP_DIVERGED_DTOL: return "DIVERGED_DTOL";
    case PB_KSP_DIVERGED_NANORINF: return "DIVERGED_NANORINF";
    case PB_KSP_DIVERGED_INDEFINITE_MAT: return "DIVERGED_INDEFINITE_MAT";
    case PB_KSP_DIVERGED_INDEFINITE_PC: return "DIVERGED_INDEFINITE_PC";
    default: return "CONVERGED_ITERATING";
  }
}

int pb_ksp_end(pb_ksp* k, pb_ksp_result* res, double* history, int64_t cap) {
  PB_CHECK_ARG(k, "ksp is NULL");
  if (!k->begun) return set_error(PB_ERR_STATE, "pb_ksp_end before pb_ksp_begin");
  pb_ctx* ctx = k->A->grid->ctx;
  PB_SYNC(ctx, "pb_ksp_end");
  if (k->lazy0 && k->host_iter == 0) {  // stopped at the setup: x = x0 = 0 was never written
    PB_HIP(hipMemsetAsync(k->x->d, 0, (size_t)k->A->grid->nlocal * sizeof(double), ctx->stream));
  }
  CgState st;
  PB_HIP(hipMemcpyAsync(&st, k->d_st, sizeof(st), hipMemcpyDeviceToHost, ctx->stream));
  PB_SYNC(ctx, "pb_ksp_end");
  if (st.pend_iter >= 0) {  // apply the still-deferred alpha_m p_m (p_m lives in pb[(m+1) % ns])
    const int ns = k->pslots();
    for (int64_t m = 0; m < st.pend_count; ++m)
      PB_TRY(launch_cg_flush(k->A->grid, k->x->d, k->pb[(st.pend_iter + m + 1) % ns], st.pa[m]));
    PB_SYNC(ctx, "pb_ksp_end");
  }
  if (res) {
    res->reason = st.reason;
    res->its = st.its;
    res->rnorm = st.dp;
    res->rnorm0 = st.rnorm0;
    res->nhist = std::min<int64_t>(st.nlog, k->nhist);
  }
  // only the norms the device logged (a breakdown exit leaves the last iteration without one)
  const int64_t nh = std::min<int64_t>(st.nlog, k->nhist);
  std::vector<double> hist((size_t)std::max<int64_t>(nh, 1));
  if (nh > 0) {
    PB_HIP(hipMemcpyAsync(hist.data(), k->d_hist, (size_t)nh * sizeof(double), hipMemcpyDeviceToHost,
                          ctx->stream));
    PB_SYNC(ctx, "pb_ksp_end");
  }
  if (history && cap > 0) memcpy(history, hist.data(), (size_t)std::min(nh, cap) * sizeof(double));
  if (ctx->rank == 0) {
    if (k->opts.monitor)
      for (int64_t i = 0; i < nh; ++i)
        printf("  %3lld KSP Residual norm %14.12e \n", (long long)i, hist[i]);
    if (k->opts.converged_reason) {
      if (st.reason > 0)
        printf("Linear solve converged due to %s iterations %lld\n", reason_name(st.reason),
               (long long)st.its);
      else
        printf("Linear solve did not converge due to %s iterations %lld\n",
               reason_name(st.reason), (long long)st.its);
    }
    fflush(stdout);
  }
  k->begun = false;
  return PB_OK;
}

int pb_ksp_solve(pb_ksp* k, const pb_vec* b, pb_vec* x, pb_ksp_result* res, double* history,
                 int64_t cap) {
  ScopedTimer tm(k->A->grid->ctx, "KSPSolve");
  PB_TRY(pb_ksp_begin(k, b, x));
  PB_TRY(pb_ksp_iterate(k, k->opts.max_it + 2 * (int64_t)k->opts.check_every));
  return pb_ksp_end(k, res, history, cap);
}

int pb_ksp_destroy(pb_ksp* k) {
  if (!k) return PB_OK;
  (void)wait_stream(k->A->grid->ctx, k->A->grid->ctx->stream, "pb_ksp_destroy");
  field_free(k->r);
  field_free(k->r2);
  for (double* p : k->pb) field_free(p);
  field_free(k->w);
  field_free(k->z);
  if (k->mg) mg_destroy(k->mg);
  fftpc_destroy(k->fft);
  if (k->d_st) (void)hipFree(k->d_st);
  if (k->d_hist) (void)hipFree(k->d_hist);
  if (k->h_done) (void)hipHostFree(k->h_done);
  for (hipEvent_t e : k->ring) (void)hipEventDestroy(e);
  delete k;
  return PB_OK;
}

int pb_ksp_pc_apply(pb_ksp* k, const pb_vec* r, pb_vec* z) {
  PB_CHECK_ARG(k && r && z && r != z, "bad pc apply args");
  pb_grid* g = k->A->grid;
  PB_CHECK_ARG(r->grid == g && z->grid == g, "vector/operator grid mismatch");
  pb_ctx* ctx = g->ctx;
  if (k->mg) {
    PB_TRY(mg_apply(k->mg, r->d, z->d));
  } else if (k->fft) {
    PB_TRY(fftpc_apply(k->fft, r->d, z->d));
  } else {
    PB_HIP(hipMemcpyAsync(z->d, r->d, (size_t)g->nlocal * sizeof(double),
                          hipMemcpyDeviceToDevice, ctx->stream));
    if (k->opts.pc_type == PB_PC_JACOBI)
      PB_TRY(vec_update(ctx, 2, z->d, nullptr, g->nlocal, 1.0 / k->P->cc));
  }
  PB_SYNC(ctx, "pb_ksp_pc_apply");
  return PB_OK;
}

int pb_ksp_pc_levels(const pb_ksp* k, int* levels) {
  PB_CHECK_ARG(k && levels, "bad args");
  *levels = k->mg ? mg_levels(k->mg) : 0;
  return PB_OK;
}

int pb_solve(pb_op* A, pb_op* P, const pb_ksp_opts* opts, const pb_vec* b, pb_vec* x,
             pb_ksp_result* res, double* history, int64_t cap) {
  pb_ksp* k = nullptr;
  PB_TRY(pb_ksp_create(A, P, opts, &k));
  int rc = pb_ksp_solve(k, b, x, res, history, cap);
  pb_ksp_destroy(k);
  return rc;
}

}  // extern "C"
