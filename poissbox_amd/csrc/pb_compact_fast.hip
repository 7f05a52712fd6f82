// pb_compact_fast.hip -- bandwidth-oriented 6th-order compact Laplacian (3-pass factorisation).
//
// The reference (src/compact_schemes.f90:17-37) evaluates lapl = div(grad f) as 16 families of
// 1-D periodic tridiagonal line solves (8 for grad :42-88, 8 for div :207-257). Every 1-D operator
// is circulant, so operators on different axes commute and the same-axis pairs compose:
//     lapl = Lx Jy Jz + Jx Ly Jz + Jx Jy Lz,   L = D+ D-  (div_1d o grad_1d),
//                                              J = I+ I-  (interp_1d_div o interp_1d)
// (SURVEY.md Appendix D). Three passes, each reading/writing whole lines once:
//     Z: f -> u = Jz f, v = Lz f            (read 8, write 16 B/DoF)
//     Y: u, v -> s = Jy u, t = Ly u + Jy v  (read 16, write 16)
//     X: s, t -> out = Lx s + Jx t          (read 16, write 8)   = 80 B/DoF algorithmic
// Each 1-D half-operator (e.g. I-) is the reference's explicit 4-point RHS (eval_1d_rhs
// :332-372) followed by the (alpha, 1, alpha) periodic solve (:197, :312), done here by parallel
// cyclic reduction with the line tile in LDS. The system is circulant, so every PCR step is ONE
// scalar k_s: d_i <- d_i - k_s (d_{i-2^s} + d_{i+2^s}); the couplings decay as rho^(2^s)
// (rho = 1/3 interp, 0.148 grad): 6 resp. 5 steps reach < 1e-26 relative, or the exact
// self-coupled end state when n is a power of two. Results agree with the reference to rounding
// (operation order differs); the bit-exact reference-order path stays in pb_compact.hip.
#include <cmath>

#include "pb_internal.hpp"

namespace pb {

static constexpr int kFT = 256;  // threads per block
static constexpr int kFC = 16;   // elements per thread (tile = 4096 elements = TL lines x n)
static constexpr int kTile = kFT * kFC;

struct Pcr {
  int S;
  double k[12];
  double inv_b;
};
struct Half {  // one 1-D half operator: RHS (a, b, sign) then solve
  double a, b, sign;
  Pcr pcr;
};
struct Op {  // J or L = Half(+1) o Half(-1)
  Half h;
};
struct Term {
  int op;  // 0 = J, 1 = L
  int in;  // input index
  int out; // output index
};
struct FastPass {
  int n;          // line length
  int TL;         // lines per tile
  int layout;     // 0: flat = e*TL + l (lines contiguous in memory); 1: flat = l*n + e
  int ninner;     // lines along the tile direction
  int nouter;
  int64_t li, lo, es;  // address of (outer, inner, e) = outer*lo + inner*li + e*es
  int ntiles_inner;
  int nterms;
  Term term[3];
  Op ops[2];
  const double* in[2];
  double* out[2];
  int nout;
  const int* skip;  // pb_ctx::op_skip (exit at entry once set)
};

static Pcr make_pcr(int64_t n, double alpha) {
  Pcr p;
  double a = alpha, b = 1.0;
  const bool pow2 = (n & (n - 1)) == 0;
  int S = 0;
  bool folded = false;
  for (; S < 12; ++S) {
    if (std::fabs(a / b) < 1e-22) break;
    const int64_t dist = (int64_t)1 << S;
    p.k[S] = a / b;
    const double a2 = -a * a / b;
    b = b - 2.0 * a * a / b;
    a = a2;
    if (pow2 && 2 * dist == n) {  // next couplings sit at distance n: fold onto the diagonal
      ++S;
      folded = true;
      break;
    }
  }
  p.S = S;
  p.inv_b = folded ? 1.0 / (b + 2.0 * a) : 1.0 / b;
  return p;
}

static Op make_op(int kind, int64_t n, double h) {
  Op o;
  if (kind == 0) {  // J: interp (src/compact_schemes.f90:303-305)
    o.h.a = 0.75;
    o.h.b = 1.0 / 20.0;
    o.h.sign = 1.0;
    o.h.pcr = make_pcr(n, 3.0 / 10.0);
  } else {  // L: grad/div (:188-190)
    o.h.a = 63.0 / 62.0 / h;
    o.h.b = 17.0 / 62.0 / (3.0 * h);
    o.h.sign = -1.0;
    o.h.pcr = make_pcr(n, 9.0 / 62.0);
  }
  return o;
}

__device__ __forceinline__ int wrapi(int e, int n) { return e < 0 ? e + n : (e >= n ? e - n : e); }

// flat index of (line l, element e) in the tile / LDS
__device__ __forceinline__ int fidx(const FastPass& p, int l, int e) {
  return p.layout == 0 ? e * p.TL + l : l * p.n + e;
}

__global__ __launch_bounds__(kFT) void compact_fast_kernel(FastPass p) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  if (p.skip && *p.skip) return;  // (uniform: the whole block leaves before any barrier)
  const int tile = blockIdx.x;
  const int outer = tile / p.ntiles_inner;
  const int inner0 = (tile % p.ntiles_inner) * p.TL;
  const int nelem = p.n * p.TL;
  // this thread's elements: flat f = threadIdx.x + kFT*m
  int le[kFC], ee[kFC];
  bool ok[kFC];
  int64_t gaddr[kFC];
#pragma unroll
  for (int m = 0; m < kFC; ++m) {
    const int f = threadIdx.x + kFT * m;
    int l, e;
    if (p.layout == 0) {
      l = f % p.TL;
      e = f / p.TL;
    } else {
      l = f / p.n;
      e = f % p.n;
    }
    ok[m] = f < nelem && inner0 + l < p.ninner;
    le[m] = l;
    ee[m] = e;
    gaddr[m] = ok[m] ? (int64_t)outer * p.lo + (int64_t)(inner0 + l) * p.li + (int64_t)e * p.es : 0;
  }
  double x[kFC], d[kFC], acc[2][kFC];
#pragma unroll
  for (int m = 0; m < kFC; ++m) acc[0][m] = acc[1][m] = 0.0;
  int loaded = -1;

  // d <- RHS(half h, stagger) of the values currently in x
  auto rhs = [&](const Half& h, int shift) {
#pragma unroll
    for (int m = 0; m < kFC; ++m)
      if (ok[m]) lds[fidx(p, le[m], ee[m])] = x[m];
    __syncthreads();
#pragma unroll
    for (int m = 0; m < kFC; ++m) {
      if (!ok[m]) continue;
      const int l = le[m], e = ee[m];
      const double f0 = lds[fidx(p, l, wrapi(e + shift, p.n))];
      const double fm1 = lds[fidx(p, l, wrapi(e - 1 + shift, p.n))];
      const double f1 = lds[fidx(p, l, wrapi(e + 1 + shift, p.n))];
      const double fm2 = lds[fidx(p, l, wrapi(e - 2 + shift, p.n))];
      d[m] = h.a * (f0 + h.sign * fm1) + h.b * (f1 + h.sign * fm2);
    }
    __syncthreads();
  };
  // d <- A^-1 d by truncated / folded parallel cyclic reduction
  auto solve = [&](const Pcr& c) {
    for (int s = 0; s < c.S; ++s) {
      const int dist = (1 << s) % p.n;
#pragma unroll
      for (int m = 0; m < kFC; ++m)
        if (ok[m]) lds[fidx(p, le[m], ee[m])] = d[m];
      __syncthreads();
      const double k = c.k[s];
#pragma unroll
      for (int m = 0; m < kFC; ++m) {
        if (!ok[m]) continue;
        const int l = le[m], e = ee[m];
        const double dm = lds[fidx(p, l, wrapi(e - dist, p.n))];
        const double dp = lds[fidx(p, l, wrapi(e + dist, p.n))];
        d[m] = d[m] - k * (dm + dp);
      }
      __syncthreads();
    }
#pragma unroll
    for (int m = 0; m < kFC; ++m) d[m] = d[m] * c.inv_b;
  };

  for (int t = 0; t < p.nterms; ++t) {
    const Term tm = p.term[t];
    if (tm.in != loaded) {
      const double* src = p.in[tm.in];
#pragma unroll
      for (int m = 0; m < kFC; ++m) x[m] = ok[m] ? src[gaddr[m]] : 0.0;
      loaded = tm.in;
    }
    const Half& h = p.ops[tm.op].h;
    rhs(h, 0);     // stagger -1 (cell -> vertex)
    solve(h.pcr);
    double keep[kFC];
#pragma unroll
    for (int m = 0; m < kFC; ++m) {
      keep[m] = x[m];
      x[m] = d[m];
    }
    rhs(h, 1);     // stagger +1 (vertex -> cell)
    solve(h.pcr);
#pragma unroll
    for (int m = 0; m < kFC; ++m) {
      x[m] = keep[m];
      if (tm.out == 0) acc[0][m] += d[m];
      else acc[1][m] += d[m];
    }
  }
  for (int o = 0; o < p.nout; ++o) {
    double* dst = p.out[o];
#pragma unroll
    for (int m = 0; m < kFC; ++m)
      if (ok[m]) __builtin_nontemporal_store(o == 0 ? acc[0][m] : acc[1][m], dst + gaddr[m]);
  }
}

static int launch_pass(pb_ctx* ctx, FastPass& p) {
  p.skip = ctx->op_skip;
  p.TL = kTile / p.n;
  if (p.TL < 1) return set_error(PB_ERR_UNSUPPORTED, "compact fast path: line length > %d", kTile);
  if (p.TL > p.ninner) p.TL = p.ninner;
  p.ntiles_inner = (p.ninner + p.TL - 1) / p.TL;
  const int64_t nblocks = (int64_t)p.ntiles_inner * p.nouter;
  const size_t lds = (size_t)p.n * p.TL * sizeof(double);
  hipLaunchKernelGGL(compact_fast_kernel, dim3((unsigned)nblocks), dim3(kFT), lds, ctx->stream, p);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

// ---- the three passes on an explicit box (nx, ny, nz) whose lines along the pass axis are
// complete: the caller's grid on one rank, the y-slab of the transposed data for the Z pass on N
// ranks. Register line solves where n = 64*C supports them, the LDS-PCR kernel otherwise. ----
static bool reg_lines(int64_t n) {
  const bool lines_ok = tune("compact_lines", 1) != 0;
  return lines_ok && compact_lines_supported(n);
}

// Z: u = Jz f, v = Lz f
int compact_pass_z(pb_ctx* ctx, const int64_t d[3], double h, const double* f, double* u, double* v) {
  const int64_t nx = d[0], ny = d[1], nz = d[2];
  if (nz > kTile) return set_error(PB_ERR_UNSUPPORTED, "compact fast path: n > %d", kTile);
  if (reg_lines(nz)) return compact_lines_pass(ctx, d, 2, h, f, nullptr, u, v);
  FastPass p{};  // lines along k; tile = consecutive i for fixed j
  p.n = (int)nz;
  p.layout = 0;
  p.ninner = (int)nx;
  p.nouter = (int)ny;
  p.li = 1;
  p.lo = nx;
  p.es = nx * ny;
  p.nterms = 2;
  p.term[0] = Term{0, 0, 0};
  p.term[1] = Term{1, 0, 1};
  p.ops[0] = make_op(0, nz, h);
  p.ops[1] = make_op(1, nz, h);
  p.in[0] = f;
  p.out[0] = u;
  p.out[1] = v;
  p.nout = 2;
  return launch_pass(ctx, p);
}

// Y: s = Jy u, t = Ly u + Jy v
int compact_pass_y(pb_ctx* ctx, const int64_t d[3], double h, const double* u, const double* v,
                   double* s_, double* t, const YSlabPlan* blk_in) {
  const int64_t nx = d[0], ny = d[1], nz = d[2];
  if (ny > kTile) return set_error(PB_ERR_UNSUPPORTED, "compact fast path: n > %d", kTile);
  if (reg_lines(ny)) return compact_lines_pass(ctx, d, 1, h, u, v, s_, t, blk_in);
  if (blk_in) return set_error(PB_ERR_ARG, "compact Y pass: blocked input needs the line solves");
  FastPass p{};  // lines along j; tile = consecutive i for fixed k
  p.n = (int)ny;
  p.layout = 0;
  p.ninner = (int)nx;
  p.nouter = (int)nz;
  p.li = 1;
  p.lo = nx * ny;
  p.es = nx;
  p.nterms = 3;
  p.term[0] = Term{0, 0, 0};  // s = Jy u
  p.term[1] = Term{1, 0, 1};  // t = Ly u
  p.term[2] = Term{0, 1, 1};  //   + Jy v
  p.ops[0] = make_op(0, ny, h);
  p.ops[1] = make_op(1, ny, h);
  p.in[0] = u;
  p.in[1] = v;
  p.out[0] = s_;
  p.out[1] = t;
  p.nout = 2;
  return launch_pass(ctx, p);
}

// X: out = Lx s + Jx t
int compact_pass_x(pb_ctx* ctx, const int64_t d[3], double h, const double* s_, const double* t,
                   double* out) {
  const int64_t nx = d[0], ny = d[1], nz = d[2];
  if (nx > kTile) return set_error(PB_ERR_UNSUPPORTED, "compact fast path: n > %d", kTile);
  if (reg_lines(nx)) return compact_lines_pass(ctx, d, 0, h, s_, t, out, nullptr);
  FastPass p{};  // lines along i (contiguous); tile = consecutive j for fixed k
  p.n = (int)nx;
  p.layout = 1;
  p.ninner = (int)ny;
  p.nouter = (int)nz;
  p.li = nx;
  p.lo = nx * ny;
  p.es = 1;
  p.nterms = 2;
  p.term[0] = Term{1, 0, 0};  // out = Lx s
  p.term[1] = Term{0, 1, 0};  //     + Jx t
  p.ops[0] = make_op(0, nx, h);
  p.ops[1] = make_op(1, nx, h);
  p.in[0] = s_;
  p.in[1] = t;
  p.out[0] = out;
  p.nout = 1;
  return launch_pass(ctx, p);
}

// work doubles: 4 N (u, v, s, t) on one rank; on N ranks also the y-slab fields and the
// transpose staging (compact_dist.cpp)
int64_t compact_fast_work_len(const pb_grid* g) {
  if (!g->ctx->split) return 4 * g->nlocal;
  return 4 * g->nlocal + compact_dist_work_len(g);
}

// lapl(f) into out
int compact_lapl_fast(pb_grid* g, const double dx[3], const double* f, double* out, double* work) {
  ScopedTimer tm(g->ctx, "compact_lapl_fast");
  const int64_t N = g->nlocal;
  double *u = work, *v = work + N, *s_ = work + 2 * N, *t = work + 3 * N;
  const int64_t d[3] = {g->n[0], g->n[1], g->nzl};
  if (!g->ctx->split) {
    PB_TRY(compact_pass_z(g->ctx, d, dx[2], f, u, v));
  } else {  // z-lines span the slabs: transpose to y-slabs, Z pass, transpose u, v back
    // (with the register line solves on y the Y pass reads u, v straight from the all-to-all
    // layout: no unpack passes)
    YSlabPlan bp;
    bool blocked = false;
    PB_TRY(compact_dist_pass_z(g, dx[2], f, u, v, work + 4 * N, reg_lines(d[1]) ? &bp : nullptr,
                               &blocked));
    PB_TRY(compact_pass_y(g->ctx, d, dx[1], u, v, s_, t, blocked ? &bp : nullptr));
    return compact_pass_x(g->ctx, d, dx[0], s_, t, out);
  }
  PB_TRY(compact_pass_y(g->ctx, d, dx[1], u, v, s_, t));
  return compact_pass_x(g->ctx, d, dx[0], s_, t, out);
}

}  // namespace pb

extern "C" int pb_compact_lapl_fast(pb_grid* g, const double dx[3], const pb_vec* f, pb_vec* out) {
  using namespace pb;
  PB_CHECK_ARG(g && dx && f && out && f != out, "bad lapl args");
  double* ws = nullptr;
  PB_TRY(ctx_scratch(g->ctx, (size_t)compact_fast_work_len(g), &ws));
  int rc = compact_lapl_fast(g, dx, f->d, out->d, ws);
  return rc;
}
