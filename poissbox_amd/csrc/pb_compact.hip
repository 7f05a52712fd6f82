// pb_compact.hip -- batched tridiagonal solvers and the 6th-order staggered compact operators.
//
// Replaces src/tridsol.f90 (tdma, tdma_periodic, fwd_sweep, bwd_sweep) and
// src/compact_schemes.f90 (grad/div/interp/interp_div/lapl and their 1-D forms).
//
// * General systems (pb_tdma_batched): one lane per line, Thomas + Sherman-Morrison in the
//   reference's exact operation order (bit-identical results with -ffp-contract=off).
// * Compact-scheme systems are constant-coefficient periodic (alpha, 1, alpha): the Thomas
//   factorisation (multipliers, modified diagonal, Sherman-Morrison vector) is the same for every
//   line, so it is computed once on the host with the reference's arithmetic and each line only
//   runs the 3 data-dependent sweeps -- again bit-identical to the reference.
// * pb_pcr_alpha_batched: parallel cyclic reduction, one line per workgroup held in LDS
//   (log2(n) steps); results agree with Thomas to rounding, not bit for bit.
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "pb_internal.hpp"

namespace pb {

// ---------------------------------------------------------------------------------------------
// General batched Thomas / periodic Thomas (src/tridsol.f90:22-115)
// ---------------------------------------------------------------------------------------------
struct LineMap {
  int64_t m1, s1, s2, es;  // base(l) = (l % m1) * s1 + (l / m1) * s2; element e at base + e*es
  __device__ __forceinline__ int64_t base(int64_t l) const { return (l % m1) * s1 + (l / m1) * s2; }
};

// The recurrences carry b'[i-1], c[i-1], d'[i-1] (and u'[i-1]) in registers, so each sweep
// touches every array once: tdma 4R+2W forward, 3R+1W backward (80 B/DoF of traffic for 48
// algorithmic); tdma_periodic 4R+3W forward, 4R+2W backward, 2R+1W correction (128 B/DoF for
// 40). The operations and their order are the reference's, element by element.
__global__ __launch_bounds__(64) void tdma_kernel(int64_t n, int64_t nb, LineMap lm,
                                                  const double* __restrict__ a,
                                                  double* __restrict__ b,
                                                  const double* __restrict__ c,
                                                  double* __restrict__ d) {
  const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= nb) return;
  const int64_t o = lm.base(l), es = lm.es;
  // fwd_sweep :90-94
  double bp = b[o], cp = c[o], dp = d[o];
  for (int64_t i = 1; i < n; ++i) {
    const int64_t e = o + i * es;
    const double w = a[e] / bp;
    bp = b[e] - w * cp;
    dp = d[e] - w * dp;
    cp = c[e];
    b[e] = bp;
    d[e] = dp;
  }
  // bwd_sweep :110-113
  double xn = dp / bp;
  d[o + (n - 1) * es] = xn;
  for (int64_t i = n - 2; i >= 0; --i) {
    const int64_t e = o + i * es;
    xn = (d[e] - c[e] * xn) / b[e];
    d[e] = xn;
  }
}

// fwd_sweep (:76-96) or bwd_sweep (:98-115) alone (the reference exports both for its tests)
__global__ __launch_bounds__(64) void tdma_sweep_kernel(int64_t n, int64_t nb, LineMap lm,
                                                        const double* __restrict__ a,
                                                        double* __restrict__ b,
                                                        const double* __restrict__ c,
                                                        double* __restrict__ d, int which) {
  const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= nb) return;
  const int64_t o = lm.base(l), es = lm.es;
  if (which == 1) {
    double bp = b[o], cp = c[o], dp = d[o];
    for (int64_t i = 1; i < n; ++i) {
      const int64_t e = o + i * es;
      const double w = a[e] / bp;
      bp = b[e] - w * cp;
      dp = d[e] - w * dp;
      cp = c[e];
      b[e] = bp;
      d[e] = dp;
    }
    return;
  }
  double xn = d[o + (n - 1) * es] / b[o + (n - 1) * es];
  d[o + (n - 1) * es] = xn;
  for (int64_t i = n - 2; i >= 0; --i) {
    const int64_t e = o + i * es;
    xn = (d[e] - c[e] * xn) / b[e];
    d[e] = xn;
  }
}

// tdma_periodic :34-74; the two auxiliary Thomas solves share one forward elimination of bmod
// (the reference recomputes bmod identically for the second solve). scratch: 2*n per line,
// element i of line l at [i*nb + l] (coalesced across lines).
__global__ __launch_bounds__(64) void tdma_periodic_kernel(int64_t n, int64_t nb, LineMap lm,
                                                           const double* __restrict__ a,
                                                           const double* __restrict__ b,
                                                           const double* __restrict__ c,
                                                           double* __restrict__ d,
                                                           double* __restrict__ scratch) {
  const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= nb) return;
  const int64_t o = lm.base(l), es = lm.es;
  double* bm = scratch + l;  // modified diagonal
  double* u = scratch + n * nb + l;
  const double a0 = a[o], cn = c[o + (n - 1) * es];
  const double gamma = -b[o];
  // bb(1) = b(1) - gamma, bb(n) = b(n) - c(n) a(1) / gamma; u = [gamma, 0, ..., 0, c(n)]
  double bp = b[o] - gamma;
  if (n == 1) bp = bp - cn * a0 / gamma;
  double up = n == 1 ? cn : gamma;
  double dp = d[o], cp = c[o];
  bm[0] = bp;
  u[0] = up;
  for (int64_t i = 1; i < n; ++i) {
    const int64_t e = o + i * es;
    double bi = b[e];
    if (i == n - 1) bi = bi - cn * a0 / gamma;
    const double ui = i == n - 1 ? cn : 0.0;
    const double w = a[e] / bp;
    bp = bi - w * cp;
    dp = d[e] - w * dp;
    up = ui - w * up;
    cp = c[e];
    bm[i * nb] = bp;
    d[e] = dp;
    u[i * nb] = up;
  }
  double yn = dp / bp, zn = up / bp;
  const double ylast = yn, zlast = zn;
  d[o + (n - 1) * es] = yn;
  u[(n - 1) * nb] = zn;
  for (int64_t i = n - 2; i >= 0; --i) {
    const int64_t e = o + i * es;
    const double ci = c[e], bi = bm[i * nb];
    yn = (d[e] - ci * yn) / bi;
    zn = (u[i * nb] - ci * zn) / bi;
    d[e] = yn;
    u[i * nb] = zn;
  }
  const double num = yn + (a0 / gamma) * ylast;
  const double den = 1.0 + (zn + (a0 / gamma) * zlast);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t e = o + i * es;
    d[e] = d[e] - (u[i * nb] * num) / den;
  }
}

// ---------------------------------------------------------------------------------------------
// Constant-coefficient (alpha, 1, alpha) periodic factorisation, computed on the host with the
// reference arithmetic of tdma_periodic (:51-70) applied to ld = ud = alpha, d = 1.
// W[i] = a_i / bm'_{i-1}, BM[i] = bm'_i, U[i] = Sherman-Morrison vector solution.
// ---------------------------------------------------------------------------------------------
struct AlphaFactor {
  double* dev = nullptr;  // [W | BM | U], 3n doubles
  double alpha, gamma, a0g, den;
};

static std::mutex g_fac_mu;
static std::map<std::pair<int, std::pair<int64_t, double>>, AlphaFactor> g_fac;

static int alpha_factor(pb_ctx* ctx, int64_t n, double alpha, AlphaFactor* out) {
  std::lock_guard<std::mutex> lk(g_fac_mu);
  auto key = std::make_pair(ctx->device, std::make_pair(n, alpha));
  auto it = g_fac.find(key);
  if (it != g_fac.end()) {
    *out = it->second;
    return PB_OK;
  }
  std::vector<double> W(n, 0.0), BM(n, 1.0), U(n, 0.0);
  const double a0 = alpha, cn = alpha;
  const double gamma = -1.0;  // -b(1), b = 1
  BM[0] = BM[0] - gamma;
  BM[n - 1] = BM[n - 1] - cn * a0 / gamma;
  U[0] = gamma;
  U[n - 1] = cn;
  for (int64_t i = 1; i < n; ++i) {
    W[i] = alpha / BM[i - 1];
    BM[i] = BM[i] - W[i] * alpha;
    U[i] = U[i] - W[i] * U[i - 1];
  }
  U[n - 1] = U[n - 1] / BM[n - 1];
  for (int64_t i = n - 2; i >= 0; --i) U[i] = (U[i] - alpha * U[i + 1]) / BM[i];
  AlphaFactor f;
  f.alpha = alpha;
  f.gamma = gamma;
  f.a0g = a0 / gamma;
  f.den = 1.0 + (U[0] + f.a0g * U[n - 1]);
  std::vector<double> all(3 * n);
  memcpy(all.data(), W.data(), n * sizeof(double));
  memcpy(all.data() + n, BM.data(), n * sizeof(double));
  memcpy(all.data() + 2 * n, U.data(), n * sizeof(double));
  PB_HIP(hipMalloc(&f.dev, 3 * n * sizeof(double)));
  // stream-ordered upload, completed before any kernel can use the cached factors (a blocking
  // hipMemcpy from pageable memory may return before the DMA lands)
  PB_HIP(hipMemcpyAsync(f.dev, all.data(), 3 * n * sizeof(double), hipMemcpyHostToDevice,
                        ctx->stream));
  PB_SYNC(ctx, "compact");
  g_fac[key] = f;
  *out = f;
  return PB_OK;
}

// Scheme parameters (src/compact_schemes.f90:188-190, :303-305)
struct Scheme {
  double a, b, alpha, sign;
};
static Scheme scheme(int kind, double dx) {
  if (kind == 0) return Scheme{63.0 / 62.0 / dx, 17.0 / 62.0 / (3.0 * dx), 9.0 / 62.0, -1.0};
  return Scheme{0.75, 1.0 / 20.0, 3.0 / 10.0, +1.0};
}

// One compact 1-D operator per line: RHS (eval_1d_rhs :332-372, periodic formula) fused into
// the forward sweep, then backward sweep and Sherman-Morrison correction. `in2` (optional) is
// added to the input first (div's Z step, :249), `addend` (optional) to the output (:250).
__global__ __launch_bounds__(64) void compact_line_kernel(
    int64_t n, int64_t nb, LineMap lm, Scheme sc, int shift, const double* __restrict__ in,
    const double* __restrict__ in2, const double* __restrict__ addend, double* out,
    const double* __restrict__ fac, double a0g, double den) {
  const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= nb) return;
  const int64_t o = lm.base(l), es = lm.es;
  const double* W = fac;
  const double* BM = fac + n;
  const double* U = fac + 2 * n;
  auto F = [&](int64_t i) -> double {  // periodic input
    i %= n;
    if (i < 0) i += n;
    double v = in[o + i * es];
    if (in2) v = v + in2[o + i * es];
    return v;
  };
  // sliding window f(i+shift-2 .. i+shift+1): one input load per point
  double fm2 = F(shift - 2), fm1 = F(shift - 1), f0 = F(shift), f1 = F(shift + 1);
  auto rhs = [&]() -> double {
    return sc.a * (f0 + sc.sign * fm1) + sc.b * (f1 + sc.sign * fm2);
  };
  auto advance = [&](int64_t i) {  // window of point i -> window of point i+1
    fm2 = fm1;
    fm1 = f0;
    f0 = f1;
    int64_t k = i + shift + 2;  // <= n + 1 (i <= n - 2)
    if (k >= n) k -= n;
    f1 = in[o + k * es];
    if (in2) f1 = f1 + in2[o + k * es];
  };
  // forward sweep: d[i] = rhs[i] - W[i] * d[i-1]
  double prev = rhs();
  out[o] = prev;
  for (int64_t i = 1; i < n; ++i) {
    advance(i - 1);
    const double di = rhs() - W[i] * prev;
    out[o + i * es] = di;
    prev = di;
  }
  // backward sweep (d[n-1] is still in a register)
  double next = prev / BM[n - 1];
  out[o + (n - 1) * es] = next;
  const double dlast = next;
  for (int64_t i = n - 2; i >= 0; --i) {
    const double di = (out[o + i * es] - sc.alpha * next) / BM[i];
    out[o + i * es] = di;
    next = di;
  }
  // Sherman-Morrison correction (:69-70), then optional addend
  const double num = next + a0g * dlast;
  for (int64_t i = 0; i < n; ++i) {
    double v = out[o + i * es] - (U[i] * num) / den;
    if (addend) v = v + addend[o + i * es];
    out[o + i * es] = v;
  }
}

static int launch_line(pb_ctx* ctx, int kind, int stagger, double dx, int64_t n, int64_t nb,
                       LineMap lm, const double* in, const double* in2, const double* addend,
                       double* out) {
  Scheme sc = scheme(kind, dx);
  AlphaFactor f;
  PB_TRY(alpha_factor(ctx, n, sc.alpha, &f));
  const int shift = stagger == -1 ? 0 : 1;
  const int64_t blocks = (nb + 63) / 64;
  hipLaunchKernelGGL(compact_line_kernel, dim3((unsigned)blocks), dim3(64), 0, ctx->stream, n, nb,
                     lm, sc, shift, in, in2, addend, out, (const double*)f.dev, f.a0g, f.den);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

// direction d of an n0*n1*n2 box (the owned slab: n2 = nzl; or a y-slab with complete z-lines)
static LineMap dir_map(const int64_t b[3], int d) {
  const int64_t nx = b[0], ny = b[1];
  if (d == 0) return LineMap{ny, nx, nx * ny, 1};
  if (d == 1) return LineMap{nx, 1, nx * ny, nx};
  return LineMap{nx * ny, 1, 0, nx * ny};
}

enum { K_GRAD = 0, K_INTERP = 1 };

static int line_box(pb_ctx* ctx, const int64_t b[3], int d, int kind, int stagger, double dx,
                    const double* in, double* out, const double* in2 = nullptr,
                    const double* addend = nullptr) {
  return launch_line(ctx, kind, stagger, dx, b[d], b[0] * b[1] * b[2] / b[d], dir_map(b, d), in,
                     in2, addend, out);
}

// x and y lines are complete in every z-slab; z lines too on one rank
static int line3(pb_grid* g, int d, int kind, int stagger, double dx, const double* in,
                 double* out, const double* in2 = nullptr, const double* addend = nullptr) {
  const int64_t b[3] = {g->n[0], g->n[1], g->nzl};
  return line_box(g->ctx, b, d, kind, stagger, dx, in, out, in2, addend);
}

// Z steps on a split grid run on y-slabs (complete z-lines; pb_compact_dist.hip transposes):
// same line kernels, same per-line operation order => bit-identical to one rank. Scratch for
// them: 4 y-slab fields + the transpose aux space.
static int64_t zsplit_len(const pb_grid* g) {
  return grid_split(g) ? 4 * yslab_len(g) + yslab_aux_len(g) : 0;
}

struct ZSplit {
  YSlabPlan p;
  double* y[4];
  int64_t b[3];
};
static int zsplit_begin(pb_grid* g, double* ws, ZSplit* z) {
  const int64_t L = yslab_len(g);
  for (int i = 0; i < 4; ++i) z->y[i] = ws + i * L;
  PB_TRY(yslab_begin(g, ws + 4 * L, &z->p));
  z->b[0] = g->n[0];
  z->b[1] = z->p.ny_me;
  z->b[2] = g->n[2];
  return PB_OK;
}

// src/compact_schemes.f90:42-88 grad; scratch 5N (+ zsplit_len)
static int grad3(pb_grid* g, const double dx[3], const double* f, double* df1, double* df2,
                 double* df3, double* ws) {
  const int64_t N = g->nlocal;
  double *dff1 = ws, *dff3 = ws + N, *dfe1 = ws + 2 * N, *dfe2 = ws + 3 * N, *dfe3 = ws + 4 * N;
  if (!grid_split(g)) {
    PB_TRY(line3(g, 2, K_INTERP, -1, 0.0, f, dff1));    // :61
    PB_TRY(line3(g, 2, K_GRAD, -1, dx[2], f, dff3));    // :63  (dff2 = dff1, :62)
  } else {
    ZSplit z;
    PB_TRY(zsplit_begin(g, ws + 5 * N, &z));
    PB_TRY(yslab_to(g, z.p, f, z.y[0]));
    PB_TRY(line_box(g->ctx, z.b, 2, K_INTERP, -1, 0.0, z.y[0], z.y[1]));
    PB_TRY(line_box(g->ctx, z.b, 2, K_GRAD, -1, dx[2], z.y[0], z.y[2]));
    PB_TRY(yslab_from(g, z.p, z.y[1], dff1));
    PB_TRY(yslab_from(g, z.p, z.y[2], dff3));
  }
  PB_TRY(line3(g, 1, K_INTERP, -1, 0.0, dff1, dfe1));   // :71
  PB_TRY(line3(g, 1, K_GRAD, -1, dx[1], dff1, dfe2));   // :72
  PB_TRY(line3(g, 1, K_INTERP, -1, 0.0, dff3, dfe3));   // :73
  PB_TRY(line3(g, 0, K_GRAD, -1, dx[0], dfe1, df1));    // :81
  PB_TRY(line3(g, 0, K_INTERP, -1, 0.0, dfe2, df2));    // :82
  PB_TRY(line3(g, 0, K_INTERP, -1, 0.0, dfe3, df3));    // :83
  return PB_OK;
}

// src/compact_schemes.f90:207-257 div; scratch 6N (+ zsplit_len)
static int div3(pb_grid* g, const double dx[3], const double* f1, const double* f2,
                const double* f3, double* out, double* ws) {
  const int64_t N = g->nlocal;
  double *dfe1 = ws, *dfe2 = ws + N, *dfe3 = ws + 2 * N;
  double *dff1 = ws + 3 * N, *dff2 = ws + 4 * N, *dff3 = ws + 5 * N;
  PB_TRY(line3(g, 0, K_GRAD, +1, dx[0], f1, dfe1));     // :227
  PB_TRY(line3(g, 0, K_INTERP, +1, 0.0, f2, dfe2));     // :228
  PB_TRY(line3(g, 0, K_INTERP, +1, 0.0, f3, dfe3));     // :229
  PB_TRY(line3(g, 1, K_INTERP, +1, 0.0, dfe1, dff1));   // :237
  PB_TRY(line3(g, 1, K_GRAD, +1, dx[1], dfe2, dff2));   // :238
  PB_TRY(line3(g, 1, K_INTERP, +1, 0.0, dfe3, dff3));   // :239
  if (!grid_split(g)) {
    double* dfc = dfe1;
    PB_TRY(line3(g, 2, K_INTERP, +1, 0.0, dff1, dfc, dff2));          // :248 interp(dff1 + dff2)
    PB_TRY(line3(g, 2, K_GRAD, +1, dx[2], dff3, out, nullptr, dfc));  // :249-250
    return PB_OK;
  }
  ZSplit z;
  PB_TRY(zsplit_begin(g, ws + 6 * N, &z));
  PB_TRY(yslab_to(g, z.p, dff1, z.y[0]));
  PB_TRY(yslab_to(g, z.p, dff2, z.y[1]));
  PB_TRY(yslab_to(g, z.p, dff3, z.y[2]));
  PB_TRY(line_box(g->ctx, z.b, 2, K_INTERP, +1, 0.0, z.y[0], z.y[3], z.y[1]));
  PB_TRY(line_box(g->ctx, z.b, 2, K_GRAD, +1, dx[2], z.y[2], z.y[0], nullptr, z.y[3]));
  return yslab_from(g, z.p, z.y[0], out);
}

int64_t compact_work_len(const pb_grid* g) { return 9 * g->nlocal + zsplit_len(g); }

// src/compact_schemes.f90:17-37 lapl = div(grad f); work: 9N (+ zsplit_len)
int compact_lapl(pb_grid* g, const double dx[3], const double* f, double* out, double* work) {
  ScopedTimer tm(g->ctx, "compact_lapl");
  const int64_t N = g->nlocal;
  double *df1 = work, *df2 = work + N, *df3 = work + 2 * N;
  PB_TRY(grad3(g, dx, f, df1, df2, df3, work + 3 * N));
  PB_TRY(div3(g, dx, df1, df2, df3, out, work + 3 * N));
  return PB_OK;
}

// ---------------------------------------------------------------------------------------------
// PCR for (alpha, 1, alpha) periodic lines: one line per workgroup, line in LDS
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pcr_alpha_kernel(int64_t n, LineMap lm, double alpha,
                                                        double* d) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* A = sm;          // sub
  double* C = sm + n;      // super
  double* D = sm + 2 * n;  // rhs
  double* B = sm + 3 * n;  // diag
  const int64_t o = lm.base(blockIdx.x), es = lm.es;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    A[i] = alpha;
    C[i] = alpha;
    B[i] = 1.0;
    D[i] = d[o + i * es];
  }
  __syncthreads();
  // periodic PCR: each step eliminates the couplings at distance s, doubling it
  for (int64_t s = 1; s < n; s <<= 1) {
    double na[16], nb_[16], nc[16], nd[16];
    int cnt = 0;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x, ++cnt) {
      const int64_t im = (i - s % n + n) % n, ip = (i + s) % n;
      const double k1 = A[i] / B[im], k2 = C[i] / B[ip];
      na[cnt] = -A[im] * k1;
      nc[cnt] = -C[ip] * k2;
      nb_[cnt] = B[i] - C[im] * k1 - A[ip] * k2;
      nd[cnt] = D[i] - D[im] * k1 - D[ip] * k2;
    }
    __syncthreads();
    cnt = 0;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x, ++cnt) {
      A[i] = na[cnt];
      C[i] = nc[cnt];
      B[i] = nb_[cnt];
      D[i] = nd[cnt];
    }
    __syncthreads();
  }
  // after log2(n) steps (n a power of two) the remaining couplings are at distance n, i.e. on the
  // row itself: (B_i + A_i + C_i) x_i = D_i
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) d[o + i * es] = D[i] / (B[i] + A[i] + C[i]);
}

}  // namespace pb

using namespace pb;

extern "C" {

int pb_tdma_batched(pb_ctx* ctx, int64_t n, int64_t nbatch, int64_t line_stride,
                    int64_t elem_stride, const double* a, double* b, const double* c, double* d,
                    int periodic) {
  PB_CHECK_ARG(ctx && a && b && c && d, "bad tdma args");
  PB_CHECK_ARG(n >= 2 && nbatch >= 1, "bad tdma sizes");
  LineMap lm{nbatch, line_stride, 0, elem_stride};
  const int64_t blocks = (nbatch + 63) / 64;
  double* scratch = nullptr;
  if (periodic) PB_TRY(ctx_scratch(ctx, (size_t)(2 * n * nbatch), &scratch));
  ScopedTimer tm(ctx, "tdma");
  if (!periodic) {
    hipLaunchKernelGGL(tdma_kernel, dim3((unsigned)blocks), dim3(64), 0, ctx->stream, n, nbatch, lm,
                       a, b, c, d);
    PB_HIP(hipGetLastError());
    return PB_OK;
  }
  hipLaunchKernelGGL(tdma_periodic_kernel, dim3((unsigned)blocks), dim3(64), 0, ctx->stream, n,
                     nbatch, lm, a, (const double*)b, c, d, scratch);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

int pb_tdma_sweeps_batched(pb_ctx* ctx, int64_t n, int64_t nbatch, int64_t line_stride,
                           int64_t elem_stride, const double* a, double* b, const double* c,
                           double* d, int which) {
  PB_CHECK_ARG(ctx && b && c && d && (which == 2 || a), "bad sweep args");
  PB_CHECK_ARG(which == 1 || which == 2, "which: 1 = fwd_sweep, 2 = bwd_sweep");
  PB_CHECK_ARG(n >= 2 && nbatch >= 1, "bad sweep sizes");
  LineMap lm{nbatch, line_stride, 0, elem_stride};
  ScopedTimer tm(ctx, "tdma");
  hipLaunchKernelGGL(tdma_sweep_kernel, dim3((unsigned)((nbatch + 63) / 64)), dim3(64), 0,
                     ctx->stream, n, nbatch, lm, a, b, c, d, which);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

int pb_pcr_alpha_batched(pb_ctx* ctx, int64_t n, int64_t nbatch, int64_t line_stride,
                         int64_t elem_stride, double alpha, double* d) {
  PB_CHECK_ARG(ctx && d, "bad pcr args");
  PB_CHECK_ARG(n >= 3 && n <= 4096 && nbatch >= 1, "pcr: 3 <= n <= 4096");
  ScopedTimer tm(ctx, "pcr");
  // register line solves where the extent allows; pcr_lines = 0 keeps the PCR kernel (tests)
  if (tune("pcr_lines", 1)) {  // register-resident factorised solve with cross-lane scans (n = 64*C)
    const int rc = lines_solve_batched(ctx, n, nbatch, line_stride, elem_stride, alpha, d);
    if (rc != PB_ERR_UNSUPPORTED) return rc;
  }
  PB_CHECK_ARG((n & (n - 1)) == 0, "pcr: n must be a power of two (or 64*{1,2,3,4,6,8,12,16})");
  LineMap lm{nbatch, line_stride, 0, elem_stride};
  hipLaunchKernelGGL(pcr_alpha_kernel, dim3((unsigned)nbatch), dim3(256), 4 * n * sizeof(double),
                     ctx->stream, n, lm, alpha, d);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

int pb_compact_1d_batched(pb_ctx* ctx, int kind, int stagger, double dx, int64_t n,
                          int64_t nbatch, int64_t line_stride, int64_t elem_stride,
                          const double* f, double* out) {
  PB_CHECK_ARG(ctx && f && out && f != out, "bad compact_1d args");
  PB_CHECK_ARG(kind == 0 || kind == 1, "kind: 0 = derivative, 1 = interpolation");
  PB_CHECK_ARG(stagger == -1 || stagger == 1, "stagger must be -1 or +1");
  PB_CHECK_ARG(n >= 3 && nbatch >= 1, "compact_1d: n >= 3");
  LineMap lm{nbatch, line_stride, 0, elem_stride};
  AlphaFactor fac;
  PB_TRY(alpha_factor(ctx, n, scheme(kind == 0 ? K_GRAD : K_INTERP, dx).alpha, &fac));  // warm cache
  ScopedTimer tm(ctx, "compact_1d");
  return launch_line(ctx, kind == 0 ? K_GRAD : K_INTERP, stagger, dx, n, nbatch, lm, f, nullptr,
                     nullptr, out);
}

int pb_compact_grad(pb_grid* g, const double dx[3], const pb_vec* f, pb_vec* const df[3]) {
  PB_CHECK_ARG(g && dx && f && df && df[0] && df[1] && df[2], "bad grad args");
  double* ws = nullptr;
  PB_TRY(ctx_scratch(g->ctx, (size_t)(5 * g->nlocal + zsplit_len(g)), &ws));
  int rc = grad3(g, dx, f->d, df[0]->d, df[1]->d, df[2]->d, ws);
  return rc;
}

int pb_compact_div(pb_grid* g, const double dx[3], const pb_vec* const f[3], pb_vec* df) {
  PB_CHECK_ARG(g && dx && f && f[0] && f[1] && f[2] && df, "bad div args");
  double* ws = nullptr;
  PB_TRY(ctx_scratch(g->ctx, (size_t)(6 * g->nlocal + zsplit_len(g)), &ws));
  int rc = div3(g, dx, f[0]->d, f[1]->d, f[2]->d, df->d, ws);
  return rc;
}

int pb_compact_interp(pb_grid* g, int stagger, const pb_vec* f, pb_vec* fi) {
  PB_CHECK_ARG(g && f && fi && f != fi, "bad interp args");
  PB_CHECK_ARG(stagger == -1 || stagger == 1, "stagger must be -1 or +1");
  double* ws = nullptr;
  const int64_t N = g->nlocal;
  PB_TRY(ctx_scratch(g->ctx, (size_t)(2 * N + zsplit_len(g)), &ws));
  int rc = PB_OK;
  if (!grid_split(g)) {
    rc = line3(g, 2, K_INTERP, stagger, 0.0, f->d, ws);             // :238
  } else {  // the Z step on y-slabs
    ZSplit z;
    rc = zsplit_begin(g, ws + 2 * N, &z);
    if (!rc) rc = yslab_to(g, z.p, f->d, z.y[0]);
    if (!rc) rc = line_box(g->ctx, z.b, 2, K_INTERP, stagger, 0.0, z.y[0], z.y[1]);
    if (!rc) rc = yslab_from(g, z.p, z.y[1], ws);
  }
  if (!rc) rc = line3(g, 1, K_INTERP, stagger, 0.0, ws, ws + N);    // :246
  if (!rc) rc = line3(g, 0, K_INTERP, stagger, 0.0, ws + N, fi->d); // :254
  return rc;
}

int pb_compact_lapl(pb_grid* g, const double dx[3], const pb_vec* f, pb_vec* out) {
  PB_CHECK_ARG(g && dx && f && out && f != out, "bad lapl args");
  double* ws = nullptr;
  PB_TRY(ctx_scratch(g->ctx, (size_t)compact_work_len(g), &ws));
  int rc = compact_lapl(g, dx, f->d, out->d, ws);
  return rc;
}

// ---------------------------------------------------------------------------------------------
// Host-array forms: the reference's module procedures (src/tridsol.f90:16-18,
// src/compact_schemes.f90:9-13) take plain process-local Fortran arrays. These stage them through
// device memory, run the same kernels and copy back (synchronous; convenience, not the fast path).
// ---------------------------------------------------------------------------------------------
namespace {
struct DevBuf {
  double* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};
int stage_in(pb_ctx* ctx, DevBuf& b, size_t n, const double* host) {
  if (hipMalloc(&b.p, std::max<size_t>(n, 1) * sizeof(double)) != hipSuccess)
    return set_error(PB_ERR_ALLOC, "host-array staging of %zu doubles: out of device memory", n);
  if (host)
    PB_HIP(hipMemcpyAsync(b.p, host, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  return PB_OK;
}
int stage_out(pb_ctx* ctx, const DevBuf& b, size_t n, double* host) {
  PB_HIP(hipMemcpyAsync(host, b.p, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  PB_SYNC(ctx, "host-array copy-out");
  return PB_OK;
}
int64_t extent(int64_t n, int64_t nbatch, int64_t ls, int64_t es) {
  return (nbatch - 1) * ls + (n - 1) * es + 1;
}
// a process-local grid of the array's shape (never split, whatever the context)
struct LocalGrid {
  pb_grid* g = nullptr;
  ~LocalGrid() {
    if (g) pb_grid_destroy(g);
  }
};
int local_grid(pb_ctx* ctx, const int64_t n[3], LocalGrid& lg) {
  for (int d = 0; d < 3; ++d) PB_CHECK_ARG(n[d] >= 3, "compact operators need n >= 3");
  PB_TRY(grid_create_part(ctx, n, nullptr, 0, n[2], &lg.g));
  lg.g->whole = true;
  return PB_OK;
}
}  // namespace

int pb_tdma_batched_host(pb_ctx* ctx, int64_t n, int64_t nbatch, int64_t line_stride,
                         int64_t elem_stride, const double* a, double* b, const double* c,
                         double* d, int periodic) {
  PB_CHECK_ARG(ctx && a && b && c && d && line_stride >= 0 && elem_stride >= 1, "bad tdma args");
  PB_CHECK_ARG(n >= 2 && nbatch >= 1, "bad tdma sizes");
  const size_t E = (size_t)extent(n, nbatch, line_stride, elem_stride);
  DevBuf da, db, dc, dd;
  PB_TRY(stage_in(ctx, da, E, a));
  PB_TRY(stage_in(ctx, db, E, b));
  PB_TRY(stage_in(ctx, dc, E, c));
  PB_TRY(stage_in(ctx, dd, E, d));
  PB_TRY(pb_tdma_batched(ctx, n, nbatch, line_stride, elem_stride, da.p, db.p, dc.p, dd.p,
                         periodic));
  if (!periodic) PB_TRY(stage_out(ctx, db, E, b));  // tdma overwrites b (src/tridsol.f90:22-32)
  return stage_out(ctx, dd, E, d);
}

int pb_tdma_sweeps_batched_host(pb_ctx* ctx, int64_t n, int64_t nbatch, int64_t line_stride,
                                int64_t elem_stride, const double* a, double* b, const double* c,
                                double* d, int which) {
  PB_CHECK_ARG(ctx && b && c && d && (which == 2 || a) && line_stride >= 0 && elem_stride >= 1,
               "bad sweep args");
  PB_CHECK_ARG(n >= 2 && nbatch >= 1, "bad sweep sizes");
  const size_t E = (size_t)extent(n, nbatch, line_stride, elem_stride);
  DevBuf da, db, dc, dd;
  if (which == 1) PB_TRY(stage_in(ctx, da, E, a));
  PB_TRY(stage_in(ctx, db, E, b));
  PB_TRY(stage_in(ctx, dc, E, c));
  PB_TRY(stage_in(ctx, dd, E, d));
  PB_TRY(pb_tdma_sweeps_batched(ctx, n, nbatch, line_stride, elem_stride, da.p, db.p, dc.p, dd.p,
                                which));
  if (which == 1) PB_TRY(stage_out(ctx, db, E, b));
  return stage_out(ctx, dd, E, d);
}

int pb_compact_1d_batched_host(pb_ctx* ctx, int kind, int stagger, double dx, int64_t n,
                               int64_t nbatch, int64_t line_stride, int64_t elem_stride,
                               const double* f, double* out) {
  PB_CHECK_ARG(ctx && f && out && line_stride >= 0 && elem_stride >= 1, "bad compact_1d args");
  PB_CHECK_ARG(n >= 3 && nbatch >= 1, "compact_1d: n >= 3");
  const size_t E = (size_t)extent(n, nbatch, line_stride, elem_stride);
  DevBuf df, dout;
  PB_TRY(stage_in(ctx, df, E, f));
  PB_TRY(stage_in(ctx, dout, E, out));  // untouched gaps of a strided layout keep their values
  PB_TRY(pb_compact_1d_batched(ctx, kind, stagger, dx, n, nbatch, line_stride, elem_stride, df.p,
                               dout.p));
  return stage_out(ctx, dout, E, out);
}

int pb_compact_grad_host(pb_ctx* ctx, const int64_t n[3], const double dx[3], const double* f,
                         double* df) {
  PB_CHECK_ARG(ctx && n && dx && f && df, "bad grad args");
  LocalGrid lg;
  PB_TRY(local_grid(ctx, n, lg));
  const size_t N = (size_t)lg.g->nlocal;
  DevBuf d, o, w;
  PB_TRY(stage_in(ctx, d, N, f));
  PB_TRY(stage_in(ctx, o, 3 * N, nullptr));
  PB_TRY(stage_in(ctx, w, 5 * N, nullptr));
  PB_TRY(grad3(lg.g, dx, d.p, o.p, o.p + N, o.p + 2 * N, w.p));
  return stage_out(ctx, o, 3 * N, df);  // df(nx, ny, nz, 3): component slowest
}

int pb_compact_div_host(pb_ctx* ctx, const int64_t n[3], const double dx[3], const double* f,
                        double* df) {
  PB_CHECK_ARG(ctx && n && dx && f && df, "bad div args");
  LocalGrid lg;
  PB_TRY(local_grid(ctx, n, lg));
  const size_t N = (size_t)lg.g->nlocal;
  DevBuf d, o, w;
  PB_TRY(stage_in(ctx, d, 3 * N, f));  // f(nx, ny, nz, 3)
  PB_TRY(stage_in(ctx, o, N, nullptr));
  PB_TRY(stage_in(ctx, w, 6 * N, nullptr));
  PB_TRY(div3(lg.g, dx, d.p, d.p + N, d.p + 2 * N, o.p, w.p));
  return stage_out(ctx, o, N, df);
}

int pb_compact_interp_host(pb_ctx* ctx, const int64_t n[3], int stagger, const double* f,
                           double* fi) {
  PB_CHECK_ARG(ctx && n && f && fi, "bad interp args");
  PB_CHECK_ARG(stagger == -1 || stagger == 1, "stagger must be -1 or +1");
  LocalGrid lg;
  PB_TRY(local_grid(ctx, n, lg));
  const size_t N = (size_t)lg.g->nlocal;
  DevBuf d, w;
  PB_TRY(stage_in(ctx, d, N, f));
  PB_TRY(stage_in(ctx, w, 2 * N, nullptr));
  PB_TRY(line3(lg.g, 2, K_INTERP, stagger, 0.0, d.p, w.p));          // :122-127
  PB_TRY(line3(lg.g, 1, K_INTERP, stagger, 0.0, w.p, w.p + N));      // :130-135
  PB_TRY(line3(lg.g, 0, K_INTERP, stagger, 0.0, w.p + N, d.p));      // :139-143
  return stage_out(ctx, d, N, fi);
}

int pb_compact_lapl_host(pb_ctx* ctx, const int64_t n[3], const double dx[3], const double* f,
                         double* out) {
  PB_CHECK_ARG(ctx && n && dx && f && out, "bad lapl args");
  LocalGrid lg;
  PB_TRY(local_grid(ctx, n, lg));
  const size_t N = (size_t)lg.g->nlocal;
  DevBuf d, o, w;
  PB_TRY(stage_in(ctx, d, N, f));
  PB_TRY(stage_in(ctx, o, N, nullptr));
  PB_TRY(stage_in(ctx, w, (size_t)compact_work_len(lg.g), nullptr));
  PB_TRY(compact_lapl(lg.g, dx, d.p, o.p, w.p));
  return stage_out(ctx, o, N, out);
}

}  // extern "C"
