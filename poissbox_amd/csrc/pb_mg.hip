// pb_mg.hip -- geometric multigrid V-cycle with red-black SOR smoothing, and symmetric red-black
// SOR alone, as CG preconditioners (the reference README.md:40-45 recommends
// GAMG + SOR through PETSc, which is absent here: this is the geometric, GPU-native analogue).
//
// Levels: the periodic 7-point operator rediscretised with h_l = 2^l h (star_coeffs, the
// reference's coefficients, src/coefficients.f90:22-48), cell-centred coarsening by 2 in every
// direction, trilinear prolongation P (weights 3/4, 1/4 per direction) and restriction
// R = P^T / 8 (weights 1/8, 3/8, 3/8, 1/8 per direction). V(1,1): pre-smoothing red then black,
// post-smoothing black then red, coarsest level `coarse_its` symmetric sweeps (red, black, red,
// [black, red]...), all from a zero initial guess -- the V-cycle is a symmetric operator, as CG
// needs. SOR update (PETSc PCSOR form): x = (1 - w) x + w (b - sum_nb c x_nb) / c_centre.
// Red = (i + j + k_global) even; every smoothed level has even extents, so a colour's
// neighbours all carry the other colour across the periodic wrap too.
//
// Slab decomposition: level l owns planes [k0 / 2^l, (k0 + nzl) / 2^l); coarsening stops before
// any rank's slab would become odd (mg_plan_levels is a function of the global grid and the rank
// count only, so every rank builds the same hierarchy). Halo planes are exchanged before every
// half-sweep, residual, restriction and prolongation on N > 1 ranks; one rank reads the periodic
// wrap planes in place.
//
// The arithmetic order of every kernel is restated in oracle/pb_oracle.c (pbo_mg_apply), which
// the tests compare bit for bit.
#include <algorithm>
#include <cmath>
#include <vector>

#include "pb_internal.hpp"

namespace pb {

struct MgGeo {
  int nx, ny, nzl;
  int64_t plane, nlocal, k0;
};

struct MgLevel {
  int64_t n[3];
  double h[3];
  Star s;
  pb_grid* g = nullptr;  // level grid (level 0: the caller's grid)
  bool own = false;
  double* x = nullptr;    // correction (level 0: the PC output z)
  double* b = nullptr;    // right-hand side (level 0: the PC input r)
  double* res = nullptr;  // residual scratch
  MgGeo geo() const {
    return MgGeo{(int)g->n[0], (int)g->n[1], (int)g->nzl, g->plane, g->nlocal, g->k0};
  }
};

struct Mg {
  pb_ctx* ctx = nullptr;
  std::vector<MgLevel> lv;
  double omega = 1.0;
  int coarse_its = 1;
  double* mem = nullptr;
};

// ---------------------------------------------------------------------------------------------
// kernels (grid-stride over the owned points of one level; i fastest)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void mg_ijk(const MgGeo& G, int64_t idx, int& i, int& j, int& k) {
  k = (int)(idx / G.plane);
  const int rem = (int)(idx - (int64_t)k * G.plane);
  j = rem / G.nx;
  i = rem - j * G.nx;
}

__device__ __forceinline__ int wrapm(int v, int n) { return v < 0 ? v + n : (v >= n ? v - n : v); }

// one red-black SOR half-sweep over colour `color`; zero_init: x starts at 0 (the other colour is
// zeroed, the neighbour sum of this colour is exactly 0)
__global__ __launch_bounds__(256) void mg_smooth_kernel(MgGeo G, double* x,
                                                        const double* __restrict__ b,
                                                        const double* lo, const double* hi, Star s,
                                                        double omega, int color, int zero_init) {
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < G.nlocal;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int i, j, k;
    mg_ijk(G, idx, i, j, k);
    const int col = (int)((i + j + G.k0 + k) & 1);
    if (col != color) {
      if (zero_init) x[idx] = 0.0;
      continue;
    }
    double nb = 0.0, xo = 0.0;
    if (!zero_init) {
      const int64_t row = idx - i;
      const double zm = k > 0 ? x[idx - G.plane] : lo[idx];
      const double zp = k < G.nzl - 1 ? x[idx + G.plane] : hi[idx - (int64_t)k * G.plane];
      const double ym = x[idx + (int64_t)(wrapm(j - 1, G.ny) - j) * G.nx];
      const double yp = x[idx + (int64_t)(wrapm(j + 1, G.ny) - j) * G.nx];
      const double xm = x[row + wrapm(i - 1, G.nx)];
      const double xp = x[row + wrapm(i + 1, G.nx)];
      nb = s.cz * zm;
      nb = nb + s.cy * ym;
      nb = nb + s.cx * xm;
      nb = nb + s.cx * xp;
      nb = nb + s.cy * yp;
      nb = nb + s.cz * zp;
      xo = x[idx];
    }
    const double t = (b[idx] - nb) / s.cc;
    x[idx] = (1.0 - omega) * xo + omega * t;
  }
}

// res = b - A x (7-point, the reference operator's summation order)
__global__ __launch_bounds__(256) void mg_residual_kernel(MgGeo G, const double* __restrict__ x,
                                                          const double* __restrict__ b,
                                                          const double* __restrict__ lo,
                                                          const double* __restrict__ hi, Star s,
                                                          double* __restrict__ res) {
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < G.nlocal;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int i, j, k;
    mg_ijk(G, idx, i, j, k);
    const int64_t row = idx - i;
    const double zm = k > 0 ? x[idx - G.plane] : lo[idx];
    const double zp = k < G.nzl - 1 ? x[idx + G.plane] : hi[idx - (int64_t)k * G.plane];
    const double ym = x[idx + (int64_t)(wrapm(j - 1, G.ny) - j) * G.nx];
    const double yp = x[idx + (int64_t)(wrapm(j + 1, G.ny) - j) * G.nx];
    const double xm = x[row + wrapm(i - 1, G.nx)];
    const double xp = x[row + wrapm(i + 1, G.nx)];
    double ax = s.cz * zm;
    ax = ax + s.cy * ym;
    ax = ax + s.cx * xm;
    ax = ax + s.cc * x[idx];
    ax = ax + s.cx * xp;
    ax = ax + s.cy * yp;
    ax = ax + s.cz * zp;
    res[idx] = b[idx] - ax;
  }
}

// b_c = R res_f, R = P^T / 8: 4 x 4 x 4 fine cells (2I-1 .. 2I+2 per direction)
__global__ __launch_bounds__(256) void mg_restrict_kernel(MgGeo F, const double* __restrict__ rf,
                                                          const double* __restrict__ lo,
                                                          const double* __restrict__ hi, MgGeo Cg,
                                                          double* __restrict__ bc) {
  const double w[4] = {0.125, 0.375, 0.375, 0.125};
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < Cg.nlocal;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int I, J, K;
    mg_ijk(Cg, idx, I, J, K);
    double sz = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int kf = 2 * K - 1 + c;
      const double* pl = kf < 0 ? lo : (kf >= F.nzl ? hi : rf + (int64_t)kf * F.plane);
      double sy = 0.0;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        const double* row = pl + (int64_t)wrapm(2 * J - 1 + bb, F.ny) * F.nx;
        double sx = 0.0;
#pragma unroll
        for (int a = 0; a < 4; ++a) sx = sx + w[a] * row[wrapm(2 * I - 1 + a, F.nx)];
        sy = sy + w[bb] * sx;
      }
      sz = sz + w[c] * sy;
    }
    bc[idx] = sz;
  }
}

// x_f += P x_c (trilinear, cell-centred: near parent 3/4, far parent 1/4 per direction)
__global__ __launch_bounds__(256) void mg_prolong_kernel(MgGeo F, double* __restrict__ xf, MgGeo Cg,
                                                         const double* __restrict__ xc,
                                                         const double* __restrict__ lo,
                                                         const double* __restrict__ hi) {
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < F.nlocal;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int i, j, k;
    mg_ijk(F, idx, i, j, k);
    const int I = i >> 1, J = j >> 1, K = k >> 1;
    const int fI = wrapm((i & 1) ? I + 1 : I - 1, Cg.nx);
    const int fJ = wrapm((j & 1) ? J + 1 : J - 1, Cg.ny);
    const int fK = (k & 1) ? K + 1 : K - 1;
    const double* pn = xc + (int64_t)K * Cg.plane;
    const double* pf = fK < 0 ? lo : (fK >= Cg.nzl ? hi : xc + (int64_t)fK * Cg.plane);
    const int64_t rn = (int64_t)J * Cg.nx, rf = (int64_t)fJ * Cg.nx;
    const double vn = 0.75 * (0.75 * pn[rn + I] + 0.25 * pn[rn + fI]) +
                      0.25 * (0.75 * pn[rf + I] + 0.25 * pn[rf + fI]);
    const double vf = 0.75 * (0.75 * pf[rn + I] + 0.25 * pf[rn + fI]) +
                      0.25 * (0.75 * pf[rf + I] + 0.25 * pf[rf + fI]);
    xf[idx] = xf[idx] + (0.75 * vn + 0.25 * vf);
  }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
static int mg_blocks(pb_ctx* ctx, int64_t n) {
  int64_t b = (n + 255) / 256;
  const int64_t cap = (int64_t)ctx->num_cus * 16;
  return (int)std::max<int64_t>(1, std::min(b, cap));
}

// ghost planes of v on level L: in place (1 rank) or exchanged (N ranks)
static int ghosts(MgLevel& L, const double* v, const double** lo, const double** hi) {
  pb_grid* g = L.g;
  if (g->ctx->nranks == 1) {
    *lo = v + (g->nzl - 1) * g->plane;
    *hi = v;
    return PB_OK;
  }
  PB_TRY(halo_exchange(g, v, v + (g->nzl - 1) * g->plane));
  *lo = g->ghost_lo;
  *hi = g->ghost_hi;
  return PB_OK;
}

static int smooth(Mg* mg, MgLevel& L, int color, bool zero_init) {
  const double *lo = nullptr, *hi = nullptr;
  if (!zero_init) PB_TRY(ghosts(L, L.x, &lo, &hi));
  const MgGeo G = L.geo();
  hipLaunchKernelGGL(mg_smooth_kernel, dim3(mg_blocks(mg->ctx, G.nlocal)), dim3(256), 0,
                     mg->ctx->stream, G, L.x, (const double*)L.b, lo, hi, L.s, mg->omega, color,
                     zero_init ? 1 : 0);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

// coarsest level: `coarse_its` symmetric red-black sweeps from zero (red, black, red, black, ...)
static int coarse_solve(Mg* mg, MgLevel& L) {
  PB_TRY(smooth(mg, L, 0, true));
  for (int it = 0; it < mg->coarse_its; ++it) {
    PB_TRY(smooth(mg, L, 1, false));
    PB_TRY(smooth(mg, L, 0, false));
  }
  return PB_OK;
}

int mg_plan_levels(const int64_t n[3], int nranks, int levels_req) {
  std::vector<int64_t> k0(nranks), nz(nranks);
  for (int r = 0; r < nranks; ++r) pb_slab_partition(n[2], nranks, r, &k0[r], &nz[r]);
  int64_t cur[3] = {n[0], n[1], n[2]};
  int L = 1;
  const int cap = levels_req > 0 ? levels_req : 64;
  while (L < cap) {
    bool ok = true;
    for (int d = 0; d < 3; ++d) ok = ok && cur[d] % 4 == 0;  // coarse extents stay even
    if (levels_req <= 0) ok = ok && std::min(cur[0], std::min(cur[1], cur[2])) > 4;
    for (int r = 0; r < nranks; ++r) ok = ok && k0[r] % 2 == 0 && nz[r] % 2 == 0;
    if (!ok) break;
    for (int d = 0; d < 3; ++d) cur[d] /= 2;
    for (int r = 0; r < nranks; ++r) {
      k0[r] /= 2;
      nz[r] /= 2;
    }
    ++L;
  }
  return L;
}

int mg_levels(const Mg* mg) { return (int)mg->lv.size(); }

void mg_destroy(Mg* mg) {
  if (!mg) return;
  (void)hipStreamSynchronize(mg->ctx->stream);
  for (auto& L : mg->lv)
    if (L.own) pb_grid_destroy(L.g);
  if (mg->mem) (void)hipFree(mg->mem);
  delete mg;
}

int mg_create(pb_grid* g, const double deltas[3], int pc_type, int levels_req, int coarse_its,
              double omega, Mg** out) {
  pb_ctx* ctx = g->ctx;
  for (int d = 0; d < 3; ++d)
    if (g->n[d] % 2)
      return set_error(PB_ERR_UNSUPPORTED,
                       "red-black SOR / multigrid needs even grid extents (got %lld x %lld x %lld)",
                       (long long)g->n[0], (long long)g->n[1], (long long)g->n[2]);
  if (!(omega > 0.0 && omega < 2.0)) return set_error(PB_ERR_ARG, "SOR omega must be in (0, 2)");
  Mg* mg = new Mg();
  mg->ctx = ctx;
  mg->omega = omega;
  const int L = pc_type == PB_PC_MG ? mg_plan_levels(g->n, ctx->nranks, levels_req) : 1;
  mg->coarse_its = pc_type == PB_PC_MG ? std::max(1, coarse_its) : 1;
  mg->lv.resize(L);
  int64_t total = 0;
  for (int l = 0; l < L; ++l) {
    MgLevel& lv = mg->lv[l];
    for (int d = 0; d < 3; ++d) {
      lv.n[d] = g->n[d] >> l;
      lv.h[d] = deltas[d] * (double)(1 << l);
    }
    lv.s = star_coeffs(lv.h);
    if (l == 0) {
      lv.g = g;
    } else {
      const int rc = grid_create_part(ctx, lv.n, g->L, g->k0 >> l, g->nzl >> l, &lv.g);
      if (rc != PB_OK) {
        mg_destroy(mg);
        return rc;
      }
      lv.own = true;
      total += 2 * lv.g->nlocal;  // x, b
    }
    if (l < L - 1) total += lv.g->nlocal;  // residual
  }
  if (total > 0 && hipMalloc(&mg->mem, (size_t)total * sizeof(double)) != hipSuccess) {
    mg_destroy(mg);
    return set_error(PB_ERR_ALLOC, "multigrid levels: out of device memory");
  }
  double* p = mg->mem;
  for (int l = 0; l < L; ++l) {
    MgLevel& lv = mg->lv[l];
    if (l > 0) {
      lv.x = p;
      p += lv.g->nlocal;
      lv.b = p;
      p += lv.g->nlocal;
    }
    if (l < L - 1) {
      lv.res = p;
      p += lv.g->nlocal;
    }
  }
  *out = mg;
  return PB_OK;
}

int mg_apply(Mg* mg, const double* r, double* z) {
  ScopedTimer tm(mg->ctx, "mg_apply");
  const int L = (int)mg->lv.size();
  mg->lv[0].b = const_cast<double*>(r);
  mg->lv[0].x = z;
  pb_ctx* ctx = mg->ctx;
  for (int l = 0; l < L - 1; ++l) {  // down: pre-smooth (red, black), residual, restrict
    MgLevel& F = mg->lv[l];
    MgLevel& Cl = mg->lv[l + 1];
    PB_TRY(smooth(mg, F, 0, true));
    PB_TRY(smooth(mg, F, 1, false));
    const double *lo, *hi;
    PB_TRY(ghosts(F, F.x, &lo, &hi));
    const MgGeo G = F.geo();
    hipLaunchKernelGGL(mg_residual_kernel, dim3(mg_blocks(ctx, G.nlocal)), dim3(256), 0,
                       ctx->stream, G, (const double*)F.x, (const double*)F.b, lo, hi, F.s, F.res);
    PB_HIP(hipGetLastError());
    PB_TRY(ghosts(F, F.res, &lo, &hi));
    const MgGeo CG = Cl.geo();
    hipLaunchKernelGGL(mg_restrict_kernel, dim3(mg_blocks(ctx, CG.nlocal)), dim3(256), 0,
                       ctx->stream, G, (const double*)F.res, lo, hi, CG, Cl.b);
    PB_HIP(hipGetLastError());
  }
  PB_TRY(coarse_solve(mg, mg->lv[L - 1]));
  for (int l = L - 2; l >= 0; --l) {  // up: prolongate + correct, post-smooth (black, red)
    MgLevel& F = mg->lv[l];
    MgLevel& Cl = mg->lv[l + 1];
    const double *lo, *hi;
    PB_TRY(ghosts(Cl, Cl.x, &lo, &hi));
    const MgGeo G = F.geo(), CG = Cl.geo();
    hipLaunchKernelGGL(mg_prolong_kernel, dim3(mg_blocks(ctx, G.nlocal)), dim3(256), 0, ctx->stream,
                       G, F.x, CG, (const double*)Cl.x, lo, hi);
    PB_HIP(hipGetLastError());
    PB_TRY(smooth(mg, F, 1, false));
    PB_TRY(smooth(mg, F, 0, false));
  }
  return PB_OK;
}

}  // namespace pb
