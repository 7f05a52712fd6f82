/* pb_oracle.c -- CPU restatement of the poissbox hot path.
 *
 * TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the checker / reported CPU baseline. The product (poissbox_amd/,
 * libpoissbox_gpu.so) never links or calls this file.
 *
 * Every function cites the reference (3decomp/poissbox) file:line it restates. Arithmetic is
 * written in the reference's evaluation order; build with -ffp-contract=off (see Makefile) so
 * that no multiply-add is fused -- the flang-built reference (oracle/_ref) on x86-64 baseline
 * has no FMA either, which is what makes the tridiagonal/compact pins bit-exact.
 */
#include "pb_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define IDX(i, j, k, nx, ny) ((i) + (nx) * ((j) + (ny) * (k)))

static inline int64_t wrap(int64_t i, int64_t n) { return i < 0 ? i + n : (i >= n ? i - n : i); }

/* ---------------------------------------------------------------------------------------------
 * Coefficients
 * ------------------------------------------------------------------------------------------- */

/* src/coefficients.f90:22-35 lapl_1d_coeffs: [1, -2, 1] / dx**2 */
void pbo_lapl_1d_coeffs(double dx, double c[3]) {
  double invdx2 = 1.0 / (dx * dx);
  c[0] = invdx2;
  c[1] = -(2.0 * invdx2);
  c[2] = invdx2;
}

/* src/coefficients.f90:38-48 lapl_star_coeffs: zero box, then the three 1-D stencils are
 * ADDED along the x, y and z lines through the centre (centre accumulates x, then y, then z). */
void pbo_lapl_star_coeffs(double dx, double dy, double dz, double c[27]) {
  double cx[3], cy[3], cz[3];
  pbo_lapl_1d_coeffs(dx, cx);
  pbo_lapl_1d_coeffs(dy, cy);
  pbo_lapl_1d_coeffs(dz, cz);
  for (int m = 0; m < 27; ++m) c[m] = 0.0;
  /* column-major (ii,jj,kk) -> ii + 3*jj + 9*kk */
  for (int t = 0; t < 3; ++t) c[t + 3 * 1 + 9 * 1] += cx[t]; /* coeffs(:, 2, 2) */
  for (int t = 0; t < 3; ++t) c[1 + 3 * t + 9 * 1] += cy[t]; /* coeffs(2, :, 2) */
  for (int t = 0; t < 3; ++t) c[1 + 3 * 1 + 9 * t] += cz[t]; /* coeffs(2, 2, :) */
}

/* Jacobi diagonal of P = centre coefficient (src/coefficients.f90:44-46 via :105) */
double pbo_diag(const double h[3]) {
  double c[27];
  pbo_lapl_star_coeffs(h[0], h[1], h[2], c);
  return c[13];
}

/* ---------------------------------------------------------------------------------------------
 * 7-point operator
 * ------------------------------------------------------------------------------------------- */

/* src/poissbox.f90:84-126 compute_lapl_pointwise + :128-148 evaluate_laplacian_pointwise:
 * for every owned point, dot_product(reshape(xdof(i-1:i+1, j-1:j+1, k-1:k+1)), reshape(coeffs))
 * with the coefficients rebuilt per point (:143) and periodic ghosts (DM_BOUNDARY_PERIODIC,
 * :192). Summation runs over all 27 entries in column-major order, starting from 0. */
static void stencil27_mt(const int64_t n[3], const double h[3], const double* x, double* y,
                         int nt) {
  const int64_t nx = n[0], ny = n[1], nz = n[2];
  (void)nt; /* points are independent: any thread count gives the same bits */
#pragma omp parallel for num_threads(nt) schedule(static) collapse(2) if (nt > 1)
  for (int64_t k = 0; k < nz; ++k)
    for (int64_t j = 0; j < ny; ++j)
      for (int64_t i = 0; i < nx; ++i) {
        double c[27];
        pbo_lapl_star_coeffs(h[0], h[1], h[2], c); /* recomputed at every point, :143 */
        double s = 0.0;
        for (int kk = 0; kk < 3; ++kk)
          for (int jj = 0; jj < 3; ++jj)
            for (int ii = 0; ii < 3; ++ii) {
              double f = x[IDX(wrap(i + ii - 1, nx), wrap(j + jj - 1, ny), wrap(k + kk - 1, nz), nx, ny)];
              s += f * c[ii + 3 * jj + 9 * kk];
            }
        y[IDX(i, j, k, nx, ny)] = s;
      }
}
void pbo_stencil_apply27(const int64_t n[3], const double h[3], const double* x, double* y) {
  stencil27_mt(n, h, x, y, 1);
}

/* Same operator with the 20 zero terms dropped. For finite x, 0*f adds +-0 to a running sum that
 * is exactly 0 until the first non-zero term, so the result is bit-identical to apply27:
 * ((((((cz*f[z-] + cy*f[y-]) + cx*f[x-]) + cc*f[c]) + cx*f[x+]) + cy*f[y+]) + cz*f[z+]). */
void pbo_stencil_apply7(const int64_t n[3], const double h[3], const double* x, double* y,
                        int nthreads) {
  const int64_t nx = n[0], ny = n[1], nz = n[2];
  double c[27];
  pbo_lapl_star_coeffs(h[0], h[1], h[2], c);
  const double cx = c[12], cy = c[10], cz = c[4], cc = c[13];
  (void)nthreads;
#pragma omp parallel for num_threads(nthreads) schedule(static) collapse(2)
  for (int64_t k = 0; k < nz; ++k)
    for (int64_t j = 0; j < ny; ++j) {
      const double* xm = x + nx * (j + ny * wrap(k - 1, nz));
      const double* xp = x + nx * (j + ny * wrap(k + 1, nz));
      const double* ym = x + nx * (wrap(j - 1, ny) + ny * k);
      const double* yp = x + nx * (wrap(j + 1, ny) + ny * k);
      const double* xc = x + nx * (j + ny * k);
      double* out = y + nx * (j + ny * k);
      for (int64_t i = 0; i < nx; ++i) {
        int64_t im = i == 0 ? nx - 1 : i - 1, ip = i == nx - 1 ? 0 : i + 1;
        double s = cz * xm[i];
        s += cy * ym[i];
        s += cx * xc[im];
        s += cc * xc[i];
        s += cx * xc[ip];
        s += cy * yp[i];
        s += cz * xp[i];
        out[i] = s;
      }
    }
}

/* One z-slab of nzl planes with explicit ghost planes below (glo) and above (ghi): the per-rank
 * view of compute_lapl_pointwise after DMGlobalToLocal (src/poissbox.f90:104-119). x/y periodic. */
void pbo_stencil_slab(const int64_t n[3], const double h[3], const double* x, const double* glo,
                      const double* ghi, double* y) {
  const int64_t nx = n[0], ny = n[1], nz = n[2];
  double c[27];
  pbo_lapl_star_coeffs(h[0], h[1], h[2], c);
  const double cx = c[12], cy = c[10], cz = c[4], cc = c[13];
  for (int64_t k = 0; k < nz; ++k)
    for (int64_t j = 0; j < ny; ++j) {
      const double* xm = k == 0 ? glo + nx * j : x + nx * (j + ny * (k - 1));
      const double* xp = k == nz - 1 ? ghi + nx * j : x + nx * (j + ny * (k + 1));
      const double* ym = x + nx * (wrap(j - 1, ny) + ny * k);
      const double* yp = x + nx * (wrap(j + 1, ny) + ny * k);
      const double* xc = x + nx * (j + ny * k);
      double* out = y + nx * (j + ny * k);
      for (int64_t i = 0; i < nx; ++i) {
        int64_t im = i == 0 ? nx - 1 : i - 1, ip = i == nx - 1 ? 0 : i + 1;
        double s = cz * xm[i];
        s += cy * ym[i];
        s += cx * xc[im];
        s += cc * xc[i];
        s += cx * xc[ip];
        s += cy * yp[i];
        s += cz * xp[i];
        out[i] = s;
      }
    }
}

static int cmp_i64(const void* a, const void* b) {
  int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
  return x < y ? -1 : x > y;
}

/* src/coefficients.f90:50-113 assemble_laplacian: one MatSetValuesStencil row of the 27 box
 * entries (20 explicit zeros) per DoF, INSERT_VALUES. MatMult sums a row's stored entries in
 * ascending column order: on one rank (SeqAIJ) ascending global column (natural ordering); on
 * `nranks` z-slabs (MPIAIJ, MatMult_MPIAIJ) first the diagonal block -- the columns this rank owns,
 * ascending -- then the off-diagonal block added onto it (MatMultAdd), columns ascending by global
 * index. The slabs follow pbo-side slab_partition (remainder planes on the low ranks, as
 * pb_slab_partition / README.md:30-32). Requires n >= 3 in every direction so the 27 columns are
 * distinct. 0 * x products of the explicit zeros leave every partial sum unchanged. */
static void slab_of(int64_t nz, int nranks, int r, int64_t* k0, int64_t* nk) {
  const int64_t q = nz / nranks, rem = nz % nranks;
  *nk = q + (r < rem ? 1 : 0);
  *k0 = r * q + (r < rem ? r : rem);
}

void pbo_assembled_apply(const int64_t n[3], const double h[3], int nranks, const double* x,
                         double* y) {
  const int64_t nx = n[0], ny = n[1], nz = n[2];
  const int64_t plane = nx * ny;
  if (nranks < 1) nranks = 1;
  double c[27];
  pbo_lapl_star_coeffs(h[0], h[1], h[2], c);
  for (int r = 0; r < nranks; ++r) {
    int64_t k0, nk;
    slab_of(nz, nranks, r, &k0, &nk);
    const int64_t lo = k0 * plane, hi = (k0 + nk) * plane; /* owned rows / columns */
    for (int64_t k = k0; k < k0 + nk; ++k)
      for (int64_t j = 0; j < ny; ++j)
        for (int64_t i = 0; i < nx; ++i) {
          int64_t key[27][2];
          for (int m = 0; m < 27; ++m) {
            int ii = m % 3, jj = (m / 3) % 3, kk = m / 9;
            const int64_t col =
                IDX(wrap(i + ii - 1, nx), wrap(j + jj - 1, ny), wrap(k + kk - 1, nz), nx, ny);
            const int64_t off = (nranks > 1 && (col < lo || col >= hi)) ? 1 : 0;
            key[m][0] = (off << 62) | col;
            key[m][1] = m;
          }
          qsort(key, 27, sizeof(key[0]), cmp_i64);
          double s = 0.0;
          for (int m = 0; m < 27; ++m)
            s += c[key[m][1]] * x[key[m][0] & (((int64_t)1 << 62) - 1)];
          y[IDX(i, j, k, nx, ny)] = s;
        }
  }
}

/* ---------------------------------------------------------------------------------------------
 * Synthetic input (same distribution as src/example.f90:180-181)
 * ------------------------------------------------------------------------------------------- */
uint64_t pbo_splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

void pbo_fill_random(int64_t count, uint64_t seed, int64_t g0, double* x) {
  for (int64_t t = 0; t < count; ++t) {
    double u = (double)(pbo_splitmix64(seed ^ (uint64_t)(g0 + t)) >> 11) * 0x1.0p-53;
    x[t] = 2.0 * (0.5 - u); /* src/example.f90:181 */
  }
}

/* ---------------------------------------------------------------------------------------------
 * KSPSolve with -ksp_type cg -pc_type jacobi and the constant null space
 * (src/poissbox.f90:269-298 -> PETSc KSPSolve_CG; semantics in SURVEY.md Appendix A)
 * ------------------------------------------------------------------------------------------- */
enum {
  KSP_CONVERGED_ITERATING = 0, KSP_CONVERGED_RTOL = 2, KSP_CONVERGED_ATOL = 3,
  KSP_DIVERGED_ITS = -3, KSP_DIVERGED_DTOL = -4, KSP_DIVERGED_NANORINF = -9,
  KSP_DIVERGED_INDEFINITE_PC = -8, KSP_DIVERGED_INDEFINITE_MAT = -10
};

static double vdot(int64_t N, const double* a, const double* b, int nt) {
  double s = 0.0;
  (void)nt;
#pragma omp parallel for num_threads(nt) reduction(+ : s) schedule(static) if (nt > 1)
  for (int64_t t = 0; t < N; ++t) s += b[t] * a[t];
  return s;
}
static double vsum(int64_t N, const double* a, int nt) {
  double s = 0.0;
  (void)nt;
#pragma omp parallel for num_threads(nt) reduction(+ : s) schedule(static) if (nt > 1)
  for (int64_t t = 0; t < N; ++t) s += a[t];
  return s;
}

/* ---------------------------------------------------------------------------------------------
 * Red-black SOR / geometric V(1,1) multigrid preconditioner -- restatement of the GPU design in
 * poissbox_amd/csrc/pb_mg.hip with the same arithmetic order (tests compare bit for bit).
 * Periodic cell-centred grid, 7-point operator per level with h_l = 2^l h (lapl_star_coeffs),
 * trilinear prolongation, restriction = P^T / 8, red = (i + j + k) even.
 * ------------------------------------------------------------------------------------------- */
static void slab_part(int64_t n, int nranks, int r, int64_t* k0, int64_t* nz) {
  const int64_t q = n / nranks, m = n % nranks; /* README.md:30-32: remainder on low ranks */
  *nz = q + (r < m ? 1 : 0);
  *k0 = r * q + (r < m ? r : m);
}

int pbo_mg_plan_levels(const int64_t n[3], int nranks, int levels_req) {
  int64_t cur[3] = {n[0], n[1], n[2]};
  int64_t* k0 = (int64_t*)malloc(sizeof(int64_t) * nranks);
  int64_t* nz = (int64_t*)malloc(sizeof(int64_t) * nranks);
  for (int r = 0; r < nranks; ++r) slab_part(n[2], nranks, r, &k0[r], &nz[r]);
  int L = 1;
  const int cap = levels_req > 0 ? levels_req : 64;
  while (L < cap) {
    int ok = cur[0] % 4 == 0 && cur[1] % 4 == 0 && cur[2] % 4 == 0;
    if (levels_req <= 0) {
      int64_t mn = cur[0] < cur[1] ? cur[0] : cur[1];
      mn = mn < cur[2] ? mn : cur[2];
      ok = ok && mn > 4;
    }
    for (int r = 0; r < nranks; ++r) ok = ok && k0[r] % 2 == 0 && nz[r] % 2 == 0;
    if (!ok) break;
    for (int d = 0; d < 3; ++d) cur[d] /= 2;
    for (int r = 0; r < nranks; ++r) {
      k0[r] /= 2;
      nz[r] /= 2;
    }
    ++L;
  }
  free(k0);
  free(nz);
  return L;
}

typedef struct {
  int64_t n[3];
  double cx, cy, cz, cc;
  double *x, *b, *res;
} mg_level;

static int64_t wrap64(int64_t v, int64_t n) { return v < 0 ? v + n : (v >= n ? v - n : v); }

static void mg_smooth(const mg_level* L, int color, int zero_init, double omega) {
  const int64_t nx = L->n[0], ny = L->n[1], nz = L->n[2];
  const double icc = 1.0 / L->cc; /* the update multiplies by the inverted diagonal (MatSOR idiag) */
  for (int64_t k = 0; k < nz; ++k)
    for (int64_t j = 0; j < ny; ++j)
      for (int64_t i = 0; i < nx; ++i) {
        const int64_t id = i + nx * (j + ny * k);
        if (((i + j + k) & 1) != color) {
          if (zero_init) L->x[id] = 0.0;
          continue;
        }
        double nb = 0.0, xo = 0.0;
        if (!zero_init) {
          const double* x = L->x;
          nb = L->cz * x[i + nx * (j + ny * wrap64(k - 1, nz))];
          nb = nb + L->cy * x[i + nx * (wrap64(j - 1, ny) + ny * k)];
          nb = nb + L->cx * x[wrap64(i - 1, nx) + nx * (j + ny * k)];
          nb = nb + L->cx * x[wrap64(i + 1, nx) + nx * (j + ny * k)];
          nb = nb + L->cy * x[i + nx * (wrap64(j + 1, ny) + ny * k)];
          nb = nb + L->cz * x[i + nx * (j + ny * wrap64(k + 1, nz))];
          xo = x[id];
        }
        const double t = (L->b[id] - nb) * icc;
        L->x[id] = (1.0 - omega) * xo + omega * t;
      }
}

static void mg_residual(const mg_level* L) {
  const int64_t nx = L->n[0], ny = L->n[1], nz = L->n[2];
  const double* x = L->x;
  for (int64_t k = 0; k < nz; ++k)
    for (int64_t j = 0; j < ny; ++j)
      for (int64_t i = 0; i < nx; ++i) {
        const int64_t id = i + nx * (j + ny * k);
        double ax = L->cz * x[i + nx * (j + ny * wrap64(k - 1, nz))];
        ax = ax + L->cy * x[i + nx * (wrap64(j - 1, ny) + ny * k)];
        ax = ax + L->cx * x[wrap64(i - 1, nx) + nx * (j + ny * k)];
        ax = ax + L->cc * x[id];
        ax = ax + L->cx * x[wrap64(i + 1, nx) + nx * (j + ny * k)];
        ax = ax + L->cy * x[i + nx * (wrap64(j + 1, ny) + ny * k)];
        ax = ax + L->cz * x[i + nx * (j + ny * wrap64(k + 1, nz))];
        L->res[id] = L->b[id] - ax;
      }
}

static void mg_restrict(const mg_level* F, const mg_level* Cl) {
  static const double w[4] = {0.125, 0.375, 0.375, 0.125};
  const int64_t fx = F->n[0], fy = F->n[1], fz = F->n[2];
  for (int64_t K = 0; K < Cl->n[2]; ++K)
    for (int64_t J = 0; J < Cl->n[1]; ++J)
      for (int64_t I = 0; I < Cl->n[0]; ++I) {
        double sz = 0.0;
        for (int c = 0; c < 4; ++c) {
          const int64_t kf = wrap64(2 * K - 1 + c, fz);
          double sy = 0.0;
          for (int bb = 0; bb < 4; ++bb) {
            const int64_t jf = wrap64(2 * J - 1 + bb, fy);
            double sx = 0.0;
            for (int a = 0; a < 4; ++a)
              sx = sx + w[a] * F->res[wrap64(2 * I - 1 + a, fx) + fx * (jf + fy * kf)];
            sy = sy + w[bb] * sx;
          }
          sz = sz + w[c] * sy;
        }
        Cl->b[I + Cl->n[0] * (J + Cl->n[1] * K)] = sz;
      }
}

static void mg_prolong(const mg_level* F, const mg_level* Cl) {
  const int64_t cx = Cl->n[0], cy = Cl->n[1], cz = Cl->n[2];
  const double* c = Cl->x;
  for (int64_t k = 0; k < F->n[2]; ++k)
    for (int64_t j = 0; j < F->n[1]; ++j)
      for (int64_t i = 0; i < F->n[0]; ++i) {
        const int64_t I = i >> 1, J = j >> 1, K = k >> 1;
        const int64_t fI = wrap64((i & 1) ? I + 1 : I - 1, cx);
        const int64_t fJ = wrap64((j & 1) ? J + 1 : J - 1, cy);
        const int64_t fK = wrap64((k & 1) ? K + 1 : K - 1, cz);
#define C3(a, b, d) c[(a) + cx * ((b) + cy * (d))]
        const double vn = 0.75 * (0.75 * C3(I, J, K) + 0.25 * C3(fI, J, K)) +
                          0.25 * (0.75 * C3(I, fJ, K) + 0.25 * C3(fI, fJ, K));
        const double vf = 0.75 * (0.75 * C3(I, J, fK) + 0.25 * C3(fI, J, fK)) +
                          0.25 * (0.75 * C3(I, fJ, fK) + 0.25 * C3(fI, fJ, fK));
#undef C3
        const int64_t id = i + F->n[0] * (j + F->n[1] * k);
        F->x[id] = F->x[id] + (0.75 * vn + 0.25 * vf);
      }
}

void pbo_mg_apply(const int64_t n[3], const double h[3], int pc_type, int levels, int coarse_its,
                  double omega, int nranks, const double* r, double* z) {
  const int L = pc_type == 3 ? pbo_mg_plan_levels(n, nranks, levels) : 1;
  const int cits = pc_type == 3 ? (coarse_its > 1 ? coarse_its : 1) : 1;
  mg_level* lv = (mg_level*)calloc((size_t)L, sizeof(mg_level));
  for (int l = 0; l < L; ++l) {
    double hl[3], c27[27];
    for (int d = 0; d < 3; ++d) {
      lv[l].n[d] = n[d] >> l;
      hl[d] = h[d] * (double)(1 << l);
    }
    pbo_lapl_star_coeffs(hl[0], hl[1], hl[2], c27);
    lv[l].cx = c27[12];
    lv[l].cy = c27[10];
    lv[l].cz = c27[4];
    lv[l].cc = c27[13];
    const int64_t m = lv[l].n[0] * lv[l].n[1] * lv[l].n[2];
    lv[l].x = l ? (double*)malloc(sizeof(double) * m) : z;
    lv[l].b = l ? (double*)malloc(sizeof(double) * m) : (double*)r;
    lv[l].res = (double*)malloc(sizeof(double) * m);
  }
  for (int l = 0; l < L - 1; ++l) {
    mg_smooth(&lv[l], 0, 1, omega);
    mg_smooth(&lv[l], 1, 0, omega);
    mg_residual(&lv[l]);
    mg_restrict(&lv[l], &lv[l + 1]);
  }
  mg_smooth(&lv[L - 1], 0, 1, omega);
  for (int it = 0; it < cits; ++it) {
    mg_smooth(&lv[L - 1], 1, 0, omega);
    mg_smooth(&lv[L - 1], 0, 0, omega);
  }
  for (int l = L - 2; l >= 0; --l) {
    mg_prolong(&lv[l], &lv[l + 1]);
    mg_smooth(&lv[l], 1, 0, omega);
    mg_smooth(&lv[l], 0, 0, omega);
  }
  for (int l = 0; l < L; ++l) {
    if (l) {
      free(lv[l].x);
      free(lv[l].b);
    }
    free(lv[l].res);
  }
  free(lv);
}

/* ---- spectral preconditioner (-pc_type fft): restates pb_fft.hip's definition, not its FFT ----
 * Both P's are sums of products of 1-D circulants with real even symbols, so the separable
 * Hartley transform H (H_d[j][k] = cas(2 pi j k / n_d), H_d H_d = n_d I) diagonalises them:
 *   P^+ = H diag(1 / (N lambda)) H.
 * 7-point star (src/coefficients.f90:22-48): lambda = sum_d (2 cos t_d - 2) / h_d^2.
 * compact lapl (src/compact_schemes.f90:17-37, coefficients :188-190 / :303-305):
 *   lambda = Lx Jy Jz + Jx Ly Jz + Jx Jy Lz,
 *   L(t) = -4 (a_d sin(t/2) + b_d sin(3t/2))^2 / (1 + 2 al_d cos t)^2   (D+ D-),
 *   J(t) =  4 (a_i cos(t/2) + b_i cos(3t/2))^2 / (1 + 2 al_i cos t)^2   (I+ I-).
 * Pinned by tests/test_oracle.py: P (pbo_stencil_apply7 / pbo_lapl, themselves pinned to the
 * reference) applied to z gives r minus its null-mode part, and a numpy complex-FFT statement of
 * the same definition agrees. */
static void fft_axis_symbols(int compact, int64_t n, double h, double* L, double* J) {
  const long double pi = 3.14159265358979323846264338327950288L;
  const long double a_d = 63.0L / 62.0L / h, b_d = 17.0L / 62.0L / (3.0L * h), al_d = 9.0L / 62.0L;
  const long double a_i = 0.75L, b_i = 1.0L / 20.0L, al_i = 3.0L / 10.0L;
  for (int64_t k = 0; k < n; ++k) {
    const long double t = 2.0L * pi * (long double)k / (long double)n;
    if (!compact) {
      L[k] = (double)((2.0L * cosl(t) - 2.0L) / ((long double)h * (long double)h));
      J[k] = 1.0;
    } else {
      const long double sd = a_d * sinl(t / 2) + b_d * sinl(1.5L * t), td = 1 + 2 * al_d * cosl(t);
      const long double si = a_i * cosl(t / 2) + b_i * cosl(1.5L * t), ti = 1 + 2 * al_i * cosl(t);
      L[k] = (double)(-4.0L * sd * sd / (td * td));
      J[k] = (double)(4.0L * si * si / (ti * ti));
    }
  }
}

/* in place: u[e] over lines of axis d (n = extent, stride) <- sum_j u[j] cas(2 pi j e / n) */
static void dht_axis_naive(const int64_t n[3], int d, double* u) {
  const long double pi = 3.14159265358979323846264338327950288L;
  const int64_t m = n[d], stride = d == 0 ? 1 : (d == 1 ? n[0] : n[0] * n[1]);
  double* cas = (double*)malloc(sizeof(double) * m);
  for (int64_t q = 0; q < m; ++q) {
    const long double t = 2.0L * pi * (long double)q / (long double)m;
    cas[q] = (double)(cosl(t) + sinl(t));
  }
  const int64_t N = n[0] * n[1] * n[2], lines = N / m;
#pragma omp parallel
  {
    double* in = (double*)malloc(sizeof(double) * m);
#pragma omp for schedule(static)
    for (int64_t l = 0; l < lines; ++l) {
      /* line l: base = (l % stride) + (l / stride) * stride * m */
      const int64_t base = (l % stride) + (l / stride) * stride * m;
      for (int64_t j = 0; j < m; ++j) in[j] = u[base + j * stride];
      for (int64_t e = 0; e < m; ++e) {
        double acc = 0.0;
        for (int64_t j = 0; j < m; ++j) acc += in[j] * cas[(j * e) % m];
        u[base + e * stride] = acc;
      }
    }
    free(in);
  }
  free(cas);
}

void pbo_fft_pc_apply(const int64_t n[3], const double h[3], int compact, const double* r,
                      double* z) {
  const int64_t N = n[0] * n[1] * n[2];
  double* L[3];
  double* J[3];
  double bound = 0.0, lmax[3], jmax[3];
  for (int d = 0; d < 3; ++d) {
    L[d] = (double*)malloc(sizeof(double) * n[d]);
    J[d] = (double*)malloc(sizeof(double) * n[d]);
    fft_axis_symbols(compact, n[d], h[d], L[d], J[d]);
    lmax[d] = jmax[d] = 0.0;
    for (int64_t k = 0; k < n[d]; ++k) {
      lmax[d] = fmax(lmax[d], fabs(L[d][k]));
      jmax[d] = fmax(jmax[d], J[d][k]);
    }
  }
  bound = lmax[0] * jmax[1] * jmax[2] + jmax[0] * lmax[1] * jmax[2] + jmax[0] * jmax[1] * lmax[2];
  const double thr = 1e-10 * bound, scale = 1.0 / ((double)n[0] * (double)n[1] * (double)n[2]);
  memcpy(z, r, sizeof(double) * N);
  for (int d = 0; d < 3; ++d) dht_axis_naive(n, d, z);
  for (int64_t k = 0; k < n[2]; ++k)
    for (int64_t j = 0; j < n[1]; ++j)
      for (int64_t i = 0; i < n[0]; ++i) {
        const double lam = (L[0][i] * J[1][j] + J[0][i] * L[1][j]) * J[2][k] +
                           J[0][i] * J[1][j] * L[2][k];
        const int64_t id = i + n[0] * (j + n[1] * k);
        z[id] = fabs(lam) > thr ? z[id] * (scale / lam) : 0.0;
      }
  for (int d = 0; d < 3; ++d) dht_axis_naive(n, d, z);
  for (int d = 0; d < 3; ++d) {
    free(L[d]);
    free(J[d]);
  }
}

/* KSP_PCApply = PCApply_Jacobi (z = diag^-1 .* r, PETSc stores the reciprocal) followed by
 * KSP_RemoveNullSpace -> MatNullSpaceRemove(has_cnst): z += VecSum(z) / (-N). */
static void pc_apply(int64_t N, const double* r, double* z, double dinv, int pc, int nsp, int nt) {
  (void)nt;
#pragma omp parallel for num_threads(nt) schedule(static) if (nt > 1)
  for (int64_t t = 0; t < N; ++t) z[t] = pc ? dinv * r[t] : r[t];
  if (nsp) {
    double shift = vsum(N, z, nt) / (-1.0 * (double)N);
#pragma omp parallel for num_threads(nt) schedule(static) if (nt > 1)
    for (int64_t t = 0; t < N; ++t) z[t] += shift;
  }
}

static void op_apply(const int64_t n[3], const double h[3], const double* x, double* y, int kind,
                     int nt) {
  if (kind == 1)
    stencil27_mt(n, h, x, y, nt); /* faithful operator; one core = one reference MPI rank */
  else if (kind == 2)
    pbo_lapl(n, x, h, y); /* compact A; P (Jacobi diag) stays the 7-point */
  else if (kind >= 3)
    pbo_assembled_apply(n, h, kind - 2, x, y); /* A = P assembled, MatMult on kind-2 z-slabs */
  else
    pbo_stencil_apply7(n, h, x, y, nt);
}

/* PCApply for every pc_type: Jacobi / none as above; SOR (2) and MG (3) through pbo_mg_apply,
 * FFT (4) through pbo_fft_pc_apply,
 * followed by the same null-space removal */
static void pc_apply_any(const int64_t n[3], const double h[3], const pbo_ksp_opts* o,
                         const double* r, double* z, double dinv, int nt) {
  const int64_t N = n[0] * n[1] * n[2];
  if (o->pc_type == 2 || o->pc_type == 3 || o->pc_type == 4) {
    if (o->pc_type == 4)
      pbo_fft_pc_apply(n, h, o->pc_compact, r, z);
    else
      pbo_mg_apply(n, h, o->pc_type, o->mg_levels, o->mg_coarse_its, o->omega,
                   o->nranks > 0 ? o->nranks : 1, r, z);
    if (o->nullspace) {
      double shift = vsum(N, z, nt) / (-1.0 * (double)N);
      for (int64_t t = 0; t < N; ++t) z[t] += shift;
    }
    return;
  }
  pc_apply(N, r, z, dinv, o->pc_type, o->nullspace, nt);
}

/* PETSc KSPSolve_CG_SingleReduction (cg.c, selected by -ksp_cg_single_reduction through
 * KSPSetFromOptions, src/poissbox.f90:295; PETSc is external and absent -- restated from its
 * published cg.c). KSP_NORM_PRECONDITIONED (KSPCG's default): identical to KSPSolve_CG in exact
 * arithmetic, with S = A z formed right after z, delta = z'S and beta = z'r taken together
 * (VecMDot), w = A p and p'w by recurrence:  w_i = s_i + (beta/betaold) w_{i-1},
 * dpi = delta - beta^2 dpiold / betaold^2  (i > 0; i = 0: w = A p, dpi = p'w).
 * form 2 keeps the recurrence for dpi and recomputes w = A p (the GPU pass's arithmetic). */
static int cg_solve_single_reduction(const int64_t n[3], const double h[3], const pbo_ksp_opts* o,
                                     const double* b, double* x, double* history,
                                     int64_t* its_out, int64_t* nlog_out) {
  const int64_t N = n[0] * n[1] * n[2];
  const int nt = o->nthreads > 0 ? o->nthreads : 1;
  const int recompute_w = o->single_reduction == 2;
  double* R = (double*)malloc(sizeof(double) * N);
  double* Z = (double*)malloc(sizeof(double) * N);
  double* P = (double*)malloc(sizeof(double) * N);
  double* S = (double*)malloc(sizeof(double) * N);
  double* W = (double*)malloc(sizeof(double) * N);
  const double dinv = 1.0 / pbo_diag(h);
  int reason = KSP_CONVERGED_ITERATING;
  int64_t its = 0, nlog = 0;
  double dp, beta, betaold = 1.0, dpi = 0.0, dpiold, delta, ttol, rnorm0;

  memset(x, 0, sizeof(double) * N); /* guess_zero */
  memcpy(R, b, sizeof(double) * N); /* r = b */
  pc_apply_any(n, h, o, R, Z, dinv, nt); /* z = B r */
  dp = sqrt(vdot(N, Z, Z, nt));          /* VecNorm(Z) */
  history[0] = dp;
  nlog = 1;
  if (dp != dp || isinf(dp)) { reason = KSP_DIVERGED_NANORINF; goto done; }
  ttol = fmax(o->rtol * dp, o->atol);
  rnorm0 = dp;
  if (dp <= ttol) { reason = dp < o->atol ? KSP_CONVERGED_ATOL : KSP_CONVERGED_RTOL; goto done; }
  op_apply(n, h, Z, S, o->op_kind, nt); /* S = A z */
  delta = vdot(N, Z, S, nt);            /* delta = z'A z */
  beta = vdot(N, Z, R, nt);             /* beta = z'r */
  if (!isfinite(beta)) { reason = KSP_DIVERGED_NANORINF; goto done; } /* KSPCheckDot */

  int64_t i = 0;
  do {
    its = i + 1;
    if (beta == 0.0) { reason = KSP_CONVERGED_ATOL; break; }
    if (i > 0 && beta * betaold < 0.0) { reason = KSP_DIVERGED_INDEFINITE_PC; break; }
    double bb = 0.0;
    if (i == 0) {
      memcpy(P, Z, sizeof(double) * N);
    } else {
      bb = beta / betaold;
#pragma omp parallel for num_threads(nt) schedule(static) if (nt > 1)
      for (int64_t t = 0; t < N; ++t) P[t] = Z[t] + bb * P[t]; /* VecAYPX(P, b, Z) */
    }
    dpiold = dpi;
    if (i == 0 || recompute_w) {
      op_apply(n, h, P, W, o->op_kind, nt); /* w = A p */
      if (i == 0) dpi = vdot(N, P, W, nt);  /* dpi = p'w */
    } else {
      const double c = beta / betaold;
#pragma omp parallel for num_threads(nt) schedule(static) if (nt > 1)
      for (int64_t t = 0; t < N; ++t) W[t] = S[t] + c * W[t]; /* VecAYPX(W, beta/betaold, S) */
    }
    if (i > 0) dpi = delta - beta * beta * dpiold / (betaold * betaold);
    betaold = beta;
    if (dpi == 0.0 || (i > 0 && dpi * dpiold <= 0.0)) {
      reason = KSP_DIVERGED_INDEFINITE_MAT;
      break;
    }
    const double a = beta / dpi;
#pragma omp parallel for num_threads(nt) schedule(static) if (nt > 1)
    for (int64_t t = 0; t < N; ++t) {
      x[t] = x[t] + a * P[t];
      R[t] = R[t] + (-a) * W[t];
    }
    pc_apply_any(n, h, o, R, Z, dinv, nt); /* z = B r */
    op_apply(n, h, Z, S, o->op_kind, nt);  /* S = A z */
    dp = sqrt(vdot(N, Z, Z, nt));
    history[i + 1] = dp;
    nlog = i + 2;
    if (dp != dp || isinf(dp)) { reason = KSP_DIVERGED_NANORINF; break; }
    if (dp <= ttol) { reason = dp < o->atol ? KSP_CONVERGED_ATOL : KSP_CONVERGED_RTOL; break; }
    if (dp >= o->dtol * rnorm0) { reason = KSP_DIVERGED_DTOL; break; }
    delta = vdot(N, Z, S, nt); /* VecMDot(Z, {S, R}) */
    beta = vdot(N, Z, R, nt);
    if (!isfinite(beta)) { reason = KSP_DIVERGED_NANORINF; break; } /* KSPCheckDot */
    i++;
  } while (i < o->max_it);
  if (i >= o->max_it) reason = KSP_DIVERGED_ITS;
done:
  *its_out = its;
  if (nlog_out) *nlog_out = nlog;
  free(R); free(Z); free(P); free(S); free(W);
  return reason;
}

int pbo_cg_solve(const int64_t n[3], const double h[3], const pbo_ksp_opts* o, const double* b,
                 double* x, double* history, int64_t* its_out, int64_t* nlog_out) {
  if (o->single_reduction) return cg_solve_single_reduction(n, h, o, b, x, history, its_out, nlog_out);
  const int64_t N = n[0] * n[1] * n[2];
  const int nt = o->nthreads > 0 ? o->nthreads : 1;
  double* R = (double*)malloc(sizeof(double) * N);
  double* Z = (double*)malloc(sizeof(double) * N);
  double* P = (double*)malloc(sizeof(double) * N);
  double* W = (double*)malloc(sizeof(double) * N);
  const double dinv = 1.0 / pbo_diag(h);
  int reason = KSP_CONVERGED_ITERATING;
  int64_t its = 0, nlog = 0; /* nlog: entries KSPLogResidualHistory wrote */
  double dp, beta, betaold = 0.0, dpi = 0.0, dpiold, ttol, rnorm0;

  memset(x, 0, sizeof(double) * N); /* KSPSolve: guess_zero => X = 0 */
  memcpy(R, b, sizeof(double) * N); /* r = b */
  pc_apply_any(n, h, o, R, Z, dinv, nt);
  dp = sqrt(vdot(N, Z, Z, nt)); /* KSP_NORM_PRECONDITIONED */
  history[0] = dp;
  nlog = 1;
  /* KSPConvergedDefault at n = 0 */
  if (dp != dp || isinf(dp)) { reason = KSP_DIVERGED_NANORINF; goto done; }
  ttol = fmax(o->rtol * dp, o->atol);
  rnorm0 = dp;
  if (dp <= ttol) { reason = dp < o->atol ? KSP_CONVERGED_ATOL : KSP_CONVERGED_RTOL; goto done; }
  beta = vdot(N, Z, R, nt);
  if (!isfinite(beta)) { reason = KSP_DIVERGED_NANORINF; goto done; } /* KSPCheckDot */

  int64_t i = 0;
  do {
    its = i + 1;
    if (beta == 0.0) { reason = KSP_CONVERGED_ATOL; break; }
    /* PETSc KSPSolve_CG (real scalars): z'r changed sign -> the PC is indefinite */
    if (i > 0 && beta * betaold < 0.0) { reason = KSP_DIVERGED_INDEFINITE_PC; break; }
    if (i == 0) {
      memcpy(P, Z, sizeof(double) * N);
    } else {
      double bb = beta / betaold;
#pragma omp parallel for num_threads(nt) schedule(static) if (nt > 1)
      for (int64_t t = 0; t < N; ++t) P[t] = Z[t] + bb * P[t]; /* VecAYPX */
    }
    dpiold = dpi;
    op_apply(n, h, P, W, o->op_kind, nt); /* KSP_MatMult -> mfmult */
    dpi = vdot(N, P, W, nt);
    if (!isfinite(dpi)) { reason = KSP_DIVERGED_NANORINF; break; } /* KSPCheckDot */
    betaold = beta;
    if (dpi == 0.0 || (i > 0 && ((dpi > 0) - (dpi < 0)) * ((dpiold > 0) - (dpiold < 0)) < 0)) {
      reason = KSP_DIVERGED_INDEFINITE_MAT;
      break;
    }
    double a = beta / dpi;
#pragma omp parallel for num_threads(nt) schedule(static) if (nt > 1)
    for (int64_t t = 0; t < N; ++t) {
      x[t] = x[t] + a * P[t];
      R[t] = R[t] + (-a) * W[t];
    }
    pc_apply_any(n, h, o, R, Z, dinv, nt);
    dp = sqrt(vdot(N, Z, Z, nt));
    history[i + 1] = dp;
    nlog = i + 2;
    if (dp != dp || isinf(dp)) { reason = KSP_DIVERGED_NANORINF; break; }
    if (dp <= ttol) { reason = dp < o->atol ? KSP_CONVERGED_ATOL : KSP_CONVERGED_RTOL; break; }
    if (dp >= o->dtol * rnorm0) { reason = KSP_DIVERGED_DTOL; break; }
    beta = vdot(N, Z, R, nt);
    if (!isfinite(beta)) { reason = KSP_DIVERGED_NANORINF; break; } /* KSPCheckDot */
    i++;
  } while (i < o->max_it);
  if (i >= o->max_it) reason = KSP_DIVERGED_ITS;
done:
  *its_out = its;
  if (nlog_out) *nlog_out = nlog;
  free(R); free(Z); free(P); free(W);
  return reason;
}

/* The CPU-baseline workload: `iters` CG iterations (same per-iteration work as pbo_cg_solve:
 * MatMult, 2 dots, 1 norm, 1 sum, AXPY x2, PC, shift, AYPX), no stopping test. */
double pbo_cg_fixed(const int64_t n[3], const double h[3], int64_t iters, int nthreads,
                    const double* b, double* x, double* work) {
  const int64_t N = n[0] * n[1] * n[2];
  const int nt = nthreads > 0 ? nthreads : 1;
  double *R = work, *Z = work + N, *P = work + 2 * N, *W = work + 3 * N;
  const double dinv = 1.0 / pbo_diag(h);
  memset(x, 0, sizeof(double) * N);
  memcpy(R, b, sizeof(double) * N);
  pc_apply(N, R, Z, dinv, 1, 1, nt);
  double dp = sqrt(vdot(N, Z, Z, nt)), beta = vdot(N, Z, R, nt), betaold = 1.0;
  for (int64_t i = 0; i < iters; ++i) {
    double bb = i == 0 ? 0.0 : beta / betaold;
#pragma omp parallel for num_threads(nt) schedule(static) if (nt > 1)
    for (int64_t t = 0; t < N; ++t) P[t] = Z[t] + bb * (i == 0 ? 0.0 : P[t]);
    pbo_stencil_apply7(n, h, P, W, nt);
    double dpi = vdot(N, P, W, nt);
    betaold = beta;
    double a = beta / dpi;
#pragma omp parallel for num_threads(nt) schedule(static) if (nt > 1)
    for (int64_t t = 0; t < N; ++t) {
      x[t] = x[t] + a * P[t];
      R[t] = R[t] + (-a) * W[t];
    }
    pc_apply(N, R, Z, dinv, 1, 1, nt);
    dp = sqrt(vdot(N, Z, Z, nt));
    beta = vdot(N, Z, R, nt);
  }
  return dp;
}

/* ---------------------------------------------------------------------------------------------
 * Tridiagonal solvers (src/tridsol.f90)
 * ------------------------------------------------------------------------------------------- */

/* src/tridsol.f90:76-96 fwd_sweep */
void pbo_fwd_sweep(int64_t n, const double* a, double* b, const double* c, double* d) {
  for (int64_t i = 1; i < n; ++i) {
    double w = a[i] / b[i - 1];
    b[i] = b[i] - w * c[i - 1];
    d[i] = d[i] - w * d[i - 1];
  }
}

/* src/tridsol.f90:98-115 bwd_sweep */
void pbo_bwd_sweep(int64_t n, const double* b, const double* c, double* d) {
  d[n - 1] = d[n - 1] / b[n - 1];
  for (int64_t i = n - 2; i >= 0; --i) d[i] = (d[i] - c[i] * d[i + 1]) / b[i];
}

/* src/tridsol.f90:22-32 tdma: b (diagonal) and d (rhs -> solution) are overwritten */
void pbo_tdma(int64_t n, const double* a, double* b, const double* c, double* d) {
  pbo_fwd_sweep(n, a, b, c, d);
  pbo_bwd_sweep(n, b, c, d);
}

/* src/tridsol.f90:34-74 tdma_periodic (Sherman-Morrison); a(1) couples x(n), c(n) couples x(1).
 * b is left unchanged (the routine works on copies bmod), d is overwritten with the solution. */
void pbo_tdma_periodic(int64_t n, const double* a, double* b, const double* c, double* d) {
  double* bmod = (double*)malloc(sizeof(double) * n);
  double* u = (double*)malloc(sizeof(double) * n);
  const double gamma = -b[0];                                   /* :51 */
  memcpy(bmod, b, sizeof(double) * n);                          /* :54-56 */
  bmod[0] = bmod[0] - gamma;
  bmod[n - 1] = bmod[n - 1] - c[n - 1] * a[0] / gamma;
  pbo_tdma(n, a, bmod, c, d);                                   /* :57 */
  memcpy(bmod, b, sizeof(double) * n);                          /* :59-61 */
  bmod[0] = bmod[0] - gamma;
  bmod[n - 1] = bmod[n - 1] - c[n - 1] * a[0] / gamma;
  for (int64_t i = 0; i < n; ++i) u[i] = 0.0;                   /* :62-65 */
  u[0] = gamma;
  u[n - 1] = c[n - 1];
  pbo_tdma(n, a, bmod, c, u);                                   /* :66 */
  const double num = d[0] + (a[0] / gamma) * d[n - 1];          /* :69-70 */
  const double den = 1.0 + (u[0] + (a[0] / gamma) * u[n - 1]);
  for (int64_t i = 0; i < n; ++i) d[i] = d[i] - (u[i] * num) / den;
  free(bmod);
  free(u);
}

/* ---------------------------------------------------------------------------------------------
 * Compact schemes (src/compact_schemes.f90)
 * ------------------------------------------------------------------------------------------- */

/* src/compact_schemes.f90:332-372 eval_1d_rhs. The reference special-cases the first/last rows;
 * every special case is the interior formula with periodic index wrap, restated here as such:
 *   stagger -1: rhs(i) = a*(f(i)   + s*f(i-1)) + b*(f(i+1) + s*f(i-2))
 *   stagger +1: rhs(i) = a*(f(i+1) + s*f(i))   + b*(f(i+2) + s*f(i-1))      (needs n >= 3) */
void pbo_eval_1d_rhs(double a, double b, int opsign, int stagger, int64_t n, const double* f,
                     double* rhs) {
  const double s = (double)opsign;
  const int64_t sh = stagger == -1 ? 0 : 1;
  for (int64_t i = 0; i < n; ++i) {
    double f0 = f[wrap(i + sh, n)], fm1 = f[wrap(i - 1 + sh, n)];
    double f1 = f[wrap(i + 1 + sh, n)], fm2 = f[wrap(i - 2 + sh, n)];
    rhs[i] = a * (f0 + s * fm1) + b * (f1 + s * fm2);
  }
}

/* (alpha, 1, alpha) periodic solve as grad_1d/interp_1d set it up (:200-205 / :315-320) */
static void solve_alpha(int64_t n, double alpha, double* rhs) {
  double* ld = (double*)malloc(sizeof(double) * n);
  double* d = (double*)malloc(sizeof(double) * n);
  double* ud = (double*)malloc(sizeof(double) * n);
  for (int64_t i = 0; i < n; ++i) { ld[i] = alpha; d[i] = 1.0; ud[i] = alpha; }
  pbo_tdma_periodic(n, ld, d, ud, rhs);
  free(ld); free(d); free(ud);
}

/* src/compact_schemes.f90:155-204 grad_1d (stagger -1 cell->vertex; +1 = div_1d :260-268) */
void pbo_grad_1d(int64_t n, const double* f, double dx, double* df, int stagger) {
  const double a = 63.0 / 62.0 / dx;                 /* :188 */
  const double b = 17.0 / 62.0 / (3.0 * dx);         /* :189 */
  const double alpha = 9.0 / 62.0;                   /* :190 */
  pbo_eval_1d_rhs(a, b, -1, stagger, n, f, df);      /* :194 */
  solve_alpha(n, alpha, df);                         /* :197 */
}

/* src/compact_schemes.f90:271-319 interp_1d (stagger +1 = interp_1d_div :322-329) */
void pbo_interp_1d(int64_t n, const double* f, double* fi, int stagger) {
  const double a = 0.75, b = 1.0 / 20.0, alpha = 3.0 / 10.0; /* :303-305 */
  pbo_eval_1d_rhs(a, b, +1, stagger, n, f, fi);               /* :309 */
  solve_alpha(n, alpha, fi);                                  /* :312 */
}

/* Apply a 1-D line operator along direction `dir` of an nx*ny*nz field. */
typedef enum { L_INTERP, L_GRAD } line_kind;
static void line_op(const int64_t n[3], int dir, line_kind kind, int stagger, double dx,
                    const double* in, double* out) {
  const int64_t nx = n[0], ny = n[1], nz = n[2];
  const int64_t len = n[dir];
  const int64_t stride = dir == 0 ? 1 : (dir == 1 ? nx : nx * ny);
  const int64_t nlines = (nx * ny * nz) / len;
  double* f = (double*)malloc(sizeof(double) * len);
  double* g = (double*)malloc(sizeof(double) * len);
  for (int64_t l = 0; l < nlines; ++l) {
    int64_t base;
    if (dir == 0) base = l * nx;                                  /* l = j + ny*k */
    else if (dir == 1) base = (l % nx) + (l / nx) * nx * ny;      /* l = i + nx*k */
    else base = l;                                                /* l = i + nx*j */
    for (int64_t t = 0; t < len; ++t) f[t] = in[base + t * stride];
    if (kind == L_INTERP) pbo_interp_1d(len, f, g, stagger);
    else pbo_grad_1d(len, f, dx, g, stagger);
    for (int64_t t = 0; t < len; ++t) out[base + t * stride] = g[t];
  }
  free(f);
  free(g);
}

/* src/compact_schemes.f90:42-88 grad: Z (interp, copy, grad) -> Y -> X */
void pbo_grad(const int64_t n[3], const double* f, const double dx[3], double* df) {
  const int64_t N = n[0] * n[1] * n[2];
  double* dff = (double*)malloc(sizeof(double) * N * 3);
  double* dfe = (double*)malloc(sizeof(double) * N * 3);
  line_op(n, 2, L_INTERP, -1, 0.0, f, dff);                /* :61 */
  memcpy(dff + N, dff, sizeof(double) * N);                /* :62 */
  line_op(n, 2, L_GRAD, -1, dx[2], f, dff + 2 * N);        /* :63 */
  line_op(n, 1, L_INTERP, -1, 0.0, dff, dfe);              /* :71 */
  line_op(n, 1, L_GRAD, -1, dx[1], dff + N, dfe + N);      /* :72 */
  line_op(n, 1, L_INTERP, -1, 0.0, dff + 2 * N, dfe + 2 * N); /* :73 */
  line_op(n, 0, L_GRAD, -1, dx[0], dfe, df);               /* :81 */
  line_op(n, 0, L_INTERP, -1, 0.0, dfe + N, df + N);       /* :82 */
  line_op(n, 0, L_INTERP, -1, 0.0, dfe + 2 * N, df + 2 * N); /* :83 */
  free(dff);
  free(dfe);
}

/* src/compact_schemes.f90:93-142 interp (Z -> Y -> X with the given stagger) */
void pbo_interp(const int64_t n[3], const double* f, double* fi, int stagger) {
  const int64_t N = n[0] * n[1] * n[2];
  double* ff = (double*)malloc(sizeof(double) * N);
  double* fe = (double*)malloc(sizeof(double) * N);
  line_op(n, 2, L_INTERP, stagger, 0.0, f, ff);
  line_op(n, 1, L_INTERP, stagger, 0.0, ff, fe);
  line_op(n, 0, L_INTERP, stagger, 0.0, fe, fi);
  free(ff);
  free(fe);
}

/* src/compact_schemes.f90:207-257 div: X -> Y -> Z, Z step interpolates dff1 + dff2 (:249) */
void pbo_div(const int64_t n[3], const double* f, const double dx[3], double* df) {
  const int64_t N = n[0] * n[1] * n[2];
  double* dfe = (double*)malloc(sizeof(double) * N * 3);
  double* dff = (double*)malloc(sizeof(double) * N * 3);
  double* dfc = (double*)malloc(sizeof(double) * N);
  line_op(n, 0, L_GRAD, +1, dx[0], f, dfe);                  /* :227 */
  line_op(n, 0, L_INTERP, +1, 0.0, f + N, dfe + N);          /* :228 */
  line_op(n, 0, L_INTERP, +1, 0.0, f + 2 * N, dfe + 2 * N);  /* :229 */
  line_op(n, 1, L_INTERP, +1, 0.0, dfe, dff);                /* :237 */
  line_op(n, 1, L_GRAD, +1, dx[1], dfe + N, dff + N);        /* :238 */
  line_op(n, 1, L_INTERP, +1, 0.0, dfe + 2 * N, dff + 2 * N); /* :239 */
  for (int64_t t = 0; t < N; ++t) dfe[t] = dff[t] + dff[N + t];
  line_op(n, 2, L_INTERP, +1, 0.0, dfe, dfc);                /* :248 */
  line_op(n, 2, L_GRAD, +1, dx[2], dff + 2 * N, df);         /* :249 */
  for (int64_t t = 0; t < N; ++t) df[t] = df[t] + dfc[t];    /* :250 */
  free(dfe);
  free(dff);
  free(dfc);
}

/* src/compact_schemes.f90:17-37 lapl = div(grad f) */
void pbo_lapl(const int64_t n[3], const double* f, const double dx[3], double* out) {
  const int64_t N = n[0] * n[1] * n[2];
  double* df = (double*)malloc(sizeof(double) * N * 3);
  pbo_grad(n, f, dx, df);
  pbo_div(n, df, dx, out);
  free(df);
}
