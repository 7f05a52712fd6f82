/* pb_oracle.h -- CPU restatement of the poissbox hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This header declares the oracle: a plain-C restatement of the reference algorithms
 * (3decomp/poissbox, Fortran + PETSc) used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the CHECKER. Nothing in poissbox_amd/ links or calls it.
 *
 * Layout everywhere: Fortran column-major (i,j,k), i fastest == C [k][j][i].
 * Vector fields of 3 components (grad output): [c][k][j][i], c slowest (Fortran df(nx,ny,nz,3)).
 *
 * Parity pins: tridiagonal + compact-scheme functions are pinned bit-for-bit against the
 * flang-built reference (oracle/_ref, fixtures in tests/golden/). The 7-point operator is pinned
 * by the reference's own known-answer tests (tests/coefficients/test_star.f90) -- the
 * PETSc-dependent sources (poissbox.f90, coefficients.f90) cannot be compiled here. The
 * KSPCG + PCJacobi + MatNullSpace restatement (PETSc is external and absent) is
 * "parity unpinned" against real PETSc: it follows SURVEY.md Appendix A.
 */
#ifndef PB_ORACLE_H
#define PB_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- coefficients (src/coefficients.f90) ---- */
void pbo_lapl_1d_coeffs(double dx, double c[3]);
void pbo_lapl_star_coeffs(double dx, double dy, double dz, double c[27]);

/* ---- 7-point operator (src/poissbox.f90:84-148) ---- */
/* faithful: 27-term dot product over the 3x3x3 box incl. zero coefficients, column-major order */
void pbo_stencil_apply27(const int64_t n[3], const double h[3], const double* x, double* y);
/* fast: the 7 non-zero terms in the same order (z-, y-, x-, c, x+, y+, z+); identical results
 * for finite inputs */
void pbo_stencil_apply7(const int64_t n[3], const double h[3], const double* x, double* y,
                        int nthreads);
/* one z-slab (n[2] = owned planes) with explicit ghost planes below/above */
void pbo_stencil_slab(const int64_t n[3], const double h[3], const double* x, const double* glo,
                      const double* ghi, double* y);
/* assembled P (src/coefficients.f90:50-113) applied as a 27-point BOX SpMV, row-wise sum over
 * the 27 stored entries in MatSetValuesStencil column order */
void pbo_assembled_apply(const int64_t n[3], const double h[3], int nranks, const double* x,
                         double* y);
double pbo_diag(const double h[3]);

/* ---- synthetic input ---- */
uint64_t pbo_splitmix64(uint64_t z);
/* x[g] = 2*(0.5 - U(seed ^ (g0+g))), g = global linear index i + nx*(j + ny*k) */
void pbo_fill_random(int64_t count, uint64_t seed, int64_t g0, double* x);

/* ---- KSPCG + PCJacobi + constant null space (PETSc cg.c semantics) ---- */
typedef struct {
  double rtol, atol, dtol;
  int64_t max_it;
  int pc_type;       /* 0 = none, 1 = jacobi */
  int nullspace;     /* 1 = remove constant mode after every PCApply */
  int op_kind;       /* 0 = 7-term stencil, 1 = faithful 27-term (slow), 2 = compact lapl,
                        3 + (R-1) = assembled P (AIJ MatMult order on R z-slabs) */
  int nthreads;      /* OpenMP threads for the 7-term operator/vector ops (1 = serial sums) */
  int mg_levels;     /* pc 3: multigrid levels (0 = automatic), pc 2 = one symmetric RB-SOR sweep */
  int mg_coarse_its; /* symmetric red-black sweeps on the coarsest level */
  double omega;      /* SOR relaxation */
  int nranks;        /* slab count the GPU run uses (only changes the automatic level count) */
  int pc_compact;    /* pc 4 (fft): invert the compact operator's symbol (P = compact), else the
                        7-point star's */
  int single_reduction; /* -ksp_cg_single_reduction: 1 = PETSc KSPSolve_CG_SingleReduction
                           (w and p'w by recurrence); 2 = the same iteration with w = A p
                           recomputed each iteration (the GPU kernels' form; equal in exact
                           arithmetic) -- 0 = KSPSolve_CG */
} pbo_ksp_opts;

/* ---- red-black SOR / geometric multigrid preconditioner (our GPU design, poissbox_amd/csrc/
 * pb_mg.hip; the reference's README.md:40-45 recommends PETSc GAMG + SOR, which is absent:
 * parity for this PC is against this restatement, unpinned against PETSc) ---- */
int pbo_mg_plan_levels(const int64_t n[3], int nranks, int levels_req);
/* z = M^-1 r from a zero initial guess; pc_type 2 (SOR) or 3 (MG) */
void pbo_mg_apply(const int64_t n[3], const double h[3], int pc_type, int levels, int coarse_its,
                  double omega, int nranks, const double* r, double* z);

/* spectral preconditioner (our design, poissbox_amd/csrc/pb_fft.hip; not in the reference):
 * z = P^+ r for the periodic operator P (7-point star, or compact lapl when compact != 0), by a
 * naive separable discrete Hartley transform (O(n) per element per axis, cas tables in long
 * double) and the operator's Fourier symbol; 1/lambda := 0 where |lambda| <= 1e-10 * bound. */
void pbo_fft_pc_apply(const int64_t n[3], const double h[3], int compact, const double* r,
                      double* z);

/* Returns PETSc KSPConvergedReason; history[0..nlog) = ||z_k||_2 (capacity max_it+1): the
 * entries KSPLogResidualHistory wrote -- its+1 normally, its after a breakdown exit (beta = 0,
 * indefinite PC / matrix, non-finite p.w), which leaves the last iteration without a norm. */
int pbo_cg_solve(const int64_t n[3], const double h[3], const pbo_ksp_opts* opts, const double* b,
                 double* x, double* history, int64_t* its, int64_t* nlog);
/* Fixed number of iterations (no stopping test) -- the CPU baseline workload. Returns dp. */
double pbo_cg_fixed(const int64_t n[3], const double h[3], int64_t iters, int nthreads,
                    const double* b, double* x, double* work /* 4*N */);

/* ---- tridiagonal (src/tridsol.f90) -- arg order (sub, diag, super, rhs) as the code uses ---- */
void pbo_fwd_sweep(int64_t n, const double* a, double* b, const double* c, double* d);
void pbo_bwd_sweep(int64_t n, const double* b, const double* c, double* d);
void pbo_tdma(int64_t n, const double* a, double* b, const double* c, double* d);
void pbo_tdma_periodic(int64_t n, const double* a, double* b, const double* c, double* d);

/* ---- compact schemes (src/compact_schemes.f90) ---- */
void pbo_eval_1d_rhs(double a, double b, int opsign, int stagger, int64_t n, const double* f,
                     double* rhs);
void pbo_grad_1d(int64_t n, const double* f, double dx, double* df, int stagger);
void pbo_interp_1d(int64_t n, const double* f, double* fi, int stagger);
void pbo_grad(const int64_t n[3], const double* f, const double dx[3], double* df);
void pbo_div(const int64_t n[3], const double* f, const double dx[3], double* df);
void pbo_interp(const int64_t n[3], const double* f, double* fi, int stagger);
void pbo_lapl(const int64_t n[3], const double* f, const double dx[3], double* out);

#ifdef __cplusplus
}
#endif
#endif
