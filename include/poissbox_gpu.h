/* poissbox_gpu.h -- C ABI of the MI355X-native poissbox KSPSolve hot path.
 *
 * Drop-in boundary for 3decomp/poissbox (reference @ /root/reference). The reference is Fortran
 * driving PETSc; each entry point below names the reference interface it replaces. Callers bind
 * it from Fortran through iso_c_binding (poissbox_amd/fortran/poissbox_gpu.f90) or from Python
 * through ctypes (poissbox_amd/api.py). Plain pointers, sizes and opaque handles only.
 *
 * Conventions
 *  - Every function returns int: 0 = PB_OK, > 0 = PB_ERR_*; pb_last_error() describes the last
 *    failure of the calling thread. The reference never checks ierr; we always return it.
 *    Solver divergence is a KSP reason code in pb_ksp_result, not an error.
 *  - Layout: Fortran column-major (i,j,k), i fastest == C [k][j][i]; fp64 everywhere
 *    (src/constants.f90:15 pb_dp). Each rank owns a z-slab of whole planes, with the remainder
 *    planes on the low ranks; the rank-contiguous global order therefore equals natural order.
 *  - One process per GPU. A context spans one GPU; multi-GPU runs create one context per rank
 *    and connect them with RCCL (pb_comm_unique_id + pb_ctx_create). Every "vector" call is
 *    collective over the ranks of the context, exactly like PETSc calls on PETSC_COMM_WORLD.
 *  - Host buffers are borrowed for the duration of a call. The library owns device memory.
 */
#ifndef POISSBOX_GPU_H
#define POISSBOX_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PB_VERSION_MAJOR 0
#define PB_VERSION_MINOR 2

enum pb_error {
  PB_OK = 0,
  PB_ERR_ARG = 1,         /* invalid argument / shape */
  PB_ERR_HIP = 2,         /* HIP runtime error (device fault, launch failure) */
  PB_ERR_COMM = 3,        /* RCCL / transport error */
  PB_ERR_ALLOC = 4,       /* out of device or host memory */
  PB_ERR_UNSUPPORTED = 5, /* option or configuration not implemented */
  PB_ERR_STATE = 6        /* call out of order */
};

typedef struct pb_ctx pb_ctx;   /* device + rank + communicator + stream          */
typedef struct pb_grid pb_grid; /* DMDA analogue: periodic 3-D grid, z-slab layout */
typedef struct pb_vec pb_vec;   /* DMCreateGlobalVector analogue (owned slab)      */
typedef struct pb_op pb_op;     /* MatShell(MATOP_MULT = mfmult) analogue           */
typedef struct pb_ksp pb_ksp;   /* KSP analogue                                    */

const char* pb_last_error(void);
int pb_version(int* major, int* minor);
/* src/coefficients.f90:22-48: lapl_1d_coeffs (c = [1, -2, 1] / dx^2) and lapl_star_coeffs (the
 * 3x3x3 box, column-major, of the 7-point star) -- the coefficients every operator here uses. */
int pb_lapl_1d_coeffs(double dx, double c[3]);
int pb_lapl_star_coeffs(double dx, double dy, double dz, double c[27]);

/* ---- context / communicator (replaces MPI_Init + PetscInitialize, src/example.f90:43-47) ---- */
/* 128-byte RCCL unique id; rank 0 creates it and the caller broadcasts it (any channel). */
int pb_comm_unique_id(unsigned char uid[128]);
/* nranks == 1: uid may be NULL. nranks > 1: uid from rank 0's pb_comm_unique_id. The RCCL
 * communicator init is bounded by PB_COMM_TIMEOUT_MS: if not every rank joins in time (a peer
 * died during start-up, or holds another id) the call returns PB_ERR_COMM instead of blocking.
 * The init then still runs on a helper thread inside RCCL's start-up handshake (RCCL's blocking
 * init cannot be cancelled; its non-blocking form would make every later RCCL call of the hot
 * path asynchronous): after PB_ERR_COMM from pb_ctx_create the process should exit rather than
 * retry in-process. */
int pb_ctx_create(int device, int rank, int nranks, const unsigned char* uid, pb_ctx** ctx);
/* Test transport: route halo exchange and allreduce through host callbacks instead of RCCL
 * (lets several ranks share one GPU in tests). Must be called before any grid is created.
 * sendrecv: send `send_lo` (first owned plane) to rank-1 and `send_hi` (last owned plane) to
 * rank+1 (periodic), receive the plane below into recv_lo and the plane above into recv_hi.
 * allreduce: in-place SUM of `count` doubles over all ranks. Return 0 on success. */
typedef int (*pb_sendrecv_fn)(void* user, const double* send_lo, const double* send_hi,
                              double* recv_lo, double* recv_hi, int64_t count);
typedef int (*pb_allreduce_fn)(void* user, double* vals, int count);
int pb_ctx_set_host_transport(pb_ctx* ctx, pb_sendrecv_fn sendrecv, pb_allreduce_fn allreduce,
                              void* user);
/* Host all-to-all for the compact operators' z-slab <-> y-slab transposes: send_counts[p]
 * doubles go to rank p (blocks contiguous in rank order in `send`), recv_counts[p] arrive from
 * rank p (contiguous in rank order in `recv`). Needed only for the compact operator on a split
 * grid with the host transport; RCCL contexts use grouped ncclSend/ncclRecv. */
typedef int (*pb_alltoallv_fn)(void* user, const double* send, const int64_t* send_counts,
                               double* recv, const int64_t* recv_counts);
int pb_ctx_set_host_alltoallv(pb_ctx* ctx, pb_alltoallv_fn alltoallv, void* user);
int pb_ctx_get_rank(const pb_ctx* ctx, int* rank, int* nranks);
/* Launcher-agnostic start (≙ MPI_Init + MPI_Comm_rank/size, src/example.f90:43-47): the rank
 * layout comes from RANK/WORLD_SIZE/LOCAL_RANK (torchrun --no-python), OMPI_COMM_WORLD_* (mpirun)
 * or PMI_RANK/PMI_SIZE; one process = rank 0 of 1 on `device` (-1: LOCAL_RANK). Several ranks
 * take GPU LOCAL_RANK mod visible GPUs (PB_DEVICE overrides) and connect over
 *   PB_TRANSPORT=rccl (default when every rank has its own GPU): rank 0's unique id is passed in
 *     a file PB_RENDEZVOUS_DIR/pb_uid_<job> (default /tmp; job = PB_JOB_ID, else MASTER_PORT,
 *     plus torchrun's TORCHELASTIC_RESTART_COUNT), removed once the communicator is up; a file
 *     last written more than PB_RENDEZVOUS_SLACK_S (120) before the reading process started is
 *     taken for a crashed run's leftover and ignored, with a line on stderr -- until the reader
 *     itself has waited longer than the slack, when it takes the file (a rank started late; a
 *     stale id then fails the bounded init with PB_ERR_COMM) (likewise the shm segment below);
 *   PB_TRANSPORT=shm (default when ranks outnumber GPUs): a built-in POSIX shared-memory host
 *     transport (halo planes and scalar sums; ranks may share one GPU; no all-to-all, so the
 *     compact operators need RCCL or a host alltoallv callback on a split grid). */
int pb_ctx_create_from_env(int device, pb_ctx** ctx);
/* In-place SUM over all ranks of `count` (<= 32) host doubles (≙ MPI_Allreduce(MPI_SUM) of the
 * reference driver's checks, src/example.f90:108,137-147,194). */
int pb_ctx_allreduce_host(pb_ctx* ctx, double* vals, int count);
int pb_ctx_sync(pb_ctx* ctx);  /* stream synchronize (≙ MPI_Barrier for device work) */
int pb_ctx_barrier(pb_ctx* ctx); /* synchronize + all ranks rendezvous */
/* Failure handling on multi-rank contexts (the reference's MPI calls would hang or abort): every
 * host wait is bounded by PB_COMM_TIMEOUT_MS (default 180000) and checks RCCL's asynchronous
 * error; a timeout, an RCCL error or a failing host-transport callback aborts the communicator
 * (ncclCommAbort) and returns PB_ERR_COMM, and every later communicating call on the context
 * returns PB_ERR_COMM at once. *failed = 1 after such a failure. */
int pb_ctx_comm_status(const pb_ctx* ctx, int* failed);
/* What the context communicates over (≙ MPI_Comm_size of PETSC_COMM_WORLD as the transport
 * itself sees it): PB_TRANSPORT_RCCL with the communicator's own ncclCommCount /
 * ncclCommUserRank, PB_TRANSPORT_HOST (host callbacks or the shm transport) with the context's
 * rank layout, or PB_TRANSPORT_NONE (one rank, wrap planes in place) with 1 / 0. */
enum pb_transport { PB_TRANSPORT_NONE = 0, PB_TRANSPORT_RCCL = 1, PB_TRANSPORT_HOST = 2 };
int pb_ctx_comm_info(const pb_ctx* ctx, int* transport, int* comm_nranks, int* comm_rank);
int pb_ctx_destroy(pb_ctx* ctx);
/* Per-kernel timing with HIP events on the context's stream (off by default). */
int pb_ctx_set_timing(pb_ctx* ctx, int enable);
/* Timing restricted to the comma-separated phase names in `only` (NULL or "": every phase), and
 * to one launch in `every` of each such phase: a timed region keeps its event records off the
 * other launches (bench.py times its roofline kernel inside the timed steps this way). */
int pb_ctx_set_timing_filter(pb_ctx* ctx, int enable, const char* only, int every);
/* name: "stencil", "cg_pass_a", "cg_pass_b", ...; returns total ms and launch count since reset */
int pb_ctx_get_timing(pb_ctx* ctx, const char* name, double* total_ms, int64_t* count);
/* The per-launch durations behind pb_ctx_get_timing (the first 65536 since the last reset):
 * copies min(cap, *count) of them into ms; *count = how many there are. Lets a caller tell the
 * launches that ran from those that exited at entry (a converged solve's enqueued-ahead work). */
int pb_ctx_get_timing_samples(pb_ctx* ctx, const char* name, float* ms, int64_t cap,
                              int64_t* count);
int pb_ctx_reset_timing(pb_ctx* ctx);
/* HBM calibration of this process's device (no reference counterpart; bench.py reports it beside
 * the matvec's rate): a flat fp64 copy of n doubles -- 16-B loads, non-temporal 16-B stores, the
 * standalone matvec's access mix without its stencil -- `reps` timed launches after two warm-ups;
 * GB/s counted as 16 B per element. Allocates and frees its own 2 x n doubles. */
int pb_ctx_copy_probe(pb_ctx* ctx, int64_t n, int reps, double* best_gbps, double* median_gbps);
/* The same copy from x into y (both of one grid; y is overwritten): the matvec's own buffers,
 * so a placement-dependent rate shows up beside the matvec x -> y. */
int pb_vec_copy_probe(const pb_vec* x, pb_vec* y, int reps, double* best_gbps,
                      double* median_gbps);

/* ---- tuning (kernel selection and launch shapes; no reference counterpart) ----
 * Process-wide table of the launchers' parameters (INTEGRATION.md lists the names: z-march
 * alternation, tile heights, multigrid kernel thresholds, spectral-PC tile shapes, ...). Unset
 * names take the measured defaults; every setting selects kernels that give the same results to
 * the bits (or, for tile heights, to the reduction order of the CG sums), so it is a speed knob,
 * never a correctness one. The library reads no such setting from the environment. Unknown names
 * return PB_ERR_ARG. Set before the calls it should affect; not thread-safe against running calls. */
int pb_tune_set(const char* name, int value);
int pb_tune_get(const char* name, int* value, int* is_set);
int pb_tune_reset(void);

/* ---- slab partition (replaces DMDACreate3d's PETSC_DECIDE split, src/poissbox.f90:191-202) ---- */
/* Pure host function: remainder planes go to the low ranks (README.md:30-32's 22/21/21). */
int pb_slab_partition(int64_t nz, int nranks, int rank, int64_t* kstart, int64_t* nk);

/* ---- grid (replaces initialise_grid, src/poissbox.f90:183-204) ---- */
/* Periodic in x, y, z; spacing h = L/n (src/example.f90:33-35). n >= 3 in every direction. */
int pb_grid_create(pb_ctx* ctx, const int64_t n[3], const double L[3], pb_grid** grid);
/* ≙ DMDAGetCorners (src/poissbox.f90:107): 0-based start and owned size of this rank */
int pb_grid_get_corners(const pb_grid* grid, int64_t start[3], int64_t size[3]);
int pb_grid_get_info(const pb_grid* grid, int64_t n[3], double h[3], int64_t* nlocal);
int pb_grid_destroy(pb_grid* grid);

/* ---- vectors (replace DMCreateGlobalVector/VecDuplicate/VecSet/VecCopy/VecAXPY/VecAYPX/
 *      VecScale/VecDot/VecNorm/VecSum/DMDAVecGetArrayF90, src/example.f90:79-83,175-195,217-231) */
int pb_vec_create(pb_grid* grid, pb_vec** v);
int pb_vec_duplicate(const pb_vec* v, pb_vec** out);
int pb_vec_destroy(pb_vec* v);
int pb_vec_set(pb_vec* v, double alpha);
int pb_vec_copy(const pb_vec* src, pb_vec* dst);
int pb_vec_axpy(pb_vec* y, double alpha, const pb_vec* x);  /* y = y + alpha*x */
int pb_vec_aypx(pb_vec* y, double beta, const pb_vec* x);   /* y = x + beta*y  */
int pb_vec_scale(pb_vec* v, double alpha);
int pb_vec_dot(const pb_vec* x, const pb_vec* y, double* out); /* global sum x.y   */
int pb_vec_norm2(const pb_vec* v, double* out);              /* global ||v||_2    */
int pb_vec_sum(const pb_vec* v, double* out);                /* global sum v      */
/* Owned values in natural (i fastest) order of this rank's slab; count = nlocal. */
int pb_vec_set_values_host(pb_vec* v, const double* owned);
int pb_vec_get_values_host(const pb_vec* v, double* owned);
/* Synthetic input: v[g] = 2*(0.5 - U), U = SplitMix64(seed ^ g) >> 11 * 2^-53,
 * g = global linear index; decomposition independent (src/example.f90:180-181 distribution). */
int pb_vec_set_random(pb_vec* v, uint64_t seed);
/* Borrowed device pointer to the owned slab (≙ DMDAVecGetArrayF90 on device memory). */
int pb_vec_device_ptr(pb_vec* v, double** dptr, int64_t* nlocal);

/* ---- operator (replaces MatCreateShell + MatShellSetOperation(MATOP_MULT, mfmult),
 *      src/poissbox.f90:242-267, and mfmult itself, :300-322) ---- */
enum pb_op_kind {
  PB_OP_STAR7 = 0,       /* 2nd-order 7-point star, compute_lapl_pointwise (:84-148)        */
  PB_OP_COMPACT = 1,     /* 6th-order compact lapl = div(grad f), compact_schemes.f90:17-37  */
  PB_OP_ASSEMBLED27 = 2  /* assembled BOX AIJ P (coefficients.f90:50-113), 27-entry rows     */
};
/* PB_OP_ASSEMBLED27 applies P x with PETSc's AIJ row sums: stored columns ascending on one rank
 * (MatMult_SeqAIJ), owned columns then off-rank columns on several (MatMult_MPIAIJ) -- so rows on
 * the periodic seams and slab boundaries differ from PB_OP_STAR7 at rounding level, and
 * src/example.f90:235-261's ||A x - P x|| is the reference's rounding-level value, not 0. As a
 * KSP operator (A = P, src/example.f90:62-64) it runs the unfused CG iteration. */
int pb_op_create(pb_grid* grid, int kind, const double deltas[3], pb_op** op);
int pb_op_apply(pb_op* op, const pb_vec* x, pb_vec* y); /* ≙ MatMult(A, x, y) */
/* ≙ assemble_laplacian(da, dx, dy, dz, M) (src/coefficients.f90:50-113): (re)set the spacings
 * the operator's coefficients are built from (lapl_star_coeffs). */
int pb_op_set_deltas(pb_op* op, const double deltas[3]);
int pb_op_get_diagonal(const pb_op* op, double* diag);  /* constant diagonal of the 7-pt P */
int pb_op_destroy(pb_op* op);
/* ≙ MatGetOwnershipRange / VecGetOwnershipRange (src/example.f90:137-147): global row range
 * [first, next) owned by this rank (rank-contiguous natural order of the z-slab split). */
int pb_op_get_ownership_range(const pb_op* op, int64_t* first, int64_t* next);
int pb_vec_get_ownership_range(const pb_vec* v, int64_t* first, int64_t* next);

/* ---- KSP (replaces solve(P, A, x, b), src/poissbox.f90:269-298 -> KSPSolve) ---- */
enum pb_ksp_type { PB_KSP_CG = 0 };
/* PB_PC_FFT (-pc_type fft): z = P^+ r by separable Hartley transforms with P's symbol (the compact
 * operator's when P is PB_OP_COMPACT, else the 7-point star's); periodic, power-of-two extents in
 * 64..1024. Not in the reference: the spectrally exact PC for config 5. */
enum pb_pc_type { PB_PC_NONE = 0, PB_PC_JACOBI = 1, PB_PC_SOR = 2, PB_PC_MG = 3, PB_PC_FFT = 4 };
/* PETSc KSPConvergedReason values */
enum pb_ksp_reason {
  PB_KSP_ITERATING = 0, PB_KSP_CONVERGED_RTOL = 2, PB_KSP_CONVERGED_ATOL = 3,
  PB_KSP_CONVERGED_ITS = 4, PB_KSP_DIVERGED_ITS = -3, PB_KSP_DIVERGED_DTOL = -4,
  PB_KSP_DIVERGED_INDEFINITE_PC = -8, PB_KSP_DIVERGED_NANORINF = -9,
  PB_KSP_DIVERGED_INDEFINITE_MAT = -10
};
typedef struct {
  double rtol;       /* -ksp_rtol   (PETSc default 1e-5)  */
  double atol;       /* -ksp_atol   (1e-50)               */
  double dtol;       /* -ksp_divtol (1e5)                 */
  int64_t max_it;    /* -ksp_max_it (10000)               */
  int ksp_type;      /* -ksp_type cg                      */
  int pc_type;       /* -pc_type none|jacobi|sor|mg       */
  int nullspace;     /* constant null space (src/poissbox.f90:285-291), default 1 */
  int monitor;       /* -ksp_monitor: print ||z_k|| per iteration after the solve (rank 0) */
  int converged_reason; /* -ksp_converged_reason */
  int check_every;   /* host polls the device convergence flag every N iterations (default 8) */
  int mg_levels;     /* -pc_mg_levels: multigrid levels (0 = as many as the grid allows)      */
  int mg_coarse_its; /* -pc_mg_coarse_its: symmetric red-black sweeps on the coarsest level (8) */
  double sor_omega;  /* -pc_sor_omega: SOR relaxation factor (1.0 = Gauss-Seidel)              */
  int cg_single_reduction; /* -ksp_cg_single_reduction (PETSc KSPCGUseSingleReduction): the
                        iteration of KSPSolve_CG_SingleReduction -- one reduction per iteration
                        (z'z, z'r, z'Az together), p'w by its recurrence. Equal to KSPSolve_CG in
                        exact arithmetic. Runs as two engine passes on the 7-point operator with
                        -pc_type jacobi|none; with other operators / PCs the KSPSolve_CG iteration
                        runs (default 0) */
} pb_ksp_opts;
typedef struct {
  int reason;
  int64_t its;
  double rnorm;      /* last ||z||_2 (KSP_NORM_PRECONDITIONED) */
  double rnorm0;
  int64_t nhist;     /* residual norms logged (≙ KSPGetResidualHistory's count): its + 1, or its
                        after a breakdown exit (beta = 0, indefinite PC / matrix) */
} pb_ksp_result;
int pb_ksp_opts_default(pb_ksp_opts* opts);
/* Parses PETSc-style options (-ksp_type, -pc_type, -ksp_rtol, -ksp_atol, -ksp_divtol,
 * -ksp_max_it, -ksp_monitor, -ksp_converged_reason, -pc_mg_levels, -pc_mg_coarse_its,
 * -pc_sor_omega, -ksp_cg_single_reduction [true|false]); unknown options are ignored.
 * -pc_type sor: one symmetric red-black SOR sweep (PETSc PCSOR default: 1 local symmetric sweep,
 * here in red-black order). -pc_type mg (or gamg): geometric V(1,1) multigrid with red-black SOR
 * smoothing on the 7-point P (README.md:40-45 recommends GAMG + SOR). Both need even extents. */
int pb_ksp_opts_parse(pb_ksp_opts* opts, int argc, const char* const* argv);

/* KSPCreate + KSPSetOperators(ksp, A, P) + options. P supplies the Jacobi diagonal. */
int pb_ksp_create(pb_op* A, pb_op* P, const pb_ksp_opts* opts, pb_ksp** ksp);
/* KSPSolve(ksp, b, x): x0 = 0 (guess_zero). history (optional, may be NULL): the res->nhist
 * logged norms ||z_k|| (k = 0 .. nhist-1), at most history_cap entries written. */
int pb_ksp_solve(pb_ksp* ksp, const pb_vec* b, pb_vec* x, pb_ksp_result* res, double* history,
                 int64_t history_cap);
/* Split form used by benchmarks: setup (r = b, z, ||z0||), then exactly `iters` iterations
 * (continuing from the current state; stopping test applies unless disabled by options). */
int pb_ksp_begin(pb_ksp* ksp, const pb_vec* b, pb_vec* x);
int pb_ksp_iterate(pb_ksp* ksp, int64_t iters);
int pb_ksp_end(pb_ksp* ksp, pb_ksp_result* res, double* history, int64_t history_cap);
int pb_ksp_destroy(pb_ksp* ksp);
/* PCApply(KSPGetPC(ksp), r, z): z = M^-1 r of the configured preconditioner (Jacobi: D^-1 r;
 * SOR / MG: from a zero initial guess), without the null-space removal KSP adds. */
int pb_ksp_pc_apply(pb_ksp* ksp, const pb_vec* r, pb_vec* z);
/* number of multigrid levels in use (1 for SOR, 0 for Jacobi / none) */
int pb_ksp_pc_levels(const pb_ksp* ksp, int* levels);
/* One-shot convenience: ≙ solve(P, A, x, b). */
int pb_solve(pb_op* A, pb_op* P, const pb_ksp_opts* opts, const pb_vec* b, pb_vec* x,
             pb_ksp_result* res, double* history, int64_t history_cap);

/* ---- tridiagonal (replaces tdma / tdma_periodic / fwd_sweep / bwd_sweep, src/tridsol.f90) ----
 * Batched over `nbatch` independent lines. Element e of line l sits at
 *   ptr[l * line_stride + e * elem_stride]        (device pointers).
 * Argument order follows the reference code: a = sub-diagonal, b = diagonal, c = super-diagonal,
 * d = rhs -> solution. tdma overwrites b and d (like the reference); tdma_periodic leaves b
 * unchanged. periodic: a[0] couples x[n-1], c[n-1] couples x[0] (src/tridsol.f90:34-74). */
int pb_tdma_batched(pb_ctx* ctx, int64_t n, int64_t nbatch, int64_t line_stride,
                    int64_t elem_stride, const double* a, double* b, const double* c, double* d,
                    int periodic);
/* fwd_sweep (which = 1: a, b, c, d -> modified b, d) or bwd_sweep (which = 2: b, c, d -> x in d;
 * a unused) alone, src/tridsol.f90:76-115 (exported by the reference for its tests). */
int pb_tdma_sweeps_batched(pb_ctx* ctx, int64_t n, int64_t nbatch, int64_t line_stride,
                           int64_t elem_stride, const double* a, double* b, const double* c,
                           double* d, int which);
/* Constant-coefficient periodic (alpha, 1, alpha) systems -- the compact-scheme solves
 * (src/compact_schemes.f90:197,312) -- by parallel cyclic reduction, in place on d. */
int pb_pcr_alpha_batched(pb_ctx* ctx, int64_t n, int64_t nbatch, int64_t line_stride,
                         int64_t elem_stride, double alpha, double* d);

/* ---- compact schemes (replace src/compact_schemes.f90:9-13 public API) ----
 * 3-D fields on the grid; grad/div take 3-component vectors as three pb_vec. stagger: -1
 * cell->vertex, +1 vertex->cell. Reference operation order (bit-identical to the reference). On a
 * split grid the Z steps run on y-slabs with complete z-lines (all-to-all transposes, as
 * pb_compact_lapl_fast), so every rank's result is bit-identical to the single-domain one. */
int pb_compact_grad(pb_grid* grid, const double dx[3], const pb_vec* f, pb_vec* const df[3]);
int pb_compact_div(pb_grid* grid, const double dx[3], const pb_vec* const f[3], pb_vec* df);
int pb_compact_interp(pb_grid* grid, int stagger, const pb_vec* f, pb_vec* fi);
int pb_compact_lapl(pb_grid* grid, const double dx[3], const pb_vec* f, pb_vec* out);
/* Same operator by the 3-pass factorisation lapl = Lx Jy Jz + Jx Ly Jz + Jx Jy Lz (SURVEY.md
 * App. D) with PCR line solves in LDS: ~80 B/DoF instead of 16 line-solve families; agrees with
 * pb_compact_lapl to rounding. This is what PB_OP_COMPACT applies inside CG. */
int pb_compact_lapl_fast(pb_grid* grid, const double dx[3], const pb_vec* f, pb_vec* out);
/* 1-D line operators on device arrays, batched like pb_tdma_batched (grad_1d/div_1d/interp_1d/
 * interp_1d_div: kind 0 = derivative, 1 = interpolation). */
int pb_compact_1d_batched(pb_ctx* ctx, int kind, int stagger, double dx, int64_t n,
                          int64_t nbatch, int64_t line_stride, int64_t elem_stride,
                          const double* f, double* out);

/* ---- host-array forms of the module procedures (src/tridsol.f90:16-18, compact_schemes.f90:9-13):
 * the reference works on process-local Fortran arrays, so these take host pointers, stage them
 * through device memory, run the kernels above and copy back (synchronous). The Fortran modules
 * `tridsol` and `compact_schemes` in poissbox_amd/fortran wrap them with the reference's
 * assumed-shape signatures. 3-D fields are whole arrays of shape n (never split, whatever the
 * context); vector fields are (nx, ny, nz, 3) with the component slowest. ---- */
int pb_tdma_batched_host(pb_ctx* ctx, int64_t n, int64_t nbatch, int64_t line_stride,
                         int64_t elem_stride, const double* a, double* b, const double* c,
                         double* d, int periodic);
int pb_tdma_sweeps_batched_host(pb_ctx* ctx, int64_t n, int64_t nbatch, int64_t line_stride,
                                int64_t elem_stride, const double* a, double* b, const double* c,
                                double* d, int which);
int pb_compact_1d_batched_host(pb_ctx* ctx, int kind, int stagger, double dx, int64_t n,
                               int64_t nbatch, int64_t line_stride, int64_t elem_stride,
                               const double* f, double* out);
int pb_compact_grad_host(pb_ctx* ctx, const int64_t n[3], const double dx[3], const double* f,
                         double* df);
int pb_compact_div_host(pb_ctx* ctx, const int64_t n[3], const double dx[3], const double* f,
                        double* df);
int pb_compact_interp_host(pb_ctx* ctx, const int64_t n[3], int stagger, const double* f,
                           double* fi);
int pb_compact_lapl_host(pb_ctx* ctx, const int64_t n[3], const double dx[3], const double* f,
                         double* out);

#ifdef __cplusplus
}
#endif
#endif /* POISSBOX_GPU_H */
