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
  // fused post-smoothing (one rank, large levels): the pre-smoothed x, kept apart from x so that
  // the prolongation + both half-sweeps can read it and write x in one pass
  double* xs = nullptr;
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
  const int* skip = nullptr;  // device flag: when set, the kernels of this apply exit at entry
  // SOR half-sweeps and residuals of levels whose planes hold >= engine_min_plane points run on
  // the z-marching stencil engine (PB_MG_ENGINE_MIN_PLANE; smaller levels: per-pair kernels,
  // whose short z-chunks would not amortise the engine's prologue)
  int64_t engine_min_plane = 256 * 256;
  // restriction and prolongation: one thread per coarse column marching in z on coarse levels of
  // >= restrict_z_min_cols columns, one thread per coarse cell (prolongation) / point
  // (restriction) below
  int64_t restrict_z_min_cols = 4096;
  bool tail_attr = false;  // mg_tail_kernel's dynamic-LDS limit raised
  // Decomposed grids (r04): the coarse levels [La, L) are gathered onto every rank once per
  // V-cycle (one all-to-all of level La's right-hand side) and run there as the one-launch tail
  // on full-grid arrays -- instead of a latency-bound halo exchange per half-sweep, residual and
  // transfer on levels of a few thousand points. La = 0: none. Every rank computes the same
  // coarse correction (same kernels, same inputs) and prolongates from its own planes of it.
  int La = 0;
  double* agg = nullptr;                   // full-grid x, b, res of levels La .. L-1; send staging
  std::vector<MgGeo> ageo;                 // their full-grid geometry (k0 = 0)
  std::vector<double*> ax, ab, ares;
  double* agg_send = nullptr;              // P copies of this rank's level-La slab
  std::vector<int64_t> agg_sc, agg_rc;     // all-to-all counts (send: own slab; recv: rank q's)
};

// ---------------------------------------------------------------------------------------------
// kernels. Every level has an even x extent, so one thread owns an (i even, i + 1) pair: 16-byte
// loads and full-line 16-byte stores; the pair holds one red and one black point.
// ---------------------------------------------------------------------------------------------
typedef double dv2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int wrapm(int v, int n) { return v < 0 ? v + n : (v >= n ? v - n : v); }

struct PairPos {
  int i0, j, k;       // pair origin (i0 even), row j, local plane k
  int64_t idx;        // linear index of (i0, j, k)
};

// 32-bit index arithmetic (a level never holds 2^32 pairs on one GPU)
__device__ __forceinline__ PairPos pair_pos(const MgGeo& G, int64_t q64) {
  const uint32_t q = (uint32_t)q64, hx = (uint32_t)G.nx >> 1;
  const uint32_t row = q / hx;
  PairPos p;
  p.i0 = (int)(q - row * hx) * 2;
  p.k = (int)(row / (uint32_t)G.ny);
  p.j = (int)(row - (uint32_t)p.k * (uint32_t)G.ny);
  p.idx = (int64_t)row * G.nx + p.i0;
  return p;
}

// value of v at (i, j +- 1) and (i, j, k +- 1) for the point at linear index id (plane offset
// pid = id - k*plane); lo / hi are the planes below / above the slab
struct Nb4 {
  double zm, ym, yp, zp;
};
__device__ __forceinline__ Nb4 nb4(const MgGeo& G, const double* v, const double* lo,
                                   const double* hi, int64_t id, int i, int j, int k) {
  const int64_t pid = id - (int64_t)k * G.plane;
  Nb4 r;
  r.zm = k > 0 ? v[id - G.plane] : lo[pid];
  r.zp = k < G.nzl - 1 ? v[id + G.plane] : hi[pid];
  r.ym = v[id + (int64_t)(wrapm(j - 1, G.ny) - j) * G.nx];
  r.yp = v[id + (int64_t)(wrapm(j + 1, G.ny) - j) * G.nx];
  (void)i;
  return r;
}

// red value after the zero-initialised first half-sweep: (1 - w) * 0 + w * ((b - 0) * (1 / c))
__device__ __forceinline__ double red0(double b, const Star& s, double omega) {
  const double t = (b - 0.0) * (1.0 / s.cc);
  return (1.0 - omega) * 0.0 + omega * t;
}

// mode 0: one red-black SOR half-sweep over `color` (x holds the current iterate).
// mode 1: the first two half-sweeps from x = 0 fused: red = w D^-1 b, then black from those red
//         values, computed from b directly (lo / hi are then b's ghost planes).
__device__ __forceinline__ void mg_smooth_body(MgGeo G, double* x, const double* __restrict__ b, const double* lo, const double* hi, Star s, double omega, int color, int mode, int64_t t0, int64_t ts) {
  const int64_t npairs = G.nlocal >> 1;
  for (int64_t q = t0; q < npairs;
       q += ts) {
    const PairPos P = pair_pos(G, q);
    const int64_t row = P.idx - P.i0;
    if (mode == 1) {
      const dv2 bp = *(const dv2*)(b + P.idx);
      const int dr = (int)((P.j + G.k0 + P.k) & 1);  // red offset in the pair
      const int ib = P.i0 + (dr ^ 1);
      const int64_t idb = row + ib;
      const double bb = dr ? bp.x : bp.y;               // black point's b
      const double br = dr ? bp.y : bp.x;
      const Nb4 n4 = nb4(G, b, lo, hi, idb, ib, P.j, P.k);
      const double bxm = ib == P.i0 + 1 ? bp.x : b[row + wrapm(ib - 1, G.nx)];
      const double bxp = ib == P.i0 ? bp.y : b[row + wrapm(ib + 1, G.nx)];
      double nb = s.cz * red0(n4.zm, s, omega);
      nb = nb + s.cy * red0(n4.ym, s, omega);
      nb = nb + s.cx * red0(bxm, s, omega);
      nb = nb + s.cx * red0(bxp, s, omega);
      nb = nb + s.cy * red0(n4.yp, s, omega);
      nb = nb + s.cz * red0(n4.zp, s, omega);
      const double t = (bb - nb) * (1.0 / s.cc);
      const double xb = (1.0 - omega) * 0.0 + omega * t;
      const double xr = red0(br, s, omega);
      dv2 o;
      o.x = dr ? xb : xr;
      o.y = dr ? xr : xb;
      *(dv2*)(x + P.idx) = o;
      continue;
    }
    const dv2 xp = *(const dv2*)(x + P.idx);
    const int d = (int)((color + P.j + G.k0 + P.k) & 1);  // offset of the updated point
    const int ic = P.i0 + d;
    const int64_t id = row + ic;
    const Nb4 n4 = nb4(G, x, lo, hi, id, ic, P.j, P.k);
    const double xm = d ? xp.x : x[row + wrapm(P.i0 - 1, G.nx)];
    const double xq = d ? x[row + wrapm(P.i0 + 2, G.nx)] : xp.y;
    double nb = s.cz * n4.zm;
    nb = nb + s.cy * n4.ym;
    nb = nb + s.cx * xm;
    nb = nb + s.cx * xq;
    nb = nb + s.cy * n4.yp;
    nb = nb + s.cz * n4.zp;
    const double xo = d ? xp.y : xp.x;
    const double t = (b[id] - nb) * (1.0 / s.cc);
    const double xn = (1.0 - omega) * xo + omega * t;
    dv2 o = xp;
    if (d) o.y = xn;
    else o.x = xn;
    *(dv2*)(x + P.idx) = o;
  }
}
__global__ __launch_bounds__(256) void mg_smooth_kernel(MgGeo G, double* x,
                                                        const double* __restrict__ b,
                                                        const double* lo, const double* hi, Star s,
                                                        double omega, int color, int mode,
                                                        const int* skip) {
  if (skip && *skip) return;
  mg_smooth_body(G, x, b, lo, hi, s, omega, color, mode, (int64_t)blockIdx.x * blockDim.x + threadIdx.x,
                  (int64_t)gridDim.x * blockDim.x);
}

// res = b - A x for both points of the pair (the reference operator's summation order)
__device__ __forceinline__ void mg_residual_body(MgGeo G, const double* __restrict__ x, const double* __restrict__ b, const double* __restrict__ lo, const double* __restrict__ hi, Star s, double* __restrict__ res, int64_t t0, int64_t ts) {
  const int64_t npairs = G.nlocal >> 1;
  for (int64_t q = t0; q < npairs;
       q += ts) {
    const PairPos P = pair_pos(G, q);
    const int64_t row = P.idx - P.i0;
    const dv2 xc = *(const dv2*)(x + P.idx);
    const dv2 bc = *(const dv2*)(b + P.idx);
    const int64_t pid = P.idx - (int64_t)P.k * G.plane;
    const dv2 zm = P.k > 0 ? *(const dv2*)(x + P.idx - G.plane) : *(const dv2*)(lo + pid);
    const dv2 zp = P.k < G.nzl - 1 ? *(const dv2*)(x + P.idx + G.plane) : *(const dv2*)(hi + pid);
    const dv2 ym = *(const dv2*)(x + P.idx + (int64_t)(wrapm(P.j - 1, G.ny) - P.j) * G.nx);
    const dv2 yp = *(const dv2*)(x + P.idx + (int64_t)(wrapm(P.j + 1, G.ny) - P.j) * G.nx);
    const double xl = x[row + wrapm(P.i0 - 1, G.nx)];
    const double xr = x[row + wrapm(P.i0 + 2, G.nx)];
    double a0 = s.cz * zm.x;
    a0 = a0 + s.cy * ym.x;
    a0 = a0 + s.cx * xl;
    a0 = a0 + s.cc * xc.x;
    a0 = a0 + s.cx * xc.y;
    a0 = a0 + s.cy * yp.x;
    a0 = a0 + s.cz * zp.x;
    double a1 = s.cz * zm.y;
    a1 = a1 + s.cy * ym.y;
    a1 = a1 + s.cx * xc.x;
    a1 = a1 + s.cc * xc.y;
    a1 = a1 + s.cx * xr;
    a1 = a1 + s.cy * yp.y;
    a1 = a1 + s.cz * zp.y;
    dv2 o;
    o.x = bc.x - a0;
    o.y = bc.y - a1;
    *(dv2*)(res + P.idx) = o;
  }
}
__global__ __launch_bounds__(256) void mg_residual_kernel(MgGeo G, const double* __restrict__ x,
                                                          const double* __restrict__ b,
                                                          const double* __restrict__ lo,
                                                          const double* __restrict__ hi, Star s,
                                                          double* __restrict__ res, const int* skip) {
  if (skip && *skip) return;
  mg_residual_body(G, x, b, lo, hi, s, res, (int64_t)blockIdx.x * blockDim.x + threadIdx.x,
                  (int64_t)gridDim.x * blockDim.x);
}

__device__ __forceinline__ void mg_ijk(const MgGeo& G, int64_t idx, int& i, int& j, int& k) {
  const uint32_t u = (uint32_t)idx, nx = (uint32_t)G.nx;
  const uint32_t row = u / nx;
  i = (int)(u - row * nx);
  k = (int)(row / (uint32_t)G.ny);
  j = (int)(row - (uint32_t)k * (uint32_t)G.ny);
}

// b_c = R res_f, R = P^T / 8: 4 x 4 x 4 fine cells (2I-1 .. 2I+2 per direction)
__device__ __forceinline__ void mg_restrict_body(MgGeo F, const double* __restrict__ rf, const double* __restrict__ lo, const double* __restrict__ hi, MgGeo Cg, double* __restrict__ bc, int64_t t0, int64_t ts) {
  const double w[4] = {0.125, 0.375, 0.375, 0.125};
  for (int64_t idx = t0; idx < Cg.nlocal;
       idx += ts) {
    int I, J, K;
    mg_ijk(Cg, idx, I, J, K);
    const int xl = wrapm(2 * I - 1, F.nx), xr = wrapm(2 * I + 2, F.nx);
    double sz = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int kf = 2 * K - 1 + c;
      const double* pl = kf < 0 ? lo : (kf >= F.nzl ? hi : rf + (int64_t)kf * F.plane);
      double sy = 0.0;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        const double* row = pl + (int64_t)wrapm(2 * J - 1 + bb, F.ny) * F.nx;
        const dv2 mid = *(const dv2*)(row + 2 * I);
        double sx = w[0] * row[xl];
        sx = sx + w[1] * mid.x;
        sx = sx + w[2] * mid.y;
        sx = sx + w[3] * row[xr];
        sy = sy + w[bb] * sx;
      }
      sz = sz + w[c] * sy;
    }
    bc[idx] = sz;
  }
}
__global__ __launch_bounds__(256) void mg_restrict_kernel(MgGeo F, const double* __restrict__ rf,
                                                          const double* __restrict__ lo,
                                                          const double* __restrict__ hi, MgGeo Cg,
                                                          double* __restrict__ bc, const int* skip) {
  if (skip && *skip) return;
  mg_restrict_body(F, rf, lo, hi, Cg, bc, (int64_t)blockIdx.x * blockDim.x + threadIdx.x,
                  (int64_t)gridDim.x * blockDim.x);
}

// The same restriction, one thread per coarse (I, J) column marching over a chunk of coarse
// planes: the x-y weighted sum sy of each fine plane is formed once and kept in a 4-plane
// window (the per-cell kernel forms it twice); the z sum is the per-cell kernel's, same order.
__device__ __forceinline__ double restrict_xy(const MgGeo& F, const double* pl, int I, int J,
                                              int xl, int xr) {
  const double w[4] = {0.125, 0.375, 0.375, 0.125};
  double sy = 0.0;
#pragma unroll
  for (int bb = 0; bb < 4; ++bb) {
    const double* row = pl + (int64_t)wrapm(2 * J - 1 + bb, F.ny) * F.nx;
    const dv2 mid = *(const dv2*)(row + 2 * I);
    double sx = w[0] * row[xl];
    sx = sx + w[1] * mid.x;
    sx = sx + w[2] * mid.y;
    sx = sx + w[3] * row[xr];
    sy = sy + w[bb] * sx;
  }
  return sy;
}

__global__ __launch_bounds__(256) void mg_restrict_z_kernel(MgGeo F, const double* __restrict__ rf,
                                                            const double* __restrict__ lo,
                                                            const double* __restrict__ hi,
                                                            MgGeo Cg, int kc,
                                                            double* __restrict__ bc,
                                                            const int* skip) {
  if (skip && *skip) return;
  const int64_t cols = (int64_t)Cg.nx * Cg.ny;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t col = t % cols;
  const int K0 = (int)(t / cols) * kc;
  if (K0 >= Cg.nzl) return;
  const int K1 = min(K0 + kc, Cg.nzl);
  const int I = (int)(col % Cg.nx), J = (int)(col / Cg.nx);
  const int xl = wrapm(2 * I - 1, F.nx), xr = wrapm(2 * I + 2, F.nx);
  auto plane = [&](int kf) {
    return kf < 0 ? lo : (kf >= F.nzl ? hi : rf + (int64_t)kf * F.plane);
  };
  double s0 = restrict_xy(F, plane(2 * K0 - 1), I, J, xl, xr);
  double s1 = restrict_xy(F, plane(2 * K0), I, J, xl, xr);
  for (int K = K0; K < K1; ++K) {
    const double s2 = restrict_xy(F, plane(2 * K + 1), I, J, xl, xr);
    const double s3 = restrict_xy(F, plane(2 * K + 2), I, J, xl, xr);
    double sz = 0.0;
    sz = sz + 0.125 * s0;
    sz = sz + 0.375 * s1;
    sz = sz + 0.375 * s2;
    sz = sz + 0.125 * s3;
    bc[(int64_t)K * Cg.plane + col] = sz;
    s0 = s2;
    s1 = s3;
  }
}

// x_f += P x_c (trilinear, cell-centred: near parent 3/4, far 1/4), one thread per coarse cell: its 2 x 2 x 2 fine children from the
// 3 x 3 x 3 coarse neighbourhood (each child by the formula above, same operation order), so a
// fine row pair is read and written with 16-byte accesses and each coarse value is fetched
// ~27/8 times per fine point instead of 6.
__device__ __forceinline__ void mg_prolong_cell_body(MgGeo F, double* __restrict__ xf, MgGeo Cg, const double* __restrict__ xc, const double* __restrict__ lo, const double* __restrict__ hi, int64_t t0, int64_t ts) {
  for (int64_t idx = t0; idx < Cg.nlocal;
       idx += ts) {
    int I, J, K;
    mg_ijk(Cg, idx, I, J, K);
    const int Im = wrapm(I - 1, Cg.nx), Ip = wrapm(I + 1, Cg.nx);
    const int Jm = wrapm(J - 1, Cg.ny), Jp = wrapm(J + 1, Cg.ny);
    const double* pn = xc + (int64_t)K * Cg.plane;
    const int64_t rn = (int64_t)J * Cg.nx;
#pragma unroll
    for (int dk = 0; dk < 2; ++dk) {
      const int fK = dk ? K + 1 : K - 1;
      const double* pf = fK < 0 ? lo : (fK >= Cg.nzl ? hi : xc + (int64_t)fK * Cg.plane);
#pragma unroll
      for (int dj = 0; dj < 2; ++dj) {
        const int64_t rf = (int64_t)(dj ? Jp : Jm) * Cg.nx;
        const double vn0 = 0.75 * (0.75 * pn[rn + I] + 0.25 * pn[rn + Im]) +
                           0.25 * (0.75 * pn[rf + I] + 0.25 * pn[rf + Im]);
        const double vf0 = 0.75 * (0.75 * pf[rn + I] + 0.25 * pf[rn + Im]) +
                           0.25 * (0.75 * pf[rf + I] + 0.25 * pf[rf + Im]);
        const double vn1 = 0.75 * (0.75 * pn[rn + I] + 0.25 * pn[rn + Ip]) +
                           0.25 * (0.75 * pn[rf + I] + 0.25 * pn[rf + Ip]);
        const double vf1 = 0.75 * (0.75 * pf[rn + I] + 0.25 * pf[rn + Ip]) +
                           0.25 * (0.75 * pf[rf + I] + 0.25 * pf[rf + Ip]);
        dv2* q = (dv2*)(xf + (int64_t)(2 * K + dk) * F.plane + (int64_t)(2 * J + dj) * F.nx + 2 * I);
        dv2 o = *q;
        o.x = o.x + (0.75 * vn0 + 0.25 * vf0);
        o.y = o.y + (0.75 * vn1 + 0.25 * vf1);
        *q = o;
      }
    }
  }
}
__global__ __launch_bounds__(256) void mg_prolong_cell_kernel(MgGeo F, double* __restrict__ xf,
                                                              MgGeo Cg,
                                                              const double* __restrict__ xc,
                                                              const double* __restrict__ lo,
                                                              const double* __restrict__ hi,
                                                              const int* skip) {
  if (skip && *skip) return;
  mg_prolong_cell_body(F, xf, Cg, xc, lo, hi, (int64_t)blockIdx.x * blockDim.x + threadIdx.x,
                  (int64_t)gridDim.x * blockDim.x);
}

// The same prolongation, one thread per coarse (I, J) column marching over a chunk of coarse
// planes: the 3 x 3 coarse values of planes K-1, K, K+1 stay in registers (each coarse value is
// loaded ~3 times per coarse cell instead of 27), children by the formula above.
// xout = xf + P xc (xout may be xf: in place).
struct Coarse9 {
  double v[3][3];  // [row Jm, J, Jp][col Im, I, Ip]
};
__device__ __forceinline__ void load9(const double* pl, int64_t rm, int64_t r0, int64_t rp, int Im,
                                      int I, int Ip, Coarse9& c) {
  const int64_t rows[3] = {rm, r0, rp};
  const int cols[3] = {Im, I, Ip};
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) c.v[a][b] = pl[rows[a] + cols[b]];
}

__global__ __launch_bounds__(256) void mg_prolong_z_kernel(MgGeo F, const double* xf,
                                                           double* xout, MgGeo Cg,
                                                           int kc, const double* __restrict__ xc,
                                                           const double* __restrict__ lo,
                                                           const double* __restrict__ hi,
                                                           const int* skip) {
  if (skip && *skip) return;
  const int64_t cols = (int64_t)Cg.nx * Cg.ny;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t col = t % cols;
  const int K0 = (int)(t / cols) * kc;
  if (K0 >= Cg.nzl) return;
  const int K1 = min(K0 + kc, Cg.nzl);
  const int I = (int)(col % Cg.nx), J = (int)(col / Cg.nx);
  const int Im = wrapm(I - 1, Cg.nx), Ip = wrapm(I + 1, Cg.nx);
  const int64_t rm = (int64_t)wrapm(J - 1, Cg.ny) * Cg.nx, r0 = (int64_t)J * Cg.nx,
                rp = (int64_t)wrapm(J + 1, Cg.ny) * Cg.nx;
  auto plane = [&](int K) {
    return K < 0 ? lo : (K >= Cg.nzl ? hi : xc + (int64_t)K * Cg.plane);
  };
  Coarse9 cm, c0, cp;
  load9(plane(K0 - 1), rm, r0, rp, Im, I, Ip, cm);
  load9(plane(K0), rm, r0, rp, Im, I, Ip, c0);
  for (int K = K0; K < K1; ++K) {
    load9(plane(K + 1), rm, r0, rp, Im, I, Ip, cp);
    // all four fine pairs are loaded before any is stored (the stores would otherwise order
    // each later load behind them)
    int64_t q[2][2];
    dv2 ov[2][2];
#pragma unroll
    for (int dk = 0; dk < 2; ++dk)
#pragma unroll
      for (int dj = 0; dj < 2; ++dj) {
        q[dk][dj] = (int64_t)(2 * K + dk) * F.plane + (int64_t)(2 * J + dj) * F.nx + 2 * I;
        ov[dk][dj] = *(const dv2*)(xf + q[dk][dj]);
      }
#pragma unroll
    for (int dk = 0; dk < 2; ++dk) {
      const Coarse9& pf = dk ? cp : cm;  // far plane: K+1 for odd fine k, K-1 for even
#pragma unroll
      for (int dj = 0; dj < 2; ++dj) {
        const int f = dj ? 2 : 0;  // far row: J+1 for odd fine j, J-1 for even
        const double vn0 = 0.75 * (0.75 * c0.v[1][1] + 0.25 * c0.v[1][0]) +
                           0.25 * (0.75 * c0.v[f][1] + 0.25 * c0.v[f][0]);
        const double vf0 = 0.75 * (0.75 * pf.v[1][1] + 0.25 * pf.v[1][0]) +
                           0.25 * (0.75 * pf.v[f][1] + 0.25 * pf.v[f][0]);
        const double vn1 = 0.75 * (0.75 * c0.v[1][1] + 0.25 * c0.v[1][2]) +
                           0.25 * (0.75 * c0.v[f][1] + 0.25 * c0.v[f][2]);
        const double vf1 = 0.75 * (0.75 * pf.v[1][1] + 0.25 * pf.v[1][2]) +
                           0.25 * (0.75 * pf.v[f][1] + 0.25 * pf.v[f][2]);
        dv2 o = ov[dk][dj];
        o.x = o.x + (0.75 * vn0 + 0.25 * vf0);
        o.y = o.y + (0.75 * vn1 + 0.25 * vf1);
        ov[dk][dj] = o;
      }
    }
#pragma unroll
    for (int dk = 0; dk < 2; ++dk)
#pragma unroll
      for (int dj = 0; dj < 2; ++dj) *(dv2*)(xout + q[dk][dj]) = ov[dk][dj];
    cm = c0;
    c0 = cp;
  }
}

// ---------------------------------------------------------------------------------------------
// The coarse tail of the V-cycle in ONE launch (one rank): every level of at most
// PB_MG_TAIL_MAX points (16^3 at 512^3: the 16^3, 8^3 and 4^3 levels) -- down-legs, the coarsest
// level's sweeps and the up-legs -- run by one workgroup, step after step with a barrier between
// them, through the same per-point bodies as the per-level kernels (same operations, bit for bit).
// Replaces ~28 launches of a few microseconds each per V-cycle.
// ---------------------------------------------------------------------------------------------
struct TailLevel {
  MgGeo G;
  double* x;
  double* b;
  double* res;
  Star s;
  int64_t ox, ob, ores;  // LDS offsets (doubles) of x, b, res when the tail runs in LDS
};
static constexpr int kTailMax = 12;
static constexpr size_t kTailLdsMax = 144 * 1024;  // LDS the tail may take (of 160 KB per CU)
struct TailArgs {
  TailLevel lv[kTailMax];
  int nl;           // levels in the tail; lv[nl-1] is the coarsest
  int coarse_its;
  double omega;
  int lds;          // 1: every tail array lives in LDS (lv[0].b copied in, lv[0].x copied out)
};

__device__ __forceinline__ const double* wrap_lo(const MgGeo& G, const double* v) {
  return v + (int64_t)(G.nzl - 1) * G.plane;  // one rank: plane -1 is the last plane
}

// With A.lds the tail's arrays live in the workgroup's LDS (the 16^3, 8^3, 4^3 levels of a 512^3
// hierarchy: 109 KB): lv[0].b is copied in, lv[0].x copied out at the end, and every step in
// between reads and writes LDS through the same bodies (generic pointers) -- same operations on
// the same values, so the same bits; LDS instead of L2 latency on each of the ~35 dependent steps.
__global__ __launch_bounds__(512) void mg_tail_kernel(TailArgs A, const int* skip) {
  if (skip && *skip) return;
  extern __shared__ __attribute__((aligned(16))) double tl[];
  const int64_t t0 = threadIdx.x, ts = blockDim.x;
  const double w = A.omega;
  // level t's arrays (LDS or global); computed per use, so no array of pointers goes to scratch
  auto X = [&](int t) { return A.lds ? tl + A.lv[t].ox : A.lv[t].x; };
  auto Bv = [&](int t) { return A.lds ? tl + A.lv[t].ob : A.lv[t].b; };
  auto RES = [&](int t) { return A.lds ? tl + A.lv[t].ores : A.lv[t].res; };
  if (A.lds) {
    const double* src = A.lv[0].b;
    double* dst = Bv(0);
    for (int64_t i = t0; i < A.lv[0].G.nlocal; i += ts) dst[i] = src[i];
    __syncthreads();
  }
  auto smooth = [&](int t, int color, int mode) {
    const TailLevel& L = A.lv[t];
    double* x = X(t);
    const double* b = Bv(t);
    const double* v = mode == 1 ? b : x;
    mg_smooth_body(L.G, x, b, wrap_lo(L.G, v), v, L.s, w, color, mode, t0, ts);
    __syncthreads();
  };
  for (int t = 0; t + 1 < A.nl; ++t) {  // down: pre-smooth, residual, restrict
    const TailLevel& F = A.lv[t];
    smooth(t, 0, 1);
    double* x = X(t);
    double* res = RES(t);
    mg_residual_body(F.G, x, Bv(t), wrap_lo(F.G, x), x, F.s, res, t0, ts);
    __syncthreads();
    mg_restrict_body(F.G, res, wrap_lo(F.G, res), res, A.lv[t + 1].G, Bv(t + 1), t0, ts);
    __syncthreads();
  }
  {  // coarsest: `coarse_its` symmetric red-black sweeps from zero (coarse_solve's order)
    const int c = A.nl - 1;
    smooth(c, 0, 1);
    smooth(c, 0, 0);
    for (int it = 1; it < A.coarse_its; ++it) {
      smooth(c, 1, 0);
      smooth(c, 0, 0);
    }
  }
  for (int t = A.nl - 2; t >= 0; --t) {  // up: prolongate + correct, post-smooth
    const TailLevel& F = A.lv[t];
    const TailLevel& Cl = A.lv[t + 1];
    double* xf = X(t);
    const double* xc = X(t + 1);
    mg_prolong_cell_body(F.G, xf, Cl.G, xc, wrap_lo(Cl.G, xc), xc, t0, ts);
    __syncthreads();
    smooth(t, 1, 0);
    smooth(t, 0, 0);
  }
  if (A.lds) {
    const double* src = X(0);
    double* dst = A.lv[0].x;
    for (int64_t i = t0; i < A.lv[0].G.nlocal; i += ts) dst[i] = src[i];
  }
}

// chunks of coarse planes for the z-marching transfer kernels: ~16 resident waves per CU, at
// least 4 coarse planes per chunk
static int transfer_chunk(pb_ctx* ctx, int64_t cols, int64_t nzl, int64_t* nchunk_out) {
  const int64_t tpc = 1024;  // threads per CU
  const int64_t minz = 4;    // coarse planes per chunk, at least
  int64_t nchunk = ((int64_t)ctx->num_cus * tpc + cols - 1) / cols;
  nchunk = std::max<int64_t>(1, std::min<int64_t>(nchunk, nzl / minz));
  const int kc = (int)((nzl + nchunk - 1) / nchunk);
  *nchunk_out = (nzl + kc - 1) / kc;
  return kc;
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
// one thread per item (no grid-stride loop unless the grid would exceed 2^30 blocks)
static int mg_blocks(pb_ctx* ctx, int64_t n) {
  (void)ctx;
  int64_t b = (n + 255) / 256;
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, (int64_t)1 << 30));
}

// ghost planes of v on level L: in place (1 rank) or exchanged (N ranks)
static int ghosts(MgLevel& L, const double* v, const double** lo, const double** hi) {
  pb_grid* g = L.g;
  if (!g->ctx->split) {
    *lo = v + (g->nzl - 1) * g->plane;
    *hi = v;
    return PB_OK;
  }
  PB_TRY(halo_exchange(g, v, v + (g->nzl - 1) * g->plane));
  *lo = g->ghost_lo;
  *hi = g->ghost_hi;
  return PB_OK;
}

// mode 0: half-sweep of `color`; mode 1: zero-initialised red + black half-sweeps fused.
// sums_st (mode 0, engine path only): also take CG's residual sums of the output (*nparts set)
static int smooth(Mg* mg, MgLevel& L, int color, int mode, const CgState* sums_st = nullptr,
                  int* nparts = nullptr) {
  const double *lo = nullptr, *hi = nullptr;
  PB_TRY(ghosts(L, mode == 1 ? L.b : L.x, &lo, &hi));
  if (L.g->plane >= mg->engine_min_plane) {
    const StencilPlanes gp{lo, hi};
    return launch_mg_sor(L.g, L.s, L.x, L.b, gp, mg->omega, color, mode == 1, mg->skip,
                         mode == 0 ? sums_st : nullptr, mode == 0 ? nparts : nullptr);
  }
  const MgGeo G = L.geo();
  hipLaunchKernelGGL(mg_smooth_kernel, dim3(mg_blocks(mg->ctx, G.nlocal / 2)), dim3(256), 0,
                     mg->ctx->stream, G, L.x, (const double*)L.b, lo, hi, L.s, mg->omega, color,
                     mode, mg->skip);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

// coarsest level: `coarse_its` symmetric red-black sweeps from zero (red, black, red, black, ...)
static int coarse_solve(Mg* mg, MgLevel& L, const CgState* sums_st, int* nparts) {
  PB_TRY(smooth(mg, L, 0, 1));  // red from zero + black
  const int its = mg->coarse_its;
  PB_TRY(smooth(mg, L, 0, 0, its == 1 ? sums_st : nullptr, nparts));
  for (int it = 1; it < its; ++it) {
    PB_TRY(smooth(mg, L, 1, 0));
    PB_TRY(smooth(mg, L, 0, 0, it == its - 1 ? sums_st : nullptr, nparts));
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
  (void)wait_stream(mg->ctx, mg->ctx->stream, "mg_destroy");
  for (auto& L : mg->lv)
    if (L.own) pb_grid_destroy(L.g);
  if (mg->mem) (void)hipFree(mg->mem);
  if (mg->agg) (void)hipFree(mg->agg);
  delete mg;
}

// levels whose planes hold at least this many points run the fused / engine passes: 256^2 on one
// rank (the 128^3 level's six per-level launches beat the fused passes there, 0.381 vs 0.409 ms);
// 128^2 on decomposed grids, where every per-level pass costs a halo exchange (force_comm 512^3
// MG-PCG 48.1 -> 47.75 ms, profiles/r04/decomposed/mg_engine_128_ab.txt)
static int64_t mg_engine_min_plane_default(const pb_ctx* ctx) {
  return ctx->split ? 128 * 128 : 256 * 256;
}

// the agglomerated coarse levels of a decomposed grid (Mg::La): the first level whose whole grid
// fits the one-launch tail (<= mg_agglomerate_max points, default PB_MG_TAIL_MAX as on one
// rank), at least level 1. Only with an all-to-all to gather them (RCCL, or a host transport
// with an alltoallv callback): the built-in shm transport keeps the halo-exchange levels
static int mg_agglomerate_setup(Mg* mg) {
  pb_ctx* ctx = mg->ctx;
  const int L = (int)mg->lv.size();
  mg->La = 0;
  if (!ctx->split || L < 2 || !tune("mg_agglomerate", 1)) return PB_OK;
  if (!ctx->comm && !ctx->h_alltoallv) return PB_OK;
  const int64_t tail_max = tune("mg_tail_max", 8192);
  int La = L;
  for (int l = L - 1; l >= 1; --l) {
    const MgLevel& v = mg->lv[l];
    if (v.n[0] * v.n[1] * v.n[2] <= tail_max) La = l;
    else break;
  }
  if (La >= L || L - La > kTailMax) return PB_OK;
  const int P = ctx->nranks;
  const MgLevel& A0 = mg->lv[La];
  int64_t total = 0;
  for (int l = La; l < L; ++l) {
    const MgLevel& v = mg->lv[l];
    total += 3 * ((v.n[0] * v.n[1] * v.n[2] + 1) & ~(int64_t)1);
  }
  const int64_t slab = A0.g->nlocal;
  total += P * slab;
  if (hipMalloc(&mg->agg, (size_t)total * sizeof(double)) != hipSuccess)
    return set_error(PB_ERR_ALLOC, "multigrid coarse levels: out of device memory");
  double* q = mg->agg;
  for (int l = La; l < L; ++l) {
    const MgLevel& v = mg->lv[l];
    const int64_t n = v.n[0] * v.n[1] * v.n[2], n2 = (n + 1) & ~(int64_t)1;
    mg->ageo.push_back(MgGeo{(int)v.n[0], (int)v.n[1], (int)v.n[2], v.n[0] * v.n[1], n, 0});
    mg->ax.push_back(q);
    mg->ab.push_back(q + n2);
    mg->ares.push_back(q + 2 * n2);
    q += 3 * n2;
  }
  mg->agg_send = q;
  mg->agg_sc.assign(P, slab);
  mg->agg_rc.resize(P);
  for (int r = 0; r < P; ++r) {
    int64_t k0 = 0, nz = 0;
    pb_slab_partition(mg->lv[0].g->n[2], P, r, &k0, &nz);
    mg->agg_rc[r] = (nz >> La) * A0.n[0] * A0.n[1];
  }
  mg->La = La;
  return PB_OK;
}

int mg_create(pb_grid* g, const double deltas[3], int pc_type, int levels_req, int coarse_its,
              double omega, Mg** out) {
  pb_ctx* ctx = g->ctx;
  for (int d = 0; d < 3; ++d)
    if (g->n[d] % 2)
      return set_error(PB_ERR_UNSUPPORTED,
                       "red-black SOR / multigrid needs even grid extents (got %lld x %lld x %lld)",
                       (long long)g->n[0], (long long)g->n[1], (long long)g->n[2]);
  if (g->nlocal >= ((int64_t)1 << 32))
    return set_error(PB_ERR_UNSUPPORTED, "multigrid: more than 2^32 points on one GPU");
  // PETSc PCSORSetOmega rejects omega outside (0, 2); PB_SOR_OMEGA_ANY=1 (diagnostics) accepts
  // it -- an indefinite SOR preconditioner, e.g. to exercise KSP_DIVERGED_INDEFINITE_PC
  if (!(omega > 0.0 && omega < 2.0) && !tune("sor_omega_any", 0))
    return set_error(PB_ERR_ARG, "SOR omega must be in (0, 2)");
  Mg* mg = new Mg();
  mg->ctx = ctx;
  mg->omega = omega;
  const int L = pc_type == PB_PC_MG ? mg_plan_levels(g->n, ctx->nranks, levels_req) : 1;
  mg->coarse_its = pc_type == PB_PC_MG ? std::max(1, coarse_its) : 1;
  mg->lv.resize(L);
  int64_t total = 0;
  // levels that take the fused post-smoothing (PB_MG_POST_FUSED, one rank): an xs array each
  // (N ranks: the unrolled fused passes with deep ghost planes, r04; mg_split_fused = 0 keeps
  // the decomposed V-cycle on the per-pass kernels)
  const bool want_post = !ctx->split || tune("mg_split_fused", 1) != 0;
  const int64_t post_min_plane = tune("mg_engine_min_plane", mg_engine_min_plane_default(ctx));
  auto takes_post = [&](const MgLevel& lv, int l) {
    return want_post && l < L - 1 && lv.g->plane >= post_min_plane && sor_sweep2_supported(lv.g);
  };
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
    if (takes_post(lv, l)) total += lv.g->nlocal;
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
    if (takes_post(lv, l)) {
      lv.xs = p;
      p += lv.g->nlocal;
    }
  }
  if (const int rc = mg_agglomerate_setup(mg); rc != PB_OK) {
    mg_destroy(mg);
    return rc;
  }
  *out = mg;
  return PB_OK;
}

// level l pre-smooths into xs and post-smooths with the fused prolongation kernel: it has an xs
// array (mg_create), the fused pre-smoothing applies, and so does the marching prolongation
static bool post_fused(const Mg* mg, int l) {
  const MgLevel& F = mg->lv[l];
  if (!F.xs || l + 1 >= (int)mg->lv.size() || F.g->plane < mg->engine_min_plane) return false;
  const MgLevel& C = mg->lv[l + 1];
  // N ranks: the unrolled kernel with deep ghosts (even slab origin, >= 2 planes per slab)
  if (mg->ctx->split && (!tune("mg_split_fused", 1) || F.g->k0 % 2 || F.g->nzl < 2 ||
                         C.g->nzl < 2))
    return false;
  return C.g->n[0] * C.g->n[1] >= mg->restrict_z_min_cols;
}

int mg_apply(Mg* mg, const double* r, double* z, const int* skip, const CgState* sums_st,
             int* nparts) {
  if (nparts) *nparts = 0;
  ScopedTimer tm(mg->ctx, "mg_apply");
  mg->skip = skip;
  mg->engine_min_plane = tune("mg_engine_min_plane", mg_engine_min_plane_default(mg->ctx));
  mg->restrict_z_min_cols = tune("mg_restrict_z_min_cols", 4096);
  const int L = (int)mg->lv.size();
  mg->lv[0].b = const_cast<double*>(r);
  mg->lv[0].x = z;
  pb_ctx* ctx = mg->ctx;
  // the coarse tail in one launch (one rank): levels Lt .. L-1 of <= PB_MG_TAIL_MAX points
  int Lt = L;
  if (mg->La > 0) Lt = mg->La;  // decomposed grid: the agglomerated levels run as the tail
  else if (!ctx->split) {
    const int64_t tail_max = tune("mg_tail_max", 8192);
    Lt = L - 1;
    while (Lt > 1 && mg->lv[Lt - 1].g->nlocal <= tail_max) --Lt;
    if (Lt < 1 || mg->lv[Lt].g->nlocal > tail_max || L - Lt > kTailMax) Lt = L;
  }
  const int Ldown = Lt < L ? Lt : L - 1;  // host down-legs l < Ldown
  for (int l = 0; l < Ldown; ++l) {  // down: pre-smooth (red, black), residual, restrict
    MgLevel& F = mg->lv[l];
    MgLevel& Cl = mg->lv[l + 1];
    // large level: zero-start red + black half-sweeps and the residual in one pass
    const bool fused = F.g->plane >= mg->engine_min_plane && sor_sweep2_supported(F.g);
    // one rank: the restriction too (the residual is never stored)
    const bool fused_r = fused && F.g->nzl % 2 == 0 &&
                         (!ctx->split || (tune("mg_split_fused", 1) && F.g->nzl >= 3 &&
                                          F.g->k0 % 2 == 0));
    if (fused_r) {
      ScopedTimer t1(ctx, l == 0 ? "mg_fine_smooth_first" : "mg_coarse_levels");
      PB_TRY(launch_presmooth_restrict(F.g, F.s, Cl.g, F.b, post_fused(mg, l) ? F.xs : F.x, Cl.b,
                                       mg->omega, mg->skip));
      continue;
    }
    {
      ScopedTimer t1(ctx, l == 0 ? "mg_fine_smooth_first" : "mg_coarse_levels");
      if (fused)
        PB_TRY(launch_presmooth_residual(F.g, F.s, F.b, post_fused(mg, l) ? F.xs : F.x, F.res,
                                         mg->omega, mg->skip));
      else
        PB_TRY(smooth(mg, F, 0, 1));  // red from zero + black
    }
    ScopedTimer t2(ctx, l == 0 ? "mg_fine_resid_restrict" : "mg_coarse_levels");
    const double *lo, *hi;
    const MgGeo G = F.geo();
    if (fused) {
      // residual already in F.res
    } else if (F.g->plane >= mg->engine_min_plane) {
      PB_TRY(ghosts(F, F.x, &lo, &hi));
      PB_TRY(launch_mg_residual(F.g, F.s, F.x, F.b, StencilPlanes{lo, hi}, F.res, mg->skip));
    } else {
      PB_TRY(ghosts(F, F.x, &lo, &hi));
      hipLaunchKernelGGL(mg_residual_kernel, dim3(mg_blocks(ctx, G.nlocal / 2)), dim3(256), 0,
                         ctx->stream, G, (const double*)F.x, (const double*)F.b, lo, hi, F.s,
                         F.res, mg->skip);
      PB_HIP(hipGetLastError());
    }
    PB_TRY(ghosts(F, F.res, &lo, &hi));
    const MgGeo CG = Cl.geo();
    const int64_t cols = (int64_t)CG.nx * CG.ny;
    if (cols >= mg->restrict_z_min_cols) {
      int64_t nchunk = 1;
      const int kc = transfer_chunk(ctx, cols, CG.nzl, &nchunk);
      hipLaunchKernelGGL(mg_restrict_z_kernel, dim3(mg_blocks(ctx, cols * nchunk)), dim3(256), 0,
                         ctx->stream, G, (const double*)F.res, lo, hi, CG, kc, Cl.b, mg->skip);
    } else {
      hipLaunchKernelGGL(mg_restrict_kernel, dim3(mg_blocks(ctx, CG.nlocal)), dim3(256), 0,
                         ctx->stream, G, (const double*)F.res, lo, hi, CG, Cl.b, mg->skip);
    }
    PB_HIP(hipGetLastError());
  }
  const bool agg = mg->La > 0;
  if (agg) {  // gather level La's right-hand side onto every rank (P copies out, P slabs in)
    ScopedTimer tg(ctx, "mg_coarse_levels");
    const MgLevel& A0 = mg->lv[mg->La];
    const size_t bytes = (size_t)A0.g->nlocal * sizeof(double);
    for (int r = 0; r < ctx->nranks; ++r)
      PB_HIP(hipMemcpyAsync(mg->agg_send + (int64_t)r * A0.g->nlocal, A0.b, bytes,
                            hipMemcpyDeviceToDevice, ctx->stream));
    PB_TRY(alltoallv_device(ctx, mg->agg_send, mg->agg_sc.data(), mg->ab[0], mg->agg_rc.data()));
  }
  if (Lt < L) {
    ScopedTimer t3(ctx, "mg_coarse_levels");
    TailArgs A{};
    A.nl = L - Lt;
    A.coarse_its = mg->coarse_its;
    A.omega = mg->omega;
    int64_t off = 0;
    for (int t = 0; t < A.nl; ++t) {
      const MgLevel& lv = mg->lv[Lt + t];
      A.lv[t] = agg ? TailLevel{mg->ageo[t], mg->ax[t], mg->ab[t], mg->ares[t], lv.s, 0, 0, 0}
                    : TailLevel{lv.geo(), lv.x, lv.b, lv.res, lv.s, 0, 0, 0};
      const int64_t n = ((agg ? mg->ageo[t].nlocal : lv.g->nlocal) + 1) & ~(int64_t)1;  // 16-byte aligned arrays
      A.lv[t].ox = off;
      A.lv[t].ob = off + n;
      A.lv[t].ores = off + 2 * n;
      off += (t + 1 < A.nl ? 3 : 2) * n;
    }
    // the tail in LDS when it fits (512^3: 109 KB of the 160 KB per CU)
    const size_t lds = (size_t)off * sizeof(double);
    A.lds = lds <= kTailLdsMax;
    if (A.lds && !mg->tail_attr) {
      PB_HIP(hipFuncSetAttribute((const void*)mg_tail_kernel,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTailLdsMax));
      mg->tail_attr = true;
    }
    hipLaunchKernelGGL(mg_tail_kernel, dim3(1), dim3(512), A.lds ? lds : 0, ctx->stream, A,
                       mg->skip);
    PB_HIP(hipGetLastError());
  } else {
    ScopedTimer t3(ctx, L > 1 ? "mg_coarse_levels" : "mg_fine_smooth_first");
    PB_TRY(coarse_solve(mg, mg->lv[L - 1], L == 1 ? sums_st : nullptr, nparts));
  }
  // up: prolongate + correct, post-smooth; with a tail, the first host up-leg prolongates from Lt
  for (int l = Lt < L ? Lt - 1 : L - 2; l >= 0; --l) {
    MgLevel& F = mg->lv[l];
    MgLevel& Cl = mg->lv[l + 1];
    ScopedTimer t4(ctx, l == 0 ? "mg_fine_prolong_post" : "mg_coarse_levels");
    if (post_fused(mg, l)) {
      // prolongation + correction + both post-smoothing half-sweeps in one pass, xs -> x
      // (agglomerated coarse level: this rank's planes of the full coarse correction)
      const bool from_agg = agg && l + 1 == mg->La;
      const double* xcp = from_agg ? mg->ax[0] + Cl.g->k0 * Cl.g->plane : Cl.x;
      PB_TRY(launch_post_sweep(F.g, F.s, Cl.g, F.xs, xcp, F.b, F.x, mg->omega, mg->skip,
                               l == 0 ? sums_st : nullptr, l == 0 ? nparts : nullptr,
                               from_agg ? mg->ax[0] : nullptr));
      continue;
    }
    const double *lo, *hi;
    const double* xc = Cl.x;
    if (agg && l + 1 == mg->La) {  // this rank's planes of the full coarse correction
      const int64_t pc = Cl.g->plane, nzc = Cl.n[2], k0c = Cl.g->k0, nzl = Cl.g->nzl;
      xc = mg->ax[0] + k0c * pc;
      lo = mg->ax[0] + ((k0c - 1 + nzc) % nzc) * pc;
      hi = mg->ax[0] + ((k0c + nzl) % nzc) * pc;
    } else {
      PB_TRY(ghosts(Cl, Cl.x, &lo, &hi));
    }
    const MgGeo G = F.geo(), CG = Cl.geo();
    const int64_t cols = (int64_t)CG.nx * CG.ny;
    bool fused = false;
    if (cols >= mg->restrict_z_min_cols) {
      int64_t nchunk = 1;
      const int kc = transfer_chunk(ctx, cols, CG.nzl, &nchunk);
      // fused post-smoothing: prolongate into the residual scratch, then both half-sweeps in one
      // pass back into F.x (which also takes CG's residual sums on level 0)
      fused = F.res && F.g->plane >= mg->engine_min_plane && sor_sweep2_supported(F.g);
      hipLaunchKernelGGL(mg_prolong_z_kernel, dim3(mg_blocks(ctx, cols * nchunk)), dim3(256), 0,
                         ctx->stream, G, (const double*)F.x, fused ? F.res : F.x, CG, kc, xc, lo,
                         hi, mg->skip);
    } else {
      hipLaunchKernelGGL(mg_prolong_cell_kernel, dim3(mg_blocks(ctx, CG.nlocal)), dim3(256), 0,
                         ctx->stream, G, F.x, CG, xc, lo, hi, mg->skip);
    }
    PB_HIP(hipGetLastError());
    if (fused) {
      PB_TRY(launch_sor_sweep2(F.g, F.s, F.res, F.b, F.x, mg->omega, 1, mg->skip,
                               l == 0 ? sums_st : nullptr, l == 0 ? nparts : nullptr));
    } else {
      PB_TRY(smooth(mg, F, 1, 0));
      PB_TRY(smooth(mg, F, 0, 0, l == 0 ? sums_st : nullptr, nparts));
    }
  }
  return PB_OK;
}

}  // namespace pb
