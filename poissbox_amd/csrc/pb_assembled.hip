// pb_assembled.hip -- MatMult of the assembled P (src/coefficients.f90:50-113, 27-entry BOX rows
// with 20 explicit zeros) in PETSc's AIJ summation order.
//
// MatMult_SeqAIJ sums a row's stored entries in ascending column order; MatMult_MPIAIJ sums the
// owned columns (diagonal block) first, ascending, then adds the off-rank columns (MatMultAdd of
// the off-diagonal block), ascending by global index. For every row away from the periodic
// seams and the slab boundaries the 7 non-zero columns sort as z-, y-, x-, c, x+, y+, z+ -- the
// stencil engine's order (src/poissbox.f90:128-148), so its result is P x bit for bit there.
// Only rows whose columns wrap (i, j or global k at 0 / n-1) or leave the slab (local planes 0
// and nzl-1 on several ranks) sort differently; this kernel re-sums exactly those rows after the
// engine has run: the two outer planes of the slab in full, the perimeter of every other plane.
// The 0 * x products of the explicit zeros leave every partial sum unchanged and are skipped.
#include "pb_internal.hpp"

namespace pb {

namespace {

__device__ __forceinline__ void cswap(int64_t& ka, double& va, int64_t& kb, double& vb) {
  if (ka > kb) {
    const int64_t tk = ka;
    ka = kb;
    kb = tk;
    const double tv = va;
    va = vb;
    vb = tv;
  }
}

// one thread per seam row; rows = 2 full planes (or nzl if nzl < 2) + the perimeter of the rest
__global__ void __launch_bounds__(256) aij_seam_kernel(int nx, int ny, int nzl, int64_t k0,
                                                       int64_t nz, int multirank, double cx,
                                                       double cy, double cz, double cc,
                                                       const double* __restrict__ x,
                                                       const double* __restrict__ glo,
                                                       const double* __restrict__ ghi,
                                                       double* __restrict__ y, int64_t nrows) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nrows) return;
  const int64_t plane = (int64_t)nx * ny;
  const int nfull = nzl < 2 ? nzl : 2;
  const int64_t perim = 2 * (int64_t)nx + 2 * (int64_t)(ny - 2);
  int i, j, k;
  if (t < nfull * plane) {
    const int f = (int)(t / plane);
    const int64_t q = t - f * plane;
    k = f == 0 ? 0 : nzl - 1;
    j = (int)(q / nx);
    i = (int)(q - (int64_t)j * nx);
  } else {
    const int64_t u = t - nfull * plane;
    k = 1 + (int)(u / perim);
    const int64_t q = u - (int64_t)(k - 1) * perim;
    if (q < nx) {
      j = 0;
      i = (int)q;
    } else if (q < 2 * nx) {
      j = ny - 1;
      i = (int)(q - nx);
    } else {
      const int64_t q2 = q - 2 * nx;
      j = 1 + (int)(q2 >> 1);
      i = (q2 & 1) ? nx - 1 : 0;
    }
  }
  const int64_t kg = k0 + k;
  const int im = i == 0 ? nx - 1 : i - 1, ip = i == nx - 1 ? 0 : i + 1;
  const int jm = j == 0 ? ny - 1 : j - 1, jp = j == ny - 1 ? 0 : j + 1;
  const int64_t kgm = kg == 0 ? nz - 1 : kg - 1, kgp = kg == nz - 1 ? 0 : kg + 1;
  const double* xc = x + (int64_t)k * plane;
  // z neighbours: in place (one rank: periodic wrap inside the slab) or the ghost planes
  const double* xm = k > 0 ? xc - plane : (glo ? glo : x + (int64_t)(nzl - 1) * plane);
  const double* xp = k < nzl - 1 ? xc + plane : (ghi ? ghi : x);
  const int64_t own_lo = k0, own_hi = k0 + nzl;
  const int64_t OFF = (int64_t)1 << 62;
  auto key = [&](int ii, int jj, int64_t kk) -> int64_t {
    const int64_t col = (int64_t)ii + (int64_t)nx * ((int64_t)jj + (int64_t)ny * kk);
    return (multirank && (kk < own_lo || kk >= own_hi)) ? (OFF | col) : col;
  };
  const int64_t jr = (int64_t)j * nx;
  int64_t k_0 = key(i, j, kgm), k_1 = key(i, jm, kg), k_2 = key(im, j, kg), k_3 = key(i, j, kg),
          k_4 = key(ip, j, kg), k_5 = key(i, jp, kg), k_6 = key(i, j, kgp);
  double v_0 = cz * xm[jr + i], v_1 = cy * xc[(int64_t)jm * nx + i], v_2 = cx * xc[jr + im],
         v_3 = cc * xc[jr + i], v_4 = cx * xc[jr + ip], v_5 = cy * xc[(int64_t)jp * nx + i],
         v_6 = cz * xp[jr + i];
  // optimal 16-comparator network for 7 keys (exhaustively checked on all 0-1 inputs)
  cswap(k_0, v_0, k_6, v_6); cswap(k_2, v_2, k_3, v_3); cswap(k_4, v_4, k_5, v_5);
  cswap(k_0, v_0, k_2, v_2); cswap(k_1, v_1, k_4, v_4); cswap(k_3, v_3, k_6, v_6);
  cswap(k_0, v_0, k_1, v_1); cswap(k_2, v_2, k_5, v_5); cswap(k_3, v_3, k_4, v_4);
  cswap(k_1, v_1, k_2, v_2); cswap(k_4, v_4, k_6, v_6);
  cswap(k_2, v_2, k_3, v_3); cswap(k_4, v_4, k_5, v_5);
  cswap(k_1, v_1, k_2, v_2); cswap(k_3, v_3, k_4, v_4); cswap(k_5, v_5, k_6, v_6);
  double s = 0.0;  // PetscSparseDensePlusDot: sum from 0 in stored order
  s += v_0;
  s += v_1;
  s += v_2;
  s += v_3;
  s += v_4;
  s += v_5;
  s += v_6;
  y[(int64_t)k * plane + jr + i] = s;
}

}  // namespace

int launch_aij_seams(pb_grid* g, const Star& s, const double* x, const double* glo,
                     const double* ghi, double* y) {
  pb_ctx* ctx = g->ctx;
  const int nx = (int)g->n[0], ny = (int)g->n[1], nzl = (int)g->nzl;
  const int nfull = nzl < 2 ? nzl : 2;
  const int64_t nrows = (int64_t)nfull * g->plane +
                        (int64_t)(nzl - nfull) * (2 * (int64_t)nx + 2 * (int64_t)(ny - 2));
  if (nrows == 0) return PB_OK;
  ScopedTimer tm(ctx, "aij_seams");
  const int64_t nb = (nrows + 255) / 256;
  hipLaunchKernelGGL(aij_seam_kernel, dim3((unsigned)nb), dim3(256), 0, ctx->stream, nx, ny, nzl,
                     g->k0, g->n[2], ctx->nranks > 1 ? 1 : 0, s.cx, s.cy, s.cz, s.cc, x, glo, ghi,
                     y, nrows);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

}  // namespace pb
