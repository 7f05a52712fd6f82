// pb_cg_generic.hip -- CG iteration kernels for operators / preconditioners without a fused
// stencil engine (the compact Laplacian as A, SOR / multigrid as PC). Same device-resident scalar
// logic (cg_finalize_kernel in pb_stencil.hip) as the fused 7-point path.
#include "pb_internal.hpp"

// ---------------------------------------------------------------------------------------------
// Generic CG iteration for operators without a fused stencil engine (the compact Laplacian):
//   p = (dinv*r - mu) + bb*p ; w = A p ; p.w ; x += a p ; r += (-a) w ; residual sums
// Same device-resident scalar logic (cg_finalize_kernel) as the fused 7-point path.
// ---------------------------------------------------------------------------------------------
namespace pb {

template <int NS>
__device__ __forceinline__ void block_sums(double* acc, double* parts) {
  __shared__ double red[4][NS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    double v = acc[s];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane == 0) red[wid][s] = v;
  }
  __syncthreads();
  if (threadIdx.x < NS)
    parts[(int64_t)blockIdx.x * NS + threadIdx.x] =
        ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

// first (the solve's first iteration, KSPSolve_CG's VecCopy(Z, P)): p = z, p_old is not read
// (it is not initialised: the stored-z setup skips the p = 0 pass)
__global__ __launch_bounds__(256) void cg_gen_p_kernel(const double* __restrict__ r, double* p,
                                                       int64_t n, const CgState* st, int first) {
  if (st->done) return;
  const double dinv = st->dinv, shift = -st->mu;
  const double bb = st->it == 0 ? 0.0 : st->beta / st->betaold;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double z = dinv * r[i];
    z = z + shift;
    p[i] = first ? z : z + bb * p[i];
  }
}

__global__ __launch_bounds__(256) void cg_gen_dot_kernel(const double* __restrict__ p,
                                                         const double* __restrict__ w, int64_t n,
                                                         double* parts, const CgState* st) {
  if (st->done) return;
  double acc[1] = {0.0};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    acc[0] += w[i] * p[i];
  block_sums<1>(acc, parts);
}

__global__ __launch_bounds__(256) void cg_gen_xr_kernel(const double* __restrict__ p,
                                                        const double* __restrict__ w, double* x,
                                                        double* r, int64_t n, double* parts,
                                                        const CgState* st) {
  if (st->done) return;
  const double a = st->alpha, dinv = st->dinv, mu = st->mu;
  double acc[4] = {0, 0, 0, 0};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    x[i] = x[i] + a * p[i];
    const double rv = r[i] + (-a) * w[i];
    r[i] = rv;
    const double t = dinv * rv - mu;
    acc[0] += t;
    acc[1] += t * t;
    acc[2] += t * rv;
    acc[3] += rv;
  }
  block_sums<4>(acc, parts);
}

// preconditioned path (z = M^-1 r from SOR / MG / FFT): x += a p ; r = r_in + (-a) w, no sums.
// first: x0 = 0 is implicit (x = a p, x not read) and r_in = b (r0 = b - A x0 = b, not copied);
// a breakdown before the update leaves x = x0 = 0
__global__ __launch_bounds__(256) void cg_pc_xr_kernel(const double* __restrict__ p,
                                                       const double* __restrict__ w, double* x,
                                                       const double* r_in, double* r, int64_t n,
                                                       const CgState* st, int first) {
  const bool done = st->done;
  if (done && !first) return;
  const double a = st->alpha;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (done) {
      x[i] = 0.0;
      continue;
    }
    x[i] = first ? a * p[i] : x[i] + a * p[i];
    r[i] = r_in[i] + (-a) * w[i];
  }
}

// sums of t = z - mu_old (t, t^2, t.r) and of r, for the null-space-projected ||z|| and z.r
// (same shifted-sum algebra as the fused pass B; at setup mu_old = 0)
__global__ __launch_bounds__(256) void cg_pc_sums_kernel(const double* __restrict__ z,
                                                         const double* __restrict__ r, int64_t n,
                                                         double* parts, const CgState* st) {
  const double mu = st->mu;
  double acc[4] = {0, 0, 0, 0};
  if (!st->done) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
      const double rv = r[i];
      const double t = z[i] - mu;
      acc[0] += t;
      acc[1] += t * t;
      acc[2] += t * rv;
      acc[3] += rv;
    }
  }
  block_sums<4>(acc, parts);
}

static int gen_blocks(pb_ctx* ctx, int64_t n) {
  int64_t b = (n + 255) / 256;
  const int64_t cap = (int64_t)ctx->num_cus * 8;
  return (int)(b > cap ? cap : (b < 1 ? 1 : b));
}

int launch_cg_generic_p(pb_grid* g, const double* r, double* p, CgState* st, int first) {
  const int nb = gen_blocks(g->ctx, g->nlocal);
  hipLaunchKernelGGL(cg_gen_p_kernel, dim3(nb), dim3(256), 0, g->ctx->stream, r, p, g->nlocal,
                     (const CgState*)st, first);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

int launch_cg_generic_dot(pb_grid* g, const double* p, const double* w, CgState* st, int* nparts) {
  const int nb = gen_blocks(g->ctx, g->nlocal);
  hipLaunchKernelGGL(cg_gen_dot_kernel, dim3(nb), dim3(256), 0, g->ctx->stream, p, w, g->nlocal,
                     g->ctx->d_partials, (const CgState*)st);
  PB_HIP(hipGetLastError());
  *nparts = nb;
  return PB_OK;
}

int launch_cg_generic_xr(pb_grid* g, const double* p, const double* w, double* x, double* r,
                         CgState* st, int* nparts) {
  const int nb = gen_blocks(g->ctx, g->nlocal);
  hipLaunchKernelGGL(cg_gen_xr_kernel, dim3(nb), dim3(256), 0, g->ctx->stream, p, w, x, r,
                     g->nlocal, g->ctx->d_partials, (const CgState*)st);
  PB_HIP(hipGetLastError());
  *nparts = nb;
  return PB_OK;
}

int launch_cg_pc_xr(pb_grid* g, const double* p, const double* w, double* x, const double* r_in,
                    double* r, CgState* st, int first) {
  const int nb = gen_blocks(g->ctx, g->nlocal);
  hipLaunchKernelGGL(cg_pc_xr_kernel, dim3(nb), dim3(256), 0, g->ctx->stream, p, w, x, r_in, r,
                     g->nlocal, (const CgState*)st, first);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

int launch_cg_pc_sums(pb_grid* g, const double* z, const double* r, CgState* st, int* nparts) {
  const int nb = gen_blocks(g->ctx, g->nlocal);
  hipLaunchKernelGGL(cg_pc_sums_kernel, dim3(nb), dim3(256), 0, g->ctx->stream, z, r, g->nlocal,
                     g->ctx->d_partials, (const CgState*)st);
  PB_HIP(hipGetLastError());
  *nparts = nb;
  return PB_OK;
}

}  // namespace pb

