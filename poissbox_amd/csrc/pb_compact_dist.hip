// pb_compact_dist.hip -- the compact Laplacian's Z pass on a z-slab decomposition.
//
// z-lines span every rank's slab, and the (alpha, 1, alpha) inverses couple whole lines (their
// kernels decay like (1/3)^|k|, ~34 planes to 1e-16: SURVEY.md §7 "compact scheme across GPUs"),
// so the Z pass runs on transposed data: rank r owns rows j in [j0_r, j0_r + nyl_r) of every
// plane (a y-slab with complete z-lines, same balanced split as the z-slabs, README.md:30-32).
//   f (z-slab) --pack--> send --alltoallv--> fy (y-slab, lands in place: blocks from rank s are
//   the planes k0_s .. k0_s + nzl_s - 1 of the y-slab)  --Z pass--> uy, vy
//   uy, vy (y-slab) --alltoallv--> recv --unpack--> u, v (z-slab)
// The Y and X passes are local to the z-slab. Exchange volume: 3 fields (24 B/DoF) per apply, as
// grouped ncclSend/ncclRecv on RCCL contexts or the host alltoallv callback in tests.
#include <vector>

#include "pb_internal.hpp"

namespace pb {

// z-slab [kl][j][i] -> send buffer: block of rank r = [kl][jl][i] for j in [j0_r, j0_r + nyl_r),
// blocks in rank order (offset nzl * nx * j0_r). dir = 0: pack (zs -> buf), 1: unpack.
__global__ __launch_bounds__(256) void slab_transpose_kernel(double* zs, double* buf, int nx,
                                                             int ny, int nzl, const int* jrank,
                                                             const int* j0, const int* nyl,
                                                             int dir) {
  const int64_t n = (int64_t)nx * ny * nzl;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t u = (uint32_t)idx;
    const uint32_t row = u / (uint32_t)nx;
    const int i = (int)(u - row * (uint32_t)nx);
    const int kl = (int)(row / (uint32_t)ny);
    const int j = (int)(row - (uint32_t)kl * (uint32_t)ny);
    const int r = jrank[j];
    const int64_t b = (int64_t)nzl * nx * j0[r] + ((int64_t)kl * nyl[r] + (j - j0[r])) * nx + i;
    if (dir == 0)
      buf[b] = zs[idx];
    else
      zs[idx] = buf[b];
  }
}

struct DistPlan {
  std::vector<int64_t> k0, nzl, j0, nyl;
  int64_t ny_me = 0;
};

static DistPlan make_plan(const pb_grid* g) {
  const int P = g->ctx->nranks;
  DistPlan d;
  d.k0.resize(P);
  d.nzl.resize(P);
  d.j0.resize(P);
  d.nyl.resize(P);
  for (int r = 0; r < P; ++r) {
    pb_slab_partition(g->n[2], P, r, &d.k0[r], &d.nzl[r]);
    pb_slab_partition(g->n[1], P, r, &d.j0[r], &d.nyl[r]);
  }
  d.ny_me = d.nyl[g->ctx->rank];
  return d;
}

// y-slab fields fy, uy, vy (3 * nx * nyl * nz), staging (max of the two slab sizes), and the
// small rank tables (j -> rank, j0, nyl) as doubles-sized slots
int64_t compact_dist_work_len(const pb_grid* g) {
  const DistPlan d = make_plan(g);
  const int64_t ny_slab = g->n[0] * d.ny_me * g->n[2];
  const int64_t tables = (g->n[1] + 2 * g->ctx->nranks + 1) / 2 + 1;
  return 3 * ny_slab + std::max<int64_t>(ny_slab, g->nlocal) + tables;
}

int compact_dist_pass_z(pb_grid* g, double h, const double* f, double* u, double* v, double* work) {
  pb_ctx* ctx = g->ctx;
  const int P = ctx->nranks, me = ctx->rank;
  if (g->n[1] < P) return set_error(PB_ERR_UNSUPPORTED, "compact operator: ny < ranks");
  const DistPlan d = make_plan(g);
  const int64_t nx = g->n[0], ny = g->n[1], nz = g->n[2];
  const int64_t ny_slab = nx * d.ny_me * nz;
  double* fy = work;
  double* uy = fy + ny_slab;
  double* vy = uy + ny_slab;
  double* stage = vy + ny_slab;
  int* tab = (int*)(stage + std::max<int64_t>(ny_slab, g->nlocal));
  // rank tables (tiny, uploaded per call on the stream)
  std::vector<int> htab(ny + 2 * P);
  for (int r = 0; r < P; ++r) {
    for (int64_t j = d.j0[r]; j < d.j0[r] + d.nyl[r]; ++j) htab[j] = r;
    htab[ny + r] = (int)d.j0[r];
    htab[ny + P + r] = (int)d.nyl[r];
  }
  PB_HIP(hipMemcpyAsync(tab, htab.data(), htab.size() * sizeof(int), hipMemcpyHostToDevice,
                        ctx->stream));
  std::vector<int64_t> zc(P), yc(P);  // z-slab block for rank p; y-slab block from rank p
  for (int p = 0; p < P; ++p) {
    zc[p] = g->nzl * nx * d.nyl[p];
    yc[p] = d.nzl[p] * nx * d.ny_me;
  }
  const int nb = (int)std::min<int64_t>((g->nlocal + 255) / 256, (int64_t)ctx->num_cus * 16);
  hipLaunchKernelGGL(slab_transpose_kernel, dim3(nb), dim3(256), 0, ctx->stream,
                     const_cast<double*>(f), stage, (int)nx, (int)ny, (int)g->nzl, tab, tab + ny,
                     tab + ny + P, 0);
  PB_HIP(hipGetLastError());
  PB_SYNC(ctx, "compact transpose");  // htab stays valid until the copy is done
  PB_TRY(alltoallv_device(ctx, stage, zc.data(), fy, yc.data()));
  const int64_t dy[3] = {nx, d.ny_me, nz};
  PB_TRY(compact_pass_z(ctx, dy, h, fy, uy, vy));
  for (int f2 = 0; f2 < 2; ++f2) {
    PB_TRY(alltoallv_device(ctx, f2 ? vy : uy, yc.data(), stage, zc.data()));
    hipLaunchKernelGGL(slab_transpose_kernel, dim3(nb), dim3(256), 0, ctx->stream, f2 ? v : u,
                       stage, (int)nx, (int)ny, (int)g->nzl, tab, tab + ny, tab + ny + P, 1);
    PB_HIP(hipGetLastError());
  }
  (void)me;
  return PB_OK;
}

}  // namespace pb
