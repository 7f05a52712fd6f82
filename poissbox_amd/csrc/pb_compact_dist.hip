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

#include "pb_device.hpp"

namespace pb {

// z-slab [kl][j][i] -> send buffer: block of rank r = [kl][jl][i] for j in [j0_r, j0_r + nyl_r),
// blocks in rank order (offset nzl * nx * j0_r). dir = 0: pack (zs -> buf), 1: unpack.
__global__ __launch_bounds__(256) void slab_transpose_kernel(double* zs, double* buf, int nx,
                                                             int ny, int nzl, const int* jrank,
                                                             const int* j0, const int* nyl,
                                                             int dir, int me, double* self) {
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
    double* bb = self && r == me ? self : buf;  // the self block: straight to / from the y-slab
    if (dir == 0)
      bb[b] = zs[idx];
    else
      zs[idx] = bb[b];
  }
}

// The same permutation by rows (even nx): row (kl, j) of the z-slab is one contiguous run of nx
// doubles in its rank's block, so a thread moves 16-byte pairs of a row and the rank lookup and
// index arithmetic are done once per row instead of once per element (force_comm 512^3 pack /
// unpack: the per-element kernel moved ~3.4 TB/s).
// cz (pack only, CG on a split grid, CgFuse::z): the packed field is CG's direction formed on the
// way, p = (dinv z - mu) + beta/beta_old p_old with p_old = zs (cg_gen_p_kernel's arithmetic, bit
// for bit), and it is also stored back into zs; with the state's done flag set zs is packed as is
struct PackP {
  const double* cz = nullptr;
  const CgState* st = nullptr;
  int first = 0;
};
__global__ __launch_bounds__(256) void slab_rows_kernel(double* zs, double* buf, int nx, int ny,
                                                        int nzl, const int* jrank, const int* j0,
                                                        const int* nyl, int dir, int me,
                                                        double* self, PackP pp) {
  const bool form_p = pp.cz && !pp.st->done;  // (uniform)
  double dinv = 1.0, shift = 0.0, bbp = 0.0;
  if (form_p) {
    dinv = pp.st->dinv;
    shift = -pp.st->mu;
    bbp = pp.st->it == 0 ? 0.0 : pp.st->beta / pp.st->betaold;
  }
  const int hp = nx >> 1;                              // pairs per row
  const int step = hp < 256 ? hp : 256;                // pair stride of a thread within its row
  const int rpb = hp < 256 ? 256 / hp : 1;             // rows per block step
  const int rin = (int)threadIdx.x / step, p0 = (int)threadIdx.x - rin * step;
  const int64_t nrows = (int64_t)nzl * ny;
  if (rin >= rpb) return;
  for (int64_t row = (int64_t)blockIdx.x * rpb + rin; row < nrows;
       row += (int64_t)gridDim.x * rpb) {
    const int kl = (int)(row / ny), j = (int)(row - (int64_t)kl * ny);
    const int r = jrank[j];
    const int64_t b = (int64_t)nzl * nx * j0[r] + ((int64_t)kl * nyl[r] + (j - j0[r])) * nx;
    const int64_t a = row * nx;
    double* bb = self && r == me ? self : buf;  // the self block: straight to / from the y-slab
    for (int q = p0; q < hp; q += step) {
      if (dir == 0 && form_p) {
        const dv2 zv = *reinterpret_cast<const dv2*>(pp.cz + a + 2 * q);
        const dv2 po = *reinterpret_cast<const dv2*>(zs + a + 2 * q);
        dv2 pv;
        double z0 = dinv * zv.x, z1 = dinv * zv.y;
        z0 = z0 + shift;
        z1 = z1 + shift;
        pv.x = pp.first ? z0 : z0 + bbp * po.x;
        pv.y = pp.first ? z1 : z1 + bbp * po.y;
        *reinterpret_cast<dv2*>(zs + a + 2 * q) = pv;
        *reinterpret_cast<dv2*>(bb + b + 2 * q) = pv;
      } else if (dir == 0)
        *reinterpret_cast<dv2*>(bb + b + 2 * q) = *reinterpret_cast<const dv2*>(zs + a + 2 * q);
      else
        *reinterpret_cast<dv2*>(zs + a + 2 * q) = *reinterpret_cast<const dv2*>(bb + b + 2 * q);
    }
  }
}

// ybuf: the y-slab buffer on the other side of the all-to-all (its self block is read / written
// here directly when p.self_direct)
// pp.cz: the pack forms CG's p on the way (even nx only; the caller checks)
static void launch_slab_transpose(pb_grid* g, const YSlabPlan& p, double* zs, int dir,
                                  const double* ybuf, const PackP& pp = PackP{}) {
  pb_ctx* ctx = g->ctx;
  double* self = p.self_direct ? const_cast<double*>(ybuf) + p.self_shift : nullptr;
  const int64_t ny = g->n[1];
  const int P = ctx->nranks;
  if (g->n[0] % 2 == 0) {
    const int64_t rows = g->nzl * ny;
    const int hp = (int)(g->n[0] / 2), rpb = hp < 256 ? 256 / hp : 1;
    const int nb = (int)std::min<int64_t>((rows + rpb - 1) / rpb, (int64_t)ctx->num_cus * 16);
    hipLaunchKernelGGL(slab_rows_kernel, dim3(nb), dim3(256), 0, ctx->stream, zs, p.stage,
                       (int)g->n[0], (int)ny, (int)g->nzl, p.tab, p.tab + ny, p.tab + ny + P, dir,
                       p.me, self, pp);
    return;
  }
  hipLaunchKernelGGL(slab_transpose_kernel, dim3(p.nb), dim3(256), 0, ctx->stream, zs, p.stage,
                     (int)g->n[0], (int)ny, (int)g->nzl, p.tab, p.tab + ny, p.tab + ny + P, dir,
                     p.me, self);
}

static void make_plan(const pb_grid* g, YSlabPlan* d) {
  const int P = g->ctx->nranks;
  d->k0.resize(P);
  d->nzl.resize(P);
  d->j0.resize(P);
  d->nyl.resize(P);
  for (int r = 0; r < P; ++r) {
    pb_slab_partition(g->n[2], P, r, &d->k0[r], &d->nzl[r]);
    pb_slab_partition(g->n[1], P, r, &d->j0[r], &d->nyl[r]);
  }
  d->ny_me = d->nyl[g->ctx->rank];
  d->ny_slab = g->n[0] * d->ny_me * g->n[2];
}

int64_t yslab_len(const pb_grid* g) {
  YSlabPlan d;
  make_plan(g, &d);
  return d.ny_slab;
}

// staging: the larger of the two slab sizes (the rank tables live with the grid)
int64_t yslab_aux_len(const pb_grid* g) { return std::max<int64_t>(yslab_len(g), g->nlocal); }

int yslab_begin(pb_grid* g, double* aux, YSlabPlan* p) {
  pb_ctx* ctx = g->ctx;
  const int P = ctx->nranks;
  if (g->n[1] < P) return set_error(PB_ERR_UNSUPPORTED, "compact operators: ny < ranks");
  make_plan(g, p);
  const int64_t nx = g->n[0], ny = g->n[1];
  p->stage = aux;
  if (!g->yslab_tab) {
    // rank tables: built and uploaded once per grid (they depend on the partition only)
    std::vector<int> htab(ny + 2 * P);
    for (int r = 0; r < P; ++r) {
      for (int64_t j = p->j0[r]; j < p->j0[r] + p->nyl[r]; ++j) htab[j] = r;
      htab[ny + r] = (int)p->j0[r];
      htab[ny + P + r] = (int)p->nyl[r];
    }
    int* tab = nullptr;
    if (hipMalloc(&tab, htab.size() * sizeof(int)) != hipSuccess)
      return set_error(PB_ERR_ALLOC, "y-slab rank tables: out of device memory");
    const hipError_t e =
        hipMemcpy(tab, htab.data(), htab.size() * sizeof(int), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      (void)hipFree(tab);
      return set_error(PB_ERR_HIP, "y-slab rank tables: %s", hipGetErrorString(e));
    }
    g->yslab_tab = tab;
  }
  p->tab = g->yslab_tab;
  p->zc.resize(P);  // z-slab block for rank q; y-slab block from rank q
  p->yc.resize(P);
  for (int q = 0; q < P; ++q) {
    p->zc[q] = g->nzl * nx * p->nyl[q];
    p->yc[q] = p->nzl[q] * nx * p->ny_me;
  }
  p->nb = (int)std::min<int64_t>((g->nlocal + 255) / 256, (int64_t)ctx->num_cus * 16);
  // the self block stays on the rank: the pack / unpack kernels read and write it in the y-slab
  // buffer directly and the all-to-all skips it (RCCL and, for the tests, the host transport)
  p->me = ctx->rank;
  p->self_direct = (ctx->comm != nullptr || P > 1) && !tune("a2a_copy_self", 0);
  int64_t zo = 0, yo = 0;
  for (int q = 0; q < ctx->rank; ++q) {
    zo += p->zc[q];
    yo += p->yc[q];
  }
  p->self_shift = yo - zo;
  return PB_OK;
}

bool yslab_blocked(const YSlabPlan& p) {
  const int64_t n = p.nyl.empty() ? 0 : p.nyl[0];
  if (n <= 0 || (n & (n - 1))) return false;
  for (int64_t v : p.nyl)
    if (v != n) return false;
  return true;
}

int yslab_to(pb_grid* g, const YSlabPlan& p, const double* f, double* fy, CgFuse* cf) {
  pb_ctx* ctx = g->ctx;
  {
    ScopedTimer tm(ctx, "slab_pack");
    PackP pp;
    if (cf && cf->z && g->n[0] % 2 == 0 && cf->p_old == f && cf->p_out == f) {
      pp.cz = cf->z;
      pp.st = cf->st;
      pp.first = cf->first;
    }
    launch_slab_transpose(g, p, const_cast<double*>(f), 0, fy, pp);
    PB_HIP(hipGetLastError());
    if (pp.cz) cf->fused_z = true;
  }
  return alltoallv_device(ctx, p.stage, p.zc.data(), fy, p.yc.data(), p.self_direct);
}

int yslab_from(pb_grid* g, const YSlabPlan& p, const double* fy, double* f) {
  pb_ctx* ctx = g->ctx;
  PB_TRY(alltoallv_device(ctx, fy, p.yc.data(), p.stage, p.zc.data(), p.self_direct));
  ScopedTimer tm(ctx, "slab_unpack");
  launch_slab_transpose(g, p, f, 1, fy);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

// y-slab fields fy, uy, vy and the transpose aux space
int64_t compact_dist_work_len(const pb_grid* g) { return 3 * yslab_len(g) + yslab_aux_len(g); }

int compact_dist_pass_z(pb_grid* g, double h, const double* f, double* u, double* v, double* work,
                        YSlabPlan* plan_out, bool* blocked) {
  const int64_t ny_slab = yslab_len(g);
  double* fy = work;
  double* uy = fy + ny_slab;
  double* vy = uy + ny_slab;
  YSlabPlan p;
  PB_TRY(yslab_begin(g, vy + ny_slab, &p));
  // CG on a split grid (CgFuse): p is formed by the pack; the y-slab Z pass must not form it
  // again, so the fusion is hidden from the passes until the transposes are done (the X pass
  // takes p . w)
  CgFuse* cf = g->ctx->cg_fuse;
  struct Hide {
    pb_ctx* c;
    CgFuse* f;
    ~Hide() { c->cg_fuse = f; }
  } hide{g->ctx, cf};
  g->ctx->cg_fuse = nullptr;
  PB_TRY(yslab_to(g, p, f, fy, cf));
  const int64_t dy[3] = {g->n[0], p.ny_me, g->n[2]};
  PB_TRY(compact_pass_z(g->ctx, dy, h, fy, uy, vy));
  if (blocked) *blocked = false;
  if (plan_out && blocked && yslab_blocked(p)) {
    // received straight into u, v (nlocal doubles each) in the all-to-all layout
    PB_TRY(alltoallv_device(g->ctx, uy, p.yc.data(), u, p.zc.data(), p.self_direct));
    PB_TRY(alltoallv_device(g->ctx, vy, p.yc.data(), v, p.zc.data(), p.self_direct));
    *plan_out = p;
    if (p.self_direct) {  // the Y pass reads the self block from uy, vy
      plan_out->alt0 = uy + p.self_shift;
      plan_out->alt1 = vy + p.self_shift;
    }
    *blocked = true;
    return PB_OK;
  }
  PB_TRY(yslab_from(g, p, uy, u));
  return yslab_from(g, p, vy, v);
}

}  // namespace pb
