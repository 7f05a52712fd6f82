// pb_cg_sr.hip -- the single-reduction CG iteration (PETSc KSPSolve_CG_SingleReduction,
// -ksp_cg_single_reduction) as ONE pass over the grid per iteration (one rank).
//
// The two-pass form (pb_stencil.hip: pass P forms p, w = A p and r' = r - alpha w; pass S forms
// t = dinv r' - mu and s = A t for the sums) reads r' a second time. Here one z-march does both:
// a wave forms p one plane ahead of w and w one plane ahead of s,
//   step k:  p(k+2) = (dinv r - mu) + b p_old          (pointwise, stored)
//            w(k+1) = A p   -> r'(k+1) = r - alpha w     (stored), t(k+1) = dinv r' - mu
//            s(k)   = A t   -> sums t, t^2, t.r', r' (plane k+1) and t.s (plane k)
// so per point it reads r, p_old and writes p, r': 32 B/DoF, the single-reduction floor without
// the x update (the iterations that carry the deferred x update run the two passes).
//
// The stencils at a wave's tile edges need p and t one point outside it. Rows: a block stacks NW
// waves of TY rows, each wave forms every stage on its own rows only, and the values one row
// out come from the neighbouring waves through LDS (published one step before use, double
// buffered by step parity, one block barrier per step); each stage loses a row at the block's
// ends, so blocks store rows 2 .. NW TY - 3 and advance by NW TY - 4 rows. Columns: a wave spans
// 64 pairs but owns lanes 4..59 (112 points), so every x-neighbour is a DPP lane shift. Work is
// split evenly over one workgroup per CU (bands of W planes of every column, then the last band's
// column-planes cut into pieces of W), each z-range warming up four planes below its start.
//
// Per-point arithmetic is pass P's and pass S's (CombineLoad, PassB<., true, false>, ZLoad,
// SrSums: reference summation order, no FMA contraction), so p, r' and every summand are
// bit-identical to the two-pass iteration; only the blocks the sums are taken over differ.
#include <type_traits>

#include "pb_cg_device.hpp"

namespace pb {

// outputs per wave segment: lanes 4 .. 59 (pairs), 896 B = seven whole 128-B lines, so no line
// is written by two waves (segments of 124 points -- lanes 1 .. 62 -- wrote partial lines at both
// ends and ran 1.07-1.16 ms at 512^3 against the 112-point segments' same segment count)
static constexpr int kSrSegOut = 112, kSrLead = 4;

struct SrGeo {
  int nx, ny, nzl;
  int64_t plane;
  int nseg, ntile;  // x segments of kSrSegOut points, y tiles of NW TY - 4 rows
  int W;            // planes of work per workgroup
  int remap, nt;
};

// the deferred solution update on the iterations that carry it (depth 4, i % 4 = 3), PassB<3>'s
// arithmetic: x += a3 p_{i-3} + a2 p_{i-2} + a1 p_{i-1} + alpha p_i, as p_i is formed
struct SrX {
  double* x;
  const double* pm2;  // p_{i-2}
  const double* pm3;  // p_{i-3}
};

template <int NW, int TY, bool XU>
__device__ __forceinline__ void sr1_range(const SrGeo& g, double cx, double cy, double cz,
                                          double cc, const double* __restrict__ r,
                                          const double* __restrict__ p_old,
                                          double* __restrict__ p_new, double* __restrict__ r_out,
                                          double dinv, double shift, double bb, double alpha,
                                          const SrX& xu, const double (&xa)[3], int seg,
                                          int tile, int kb, int ke,
                                          dv2 (&xch)[2][4][NW][64], double (&acc)[5]) {
  constexpr int RB = NW * TY;
  constexpr int SB = RB - 4;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nx = g.nx, ny = g.ny, nz = g.nzl;
  const int g0 = tile * SB - 2;  // global row of block row 0
  const int br0 = wid * TY;
  const int j0 = g0 + br0;
  auto wrap = [](int v, int n) { v %= n; return v < 0 ? v + n : v; };
  const int o = seg * kSrSegOut + 2 * (lane - kSrLead);  // this lane's pair (output index)
  const int ip = wrap(o, nx);  // (nx even: a pair never straddles the wrap)
  const bool out_ok = lane >= kSrLead && lane < kSrLead + kSrSegOut / 2 && o < nx;
  int64_t ro[TY];
  unsigned row_ok = 0;
#pragma unroll
  for (int q = 0; q < TY; ++q) {
    ro[q] = (int64_t)wrap(j0 + q, ny) * nx;
    const int brow = br0 + q;
    if (out_ok && brow >= 2 && brow < RB - 2 && g0 + brow < ny) row_ok |= 1u << q;
  }
  const unsigned boff = (unsigned)ip * 8u;
  auto rix = [&](int64_t row) { return RowIx{row, boff}; };
  auto pl = [&](int kk) -> int64_t { return (int64_t)wrap(kk, nz) * g.plane; };
  const int wm = wid > 0 ? wid - 1 : wid, wp = wid < NW - 1 ? wid + 1 : wid;

  // rings of four register slots whose roles rotate with the unrolled step (no copies):
  double P[4][TY][2];   // p of planes k, k+1, k+2 at slots Q, Q+1, Q+2
  double R[4][TY][2];   // r of planes k+1 .. k+3 at slots Q+1 .. Q+3; slot Q receives plane k+4
  double T[4][TY][2];   // t of planes k-1, k, k+1 at slots Q, Q+1, Q+2
  double PO[4][TY][2];  // p_old of planes k+2, k+3 at slots Q+2, Q+3; slot Q receives k+4
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int q = 0; q < TY; ++q)
#pragma unroll
      for (int e = 0; e < 2; ++e) P[s][q][e] = R[s][q][e] = T[s][q][e] = PO[s][q][e] = 0.0;
  auto ld = [&](const double* src, int kk, double (&dst)[TY][2]) {
    const int64_t base = pl(kk);
#pragma unroll
    for (int q = 0; q < TY; ++q) load_row<2>(src, rix(base + ro[q]), dst[q]);
  };
  // the first step (k = kb - 4, Q = 0) forms p(kb - 2); plane kb - 1 is in flight
  ld(r, kb - 2, R[2]);
  ld(p_old, kb - 2, PO[2]);
  ld(r, kb - 1, R[3]);
  ld(p_old, kb - 1, PO[3]);

  auto body = [&](auto Qc, int k) {
    constexpr int Q = decltype(Qc)::value;
    double (&pk)[TY][2] = P[Q];
    double (&pk1)[TY][2] = P[(Q + 1) & 3];
    double (&pk2)[TY][2] = P[(Q + 2) & 3];
    double (&rk1)[TY][2] = R[(Q + 1) & 3];
    double (&rk2)[TY][2] = R[(Q + 2) & 3];
    double (&tkm)[TY][2] = T[Q];
    double (&tk)[TY][2] = T[(Q + 1) & 3];
    double (&tk1)[TY][2] = T[(Q + 2) & 3];
    // planes k+4 in flight for two steps (plane k+3's loads are already on their way)
    ld(r, k + 4, R[Q]);
    ld(p_old, k + 4, PO[Q]);
    // x-update operands of plane k+2 (consumed at the end of this step)
    double XX[XU ? TY : 1][2], M2[XU ? TY : 1][2], M3[XU ? TY : 1][2];
    if constexpr (XU) {
      ld(xu.x, k + 2, XX);
      ld(xu.pm2, k + 2, M2);
      ld(xu.pm3, k + 2, M3);
    }
    // p(k+2) = (dinv r - mu) + b p_old (CombineLoad::f)
#pragma unroll
    for (int q = 0; q < TY; ++q)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        double z = dinv * rk2[q][e];
        z = z + shift;
        pk2[q][e] = z + bb * PO[(Q + 2) & 3][q][e];
      }
    __syncthreads();
    // rows -1 / TY of p(k+1) and t(k): published by the neighbouring waves at step k-1
    const int rp = (k + 1) & 1, cur = k & 1;
    const dv2 phl = xch[rp][1][wm][lane], phh = xch[rp][0][wp][lane];
    const dv2 thl = xch[rp][3][wm][lane], thh = xch[rp][2][wp][lane];
    xch[cur][0][wid][lane] = dv2{pk2[0][0], pk2[0][1]};
    xch[cur][1][wid][lane] = dv2{pk2[TY - 1][0], pk2[TY - 1][1]};
    const bool in2 = k + 2 >= kb && k + 2 < ke, in1 = k + 1 >= kb && k + 1 < ke,
               in0 = k >= kb && k < ke;
    if (in2) {
      const int64_t base = pl(k + 2);
#pragma unroll
      for (int q = 0; q < TY; ++q)
        if (row_ok >> q & 1u) store_row<2>(p_new, rix(base + ro[q]), pk2[q], g.nt);
    }
    // w(k+1) = A p (z-, y-, x-, c, x+, y+, z+), r' = r - alpha w, t = dinv r' - mu
    const int64_t base1 = pl(k + 1);
#pragma unroll
    for (int q = 0; q < TY; ++q) {
      const double lo = dpp_from_lower(pk1[q][1]);
      const double hi = dpp_from_upper(pk1[q][0]);
      double rv[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const double xm = e == 0 ? lo : pk1[q][0];
        const double xp = e == 1 ? hi : pk1[q][1];
        const double ym = q == 0 ? phl[e] : pk1[q == 0 ? 0 : q - 1][e];
        const double yp = q == TY - 1 ? phh[e] : pk1[q == TY - 1 ? q : q + 1][e];
        double w = cz * pk[q][e];
        w = w + cy * ym;
        w = w + cx * xm;
        w = w + cc * pk1[q][e];
        w = w + cx * xp;
        w = w + cy * yp;
        w = w + cz * pk2[q][e];
        rv[e] = rk1[q][e] + (-alpha) * w;
        double z = dinv * rv[e];
        tk1[q][e] = z + shift;
      }
      if (in1 && (row_ok >> q & 1u)) {
        store_row<2>(r_out, rix(base1 + ro[q]), rv, g.nt);
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const double t = tk1[q][e];
          acc[0] += t;
          acc[1] += t * t;
          acc[2] += t * rv[e];
          acc[3] += rv[e];
        }
      }
    }
    xch[cur][2][wid][lane] = dv2{tk1[0][0], tk1[0][1]};
    xch[cur][3][wid][lane] = dv2{tk1[TY - 1][0], tk1[TY - 1][1]};
    // s(k) = A t, delta sum t.s
    if (in0) {
#pragma unroll
      for (int q = 0; q < TY; ++q) {
        const double lo = dpp_from_lower(tk[q][1]);
        const double hi = dpp_from_upper(tk[q][0]);
        if (row_ok >> q & 1u) {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const double xm = e == 0 ? lo : tk[q][0];
            const double xp = e == 1 ? hi : tk[q][1];
            const double ym = q == 0 ? thl[e] : tk[q == 0 ? 0 : q - 1][e];
            const double yp = q == TY - 1 ? thh[e] : tk[q == TY - 1 ? q : q + 1][e];
            double sv = cz * tkm[q][e];
            sv = sv + cy * ym;
            sv = sv + cx * xm;
            sv = sv + cc * tk[q][e];
            sv = sv + cx * xp;
            sv = sv + cy * yp;
            sv = sv + cz * tk1[q][e];
            acc[4] += tk[q][e] * sv;
          }
        }
      }
    }
    if constexpr (XU) {  // x(k+2) += a3 p_{i-3} + a2 p_{i-2} + a1 p_{i-1} + alpha p_i
      if (in2) {
        const int64_t base = pl(k + 2);
#pragma unroll
        for (int q = 0; q < TY; ++q) {
          double xv[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            double u = xa[0] * M3[q][e];
            u = u + xa[1] * M2[q][e];
            u = u + xa[2] * PO[(Q + 2) & 3][q][e];
            u = u + alpha * pk2[q][e];
            xv[e] = XX[q][e] + u;
          }
          if (row_ok >> q & 1u) store_row<2>(xu.x, rix(base + ro[q]), xv, g.nt);
        }
      }
    }
  };
  // steps kb-4 .. ke-1 (padded to whole four-step rounds: the spare steps store and sum nothing)
#pragma unroll 1
  for (int k = kb - 4; k < ke; k += 4) {
    body(std::integral_constant<int, 0>{}, k);
    body(std::integral_constant<int, 1>{}, k + 1);
    body(std::integral_constant<int, 2>{}, k + 2);
    body(std::integral_constant<int, 3>{}, k + 3);
  }
}

template <int NW, int TY, bool XU>
__global__ __launch_bounds__(64 * NW) void cg_sr1_kernel(SrGeo g, double cx, double cy, double cz,
                                                         double cc, const double* __restrict__ r,
                                                         const double* __restrict__ p_old,
                                                         double* __restrict__ p_new,
                                                         double* __restrict__ r_out, SrX xu,
                                                         double* parts, Fold fold) {
  __shared__ dv2 xch[2][4][NW][64];
  CgState st;
  fold_prologue(fold, st);  // every wave: the previous residual-sum stage + this iteration's top
  if (st.done) return;      // (uniform: every wave computed the same state)
  const double dinv = st.dinv, shift = -st.mu, bb = st.bbp, alpha = st.alpha;
  const double xa[3] = {st.pa[0], st.pa[1], st.pa[2]};  // pending alphas of i-3, i-2, i-1
  double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  const int bid = xcd_block(g.remap);
  const int ncol = g.nseg * g.ntile, W = g.W, T = g.nzl / W;
  auto run = [&](int col, int kb, int ke) {
    sr1_range<NW, TY, XU>(g, cx, cy, cz, cc, r, p_old, p_new, r_out, dinv, shift, bb, alpha, xu,
                          xa, col % g.nseg, col / g.nseg, kb, ke, xch, acc);
  };
  if (bid < T * ncol) {  // bands of W planes of every column
    const int kb = (bid / ncol) * W;
    run(bid % ncol, kb, kb + W);
  } else {  // the last band [T W, nzl) of all columns end to end, in pieces of W
    const int k0 = T * W, h = g.nzl - k0;
    if (h > 0) {
      const int64_t total = (int64_t)ncol * h;
      const int64_t e = min(total, (int64_t)(bid - T * ncol + 1) * W);
      for (int64_t s = (int64_t)(bid - T * ncol) * W; s < e;) {
        const int col = (int)(s / h);
        const int kb = (int)(s - (int64_t)col * h);
        const int ke = (int)min((int64_t)h, kb + (e - s));
        run(col, k0 + kb, k0 + ke);
        s += ke - kb;
        __syncthreads();  // the next range rewrites the exchange slots
      }
    }
  }
  block_partials<5>(acc, parts);
}


bool cg_sr1_supported(const pb_grid* g) {
  return !g->ctx->split && g->n[0] % 2 == 0 && tune("cg_sr_fused", 1) != 0;
}

template <int NW, int TY>
static int launch_sr1_t(pb_grid* g, const Star& s, const double* r, const double* p_old,
                        double* p_new, double* r_out, const SrX* xu, const SrFold& sf,
                        const double* parts_in, double* parts_out, int64_t host_iter,
                        int* nblocks) {
  pb_ctx* ctx = g->ctx;
  SrGeo geo;
  geo.nx = (int)g->n[0];
  geo.ny = (int)g->n[1];
  geo.nzl = (int)g->nzl;
  geo.plane = g->plane;
  geo.nseg = (geo.nx + kSrSegOut - 1) / kSrSegOut;
  geo.ntile = (geo.ny + NW * TY - 5) / (NW * TY - 4);
  geo.remap = 1;
  geo.nt = 1;
  const int64_t work = (int64_t)geo.nseg * geo.ntile * geo.nzl;  // column-planes
  const int64_t want = (int64_t)(ctx->num_cus);
  geo.W = (int)std::max<int64_t>(1, (work + want - 1) / want);
  const int64_t nb = (work + geo.W - 1) / geo.W;
  if (nb * 5 > ctx->partials_cap / 2)
    return set_error(PB_ERR_UNSUPPORTED, "single-reduction pass of %lld blocks", (long long)nb);
  Fold f;
  f.stage = sf.fold_sums ? 3 : 4;
  f.nparts = sf.nparts_s;
  f.width = 5;
  f.parts = parts_in;
  f.in = sf.in;
  f.out = sf.out;
  f.hist = sf.hist;
  f.h_done = sf.h_done;
  f.host_iter = host_iter - 1;
  if (xu)
    hipLaunchKernelGGL((cg_sr1_kernel<NW, TY, true>), dim3((unsigned)nb), dim3(64 * NW), 0,
                       ctx->stream, geo, s.cx, s.cy, s.cz, s.cc, r, p_old, p_new, r_out, *xu,
                       parts_out, f);
  else
    hipLaunchKernelGGL((cg_sr1_kernel<NW, TY, false>), dim3((unsigned)nb), dim3(64 * NW), 0,
                       ctx->stream, geo, s.cx, s.cy, s.cz, s.cc, r, p_old, p_new, r_out,
                       SrX{nullptr, nullptr, nullptr}, parts_out, f);
  PB_HIP(hipGetLastError());
  *nblocks = (int)nb;
  return PB_OK;
}

int launch_cg_sr1(pb_grid* g, const Star& s, const double* r, const double* p_old,
                  double* p_new, double* r_out, double* x, const double* p_m2, const double* p_m3,
                  const SrFold& sf, const double* parts_in, double* parts_out, int64_t host_iter,
                  int* nblocks) {
  ScopedTimer tm(g->ctx, x ? "cg_sr1_x4" : "cg_sr1");
  const SrX xv{x, p_m2, p_m3};
  const SrX* xu = x ? &xv : nullptr;
  switch (tune("cg_sr_shape", 0)) {
    case 1:  // 12 waves of 2 rows: three waves per SIMD
      return launch_sr1_t<12, 2>(g, s, r, p_old, p_new, r_out, xu, sf, parts_in, parts_out,
                                 host_iter, nblocks);
    case 3:
      return launch_sr1_t<8, 3>(g, s, r, p_old, p_new, r_out, xu, sf, parts_in, parts_out,
                                host_iter, nblocks);
    default:  // 8 waves of 2 rows: two waves per SIMD
      return launch_sr1_t<8, 2>(g, s, r, p_old, p_new, r_out, xu, sf, parts_in, parts_out,
                                host_iter, nblocks);
  }
}

}  // namespace pb
