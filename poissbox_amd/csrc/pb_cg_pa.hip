// pb_cg_pa.hip -- KSPSolve_CG's pass A on one rank as a ring-buffered z-march with the plane loads
// two steps ahead: p = (dinv r - mu) + b p_old formed on load (CombineLoad::f), w = A p, and the
// partial sums of p.w (PassAT<false>: read r and p_old, 16 B/DoF, nothing stored).
//
// The engine's pass A (pb_stencil.hip) runs one workgroup of 4 waves per CU -- one wave per SIMD --
// and loads each plane one step ahead; it spends 46 % of its wave cycles waiting on memory
// (SQ_WAIT_ANY; the pass B forms, bandwidth-bound, 14-17 %), and more workgroups per CU with
// shorter z-chunks ran slower. Here 8 waves of 2 rows (two waves per SIMD) march
// with three-slot rings whose roles rotate with the unrolled step (no copies, no control flow in
// the step): plane k+3's rows are requested while p(k+1) is formed and w(k) computed.
// Rows: a block stacks NW waves of TY rows; the row one step outside a wave comes from its
// neighbour through LDS (published one step before use, double buffered, one barrier per step);
// the block's first and last rows are halo rows (formed, not summed): blocks sum rows 1 .. NW TY - 2
// and advance by NW TY - 2 rows. Columns: 128 points per wave (whole lines); lane 0's left and
// lane 63's right neighbours come from "halo pairs" held in one more register set (lane q: row
// q's left pair, lane 64 - TY + q its right pair, pb_cg_sr.hip). Work: bands of W planes of every
// column, then the last band's column-planes in pieces of W, one workgroup per CU's worth.
//
// MEASURED SLOWER than the engine's pass A at 512^3 (0.444-0.484 ms with 2 or 4 rows per wave vs
// 0.383-0.387, profiles/r05/passa_ring_ab.txt): off by default (tuning cg_pa_ring = 1 selects it),
// kept as the parity-tested record of the two-plane-prefetch experiment.
//
// Per-point arithmetic is the engine's (CombineLoad::f, the reference summation order, w * c
// summed per point, no contraction); only the blocks the sums are taken over differ, so the
// history matches the engine's to rounding. Folded: every wave runs the previous iteration's
// residual-sum stage in its prologue (Fold stage 2) exactly as the engine's pass A does.
#include "pb_cg_device.hpp"

namespace pb {

static constexpr int kPaSeg = 128;  // points per wave segment

struct PaGeo {
  int nx, ny, nzl;
  int64_t plane;
  int nseg, ntile;  // x segments of kPaSeg points, y tiles of NW TY - 2 rows
  int W;            // planes of work per workgroup
};

template <int NW>
struct PaLds {
  dv2 xch[2][2][NW][64];  // [step parity][row 0, row TY-1][wave][lane]: p of the wave's edge rows
};

template <int NW, int TY>
__device__ __forceinline__ void pa_range(const PaGeo& g, double cx, double cy, double cz,
                                         double cc, const double* __restrict__ r,
                                         const double* __restrict__ p_old, double dinv,
                                         double shift, double bb, int seg, int tile, int kb,
                                         int ke, PaLds<NW>& L, double& acc) {
  constexpr int RB = NW * TY;
  constexpr int SB = RB - 2;
  constexpr int U = 3;  // ring slots: p(k-1), p(k), p(k+1); planes k+1 .. k+3 of r and p_old
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nx = g.nx, ny = g.ny, nz = g.nzl;
  const int g0 = tile * SB - 1;  // global row of block row 0
  const int br0 = wid * TY;
  const int j0 = g0 + br0;
  auto wrap = [](int v, int n) { v %= n; return v < 0 ? v + n : v; };
  const int x0 = seg * kPaSeg;
  const int o = x0 + 2 * lane;
  const int ip = wrap(o, nx);  // (nx even: a pair never straddles the wrap)
  const bool out_ok = o < nx;
  const bool left = lane < 32;  // halo pair: left (x0 - 2, x0 - 1) or right (x0 + 128, x0 + 129)
  const int qh = left ? lane % TY : (lane - (64 - TY)) % TY;  // the halo lane's row (others: any)
  const int ih = wrap(left ? x0 - 2 : x0 + kPaSeg, nx);
  int64_t ro[TY];
  double m[TY];  // 1: a summed row of this lane, 0: a halo row / a lane or row past the grid
#pragma unroll
  for (int q = 0; q < TY; ++q) {
    ro[q] = (int64_t)wrap(j0 + q, ny) * nx;
    const int brow = br0 + q;
    m[q] = out_ok && brow >= 1 && brow < RB - 1 && g0 + brow < ny ? 1.0 : 0.0;
  }
  const unsigned boff = (unsigned)ip * 8u;
  unsigned hoff = 0;
#pragma unroll
  for (int q = 0; q < TY; ++q)
    if (qh == q) hoff = (unsigned)((ro[q] + ih) * 8);
  auto pl = [&](int kk) -> int64_t { return (int64_t)wrap(kk, nz) * g.plane; };
  const int wm = wid > 0 ? wid - 1 : wid, wp = wid < NW - 1 ? wid + 1 : wid;
  auto inner = [&](const double (&v)[2]) { return left ? v[1] : v[0]; };

  double P[U][TY][2], PH[U][2];
  double R[U][TY][2], RH[U][2];
  double PO[U][TY][2], POH[U][2];
#pragma unroll
  for (int s = 0; s < U; ++s)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      PH[s][e] = RH[s][e] = POH[s][e] = 0.0;
#pragma unroll
      for (int q = 0; q < TY; ++q) P[s][q][e] = R[s][q][e] = PO[s][q][e] = 0.0;
    }
  auto ld = [&](const double* src, int kk, double (&dst)[TY][2], double (&dsth)[2]) {
    const int64_t base = pl(kk);
#pragma unroll
    for (int q = 0; q < TY; ++q) load_row<2>(src, RowIx{base + ro[q], boff}, dst[q]);
    load_row<2>(src, RowIx{base, hoff}, dsth);
  };
  // lane 0's left / lane 63's right x-neighbour of row q from the halo lanes (pb_cg_sr.hip)
  auto x_lo = [&](const double (&pair)[2], double hv, auto qc) {
    constexpr int q = decltype(qc)::value;
    return dpp_shr1_keep(dpp_row_shl<q>(hv), pair[1]);
  };
  auto x_hi = [&](const double (&pair)[2], double hv, auto qc) {
    constexpr int q = decltype(qc)::value;
    return dpp_shl1_keep(dpp_row_shr<TY - 1 - q>(hv), pair[0]);
  };
  // no loads before the loop: two load-only steps (k = kb - 4, kb - 3) start the ring, so the
  // loop head sees one issue order (preloads ahead of it were reordered past the loop's own loads
  // and its wait counts then merged to the stricter ones)

  auto body = [&](auto Qc, int k) {
    constexpr int Q = decltype(Qc)::value;
    constexpr int Q1 = (Q + 1) % U, Q2 = (Q + 2) % U;
    double (&pk)[TY][2] = P[Q1];   // p(k)
    double (&pk1)[TY][2] = P[Q2];  // p(k+1), formed this step
    double (&pkm)[TY][2] = P[Q];   // p(k-1)
    // (no instruction crosses a step: the scheduler otherwise hoists the next step's p(k+2) into
    // this step, which waits for the loads issued last -- vmcnt(0) at the loop head)
    __builtin_amdgcn_sched_barrier(0);
    // plane k+3 in flight for two steps (slot Q held plane k, consumed at step k-1)
    ld(r, k + 3, R[Q], RH[Q]);
    ld(p_old, k + 3, PO[Q], POH[Q]);
    // p(k+1) = (dinv r - mu) + b p_old (CombineLoad::f), halo pair included
#pragma unroll
    for (int q = 0; q < TY; ++q)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        double z = dinv * R[Q1][q][e];
        z = z + shift;
        pk1[q][e] = z + bb * PO[Q1][q][e];
      }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      double zh = dinv * RH[Q1][e];
      zh = zh + shift;
      PH[Q2][e] = zh + bb * POH[Q1][e];
    }
    __syncthreads();
    // rows -1 / TY of p(k) (and the halo lanes' p(k)), published by the neighbours at step k-1
    const int rp = (k + 1) & 1, cur = k & 1;
    const dv2 phl = L.xch[rp][1][wm][lane], phh = L.xch[rp][0][wp][lane];
    L.xch[cur][0][wid][lane] = dv2{pk1[0][0], pk1[0][1]};
    L.xch[cur][1][wid][lane] = dv2{pk1[TY - 1][0], pk1[TY - 1][1]};
    // w(k) = A p(k) (z-, y-, x-, c, x+, y+, z+), sum w * p
    const bool in = k >= kb && k < ke;
    const double hc = inner(PH[Q1]);  // the halo lanes' p(k)
    unroll_steps(std::make_integer_sequence<int, TY>{}, [&](auto qc) {
      constexpr int q = decltype(qc)::value;
      const double lo = x_lo(pk[q], hc, qc);
      const double hi = x_hi(pk[q], hc, qc);
      const double mq = in ? m[q] : 0.0;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const double xm = e == 0 ? lo : pk[q][0];
        const double xp = e == 1 ? hi : pk[q][1];
        const double ym = q == 0 ? phl[e] : pk[q == 0 ? 0 : q - 1][e];
        const double yp = q == TY - 1 ? phh[e] : pk[q == TY - 1 ? q : q + 1][e];
        const double w = star7_sum(cx, cy, cz, cc, pkm[q][e], ym, xm, pk[q][e], xp, yp, pk1[q][e]);
        acc += (w * pk[q][e]) * mq;  // (PassAT: w * c; masked rows hold finite values)
      }
    });
  };
  // steps kb-4 .. ke-1 (padded to whole rounds of U steps: the spare steps sum nothing); step
  // kb-2 forms p(kb-1), the first plane w(kb) needs
#pragma unroll 1
  for (int k = kb - 4; k < ke; k += U)
    unroll_steps(std::make_integer_sequence<int, U>{},
                 [&](auto Qc) { body(Qc, k + decltype(Qc)::value); });
}

template <int NW, int TY>
__global__ __launch_bounds__(64 * NW) void cg_pa_kernel(PaGeo g, double cx, double cy, double cz,
                                                        double cc, const double* __restrict__ r,
                                                        const double* __restrict__ p_old,
                                                        double* parts, const CgState* st_in,
                                                        Fold fold) {
  __shared__ PaLds<NW> lds;
  CgState st;
  if (fold.stage) {
    fold_prologue(fold, st);  // every wave: the previous iteration's residual-sum stage
  } else {
    cg_copy(st, *st_in);
  }
  if (st.done) return;  // (uniform)
  {  // zero the exchange (warm-up steps read it first; see pb_cg_sr.hip)
    double* z = reinterpret_cast<double*>(&lds);
    constexpr int nd = (int)(sizeof(PaLds<NW>) / sizeof(double));
    for (int i = threadIdx.x; i < nd; i += 64 * NW) z[i] = 0.0;
  }
  // (CombineLoad::prepare_from: the b of this iteration's pass A)
  const double dinv = st.dinv, shift = -st.mu, bb = st.it == 0 ? 0.0 : st.beta / st.betaold;
  double acc = 0.0;
  const int bid = xcd_block(1);
  const int ncol = g.nseg * g.ntile, W = g.W, T = g.nzl / W;
  auto run = [&](int col, int kb, int ke) {
    pa_range<NW, TY>(g, cx, cy, cz, cc, r, p_old, dinv, shift, bb, col % g.nseg, col / g.nseg,
                     kb, ke, lds, acc);
  };
  if (bid < T * ncol) {
    const int kb = (bid / ncol) * W;
    run(bid % ncol, kb, kb + W);
  } else {
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
        __syncthreads();
      }
    }
  }
  block_partials<1>(&acc, parts);
}

bool cg_pa_supported(const pb_grid* g) {
  return !g->ctx->split && g->n[0] % 2 == 0 && g->n[1] >= 2 && tune("cg_pa_ring", 0) != 0;
}

int launch_cg_pa(pb_grid* g, const Star& s, const double* r, const double* p_old,
                 const CgState* st, const Fold& fold, int* nblocks) {
#ifndef PB_PA_TY
#define PB_PA_TY 2
#endif
  constexpr int NW = 8, TY = PB_PA_TY;
  pb_ctx* ctx = g->ctx;  // (timed by the caller: launch_cg_pass_a*)
  PaGeo geo;
  geo.nx = (int)g->n[0];
  geo.ny = (int)g->n[1];
  geo.nzl = (int)g->nzl;
  geo.plane = g->plane;
  geo.nseg = (geo.nx + kPaSeg - 1) / kPaSeg;
  geo.ntile = (geo.ny + NW * TY - 3) / (NW * TY - 2);
  const int64_t work = (int64_t)geo.nseg * geo.ntile * geo.nzl;
  geo.W = (int)std::max<int64_t>(1, (work + ctx->num_cus - 1) / ctx->num_cus);
  const int64_t nb = (work + geo.W - 1) / geo.W;
  if (nb > kFoldMaxParts || nb > ctx->partials_cap / 8)  // (pass B's partials follow, folded)
    return set_error(PB_ERR_UNSUPPORTED, "ring pass A of %lld blocks", (long long)nb);
  hipLaunchKernelGGL((cg_pa_kernel<NW, TY>), dim3((unsigned)nb), dim3(64 * NW), 0, ctx->stream,
                     geo, s.cx, s.cy, s.cz, s.cc, r, p_old, ctx->d_partials, st, fold);
  PB_HIP(hipGetLastError());
  *nblocks = (int)nb;
  return PB_OK;
}

}  // namespace pb
