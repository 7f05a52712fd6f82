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
// the x update (the iterations that carry the deferred x update run the two passes: pass P's
// x-update form streams at the copy rate, a fused form would not fit the register budget).
//
// The stencils at a wave's tile edges need p two points and t one point outside it.
// Rows: a block stacks NW waves of TY rows, each wave forms every stage on its own rows only, and
// the values one row out come from the neighbouring waves through LDS (published one step before
// use, double buffered by step parity, one block barrier per step); each stage loses a row at the
// block's ends, so blocks store rows 2 .. NW TY - 3 and advance by NW TY - 4 rows (with delta in
// the difference form, below: rows 1 .. NW TY - 3, advancing by NW TY - 3).
// Columns: a wave owns 64 V points (V = 2, the default: 64 lanes x one 16-B pair, whole 128-B
// lines, segments that tile a 512-point row exactly; V = 1 with 3- or 4-row waves, PB_SR_TY /
// PB_SR_V, measured slower). The two points either side of each row are a "halo pair", all of a wave's halo pairs
// in ONE more register set: lane q holds row q's left pair (x0 - 2, x0 - 1), lane 64 - TY + q row
// q's right pair (x0 + 64 V, x0 + 64 V + 1). The halo's inner point gets
// p, w, r', t like any other point: its x-neighbours are its outer point and the segment's edge
// value (read from lane 0 / 63), its y-neighbours the next lanes (DPP; across waves through LDS),
// its z-neighbours the same register of the next planes. Lane 0's left and lane 63's right
// neighbours are then read from the halo lanes; every other x-neighbour is a DPP lane shift.
// Work is split evenly over one workgroup per CU (bands of W planes of every column, then the
// last band's column-planes cut into pieces of W), each z-range warming up four planes below its
// start.
//
// Per-point arithmetic is pass P's and pass S's (CombineLoad, PassB<., true, false>, ZLoad,
// SrSums: reference summation order, no FMA contraction), so p, r' and every summand are
// bit-identical to the two-pass iteration; only the blocks the sums are taken over differ.
#include <type_traits>
#include <utility>

#include "pb_cg_device.hpp"

namespace pb {

struct SrGeo {
  int nx, ny, nzl;
  int64_t plane;
  int nseg, ntile;  // x segments of 64 V points, y tiles of NW TY - SrRows::kHalo rows
  int W;            // planes of work per workgroup
  int remap;
};

// delta = t'A t in the difference form (r06): -sum (cx dx^2 + cy dy^2 + cz dz^2) over
// forward differences of t, plus (cc + 2 cx + 2 cy + 2 cz) sum t^2 (~0), equal to t'A t in exact
// arithmetic on the periodic grid. It needs t one row further on one side only, so a block stores
// NW TY - 3 of its NW TY rows instead of NW TY - 4 (fewer rows fetched twice by neighbouring
// tiles). 0: delta = t . (A t) with the stencil, two rows of halo each side (r05).
// (template flag DD; tuning sr_ddiff, default: see launch_cg_sr1)
template <bool DD>
struct SrRows {
  static constexpr int kHalo = DD ? 3 : 4;  // block rows not stored (both sides)
  static constexpr int kLead = DD ? 1 : 2;  // block rows below the first stored one
};

// p, r' stores non-temporal (buffer-store aux 2), like the stencil engine's outputs: 0.874-0.904
// against 0.937-0.949 ms for cached stores at 512^3, and the next x-update pass P 0.193 against
// 0.207-0.213 ms at 256^3 (profiles/r05/sr/sr_store_nt_ab.txt); 0: cached
#ifndef PB_SR_STORE_AUX
#define PB_SR_STORE_AUX 2
#endif
template <int V>
using lane_pts = std::conditional_t<V == 2, dv2, double>;
template <int V>
__device__ __forceinline__ lane_pts<V> pack_pts(const double (&v)[V]) {
  if constexpr (V == 2) return dv2{v[0], v[1]};
  else return v[0];
}
template <int V>
__device__ __forceinline__ double pt(const lane_pts<V>& x, int e) {
  if constexpr (V == 2) return x[e];
  else return x;
}

// v, or +0 where the mask is 0 (bitwise, exact; +0 leaves a sum that started at +0 bit-identical)
__device__ __forceinline__ double keep_if(double v, long long mk) {
  return __builtin_bit_cast(double, __builtin_bit_cast(long long, v) & mk);
}

template <int NW, int TY, int V>
struct SrLds {
  // [step parity][p row 0, p row TY-1, t row 0, t row TY-1][wave][lane]
  lane_pts<V> xch[2][4][NW][64];
  double xh[2][NW][64];  // [step parity][wave][lane]: the halo lanes' p
};

template <int NW, int TY, int V, bool DD>
__device__ __forceinline__ void sr1_range(const SrGeo& g, double cx, double cy, double cz,
                                          double cc, const double* __restrict__ r,
                                          const double* __restrict__ p_old,
                                          double* __restrict__ p_new, double* __restrict__ r_out,
                                          double dinv, double shift, double bb, double alpha,
                                          int seg, int tile, int kb, int ke, SrLds<NW, TY, V>& L,
                                          double (&acc)[5]) {
  constexpr int RB = NW * TY;
  constexpr int SB = RB - SrRows<DD>::kHalo;
  constexpr int kSrLead = SrRows<DD>::kLead;
  constexpr int SEG = 64 * V;  // points per wave segment
  const double ce = ((cc + 2.0 * cx) + 2.0 * cy) + 2.0 * cz;  // (difference form: ~0)
  // register ring slots: plane loads D = U - 2 steps ahead of the step that forms p from them.
  // U = 3 (one step ahead) fits the 256-register budget; at U = 4 the x-halo registers spill
  // (two-step prefetch measured within noise before the halo lanes: 0.86-0.93 vs 0.87-0.90 ms)
  constexpr int U = 3;
  constexpr int D = U - 2;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nx = g.nx, ny = g.ny, nz = g.nzl;
  const int g0 = tile * SB - kSrLead;  // global row of block row 0
  const int br0 = wid * TY;
  const int j0 = g0 + br0;
  auto wrap = [](int v, int n) { v %= n; return v < 0 ? v + n : v; };
  const int x0 = seg * SEG;
  const int o = x0 + V * lane;  // this lane's points
  const int ip = wrap(o, nx);   // (nx even: a pair never straddles the wrap)
  const bool out_ok = o < nx;
  const bool left = lane < 32;  // halo pair: left (x0 - 2, x0 - 1) or right (x0 + SEG, x0 + SEG + 1)
  const int qh = left ? lane % TY : (lane - (64 - TY)) % TY;  // the halo lane's row (other lanes: any)
  const int ih = wrap(left ? x0 - 2 : x0 + SEG, nx);
  int64_t ro[TY];
  unsigned row_ok = 0;
#pragma unroll
  for (int q = 0; q < TY; ++q) {
    ro[q] = (int64_t)wrap(j0 + q, ny) * nx;
    const int brow = br0 + q;
    if (out_ok && brow >= kSrLead && brow < kSrLead + SB && g0 + brow < ny) row_ok |= 1u << q;
  }
  const unsigned boff = (unsigned)ip * 8u;
  auto pl = [&](int kk) -> int64_t { return (int64_t)wrap(kk, nz) * g.plane; };
  // stores: buffer stores through a descriptor of the plane (out-of-range offsets are dropped by
  // the range check), so that no store sits under a branch -- control flow in the step made the
  // compiler's wait counts drain the two-plane prefetch
  unsigned roff[TY];
#pragma unroll
  for (int q = 0; q < TY; ++q) roff[q] = (unsigned)(ro[q] * 8) + boff;
  const int pbytes = (int)(g.plane * 8);
  auto plane_rsrc = [&](double* base, int kk) { return buf_rsrc(base + pl(kk), pbytes); };
  unsigned hoff = 0;  // the halo lane's byte offset in a plane
#pragma unroll
  for (int q = 0; q < TY; ++q)
    if (qh == q) hoff = (unsigned)((ro[q] + ih) * 8);
  // LDS lanes of the halo rows TY-1 (read by row 0) and 0 (read by row TY-1), same side
  const int hl_lo = left ? TY - 1 : 63, hl_hi = left ? 0 : 64 - TY;
  const int wm = wid > 0 ? wid - 1 : wid, wp = wid < NW - 1 ? wid + 1 : wid;
  // halo pair: inner point (next to the segment) and outer point
  auto inner = [&](const double (&v)[2]) { return left ? v[1] : v[0]; };  // next to the segment
  auto outer = [&](const double (&v)[2]) { return left ? v[0] : v[1]; };

  // rings of U register slots whose roles rotate with the unrolled step (no copies); *H = the
  // halo lanes' pairs
  double P[U][TY][V], PH[U][2];    // p of planes k, k+1, k+2 at slots Q, Q+1, Q+2
  double R[U][TY][V], RH[U][2];    // r of planes k+1 .. k+1+D; slot Q receives plane k+2+D
  double T[U][TY][V], TH[U];       // t of planes k-1, k, k+1 (halo: inner point only)
  double PO[U][TY][V], POH[U][2];  // p_old of planes k+2 .. k+1+D; slot Q receives k+2+D
#pragma unroll
  for (int s = 0; s < U; ++s) {
    TH[s] = 0.0;
#pragma unroll
    for (int e = 0; e < 2; ++e) PH[s][e] = RH[s][e] = POH[s][e] = 0.0;
#pragma unroll
    for (int e = 0; e < V; ++e)
#pragma unroll
      for (int q = 0; q < TY; ++q) P[s][q][e] = R[s][q][e] = T[s][q][e] = PO[s][q][e] = 0.0;
  }
  auto ld = [&](const double* src, int kk, double (&dst)[TY][V], double (&dsth)[2]) {
    const int64_t base = pl(kk);
#pragma unroll
    for (int q = 0; q < TY; ++q) load_row<V>(src, RowIx{base + ro[q], boff}, dst[q]);
    load_row<2>(src, RowIx{base, hoff}, dsth);
  };
  // Cross-lane moves are DPP only (row shifts within a 16-lane row, wave shifts by one) and every
  // choice a per-lane select: a readlane under a per-lane condition becomes a branch, and any
  // control flow in the step drains the prefetch (the compiler's wait counts merge at joins).
  // the segment's edge value of row q (lane 0's first / lane 63's second point) in the halo lanes
  auto edge = [&](const double (&v)[TY][V]) {
    double e = 0.0;
    unroll_steps(std::make_integer_sequence<int, TY>{}, [&](auto qc) {
      constexpr int q = decltype(qc)::value;
      const double a = dpp_row_shr<q>(v[q][0]);            // lane q <- lane 0
      const double b = dpp_row_shl<TY - 1 - q>(v[q][V - 1]);  // lane 64 - TY + q <- lane 63
      e = qh == q ? (left ? a : b) : e;
    });
    return e;
  };
  // x-neighbours of row q's pairs: lane 0's left and lane 63's right come from the halo lanes
  // (wave shifts keep the old value where the source lane is outside the wave)
  auto x_lo = [&](const double (&pts)[V], double hv, auto qc) {
    constexpr int q = decltype(qc)::value;
    return dpp_shr1_keep(dpp_row_shl<q>(hv), pts[V - 1]);  // lane 0 <- halo lane q
  };
  auto x_hi = [&](const double (&pts)[V], double hv, auto qc) {
    constexpr int q = decltype(qc)::value;
    return dpp_shl1_keep(dpp_row_shr<TY - 1 - q>(hv), pts[0]);  // lane 63 <- 64 - TY + q
  };
  // the first step (k = kb - 4, Q = 0) forms p(kb - 2); planes kb - 1 .. kb - 3 + D are in flight
#pragma unroll
  for (int m = 0; m < D; ++m) {
    ld(r, kb - 2 + m, R[(2 + m) % U], RH[(2 + m) % U]);
    ld(p_old, kb - 2 + m, PO[(2 + m) % U], POH[(2 + m) % U]);
  }

  auto body = [&](auto Qc, int k) {
    constexpr int Q = decltype(Qc)::value;
    constexpr int Q1 = (Q + 1) % U, Q2 = (Q + 2) % U;
    double (&pk)[TY][V] = P[Q];
    double (&pk1)[TY][V] = P[Q1];
    double (&pk2)[TY][V] = P[Q2];
    double (&hk)[2] = PH[Q];
    double (&hk1)[2] = PH[Q1];
    double (&hk2)[2] = PH[Q2];
    double (&tkm)[TY][V] = T[Q];
    double (&tk)[TY][V] = T[Q1];
    double (&tk1)[TY][V] = T[Q2];
    // planes k+2+D in flight for D steps
    ld(r, k + 2 + D, R[Q], RH[Q]);
    ld(p_old, k + 2 + D, PO[Q], POH[Q]);
    // p(k+2) = (dinv r - mu) + b p_old (CombineLoad::f), halo pair included
#pragma unroll
    for (int q = 0; q < TY; ++q)
#pragma unroll
      for (int e = 0; e < V; ++e) {
        double z = dinv * R[Q2][q][e];
        z = z + shift;
        pk2[q][e] = z + bb * PO[Q2][q][e];
      }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      double zh = dinv * RH[Q2][e];
      zh = zh + shift;
      hk2[e] = zh + bb * POH[Q2][e];
    }
    __syncthreads();
    // rows -1 / TY of p(k+1) and t(k): published by the neighbouring waves at step k-1
    const int rp = (k + 1) & 1, cur = k & 1;
    const lane_pts<V> phl = L.xch[rp][1][wm][lane], phh = L.xch[rp][0][wp][lane];
    const lane_pts<V> thh = L.xch[rp][2][wp][lane];
    const lane_pts<V> thl = DD ? thh : L.xch[rp][3][wm][lane];  // (DD: unused)
    const double hhl = L.xh[rp][wm][hl_lo], hhh = L.xh[rp][wp][hl_hi];
    L.xch[cur][0][wid][lane] = pack_pts<V>(pk2[0]);
    L.xch[cur][1][wid][lane] = pack_pts<V>(pk2[TY - 1]);
    L.xh[cur][wid][lane] = inner(hk2);
    const bool in2 = k + 2 >= kb && k + 2 < ke, in1 = k + 1 >= kb && k + 1 < ke,
               in0 = k >= kb && k < ke;
    {
      const auto rs = plane_rsrc(p_new, k + 2);
#pragma unroll
      for (int q = 0; q < TY; ++q)
        store_pts<V, PB_SR_STORE_AUX>(rs, in2 && (row_ok >> q & 1u) ? roff[q] : kOob, pk2[q]);
    }
    // w(k+1) = A p, r' = r - alpha w, t = dinv r' - mu: the halo lanes' inner points first
    const double hc = inner(hk1);
    {
      const double eg = edge(pk1);
      const double xm = left ? outer(hk1) : eg;
      const double xp = left ? eg : outer(hk1);
      const double dl = dpp_from_lower(hc), du = dpp_from_upper(hc);
      const double ym = qh == 0 ? hhl : dl;
      const double yp = qh == TY - 1 ? hhh : du;
      const double w = star7_sum(cx, cy, cz, cc, inner(hk), ym, xm, hc, xp, yp, inner(hk2));
      const double rv = inner(RH[Q1]) + (-alpha) * w;
      const double z = dinv * rv;
      TH[Q2] = z + shift;
    }
    const auto rs1 = plane_rsrc(r_out, k + 1);
    unroll_steps(std::make_integer_sequence<int, TY>{}, [&](auto qc) {
      constexpr int q = decltype(qc)::value;
      const double lo = x_lo(pk1[q], hc, qc);
      const double hi = x_hi(pk1[q], hc, qc);
      double rv[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const double xm = e == 0 ? lo : pk1[q][e == 0 ? 0 : e - 1];
        const double xp = e == V - 1 ? hi : pk1[q][e == V - 1 ? e : e + 1];
        const double ym = q == 0 ? pt<V>(phl, e) : pk1[q == 0 ? 0 : q - 1][e];
        const double yp = q == TY - 1 ? pt<V>(phh, e) : pk1[q == TY - 1 ? q : q + 1][e];
        const double w = star7_sum(cx, cy, cz, cc, pk[q][e], ym, xm, pk1[q][e], xp, yp, pk2[q][e]);
        rv[e] = R[Q1][q][e] + (-alpha) * w;
        double z = dinv * rv[e];
        tk1[q][e] = z + shift;
      }
      const bool ok = in1 && (row_ok >> q & 1u);
      store_pts<V, PB_SR_STORE_AUX>(rs1, ok ? roff[q] : kOob, rv);
      // summands of masked rows become +0 by a bit mask (no branch -- selects here became
      // branches and spills; a multiply by 0 would let a NaN / Inf of a masked row through)
      const long long mk = ok ? -1LL : 0LL;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const double t = tk1[q][e];
        acc[0] += keep_if(t, mk);
        acc[1] += keep_if(t * t, mk);
        acc[2] += keep_if(t * rv[e], mk);
        acc[3] += keep_if(rv[e], mk);
      }
    });
    L.xch[cur][2][wid][lane] = pack_pts<V>(tk1[0]);
    if constexpr (DD) {
    // delta of plane k in the difference form: forward differences of t in x (past lane 63: the
    // halo lanes), y (past the wave's top row: the wave above's row 0, thh) and z (t(k+1))
    unroll_steps(std::make_integer_sequence<int, TY>{}, [&](auto qc) {
      constexpr int q = decltype(qc)::value;
      const double hi = x_hi(tk[q], TH[Q1], qc);
      const long long mk = in0 && (row_ok >> q & 1u) ? -1LL : 0LL;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const double tc = tk[q][e];
        const double xp = e == V - 1 ? hi : tk[q][e == V - 1 ? e : e + 1];
        const double yp = q == TY - 1 ? pt<V>(thh, e) : tk[q == TY - 1 ? q : q + 1][e];
        const double dxv = xp - tc, dyv = yp - tc, dzv = tk1[q][e] - tc;
        double v = ce * (tc * tc);
        v = v - cx * (dxv * dxv);
        v = v - cy * (dyv * dyv);
        v = v - cz * (dzv * dzv);
        acc[4] += keep_if(v, mk);
      }
    });
    (void)thl;
    (void)tkm;
    } else {
    L.xch[cur][3][wid][lane] = pack_pts<V>(tk1[TY - 1]);
    // s(k) = A t, delta sum t.s
    unroll_steps(std::make_integer_sequence<int, TY>{}, [&](auto qc) {
      constexpr int q = decltype(qc)::value;
      const double lo = x_lo(tk[q], TH[Q1], qc);
      const double hi = x_hi(tk[q], TH[Q1], qc);
      const long long mk = in0 && (row_ok >> q & 1u) ? -1LL : 0LL;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const double xm = e == 0 ? lo : tk[q][e == 0 ? 0 : e - 1];
        const double xp = e == V - 1 ? hi : tk[q][e == V - 1 ? e : e + 1];
        const double ym = q == 0 ? pt<V>(thl, e) : tk[q == 0 ? 0 : q - 1][e];
        const double yp = q == TY - 1 ? pt<V>(thh, e) : tk[q == TY - 1 ? q : q + 1][e];
        const double sv = star7_sum(cx, cy, cz, cc, tkm[q][e], ym, xm, tk[q][e], xp, yp, tk1[q][e]);
        acc[4] += keep_if(tk[q][e] * sv, mk);
      }
    });
    }
  };
  // steps kb-4 .. ke-1 (padded to whole rounds of U steps: the spare steps store and sum nothing)
#pragma unroll 1
  for (int k = kb - 4; k < ke; k += U)
    unroll_steps(std::make_integer_sequence<int, U>{},
                 [&](auto Qc) { body(Qc, k + decltype(Qc)::value); });
}

template <int NW, int TY, int V, bool DD>
__global__ __launch_bounds__(64 * NW) void cg_sr1_kernel(SrGeo g, double cx, double cy, double cz,
                                                         double cc, const double* __restrict__ r,
                                                         const double* __restrict__ p_old,
                                                         double* __restrict__ p_new,
                                                         double* __restrict__ r_out,
                                                         double* parts, Fold fold) {
  __shared__ SrLds<NW, TY, V> lds;
  CgState st;
  fold_prologue(fold, st);  // every wave: the previous residual-sum stage + this iteration's top
  if (st.done) return;      // (uniform: every wave computed the same state)
  {  // zero the exchange: warm-up steps read it before any wave wrote it (stale LDS of earlier
     // kernels, possibly NaN, which the masked sums' factor 0 would not cancel); the first step's
     // barrier orders these stores before every read
    double* z = reinterpret_cast<double*>(&lds);
    constexpr int nd = (int)(sizeof(SrLds<NW, TY, V>) / sizeof(double));
    for (int i = threadIdx.x; i < nd; i += 64 * NW) z[i] = 0.0;
  }
  const double dinv = st.dinv, shift = -st.mu, bb = st.bbp, alpha = st.alpha;
  double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  const int bid = xcd_block(g.remap);
  const int ncol = g.nseg * g.ntile, W = g.W, T = g.nzl / W;
  auto run = [&](int col, int kb, int ke) {
    sr1_range<NW, TY, V, DD>(g, cx, cy, cz, cc, r, p_old, p_new, r_out, dinv, shift, bb, alpha,
                      col % g.nseg, col / g.nseg, kb, ke, lds, acc);
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
  // (plane byte offsets in 31 bits: buffer-store descriptors per plane)
  return !g->ctx->split && g->n[0] % 2 == 0 && g->plane * 8 < ((int64_t)1 << 31) &&
         tune("cg_sr_fused", 1) != 0;
}

int launch_cg_sr1(pb_grid* g, const Star& s, const double* r, const double* p_old,
                  double* p_new, double* r_out, const SrFold& sf, const double* parts_in,
                  double* parts_out, int64_t host_iter, int* nblocks) {
#ifndef PB_SR_TY
#define PB_SR_TY 2
#endif
  // 8 waves (two per SIMD, one block per CU) of TY rows of 64 V points (TY V = 4: the register
  // budget)
#ifndef PB_SR_V
#define PB_SR_V (4 / PB_SR_TY)
#endif
  constexpr int NW = 8, TY = PB_SR_TY, V = PB_SR_V;
  pb_ctx* ctx = g->ctx;
  ScopedTimer tm(ctx, "cg_sr1");
  SrGeo geo;
  geo.nx = (int)g->n[0];
  geo.ny = (int)g->n[1];
  geo.nzl = (int)g->nzl;
  geo.plane = g->plane;
  geo.nseg = (geo.nx + 64 * V - 1) / (64 * V);
  // delta in the difference form: 256^3 0.1518-0.1525 against 0.1581-0.1599 ms/iteration, but
  // 512^3 1.107-1.115 against 1.096-1.097 (profiles/r06/sr_ddiff_ab.txt): by default on planes
  // below 512^2 points
  const int ddt = tune("sr_ddiff", -1);
  const bool dd = ddt < 0 ? g->plane < 512 * 512 : ddt != 0;
  const int halo = dd ? SrRows<true>::kHalo : SrRows<false>::kHalo;
  geo.ntile = (geo.ny + NW * TY - halo - 1) / (NW * TY - halo);
  geo.remap = 1;
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
  if (dd)
    hipLaunchKernelGGL((cg_sr1_kernel<NW, TY, V, true>), dim3((unsigned)nb), dim3(64 * NW), 0,
                       ctx->stream, geo, s.cx, s.cy, s.cz, s.cc, r, p_old, p_new, r_out, parts_out,
                       f);
  else
    hipLaunchKernelGGL((cg_sr1_kernel<NW, TY, V, false>), dim3((unsigned)nb), dim3(64 * NW), 0,
                       ctx->stream, geo, s.cx, s.cy, s.cz, s.cc, r, p_old, p_new, r_out, parts_out,
                       f);
  PB_HIP(hipGetLastError());
  *nblocks = (int)nb;
  return PB_OK;
}

}  // namespace pb
