// pb_mg_sweep.hip -- fused red-black SOR passes for the multigrid preconditioner (pb_mg.hip), on
// one rank or N (two-deep z ghosts exchanged per pass):
// both half-sweeps of a post-smoothing in one pass, and the zero-start pre-smoothing fused with
// the residual. Same per-point arithmetic as the half-sweep / residual kernels (SorHalf, ResidEpi
// in pb_stencil.hip, restated in oracle/pb_oracle.c pbo_mg_apply), hence bit-identical results.
#include <algorithm>
#include <type_traits>

#include "pb_device.hpp"

namespace pb {

// ---------------------------------------------------------------------------------------------
// Fused red-black SOR sweep: both half-sweeps (colour c1, then 1 - c1) in ONE pass, out of place
// (xout != xin), one rank. The second half-sweep at point p needs first-half values S1 at p's
// neighbours, and S1 needs xin at distance 1 from those: a wave holds xin for TY2 + 4 rows and
// three planes, computes S1 for the TY2 + 2 middle rows one plane ahead, and the second half for
// its TY2 own rows. x-halo by overlap: a wave spans 64 pairs but stores only lanes 4..59 (112
// points, whole 128-B lines; neighbouring segments overlap), so every x-neighbour is a DPP shift.
// Per point: read xin and b once, write xout once (24 B/DoF instead of 2 x 24). Arithmetic per
// point is the two half-sweeps' (SorHalf / mg_smooth_kernel), so results are bit-identical.
// ---------------------------------------------------------------------------------------------
#ifndef PB_SWEEP2_TY
#define PB_SWEEP2_TY 3  // measured: 3 beats 2 (0.97 vs 1.09 ms at 512^3) and 1 (1.24)
#endif
static constexpr int kTY2 = PB_SWEEP2_TY;  // own rows per wave
static constexpr int kRW = kTY2 + 4;    // xin rows held: j0-2 .. j0+TY2+1
static constexpr int kSegOut = 112;     // outputs per wave segment (lanes 4..59): 896 B, whole
                                        // 128-B lines, so no line is written by two waves
static constexpr int kSegLead = 4;      // halo pairs left of the outputs (>= 1 needed)

// v[1] if e1 else v[0], as bit operations: a `?:` between two elements of a register array can
// become a computed address, which moves the whole array to scratch
__device__ __forceinline__ double pick(bool e1, const double (&v)[2]) {
  const long long m = -(long long)e1;
  return __builtin_bit_cast(double, (__builtin_bit_cast(long long, v[1]) & m) |
                                        (__builtin_bit_cast(long long, v[0]) & ~m));
}

struct Sweep2Geo {
  int nx, ny, nzl;
  int64_t plane;
  int nseg, ntile, kc, nchunk;
  int k0, remap, nt;
  // N ranks (split): xin's planes -2, -1, nzl, nzl+1 at xg[0..3], b's planes -1 / nzl at
  // bg_lo / bg_hi; one rank reads the periodic wrap in place
  int split;
  int wsplit = 0;  // > 0: planes per workgroup of the balanced work split (the u4 kernels)
  const double* xg;
  const double* bg_lo;
  const double* bg_hi;
};

// SOR sweep (first colour c1, then the other) of xin -> xout.
template <bool SUMS, bool SPLIT>
__global__ __launch_bounds__(kThreads) void sor_sweep2_kernel(Sweep2Geo g, double cx, double cy,
                                                               double cz, double cc, double omega,
                                                               int c1, const double* __restrict__ xin,
                                                               const double* __restrict__ b,
                                                               double* __restrict__ xout,
                                                               const CgState* st, double* parts,
                                                               const int* skip) {
  if (skip && *skip) return;
  const double icc = 1.0 / cc;  // SOR: multiply by the inverted diagonal
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  const double mu = SUMS ? st->mu : 0.0;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int bid = xcd_block(g.remap);
  const int seg = bid % g.nseg;
  bid /= g.nseg;
  const int tile = bid % g.ntile;
  const int chunk = bid / g.ntile;
  const int j0 = (tile * kWaves + wid) * kTY2;
  const int kb = chunk * g.kc;
  const int ke = min(kb + g.kc, g.nzl);
  const int nx = g.nx, ny = g.ny, nz = g.nzl;
  int ip = seg * kSegOut + 2 * (lane - kSegLead);  // this lane's pair (x wraps periodically)
  if (ip < 0) ip += nx;
  if (ip >= nx) ip -= nx;
  const int o = seg * kSegOut + 2 * (lane - kSegLead);  // output pair
  const bool out_ok = lane >= kSegLead && lane < kSegLead + kSegOut / 2 && o < nx;
  if (j0 < ny && kb < nz) {
    int64_t ro[kRW];  // wave-uniform row offsets; the lane's pair is the byte offset boff
    int par_row[kRW];  // (i + j) parity base of each row for element 0
#pragma unroll
    for (int r = 0; r < kRW; ++r) {
      int j = j0 - 2 + r;
      if (j < 0) j += ny;
      if (j >= ny) j -= ny;
      ro[r] = (int64_t)j * nx;
      par_row[r] = (ip + j) & 1;
    }
    const unsigned boff = (unsigned)ip * 8u;
    auto rix = [&](int64_t row) { return RowIx{row, boff}; };
    // one rank: periodic plane offsets into xin / b; N ranks: own planes or the ghost planes
    auto pl = [&](int kk) -> int64_t {
      if constexpr (!SPLIT) kk = kk < 0 ? kk + nz : (kk >= nz ? kk - nz : kk);
      return (int64_t)kk * g.plane;
    };
    auto kpar = [&](int kk) -> int {  // colour parity of plane kk (global index)
      if constexpr (!SPLIT) kk = kk < 0 ? kk + nz : (kk >= nz ? kk - nz : kk);
      return (g.k0 + kk) & 1;
    };
    auto xplane = [&](int kk) -> const double* {  // N ranks: xin plane kk in [-2, nzl+1]
      if (kk >= 0 && kk < nz) return xin + (int64_t)kk * g.plane;
      return g.xg + (int64_t)(kk < 0 ? kk + 2 : kk - nz + 2) * g.plane;
    };
    auto bplane = [&](int kk) -> const double* {  // N ranks: b plane kk in [-1, nzl]
      if (kk >= 0 && kk < nz) return b + (int64_t)kk * g.plane;
      return kk < 0 ? g.bg_lo : g.bg_hi;
    };
    double xq[3][kRW][2];  // xin planes k, k+1, k+2
    double xn[kRW][2];     // prefetch: plane k+3
    double s1[3][kRW][2];  // S1 planes k-1, k, k+1 (rows 1 .. kRW-2)
    double bq[2][kRW][2];  // b planes k, k+1 (rows 1 .. kRW-2)
    double bn[kRW][2];     // prefetch: b plane k+2
    auto ldx = [&](double (&dst)[kRW][2], int kk) {
      if constexpr (SPLIT) {
        const double* P = xplane(kk);
#pragma unroll
        for (int r = 0; r < kRW; ++r) load_row<2>(P, rix(ro[r]), dst[r]);
      } else {
        const int64_t base = pl(kk);
#pragma unroll
        for (int r = 0; r < kRW; ++r) load_row<2>(xin, rix(base + ro[r]), dst[r]);
      }
    };
    auto ldb = [&](double (&dst)[kRW][2], int kk) {
      if constexpr (SPLIT) {
        const double* P = bplane(kk);
#pragma unroll
        for (int r = 1; r < kRW - 1; ++r) load_row<2>(P, rix(ro[r]), dst[r]);
      } else {
        const int64_t base = pl(kk);
#pragma unroll
        for (int r = 1; r < kRW - 1; ++r) load_row<2>(b, rix(base + ro[r]), dst[r]);
      }
    };
    // first half-sweep at plane kk (rows 1 .. kRW-2): x planes xm (kk-1), xc (kk), xp (kk+1)
    auto half1 = [&](const double (&xm)[kRW][2], const double (&xc)[kRW][2],
                     const double (&xp)[kRW][2], const double (&bb)[kRW][2], int kk,
                     double (&out)[kRW][2]) {
      const int kp = kpar(kk);
#pragma unroll
      for (int r = 1; r < kRW - 1; ++r) {
        // the pair holds one point of each colour; which element is c1 is wave-uniform (pairs
        // start at even i), so only that element is updated -- one division per pair
        const bool a1 = ((par_row[r] + kp) & 1) != c1;  // c1 point is element 1
        const double lo = dpp_from_lower(xc[r][1]);
        const double hi = dpp_from_upper(xc[r][0]);
        const double xl = a1 ? xc[r][0] : lo;
        const double xr = a1 ? hi : xc[r][1];
        const double zm = a1 ? xm[r][1] : xm[r][0];
        const double ym = a1 ? xc[r - 1][1] : xc[r - 1][0];
        const double yp = a1 ? xc[r + 1][1] : xc[r + 1][0];
        const double zp = a1 ? xp[r][1] : xp[r][0];
        const double bv = a1 ? bb[r][1] : bb[r][0];
        const double xo = a1 ? xc[r][1] : xc[r][0];
        double nb = cz * zm;
        nb = nb + cy * ym;
        nb = nb + cx * xl;
        nb = nb + cx * xr;
        nb = nb + cy * yp;
        nb = nb + cz * zp;
        const double t = (bv - nb) * icc;
        const double v = (1.0 - omega) * xo + omega * t;
        out[r][0] = a1 ? xc[r][0] : v;
        out[r][1] = a1 ? v : xc[r][1];
      }
    };
    // prologue: S1 at planes kb-1 and kb
    {
      double xa[kRW][2], bb[kRW][2];
      ldx(xa, kb - 2);
      ldx(xq[0], kb - 1);
      ldx(xq[1], kb);
      ldb(bb, kb - 1);
      half1(xa, xq[0], xq[1], bb, kb - 1, s1[0]);
      ldx(xq[2], kb + 1);
      ldb(bq[0], kb);
      half1(xq[0], xq[1], xq[2], bq[0], kb, s1[1]);
      // shift x queue to (kb, kb+1, kb+2)
#pragma unroll
      for (int r = 0; r < kRW; ++r)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          xq[0][r][e] = xq[1][r][e];
          xq[1][r][e] = xq[2][r][e];
        }
      ldx(xq[2], kb + 2);
      ldb(bq[1], kb + 1);
    }
    for (int k = kb; k < ke; ++k) {
      const bool more = k + 1 < ke;
      // unconditional (the chunk's last step re-loads valid planes, unused): a load under a
      // branch made the compiler copy the prefetch registers at the join, waiting for the loads
      ldx(xn, more ? k + 3 : k + 2);
      ldb(bn, more ? k + 2 : k + 1);
      half1(xq[0], xq[1], xq[2], bq[1], k + 1, s1[2]);  // S1 at plane k+1
      // second half-sweep at plane k, own rows 2 .. 2+TY2-1
      const int kp = kpar(k);
      const int64_t base = pl(k);
#pragma unroll
      for (int r = 2; r < 2 + kTY2; ++r) {
        const bool a1 = ((par_row[r] + kp) & 1) == c1;  // second-colour point is element 1
        const double lo = dpp_from_lower(s1[1][r][1]);
        const double hi = dpp_from_upper(s1[1][r][0]);
        const double xl = a1 ? s1[1][r][0] : lo;
        const double xr = a1 ? hi : s1[1][r][1];
        const double zm = a1 ? s1[0][r][1] : s1[0][r][0];
        const double ym = a1 ? s1[1][r - 1][1] : s1[1][r - 1][0];
        const double yp = a1 ? s1[1][r + 1][1] : s1[1][r + 1][0];
        const double zp = a1 ? s1[2][r][1] : s1[2][r][0];
        const double bv = a1 ? bq[0][r][1] : bq[0][r][0];
        const double xo = a1 ? xq[0][r][1] : xq[0][r][0];
        double nb = cz * zm;
        nb = nb + cy * ym;
        nb = nb + cx * xl;
        nb = nb + cx * xr;
        nb = nb + cy * yp;
        nb = nb + cz * zp;
        const double t = (bv - nb) * icc;
        const double v = (1.0 - omega) * xo + omega * t;
        double ov[2];
        ov[0] = a1 ? s1[1][r][0] : v;
        ov[1] = a1 ? v : s1[1][r][1];
        if (out_ok && j0 + r - 2 < ny) {  // rows past ny (last tile) would wrap: not ours
          store_row<2>(xout, rix(base + ro[r]), ov, g.nt);
          if constexpr (SUMS) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const double rv = bq[0][r][e];
              const double t2 = ov[e] - mu;
              acc[0] += t2;
              acc[1] += t2 * t2;
              acc[2] += t2 * rv;
              acc[3] += rv;
            }
          }
        }
      }
      // rotate queues
#pragma unroll
      for (int r = 0; r < kRW; ++r)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          s1[0][r][e] = s1[1][r][e];
          s1[1][r][e] = s1[2][r][e];
          xq[0][r][e] = xq[1][r][e];
          xq[1][r][e] = xq[2][r][e];
          xq[2][r][e] = xn[r][e];
          bq[0][r][e] = bq[1][r][e];
          bq[1][r][e] = bn[r][e];
        }
    }
  }
  if constexpr (SUMS) block_partials<4>(acc, parts);
}

// ---------------------------------------------------------------------------------------------
// Pre-smoothing from x = 0 fused with the residual, slim form of sor_sweep2_kernel<.., 1, ..>:
// after the zero-start red half-sweep every pair holds ONE non-zero (its red point, w b / c), and
// the black half-sweep reads only red values -- so the x queue keeps one double per pair (the red
// value) instead of two, and b is loaded once per plane (the red values are formed from the raw
// rows that also serve as the b operand). Same per-point operations as the zero-start sweeps
// (Red0Load + SorHalf, then ResidEpi's order): bit-identical. 42 fewer VGPRs -> two waves per SIMD
// instead of one.
// ---------------------------------------------------------------------------------------------
template <bool SPLIT>
__global__ __launch_bounds__(kThreads) void presmooth_resid_kernel(
    Sweep2Geo g, double cx, double cy, double cz, double cc, double omega,
    const double* __restrict__ b, double* __restrict__ xout, double* __restrict__ res,
    const int* skip) {
  if (skip && *skip) return;
  const double icc = 1.0 / cc;  // SOR: multiply by the inverted diagonal
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int bid = xcd_block(g.remap);
  const int seg = bid % g.nseg;
  bid /= g.nseg;
  const int tile = bid % g.ntile;
  const int chunk = bid / g.ntile;
  const int j0 = (tile * kWaves + wid) * kTY2;
  const int kb = chunk * g.kc;
  const int ke = min(kb + g.kc, g.nzl);
  const int nx = g.nx, ny = g.ny, nz = g.nzl;
  int ip = seg * kSegOut + 2 * (lane - kSegLead);
  if (ip < 0) ip += nx;
  if (ip >= nx) ip -= nx;
  const int o = seg * kSegOut + 2 * (lane - kSegLead);
  const bool out_ok = lane >= kSegLead && lane < kSegLead + kSegOut / 2 && o < nx;
  if (!(j0 < ny && kb < nz)) return;
  int64_t ro[kRW];
  int par_row[kRW];
#pragma unroll
  for (int r = 0; r < kRW; ++r) {
    int j = j0 - 2 + r;
    if (j < 0) j += ny;
    if (j >= ny) j -= ny;
    ro[r] = (int64_t)j * nx;
    par_row[r] = (ip + j) & 1;
  }
  const unsigned boff = (unsigned)ip * 8u;
  auto rix = [&](int64_t row) { return RowIx{row, boff}; };
  auto kpar = [&](int kk) -> int {
    if constexpr (!SPLIT) kk = kk < 0 ? kk + nz : (kk >= nz ? kk - nz : kk);
    return (g.k0 + kk) & 1;
  };
  // b plane kk in [-2, nzl+1]: own planes or (N ranks) the two-deep ghosts of b
  auto bplane = [&](int kk) -> const double* {
    if constexpr (!SPLIT) {
      kk = kk < 0 ? kk + nz : (kk >= nz ? kk - nz : kk);
      return b + (int64_t)kk * g.plane;
    } else {
      if (kk >= 0 && kk < nz) return b + (int64_t)kk * g.plane;
      return g.xg + (int64_t)(kk < 0 ? kk + 2 : kk - nz + 2) * g.plane;
    }
  };
  auto ldraw = [&](double (&dst)[kRW][2], int kk) {
    const double* P = bplane(kk);
#pragma unroll
    for (int r = 0; r < kRW; ++r) load_row<2>(P, rix(ro[r]), dst[r]);
  };
  // raw b rows of plane kk -> the red value of each pair (Red0Load's arithmetic)
  auto redv = [&](const double (&v)[kRW][2], int kk, double (&red)[kRW]) {
    const int kp = kpar(kk);
#pragma unroll
    for (int r = 0; r < kRW; ++r) {
      const long long m = -(long long)(((par_row[r] + kp) & 1) != 0);  // red point is element 1
      const double bv = __builtin_bit_cast(
          double, (__builtin_bit_cast(long long, v[r][1]) & m) |
                      (__builtin_bit_cast(long long, v[r][0]) & ~m));  // (see half1)
      const double t = (bv - 0.0) * icc;
      red[r] = (1.0 - omega) * 0.0 + omega * t;
    }
  };
  auto keepb = [&](const double (&v)[kRW][2], double (&bb)[kRW][2]) {
#pragma unroll
    for (int r = 1; r < kRW - 1; ++r) {
      bb[r][0] = v[r][0];
      bb[r][1] = v[r][1];
    }
  };
  // black half-sweep at plane kk (rows 1 .. kRW-2) from the red values of planes kk-1, kk, kk+1:
  // the pair's full values (red, new black) -> out. sor_sweep2's half1 with c1 = 1, x_old = 0.
  auto half1 = [&](const double (&rm)[kRW], const double (&rc)[kRW], const double (&rp)[kRW],
                   const double (&bb)[kRW][2], int kk, double (&out)[kRW][2]) {
    const int kp = kpar(kk);
#pragma unroll
    for (int r = 1; r < kRW - 1; ++r) {
      const bool a1 = ((par_row[r] + kp) & 1) != 1;  // the black point is element 1
      const double lo = dpp_from_lower(rc[r]);
      const double hi = dpp_from_upper(rc[r]);
      const double xl = a1 ? rc[r] : lo;
      const double xr = a1 ? hi : rc[r];
      double nb = cz * rm[r];
      nb = nb + cy * rc[r - 1];
      nb = nb + cx * xl;
      nb = nb + cx * xr;
      nb = nb + cy * rc[r + 1];
      nb = nb + cz * rp[r];
      // (bitwise select: a `?:` on the two array elements became a computed address, which put
      // the array in scratch)
      const long long m = -(long long)a1;
      const double bv = __builtin_bit_cast(
          double, (__builtin_bit_cast(long long, bb[r][1]) & m) |
                      (__builtin_bit_cast(long long, bb[r][0]) & ~m));
      const double t = (bv - nb) * icc;
      const double v = (1.0 - omega) * 0.0 + omega * t;
      out[r][0] = a1 ? rc[r] : v;
      out[r][1] = a1 ? v : rc[r];
    }
  };
  double rq[3][kRW];      // red values, planes k, k+1, k+2
  double nraw[kRW][2];    // prefetch: raw b, plane k+3
  double s1[3][kRW][2];   // S1 planes k-1, k, k+1 (rows 1 .. kRW-2)
  double bq[3][kRW][2];   // raw b planes k, k+1, k+2 (rows 1 .. kRW-2)
  {
    double raw[kRW][2] = {}, ra[kRW] = {};
    ldraw(raw, kb - 2);
    redv(raw, kb - 2, ra);
    ldraw(raw, kb - 1);
    redv(raw, kb - 1, rq[0]);
    double bm[kRW][2] = {};
    keepb(raw, bm);
    ldraw(raw, kb);
    redv(raw, kb, rq[1]);
    keepb(raw, bq[0]);
    half1(ra, rq[0], rq[1], bm, kb - 1, s1[0]);
    ldraw(raw, kb + 1);
    redv(raw, kb + 1, rq[2]);
    keepb(raw, bq[1]);
    half1(rq[0], rq[1], rq[2], bq[0], kb, s1[1]);
    // queue to (kb, kb+1, kb+2)
#pragma unroll
    for (int r = 0; r < kRW; ++r) {
      rq[0][r] = rq[1][r];
      rq[1][r] = rq[2][r];
    }
    ldraw(raw, kb + 2);
    redv(raw, kb + 2, rq[2]);
    keepb(raw, bq[2]);
  }
  for (int k = kb; k < ke; ++k) {
    const bool more = k + 1 < ke;
    ldraw(nraw, more ? k + 3 : k + 2);  // unconditional: see sor_sweep2_kernel
    half1(rq[0], rq[1], rq[2], bq[1], k + 1, s1[2]);  // S1 at plane k+1
    // x = S1; res = b - A S1 at plane k (z-, y-, x-, c, x+, y+, z+)
    const int64_t base = (int64_t)k * g.plane;
#pragma unroll
    for (int r = 2; r < 2 + kTY2; ++r) {
      const double lo = dpp_from_lower(s1[1][r][1]);
      const double hi = dpp_from_upper(s1[1][r][0]);
      double rv[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const double xl = e == 0 ? lo : s1[1][r][0];
        const double xr = e == 1 ? hi : s1[1][r][1];
        double a = cz * s1[0][r][e];
        a = a + cy * s1[1][r - 1][e];
        a = a + cx * xl;
        a = a + cc * s1[1][r][e];
        a = a + cx * xr;
        a = a + cy * s1[1][r + 1][e];
        a = a + cz * s1[2][r][e];
        rv[e] = bq[0][r][e] - a;
      }
      if (out_ok && j0 + r - 2 < ny) {
        store_row<2>(xout, rix(base + ro[r]), s1[1][r], g.nt);
        store_row<2>(res, rix(base + ro[r]), rv, g.nt);
      }
    }
    // rotate: red (k+1, k+2, k+3), b (k+1, k+2, k+3), S1 (k, k+1, .)
    double rn[kRW];
    redv(nraw, k + 3, rn);
#pragma unroll
    for (int r = 0; r < kRW; ++r) {
      rq[0][r] = rq[1][r];
      rq[1][r] = rq[2][r];
      rq[2][r] = rn[r];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        s1[0][r][e] = s1[1][r][e];
        s1[1][r][e] = s1[2][r][e];
        bq[0][r][e] = bq[1][r][e];
        bq[1][r][e] = bq[2][r][e];
      }
    }
    keepb(nraw, bq[2]);
  }
}

// ---------------------------------------------------------------------------------------------
// Pre-smoothing from x = 0, residual AND restriction in one pass (one rank, or N ranks with
// three-deep ghosts of b): the residual is never stored. Per fine point: read b, write x (+ 1/8 of
// a coarse b) -- 17 B/DoF instead of the pre-smoothing pass's 24 plus the restriction's 9.
// Arithmetic: the slim pre-smoothing kernel's (red, black, residual) and mg_restrict_z_kernel's
// (restrict_xy, then the z sum in the same order), so results are bit-identical.
// Rows shared between the waves of a block (r03): a block of NW waves stacks NW x TY rows (TY / 2
// coarse rows per wave) and each wave forms red, black and residual values on its own rows only;
// the values one row out come from the neighbouring waves through LDS (red values, the smoothed
// pairs, and the residual's x sums), one block barrier per plane. Each step loses a row at the
// block's ends (red -> black -> residual -> y sum), so a block stores its fine rows 4 .. NW TY - 5
// and blocks advance by NW TY - 8 rows. The plane loop is unrolled by four: the queues (red
// values, smoothed pairs, b rows, x sums, halo values) are rings of four or two register slots
// whose roles rotate with the unrolled copy, so no value is copied from one iteration to the
// next, and each copy knows its plane's parity: with an even slab origin k0 (one rank: 0; N ranks: the MG
// plan keeps every level's slab origins even) and even extents, pair origins and
// row origins, the colour of every element is known at compile time, so the colour choices are
// register choices instead of selects and each half-sweep needs one DPP shift per row, not two.
// A chunk runs a whole number of four-plane steps (up to three planes more than it needs; they
// store nothing). Same operations on the same operands: bit-identical.
// ---------------------------------------------------------------------------------------------
// one z-range [kb, ke) of one column (x-segment seg, row tile) of presmooth_restrict_u4_kernel
template <int NW, int TY>
__device__ __forceinline__ void presmooth_restrict_u4_range(
    const Sweep2Geo& g, int ncx, int64_t cplane, double cx, double cy, double cz, double cc,
    double omega, const double* __restrict__ b, double* __restrict__ xout,
    double* __restrict__ bc, int seg, int tile, int kb, int ke, double (&xch)[2][8][NW][64]) {
  static_assert(TY % 2 == 0 && TY >= 2, "whole coarse rows per wave");
  constexpr int RB = NW * TY;
  constexpr int LO = 4;  // first stored block row
  constexpr int SB = RB - 2 * LO;
  constexpr int NCR = TY / 2;
  const double icc = 1.0 / cc;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nx = g.nx, ny = g.ny, nz = g.nzl;
  if (kb >= nz) return;
  const int g0 = tile * SB - LO;
  const int br0 = wid * TY;
  const int j0 = g0 + br0;  // even
  auto wrap = [](int v, int n) { v %= n; return v < 0 ? v + n : v; };
  int ip = seg * kSegOut + 2 * (lane - kSegLead);  // even
  if (ip < 0) ip += nx;
  if (ip >= nx) ip -= nx;
  const int o = seg * kSegOut + 2 * (lane - kSegLead);
  const bool out_ok = lane >= kSegLead && lane < kSegLead + kSegOut / 2 && o < nx;
  int64_t ro[TY];
  unsigned row_ok = 0;
#pragma unroll
  for (int r = 0; r < TY; ++r) {
    ro[r] = (int64_t)wrap(j0 + r, ny) * nx;
    const int brow = br0 + r;
    if (brow >= LO && brow < RB - LO && g0 + brow < ny) row_ok |= 1u << r;
  }
  const unsigned boff = (unsigned)ip * 8u;
  auto rix = [&](int64_t row) { return RowIx{row, boff}; };
  // planes up to a few steps past the chunk (the last step's spare planes): any distance
  auto wrapk = [&](int kk) { kk %= nz; return kk < 0 ? kk + nz : kk; };
  // b's plane kk: one rank wraps periodically; N ranks (g.split) read planes -3 .. -1 and
  // nz .. nz+2 from the ghost buffer g.xg (six planes, in that order) -- the spare planes of the
  // last unrolled step beyond those clamp (their values are never stored)
  auto bplane = [&](int kk) -> const double* {
    if (!g.split) return b + (int64_t)wrapk(kk) * g.plane;
    if (kk >= 0 && kk < nz) return b + (int64_t)kk * g.plane;
    const int gi = kk < 0 ? max(kk + 3, 0) : 3 + min(kk - nz, 2);
    return g.xg + (int64_t)gi * g.plane;
  };
  auto ldraw = [&](double (&dst)[TY][2], int kk) {
    const double* src = bplane(kk);
#pragma unroll
    for (int r = 0; r < TY; ++r) load_row<2>(src, rix(ro[r]), dst[r]);
  };
  // element holding the red point of own row r on a plane of parity P (pair origin i even, row
  // origin j0 even, k0 even): ((i + j) & 1) + kpar != 0
  auto red_e = [](int r, int P) { return (r + P) & 1; };

  auto redv = [&](auto Pc, const double (&v)[TY][2], double (&red)[TY]) {
    constexpr int P = decltype(Pc)::value;
#pragma unroll
    for (int r = 0; r < TY; ++r) {
      const double t = (v[r][red_e(r, P)] - 0.0) * icc;
      red[r] = (1.0 - omega) * 0.0 + omega * t;
    }
  };
  auto black = [&](auto Pc, const double (&rm)[TY], const double (&rc)[TY],
                   const double (&rp)[TY], const double (&rh)[2], const double (&bb)[TY][2],
                   double (&out)[TY][2]) {
    constexpr int P = decltype(Pc)::value;
#pragma unroll
    for (int r = 0; r < TY; ++r) {
      const int be = 1 - red_e(r, P);  // the black point's element
      const double xl = be ? rc[r] : dpp_from_lower(rc[r]);
      const double xr = be ? dpp_from_upper(rc[r]) : rc[r];
      double nb = cz * rm[r];
      nb = nb + cy * (r == 0 ? rh[0] : rc[r == 0 ? 0 : r - 1]);
      nb = nb + cx * xl;
      nb = nb + cx * xr;
      nb = nb + cy * (r == TY - 1 ? rh[1] : rc[r == TY - 1 ? r : r + 1]);
      nb = nb + cz * rp[r];
      const double t = (bb[r][be] - nb) * icc;
      const double v = (1.0 - omega) * 0.0 + omega * t;
      out[r][1 - be] = rc[r];
      out[r][be] = v;
    }
  };
  const int wm = wid > 0 ? wid - 1 : wid, wp = wid < NW - 1 ? wid + 1 : wid;
  const int J0 = j0 >> 1;
  const int I = o >> 1;
  const double w[4] = {0.125, 0.375, 0.375, 0.125};
  double R[4][TY];     // red values: planes k, k+1, k+2 and (new) k+3 at slots Q .. Q+3
  double S[4][TY][2];  // smoothed pairs: planes k-1, k, k+1 at slots Q .. Q+2
  double B[4][TY][2];  // b rows: planes k .. k+3 at slots Q .. Q+3
  double X[2][TY];     // residual x sums: planes k-1, k at slots Q, Q+1
  double H[2][2];      // red values of rows -1 / TY: planes k+1, k+2 at slots Q, Q+1
  double accA[NCR], accB[NCR];
  ldraw(B[3], kb - 3);
  redv(std::integral_constant<int, 1>{}, B[3], R[0]);  // planes kb-3 (odd), kb-2, kb-1
  ldraw(B[1], kb - 2);
  redv(std::integral_constant<int, 0>{}, B[1], R[1]);
  ldraw(B[2], kb - 1);
  redv(std::integral_constant<int, 1>{}, B[2], R[2]);
  xch[1][0][wid][lane] = R[1][0];
  xch[1][1][wid][lane] = R[1][TY - 1];
  __syncthreads();
  H[0][0] = xch[1][1][wm][lane];
  H[0][1] = xch[1][0][wp][lane];
  xch[0][0][wid][lane] = R[2][0];
  xch[0][1][wid][lane] = R[2][TY - 1];
#pragma unroll
  for (int r = 0; r < TY; ++r) {
    X[0][r] = 0.0;
#pragma unroll
    for (int e = 0; e < 2; ++e) S[0][r][e] = S[1][r][e] = B[0][r][e] = 0.0;
  }
#pragma unroll
  for (int c = 0; c < NCR; ++c) accA[c] = accB[c] = 0.0;
  // one plane: k = kb - 3 + Q (mod 4), parity KP = (Q + 1) & 1 (kb even)
  auto body = [&](auto Qc, int k) {
    constexpr int Q = decltype(Qc)::value;
    constexpr int KP = (Q + 1) & 1;
    double (&rq0)[TY] = R[Q];
    double (&rq1)[TY] = R[(Q + 1) & 3];
    double (&rq2)[TY] = R[(Q + 2) & 3];
    double (&rn)[TY] = R[(Q + 3) & 3];
    double (&s1m)[TY][2] = S[Q];
    double (&s1c)[TY][2] = S[(Q + 1) & 3];
    double (&s1p)[TY][2] = S[(Q + 2) & 3];
    double (&bq0)[TY][2] = B[Q];
    double (&bq1)[TY][2] = B[(Q + 1) & 3];
    double (&raw)[TY][2] = B[(Q + 3) & 3];
    double (&sxp)[TY] = X[Q & 1];
    double (&sxc)[TY] = X[(Q + 1) & 1];
    double (&rh1)[2] = H[Q & 1];
    double (&rh2)[2] = H[(Q + 1) & 1];
    ldraw(raw, k + 3);
    __syncthreads();
    double sh[2][2], sxh[2];
    {
      constexpr int rp = KP ^ 1;  // written by plane k-1
      rh2[0] = xch[rp][1][wm][lane];
      rh2[1] = xch[rp][0][wp][lane];
      sh[0][0] = xch[rp][4][wm][lane];
      sh[0][1] = xch[rp][5][wm][lane];
      sh[1][0] = xch[rp][2][wp][lane];
      sh[1][1] = xch[rp][3][wp][lane];
      sxh[0] = xch[rp][7][wm][lane];
      sxh[1] = xch[rp][6][wp][lane];
    }
    black(std::integral_constant<int, KP ^ 1>{}, rq0, rq1, rq2, rh1, bq1, s1p);  // plane k+1
    xch[KP][2][wid][lane] = s1p[0][0];
    xch[KP][3][wid][lane] = s1p[0][1];
    xch[KP][4][wid][lane] = s1p[TY - 1][0];
    xch[KP][5][wid][lane] = s1p[TY - 1][1];
    if (k >= kb - 1 && k <= ke) {
#pragma unroll
      for (int r = 0; r < TY; ++r) {
        const double lo = dpp_from_lower(s1c[r][1]);
        const double hi = dpp_from_upper(s1c[r][0]);
        double rv[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const double xl = e == 0 ? lo : s1c[r][0];
          const double xr = e == 1 ? hi : s1c[r][1];
          const double ym = r == 0 ? sh[0][e] : s1c[r == 0 ? 0 : r - 1][e];
          const double yp = r == TY - 1 ? sh[1][e] : s1c[r == TY - 1 ? r : r + 1][e];
          double a = cz * s1m[r][e];
          a = a + cy * ym;
          a = a + cx * xl;
          a = a + cc * s1c[r][e];
          a = a + cx * xr;
          a = a + cy * yp;
          a = a + cz * s1p[r][e];
          rv[e] = bq0[r][e] - a;
        }
        const double rlo = dpp_from_lower(rv[1]);
        const double rhi = dpp_from_upper(rv[0]);
        double sx = w[0] * rlo;
        sx = sx + w[1] * rv[0];
        sx = sx + w[2] * rv[1];
        sx = sx + w[3] * rhi;
        sxc[r] = sx;
      }
      if (k >= kb && k < ke && out_ok) {
        const int64_t base = (int64_t)k * g.plane;
#pragma unroll
        for (int r = 0; r < TY; ++r)
          if (row_ok >> r & 1u) store_row<2>(xout, rix(base + ro[r]), s1c[r], g.nt);
      }
    } else {
#pragma unroll
      for (int r = 0; r < TY; ++r) sxc[r] = 0.0;
    }
    xch[KP][6][wid][lane] = sxc[0];
    xch[KP][7][wid][lane] = sxc[TY - 1];
    const int kr = k - 1;  // restriction of plane k-1 (parity KP ^ 1)
    if (kr >= kb - 1) {
#pragma unroll
      for (int c = 0; c < NCR; ++c) {
        double sy = 0.0;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
          const int r = 2 * c - 1 + bb;
          const double sxv = r < 0 ? sxh[0] : (r >= TY ? sxh[1] : sxp[r < 0 ? 0 : (r >= TY ? 0 : r)]);
          sy = sy + w[bb] * sxv;
        }
        if constexpr ((KP ^ 1) == 1) {  // kr = 2K-1
          accB[c] = accB[c] + 0.375 * sy;
          accA[c] = 0.0;
          accA[c] = accA[c] + 0.125 * sy;
        } else {  // kr = 2K
          accB[c] = accB[c] + 0.125 * sy;
          if (kr >= kb + 2 && kr <= ke && out_ok && (row_ok >> (2 * c) & 1u))
            bc[(int64_t)((kr >> 1) - 1) * cplane + (int64_t)wrap(J0 + c, ny >> 1) * ncx + I] =
                accB[c];
          accA[c] = accA[c] + 0.375 * sy;
          accB[c] = accA[c];
        }
      }
    }
    redv(std::integral_constant<int, KP ^ 1>{}, raw, rn);  // plane k+3
    xch[KP][0][wid][lane] = rn[0];
    xch[KP][1][wid][lane] = rn[TY - 1];
  };
#pragma unroll 1
  for (int k = kb - 3; k <= ke + 1; k += 4) {
    body(std::integral_constant<int, 0>{}, k);
    body(std::integral_constant<int, 1>{}, k + 1);
    body(std::integral_constant<int, 2>{}, k + 2);
    body(std::integral_constant<int, 3>{}, k + 3);
  }
}

// Work split (g.wsplit = W > 0): every workgroup gets W planes of work whatever the column count
// (512^3: 110 columns of 512 planes as 2 chunks each leave 36 of 256 CUs idle). Bands first:
// band t = planes [t W, (t + 1) W) of every column, one workgroup per column and band, so the
// workgroups running together stay at a few z-positions (pieces at scattered planes were 30 %
// slower at 512^3); then the last, lower band [T W, nz) of all columns laid end to end
// (column-major) and cut into pieces of W planes -- a piece may run the end of one column and
// the start of the next, each z-range with its own few warm-up planes. fn(col, kb, ke) per range.
template <class F>
__device__ __forceinline__ void split_ranges(const Sweep2Geo& g, int bid, F&& fn) {
  const int ncol = g.nseg * g.ntile, W = g.wsplit, T = g.nzl / W;
  if (bid < T * ncol) {
    const int kb = (bid / ncol) * W;
    fn(bid % ncol, kb, kb + W);
    return;
  }
  const int k0 = T * W, h = g.nzl - k0;
  if (h <= 0) return;
  const int64_t total = (int64_t)ncol * h;
  const int64_t e = min(total, (int64_t)(bid - T * ncol + 1) * W);
  for (int64_t s = (int64_t)(bid - T * ncol) * W; s < e;) {
    const int col = (int)(s / h);
    const int kb = (int)(s - (int64_t)col * h);
    const int ke = (int)min((int64_t)h, kb + (e - s));
    fn(col, k0 + kb, k0 + ke);
    s += ke - kb;
  }
}

template <int NW, int TY>
__global__ __launch_bounds__(64 * NW) void presmooth_restrict_u4_kernel(
    Sweep2Geo g, int ncx, int64_t cplane, double cx, double cy, double cz, double cc,
    double omega, const double* __restrict__ b, double* __restrict__ xout,
    double* __restrict__ bc, const int* skip) {
  // per plane parity, per wave: red values of own rows 0 / TY-1 (plane k+3), smoothed pairs of
  // rows 0 / TY-1 (plane k+1: e0, e1 each), residual x sums of rows 0 / TY-1 (plane k)
  __shared__ double xch[2][8][NW][64];
  if (skip && *skip) return;
  int bid = xcd_block(g.remap);
  if (g.wsplit > 0) {  // ranges start on even planes (W, nzl even)
    split_ranges(g, bid, [&](int col, int kb, int ke) {
      presmooth_restrict_u4_range<NW, TY>(g, ncx, cplane, cx, cy, cz, cc, omega, b, xout, bc,
                                          col % g.nseg, col / g.nseg, kb, ke, xch);
      __syncthreads();  // the next range rewrites the exchange slots
    });
    return;
  }
  const int seg = bid % g.nseg;
  bid /= g.nseg;
  const int tile = bid % g.ntile;
  const int chunk = bid / g.ntile;
  const int kb = chunk * g.kc;  // even (kc even)
  presmooth_restrict_u4_range<NW, TY>(g, ncx, cplane, cx, cy, cz, cc, omega, b, xout, bc, seg,
                                      tile, kb, min(kb + g.kc, g.nzl), xch);
}

// ---------------------------------------------------------------------------------------------
// Post-smoothing with the prolongation folded in (one rank; the unrolled form also on N ranks with
// deep ghost planes, r04): the sweep's input
// xin = x_s + P x_c is formed as the planes arrive -- x_s (the pre-smoothed iterate) and the
// coarse correction x_c are read, the prolongated input is never stored. Then both half-sweeps
// (c1 = 1 first, then the other colour) out of place into xout, CG's residual sums optional.
// Per fine point: read x_s and b, write xout (+ 1/8 of a coarse value): 24 B/DoF instead of the
// prolongation pass's 16 plus the sweep's 24. Arithmetic: mg_prolong_z_kernel's interpolation
// (x-stage, then y, then z, same operation order) and sor_sweep2_kernel's half-sweeps, so the
// result is bit-identical. The first-half queue keeps only the c1 value of each pair (the
// second half-sweep reads only c1 points; the c2 values are the input's), which pays for the
// coarse-value prefetch in registers.
// ---------------------------------------------------------------------------------------------
struct PostGeo {
  int ncx, ncy, ncz;   // coarse extents (one rank: the whole coarse grid; N ranks: the slab)
  int64_t cplane;
  // N ranks (post_sweep_u4_kernel): the coarse correction's planes -2, -1, ncz, ncz+1 (in that
  // order) at cgh[0..3]; the fine x_s ghosts (-2, -1, nz, nz+1) in Sweep2Geo::xg, b's in bg_lo /
  // bg_hi
  int split;
  const double* cgh[4];
};

// ---------------------------------------------------------------------------------------------
// The post-smoothing pass (r03): rows shared between the waves of a block through LDS as in
// presmooth_restrict_u4_kernel -- a wave loads its own input rows only, the rows one out (the
// prolongated input and the first-half values) come from the neighbouring waves, published one
// plane before use, one barrier per plane; a block stores rows 2 .. NW TY - 3 -- and the plane
// loop unrolled by four: the queues (input planes with their halo rows, first-half values,
// c2 inputs and right-hand sides, halo first-half values) are rings of four or two register slots
// whose roles rotate with the unrolled copy, and each copy knows its plane's parity (even k0,
// even extents and origins), so the colour choices are register choices and each half-sweep
// shifts one value per row. A chunk runs a whole number of four-plane steps (the last step's
// extra planes store nothing). Same operations on the same operands: bit-identical.
// ---------------------------------------------------------------------------------------------
// one z-range [kb, ke) (kb a multiple of 4) of one column of post_sweep_u4_kernel; CG's
// residual sums accumulate into acc
template <bool SUMS, int NW, int TY>
__device__ __forceinline__ void post_sweep_u4_range(
    const Sweep2Geo& g, const PostGeo& cgeo, double cx, double cy, double cz, double cc,
    double omega, const double* __restrict__ xs, const double* __restrict__ xc,
    const double* __restrict__ b, double* __restrict__ xout, double mu, int seg, int tile, int kb,
    int ke, double (&xch)[2][6][NW][64], double (&acc)[4]) {
  static_assert(TY % 2 == 0 && TY >= 2, "own rows start on an even fine row");
  constexpr int RB = NW * TY;
  constexpr int SB = RB - 4;
  constexpr int NC = TY / 2 + 2;
  const double icc = 1.0 / cc;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nx = g.nx, ny = g.ny, nz = g.nzl;
  if (kb < nz) {
    const int g0 = tile * SB - 2;
    const int br0 = wid * TY;
    const int j0 = g0 + br0;  // even
    auto wrap = [](int v, int n) { v %= n; return v < 0 ? v + n : v; };
    int ip = seg * kSegOut + 2 * (lane - kSegLead);  // even
    if (ip < 0) ip += nx;
    if (ip >= nx) ip -= nx;
    const int o = seg * kSegOut + 2 * (lane - kSegLead);
    const bool out_ok = lane >= kSegLead && lane < kSegLead + kSegOut / 2 && o < nx;
    int64_t ro[TY];
    unsigned row_ok = 0;
#pragma unroll
    for (int r = 0; r < TY; ++r) {
      ro[r] = (int64_t)wrap(j0 + r, ny) * nx;
      const int brow = br0 + r;
      if (brow >= 2 && brow < RB - 2 && g0 + brow < ny) row_ok |= 1u << r;
    }
    const unsigned boff = (unsigned)ip * 8u;
    auto rix = [&](int64_t row) { return RowIx{row, boff}; };
    // planes up to a few steps past the chunk (the last step's spare planes): any distance
    auto wrapk = [&](int kk) { kk %= nz; return kk < 0 ? kk + nz : kk; };
    auto pl = [&](int kk) -> int64_t { return (int64_t)wrapk(kk) * g.plane; };
    int64_t crow[NC];
#pragma unroll
    for (int t = 0; t < NC; ++t) crow[t] = (int64_t)wrap((j0 >> 1) - 1 + t, cgeo.ncy) * cgeo.ncx;
    const unsigned cboff = (unsigned)(ip >> 1) * 8u;
    // x_s rows of plane kk into rows 1 .. TY of dst
    // N ranks (g.split): planes outside the slab from the ghost buffers (x_s two deep, b one
    // deep, the coarse correction two deep); the last unrolled step's spare planes clamp
    auto xsplane = [&](int kk) -> const double* {
      if (!g.split) return xs + pl(kk);
      if (kk >= 0 && kk < nz) return xs + (int64_t)kk * g.plane;
      const int gi = kk < 0 ? max(kk + 2, 0) : 2 + min(kk - nz, 1);
      return g.xg + (int64_t)gi * g.plane;
    };
    auto ldx = [&](double (&dst)[TY + 2][2], int kk) {
      const double* src = xsplane(kk);
#pragma unroll
      for (int r = 0; r < TY; ++r) load_row<2>(src, rix(ro[r]), dst[r + 1]);
    };
    // coarse plane K (periodic) under the own rows
    auto ldc = [&](double (&cv)[NC], int K) {
      const double* cp;
      if (!cgeo.split) {
        K %= cgeo.ncz;
        if (K < 0) K += cgeo.ncz;
        cp = xc + (int64_t)K * cgeo.cplane;
      } else if (K >= 0 && K < cgeo.ncz) {
        cp = xc + (int64_t)K * cgeo.cplane;
      } else {
        const int gi = K < 0 ? max(K + 2, 0) : 2 + min(K - cgeo.ncz, 1);
        cp = cgeo.cgh[gi];
      }
#pragma unroll
      for (int t = 0; t < NC; ++t)
        cv[t] = *reinterpret_cast<const double*>(reinterpret_cast<const char*>(cp + crow[t]) + cboff);
    };
    // one coarse plane interpolated in x, then in y onto each own row (mg_prolong_z_kernel's
    // operations, formed once per coarse plane instead of once per fine plane that reads it --
    // each serves the two fine planes it is near to and the two it is far from)
    auto yinterp = [&](const double (&cv)[NC], double (&Y)[TY][2]) {
      double xi[NC][2];
#pragma unroll
      for (int t = 0; t < NC; ++t) {
        const double c = cv[t];
        xi[t][0] = 0.75 * c + 0.25 * dpp_from_lower(c);
        xi[t][1] = 0.75 * c + 0.25 * dpp_from_upper(c);
      }
#pragma unroll
      for (int r = 0; r < TY; ++r) {
        const int tJ = 1 + (r >> 1);
        const int tf = (r & 1) ? tJ + 1 : tJ - 1;
#pragma unroll
        for (int e = 0; e < 2; ++e) Y[r][e] = 0.75 * xi[tJ][e] + 0.25 * xi[tf][e];
      }
    };
    // x_s + P x_c on the own rows: Yn, Yf = the near / far coarse planes' interpolants
    auto prolong = [&](double (&v)[TY + 2][2], const double (&Yn)[TY][2],
                       const double (&Yf)[TY][2]) {
#pragma unroll
      for (int r = 0; r < TY; ++r)
#pragma unroll
        for (int e = 0; e < 2; ++e) v[r + 1][e] = v[r + 1][e] + (0.75 * Yn[r][e] + 0.25 * Yf[r][e]);
    };
    auto ldb = [&](double (&dst)[TY][2], int kk) {
      const double* src = !g.split ? b + pl(kk)
                          : (kk >= 0 && kk < nz ? b + (int64_t)kk * g.plane
                                                : (kk < 0 ? g.bg_lo : g.bg_hi));
#pragma unroll
      for (int r = 0; r < TY; ++r) load_row<2>(src, rix(ro[r]), dst[r]);
    };
    // element of the c1 (first-half) point of own row r on a plane of parity P (((i + j) & 1) =
    // r & 1, c1 = 1)
    auto e1 = [](int r, int P) { return ((r + P) & 1) ^ 1; };
    auto half1 = [&](auto Pc, const double (&zmv)[TY], const double (&xcn)[TY + 2][2],
                     const double (&xp)[TY + 2][2], const double (&bb)[TY][2],
                     double (&out)[TY]) {
      constexpr int P = decltype(Pc)::value;
#pragma unroll
      for (int r = 0; r < TY; ++r) {
        const int e = e1(r, P);
        const double xl = e ? xcn[r + 1][0] : dpp_from_lower(xcn[r + 1][1]);
        const double xr = e ? dpp_from_upper(xcn[r + 1][0]) : xcn[r + 1][1];
        double nb = cz * zmv[r];
        nb = nb + cy * xcn[r][e];
        nb = nb + cx * xl;
        nb = nb + cx * xr;
        nb = nb + cy * xcn[r + 2][e];
        nb = nb + cz * xp[r + 1][e];
        const double t = (bb[r][e] - nb) * icc;
        out[r] = (1.0 - omega) * xcn[r + 1][e] + omega * t;
      }
    };
    auto half2 = [&](auto Pc, int kk, const double (&sm)[TY], const double (&sc)[TY],
                     const double (&sp)[TY], const double (&sh)[2], const double (&xo)[TY],
                     const double (&bo)[TY], const double (&bc1)[SUMS ? TY : 1]) {
      constexpr int P = decltype(Pc)::value;
      const int64_t base = pl(kk);
#pragma unroll
      for (int r = 0; r < TY; ++r) {
        const int e2 = e1(r, P) ^ 1;  // the second-colour point's element
        const double cself = sc[r];
        const double xl = e2 ? cself : dpp_from_lower(cself);
        const double xr = e2 ? dpp_from_upper(cself) : cself;
        double nb = cz * sm[r];
        nb = nb + cy * (r == 0 ? sh[0] : sc[r == 0 ? 0 : r - 1]);
        nb = nb + cx * xl;
        nb = nb + cx * xr;
        nb = nb + cy * (r == TY - 1 ? sh[1] : sc[r == TY - 1 ? r : r + 1]);
        nb = nb + cz * sp[r];
        const double t = (bo[r] - nb) * icc;
        const double v = (1.0 - omega) * xo[r] + omega * t;
        double ov[2];
        ov[e2] = v;
        ov[e2 ^ 1] = cself;
        if (out_ok && (row_ok >> r & 1u)) {
          store_row<2>(xout, rix(base + ro[r]), ov, g.nt);
          if constexpr (SUMS) {
            double rv2[2];
            rv2[e2] = bo[r];
            rv2[e2 ^ 1] = bc1[r];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const double t2 = ov[e] - mu;
              acc[0] += t2;
              acc[1] += t2 * t2;
              acc[2] += t2 * rv2[e];
              acc[3] += rv2[e];
            }
          }
        }
      }
    };
    const int wm = wid > 0 ? wid - 1 : wid, wp = wid < NW - 1 ? wid + 1 : wid;
    auto put_x = [&](int par, const double (&v)[TY + 2][2]) {
      xch[par][0][wid][lane] = v[1][0];
      xch[par][1][wid][lane] = v[1][1];
      xch[par][2][wid][lane] = v[TY][0];
      xch[par][3][wid][lane] = v[TY][1];
    };
    double XQ[2][TY + 2][2];  // input planes k+1 (rows -1 .. TY), k+2 (own rows) at Q, Q+1
    double XM[2][TY];         // input c2 values: planes k-1, k at Q, Q+1
    double S1[4][TY];         // first-half values: planes k-2 .. k+1 at Q .. Q+3
    double SH[2][2];          // first-half values of rows -1 / TY: planes k-1, k at Q, Q+1
    double BB[2][TY];         // b at c2 points: planes k-1, k at Q, Q+1
    double BB1[2][SUMS ? TY : 1];  // b at c1 points (sums only)
    // coarse interpolants: slot K & 1 holds coarse plane K (kb a multiple of 4, K0 = kb / 2 even)
    double YC[2][TY][2];
    const int K0 = kb >> 1;
    {
      double cv[NC];
      ldc(cv, K0 - 2);
      yinterp(cv, YC[0]);
      ldc(cv, K0 - 1);
      yinterp(cv, YC[1]);
      ldx(XQ[1], kb - 2);  // plane kb-2 (even; near K0-1, far K0-2): its c2 values only
      prolong(XQ[1], YC[1], YC[0]);
#pragma unroll
      for (int r = 0; r < TY; ++r) XM[1][r] = XQ[1][r + 1][e1(r, 0) ^ 1];
      ldc(cv, K0);
      yinterp(cv, YC[0]);
      ldx(XQ[0], kb - 1);  // plane kb-1 (near K0-1, far K0)
      prolong(XQ[0], YC[1], YC[0]);
      put_x(1, XQ[0]);  // as if iteration kb-3 (odd) had formed plane kb-1
    }
#pragma unroll
    for (int r = 0; r < TY; ++r) {
      XM[0][r] = BB[0][r] = BB[1][r] = 0.0;
      S1[0][r] = S1[1][r] = S1[2][r] = 0.0;
      if constexpr (SUMS) BB1[0][r] = BB1[1][r] = 0.0;
    }
    SH[0][0] = SH[0][1] = 0.0;
    // one plane: k = kb - 2 + Q (mod 4), parity Q & 1
    auto body = [&](auto Qc, int k) {
      constexpr int Q = decltype(Qc)::value;
      constexpr int KP = Q & 1;
      double (&xq1)[TY + 2][2] = XQ[Q & 1];
      double (&xq2)[TY + 2][2] = XQ[(Q + 1) & 1];
      double (&xm)[TY] = XM[Q & 1];
      double (&x0)[TY] = XM[(Q + 1) & 1];
      double (&bm)[TY] = BB[Q & 1];  // (plane k's sits in the other slot until the next copy)
      double (&bm1)[SUMS ? TY : 1] = BB1[Q & 1];
      double (&shp)[2] = SH[Q & 1];
      double (&shc)[2] = SH[(Q + 1) & 1];
      // plane k+2 = kb + 4m + Q: even (Q even) -> near K, far K-1; odd -> near K, far K+1 (new),
      // K = (k + 2) >> 1 = K0 + 2m + (Q >> 1)
      constexpr int KN = Q >> 1;  // near coarse plane's slot (K0 even)
      double bq1[TY][2], cv[NC];
      ldx(xq2, k + 2);
      if constexpr (Q & 1) ldc(cv, ((k + 2) >> 1) + 1);
      ldb(bq1, k + 1);
      __syncthreads();
      {
        constexpr int rp = KP ^ 1;
        xq1[0][0] = xch[rp][2][wm][lane];
        xq1[0][1] = xch[rp][3][wm][lane];
        xq1[TY + 1][0] = xch[rp][0][wp][lane];
        xq1[TY + 1][1] = xch[rp][1][wp][lane];
        shc[0] = xch[rp][5][wm][lane];
        shc[1] = xch[rp][4][wp][lane];
      }
      if (k > kb && k <= ke)
        half2(std::integral_constant<int, KP ^ 1>{}, k - 1, S1[Q], S1[(Q + 1) & 3],
              S1[(Q + 2) & 3], shp, xm, bm, bm1);
      if constexpr (Q & 1) yinterp(cv, YC[KN ^ 1]);
      prolong(xq2, YC[KN], YC[KN ^ 1]);
      put_x(KP, xq2);
      double (&s1n)[TY] = S1[(Q + 3) & 3];
      half1(std::integral_constant<int, KP ^ 1>{}, x0, xq1, xq2, bq1, s1n);  // plane k+1
      xch[KP][4][wid][lane] = s1n[0];
      xch[KP][5][wid][lane] = s1n[TY - 1];
      // plane k+1's c2 input values and right-hand side replace plane k-1's
#pragma unroll
      for (int r = 0; r < TY; ++r) {
        const int e = e1(r, KP ^ 1);
        xm[r] = xq1[r + 1][e ^ 1];
        bm[r] = bq1[r][e ^ 1];
        if constexpr (SUMS) bm1[r] = bq1[r][e];
      }
    };
#pragma unroll 1
    for (int k = kb - 2; k <= ke; k += 4) {
      body(std::integral_constant<int, 0>{}, k);
      body(std::integral_constant<int, 1>{}, k + 1);
      body(std::integral_constant<int, 2>{}, k + 2);
      body(std::integral_constant<int, 3>{}, k + 3);
    }
  }
}

// g.wsplit > 0: the balanced work split of presmooth_restrict_u4_kernel (split_ranges; W a
// multiple of 4, so every z-range starts on a multiple of 4)
template <bool SUMS, int NW, int TY>
__global__ __launch_bounds__(64 * NW) void post_sweep_u4_kernel(
    Sweep2Geo g, PostGeo cgeo, double cx, double cy, double cz, double cc, double omega,
    const double* __restrict__ xs, const double* __restrict__ xc, const double* __restrict__ b,
    double* __restrict__ xout, const CgState* st, double* parts, const int* skip) {
  // per plane parity, per wave: the prolongated input of own rows 0 / TY-1 (e0, e1 each), the
  // first-half values of rows 0 / TY-1
  __shared__ double xch[2][6][NW][64];
  if (skip && *skip) return;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  const double mu = SUMS ? st->mu : 0.0;
  int bid = xcd_block(g.remap);
  if (g.wsplit > 0) {  // ranges start on multiples of 4 (W, nzl multiples of 4)
    split_ranges(g, bid, [&](int col, int kb, int ke) {
      post_sweep_u4_range<SUMS, NW, TY>(g, cgeo, cx, cy, cz, cc, omega, xs, xc, b, xout, mu,
                                        col % g.nseg, col / g.nseg, kb, ke, xch, acc);
      __syncthreads();  // the next range rewrites the exchange slots
    });
  } else {
    const int seg = bid % g.nseg;
    bid /= g.nseg;
    const int tile = bid % g.ntile;
    const int chunk = bid / g.ntile;
    const int kb = chunk * g.kc;
    post_sweep_u4_range<SUMS, NW, TY>(g, cgeo, cx, cy, cz, cc, omega, xs, xc, b, xout, mu, seg,
                                      tile, kb, min(kb + g.kc, g.nzl), xch, acc);
  }
  if constexpr (SUMS) block_partials<4>(acc, parts);
}

// even extents, nx >= 128, >= 4 planes per rank: the fused sweep applies (else two half-sweeps)
bool sor_sweep2_supported(const pb_grid* g) {
  return g->n[0] >= 128 && g->n[0] % 2 == 0 && g->n[1] % 2 == 0 && g->n[1] >= 8 &&
         g->nzl >= 4 && tune("mg_sweep2", 1) != 0;
}

// the six-plane deep-ghost buffer of a grid (pb_grid::ghost2)
static int ensure_ghost2(pb_grid* g) {
  if (!g->ghost2 && hipMalloc(&g->ghost2, 6 * (size_t)g->plane * sizeof(double)) != hipSuccess)
    return set_error(PB_ERR_ALLOC, "deep ghost planes: out of device memory");
  return PB_OK;
}

// N ranks: two-deep ghosts of xin (and, when b is another array, one-deep ghosts of b)
static int sweep2_ghosts(pb_grid* g, const double* xin, const double* b, Sweep2Geo& geo) {
  geo.split = g->ctx->split ? 1 : 0;
  geo.xg = geo.bg_lo = geo.bg_hi = nullptr;
  if (!geo.split) return PB_OK;
  PB_TRY(ensure_ghost2(g));
  PB_TRY(halo_exchange_n(g, xin, xin + (g->nzl - 2) * g->plane, 2, g->ghost2,
                         g->ghost2 + 2 * g->plane));
  geo.xg = g->ghost2;
  if (b == xin) {
    geo.bg_lo = g->ghost2 + g->plane;      // plane -1
    geo.bg_hi = g->ghost2 + 2 * g->plane;  // plane nzl
  } else {
    PB_TRY(halo_exchange(g, b, b + (g->nzl - 1) * g->plane));
    geo.bg_lo = g->ghost_lo;
    geo.bg_hi = g->ghost_hi;
  }
  return PB_OK;
}

static int64_t sweep2_geo(pb_grid* g, Sweep2Geo& geo) {
  geo.nx = (int)g->n[0];
  geo.ny = (int)g->n[1];
  geo.nzl = (int)g->nzl;
  geo.plane = g->plane;
  geo.nseg = (geo.nx + kSegOut - 1) / kSegOut;
  geo.ntile = (geo.ny + kWaves * kTY2 - 1) / (kWaves * kTY2);
  geo.k0 = (int)g->k0;
  geo.remap = 1;
  geo.nt = 1;
  const int columns = geo.nseg * geo.ntile;
  // chunks: ~PB_SWEEP2_WGCU (16) workgroups per CU (many rounds: the loop is latency-bound),
  // at least 16 planes per chunk
  const int target = 16 * g->ctx->num_cus;
  int nchunk = std::max(1, (target + columns - 1) / columns);
  nchunk = std::min(nchunk, std::max(1, geo.nzl / 16));
  geo.kc = (geo.nzl + nchunk - 1) / nchunk;
  geo.nchunk = (geo.nzl + geo.kc - 1) / geo.kc;
  return (int64_t)columns * geo.nchunk;
}

int launch_sor_sweep2(pb_grid* g, const Star& s, const double* xin, const double* b, double* xout,
                      double omega, int c1, const int* skip, const CgState* sums_st, int* nparts) {
  ScopedTimer tm(g->ctx, "mg_sor_sweep2");
  if (xin == xout) return set_error(PB_ERR_ARG, "fused SOR sweep must run out of place");
  Sweep2Geo geo;
  const int64_t nblocks = sweep2_geo(g, geo);
  PB_TRY(sweep2_ghosts(g, xin, b, geo));
  if (sums_st) {
    if (nblocks * 4 > g->ctx->partials_cap)
      return set_error(PB_ERR_UNSUPPORTED, "fused sweep of %lld blocks exceeds partials capacity",
                       (long long)nblocks);
    auto kern = geo.split ? sor_sweep2_kernel<true, true> : sor_sweep2_kernel<true, false>;
    hipLaunchKernelGGL(kern, dim3((unsigned)nblocks), dim3(kThreads), 0,
                       g->ctx->stream, geo, s.cx, s.cy, s.cz, s.cc, omega, c1, xin, b, xout,
                       sums_st, g->ctx->d_partials, skip);
    if (nparts) *nparts = (int)nblocks;
  } else {
    auto kern = geo.split ? sor_sweep2_kernel<false, true> : sor_sweep2_kernel<false, false>;
    hipLaunchKernelGGL(kern, dim3((unsigned)nblocks), dim3(kThreads), 0,
                       g->ctx->stream, geo, s.cx, s.cy, s.cz, s.cc, omega, c1, xin, b, xout,
                       (const CgState*)nullptr, (double*)nullptr, skip);
  }
  PB_HIP(hipGetLastError());
  return PB_OK;
}

// The u4 kernels' balanced work split (Sweep2Geo::wsplit): per_cu workgroups per CU, pieces of a
// multiple of `align` planes (the kernels' chunk-start parity); per_cu = 0 keeps the chunks.
// Returns the workgroup count.
static int64_t balanced_split(const pb_grid* g, Sweep2Geo& geo, int per_cu, int align,
                              int64_t nblocks) {
  geo.wsplit = 0;
  if (per_cu <= 0 || geo.nzl % align) return nblocks;
  const int64_t ncol = (int64_t)geo.nseg * geo.ntile, total = ncol * geo.nzl;
  int64_t w = (total + (int64_t)per_cu * g->ctx->num_cus - 1) / ((int64_t)per_cu * g->ctx->num_cus);
  w = std::min<int64_t>((w + align - 1) / align * align, geo.nzl);
  geo.wsplit = (int)w;
  const int64_t T = geo.nzl / w, h = geo.nzl - T * w;  // split_ranges: T bands, then the rest
  return T * ncol + (ncol * h + w - 1) / w;
}

int launch_post_sweep(pb_grid* g, const Star& s, const pb_grid* cg, const double* xs,
                      const double* xc, const double* b, double* xout, double omega,
                      const int* skip, const CgState* sums_st, int* nparts,
                      const double* xc_full) {
  ScopedTimer tm(g->ctx, "mg_post_sweep");
  const bool split = g->ctx->split;
  if (xs == xout) return set_error(PB_ERR_ARG, "fused post-smoothing must run out of place");
  if (cg->n[0] * 2 != g->n[0] || cg->n[1] * 2 != g->n[1] || cg->nzl * 2 != g->nzl)
    return set_error(PB_ERR_ARG, "fused post-smoothing: coarse grid is not half the fine one");
  Sweep2Geo geo;
  int64_t nblocks = sweep2_geo(g, geo);
  geo.split = 0;
  geo.xg = geo.bg_lo = geo.bg_hi = nullptr;
  PostGeo cgeo{(int)cg->n[0], (int)cg->n[1], (int)cg->nzl, cg->plane, 0,
                {nullptr, nullptr, nullptr, nullptr}};
  if (split) {  // x_s two deep, b one deep, the coarse correction two deep
    pb_grid* gc = const_cast<pb_grid*>(cg);
    if (g->nzl < 2 || gc->nzl < 2)
      return set_error(PB_ERR_UNSUPPORTED, "fused post-smoothing: slabs of < 2 planes");
    PB_TRY(ensure_ghost2(g));
    PB_TRY(ensure_ghost2(gc));
    PB_TRY(halo_exchange_n(g, xs, xs + (g->nzl - 2) * g->plane, 2, g->ghost2,
                           g->ghost2 + 2 * g->plane));
    PB_TRY(halo_exchange(g, b, b + (g->nzl - 1) * g->plane));
    geo.split = 1;
    geo.xg = g->ghost2;
    geo.bg_lo = g->ghost_lo;
    geo.bg_hi = g->ghost_hi;
    cgeo.split = 1;
    if (xc_full) {
      // the agglomerated coarse level: every rank holds the whole coarse correction, so its
      // planes -2, -1, nzl, nzl+1 are read in place (no coarse halo exchange)
      const int64_t nzc = gc->n[2];
      for (int i = 0; i < 4; ++i) {
        const int64_t kk = i < 2 ? gc->k0 - 2 + i : gc->k0 + gc->nzl + (i - 2);
        cgeo.cgh[i] = xc_full + ((kk % nzc + nzc) % nzc) * gc->plane;
      }
    } else {
      PB_TRY(halo_exchange_n(gc, xc, xc + (gc->nzl - 2) * gc->plane, 2, gc->ghost2,
                             gc->ghost2 + 2 * gc->plane));
      for (int i = 0; i < 4; ++i) cgeo.cgh[i] = gc->ghost2 + (int64_t)i * gc->plane;
    }
  }
  // 8 waves x 4 rows (unrolled: compile-time colours need an even k0, chunks start at multiples
  // of 4)
  constexpr int nw = 8, ty = 4;
  geo.ntile = (geo.ny + nw * ty - 5) / (nw * ty - 4);
  const int columns = geo.nseg * geo.ntile;
  // z-chunks: every chunk re-reads two planes and runs up to five spare ones, so chunks stay
  // >= 64 planes where the grid has 512 (measured: 0.733 -> 0.700 ms at 512^3 against 16) and
  // >= nz / 8 on shallower grids, which need the workgroups (~8 per CU)
  const int target = 8 * g->ctx->num_cus;
  int nchunk = std::max(1, (target + columns - 1) / columns);
  const int minz = std::min(64, std::max(16, geo.nzl / 8));
  nchunk = std::min(nchunk, std::max(1, geo.nzl / minz));
  geo.kc = (geo.nzl + nchunk - 1) / nchunk;
  geo.kc = (geo.kc + 3) & ~3;
  geo.nchunk = (geo.nzl + geo.kc - 1) / geo.kc;
  nblocks = (int64_t)columns * geo.nchunk;
  if (g->k0 % 2 != 0)
    return set_error(PB_ERR_UNSUPPORTED, "fused post-smoothing: odd slab origin");
  // (mg_u4_split: the balanced work split, tests only -- slower here at any count, r04)
  nblocks = balanced_split(g, geo, std::max(0, tune("mg_u4_split", 0)), 4, nblocks);
  if (sums_st && nblocks * 4 > g->ctx->partials_cap)
    return set_error(PB_ERR_UNSUPPORTED, "fused sweep of %lld blocks exceeds partials capacity",
                     (long long)nblocks);
  auto kern = sums_st ? post_sweep_u4_kernel<true, nw, ty> : post_sweep_u4_kernel<false, nw, ty>;
  hipLaunchKernelGGL(kern, dim3((unsigned)nblocks), dim3(64 * nw), 0, g->ctx->stream, geo, cgeo,
                     s.cx, s.cy, s.cz, s.cc, omega, xs, xc, b, xout, sums_st,
                     sums_st ? g->ctx->d_partials : (double*)nullptr, skip);
  if (sums_st && nparts) *nparts = (int)nblocks;
  PB_HIP(hipGetLastError());
  return PB_OK;
}

int launch_presmooth_restrict(pb_grid* g, const Star& s, const pb_grid* cg, const double* b,
                              double* xout, double* bc, double omega, const int* skip) {
  ScopedTimer tm(g->ctx, "mg_presmooth_restrict");
  const bool split = g->ctx->split;
  if (split && g->nzl < 3)
    return set_error(PB_ERR_UNSUPPORTED, "fused restriction on N ranks: >= 3 planes per slab");
  if (b == xout) return set_error(PB_ERR_ARG, "fused pre-smoothing must run out of place");
  if (!sor_sweep2_supported(g) || g->nzl % 2)
    return set_error(PB_ERR_UNSUPPORTED, "fused restriction: grid not supported");
  if (cg->n[0] * 2 != g->n[0] || cg->n[1] * 2 != g->n[1] || cg->nzl * 2 != g->nzl)
    return set_error(PB_ERR_ARG, "fused restriction: coarse grid is not half the fine one");
  Sweep2Geo geo;
  sweep2_geo(g, geo);
  geo.split = 0;
  geo.xg = geo.bg_lo = geo.bg_hi = nullptr;
  if (split) {  // b three deep (planes -3 .. -1 | nzl .. nzl+2)
    PB_TRY(ensure_ghost2(g));
    PB_TRY(halo_exchange_n(g, b, b + (g->nzl - 3) * g->plane, 3, g->ghost2,
                           g->ghost2 + 3 * g->plane));
    geo.split = 1;
    geo.xg = g->ghost2;
  }
  // 8 waves x 4 rows, the plane loop unrolled by four (compile-time colours: even k0, even
  // chunk starts)
  constexpr int nw = 8, ty = 4;
  geo.ntile = (geo.ny + nw * ty - 9) / (nw * ty - 8);
  const int columns = geo.nseg * geo.ntile;
  // z-chunks: each chunk forms red, black and residual values on five planes outside it, and
  // the pass is latency-bound at two waves per SIMD, so (measured at 512^3, one box) few long
  // chunks at most one workgroup per CU win (2 chunks of 256 planes, 220 workgroups: 0.503 ms)
  // over many (10 of 52, 1100 workgroups: 0.566 ms) -- while a count just above one per CU
  // leaves some CUs two workgroups (3 chunks of 172, 330 workgroups: 0.685 vs 0.609 on another
  // box). So: at most one workgroup per CU when that keeps chunks of >= 128 planes, else ~4 per
  // CU (256^3 and smaller grids), chunks of >= 16 planes
  int nchunk = std::max(1, g->ctx->num_cus / columns);
  if (geo.nzl / nchunk < 128) nchunk = std::max(1, (4 * g->ctx->num_cus + columns - 1) / columns);
  nchunk = std::min(nchunk, std::max(1, geo.nzl / 16));
  geo.kc = (geo.nzl + nchunk - 1) / nchunk;
  geo.kc += geo.kc & 1;
  geo.nchunk = (geo.nzl + geo.kc - 1) / geo.kc;
  int64_t nblocks = (int64_t)columns * geo.nchunk;
  if (g->k0 % 2 != 0)
    return set_error(PB_ERR_UNSUPPORTED, "fused restriction: odd slab origin");
  // balanced split (one workgroup per CU where the chunks above need more than one round of
  // workgroups -- this pass runs one per CU (254 VGPRs): 512^3's 256^3 level, 528 workgroups,
  // 0.405 -> 0.382 ms for the coarse levels; on the 512^3 level itself, 220 workgroups in one
  // round, the split was slower, 0.506 -> 0.521 ms, r04/mg/split_ab.jsonl)
  const int ps = tune("mg_u4_split", -1);
  nblocks = balanced_split(g, geo, ps >= 0 ? ps : (nblocks > g->ctx->num_cus ? 1 : 0), 2,
                           nblocks);
  hipLaunchKernelGGL((presmooth_restrict_u4_kernel<nw, ty>), dim3((unsigned)nblocks),
                     dim3(64 * nw), 0, g->ctx->stream, geo, (int)cg->n[0], cg->plane, s.cx, s.cy,
                     s.cz, s.cc, omega, b, xout, bc, skip);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

int launch_presmooth_residual(pb_grid* g, const Star& s, const double* b, double* x, double* res,
                              double omega, const int* skip) {
  ScopedTimer tm(g->ctx, "mg_presmooth_residual");
  if (b == x || b == res || x == res)
    return set_error(PB_ERR_ARG, "fused pre-smoothing + residual must run out of place");
  Sweep2Geo geo;
  const int64_t nblocks = sweep2_geo(g, geo);
  PB_TRY(sweep2_ghosts(g, b, b, geo));
  auto kern = geo.split ? presmooth_resid_kernel<true> : presmooth_resid_kernel<false>;
  hipLaunchKernelGGL(kern, dim3((unsigned)nblocks), dim3(kThreads), 0, g->ctx->stream, geo,
                     s.cx, s.cy, s.cz, s.cc, omega, b, x, res, skip);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

}  // namespace pb
