// pb_compact_lines.hip -- register-resident line solves for the 3-pass compact Laplacian.
//
// Same factorisation as pb_compact_fast.hip (lapl = Lx Jy Jz + Jx Ly Jz + Jx Jy Lz, SURVEY.md
// Appendix D; reference src/compact_schemes.f90:17-37), but each 1-D line of n = 64*C points is
// owned by ONE wave with C consecutive points per lane, so both the explicit RHS and the periodic
// (alpha, 1, alpha) solve run in registers:
//
//   (alpha,1,alpha) = kappa (1 + q S^-1)(1 + q S),  q = 2 alpha / (1 + sqrt(1 - 4 alpha^2)),
//                                                   kappa = alpha / q
// so the solve is a causal first-order recursion y_i = d_i - q y_{i-1} followed by the
// anti-causal z_i = y_i - q z_{i+1}, each periodic. A lane runs its chunk with zero initial state,
// then the chunk-end values are combined across lanes by a cyclic Kogge-Stone scan with
// multiplier G = (-q)^C (truncated once G^(2^s) < 1e-24, or the exact periodic factor
// 1/(1 - G^64) when the scan covers the whole line), and each point is corrected by
// (-q)^(m+1) * carry. Nothing touches LDS except the tile transpose that gives coalesced HBM
// rows for the strided (Y, Z) passes. HBM traffic is the 80 B/DoF of the factorisation.
//
// Line sets: Z pass (lines along k, tile = TL consecutive i at fixed j), Y pass (along j, tile =
// TL consecutive i at fixed k), X pass (along i, tile = TL consecutive contiguous lines).
// The results match the reference to rounding (operation order differs from Thomas + Sherman-
// Morrison in src/tridsol.f90:34-74); the bit-exact reference-order path stays in pb_compact.hip.
#include <algorithm>
#include <cmath>

#include "pb_internal.hpp"
#include "pb_device.hpp"

#pragma clang fp contract(fast)

namespace pb {


struct LineOp {
  double a, b, sign;  // explicit 4-point RHS (src/compact_schemes.f90:332-372)
  double mq;          // -q
  double inv_kappa;
  double corr;        // 1 / (1 - G^64) if the scan wraps the whole line, else 1
  double gs[6];       // G^(2^s)
  double pw[16];      // (-q)^(m+1)
  int nsteps;
};

struct LinePass {
  const double* in0;
  const double* in1;
  double* out0;
  double* out1;
  int64_t li, lo, es;  // address of (outer, inner line, element e) = outer*lo + inner*li + e*es
  int ninner, ntiles_inner, nouter, TL, P;
  int ablate;  // tuning only (PB_LINES_ABLATE=1): copy lines through, no solves (the build flag
               // -DPB_LINES_ABLATE_TRAFFIC=1 drops the tiled passes' global loads / stores instead)
  int remap;   // XCD-aware tile order: off (Z pass 0.74-0.78 vs 0.715-0.72 ms with it at 512^3,
               // profiles/r02/ab_remap_compact.jsonl)
  LineOp J, L;
  const int* skip;  // pb_ctx::op_skip (exit at entry once set)
  // CG fusions (CgFuse): Z pass forming p from in0 = z and in1 = p_old (CGP kernels), X pass
  // taking p . w partial sums (DOT kernels)
  double* p_out;
  const CgState* st;
  int first;
  const double* dot_p;
  double* parts;
  // blocked inputs (lo_in > 0): the decomposed Y pass reads the all-to-all receive buffers --
  // outer stride lo_in, element e at (e >> esh_in) * ebs_in + (e & (2^esh_in - 1)) * es
  int64_t lo_in, ebs_in;
  int esh_in;
  // the self block of a blocked input (YSlabPlan::self_direct): block alt_blk of in0 / in1 is read
  // from alt0 / alt1 (the Z pass's y-slab outputs; the all-to-all did not copy it); -1: none
  const double* alt0 = nullptr;
  const double* alt1 = nullptr;
  int alt_blk = -1;
};

static LineOp make_line_op(int kind, int C, double h) {
  LineOp o{};
  double alpha;
  if (kind == 0) {  // J: interp (:303-305)
    o.a = 0.75;
    o.b = 1.0 / 20.0;
    o.sign = 1.0;
    alpha = 3.0 / 10.0;
  } else {  // L: grad / div (:188-190)
    o.a = 63.0 / 62.0 / h;
    o.b = 17.0 / 62.0 / (3.0 * h);
    o.sign = -1.0;
    alpha = 9.0 / 62.0;
  }
  const double q = 2.0 * alpha / (1.0 + std::sqrt(1.0 - 4.0 * alpha * alpha));
  o.mq = -q;
  o.inv_kappa = q / alpha;
  double p = 1.0;
  for (int m = 0; m < C; ++m) {
    p *= -q;
    o.pw[m] = p;
  }
  const double G = p;  // (-q)^C
  double g = G;
  int s = 0;
  for (; s < 6; ++s) {
    if (std::fabs(g) < 1e-24) break;
    o.gs[s] = g;
    g = g * g;
  }
  o.nsteps = s;
  o.corr = s == 6 ? 1.0 / (1.0 - g) : 1.0;  // g = G^64 here
  return o;
}

__device__ __forceinline__ double lane_shfl(double v, int src) { return __shfl(v, src & 63, 64); }
// the wave rotations by one lane as DPP moves (VALU, no LDS round trip like __shfl's
// ds_bpermute): lane l <- lane l-1 (lane 0 <- 63: wave_ror:1) / lane l+1 (lane 63 <- 0: wave_rol:1).
// The same values as lane_shfl(v, lane -/+ 1), so the results do not change.
template <int CTRL>
__device__ __forceinline__ double lane_rot(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double lane_from_lower(double v) { return lane_rot<0x13C>(v); }
__device__ __forceinline__ double lane_from_upper(double v) { return lane_rot<0x134>(v); }

// d <- explicit RHS of x (stagger -1: cell -> vertex, +1: vertex -> cell), eval_1d_rhs order
template <int C>
__device__ __forceinline__ void line_rhs(const double (&x)[C], double (&d)[C], const LineOp& o,
                                         int stagger, int lane) {
  double xm2, xm1, xp0, xp1;  // x at local offsets -2, -1, C, C+1
  (void)lane;
  xm1 = lane_from_lower(x[C - 1]);
  xp0 = lane_from_upper(x[0]);
  if constexpr (C >= 2) {
    if (stagger < 0) {
      xm2 = lane_from_lower(x[C - 2]);
      xp1 = 0.0;
    } else {
      xp1 = lane_from_upper(x[1]);
      xm2 = 0.0;
    }
  } else {
    if (stagger < 0) {
      xm2 = lane_from_lower(xm1);
      xp1 = 0.0;
    } else {
      xp1 = lane_from_upper(xp0);
      xm2 = 0.0;
    }
  }
  auto at = [&](int o2) -> double {  // o2 is a compile-time constant after unrolling
    if (o2 == -2) return xm2;
    if (o2 == -1) return xm1;
    if (o2 == C) return xp0;
    if (o2 == C + 1) return xp1;
    return x[o2];
  };
  const double a = o.a, b = o.b, s = o.sign;
#pragma unroll
  for (int m = 0; m < C; ++m) {
    if (stagger < 0)
      d[m] = a * (at(m) + s * at(m - 1)) + b * (at(m + 1) + s * at(m - 2));
    else
      d[m] = a * (at(m + 1) + s * at(m)) + b * (at(m + 2) + s * at(m - 1));
  }
}

// d <- (alpha, 1, alpha)^-1 d on the periodic line (64 lanes x C points)
template <int C>
__device__ __forceinline__ void line_solve(double (&d)[C], const LineOp& o, int lane) {
  const double mq = o.mq;
  // causal sweep y_i = d_i - q y_{i-1}
#pragma unroll
  for (int m = 1; m < C; ++m) d[m] = d[m] + mq * d[m - 1];
  double T = d[C - 1];
  // the scan's distance-1 step and the carries as DPP rotations (chains of them for distances 2
  // and 4 measured no faster than ds_bpermute, profiles/r03/compact_dpp_*.jsonl)
  if (o.nsteps > 0) T = T + o.gs[0] * lane_from_lower(T);
  for (int s = 1; s < o.nsteps; ++s) T = T + o.gs[s] * lane_shfl(T, lane - (1 << s));
  T *= o.corr;
  double cin = lane_from_lower(T);
#pragma unroll
  for (int m = 0; m < C; ++m) d[m] = d[m] + o.pw[m] * cin;
  // anti-causal sweep z_i = y_i - q z_{i+1}
#pragma unroll
  for (int m = C - 2; m >= 0; --m) d[m] = d[m] + mq * d[m + 1];
  T = d[0];
  if (o.nsteps > 0) T = T + o.gs[0] * lane_from_upper(T);
  for (int s = 1; s < o.nsteps; ++s) T = T + o.gs[s] * lane_shfl(T, lane + (1 << s));
  T *= o.corr;
  cin = lane_from_upper(T);
#pragma unroll
  for (int m = 0; m < C; ++m) d[m] = (d[m] + o.pw[C - 1 - m] * cin) * o.inv_kappa;
}

// r <- (I+ I-) x  (J or L: cell -> vertex half, then vertex -> cell half)
template <int C>
__device__ __forceinline__ void line_op(const double (&x)[C], double (&r)[C], const LineOp& o,
                                        int lane, int ablate) {
  if (ablate) {
#pragma unroll
    for (int m = 0; m < C; ++m) r[m] = x[m];
    return;
  }
  double t[C];
  line_rhs<C>(x, t, o, -1, lane);
  line_solve<C>(t, o, lane);
  line_rhs<C>(t, r, o, +1, lane);
  line_solve<C>(r, o, lane);
}

// LDS word of (line l, element e): lanes own C consecutive points; chunk pitch odd -> no conflicts
template <int C>
struct Lds {
  static constexpr int CP = (C % 2 == 0) ? C + 1 : C;
  // line pitch (doubles): 64 CP + 1 = 1 mod 16, so the tile copies' 16-lane groups (8 lines x 2
  // elements) hit 16 distinct banks; the r01/r02 pitch 64 CP + 4 put lines 0, 4, 8, 12 on one bank
  // (4-way conflicts on every tile write: 4x the LDS write cycles of the copy, by a bank model)
  static constexpr int LP = 64 * CP + 1;
  __device__ static __forceinline__ int word(int l, int e) { return l * LP + (e / C) * CP + (e % C); }
};

// global <-> LDS tile copies, fully unrolled so every load of the tile is in flight at once.
// LAYOUT 0: lines run across rows (li == 1, coalesced along l); LAYOUT 1: lines contiguous
// (es == 1, li == n). V = 2 moves 16-byte pairs along the contiguous direction (needs an even
// row length); the pair (l, l+1) of LAYOUT 0 sits in two different LDS lines.
typedef double dv2 __attribute__((ext_vector_type(2)));

template <int C, int LAYOUT, int TL, int V>
__device__ __forceinline__ void tile_coord(int f, int& l, int& e) {
  constexpr int n = 64 * C;
  if (LAYOUT == 0) {
    l = (f % (TL / V)) * V;
    e = f / (TL / V);
  } else {
    l = (f * V) / n;
    e = (f * V) % n;
  }
}

template <int C, int LAYOUT, int TL, int V, int NT>
struct TileRegs {
  static constexpr int NF = TL * 64 * C / V;  // pairs (or singles) in the tile
  static constexpr int R = (NF + NT - 1) / NT;
  double v[R][V];
};

// issue every global load of the tile (no wait: the registers are consumed by tile_put later).
// Every load is unconditional, from a valid address (pairs past the tile re-load line 0 / the
// tile's first element; tile_put ignores them): a load under a runtime `if` made the compiler
// wait for each load before issuing the next (s_waitcnt vmcnt(0) ahead of every
// global_load_dwordx4 in the r02 ISA of the persistent Z / Y passes), i.e. one HBM round trip per
// pair instead of the whole tile in flight.
#ifndef PB_LINES_ABLATE_TRAFFIC
#define PB_LINES_ABLATE_TRAFFIC 0  // timing builds only: no global loads / stores in tiled passes
#endif
// BLK: the input is an all-to-all receive buffer in its blocked layout (LinePass::lo_in, esh_in,
// ebs_in; the decomposed Y pass, PASS 4); base is the output layout's
template <bool BLK = false, int C, int LAYOUT, int TL, int V, int NT>
__device__ __forceinline__ void tile_fetch(const LinePass& p, const double* __restrict__ src,
                                           int64_t base, int nl, TileRegs<C, LAYOUT, TL, V, NT>& t) {
  using T = TileRegs<C, LAYOUT, TL, V, NT>;
  if (PB_LINES_ABLATE_TRAFFIC) return;
  int64_t b_in = base;
  if constexpr (BLK) {
    const int64_t outer = base / p.lo;
    b_in = outer * p.lo_in + (base - outer * p.lo);
  }
#pragma unroll
  for (int r = 0; r < T::R; ++r) {
    int l, e;
    const int f = threadIdx.x + NT * r;
    tile_coord<C, LAYOUT, TL, V>(f, l, e);
    const bool ok = (T::NF % NT == 0 || f < T::NF) && l < nl;
    const int lc = ok ? l : 0, ec = ok ? e : 0;  // selects, not a branch around the load
    int64_t eo = (int64_t)ec * p.es;
    const double* s = src;
    if constexpr (BLK) {
      eo = (int64_t)(ec >> p.esh_in) * p.ebs_in + (int64_t)(ec & ((1 << p.esh_in) - 1)) * p.es;
      if ((ec >> p.esh_in) == p.alt_blk) s = src == p.in0 ? p.alt0 : p.alt1;  // (a select)
    }
    const double* a = s + b_in + lc * p.li + eo;
    if (V == 2) {
      const dv2 w = __builtin_nontemporal_load((const dv2*)a);
      t.v[r][0] = w.x;
      t.v[r][V - 1] = w.y;
    } else {
      t.v[r][0] = __builtin_nontemporal_load(a);
    }
  }
}

template <int C, int LAYOUT, int TL, int V, int NT>
__device__ __forceinline__ void tile_put(double* lds, int nl, const TileRegs<C, LAYOUT, TL, V, NT>& t) {
  using T = TileRegs<C, LAYOUT, TL, V, NT>;
  constexpr int dl = LAYOUT == 0 ? 1 : 0, de = LAYOUT == 0 ? 0 : 1;  // step of the pair partner
#pragma unroll
  for (int r = 0; r < T::R; ++r) {
    int l, e;
    const int f = threadIdx.x + NT * r;
    tile_coord<C, LAYOUT, TL, V>(f, l, e);
    if ((T::NF % NT == 0 || f < T::NF) && l < nl) {
      lds[Lds<C>::word(l, e)] = t.v[r][0];
      if (V == 2) lds[Lds<C>::word(l + dl, e + de)] = t.v[r][V - 1];
    }
  }
}

template <int C, int LAYOUT, int TL, int V, int NT>
__device__ __forceinline__ void tile_store(const LinePass& p, double* __restrict__ dst,
                                           const double* lds, int64_t base, int nl) {
  constexpr int NF = TL * 64 * C / V;
  constexpr int R = (NF + NT - 1) / NT;
  constexpr int dl = LAYOUT == 0 ? 1 : 0, de = LAYOUT == 0 ? 0 : 1;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    int l, e;
    const int f = threadIdx.x + NT * r;
    tile_coord<C, LAYOUT, TL, V>(f, l, e);
    if ((NF % NT == 0 || f < NF) && l < nl) {
      double* a = dst + base + l * p.li + e * p.es;
      if (V == 2) {
        dv2 w;
        w.x = lds[Lds<C>::word(l, e)];
        w.y = lds[Lds<C>::word(l + dl, e + de)];
        if (PB_LINES_ABLATE_TRAFFIC) {
          if (w.x == 12345.678) *a = w.y;  // keeps the LDS reads (never true on real data)
          continue;
        }
        __builtin_nontemporal_store(w, (dv2*)a);
      } else {
        __builtin_nontemporal_store(lds[Lds<C>::word(l, e)], a);
      }
    }
  }
}

// CGP: p = (dinv z - mu) + (beta / beta_old) p_old on the tile's pairs (z in `pre`, p_old in
// `pold`), written back into `pre` and stored to p_out at the pairs' own addresses. The products
// and sums round separately, as cg_gen_p_kernel's (built without contraction): bit-identical.
template <int C, int LAYOUT, int TL, int V, int NT>
__device__ __forceinline__ void cg_form_p(const LinePass& p, int64_t base, int nl,
                                          TileRegs<C, LAYOUT, TL, V, NT>& pre,
                                          const TileRegs<C, LAYOUT, TL, V, NT>& pold) {
  using T = TileRegs<C, LAYOUT, TL, V, NT>;
  const CgState* st = p.st;
  const double dinv = st->dinv, shift = -st->mu;
  const double bb = st->it == 0 ? 0.0 : st->beta / st->betaold;
#pragma unroll
  for (int r = 0; r < T::R; ++r) {
    int l, e;
    const int f = threadIdx.x + NT * r;
    tile_coord<C, LAYOUT, TL, V>(f, l, e);
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const double z = __dadd_rn(__dmul_rn(dinv, pre.v[r][q]), shift);
      pre.v[r][q] = p.first ? z : __dadd_rn(z, __dmul_rn(bb, pold.v[r][q]));
    }
    if ((T::NF % NT == 0 || f < T::NF) && l < nl && !PB_LINES_ABLATE_TRAFFIC) {
      dv2 w;
      w.x = pre.v[r][0];
      w.y = pre.v[r][V - 1];
      __builtin_nontemporal_store(w, (dv2*)(p.p_out + base + l * p.li + e * p.es));
    }
  }
}

template <int C>
__device__ __forceinline__ void chunk_read(const double* lds, int l, int lane, double (&x)[C]) {
  const int w0 = l * Lds<C>::LP + lane * Lds<C>::CP;
#pragma unroll
  for (int m = 0; m < C; ++m) x[m] = lds[w0 + m];
}
template <int C>
__device__ __forceinline__ void chunk_write(double* lds, int l, int lane, const double (&x)[C]) {
  const int w0 = l * Lds<C>::LP + lane * Lds<C>::CP;
#pragma unroll
  for (int m = 0; m < C; ++m) lds[w0 + m] = x[m];
}

// PASS 0 (Z): out0 = J in0, out1 = L in0.   PASS 1 (Y): out0 = J in0, out1 = L in0 + J in1.
// PASS 2 (X): out0 = L in0 + J in1.
// K = launch shape: TL lines per tile, NW waves per block (NW divides TL), PF = 1 for persistent
// blocks that fetch the next input tile into registers while the current one is solved and
// stored (HBM reads overlap the line solves and the write-back), PF = 0 for one tile per block.
template <int TL_, int NW_, int PF_>
struct LineCfg {
  static constexpr int TL = TL_, NW = NW_, PF = PF_, NT = 64 * NW_, LPW = TL_ / NW_;
};

// CGP (PASS 0, V = 2): in0 = z, in1 = p_old; the tile's input is p = (dinv z - mu) + beta/
// beta_old p_old (cg_gen_p_kernel's operations, unfused roundings: bit-identical), also stored to
// p_out as it goes into LDS
// PASS_ 4: PASS 1 with its inputs read from the all-to-all receive buffers (tile_fetch BLK)
template <int C, int LAYOUT, int PASS_, class K, int V, bool CGP = false>
__global__ __launch_bounds__(K::NT) void compact_lines_kernel(LinePass p) {
  constexpr bool BLK = PASS_ == 4;
  constexpr int PASS = BLK ? 1 : PASS_;
  static_assert(!CGP || (PASS == 0 && V == 2 && K::PF == 1), "CGP: Z pass, pairs, prefetch");
  if (p.skip && *p.skip) return;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int TL = K::TL, LPW = K::LPW, NT = K::NT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ntiles = p.ntiles_inner * p.nouter;
  auto tile_of = [&](int t, int64_t& base, int& nl) {
    const int outer = t / p.ntiles_inner;
    const int inner0 = (t % p.ntiles_inner) * TL;
    nl = min(TL, p.ninner - inner0);
    base = (int64_t)outer * p.lo + (int64_t)inner0 * p.li;
  };
  int t = xcd_block(p.remap);
  if (t >= ntiles) return;
  double keep[LPW][C];
  TileRegs<C, LAYOUT, TL, V, NT> pold;  // CGP: p_old of the prefetched tile (dead otherwise)
  // one tile: its input registers `pre` go to LDS, then (PF) tile tn's input is fetched into them
  // while this tile is solved and stored
  auto step = [&](int t, TileRegs<C, LAYOUT, TL, V, NT>& pre, int tn) {
    int64_t base, base_n = 0;
    int nl, nl_n = 0;
    tile_of(t, base, nl);
    if (K::PF && tn < ntiles) tile_of(tn, base_n, nl_n);
    __syncthreads();  // previous tile's LDS reads are done
    if (!K::PF) tile_fetch<BLK>(p, p.in0, base, nl, pre);
    if constexpr (CGP) cg_form_p<C, LAYOUT, TL, V, NT>(p, base, nl, pre, pold);
    tile_put(lds, nl, pre);
    __syncthreads();
    if (K::PF) {
      if (PASS == 0 || PASS == 3) {
        if (tn < ntiles) {
          tile_fetch<BLK>(p, p.in0, base_n, nl_n, pre);
          // (the first iteration of a lazy-start solve has no p_old: p = z - mu, 8 B/DoF fewer)
          if constexpr (CGP)
            if (!p.first) tile_fetch<BLK>(p, p.in1, base_n, nl_n, pold);
        }
      } else {
        tile_fetch<BLK>(p, p.in1, base, nl, pre);
      }
    }
#pragma unroll
    for (int j = 0; j < LPW; ++j) {
      const int l = wave * LPW + j;
      if (l >= nl) continue;
      double x[C], r[C];
      chunk_read<C>(lds, l, lane, x);
      if (PASS == 3) {  // batched (alpha, 1, alpha) periodic solve
#pragma unroll
        for (int m = 0; m < C; ++m) r[m] = x[m];
        line_solve<C>(r, p.J, lane);
        chunk_write<C>(lds, l, lane, r);
        continue;  // (per line)
      }
      if (PASS != 2) {
        line_op<C>(x, r, p.J, lane, p.ablate);
        chunk_write<C>(lds, l, lane, r);
      }
      line_op<C>(x, keep[j], p.L, lane, p.ablate);
    }
    __syncthreads();
    if (PASS == 3) {
      tile_store<C, LAYOUT, TL, V, NT>(p, p.out0, lds, base, nl);
      return;
    }
    if (PASS == 0) {
      tile_store<C, LAYOUT, TL, V, NT>(p, p.out0, lds, base, nl);
      __syncthreads();
#pragma unroll
      for (int j = 0; j < LPW; ++j) {
        const int l = wave * LPW + j;
        if (l < nl) chunk_write<C>(lds, l, lane, keep[j]);
      }
      __syncthreads();
      tile_store<C, LAYOUT, TL, V, NT>(p, p.out1, lds, base, nl);
      return;
    }
    if (PASS == 1) {
      tile_store<C, LAYOUT, TL, V, NT>(p, p.out0, lds, base, nl);
      __syncthreads();
    }
    if (!K::PF) tile_fetch<BLK>(p, p.in1, base, nl, pre);
    tile_put(lds, nl, pre);
    __syncthreads();
    if (K::PF && tn < ntiles) tile_fetch<BLK>(p, p.in0, base_n, nl_n, pre);
#pragma unroll
    for (int j = 0; j < LPW; ++j) {
      const int l = wave * LPW + j;
      if (l >= nl) continue;
      double x[C], r[C];
      chunk_read<C>(lds, l, lane, x);
      line_op<C>(x, r, p.J, lane, p.ablate);
#pragma unroll
      for (int m = 0; m < C; ++m) r[m] = keep[j][m] + r[m];
      chunk_write<C>(lds, l, lane, r);
    }
    __syncthreads();
    tile_store<C, LAYOUT, TL, V, NT>(p, PASS == 1 ? p.out1 : p.out0, lds, base, nl);
  };
  if constexpr (K::PF == 2) {  // two tiles' inputs in flight (single-input passes)
    static_assert(PASS == 0 || PASS == 3, "PF = 2: single-input passes only");
    const int G = gridDim.x;
    TileRegs<C, LAYOUT, TL, V, NT> ra, rb;
    int64_t b0;
    int n0;
    tile_of(t, b0, n0);
    tile_fetch<BLK>(p, p.in0, b0, n0, ra);
    if (t + G < ntiles) {
      tile_of(t + G, b0, n0);
      tile_fetch<BLK>(p, p.in0, b0, n0, rb);
    }
    for (; t < ntiles; t += 2 * G) {
      step(t, ra, t + 2 * G);
      if (t + G >= ntiles) break;
      step(t + G, rb, t + 3 * G);
    }
  } else {
    TileRegs<C, LAYOUT, TL, V, NT> pre;
    if (K::PF) {
      int64_t b0;
      int n0;
      tile_of(t, b0, n0);
      tile_fetch<BLK>(p, p.in0, b0, n0, pre);
      if constexpr (CGP)
        if (!p.first) tile_fetch(p, p.in1, b0, n0, pold);
    }
    for (; t < ntiles; t += gridDim.x) step(t, pre, t + gridDim.x);
  }
}

// X pass without block barriers: the lines are contiguous, so each wave owns whole lines and
// re-distributes them through a wave-private LDS strip (coalesced 16-byte loads -> C consecutive
// points per lane -> coalesced stores). One wave per line: out = L in0 + J in1.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int C, bool DOT>
__device__ __forceinline__ void x_direct_line(const LinePass& p, int64_t line, double* sl,
                                              int lane, double& acc) {
  constexpr int LP = Lds<C>::LP, CP = Lds<C>::CP;
  const int64_t off = line * (64 * C);
  constexpr int NP = 32 * C;  // 16-byte pieces per line
  constexpr int R = (NP + 63) / 64;
  dv2 a[R], b[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int q = lane + 64 * r;
    if (NP % 64 == 0 || q < NP) {
      a[r] = __builtin_nontemporal_load((const dv2*)(p.in0 + off) + q);
      b[r] = __builtin_nontemporal_load((const dv2*)(p.in1 + off) + q);
    }
  }
  auto w = [&](int e) { return (e / C) * CP + (e % C); };
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int q = lane + 64 * r;
    if (NP % 64 == 0 || q < NP) {
      sl[w(2 * q)] = a[r].x;
      sl[w(2 * q + 1)] = a[r].y;
      sl[LP + w(2 * q)] = b[r].x;
      sl[LP + w(2 * q + 1)] = b[r].y;
    }
  }
  wave_sync();
  double x[C], y[C], r1[C], r2[C];
#pragma unroll
  for (int m = 0; m < C; ++m) {
    x[m] = sl[lane * CP + m];
    y[m] = sl[LP + lane * CP + m];
  }
  line_op<C>(x, r1, p.L, lane, p.ablate);
  line_op<C>(y, r2, p.J, lane, p.ablate);
  wave_sync();
#pragma unroll
  for (int m = 0; m < C; ++m) sl[lane * CP + m] = r1[m] + r2[m];
  wave_sync();
  dv2 pp[R];
  if constexpr (DOT) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int q = lane + 64 * r;
      pp[r] = __builtin_nontemporal_load((const dv2*)(p.dot_p + off) + (NP % 64 == 0 || q < NP ? q : 0));
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int q = lane + 64 * r;
    if (NP % 64 == 0 || q < NP) {
      dv2 o;
      o.x = sl[w(2 * q)];
      o.y = sl[w(2 * q + 1)];
      __builtin_nontemporal_store(o, (dv2*)(p.out0 + off) + q);
      if constexpr (DOT) {
        acc += o.x * pp[r].x;
        acc += o.y * pp[r].y;
      }
    }
  }
  wave_sync();  // the strip is reused by the wave's next line
}

// DOT: CG's p . w partial sums as w is written (p = p.dot_p): the waves walk lines
// grid-stride (line = 4 block + wave + 4 grid k), each lane sums its w p products in order, then a
// fixed-order block reduction (lane butterflies, waves in order) -> p.parts[block]
template <int C, bool DOT = false>
__global__ __launch_bounds__(256) void compact_lines_x_direct(LinePass p, int64_t nlines) {
  if (p.skip && *p.skip) return;
  constexpr int LP = Lds<C>::LP;
  __shared__ double strip[4][2 * LP];
  __shared__ double red[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double acc = 0.0;
  for (int64_t line = (int64_t)blockIdx.x * 4 + wave; line < nlines;
       line += DOT ? (int64_t)gridDim.x * 4 : nlines) {
    x_direct_line<C, DOT>(p, line, strip[wave], lane, acc);
  }
  if constexpr (DOT) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) red[wave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) p.parts[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
  }
}


template <int C>
static int launch_x_direct(pb_ctx* ctx, LinePass& p, int64_t nlines) {
  CgFuse* cf = ctx->cg_fuse;
  if (cf && cf->dot_p) {  // p . w partial sums: a fixed grid of at most 16 blocks per CU
    // (x_dot_cu, A/B: blocks per CU of that grid; 0: one line per wave like the plain X pass)
    const int per_cu = tune("x_dot_cu", 16);
    const int64_t nb = per_cu > 0 ? std::min<int64_t>((nlines + 3) / 4, (int64_t)ctx->num_cus * per_cu)
                                   : (nlines + 3) / 4;
    if (nb > ctx->partials_cap) return set_error(PB_ERR_UNSUPPORTED, "x pass: partials");
    p.dot_p = cf->dot_p;
    p.parts = ctx->d_partials;
    hipLaunchKernelGGL((compact_lines_x_direct<C, true>), dim3((unsigned)nb), dim3(256), 0,
                       ctx->stream, p, nlines);
    PB_HIP(hipGetLastError());
    cf->nparts = (int)nb;
    cf->fused_dot = true;
    return PB_OK;
  }
  hipLaunchKernelGGL(compact_lines_x_direct<C>, dim3((unsigned)((nlines + 3) / 4)), dim3(256), 0,
                     ctx->stream, p, nlines);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

// batched solve on contiguous lines (element stride 1, line stride li): one wave per line,
// redistributed through a wave-private LDS strip like the X pass
template <int C>
__global__ __launch_bounds__(256) void lines_solve_direct(LinePass p, int64_t nlines) {
  if (p.skip && *p.skip) return;
  constexpr int LP = Lds<C>::LP, CP = Lds<C>::CP;
  __shared__ double strip[4][LP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t line = (int64_t)blockIdx.x * 4 + wave;
  if (line >= nlines) return;
  double* sl = strip[wave];
  const int64_t off = line * p.li;
  constexpr int NP = 32 * C;
  constexpr int R = (NP + 63) / 64;
  dv2 a[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int q = lane + 64 * r;
    if (NP % 64 == 0 || q < NP) a[r] = __builtin_nontemporal_load((const dv2*)(p.in0 + off) + q);
  }
  auto w = [&](int e) { return (e / C) * CP + (e % C); };
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int q = lane + 64 * r;
    if (NP % 64 == 0 || q < NP) {
      sl[w(2 * q)] = a[r].x;
      sl[w(2 * q + 1)] = a[r].y;
    }
  }
  wave_sync();
  double x[C];
#pragma unroll
  for (int m = 0; m < C; ++m) x[m] = sl[lane * CP + m];
  line_solve<C>(x, p.J, lane);
  wave_sync();
#pragma unroll
  for (int m = 0; m < C; ++m) sl[lane * CP + m] = x[m];
  wave_sync();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int q = lane + 64 * r;
    if (NP % 64 == 0 || q < NP) {
      dv2 o;
      o.x = sl[w(2 * q)];
      o.y = sl[w(2 * q + 1)];
      __builtin_nontemporal_store(o, (dv2*)(p.out0 + off) + q);
    }
  }
}

template <int C>
static int launch_solve_direct(pb_ctx* ctx, LinePass& p, int64_t nlines) {
  hipLaunchKernelGGL(lines_solve_direct<C>, dim3((unsigned)((nlines + 3) / 4)), dim3(256), 0,
                     ctx->stream, p, nlines);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

static LineOp make_solve_op(double alpha, int C) {
  LineOp o{};
  const double q = 2.0 * alpha / (1.0 + std::sqrt(1.0 - 4.0 * alpha * alpha));
  o.mq = -q;
  o.inv_kappa = q / alpha;
  double pw = 1.0;
  for (int m = 0; m < C; ++m) {
    pw *= -q;
    o.pw[m] = pw;
  }
  double g = pw;
  int s = 0;
  for (; s < 6; ++s) {
    if (std::fabs(g) < 1e-24) break;
    o.gs[s] = g;
    g = g * g;
  }
  o.nsteps = s;
  o.corr = s == 6 ? 1.0 / (1.0 - g) : 1.0;
  return o;
}

// the CgFuse passes apply: one rank (no z-slab <-> y-slab transposes), register line solves in
// every direction, the Z pass with prefetch (lines of <= 512 points) on an even x extent, default
// launch shapes
// (the same conditions the Z and X passes test below and in compact_pass_*: the solver falls back
// to the unfused iteration when a pass reports it did not fuse)
bool compact_cg_fusable(const pb_grid* g) {
  return !grid_split(g) && !g->ctx->split && tune("compact_lines", 1) &&
         compact_lines_supported(g->n[0]) && compact_lines_supported(g->n[1]) &&
         compact_lines_supported(g->n[2]) && g->n[2] <= 512 && g->n[0] % 2 == 0 &&
         tune("cg_fuse", 1);
}

// split grids (z-slab <-> y-slab transposes, r06): p is formed by the pack of the transpose
// (pb_compact_dist.hip, even nx) and p . w taken by the X pass (register line solves in x);
// a pass that does not fuse is reported and the solver runs the separate kernels for it
bool compact_cg_fusable_split(const pb_grid* g) {
  return g->ctx->split && tune("compact_lines", 1) && compact_lines_supported(g->n[0]) &&
         g->n[0] % 2 == 0 && tune("cg_fuse", 1);
}

bool compact_lines_supported(int64_t n) {
  if (n % 64) return false;
  const int64_t C = n / 64;
  return C == 1 || C == 2 || C == 3 || C == 4 || C == 6 || C == 8 || C == 12 || C == 16;
}

template <int C, int LAYOUT, int PASS, class K, int V, bool CGP = false>
static int launch_lines_v(pb_ctx* ctx, LinePass& p, int64_t nouter) {
  p.TL = K::TL;
  p.P = Lds<C>::LP;
  p.ntiles_inner = (p.ninner + K::TL - 1) / K::TL;
  p.nouter = (int)nouter;
  const int64_t ntiles = (int64_t)p.ntiles_inner * nouter;
  const size_t lds = (size_t)K::TL * Lds<C>::LP * sizeof(double);
  auto kern = compact_lines_kernel<C, LAYOUT, PASS, K, V, CGP>;
  static int occ = 0;
  if (!occ) {
    PB_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds));
    PB_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, K::NT, lds));
    if (occ < 1) occ = 1;
  }
  int64_t nblocks = K::PF ? (int64_t)occ * ctx->num_cus : ntiles;
  if (nblocks > ntiles) nblocks = ntiles;
  hipLaunchKernelGGL(kern, dim3((unsigned)nblocks), dim3(K::NT), lds, ctx->stream, p);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

// 16-byte pairs when the contiguous direction has even length (always for LAYOUT 1, n = 64*C)
template <int C, int LAYOUT, int PASS, class K>
static int launch_lines_k(pb_ctx* ctx, LinePass& p, int64_t nouter) {
  if (LAYOUT == 1 || (p.ninner % 2 == 0 && p.li == 1 && p.lo % 2 == 0 && p.es % 2 == 0 &&
                      ((uintptr_t)p.in0 & 15) == 0 && ((uintptr_t)p.out0 & 15) == 0))
    return launch_lines_v<C, LAYOUT, PASS, K, 2>(ctx, p, nouter);
  return launch_lines_v<C, LAYOUT, PASS, K, 1>(ctx, p, nouter);
}

// Launch shapes (measured at 512^3, profiles/r01/tune_compact*.jsonl): strided passes use 16-line
// tiles (128-B row segments, two blocks per CU), the contiguous X pass 8-line tiles; the batched
// interleaved solve (PASS 3: little compute per tile to hide the next tile's loads under) 32-line
// tiles with two tiles' inputs in flight. C > 8 keeps 8-line tiles for LDS.
template <int C, int LAYOUT, int PASS>
static int launch_lines_c(pb_ctx* ctx, LinePass& p, int64_t nouter) {
  if constexpr (LAYOUT == 0 && C <= 8 && PASS == 3)  // batched solve: 0.62 -> 0.48 ms at 512
    return launch_lines_k<C, LAYOUT, PASS, LineCfg<32, 16, 2>>(ctx, p, nouter);
  else if constexpr (LAYOUT == 0 && C <= 8)
    return launch_lines_k<C, LAYOUT, PASS, LineCfg<16, 16, 1>>(ctx, p, nouter);
  else
    return launch_lines_k<C, LAYOUT, PASS, LineCfg<8, 8, 0>>(ctx, p, nouter);
}

template <int LAYOUT, int PASS>
static int launch_lines(pb_ctx* ctx, LinePass& p, int64_t n, int64_t nouter) {
  switch (n / 64) {
    case 1: return launch_lines_c<1, LAYOUT, PASS>(ctx, p, nouter);
    case 2: return launch_lines_c<2, LAYOUT, PASS>(ctx, p, nouter);
    case 3: return launch_lines_c<3, LAYOUT, PASS>(ctx, p, nouter);
    case 4: return launch_lines_c<4, LAYOUT, PASS>(ctx, p, nouter);
    case 6: return launch_lines_c<6, LAYOUT, PASS>(ctx, p, nouter);
    case 8: return launch_lines_c<8, LAYOUT, PASS>(ctx, p, nouter);
    case 12: return launch_lines_c<12, LAYOUT, PASS>(ctx, p, nouter);
    case 16: return launch_lines_c<16, LAYOUT, PASS>(ctx, p, nouter);
  }
  return set_error(PB_ERR_UNSUPPORTED, "compact line solver: n = %lld", (long long)n);
}

// One pass of the factorised Laplacian with register line solves. axis: 2 = Z, 1 = Y, 0 = X.
int compact_lines_pass(pb_ctx* ctx, const int64_t dims[3], int axis, double h, const double* in0,
                       const double* in1, double* out0, double* out1, const YSlabPlan* blk_in) {
  const int64_t nx = dims[0], ny = dims[1], nz = dims[2];
  const int64_t n = axis == 2 ? nz : (axis == 1 ? ny : nx);
  const int C = (int)(n / 64);
  static const char* names[3] = {"compact_lines_x", "compact_lines_y", "compact_lines_z"};
  ScopedTimer tm(ctx, names[axis]);
  LinePass p{};
  p.skip = ctx->op_skip;
  p.remap = 0;
  const int ablate = PB_ABLATE_LINES;
  p.ablate = ablate;
  p.in0 = in0;
  p.in1 = in1;
  p.out0 = out0;
  p.out1 = out1;
  p.J = make_line_op(0, C, h);
  p.L = make_line_op(1, C, h);
  if (axis == 2) {
    p.li = 1;
    p.lo = nx;
    p.es = nx * ny;
    p.ninner = (int)nx;
    CgFuse* cf = ctx->cg_fuse;
    if (cf && cf->z && C <= 8 && nx % 2 == 0 && ((uintptr_t)cf->z & 15) == 0 &&
        ((uintptr_t)out0 & 15) == 0) {
      // CG's p formed by the Z pass from z and p_old (CgFuse); in0 is not read
      p.in0 = cf->z;
      p.in1 = cf->p_old;
      p.p_out = cf->p_out;
      p.st = cf->st;
      p.first = cf->first;
      int rc = PB_ERR_UNSUPPORTED;
      switch (C) {
        case 1: rc = launch_lines_v<1, 0, 0, LineCfg<16, 16, 1>, 2, true>(ctx, p, ny); break;
        case 2: rc = launch_lines_v<2, 0, 0, LineCfg<16, 16, 1>, 2, true>(ctx, p, ny); break;
        case 3: rc = launch_lines_v<3, 0, 0, LineCfg<16, 16, 1>, 2, true>(ctx, p, ny); break;
        case 4: rc = launch_lines_v<4, 0, 0, LineCfg<16, 16, 1>, 2, true>(ctx, p, ny); break;
        case 6: rc = launch_lines_v<6, 0, 0, LineCfg<16, 16, 1>, 2, true>(ctx, p, ny); break;
        case 8: rc = launch_lines_v<8, 0, 0, LineCfg<16, 16, 1>, 2, true>(ctx, p, ny); break;
      }
      if (rc == PB_OK) cf->fused_z = true;
      return rc;
    }
    return launch_lines<0, 0>(ctx, p, n, ny);
  }
  if (axis == 1) {
    p.li = 1;
    p.lo = nx * ny;
    p.es = nx;
    p.ninner = (int)nx;
    if (blk_in) {  // row (kl, j) at block j >> k, row kl * nyl + (j & (nyl - 1))
      const int64_t nyl = blk_in->nyl[0];
      int sh = 0;
      while (((int64_t)1 << sh) < nyl) ++sh;
      p.lo_in = nyl * nx;
      p.esh_in = sh;
      p.ebs_in = nz * nyl * nx;
      if (blk_in->self_direct) {
        p.alt_blk = blk_in->me;
        p.alt0 = blk_in->alt0;
        p.alt1 = blk_in->alt1;
      }
      return launch_lines<0, 4>(ctx, p, n, nz);
    }
    return launch_lines<0, 1>(ctx, p, n, nz);
  }
  if (blk_in) return set_error(PB_ERR_ARG, "compact lines: blocked input on the Y pass only");
  p.li = nx;
  p.lo = nx * ny;
  p.es = 1;
  p.ninner = (int)ny;
  switch (C) {
    case 1: return launch_x_direct<1>(ctx, p, ny * nz);
    case 2: return launch_x_direct<2>(ctx, p, ny * nz);
    case 3: return launch_x_direct<3>(ctx, p, ny * nz);
    case 4: return launch_x_direct<4>(ctx, p, ny * nz);
    case 6: return launch_x_direct<6>(ctx, p, ny * nz);
    case 8: return launch_x_direct<8>(ctx, p, ny * nz);
    case 12: return launch_x_direct<12>(ctx, p, ny * nz);
    case 16: return launch_x_direct<16>(ctx, p, ny * nz);
  }
  return set_error(PB_ERR_UNSUPPORTED, "compact lines: X extent %lld", (long long)nx);
}

// Batched periodic (alpha, 1, alpha) solve, in place, n = 64*C points per line: contiguous
// lines (elem_stride 1) one wave each; interleaved lines (line_stride 1) through the LDS tile
// transpose. Returns PB_ERR_UNSUPPORTED for other layouts (the caller falls back to LDS PCR).
int lines_solve_batched(pb_ctx* ctx, int64_t n, int64_t nbatch, int64_t line_stride,
                        int64_t elem_stride, double alpha, double* d) {
  if (!compact_lines_supported(n) || !(alpha > 0.0 && alpha < 0.5))
    return PB_ERR_UNSUPPORTED;
  const int C = (int)(n / 64);
  LinePass p{};
  p.skip = ctx->op_skip;
  p.remap = 0;
  p.in0 = d;
  p.out0 = d;
  p.J = make_solve_op(alpha, C);
  const bool al16 = ((uintptr_t)d & 15) == 0;
  if (elem_stride == 1 && line_stride % 2 == 0 && al16 && line_stride >= n) {
    p.li = line_stride;
    switch (C) {
      case 1: return launch_solve_direct<1>(ctx, p, nbatch);
      case 2: return launch_solve_direct<2>(ctx, p, nbatch);
      case 3: return launch_solve_direct<3>(ctx, p, nbatch);
      case 4: return launch_solve_direct<4>(ctx, p, nbatch);
      case 6: return launch_solve_direct<6>(ctx, p, nbatch);
      case 8: return launch_solve_direct<8>(ctx, p, nbatch);
      case 12: return launch_solve_direct<12>(ctx, p, nbatch);
      case 16: return launch_solve_direct<16>(ctx, p, nbatch);
    }
  }
  if (line_stride == 1 && elem_stride >= nbatch) {
    p.li = 1;
    p.lo = 0;
    p.es = elem_stride;
    p.ninner = (int)nbatch;
    return launch_lines<0, 3>(ctx, p, n, 1);
  }
  return PB_ERR_UNSUPPORTED;
}

}  // namespace pb
