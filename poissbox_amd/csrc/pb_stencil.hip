// pb_stencil.hip -- 7-point periodic Laplacian engine for gfx950 (MI355X) and the fused CG passes.
//
// Replaces the reference hot loop src/poissbox.f90:112-119 (compute_lapl_pointwise ->
// evaluate_laplacian_pointwise, :128-148) and the PETSc KSPSolve_CG vector kernels around it
// (SURVEY.md Appendix A).
//
// Work decomposition (HBM-bound, AI ~ 0.8 flop/B, MFMA unused):
//   * a wave owns an x-segment of 64*V points (V = 2 -> one 16-B load per lane, 1 KiB per
//     wave-instruction) of TY consecutive y-rows and marches in z over a chunk of planes, keeping
//     planes k-1, k, k+1 of its rows in registers (each plane is read from HBM once per chunk);
//   * software pipeline: while plane k is computed, plane k+2 of the z-queue and the halo rows,
//     segment edges and epilogue operands (r, x, p_prev in CG pass B; non-temporal loads, they
//     are read once) of plane k+1 are in flight -- the grid is one resident round of 1-3
//     workgroups per CU (Epi::WGCU), so registers, not occupancy, buy the latency hiding;
//   * each chunk is marched upwards or downwards (Geo::rev): consecutive kernels start on the
//     planes their predecessor touched last, still in the Infinity Cache;
//   * x-neighbours come from the neighbouring lane (DPP wave shift); the two segment-end values
//     of all TY rows come from ONE masked load, broadcast with readlane; y-neighbours come from
//     the wave's own rows, the tile's top/bottom rows from the neighbouring tile (L2 hit: tiles
//     are remapped so neighbours share an XCD);
//   * z ghosts (periodic wrap or the neighbouring rank's plane) are read through plane pointers
//     chosen per plane, or (Geo::wrap, one rank) as the wrap planes of the raw input arrays, so no
//     ghost copy is made on one rank.
// Summation order per point matches the reference dot product with its zero terms dropped:
// z-, y-, x-, centre, x+, y+, z+ (built with -ffp-contract=off => bit-identical to the oracle).
#include "pb_cg_device.hpp"

namespace pb {

struct Geo {
  int nx, ny, nzl;
  int64_t plane;
  int nsegx, ntile, nchunk, kc, ty;
  int k_lo, k_hi, kstride;  // chunk c covers planes [k_lo + c*kstride, min(+kc, k_hi))
  int remap;  // XCD-aware block remap on/off (PB_XCD_REMAP, default on)
  int nt;     // non-temporal output stores (PB_STENCIL_NT, default on)
  int rev;    // march each chunk downwards (k from the top plane to the bottom one)
  int k0;     // global index of local plane 0 (red-black colouring)
  int wrap;   // planes -1 / nzl are the periodic wrap of the raw arrays (StencilPlanes::wrap)
};

// ---------------------------------------------------------------------------------------------
// Loaders: NR raw arrays per point, combined into the field value by value().
// ---------------------------------------------------------------------------------------------
struct PlainLoad {
  static constexpr int NR = 1;
  static constexpr bool GHOST_RAW = false;  // ghost planes hold raw values to transform
  const double* __restrict__ x;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ const double* src(int) const { return x; }
  __device__ __forceinline__ double value(const double* raw) const { return raw[0]; }
};

// p_new = (dinv*r + shift) + bb*p_old  -- PCApply_Jacobi + MatNullSpaceRemove + VecAYPX fused
struct CgState;
__device__ __forceinline__ double cg_bb(const CgState* st);
struct CombineLoad {
  static constexpr int NR = 2;
  static constexpr bool GHOST_RAW = false;
  const double* __restrict__ r;
  const double* __restrict__ p;
  const CgState* st;
  double dinv, shift, bb;
  // 1: the state is past stage 1 (betaold already overwritten): take pass A's beta/betaold from
  // bbp, which stage 1 computed with the same operands (pass B re-forming p, PB_CG_PSTORE_B)
  int after1 = 0;
  __device__ __forceinline__ void prepare() { prepare_from(*st); }
  template <class S>
  __device__ __forceinline__ void prepare_from(const S& s) {
    dinv = s.dinv;
    shift = -s.mu;
    bb = after1 ? s.bbp : (s.it == 0 ? 0.0 : s.beta / s.betaold);
  }
  __device__ __forceinline__ const double* src(int a) const { return a == 0 ? r : p; }
  __device__ __forceinline__ double f(double rv, double pv) const {
    double z = dinv * rv;
    z = z + shift;
    return z + bb * pv;
  }
  __device__ __forceinline__ double value(const double* raw) const { return f(raw[0], raw[1]); }
  __device__ __forceinline__ double one(int64_t idx) const { return f(r[idx], p[idx]); }
};

// ---------------------------------------------------------------------------------------------
// Epilogues: NE operand arrays prefetched one plane ahead; put() consumes centre value c,
// Laplacian w and the operands at owned index idx.
// ---------------------------------------------------------------------------------------------
struct StoreY {
  static constexpr int NS = 0, NE = 0;
  static constexpr bool RAW = false, TALL = true;
  static constexpr int WGCU = 3;  // workgroups per CU the grid is sized for
  static constexpr bool PREFETCH = true;
  double* __restrict__ y;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ const double* src(int) const { return nullptr; }
  template <int V>
  __device__ __forceinline__ void put(RowIx idx, const double (&c)[V], const double (&w)[V],
                                      double (&)[1][V], double*, int nt) const {
    store_row<V>(y, idx, w, nt);
    (void)c;
  }
};

// CG pass A: store p_new, accumulate p.w (VecXDot(P, W)). STORE = false: the
// p store moves to pass B, which re-forms p from r and p_old on load (PB_CG_PSTORE_B): pass A
// becomes read-only (16 B/DoF) and pass B reads 2 / writes 2 arrays (32 B/DoF), same 48 B/DoF.
// Read-only (STORE = false): 4-row tiles, one workgroup per CU (z-chunks of half the slab at
// 512^3), measured 0.378 vs 0.391 ms for 8-row tiles (profiles/r02/ab_pst_defer_512.jsonl).
#ifndef PB_PASSA_TALL
#define PB_PASSA_TALL 0
#endif
template <bool STORE>
struct PassAT {
  static constexpr int NS = 1, NE = 0;
  static constexpr bool RAW = false, TALL = STORE || PB_PASSA_TALL;  // put() takes the Laplacian; 8-row tiles
  static constexpr int WGCU = STORE ? 3 : 1;        // (4-row tiles; 1 with 8 rows)
  static constexpr bool CAP = !STORE, WIDE8 = !STORE;
  static constexpr bool PREFETCH = true;
  // (p stores non-temporal like every engine output: cached stores, which pass B could re-read
  // from the Infinity Cache, measured within noise, profiles/r01/ab_passa_nt.txt)
  double* __restrict__ p_new;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ const double* src(int) const { return nullptr; }
  template <int V>
  __device__ __forceinline__ void put(RowIx idx, const double (&c)[V], const double (&w)[V],
                                      double (&)[1][V], double* acc, int nt) const {
    if constexpr (STORE) store_row<V>(p_new, idx, c, nt);
#pragma unroll
    for (int e = 0; e < V; ++e) acc[0] += w[e] * c[e];
  }
};
using PassA = PassAT<true>;

// CG pass B: r += (-a) w with w = A p recomputed; then the PC/null-space sums of the new
// residual: s = dinv*r, t = s - mu_old:  sum t, sum t^2, sum t*r, sum r.
// The solution update is deferred over D iterations (x is not part of the recurrence; D = 4 by
// default, 2 or 0 by PB_CG_DEFER_X), the directions kept in a ring of D p buffers:
//   XU = 0 (i % D < D-1):      no x traffic, alpha_i p_i stays pending;
//   XU = 3 (D = 4, i % 4 = 3): x += a_{i-3} p_{i-3} + a_{i-2} p_{i-2} + a_{i-1} p_{i-1} + a_i p_i
//   XU = 1 (D = 2, odd i):     x += (alpha_{i-1} p_{i-1} + alpha_i p_i);
//   XU = 2 (no deferral):      x += alpha_i p_i every iteration.
// Operands are prefetched one plane ahead (XU = 1: 3 operand rows, 238 VGPRs -- one workgroup
// per CU is all the grid uses; measured 2 % faster than loading them in the plane's own step).
#ifndef PB_PSTB_WGCU
#define PB_PSTB_WGCU 1
#endif
#ifndef PB_PSTB_TALL
#define PB_PSTB_TALL 0
#endif
// PST (PB_CG_PSTORE_B): the field is p re-formed from (r, p_old) by CombineLoad, stored to p_out;
// r is read from op[0] (= r) and written to r_out (another buffer: neighbouring waves still read
// r through the z-queue, an in-place update would race with them).
// SUMS = false: the single-reduction iteration's pass P (the residual sums move to pass S)
template <int XU, bool PST = false, bool SUMS = true>
struct PassB {
  static constexpr int NS = SUMS ? 4 : 0, NE = XU == 1 ? 3 : (XU == 2 ? 2 : (XU == 3 ? 5 : 1));
  static constexpr bool RAW = false;  // put() takes the Laplacian, not the 7 values
  // one workgroup per CU (z-chunks of half the slab at 512^3): 8-10 % faster than 3 per CU
  static constexpr int WGCU = PST ? PB_PSTB_WGCU : 1;
  static constexpr bool TALL = PST && XU == 0 && PB_PSTB_TALL;  // (A/B builds)
  static constexpr bool CAP = true, WIDE8 = PST && XU == 0;
  static constexpr bool PREFETCH = true;
  double* __restrict__ x;
  double* __restrict__ r;
  const double* __restrict__ p_prev;  // p of iteration i-1
  const double* __restrict__ p_m2;    // XU = 3: p of iterations i-2, i-3
  const double* __restrict__ p_m3;
  const CgState* st;
  double alpha, alpha_prev, dinv, mu, a2, a3;
  double* __restrict__ r_out = nullptr;  // PST only
  double* __restrict__ p_out = nullptr;
  // PST: operands r (op 0) and p_{i-1} = p_old (op 2) are the centre plane's raw z-queue values
  // (CombineLoad arrays 0 and 1) -- taken from the queue instead of loaded again
  static constexpr int qop(int a) { return !PST ? -1 : (a == 0 ? 0 : (a == 2 ? 1 : -1)); }
  __device__ __forceinline__ void prepare() { prepare_from(*st); }
  template <class S>
  __device__ __forceinline__ void prepare_from(const S& s) {
    alpha = s.alpha;
    alpha_prev = s.alpha_prev;
    dinv = s.dinv;
    mu = s.mu;
    if constexpr (XU == 3) {  // pending alphas of iterations i-3, i-2, i-1
      a3 = s.pa[0];
      a2 = s.pa[1];
      alpha_prev = s.pa[2];
    }
  }
  __device__ __forceinline__ const double* src(int a) const {
    return a == 0 ? r : (a == 1 ? x : (a == 2 ? p_prev : (a == 3 ? p_m2 : p_m3)));
  }
  template <int V>
  __device__ __forceinline__ void put(RowIx idx, const double (&c)[V], const double (&w)[V],
                                      double (&op)[NE][V], double* acc, int nt) const {
    double rv[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      rv[e] = op[0][e] + (-alpha) * w[e];
      if constexpr (SUMS) {
        const double s = dinv * rv[e];
        const double t = s - mu;
        acc[0] += t;
        acc[1] += t * t;
        acc[2] += t * rv[e];
        acc[3] += rv[e];
      }
    }
    (void)acc;
    if constexpr (PST) {
      store_row<V>(r_out, idx, rv, nt);
      store_row<V>(p_out, idx, c, nt);
    } else {
      store_row<V>(r, idx, rv, nt);
    }
    if constexpr (XU == 1) {
      double xv[V];
#pragma unroll
      for (int e = 0; e < V; ++e) xv[e] = op[1][e] + (alpha_prev * op[2][e] + alpha * c[e]);
      store_row<V>(x, idx, xv, nt);
    } else if constexpr (XU == 2) {
      double xv[V];
#pragma unroll
      for (int e = 0; e < V; ++e) xv[e] = op[1][e] + alpha * c[e];
      store_row<V>(x, idx, xv, nt);
    } else if constexpr (XU == 3) {  // x += a3 p_{i-3} + a2 p_{i-2} + alpha_prev p_{i-1} + alpha p_i
      double xv[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        double u = a3 * op[4][e];
        u = u + a2 * op[3][e];
        u = u + alpha_prev * op[2][e];
        u = u + alpha * c[e];
        xv[e] = op[1][e] + u;
      }
      store_row<V>(x, idx, xv, nt);
    }
  }
};

// Single-reduction CG pass S (PETSc KSPSolve_CG_SingleReduction: z = B r, S = A z, then z'z,
// z'r and z'S in one reduction): the field is t = dinv r' - mu_old, formed on load (ghost planes
// of a split grid hold raw r' and are transformed too); the engine's Laplacian is s = A t. Sums
// t, t^2, t.r', r' (norm, beta and the mean as pass B's) and t.s (delta = z'A z: z = t - const
// and A annihilates constants, so t'A t is z'A z up to rounding). Read-only: 8 B/DoF.
struct ZLoad {
  static constexpr int NR = 1;
  static constexpr bool GHOST_RAW = true;
  const double* __restrict__ r;
  const CgState* st;
  double dinv = 1.0, shift = 0.0;
  __device__ __forceinline__ void prepare() { prepare_from(*st); }
  template <class S>
  __device__ __forceinline__ void prepare_from(const S& s) {
    dinv = s.dinv;
    shift = -s.mu;
  }
  __device__ __forceinline__ const double* src(int) const { return r; }
  __device__ __forceinline__ double value(const double* raw) const {
    double z = dinv * raw[0];
    return z + shift;
  }
};
struct SrSums {
  static constexpr int NS = 5, NE = 1;
  static constexpr bool RAW = false;
  static constexpr int WGCU = 1;
  static constexpr bool CAP = true, WIDE8 = true;
  static constexpr bool PREFETCH = true;
  // operand 0 (r') is the centre plane's raw queue value
  static constexpr int qop(int a) { return a == 0 ? 0 : -1; }
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ const double* src(int) const { return nullptr; }
  template <int V>
  __device__ __forceinline__ void put(RowIx, const double (&c)[V], const double (&w)[V],
                                      double (&op)[1][V], double* acc, int) const {
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const double t = c[e], rv = op[0][e];
      acc[0] += t;
      acc[1] += t * t;
      acc[2] += t * rv;
      acc[3] += rv;
      acc[4] += t * w[e];
    }
  }
};


// Epi::qop(a) (optional): operand a is raw z-queue array qop(a) of the centre plane (-1: loaded)
template <class E, class = void>
struct HasQop {
  static constexpr bool v = false;
};
template <class E>
struct HasQop<E, std::void_t<decltype(E::qop(0))>> {
  static constexpr bool v = true;
};
template <class E>
__device__ __forceinline__ constexpr int qop_of(int a) {
  if constexpr (HasQop<E>::v) return E::qop(a);
  else return -1;
}

// Load / Epi structs that read CG scalars have prepare_from(state): fed the register copy
template <class T>
__device__ __forceinline__ auto prepare_state(T& t, const CgState& s, int)
    -> decltype(t.prepare_from(s), void()) {
  t.prepare_from(s);
}
template <class T>
__device__ __forceinline__ void prepare_state(T& t, const CgState&, long) {
  t.prepare();
}

// ---------------------------------------------------------------------------------------------
// The stencil engine
// ---------------------------------------------------------------------------------------------
template <int V, int TY, class Load, class Epi>
__global__ __launch_bounds__(kThreads) void star7_kernel(Geo g, double cx, double cy, double cz,
                                                         double cc, Load ld0,
                                                         const double* __restrict__ ghost_lo,
                                                         const double* __restrict__ ghost_hi,
                                                         Epi ep0, double* parts,
                                                         const int* __restrict__ skip, Fold fold) {
  Load ld = ld0;
  Epi ep = ep0;
  if (!fold.stage) {
    if (skip && *skip) return;  // device-side convergence flag (uniform)
    ld.prepare();
    ep.prepare();
  }
  // folded finalize: run after the first planes' loads are issued (they need no CG scalar), so
  // the partial-sum loads and the plane loads are in flight together
  auto do_fold = [&]() -> bool {
    CgState sst;  // register copy
    fold_prologue(fold, sst);
    if (sst.done) return false;  // uniform: every wave computed the same state
    prepare_state(ld, sst, 0);
    prepare_state(ep, sst, 0);
    return true;
  };
  constexpr int NS = Epi::NS, NR = Load::NR;
  constexpr int NE = Epi::NE > 0 ? Epi::NE : 1;
  double acc[NS > 0 ? NS : 1];
#pragma unroll
  for (int s = 0; s < (NS > 0 ? NS : 1); ++s) acc[s] = 0.0;

  // wave index as a scalar: row addresses are wave-uniform (SGPR base + one lane offset, RowIx)
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware remap (speed only): the dispatcher deals blocks round-robin over the 8 XCDs, so
  // give each XCD a contiguous range of logical tiles -- y/x-neighbouring tiles then share the
  // XCD's L2 and their halo rows hit there. Bijective for any grid size.
  int b = xcd_block(g.remap);
  const int seg = b % g.nsegx;
  b /= g.nsegx;
  const int tile = b % g.ntile;
  const int chunk = b / g.ntile;
  const int j0 = (tile * kWaves + wid) * TY;
  const int kb = g.k_lo + chunk * g.kstride;
  const int ke = min(kb + g.kc, g.k_hi);
  const int nx = g.nx;
  const int i0 = seg * 64 * V + lane * V;
  const bool active = i0 < nx;
  const bool wave_on = j0 < g.ny && kb < g.k_hi;
  const int ic = active ? i0 : 0;  // clamp addresses of idle lanes
  // x-edges: lane 0 needs x[seg0-1]; the last active lane needs x[seg_end] (periodic wrap).
  // One masked load per plane and array fetches them for all TY rows: lane t < TY the left edge
  // of row t, lane 32 + t the right edge; they are broadcast with readlane.
  const int seg0 = seg * 64 * V;
  const int seg_end = min(seg0 + 64 * V, nx);
  const bool needL = lane == 0;
  const bool needR = active && (lane == 63 || i0 + V >= nx);
  const int edge_row = lane < 32 ? lane : lane - 32;
  const bool edge_lane = edge_row < TY;
  const int edge_i = lane < 32 ? (seg0 == 0 ? nx - 1 : seg0 - 1) : (seg_end >= nx ? 0 : seg_end);
  const int64_t edge_off = (int64_t)(j0 + (edge_lane ? edge_row : 0)) * nx + edge_i;
  const unsigned boff = (unsigned)ic * 8u;  // lane byte offset inside a row
  const int64_t row_dn = (int64_t)(j0 == 0 ? g.ny - 1 : j0 - 1) * nx;
  const int64_t row_up = (int64_t)((j0 + TY >= g.ny) ? 0 : j0 + TY) * nx;
  auto rix = [&](int64_t row) { return RowIx{row, boff}; };
  if (fold.stage && !wave_on && !do_fold()) return;

  if (wave_on) {
    // combined z-queue (planes k-1, k, k+1) and raw prefetch of plane k+2
    double q0[TY][V], q1[TY][V], q2[TY][V];
    double zr[NR][TY][V];
    bool zr_ghost = false;
    // plane-k operands (combined) and their plane-(k+1) prefetch (raw)
    double hdn[V], hup[V], edge = 0.0;
    double hdn_r[NR][V], hup_r[NR][V], edge_r[NR];
    double opc[TY][NE][V], opn[Epi::PREFETCH ? TY : 1][NE][V];

    // Every load below is issued unconditionally (ghost planes by a uniform pointer select, the
    // chunk's last step re-loading valid planes): no branch around a load, so the compiler keeps
    // the prefetch registers stable instead of copying them at control-flow joins -- such copies
    // must wait for the loads and serialised the software pipeline (pass A ran ~10 % slower).
    // raw rows of plane kk in [-1, nzl] -> dst (ghost: the plane is a ghost buffer)
    auto issue_rows = [&](int kk, double (&dst)[NR][TY][V], bool& ghost) {
      if (g.wrap) kk = kk < 0 ? kk + g.nzl : (kk >= g.nzl ? kk - g.nzl : kk);
      ghost = kk < 0 || kk >= g.nzl;
      const double* gp = kk < 0 ? ghost_lo : ghost_hi;
      const int64_t base = ghost ? 0 : (int64_t)kk * g.plane;
#pragma unroll
      for (int a = 0; a < NR; ++a) {
        const double* src = ghost ? gp : ld.src(a);
#pragma unroll
        for (int t = 0; t < TY; ++t) load_row<V>(src, rix(base + (int64_t)(j0 + t) * nx), dst[a][t]);
      }
    };
    auto take_rows = [&](const double (&src)[NR][TY][V], bool ghost, double (&q)[TY][V]) {
#pragma unroll
      for (int t = 0; t < TY; ++t)
#pragma unroll
        for (int e = 0; e < V; ++e) {
          double raw[NR];
#pragma unroll
          for (int a = 0; a < NR; ++a) raw[a] = src[a][t][e];
          q[t][e] = (ghost && !Load::GHOST_RAW) ? src[0][t][e] : ld.value(raw);
        }
    };
    auto issue_zrow = [&](int kk) { issue_rows(kk, zr, zr_ghost); };
    auto take_zrow = [&](double (&q)[TY][V]) { take_rows(zr, zr_ghost, q); };
    auto issue_plane_ops = [&](int kk) {  // halo rows, edges, epilogue operands of own plane kk
      const int64_t base = (int64_t)kk * g.plane;
#pragma unroll
      for (int a = 0; a < NR; ++a) {
#ifdef PB_ABLATE_HALO  // timing experiments only (wrong results): y-halo rows from own rows
        load_row<V>(ld.src(a), rix(base + (int64_t)j0 * nx), hdn_r[a]);
        load_row<V>(ld.src(a), rix(base + (int64_t)(j0 + TY - 1) * nx), hup_r[a]);
#else
        load_row<V>(ld.src(a), rix(base + row_dn), hdn_r[a]);
        load_row<V>(ld.src(a), rix(base + row_up), hup_r[a]);
#endif
        edge_r[a] = 0.0;
#ifndef PB_ABLATE_EDGES  // timing experiments only (wrong results): no segment-edge loads
        edge_r[a] = ld.src(a)[base + edge_off];  // (all lanes: valid address, only edge lanes read)
#endif
      }
      if constexpr (Epi::NE > 0 && Epi::PREFETCH) {
#pragma unroll
        for (int t = 0; t < TY; ++t)
#pragma unroll
          for (int a = 0; a < Epi::NE; ++a)
            if (qop_of<Epi>(a) < 0)
              load_row_nt<V>(ep.src(a), rix(base + (int64_t)(j0 + t) * nx), opn[t][a]);
      }
    };
    // operands that are raw queue values of a plane (Epi::qop): copied, not loaded
    auto take_queue_ops = [&](const double (&raw)[NR][TY][V]) {
      if constexpr (Epi::NE > 0 && Epi::PREFETCH && HasQop<Epi>::v) {
#pragma unroll
        for (int t = 0; t < TY; ++t)
#pragma unroll
          for (int a = 0; a < Epi::NE; ++a)
            if (qop_of<Epi>(a) >= 0)
#pragma unroll
              for (int e = 0; e < V; ++e) opn[t][a][e] = raw[qop_of<Epi>(a)][t][e];
      }
    };
    auto issue_ops_now = [&](int kk) {  // operands without prefetch: plane kk straight to opc
      if constexpr (Epi::NE > 0 && !Epi::PREFETCH) {
        const int64_t base = (int64_t)kk * g.plane;
#pragma unroll
        for (int t = 0; t < TY; ++t)
#pragma unroll
          for (int a = 0; a < Epi::NE; ++a)
            load_row_nt<V>(ep.src(a), rix(base + (int64_t)(j0 + t) * nx), opc[t][a]);
      }
    };
    auto take_plane_ops = [&]() {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        double rd[NR], ru[NR];
#pragma unroll
        for (int a = 0; a < NR; ++a) {
          rd[a] = hdn_r[a][e];
          ru[a] = hup_r[a][e];
        }
        hdn[e] = ld.value(rd);
        hup[e] = ld.value(ru);
      }
      edge = ld.value(edge_r);
      if constexpr (Epi::NE > 0 && Epi::PREFETCH) {
#pragma unroll
        for (int t = 0; t < TY; ++t)
#pragma unroll
          for (int a = 0; a < Epi::NE; ++a)
#pragma unroll
            for (int e = 0; e < V; ++e) opc[t][a][e] = opn[t][a][e];
      }
    };

    // prologue: planes kf-dir, kf combined; raw plane kf+dir and plane kf's operands in flight.
    // Marching downwards (g.rev) lets a kernel start on the planes its predecessor touched last
    // (still in the 256 MiB Infinity Cache); per-point arithmetic is unchanged (zm/zp swap).
    const int dir = g.rev ? -1 : 1;
    const int kf = g.rev ? ke - 1 : kb;
    const int nk = ke - kb;
    // The first planes' loads go out together (one wait instead of one per plane; the
    // prologue is ~10 % of a 32-plane chunk): one array through the queue -- planes kf-dir, kf,
    // kf+dir and plane kf's operands all in flight; two -- kf-dir and kf, then the rest.
    {
      double r0[NR][TY][V], r1[NR][TY][V];
      bool g0 = false, g1 = false;
      issue_rows(kf - dir, r0, g0);
      issue_rows(kf, r1, g1);
      if constexpr (NR == 1) {
        issue_plane_ops(kf);
        issue_zrow(kf + dir);
      }
      if (fold.stage && !do_fold()) return;
      take_rows(r0, g0, q0);
      take_rows(r1, g1, q1);
      take_queue_ops(r1);  // plane kf (owned, never a ghost)
      if constexpr (NR != 1) {
        issue_plane_ops(kf);
        issue_zrow(kf + dir);
      }
    }
    for (int m = 0; m < nk; ++m) {
      const int k = kf + m * dir;
      take_zrow(q2);                    // plane k+dir (in flight since the previous step)
      take_plane_ops();                 // halo/edges/operands of plane k
      take_queue_ops(zr);               // queue-sourced operands of plane k+dir
      issue_ops_now(k);
      issue_zrow(m + 2 <= nk ? k + 2 * dir : k + dir);  // (last step: a valid plane, unused)
      issue_plane_ops(m + 1 < nk ? k + dir : k);
      const int64_t base = (int64_t)k * g.plane;
#pragma unroll
      for (int t = 0; t < TY; ++t) {
        const double eL = readlane_d(edge, t);
        const double eR = readlane_d(edge, 32 + t);
        const double fromL = dpp_from_lower(q1[t][V - 1]);
        const double fromR = dpp_from_upper(q1[t][0]);
        const double xl0 = needL ? eL : fromL;
        const double xrl = needR ? eR : fromR;
        if constexpr (Epi::RAW) {  // the epilogue combines the 7 values itself
          double nzm[V], nym[V], nxm[V], nxp[V], nyp[V], nzp[V];
#pragma unroll
          for (int e = 0; e < V; ++e) {
            nxm[e] = e == 0 ? xl0 : q1[t][e - 1];
            nxp[e] = e == V - 1 ? xrl : q1[t][e + 1];
            nym[e] = t == 0 ? hdn[e] : q1[t - 1][e];
            nyp[e] = t == TY - 1 ? hup[e] : q1[t + 1][e];
            nzm[e] = g.rev ? q2[t][e] : q0[t][e];
            nzp[e] = g.rev ? q0[t][e] : q2[t][e];
          }
          if (active)
            ep.template put_raw<V>(rix(base + (int64_t)(j0 + t) * nx), i0 + j0 + t + g.k0 + k,
                                   nzm, nym, nxm, q1[t], nxp, nyp, nzp, opc[t], acc, g.nt);
        } else {
          double w[V];
#pragma unroll
          for (int e = 0; e < V; ++e) {
            const double xm = e == 0 ? xl0 : q1[t][e - 1];
            const double xp = e == V - 1 ? xrl : q1[t][e + 1];
            const double ym = t == 0 ? hdn[e] : q1[t - 1][e];
            const double yp = t == TY - 1 ? hup[e] : q1[t + 1][e];
            const double zm = g.rev ? q2[t][e] : q0[t][e];
            const double zp = g.rev ? q0[t][e] : q2[t][e];
            double s = cz * zm;
            s = s + cy * ym;
            s = s + cx * xm;
            s = s + cc * q1[t][e];
            s = s + cx * xp;
            s = s + cy * yp;
            s = s + cz * zp;
            w[e] = s;
          }
          if (active)
            ep.template put<V>(rix(base + (int64_t)(j0 + t) * nx), q1[t], w, opc[t], acc, g.nt);
        }
      }
#pragma unroll
      for (int t = 0; t < TY; ++t)
#pragma unroll
        for (int e = 0; e < V; ++e) {
          q0[t][e] = q1[t][e];
          q1[t][e] = q2[t][e];
        }
    }
  }
  block_partials<NS>(acc, parts);
}

// ---------------------------------------------------------------------------------------------
// Launch configuration
// ---------------------------------------------------------------------------------------------
// Plane sets: PLANES_ALL = [0, nzl); PLANES_INTERIOR = [1, nzl-1) (no ghost plane is read);
// PLANES_BOUNDARY = {0, nzl-1} (the two planes that read ghosts) -- the split lets the halo
// exchange of a multi-rank step overlap the interior.
static Geo make_geo(pb_grid* g, int V, int TY, int mode, int rev, int wgcu, int skew) {
  Geo geo;
  geo.rev = rev;
  geo.k0 = (int)g->k0;
  geo.wrap = 0;
  geo.nx = (int)g->n[0];
  geo.ny = (int)g->n[1];
  geo.nzl = (int)g->nzl;
  geo.plane = g->plane;
  geo.ty = TY;
  geo.remap = 1;  // XCD-aware block remap
  geo.nt = 1;     // non-temporal output stores
  geo.nsegx = (geo.nx + 64 * V - 1) / (64 * V);
  geo.ntile = (geo.ny + kWaves * TY - 1) / (kWaves * TY);
  if (mode == PLANES_BOUNDARY) {
    geo.k_lo = 0;
    geo.k_hi = geo.nzl;
    geo.kc = 1;
    geo.kstride = geo.nzl - 1;
    geo.nchunk = 2;
    return geo;
  }
  geo.k_lo = mode == PLANES_INTERIOR ? 1 : 0;
  geo.k_hi = mode == PLANES_INTERIOR ? geo.nzl - 1 : geo.nzl;
  const int nk = geo.k_hi - geo.k_lo;
  const int columns = geo.nsegx * geo.ntile;
  // wgcu (the epilogue's WGCU) workgroups per CU: long z-chunks, few chunk-boundary re-reads.
  // Measured at 512^3: 3 per CU for the matvec and pass A (768 blocks beat 512 even where the
  // registers allow only 2 resident), 1 per CU for pass B
  int target = wgcu * g->ctx->num_cus;
  int nchunk = (target + columns - 1) / columns;
  // z-chunks shorter than 64 planes re-read too many boundary planes (2 per
  // chunk): use fewer, longer chunks, but keep at least one workgroup per CU (256^3: 8 chunks of
  // 32 planes instead of 24 of 11, measured 8-15 % faster)
  const int kcmin = 64;
  if (nk / nchunk < kcmin) {
    const int floor_cu = (g->ctx->num_cus + columns - 1) / columns;
    nchunk = std::max(nk / kcmin, floor_cu);
  }
  if (nchunk > nk) nchunk = nk;
  if (nchunk < 1) nchunk = 1;
  geo.kc = (nk + nchunk - 1) / nchunk;
  // chunk skew (in 64ths of a chunk): longer chunks and a shorter last one, so that the planes
  // the chunks march through together are not a power-of-two number of planes apart. The
  // standalone matvec's four 128-plane chunks at 512^3 ran 0.37-0.42 ms depending on where its x
  // and y sat (pairs of buffers: one slow, one fast group); chunks of 136 planes ran 0.36-0.38
  // over the same pairs (profiles/r06/placement/). The CG passes' two 256-plane chunks gained
  // nothing from it (skew 2: within noise, 4 / 8: slower) and keep 0. Only for chunks at least
  // 128 MiB of planes apart: 256^3's matvec (eight 32-plane chunks, 16 MiB apart) ran 0.0439
  // against 0.0414 ms with the skew (profiles/r06/placement/cgcfg256.jsonl)
  if (nchunk > 1 && skew > 0 && (int64_t)geo.kc * g->plane * 8 >= ((int64_t)128 << 20)) {
    const int kc = geo.kc + std::max(1, geo.kc * skew / 64);
    if ((int64_t)kc * (nchunk - 1) < nk) geo.kc = kc;
  }
  geo.kstride = geo.kc;
  geo.nchunk = (nk + geo.kc - 1) / geo.kc;
  return geo;
}

static int pick_ty(int ny) {
  if (ny % 4 == 0) return 4;
  if (ny % 2 == 0) return 2;
  return 1;
}

// Epi::CAP (optional trait): keep at most WGCU workgroups resident per CU (launch_t)
template <class E, class = void>
struct CapOf {
  static constexpr bool v = false;
};
template <class E>
struct CapOf<E, std::void_t<decltype(E::CAP)>> {
  static constexpr bool v = E::CAP;
};
constexpr size_t kLdsPerCu = 160 * 1024;

template <int V, int TY, class Load, class Epi>
static int launch_t(pb_grid* g, const Star& s, const Load& ld, const StencilPlanes& gp,
                    const Epi& ep, const int* skip, int mode, int part_off, int* nb_out, int rev,
                    int wgcu, const Fold& fold, int64_t part_end) {
  Geo geo = make_geo(g, V, TY, mode, rev, wgcu > 0 ? wgcu : Epi::WGCU,
                     std::is_same_v<Epi, StoreY> ? tune("stencil_kc_skew", 4)
                                                 : tune("engine_kc_skew", 0));
  geo.wrap = gp.wrap && !g->ctx->split ? 1 : 0;
  if constexpr (std::is_same_v<Epi, StoreY>) {  // (A/B runs)
    geo.nt = tune("stencil_nt", 1);
    const int kc = tune("stencil_kc", 0);
    if (kc > 0 && mode != PLANES_BOUNDARY) {
      const int nk = geo.k_hi - geo.k_lo;
      geo.kc = std::min(kc, nk);
      geo.kstride = geo.kc;
      geo.nchunk = (nk + geo.kc - 1) / geo.kc;
    }
  }
  const int64_t nblocks = (int64_t)geo.nsegx * geo.ntile * geo.nchunk;
  constexpr int NS = Epi::NS > 0 ? Epi::NS : 1;
  // part_end (in blocks, 0: the whole buffer): the end of the caller's partial-sum region
  const int64_t end = part_end > 0 ? part_end * NS : g->ctx->partials_cap;
  if ((part_off + nblocks) * NS > std::min(end, g->ctx->partials_cap))
    return set_error(PB_ERR_UNSUPPORTED, "stencil grid of %lld blocks exceeds partials capacity",
                     (long long)nblocks);
  // Residency cap (Epi::CAP, the CG passes): a grid with more columns than the epilogue's WGCU
  // workgroups per CU (planes of 1024^2 points: 512 columns of 4-row tiles, twice the 1-per-CU
  // count) would run two workgroups per CU side by side; an LDS request no kernel uses keeps it at
  // WGCU resident per CU, the rest following as slots free. 1024x1024x128 (config 4's per-GPU
  // slab): pass B 0.847 -> 0.772 ms, iteration 1.47 -> 1.40 ms (profiles/r04/shapes_r4.txt).
  size_t lds = 0;
  if constexpr (CapOf<Epi>::v) {
    const int w = wgcu > 0 ? wgcu : Epi::WGCU;
    if (nblocks > (int64_t)w * g->ctx->num_cus) lds = kLdsPerCu / (size_t)(w + 1) + 4096;
  }
  hipLaunchKernelGGL((star7_kernel<V, TY, Load, Epi>), dim3((unsigned)nblocks), dim3(kThreads),
                     lds, g->ctx->engine_stream ? g->ctx->engine_stream : g->ctx->stream, geo, s.cx,
                     s.cy, s.cz, s.cc, ld, gp.ghost_lo, gp.ghost_hi, ep,
                     g->ctx->d_partials + (int64_t)part_off * NS, skip, fold);
  PB_HIP(hipGetLastError());
  if (nb_out) *nb_out = (int)nblocks;
  return PB_OK;
}

// Epi::TALL (optional trait): on planes of >= 512^2 points the epilogue runs 8 rows per wave
// with one workgroup per CU (at 512^3: matvec 0.402 -> 0.386 ms, pass A 0.616 -> 0.586 ms; the
// pass B variants are slower that way and keep 4 rows, profiles/r01/tune_ty8.txt)
template <class E, class = void>
struct TallOf {
  static constexpr bool v = false;
};
template <class E>
struct TallOf<E, std::void_t<decltype(E::TALL)>> {
  static constexpr bool v = E::TALL;
};

// Epi::WIDE8 (optional trait): 8 rows per wave when 4-row tiles would leave more columns than
// WGCU workgroups per CU (planes 1024 or more points wide): the CG passes then run one column per
// CU as at 512^3. 1024x1024x128: pass A 0.412 -> 0.389 ms, pass B 0.759 -> 0.720 ms, iteration
// 1.39 -> 1.33 ms, the 512^3 rate; at 512^3 itself 4-row tiles stay faster
// (profiles/r04/shapes_r4b.txt)
template <class E, class = void>
struct Wide8Of {
  static constexpr bool v = false;
};
template <class E>
struct Wide8Of<E, std::void_t<decltype(E::WIDE8)>> {
  static constexpr bool v = E::WIDE8;
};

template <class Load, class Epi>
static int launch_any(pb_grid* g, const Star& s, const Load& ld, const StencilPlanes& gp,
                      const Epi& ep, const int* skip, int mode = PLANES_ALL, int part_off = 0,
                      int* nb_out = nullptr, int rev = 0, int wgcu = 0,
                      const Fold& fold = Fold{}, int64_t part_end = 0) {
  const bool vec2 = (g->n[0] % 2) == 0;
  const int ty = pick_ty((int)g->n[1]);
  if constexpr (Wide8Of<Epi>::v) {
    const int64_t cols4 = ((g->n[0] + 127) / 128) * ((g->n[1] + kWaves * 4 - 1) / (kWaves * 4));
    const int w = wgcu > 0 ? wgcu : Epi::WGCU;
    if (vec2 && ty == 4 && g->n[1] % 8 == 0 && cols4 > (int64_t)w * g->ctx->num_cus)
      return launch_t<2, 8>(g, s, ld, gp, ep, skip, mode, part_off, nb_out, rev, wgcu, fold, part_end);
  }
  if constexpr (TallOf<Epi>::v) {
    if (vec2 && ty == 4 && g->n[1] % 8 == 0 && g->plane >= 512 * 512 &&
        tune("stencil_tall", 1) != 0)
      return launch_t<2, 8>(g, s, ld, gp, ep, skip, mode, part_off, nb_out, rev,
                            wgcu > 0 ? wgcu : 1, fold, part_end);
  }
  if (vec2) {
    switch (ty) {
      case 4: return launch_t<2, 4>(g, s, ld, gp, ep, skip, mode, part_off, nb_out, rev, wgcu, fold, part_end);
      case 2: return launch_t<2, 2>(g, s, ld, gp, ep, skip, mode, part_off, nb_out, rev, wgcu, fold, part_end);
      default: return launch_t<2, 1>(g, s, ld, gp, ep, skip, mode, part_off, nb_out, rev, wgcu, fold, part_end);
    }
  }
  switch (ty) {
    case 4: return launch_t<1, 4>(g, s, ld, gp, ep, skip, mode, part_off, nb_out, rev, wgcu, fold, part_end);
    case 2: return launch_t<1, 2>(g, s, ld, gp, ep, skip, mode, part_off, nb_out, rev, wgcu, fold, part_end);
    default: return launch_t<1, 1>(g, s, ld, gp, ep, skip, mode, part_off, nb_out, rev, wgcu, fold, part_end);
  }
}

// Timer names: a whole-grid launch is "<name>"; the two launches of a split apply (interior
// planes, then the boundary planes after the halo exchange) are "<name>_interior" and
// "<name>_boundary", and the caller times the apply as a whole under "<name>" (pb_solver.cpp),
// so "<name>" always averages complete applies over all owned planes.
static const char* timer_name(int mode, const char* all, const char* interior,
                              const char* boundary) {
  return mode == PLANES_ALL ? all : (mode == PLANES_INTERIOR ? interior : boundary);
}

int launch_star7_apply(pb_grid* g, const Star& s, const double* x, double* y,
                       const StencilPlanes& gp, int mode) {
  ScopedTimer tm(g->ctx, timer_name(mode, "stencil", "stencil_interior", "stencil_boundary"));
  // alternate the march direction between applies (the boundary launch of a split apply is one
  // plane per chunk, direction-free, and does not flip it)
  const int rev = g->ctx->zflip;
  if (mode != PLANES_BOUNDARY) g->ctx->zflip ^= 1;
  return launch_any(g, s, PlainLoad{x}, gp, StoreY{y}, g->ctx->op_skip, mode, 0, nullptr, rev,
                    tune("stencil_wgcu", 0));
}

// ---------------------------------------------------------------------------------------------
// Red-black SOR smoothing and the multigrid residual on the engine (pb_mg.hip; oracle
// pbo_mg_apply). PETSc PCSOR update form x = (1 - w) x + w (b - sum_nb c x_nb) / c_centre,
// neighbour sum in the order z-, y-, x-, x+, y+, z+. A half-sweep updates the points with
// (i + j + k_global) % 2 == color in place: their neighbours all carry the other colour, which
// the half-sweep does not modify, so halo rows read from other waves are the same whether or not
// those waves have stored their plane yet (the stored other-colour values are bit-identical).
// ---------------------------------------------------------------------------------------------
// the red values of the first half-sweep from x = 0: (1 - w) * 0 + w * ((b - 0) * (1 / c))
struct Red0Load {
  static constexpr int NR = 1;
  static constexpr bool GHOST_RAW = true;  // ghost planes are b's: transform them too
  const double* __restrict__ b;
  double icc, omega;  // icc = 1 / c (the SOR update multiplies by the inverted diagonal)
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ const double* src(int) const { return b; }
  __device__ __forceinline__ double value(const double* raw) const {
    const double t = (raw[0] - 0.0) * icc;
    return (1.0 - omega) * 0.0 + omega * t;
  }
};

// SUMS: the last half-sweep of a preconditioner apply inside CG also takes the residual sums of
// its output z against r = b (t = z - mu_old: sum t, t^2, t.r, r -- cg_pc_sums_kernel's)
template <bool SUMS>
struct SorHalfT {
  static constexpr int NS = SUMS ? 4 : 0, NE = 1;
  static constexpr bool PREFETCH = true, RAW = true;
  static constexpr int WGCU = 1;  // (the zero-start sweep overrides: 3)
  double* x;
  const double* __restrict__ b;
  double cx, cy, cz, icc, omega;  // icc = 1 / c
  int color;  // points with (i + j + k_global) % 2 == color are updated
  int first;  // 1: black half-sweep after the zero-start red one (x_old = 0, field = Red0Load)
  const CgState* st;
  double mu;
  __device__ __forceinline__ void prepare();
  __device__ __forceinline__ const double* src(int) const { return b; }
  template <int V>
  __device__ __forceinline__ void put_raw(RowIx idx, int par, const double (&zm)[V],
                                          const double (&ym)[V], const double (&xm)[V],
                                          const double (&c)[V], const double (&xp)[V],
                                          const double (&yp)[V], const double (&zp)[V],
                                          const double (&op)[1][V], double* acc, int nt) const {
    double o[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      double nb = cz * zm[e];
      nb = nb + cy * ym[e];
      nb = nb + cx * xm[e];
      nb = nb + cx * xp[e];
      nb = nb + cy * yp[e];
      nb = nb + cz * zp[e];
      const double t = (op[0][e] - nb) * icc;
      const double xo = first ? 0.0 : c[e];
      const double xn = (1.0 - omega) * xo + omega * t;
      o[e] = ((par + e) & 1) == color ? xn : c[e];
      if constexpr (SUMS) {
        const double rv = op[0][e];
        const double t2 = o[e] - mu;
        acc[0] += t2;
        acc[1] += t2 * t2;
        acc[2] += t2 * rv;
        acc[3] += rv;
      }
    }
    store_row<V>(x, idx, o, nt);
    (void)acc;
  }
};
typedef SorHalfT<false> SorHalf;

// res = b - A x (the reference operator's summation order)
struct ResidEpi {
  static constexpr int NS = 0, NE = 1;
  static constexpr bool PREFETCH = true, RAW = false;
  static constexpr int WGCU = 1;
  double* __restrict__ res;
  const double* __restrict__ b;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ const double* src(int) const { return b; }
  template <int V>
  __device__ __forceinline__ void put(RowIx idx, const double (&c)[V], const double (&w)[V],
                                      double (&op)[1][V], double*, int nt) const {
    double o[V];
#pragma unroll
    for (int e = 0; e < V; ++e) o[e] = op[0][e] - w[e];
    store_row<V>(res, idx, o, nt);
    (void)c;
  }
};

int launch_mg_sor(pb_grid* g, const Star& s, double* x, const double* b, const StencilPlanes& gp,
                  double omega, int color, int first, const int* skip, const CgState* sums_st,
                  int* nparts) {
  ScopedTimer tm(g->ctx, "mg_sor");
  if (sums_st) {  // partial sums -> ctx->d_partials[0 .. nparts*4)
    SorHalfT<true> ep{x, b, s.cx, s.cy, s.cz, 1.0 / s.cc, omega, color, 0, sums_st, 0.0};
    return launch_any(g, s, PlainLoad{x}, gp, ep, skip, PLANES_ALL, 0, nparts);
  }
  SorHalf ep{x, b, s.cx, s.cy, s.cz, 1.0 / s.cc, omega, first ? 1 : color, first, nullptr, 0.0};
  if (first)  // measured: the zero-start sweep prefers 3 workgroups per CU, the others 1
    return launch_any(g, s, Red0Load{b, 1.0 / s.cc, omega}, gp, ep, skip, PLANES_ALL, 0, nullptr, 0, 3);
  return launch_any(g, s, PlainLoad{x}, gp, ep, skip);
}

int launch_mg_residual(pb_grid* g, const Star& s, const double* x, const double* b,
                       const StencilPlanes& gp, double* res, const int* skip) {
  ScopedTimer tm(g->ctx, "mg_residual");
  return launch_any(g, s, PlainLoad{x}, gp, ResidEpi{res, b}, skip);
}

// ---------------------------------------------------------------------------------------------
// CG (PETSc KSPSolve_CG + PCJacobi + MatNullSpace), device-resident state
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double cg_bb(const CgState* st) {
  return st->it == 0 ? 0.0 : st->beta / st->betaold;
}

template <bool SUMS>
__device__ __forceinline__ void SorHalfT<SUMS>::prepare() {
  if constexpr (SUMS) mu = st->mu;
}


// r = b, x = 0, p = 0 and the sums of s = dinv*r (t = s - 0)
__global__ __launch_bounds__(256) void cg_init_kernel(const double* __restrict__ b,
                                                      double* __restrict__ x,
                                                      double* __restrict__ r,
                                                      double* __restrict__ p, int64_t n,
                                                      double dinv, double* parts) {
  double acc[4] = {0, 0, 0, 0};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double rv = b[i];
    r[i] = rv;
    x[i] = 0.0;
    p[i] = 0.0;
    double s = dinv * rv;
    acc[0] += s;
    acc[1] += s * s;
    acc[2] += s * rv;
    acc[3] += rv;
  }
  block_partials<4>(acc, parts);
}

// boundary planes of p_new (for the halo exchange / periodic self-wrap)
// fold.stage = 2 (split grids): every wave first runs the previous iteration's stage 2 from the
// allreduced sums (a one-block partial) and the lead lane stores the state (fold.out)
__global__ __launch_bounds__(256) void cg_boundary_kernel(const double* __restrict__ r,
                                                          const double* __restrict__ p,
                                                          int64_t plane, int64_t last_off,
                                                          double* __restrict__ lo,
                                                          double* __restrict__ hi,
                                                          const CgState* st, Fold fold) {
  // the first PER points of both planes are loaded before the state (prologue) is ready: the
  // loads do not depend on it, so their latency hides the prologue's (r05: 23.7 -> 13.3 us with
  // one block per CU alone, at 512^2)
  constexpr int PER = 4;
  const int64_t gs = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double vr[2][PER], vp[2][PER];
  auto fetch = [&](int64_t base) {
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int64_t i = min(base + q * gs, plane - 1);  // (clamped: valid address, unused)
      vr[0][q] = r[i];
      vp[0][q] = p[i];
      vr[1][q] = r[last_off + i];
      vp[1][q] = p[last_off + i];
    }
  };
  fetch(i0);
  CgState sst;
  if (fold.stage) {
    fold_prologue(fold, sst);
    st = &sst;
  }
  if (st->done) return;
  CombineLoad c{r, p, nullptr, 0.0, 0.0, 0.0};
  c.prepare_from(*st);
  for (int64_t base = i0; base < plane; base += PER * gs) {
    if (base != i0) fetch(base);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int64_t i = base + q * gs;
      if (i < plane) {
        lo[i] = c.f(vr[0][q], vp[0][q]);
        hi[i] = c.f(vr[1][q], vp[1][q]);
      }
    }
  }
}


// Finalize: deterministic fixed-order reduction of the per-block partials, then the PETSc CG
// scalar logic (KSPSolve_CG + KSPConvergedDefault) on the device. mode bit 1 = reduce partials
// into sums[], bit 2 = update the state from sums[] (split around the RCCL allreduce).
// stage 0 = after init, 1 = after pass A (p.w), 2 = after pass B (residual sums), 3 = delta only.
__global__ __launch_bounds__(256) void cg_finalize_kernel(const double* __restrict__ parts,
                                                          int nparts, int width, double* sums,
                                                          int mode, int stage, CgState* st,
                                                          double* hist, int* h_done,
                                                          int64_t host_iter) {
  double S[kMaxSums];
  if ((mode & 1) && nparts > kFoldMaxParts) {
    // many partials (elementwise / multigrid kernels): 256-thread fixed-order tree
    __shared__ double red[256][kMaxSums];
    for (int s = 0; s < width; ++s) {
      double v = 0.0;
      for (int b = threadIdx.x; b < nparts; b += 256) v += parts[(int64_t)b * width + s];
      red[threadIdx.x][s] = v;
    }
    __syncthreads();
    for (int off = 128; off >= 1; off >>= 1) {
      if ((int)threadIdx.x < off)
        for (int s = 0; s < width; ++s) red[threadIdx.x][s] += red[threadIdx.x + off][s];
      __syncthreads();
    }
    if (threadIdx.x == 0)
      for (int s = 0; s < width; ++s) sums[s] = red[0][s];
  } else if (mode & 1) {
    // up to kFoldMaxParts: one wave, the folded prologues' order (folded == unfolded bits)
    if (threadIdx.x >= 64) return;
    wave_reduce_parts(parts, nparts, width, S);
    if (threadIdx.x == 0)
      for (int s = 0; s < width; ++s) sums[s] = S[s];
  }
  if (!(mode & 2) || threadIdx.x != 0) return;
  for (int s = 0; s < kMaxSums; ++s) S[s] = s < width ? sums[s] : 0.0;
  if (stage == 0) cg_stage0(*st, S, hist, h_done);
  else if (stage == 1) cg_stage1(*st, S[0]);
  else if (stage == 2) cg_stage2(*st, S, hist, h_done, host_iter);
  else st->delta = S[4];  // 3: the single-reduction setup's delta = z0'A z0
}


static int cg_reduce_update(pb_ctx* ctx, int stage, int nparts, int width, CgState* st,
                            double* hist, int* h_done, int64_t host_iter,
                            const double* parts = nullptr) {
  double* sums = ctx->d_scalars;
  if (!parts) parts = ctx->d_partials;
  if (!ctx->split) {
    hipLaunchKernelGGL(cg_finalize_kernel, dim3(1), dim3(256), 0, ctx->stream, parts,
                       nparts, width, sums, 3, stage, st, hist, h_done, host_iter);
    PB_HIP(hipGetLastError());
    return PB_OK;
  }
  hipLaunchKernelGGL(cg_finalize_kernel, dim3(1), dim3(256), 0, ctx->stream, parts,
                     nparts, width, sums, 1, stage, st, hist, h_done, host_iter);
  PB_HIP(hipGetLastError());
  PB_TRY(allreduce_device(ctx, sums, width));
  hipLaunchKernelGGL(cg_finalize_kernel, dim3(1), dim3(256), 0, ctx->stream, parts,
                     nparts, width, sums, 2, stage, st, hist, h_done, host_iter);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

static int elementwise_blocks(pb_ctx* ctx, int64_t n) {
  int64_t b = (n + 255) / 256;
  int64_t cap = (int64_t)ctx->num_cus * 8;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

int launch_cg_init(pb_grid* g, const double* b, double* x, double* r, double* p, CgState* st,
                   double dinv, double* hist, int* h_done) {
  pb_ctx* ctx = g->ctx;
  ScopedTimer tm(ctx, "cg_init");
  const int nb = elementwise_blocks(ctx, g->nlocal);
  hipLaunchKernelGGL(cg_init_kernel, dim3(nb), dim3(256), 0, ctx->stream, b, x, r, p, g->nlocal,
                     dinv, ctx->d_partials);
  PB_HIP(hipGetLastError());
  return cg_reduce_update(ctx, 0, nb, 4, st, hist, h_done, -1);
}

int launch_cg_boundary(pb_grid* g, const double* r, const double* p_old, CgState* st,
                       const Fold& fold, hipStream_t stream) {
  pb_ctx* ctx = g->ctx;
  hipStream_t sm = stream ? stream : ctx->stream;
  hipEvent_t tev = nullptr;
  const bool timed = ctx->timing && timer_wanted(ctx, "cg_boundary");
  if (timed) timer_begin(ctx, "cg_boundary", &tev, sm);
  // one block per CU at most, four points of each plane per thread (every wave of the folded
  // form runs the stage-2 prologue first)
  const int nb = (int)std::max<int64_t>(
      1, std::min<int64_t>(ctx->num_cus, (g->plane + 256 * 4 - 1) / (256 * 4)));
  hipLaunchKernelGGL(cg_boundary_kernel, dim3(nb), dim3(256), 0, sm, r, p_old, g->plane,
                     (g->nzl - 1) * g->plane, g->bnd_lo, g->bnd_hi, (const CgState*)st, fold);
  PB_HIP(hipGetLastError());
  if (timed) timer_end(ctx, "cg_boundary", tev, sm);
  return PB_OK;
}

int launch_cg_boundary(pb_grid* g, const double* r, const double* p_old, CgState* st) {
  return launch_cg_boundary(g, r, p_old, st, Fold{});
}

int launch_cg_pass_a(pb_grid* g, const Star& s, const double* r, const double* p_old,
                     double* p_new, const StencilPlanes& gp, CgState* st, int mode, int part_off,
                     int* nblocks, bool store) {
  ScopedTimer tm(g->ctx,
                 timer_name(mode, "cg_pass_a", "cg_pass_a_interior", "cg_pass_a_boundary"));
  const CombineLoad ld{r, p_old, st, 0.0, 0.0, 0.0};
  if (!store)
    return launch_any(g, s, ld, gp, PassAT<false>{p_new}, &st->done, mode, part_off, nblocks);
  return launch_any(g, s, ld, gp, PassA{p_new}, &st->done, mode, part_off, nblocks);
}

// Folded iteration (one rank, Jacobi): partial sums of pass A at block 0, of pass B at
// fold_parts_b_off(); state slots st2[0] (read by pass B, written by pass A) and st2[1].
static int64_t fold_parts_b_off(const pb_ctx* ctx) { return ctx->partials_cap / 8; }

int launch_cg_pass_a_folded(pb_grid* g, const Star& s, const double* r, const double* p_old,
                            double* p_new, const StencilPlanes& gp, CgState* st2, int nparts_b,
                            double* hist, int* h_done, int64_t host_iter, int* nblocks,
                            bool store) {
  ScopedTimer tm(g->ctx, "cg_pass_a");
  pb_ctx* ctx = g->ctx;
  Fold f;
  f.stage = 2;
  f.nparts = nparts_b;
  f.width = 4;
  f.parts = ctx->d_partials + fold_parts_b_off(ctx) * 4;
  f.in = st2 + 1;
  f.out = st2;
  f.hist = hist;
  f.h_done = h_done;
  f.host_iter = host_iter - 1;  // stage 2 of the previous iteration
  const CombineLoad ld{r, p_old, nullptr, 0.0, 0.0, 0.0};
  if (!store)
    return launch_any(g, s, ld, gp, PassAT<false>{p_new}, nullptr, PLANES_ALL, 0, nblocks, 0,
                      0, f);
  return launch_any(g, s, ld, gp, PassA{p_new}, nullptr, PLANES_ALL, 0, nblocks, 0, 0, f);
}

int launch_cg_pass_a_fold(pb_grid* g, const Star& s, const double* r, const double* p_old,
                          double* p_new, const StencilPlanes& gp, const Fold& fold, int mode,
                          int part_off, int* nblocks, bool store) {
  ScopedTimer tm(g->ctx,
                 timer_name(mode, "cg_pass_a", "cg_pass_a_interior", "cg_pass_a_boundary"));
  const CombineLoad ld{r, p_old, nullptr, 0.0, 0.0, 0.0};
  if (!store)
    return launch_any(g, s, ld, gp, PassAT<false>{p_new}, nullptr, mode, part_off, nblocks, 0, 0,
                      fold);
  return launch_any(g, s, ld, gp, PassA{p_new}, nullptr, mode, part_off, nblocks, 0, 0, fold);
}

// split grids, folded iteration: reduce a pass's partials and allreduce them into d_scalars, where
// the next kernel's prologue reads them as a one-block partial (pass A's -> pass B; pass B's ->
// the next boundary-plane kernel); b_region: pass B's partials (fold_parts_b_off)
int cg_reduce_allreduce(pb_ctx* ctx, int nparts, int width, bool b_region) {
  return cg_reduce_allreduce(ctx, ctx->d_partials + (b_region ? fold_parts_b_off(ctx) * 4 : 0),
                             nparts, width);
}

int cg_reduce_allreduce(pb_ctx* ctx, const double* parts, int nparts, int width) {
  hipLaunchKernelGGL(cg_finalize_kernel, dim3(1), dim3(256), 0, ctx->stream, parts, nparts, width,
                     ctx->d_scalars, 1, 0, (CgState*)nullptr, (double*)nullptr, (int*)nullptr,
                     (int64_t)0);
  PB_HIP(hipGetLastError());
  return allreduce_device(ctx, ctx->d_scalars, width);
}

// the residual-sum stage (2) on st in place from sums already allreduced into d_scalars
int cg_stage2_from_sums(pb_ctx* ctx, int width, CgState* st, double* hist, int* h_done,
                        int64_t host_iter) {
  hipLaunchKernelGGL(cg_finalize_kernel, dim3(1), dim3(256), 0, ctx->stream,
                     (const double*)nullptr, 0, width, ctx->d_scalars, 2, 2, st, hist, h_done,
                     host_iter);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

int cg_finalize_init(pb_ctx* ctx, int nparts, CgState* st, double* hist, int* h_done) {
  return cg_reduce_update(ctx, 0, nparts, 4, st, hist, h_done, -1);
}

int cg_finalize_pass_a(pb_ctx* ctx, int nparts, CgState* st) {
  return cg_reduce_update(ctx, 1, nparts, 1, st, nullptr, nullptr, 0);
}

int cg_finalize_stage2(pb_ctx* ctx, int nparts, CgState* st, double* hist, int* h_done,
                       int64_t host_iter) {
  return cg_reduce_update(ctx, 2, nparts, 4, st, hist, h_done, host_iter);
}

// pass B variants by the x-update position; fold.stage = 1: stage 1 in the prologue (partials
// of pass A at block 0, state st2[0] -> st2[1]) and the partials written at fold_parts_b_off().
// ps.r_out != nullptr (PB_CG_PSTORE_B): pass B re-forms p = CombineLoad(ps.zsrc, p_old) on load,
// stores it to p, reads r and writes the new residual to ps.r_out.
template <int XU, bool PST>
static int pass_b_one(pb_grid* g, const Star& s, const double* p, const double* const* p_prev,
                      double* x, double* r, const StencilPlanes& gp, CgState* st, const Fold& f,
                      const PStore& ps, int* nparts) {
  const int* skip = f.stage ? nullptr : &st->done;
  const int off = f.stage ? (int)fold_parts_b_off(g->ctx) : 0;
  PassB<XU, PST> ep{x, r, p_prev[0], XU == 3 ? p_prev[1] : nullptr, XU == 3 ? p_prev[2] : nullptr,
                    st, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  if constexpr (PST) {
    ep.r_out = ps.r_out;
    ep.p_out = const_cast<double*>(p);
    CombineLoad ld{ps.zsrc, p_prev[0], st, 0.0, 0.0, 0.0};
    ld.after1 = 1;
    return launch_any(g, s, ld, gp, ep, skip, PLANES_ALL, off, nparts, 1, 0, f);
  } else {
    return launch_any(g, s, PlainLoad{p}, gp, ep, skip, PLANES_ALL, off, nparts, 1, 0, f);
  }
}

template <bool PST>
static int pass_b_pick(pb_grid* g, const Star& s, const double* p, const double* const* p_prev,
                       double* x, double* r, const StencilPlanes& gp, CgState* st,
                       int64_t host_iter, int defer, const Fold& f, const PStore& ps, int* nparts) {
  if (defer == 0) {
    ScopedTimer tm(g->ctx, "cg_pass_b");
    return pass_b_one<2, PST>(g, s, p, p_prev, x, r, gp, st, f, ps, nparts);
  }
  if (host_iter % defer != defer - 1) {
    ScopedTimer tm(g->ctx, "cg_pass_b_even");
    return pass_b_one<0, PST>(g, s, p, p_prev, x, r, gp, st, f, ps, nparts);
  }
  if (defer == 2) {
    ScopedTimer tm(g->ctx, "cg_pass_b_odd");
    return pass_b_one<1, PST>(g, s, p, p_prev, x, r, gp, st, f, ps, nparts);
  }
  ScopedTimer tm(g->ctx, "cg_pass_b_x4");
  return pass_b_one<3, PST>(g, s, p, p_prev, x, r, gp, st, f, ps, nparts);
}

static int pass_b_launch(pb_grid* g, const Star& s, const double* p, const double* const* p_prev,
                         double* x, double* r, const StencilPlanes& gp, CgState* st,
                         int64_t host_iter, int defer, const Fold& f, const PStore& ps,
                         int* nparts) {
  if (ps.r_out)
    return pass_b_pick<true>(g, s, p, p_prev, x, r, gp, st, host_iter, defer, f, ps, nparts);
  return pass_b_pick<false>(g, s, p, p_prev, x, r, gp, st, host_iter, defer, f, ps, nparts);
}

int launch_cg_pass_b(pb_grid* g, const Star& s, const double* p, const double* const* p_prev,
                     double* x, double* r, const StencilPlanes& gp, CgState* st, double* hist,
                     int* h_done, int64_t host_iter, int defer, bool finalize, const PStore& ps) {
  int nparts = 0;
  PB_TRY(pass_b_launch(g, s, p, p_prev, x, r, gp, st, host_iter, defer, Fold{}, ps, &nparts));
  if (!finalize) return PB_OK;  // preconditioned path: the sums come from z = M^-1 r later
  return cg_reduce_update(g->ctx, 2, nparts, 4, st, hist, h_done, host_iter);
}

int launch_cg_pass_b_folded(pb_grid* g, const Star& s, const double* p,
                            const double* const* p_prev, double* x, double* r,
                            const StencilPlanes& gp, CgState* st2, int nparts_a, int64_t host_iter,
                            int defer, int* nparts_b, const PStore& ps, const double* parts_a) {
  Fold f;
  f.stage = 1;
  f.nparts = nparts_a;
  f.width = 1;
  f.parts = parts_a ? parts_a : g->ctx->d_partials;
  f.in = st2;
  f.out = st2 + 1;
  return pass_b_launch(g, s, p, p_prev, x, r, gp, nullptr, host_iter, defer, f, ps, nparts_b);
}

// after the last folded iteration of a pb_ksp_iterate call: its stage 2 (in place on st2[1]),
// then st2[0] = st2[1], so the unfolded entry points find the complete state in slot 0
int cg_fold_tail(pb_ctx* ctx, int nparts_b, CgState* st2, double* hist, int* h_done,
                 int64_t host_iter) {
  // split grids: pass B's sums are already reduced and allreduced into d_scalars (mode 2 only)
  hipLaunchKernelGGL(cg_finalize_kernel, dim3(1), dim3(256), 0, ctx->stream,
                     ctx->d_partials + fold_parts_b_off(ctx) * 4, nparts_b, 4, ctx->d_scalars,
                     ctx->split ? 2 : 3, 2, st2 + 1, hist, h_done, host_iter);
  PB_HIP(hipGetLastError());
  PB_HIP(hipMemcpyAsync(st2, st2 + 1, sizeof(CgState), hipMemcpyDeviceToDevice, ctx->stream));
  return PB_OK;
}

// ---------------------------------------------------------------------------------------------
// Single-reduction CG (-ksp_cg_single_reduction): pass P (p, r' and the deferred x update; no
// sums) and pass S (t = dinv r' - mu, s = A t, five sums). 32 + 8 B/DoF per iteration (+ the x
// update's 32 every fourth), one reduction -- against 16 + 32 and two for the KSPSolve_CG passes.
// ---------------------------------------------------------------------------------------------
template <int XU>
static int sr_pass_p_one(pb_grid* g, const Star& s, const double* r, const double* const* p_prev,
                         double* p_new, double* x, double* r_out, const StencilPlanes& gp,
                         const Fold& f, int mode) {
  PassB<XU, true, false> ep{x, nullptr, p_prev[0], XU == 3 ? p_prev[1] : nullptr,
                            XU == 3 ? p_prev[2] : nullptr, nullptr, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  ep.r_out = r_out;
  ep.p_out = p_new;
  CombineLoad ld{r, p_prev[0], nullptr, 0.0, 0.0, 0.0};
  ld.after1 = 1;  // b = beta / betaold as the prologue's top found it (bbp)
  return launch_any(g, s, ld, gp, ep, nullptr, mode, 0, nullptr, 1, 0, f);
}

int launch_cg_sr_pass_p(pb_grid* g, const Star& s, const double* r, const double* const* p_prev,
                        double* p_new, double* x, double* r_out, const StencilPlanes& gp,
                        const SrFold& sf, int mode, int64_t host_iter, int defer) {
  Fold f;
  f.stage = sf.fold_sums ? 3 : 4;
  f.nparts = sf.nparts_s;
  f.width = 5;
  f.parts = sf.parts ? sf.parts : g->ctx->d_partials;
  f.in = sf.in;
  f.out = sf.out;
  f.hist = sf.hist;
  f.h_done = sf.h_done;
  f.host_iter = host_iter - 1;  // the residual-sum stage of the previous iteration
  if (defer == 4 && host_iter % 4 == 3) {
    ScopedTimer tm(g->ctx, timer_name(mode, "cg_sr_p_x4", "cg_sr_p_x4_interior", "cg_sr_p_x4_boundary"));
    return sr_pass_p_one<3>(g, s, r, p_prev, p_new, x, r_out, gp, f, mode);
  }
  if (defer == 4) {
    ScopedTimer tm(g->ctx, timer_name(mode, "cg_sr_p", "cg_sr_p_interior", "cg_sr_p_boundary"));
    return sr_pass_p_one<0>(g, s, r, p_prev, p_new, x, r_out, gp, f, mode);
  }
  if (defer == 2 && host_iter % 2 == 1) {
    ScopedTimer tm(g->ctx, timer_name(mode, "cg_sr_p_x2", "cg_sr_p_x2_interior", "cg_sr_p_x2_boundary"));
    return sr_pass_p_one<1>(g, s, r, p_prev, p_new, x, r_out, gp, f, mode);
  }
  if (defer == 2) {
    ScopedTimer tm(g->ctx, timer_name(mode, "cg_sr_p", "cg_sr_p_interior", "cg_sr_p_boundary"));
    return sr_pass_p_one<0>(g, s, r, p_prev, p_new, x, r_out, gp, f, mode);
  }
  ScopedTimer tm(g->ctx, timer_name(mode, "cg_sr_p_x1", "cg_sr_p_x1_interior", "cg_sr_p_x1_boundary"));
  return sr_pass_p_one<2>(g, s, r, p_prev, p_new, x, r_out, gp, f, mode);
}

int launch_cg_sr_pass_s(pb_grid* g, const Star& s, const double* r, const StencilPlanes& gp,
                        const CgState* st, int mode, int part_off, int part_end, int* nblocks) {
  ScopedTimer tm(g->ctx, timer_name(mode, "cg_sr_s", "cg_sr_s_interior", "cg_sr_s_boundary"));
  // (marches upwards after pass P marched downwards: it starts on the planes P wrote last)
  // 4-row tiles, two workgroups per CU (a single read-only stream: 0.218-0.221 ms at 512^3 against
  // 0.247 with one per CU, 0.223-0.228 with three, 0.224 with 8-row tiles; gpurun_out sr2/sr3)
  return launch_any(g, s, ZLoad{r, st}, gp, SrSums{}, &st->done, mode, part_off, nblocks, 0, 2,
                    Fold{}, part_end);
}

int cg_sr_finalize(pb_ctx* ctx, const double* parts, int nparts, CgState* st, double* hist,
                   int* h_done, int64_t host_iter, bool stage_delta0) {
  return cg_reduce_update(ctx, stage_delta0 ? 3 : 2, nparts, 5, st, hist, h_done, host_iter,
                          parts);
}

// x += alpha * p (the pending half of the deferred solution update)
__global__ __launch_bounds__(256) void cg_flush_kernel(double* __restrict__ x,
                                                       const double* __restrict__ p, int64_t n,
                                                       double alpha) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    x[i] = x[i] + alpha * p[i];
}

int launch_cg_flush(pb_grid* g, double* x, const double* p, double alpha) {
  const int nb = elementwise_blocks(g->ctx, g->nlocal);
  hipLaunchKernelGGL(cg_flush_kernel, dim3(nb), dim3(256), 0, g->ctx->stream, x, p, g->nlocal, alpha);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

}  // namespace pb
