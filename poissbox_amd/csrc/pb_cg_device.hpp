// pb_cg_device.hpp -- device-side CG scalar logic shared by the stencil engine's fused passes
// (pb_stencil.hip) and the single-reduction one-pass kernel (pb_cg_sr.hip): PETSc KSPSolve_CG /
// KSPSolve_CG_SingleReduction stages on a register copy of CgState, the fixed-order reduction of
// per-block partial sums, and the finalize folded into a pass prologue (Fold).
#pragma once

#include <type_traits>
#include <utility>
#include "pb_device.hpp"

namespace pb {

// ---------------------------------------------------------------------------------------------
// CG scalar logic (PETSc KSPSolve_CG + KSPConvergedDefault), shared by the finalize kernel and
// the folded pass prologues
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool finite(double v) { return v == v && v - v == 0.0; }
// ||z|| from the shifted sum of squares: a rounding-negative sum clamps to 0, a NaN stays NaN (so
// the norm test below reports DIVERGED_NANORINF like PETSc's KSPCheckNorm; a clamp written as
// zz > 0 ? zz : 0 turned a NaN into CONVERGED_ATOL)
__device__ __forceinline__ double norm_from_sq(double zz) { return sqrt(zz < 0.0 ? 0.0 : zz); }
// timing-only ablation builds (wrong results): every exit but the iteration limit is ignored
template <class S>
__device__ __forceinline__ void ablate_keep_going(S& st) {
#ifdef PB_ABLATE_NO_EXITS
  if (st.reason != PB_KSP_DIVERGED_ITS) st.reason = 0, st.done = 0;
#endif
}

// partial counts up to which the finalize kernel reduces with one wave in this order (the CG
// passes: one workgroup per CU); beyond it, a 256-thread tree (a lone wave took 29 us over the
// 2048 partials of the elementwise kernels of the preconditioned CG)
static constexpr int kFoldMaxParts = 1024;
static constexpr int kMaxSums = 5;  // partial sums per block (single-reduction pass S: 5)
// fixed-order reduction of nparts x width partials by ONE wave: lane l sums blocks l, l+64, ...
// in order, then an xor butterfly (every lane ends with the same bits). Used by the finalize
// kernel (wave 0) and by every wave of a folded pass prologue, so both paths round alike.
__device__ __forceinline__ void wave_reduce_parts(const double* __restrict__ parts, int nparts,
                                                  int width, double* S) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < kMaxSums; ++s) {
    double v = 0.0;
    if (s < width)
      for (int b = lane; b < nparts; b += 64) v += parts[(int64_t)b * width + s];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    S[s] = v;
  }
}

// stage 0 (after init / the first PC apply): S = (sum t, sum t^2, sum t.r, sum r)
__device__ __forceinline__ void cg_stage0(CgState& st, const double* S, double* hist,
                                          int* h_done) {
  const double N = st.ntot;
  double mu = 0.0, zz = S[1], zr = S[2];
  if (st.nullspace) {
    const double delta = S[0] / N;
    mu = delta;
    zz = S[1] - N * delta * delta;
    zr = S[2] - delta * S[3];
  }
  const double dp = norm_from_sq(zz);
  st.mu = mu;
  st.dp = dp;
  st.rnorm0 = dp;
  st.it = 0;
  st.its = 0;
  st.dpi = 0.0;
  st.alpha = 0.0;
  st.alpha_prev = 0.0;
  st.pend_iter = -1;
  st.pend_count = 0;
  st.reason = 0;
  st.done = 0;
  if (st.nhist > 0 && hist) hist[0] = dp;
  st.nlog = st.nhist > 0 ? 1 : 0;
  if (!finite(dp)) {
    st.reason = PB_KSP_DIVERGED_NANORINF;
    st.done = 1;
  } else {
    st.ttol = fmax(st.rtol * dp, st.atol);
    if (dp <= st.ttol) {
      st.reason = dp < st.atol ? PB_KSP_CONVERGED_ATOL : PB_KSP_CONVERGED_RTOL;
      st.done = 1;
    } else {
      st.beta = zr;
      if (!finite(zr)) {
        st.reason = PB_KSP_DIVERGED_NANORINF;
        st.done = 1;
      } else if (zr == 0.0) {
        st.its = 1;
        st.reason = PB_KSP_CONVERGED_ATOL;
        st.done = 1;
      } else if (st.max_it <= 0) {
        st.reason = PB_KSP_DIVERGED_ITS;
        st.done = 1;
      }
    }
  }
  if (h_done) h_done[0] = st.done;
}

// stage 1 (after pass A): dpi = p.w -> alpha, or an INDEFINITE_MAT / NaN exit. check_dot:
// KSPSolve_CG's KSPCheckDot on p.w; PETSc's single-reduction iteration checks only beta, so a
// non-finite recurrence dpi runs one more pass and ends at the next norm test (oracle alike)
__device__ __forceinline__ void cg_stage1(CgState& st, double dpi, bool check_dot = true) {
  if (st.done) return;
  const int64_t i = st.it;
  const double sp = (double)((dpi > 0) - (dpi < 0)), so = (double)((st.dpi > 0) - (st.dpi < 0));
  if (check_dot && !finite(dpi)) {
    st.its = i + 1;
    st.reason = PB_KSP_DIVERGED_NANORINF;
    st.done = 1;
  } else if (dpi == 0.0 || (i > 0 && sp * so < 0.0)) {
    st.its = i + 1;
    st.reason = PB_KSP_DIVERGED_INDEFINITE_MAT;
    st.done = 1;
  } else {
    st.dpiold = st.dpi;
    st.dpi = dpi;
    st.bbp = i == 0 ? 0.0 : st.beta / st.betaold;  // CombineLoad's bb of this pass A
    st.betaold = st.beta;
    st.alpha_prev = st.alpha;
    st.alpha = st.beta / dpi;
  }
  ablate_keep_going(st);
}

// iterations i % D < D-1 leave alpha_i p_i pending in x; the last of each D applied them all
// (PassB<XU>)
__device__ __forceinline__ void cg_pend(CgState& st) {
  const int64_t i = st.it;
  const int D = st.defer_x;
  const int m = D > 0 ? (int)(i % D) : 0;
  if (D > 0 && m < D - 1) {
    // (value selects, no computed index: st may be a register copy)
    st.pa[0] = m == 0 ? st.alpha : st.pa[0];
    st.pa[1] = m == 1 ? st.alpha : st.pa[1];
    st.pa[2] = m == 2 ? st.alpha : st.pa[2];
    st.pend_iter = i - m;
    st.pend_count = m + 1;
  } else {
    st.pend_iter = -1;
    st.pend_count = 0;
  }
}

// stage 2 (after pass B / the PC apply): residual sums -> norm, convergence tests, next beta
__device__ __forceinline__ void cg_stage2(CgState& st, const double* S, double* hist, int* h_done,
                                          int64_t host_iter) {
  if (!st.done) {
    const double N = st.ntot;
    const int64_t i = st.it;
    double mu = st.mu, zz = S[1], zr = S[2];
    if (st.nullspace) {
      const double delta = S[0] / N;
      mu = st.mu + delta;
      zz = S[1] - N * delta * delta;
      zr = S[2] - delta * S[3];
    }
    const double dp = norm_from_sq(zz);
    // (single reduction: alpha_i was booked by cg_sr_top, before pass P applied it)
    if (!st.sr) cg_pend(st);
    st.dp = dp;
    st.its = i + 1;
    if (i + 1 < st.nhist) {
      if (hist) hist[i + 1] = dp;
      st.nlog = i + 2;
    }
    if (!finite(dp)) {
      st.reason = PB_KSP_DIVERGED_NANORINF;
      st.done = 1;
    } else if (dp <= st.ttol) {
      st.reason = dp < st.atol ? PB_KSP_CONVERGED_ATOL : PB_KSP_CONVERGED_RTOL;
      st.done = 1;
    } else if (dp >= st.dtol * st.rnorm0) {
      st.reason = PB_KSP_DIVERGED_DTOL;
      st.done = 1;
    } else {
      st.beta = zr;
      st.mu = mu;
      st.delta = S[4];  // (single reduction: z'A z, read by the next cg_sr_top)
      st.it = i + 1;
      if (!finite(zr)) {
        st.reason = PB_KSP_DIVERGED_NANORINF;
        st.done = 1;
      } else if (st.it >= st.max_it) {
        st.reason = PB_KSP_DIVERGED_ITS;
        st.done = 1;
      } else if (zr == 0.0) {
        st.its = st.it + 1;
        st.reason = PB_KSP_CONVERGED_ATOL;
        st.done = 1;
      } else if (zr * st.betaold < 0.0) {
        // PETSc KSPSolve_CG, top of iteration i+1 (real scalars): beta*betaold < 0 -> the
        // preconditioner is indefinite (betaold = the beta iteration i used, stage 1)
        st.its = st.it + 1;
        st.reason = PB_KSP_DIVERGED_INDEFINITE_PC;
        st.done = 1;
      }
    }
  }
  ablate_keep_going(st);
  if (h_done) h_done[host_iter + 1] = st.done;
}

// Top of a single-reduction iteration (PETSc KSPSolve_CG_SingleReduction, real scalars): the
// beta checks ran with the residual-sum stage (cg_stage0 / cg_stage2, as in KSPSolve_CG); here
// p'w = delta (i = 0: p = z, w = A z) or delta - beta^2 dpiold / betaold^2, then stage 1's
// INDEFINITE_MAT / NaN exits and alpha, and alpha_i's deferred-x bookkeeping (pass P applies it)
__device__ __forceinline__ void cg_sr_top(CgState& st) {
  if (st.done) return;
  const double dpi = st.it == 0 ? st.delta
                                : st.delta - st.beta * st.beta * st.dpi / (st.betaold * st.betaold);
  cg_stage1(st, dpi, false);
  if (!st.done) cg_pend(st);
}

// ---------------------------------------------------------------------------------------------
// Finalize folded into the next pass's prologue (one rank, Jacobi CG): EVERY WAVE reduces the
// previous pass's partials in the finalize kernel's fixed order (lane-strided sums, xor
// butterfly: bit-identical in every lane) and runs the PETSc scalar step (stage 1 before pass B,
// stage 2 of the previous iteration before pass A) on a register copy of the state -- no LDS, no
// barrier; lane 0 of block 0 stores the result into the OTHER state slot, so the slot this launch
// reads is never written while it runs. Removes the two finalize launches (and their kernel
// boundaries) from every iteration.
// ---------------------------------------------------------------------------------------------
// (struct Fold: pb_internal.hpp)

// field-wise copy (an aggregate copy becomes a memcpy that pins the register copy in scratch)
__device__ __forceinline__ void cg_copy(CgState& d, const CgState& s) {
  d.beta = s.beta, d.betaold = s.betaold, d.dpi = s.dpi, d.dpiold = s.dpiold;
  d.alpha = s.alpha, d.alpha_prev = s.alpha_prev, d.mu = s.mu, d.dp = s.dp, d.ttol = s.ttol;
  d.rnorm0 = s.rnorm0, d.pa[0] = s.pa[0], d.pa[1] = s.pa[1], d.pa[2] = s.pa[2];
  d.rtol = s.rtol, d.atol = s.atol, d.dtol = s.dtol, d.dinv = s.dinv, d.ntot = s.ntot;
  d.it = s.it, d.its = s.its, d.max_it = s.max_it, d.nhist = s.nhist, d.pend_iter = s.pend_iter;
  d.pend_count = s.pend_count, d.nlog = s.nlog;
  d.reason = s.reason, d.done = s.done, d.pc = s.pc, d.nullspace = s.nullspace;
  d.defer_x = s.defer_x;
  d.bbp = s.bbp;
  d.delta = s.delta, d.sr = s.sr;
}
static_assert(sizeof(CgState) == 248, "cg_copy lists every CgState field");

__device__ __forceinline__ void fold_prologue(const Fold& f, CgState& st) {
  double S[kMaxSums];
  cg_copy(st, *f.in);
  // (garbage if done: the stages ignore it)
  if (f.stage != 4) wave_reduce_parts(f.parts, f.nparts, f.width, S);
  const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
  if (f.stage == 1) {
    cg_stage1(st, S[0]);
  } else if (f.stage == 2) {
    cg_stage2(st, S, lead ? f.hist : nullptr, lead ? f.h_done : nullptr, f.host_iter);
  } else {
    if (f.stage == 3)
      cg_stage2(st, S, lead ? f.hist : nullptr, lead ? f.h_done : nullptr, f.host_iter);
    cg_sr_top(st);
  }
  if (lead && f.out) cg_copy(*f.out, st);  // (out null: the state in registers only)
}

// ---------------------------------------------------------------------------------------------
// z-march helpers of the ring-buffered CG kernel (pb_cg_sr.hip)
// ---------------------------------------------------------------------------------------------
template <int... Qs, class F>
__device__ __forceinline__ void unroll_steps(std::integer_sequence<int, Qs...>, F&& f) {
  (f(std::integral_constant<int, Qs>{}), ...);
}

// one 7-point sum in the reference order (z-, y-, x-, c, x+, y+, z+)
__device__ __forceinline__ double star7_sum(double cx, double cy, double cz, double cc,
                                            double zm, double ym, double xm, double c, double xp,
                                            double yp, double zp) {
  double w = cz * zm;
  w = w + cy * ym;
  w = w + cx * xm;
  w = w + cc * c;
  w = w + cx * xp;
  w = w + cy * yp;
  w = w + cz * zp;
  return w;
}

// DPP moves of a double: row shifts by N lanes within 16-lane rows (N = 0: the value itself)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
template <int N>
__device__ __forceinline__ double dpp_row_shl(double v) {  // lane l <- lane l + N
  if constexpr (N == 0) return v;
  else return dpp_d<0x100 + N>(v);
}
template <int N>
__device__ __forceinline__ double dpp_row_shr(double v) {  // lane l <- lane l - N
  if constexpr (N == 0) return v;
  else return dpp_d<0x110 + N>(v);
}
// wave shifts by one lane that keep `old` where the source lane is outside the wave (lane 0 for
// shr, lane 63 for shl)
template <int CTRL>
__device__ __forceinline__ double dpp_keep(double old, double v) {
  const long long b = __builtin_bit_cast(long long, v), o = __builtin_bit_cast(long long, old);
  const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double dpp_shr1_keep(double old, double v) {  // lane l <- lane l-1
  return dpp_keep<0x138>(old, v);
}
__device__ __forceinline__ double dpp_shl1_keep(double old, double v) {  // lane l <- lane l+1
  return dpp_keep<0x130>(old, v);
}

}  // namespace pb
