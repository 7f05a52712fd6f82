// pb_fft.hip -- spectral preconditioner (-pc_type fft): z = P^+ r for the periodic
// constant-coefficient operators of this library, by separable discrete Hartley transforms.
//
// Every operator here is a sum of products of 1-D circulant operators with real, even symbols:
//   7-point star (src/coefficients.f90:22-48):   lambda = sum_d (2 cos t_d - 2) / h_d^2
//   compact lapl (src/compact_schemes.f90:17-37): lambda = Lx Jy Jz + Jx Ly Jz + Jx Jy Lz, with
//     J(t) = (I+ I-)(t) = 4 (a_i cos(t/2) + b_i cos(3t/2))^2 / (1 + 2 alpha_i cos t)^2
//     L(t) = (D+ D-)(t) = -4 (a_d sin(t/2) + b_d sin(3t/2))^2 / (1 + 2 alpha_d cos t)^2
//     (coefficients :188-190, :303-305; D+ = -D-^T, I+ = I-^T, so lambda is real and <= 0)
// A symbol even in each t_d separately is diagonalised by the separable real Hartley transform
// H = Hx Hy Hz (H_d: cas(2 pi j k / n_d) = cos + sin, H_d H_d = n_d I), so
//   P^+ = H diag(1 / (N lambda)) H,  1/lambda := 0 on the null modes (|lambda| <= 1e-10 max|lambda|:
//   the constants, and for the compact operator every mode with two or more Nyquist components --
//   the near-null modes that stall Jacobi- or 7-point-MG-preconditioned CG on config 5).
// CG with this PC converges in a handful of iterations on any grid size.
//
// Passes (5 line passes, 16 B/DoF each, in place after the first): X forward (r -> z), Y forward,
// Z forward * 1/(N lambda) * Z inverse (one kernel), Y inverse, X inverse. On a split grid the Z
// pass runs on y-slabs with complete z-lines (the compact operators' z-slab <-> y-slab transposes).
//
// Line kernel: a block loads a tile of TL lines into LDS (coalesced rows), each wave takes two
// real lines x, y and runs ONE complex FFT of z = x + i y of length n = 64*C: C-point DFTs in
// registers (lane owns elements lane + 64 m), twiddles, then a 64-point DFT across the lanes by six
// radix-2 decimation-in-frequency stages over wave shuffles (output in bit-reversed lane order);
// the two Hartley spectra follow from Z(k) and Z(-k) (one more shuffle), and go back to LDS in
// natural order for the coalesced store. Twiddles come from a per-axis table exp(-2 pi i k / n).
#include <algorithm>
#include <cmath>
#include <vector>

#include "pb_internal.hpp"
#include "pb_device.hpp"


#ifndef PB_FFT_TW_LAZY
#define PB_FFT_TW_LAZY 0
#endif
// loads / stores of a tile in flight per thread (#pragma unroll count of the tile copy loops)
#ifndef PB_FFT_TILE_UNROLL
#define PB_FFT_TILE_UNROLL 4
#endif
#define PB_FFT_STR(x) #x
#define PB_FFT_UNROLL(n) _Pragma(PB_FFT_STR(unroll n))
#ifndef PB_FFT_X_WAVE
#define PB_FFT_X_WAVE 1
#endif
#ifndef PB_FFT_SCALE_LDS
#define PB_FFT_SCALE_LDS 1
#endif

namespace pb {

namespace {

struct DhtPass {
  const double* in;   // tile source (X forward: r), else == out
  double* out;
  int64_t li, lo, es;  // element e of line (outer, inner) at outer*lo + inner*li + e*es
  int ninner, nouter, ntiles_inner;
  const double* w;    // twiddles of the line axis: (re, im) of exp(-2 pi i k / n), k < n
  const double* tab;  // [Lx | Jx | Ly | Jy | Lz | Jz] (SCALE only)
  int nx, ny, j0;     // global x / y sizes, global y of the box's row 0 (SCALE only)
  double scale, thr;  // 1 / (nx ny nz) and the null-mode threshold (SCALE only)
  int remap;          // XCD-aware tile order (PB_FFT_REMAP, default on): consecutive tiles share an
                      // XCD; Z pass 1.35-1.36 vs 1.375-1.378 ms at 512^3 (ab_remap_fft.jsonl)
  // CG's residual sums taken by the last pass (X inverse) as it writes z: t = z - mu, over the
  // tile, against r = sr -> parts[block * 4 + (t, t^2, t r, r)] (cg_pc_sums_kernel's sums)
  const double* sr;
  double* parts;
  const CgState* st;
  int nparts_out;     // (host) partial blocks written
};

struct cplx {
  double re, im;
};
__device__ __forceinline__ cplx cmul(cplx a, cplx b) {
  return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
__device__ __forceinline__ cplx tw(const double* w, int k) { return {w[2 * k], w[2 * k + 1]}; }

__host__ __device__ constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v >> 1); }
__host__ __device__ constexpr int bitrev(int v, int bits) {
  int r = 0;
  for (int b = 0; b < bits; ++b) r |= ((v >> b) & 1) << (bits - 1 - b);
  return r;
}

// ---- lane exchanges without LDS: value of lane ^ H (H = 1..32) and of lane ^ 63 ----
// H = 1, 2: DPP quad_perm; 4, 8: DPP row shifts up / down and a select; 16, 32: the gfx950
// permlane swaps. All VALU: no LDS round trip per FFT stage (the r02 first cut used
// __shfl_xor = ds_bpermute, twice per double).
template <int CTRL>
__device__ __forceinline__ int dpp32(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, true);  // bound_ctrl: no old operand
}
template <int H>
__device__ __forceinline__ int xor_lane32(int v, int lane) {
  if constexpr (H == 1) return dpp32<0xB1>(v);  // quad_perm [1, 0, 3, 2]
  else if constexpr (H == 2) return dpp32<0x4E>(v);  // quad_perm [2, 3, 0, 1]
  else if constexpr (H == 4 || H == 8) {
    const int up = dpp32<0x100 + H>(v);  // row_shl:H -> lane + H
    const int dn = dpp32<0x110 + H>(v);  // row_shr:H -> lane - H
    return (lane & H) ? dn : up;
  } else if constexpr (H == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane & 16) ? (int)r[0] : (int)r[1];
  } else {
    static_assert(H == 32, "xor_lane32: H in {1, 2, 4, 8, 16, 32}");
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (lane & 32) ? (int)r[0] : (int)r[1];
  }
}
template <int H>
__device__ __forceinline__ double xor_lane(double v, int lane) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = xor_lane32<H>((int)b, lane), hi = xor_lane32<H>((int)(b >> 32), lane);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
// lane ^ 63 = row_mirror (lane ^ 15), then ^ 16, ^ 32
__device__ __forceinline__ double mirror_lane(double v, int lane) {
  const long long b = __builtin_bit_cast(long long, v);
  int lo = dpp32<0x140>((int)b), hi = dpp32<0x140>((int)(b >> 32));
  lo = xor_lane32<32>(xor_lane32<16>(lo, lane), lane);
  hi = xor_lane32<32>(xor_lane32<16>(hi, lane), lane);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// lane-dependent twiddles of fft_wave, loaded once per wave before the tile arrives
template <int C, bool LAZY = false>
struct WaveTw {
  cplx t2_[C];   // exp(-2 pi i lane k2 / n), k2 >= 1
  cplx st_[6];   // stage h = 32 >> s: exp(-2 pi i (lane & (h-1)) n / (2h) / n)
  __device__ __forceinline__ void load(const double* w, int lane) {
    constexpr int n = 64 * C;
#pragma unroll
    for (int k2 = 1; k2 < C; ++k2) t2_[k2] = tw(w, (lane * k2) & (n - 1));
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const int h = 32 >> s;
      st_[s] = tw(w, (lane & (h - 1)) * (n / (2 * h)));
    }
  }
  __device__ __forceinline__ cplx t2(int k2) const { return t2_[k2]; }
  __device__ __forceinline__ cplx st(int s) const { return st_[s]; }
};
// LAZY (PB_FFT_TW_LAZY builds, Z pass): the twiddles are read from the (L1/L2-resident) table
// where they are used instead of being held in 52 VGPRs for the whole kernel. With the symbol
// scaling in the transform's epilogue the Z pass took 182 VGPRs and LAZY gained (144 VGPRs, 512^3
// 1.356 -> 1.28 ms, profiles/r02/ab_fft_twlazy.jsonl); with the scaling as its own LDS step
// (scale_pair) the pass takes 128 VGPRs either way and the register twiddles are faster
// (1.09 vs 1.19 ms, ab_fft_scale.jsonl)
template <int C>
struct WaveTw<C, true> {
  const double* w_;
  int lane_;
  __device__ __forceinline__ void load(const double* w, int lane) {
    w_ = w;
    lane_ = lane;
  }
  __device__ __forceinline__ cplx t2(int k2) const { return tw(w_, (lane_ * k2) & (64 * C - 1)); }
  __device__ __forceinline__ cplx st(int s) const {
    const int h = 32 >> s;
    return tw(w_, (lane_ & (h - 1)) * (64 * C / (2 * h)));
  }
};

template <int H, int C>
__device__ __forceinline__ void dif_stage(cplx (&z)[C], const cplx wh, int lane) {
  const bool upper = lane & H;
#pragma unroll
  for (int k2 = 0; k2 < C; ++k2) {
    const cplx p = {xor_lane<H>(z[k2].re, lane), xor_lane<H>(z[k2].im, lane)};
    if (upper)
      z[k2] = cmul({p.re - z[k2].re, p.im - z[k2].im}, wh);
    else
      z[k2] = {z[k2].re + p.re, z[k2].im + p.im};
  }
}

// z (lane owns elements lane + 64 m, m < C) -> spectrum: lane L holds Z[k2 + C bitrev6(L)] in
// z[k2]. n = 64 C, w = exp(-2 pi i k / n).
template <int C, class TW>
__device__ __forceinline__ void fft_wave(cplx (&z)[C], const double* w, const TW& T,
                                         int lane) {
  constexpr int n = 64 * C, LB = ilog2(C);
  // (1) C-point DFT over m in registers (radix-2 DIT, bit-reversed input order)
  cplx t[C];
#pragma unroll
  for (int i = 0; i < C; ++i) t[i] = z[bitrev(i, LB)];
#pragma unroll
  for (int len = 2; len <= C; len <<= 1)
#pragma unroll
    for (int i = 0; i < C; i += len)
#pragma unroll
      for (int j = 0; j < len / 2; ++j) {
        const cplx u = t[i + j], v = cmul(t[i + j + len / 2], tw(w, j * (n / len)));
        t[i + j] = {u.re + v.re, u.im + v.im};
        t[i + j + len / 2] = {u.re - v.re, u.im - v.im};
      }
  // (2) twiddles exp(-2 pi i lane k2 / n)
#pragma unroll
  for (int k2 = 0; k2 < C; ++k2) z[k2] = k2 ? cmul(t[k2], T.t2(k2)) : t[k2];
  // (3) 64-point DFT across lanes: radix-2 DIF, partner lane ^ h
  dif_stage<32>(z, T.st(0), lane);
  dif_stage<16>(z, T.st(1), lane);
  dif_stage<8>(z, T.st(2), lane);
  dif_stage<4>(z, T.st(3), lane);
  dif_stage<2>(z, T.st(4), lane);
  dif_stage<1>(z, T.st(5), lane);
}

// Hartley spectra of the two real lines packed in z (spectrum layout of fft_wave): hx, hy at
// k = k2 + C bitrev6(lane)
template <int C>
__device__ __forceinline__ void hartley_split(const cplx (&z)[C], double (&hx)[C], double (&hy)[C],
                                              int lane) {
  const int k1 = bitrev(lane, 6);
#pragma unroll
  for (int k2 = 0; k2 < C; ++k2) {
    // partner -k mod n: k2 = 0 -> (0, -k1 mod 64), lane bitrev6((64 - k1) & 63) (a bpermute);
    // else (C - k2, 63 - k1), lane bitrev6(63 - k1) = lane ^ 63
    const int k2p = k2 == 0 ? 0 : C - k2;
    cplx m;
    if (k2 == 0) {
      const int src = bitrev((64 - k1) & 63, 6);
      m = {__shfl(z[0].re, src, 64), __shfl(z[0].im, src, 64)};
    } else {
      m = {mirror_lane(z[k2p].re, lane), mirror_lane(z[k2p].im, lane)};
    }
    hx[k2] = 0.5 * ((z[k2].re + m.re) - (z[k2].im - m.im));
    hy[k2] = 0.5 * ((z[k2].im + m.im) + (z[k2].re - m.re));
  }
}

template <int C, int TL_>
struct DhtTile {
  static constexpr int n = 64 * C;
  static constexpr int TL = TL_;       // lines per tile (LDS: TL * (n + 1) doubles)
  static constexpr int NW = TL / 2;    // waves: two lines each
  static constexpr int NT = 64 * NW;
  static constexpr int LP = n + 1;     // odd line pitch: column writes spread over banks
  static constexpr size_t LDS = (size_t)TL * LP * sizeof(double);
};

// one DHT of the wave's two lines (pair p) in LDS, in place; SCALE: multiply by s(k) before the
// write-back (callers run the inverse transform again afterwards)
template <int C, bool SCALE, class TW>
__device__ __forceinline__ void dht_pair(double* lds, int l0, const DhtPass& p, const TW& T,
                                         int lane, int64_t outer, int inner0) {
  constexpr int LP = 64 * C + 1;
  constexpr int n = 64 * C;
  cplx z[C];
#pragma unroll
  for (int m = 0; m < C; ++m) z[m] = {lds[l0 * LP + lane + 64 * m], lds[(l0 + 1) * LP + lane + 64 * m]};
  fft_wave<C>(z, p.w, T, lane);
  double hx[C], hy[C];
  hartley_split<C>(z, hx, hy, lane);
  const int k1 = bitrev(lane, 6);
  if constexpr (SCALE) {  // Z pass: line (i, j) -> kx = i, ky = j; element -> kz
    const int nx = p.nx, ny = p.ny;
    const int i0 = inner0 + l0, j = p.j0 + (int)outer;
    const double* Lx = p.tab;
    const double* Jx = Lx + nx;
    const double* Ly = Jx + nx;
    const double* Jy = Ly + ny;
    const double* Lz = Jy + ny;
    const double* Jz = Lz + n;
    const double ly = Ly[j], jy = Jy[j];
    const double a0 = Lx[i0] * jy + Jx[i0] * ly, c0 = Jx[i0] * jy;
    const double a1 = Lx[i0 + 1] * jy + Jx[i0 + 1] * ly, c1 = Jx[i0 + 1] * jy;
#pragma unroll
    for (int k2 = 0; k2 < C; ++k2) {
      const int k = k2 + C * k1;
      const double lam0 = a0 * Jz[k] + c0 * Lz[k], lam1 = a1 * Jz[k] + c1 * Lz[k];
      hx[k2] = fabs(lam0) > p.thr ? hx[k2] * (p.scale / lam0) : 0.0;
      hy[k2] = fabs(lam1) > p.thr ? hy[k2] * (p.scale / lam1) : 0.0;
    }
  }
#pragma unroll
  for (int k2 = 0; k2 < C; ++k2) {
    const int k = k2 + C * k1;
    lds[l0 * LP + k] = hx[k2];
    lds[(l0 + 1) * LP + k] = hy[k2];
  }
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The Z pass's 1/(N lambda) scaling as its own step over the wave's two spectra in LDS (element k
// of both lines per lane, k = lane + 64 m: coalesced symbol-table reads), between two unscaled
// transforms -- the same arithmetic as the SCALE epilogue of dht_pair, without its symbol values
// and spectra live in registers beside the transform's (PB_FFT_SCALE_LDS): 512^3 Z pass 182 -> 128
// VGPRs, 2 -> 4 waves per SIMD, 1.356 -> 1.09 ms; 256^3 124 -> 88 VGPRs (ab_fft_scale.jsonl)
template <int C>
__device__ __forceinline__ void scale_pair(double* lds, int l0, const DhtPass& p, int lane,
                                           int64_t outer, int inner0) {
  constexpr int LP = 64 * C + 1;
  constexpr int n = 64 * C;
  const int nx = p.nx, ny = p.ny;
  const int i0 = inner0 + l0, j = p.j0 + (int)outer;
  const double* Lx = p.tab;
  const double* Jx = Lx + nx;
  const double* Ly = Jx + nx;
  const double* Jy = Ly + ny;
  const double* Lz = Jy + ny;
  const double* Jz = Lz + n;
  const double ly = Ly[j], jy = Jy[j];
  const double a0 = Lx[i0] * jy + Jx[i0] * ly, c0 = Jx[i0] * jy;
  const double a1 = Lx[i0 + 1] * jy + Jx[i0 + 1] * ly, c1 = Jx[i0 + 1] * jy;
#pragma unroll
  for (int m = 0; m < C; ++m) {
    const int k = lane + 64 * m;
    const double lam0 = a0 * Jz[k] + c0 * Lz[k], lam1 = a1 * Jz[k] + c1 * Lz[k];
    const double hx = lds[l0 * LP + k], hy = lds[(l0 + 1) * LP + k];
    lds[l0 * LP + k] = fabs(lam0) > p.thr ? hx * (p.scale / lam0) : 0.0;
    lds[(l0 + 1) * LP + k] = fabs(lam1) > p.thr ? hy * (p.scale / lam1) : 0.0;
  }
}

// LAYOUT 0: the tile's lines are adjacent (li = 1), elements strided (rows of TL doubles);
// LAYOUT 1: lines contiguous (es = 1). MODE 0: one DHT; MODE 1: DHT, 1/(N lambda), DHT.
// One tile per block (a persistent form that prefetched the next tile into registers during the
// transforms measured 10-30 % slower: twice the VGPRs, half the resident waves).
template <int C, int TL, int LAYOUT, int MODE, bool SUMS = false>
__global__ __launch_bounds__(32 * TL) void dht_lines_kernel(DhtPass p, const int* skip) {
  using T = DhtTile<C, TL>;
  constexpr int n = T::n, NT = T::NT, LP = T::LP;
  if (skip && *skip) return;  // CG's device convergence flag (uniform)
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int tile = xcd_block(p.remap);
  const int64_t outer = tile / p.ntiles_inner;
  const int inner0 = (tile % p.ntiles_inner) * TL;
  const int64_t base = outer * p.lo + (int64_t)inner0 * p.li;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  WaveTw<C, MODE == 1 && PB_FFT_TW_LAZY> twv;
  twv.load(p.w, lane);  // in flight while the tile loads
  typedef double dv2 __attribute__((ext_vector_type(2)));
  // tile -> LDS (16-byte pairs along the contiguous direction). WAVE (X pass, contiguous lines of
  // <= 256 points): each wave loads and stores only its own two lines, so the block needs no
  // barrier around the transforms and its waves run independently (PB_FFT_X_WAVE): 256^3 X pass
  // 0.078 -> 0.062 ms; on 512-point lines it takes 136 VGPRs (3 waves per SIMD) and is slower,
  // 0.56 vs 0.49 ms (profiles/r02/ab_fft_xwave.jsonl)
  constexpr bool WAVE = LAYOUT == 1 && PB_FFT_X_WAVE && C <= 4;
  constexpr int NP = WAVE ? n : TL * n / 2;  // pairs moved by the block (WAVE: by the wave)
  constexpr int NS = WAVE ? 64 : NT;
  const int fid = WAVE ? lane : (int)threadIdx.x;
  const int l0 = 2 * wave;
  PB_FFT_UNROLL(PB_FFT_TILE_UNROLL)
  for (int f = fid; f < NP; f += NS) {
    int l, e;
    if (WAVE) {
      l = l0 + f / (n / 2);
      e = (f % (n / 2)) * 2;
    } else if (LAYOUT == 0) {
      l = (f % (TL / 2)) * 2;
      e = f / (TL / 2);
    } else {
      l = f / (n / 2);
      e = (f % (n / 2)) * 2;
    }
    const dv2 v = __builtin_nontemporal_load((const dv2*)(p.in + base + l * p.li + e * p.es));
    if (LAYOUT == 0) {
      lds[l * LP + e] = v.x;
      lds[(l + 1) * LP + e] = v.y;
    } else {
      lds[l * LP + e] = v.x;
      lds[l * LP + e + 1] = v.y;
    }
  }
  if (WAVE)
    wave_sync_lds();
  else
    __syncthreads();
  if (l0 < p.ninner - inner0) {
    dht_pair<C, MODE == 1 && !PB_FFT_SCALE_LDS>(lds, l0, p, twv, lane, outer, inner0);
    if (MODE == 1) {
      wave_sync_lds();
      if (PB_FFT_SCALE_LDS) {
        scale_pair<C>(lds, l0, p, lane, outer, inner0);
        wave_sync_lds();
      }
      dht_pair<C, false>(lds, l0, p, twv, lane, outer, inner0);
    }
  }
  if (WAVE)
    wave_sync_lds();
  else
    __syncthreads();
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  const double mu = SUMS ? p.st->mu : 0.0;
  PB_FFT_UNROLL(PB_FFT_TILE_UNROLL)
  for (int f = fid; f < NP; f += NS) {
    int l, e;
    if (WAVE) {
      l = l0 + f / (n / 2);
      e = (f % (n / 2)) * 2;
    } else if (LAYOUT == 0) {
      l = (f % (TL / 2)) * 2;
      e = f / (TL / 2);
    } else {
      l = f / (n / 2);
      e = (f % (n / 2)) * 2;
    }
    dv2 v;
    if (LAYOUT == 0) {
      v.x = lds[l * LP + e];
      v.y = lds[(l + 1) * LP + e];
    } else {
      v.x = lds[l * LP + e];
      v.y = lds[l * LP + e + 1];
    }
    const int64_t a = base + l * p.li + e * p.es;
    __builtin_nontemporal_store(v, (dv2*)(p.out + a));
    if constexpr (SUMS) {
      const dv2 rv = __builtin_nontemporal_load((const dv2*)(p.sr + a));
      const double t0 = v.x - mu, t1 = v.y - mu;
      acc[0] += t0;
      acc[1] += t0 * t0;
      acc[2] += t0 * rv.x;
      acc[3] += rv.x;
      acc[0] += t1;
      acc[1] += t1 * t1;
      acc[2] += t1 * rv.y;
      acc[3] += rv.y;
    }
  }
  if constexpr (SUMS) {  // fixed-order block reduction: wave butterflies, then waves in order
    __syncthreads();     // the tile's LDS reads are done
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      double v = acc[q];
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
      if (lane == 0) lds[wave * 4 + q] = v;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
      double v = lds[threadIdx.x];
      for (int w = 1; w < NT / 64; ++w) v += lds[w * 4 + threadIdx.x];
      p.parts[(int64_t)blockIdx.x * 4 + threadIdx.x] = v;
    }
  }
}

template <int C, int TL, int LAYOUT, int MODE>
int launch_dht_tl(pb_ctx* ctx, DhtPass& p, const int* skip) {
  using T = DhtTile<C, TL>;
  p.ntiles_inner = p.ninner / TL;
  const int64_t ntiles = (int64_t)p.ntiles_inner * p.nouter;
  auto kern = dht_lines_kernel<C, TL, LAYOUT, MODE>;
  auto kern_s = dht_lines_kernel<C, TL, LAYOUT, MODE, LAYOUT == 1 && MODE == 0>;
  static bool attr = false;
  if (!attr) {
    PB_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)T::LDS));
    PB_HIP(hipFuncSetAttribute((const void*)kern_s, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)T::LDS));
    attr = true;
  }
  if (p.parts) {
    if (LAYOUT != 1 || MODE != 0)
      return set_error(PB_ERR_STATE, "fft pc: residual sums on the X pass only");
    if (ntiles * 4 > ctx->partials_cap)
      return set_error(PB_ERR_UNSUPPORTED, "fft pc: %lld tiles exceed the partials capacity",
                       (long long)ntiles);
    p.nparts_out = (int)ntiles;
    kern = kern_s;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)ntiles), dim3(T::NT), T::LDS, ctx->stream, p, skip);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

// lines per tile by pass (PB_FFT_TL_X / _Y / _Z; default 16, 8 for the Z pass on lines of >= 512
// points -- measured at 512^3: X/Y 16 vs 8 vs 32 lines 0.52 / 0.57 / 0.66 ms, Z 8 lines 1.28 ms
// vs 1.65 with 16; at 256^3 the Z pass is faster with 16, 0.121 vs 0.132 ms -- and 8 for
// 1024-long lines): a power of two dividing ninner (>= 64)
template <int C, int LAYOUT, int MODE>
int launch_dht_c(pb_ctx* ctx, DhtPass& p, const int* skip) {
  const char* knob = LAYOUT == 1 ? "PB_FFT_TL_X" : (MODE == 1 ? "PB_FFT_TL_Z" : "PB_FFT_TL_Y");
  int tl = env_int(knob, (LAYOUT == 0 && MODE == 1 && C >= 8) ? 8 : 16);
  if (C >= 16 && tl > 8) tl = 8;
  while (tl > 4 && p.ninner % tl) tl /= 2;
  if (p.ninner % tl)
    return set_error(PB_ERR_UNSUPPORTED, "fft pc: %d lines do not tile", p.ninner);
  switch (tl) {
    case 32:
      if constexpr (C < 16) return launch_dht_tl<C, 32, LAYOUT, MODE>(ctx, p, skip);
      break;
    case 16: return launch_dht_tl<C, 16, LAYOUT, MODE>(ctx, p, skip);
    case 8: return launch_dht_tl<C, 8, LAYOUT, MODE>(ctx, p, skip);
    default: return launch_dht_tl<C, 4, LAYOUT, MODE>(ctx, p, skip);
  }
  return launch_dht_tl<C, 8, LAYOUT, MODE>(ctx, p, skip);
}

template <int LAYOUT, int MODE>
int launch_dht(pb_ctx* ctx, int64_t n, DhtPass& p, const int* skip) {
  switch (n) {
    case 64: return launch_dht_c<1, LAYOUT, MODE>(ctx, p, skip);
    case 128: return launch_dht_c<2, LAYOUT, MODE>(ctx, p, skip);
    case 256: return launch_dht_c<4, LAYOUT, MODE>(ctx, p, skip);
    case 512: return launch_dht_c<8, LAYOUT, MODE>(ctx, p, skip);
    case 1024: return launch_dht_c<16, LAYOUT, MODE>(ctx, p, skip);
  }
  return set_error(PB_ERR_UNSUPPORTED, "fft pc: line length %lld (64..1024, power of two)",
                   (long long)n);
}

bool dht_length_ok(int64_t n) { return n >= 64 && n <= 1024 && (n & (n - 1)) == 0; }

}  // namespace

struct FftPc {
  pb_grid* g = nullptr;
  double* dev = nullptr;  // twiddles (2 nx | 2 ny | 2 nz) then symbol tables (2 nx | 2 ny | 2 nz)
  double* tw[3] = {nullptr, nullptr, nullptr};
  double* tab = nullptr;
  double* ybuf = nullptr;  // split grids: one y-slab field + the transpose aux space
  double thr = 0.0;
};

// per-axis symbol factors (L, J) of the operator kind at wavenumber t = 2 pi k / n
static void axis_symbols(int compact, int64_t n, double h, double* L, double* J) {
  const double a_d = 63.0 / 62.0 / h, b_d = 17.0 / 62.0 / (3.0 * h), al_d = 9.0 / 62.0;
  const double a_i = 0.75, b_i = 1.0 / 20.0, al_i = 3.0 / 10.0;
  for (int64_t k = 0; k < n; ++k) {
    const long double t = 2.0L * 3.14159265358979323846264338327950288L * (long double)k / (long double)n;
    if (!compact) {
      L[k] = (double)((2.0L * cosl(t) - 2.0L) / ((long double)h * (long double)h));
      J[k] = 1.0;
      continue;
    }
    const long double sd = a_d * sinl(t / 2) + b_d * sinl(1.5L * t);
    const long double td = 1.0L + 2.0L * al_d * cosl(t);
    const long double si = a_i * cosl(t / 2) + b_i * cosl(1.5L * t);
    const long double ti = 1.0L + 2.0L * al_i * cosl(t);
    L[k] = (double)(-4.0L * sd * sd / (td * td));
    J[k] = (double)(4.0L * si * si / (ti * ti));
  }
}

int fftpc_create(pb_grid* g, const double deltas[3], int compact, FftPc** out) {
  for (int d = 0; d < 3; ++d)
    if (!dht_length_ok(g->n[d]))
      return set_error(PB_ERR_UNSUPPORTED,
                       "-pc_type fft: every grid extent must be a power of two in 64..1024 "
                       "(got %lld x %lld x %lld)",
                       (long long)g->n[0], (long long)g->n[1], (long long)g->n[2]);
  if (grid_split(g) && g->n[1] < g->ctx->nranks)
    return set_error(PB_ERR_UNSUPPORTED, "-pc_type fft: ny < ranks");
  FftPc* f = new FftPc();
  f->g = g;
  const int64_t nsum = g->n[0] + g->n[1] + g->n[2];
  std::vector<double> host(4 * nsum);
  double* ht = host.data();
  double* hs = host.data() + 2 * nsum;
  double lmax[3], jmax[3];
  int64_t off = 0;
  for (int d = 0; d < 3; ++d) {
    const int64_t n = g->n[d];
    for (int64_t k = 0; k < n; ++k) {
      const long double t = -2.0L * 3.14159265358979323846264338327950288L * (long double)k / (long double)n;
      ht[2 * (off + k)] = (double)cosl(t);
      ht[2 * (off + k) + 1] = (double)sinl(t);
    }
    double* L = hs + 2 * off;
    double* J = L + n;
    axis_symbols(compact, n, deltas[d], L, J);
    lmax[d] = jmax[d] = 0.0;
    for (int64_t k = 0; k < n; ++k) {
      lmax[d] = std::max(lmax[d], std::fabs(L[k]));
      jmax[d] = std::max(jmax[d], J[k]);
    }
    off += n;
  }
  // |lambda| <= sum_d max|L_d| prod_{e != d} max J_e
  const double bound = lmax[0] * jmax[1] * jmax[2] + jmax[0] * lmax[1] * jmax[2] +
                       jmax[0] * jmax[1] * lmax[2];
  f->thr = 1e-10 * bound;
  if (hipMalloc(&f->dev, host.size() * sizeof(double)) != hipSuccess) {
    delete f;
    return set_error(PB_ERR_ALLOC, "fft pc tables: out of device memory");
  }
  pb_ctx* ctx = g->ctx;
  PB_HIP(hipMemcpyAsync(f->dev, host.data(), host.size() * sizeof(double), hipMemcpyHostToDevice,
                        ctx->stream));
  PB_SYNC(ctx, "fft pc tables");
  f->tw[0] = f->dev;
  f->tw[1] = f->dev + 2 * g->n[0];
  f->tw[2] = f->dev + 2 * (g->n[0] + g->n[1]);
  f->tab = f->dev + 2 * nsum;
  if (grid_split(g)) {
    const int64_t len = yslab_len(g) + yslab_aux_len(g);
    if (hipMalloc(&f->ybuf, (size_t)len * sizeof(double)) != hipSuccess) {
      (void)hipFree(f->dev);
      delete f;
      return set_error(PB_ERR_ALLOC, "fft pc y-slab buffer: out of device memory");
    }
  }
  *out = f;
  return PB_OK;
}

// one DHT along an axis of the box b (b[2] = planes), in place or from `in`
static int dht_axis(pb_ctx* ctx, const FftPc* f, const int64_t b[3], int axis, const double* in,
                    double* out, const int* skip, int j0 = 0, const double* sr = nullptr,
                    const CgState* st = nullptr, int* np = nullptr) {
  static const char* names[3] = {"pc_fft_x", "pc_fft_y", "pc_fft_z"};
  ScopedTimer tm(ctx, names[axis]);
  DhtPass p{};
  p.remap = env_int("PB_FFT_REMAP", 1);
  p.in = in;
  p.out = out;
  p.w = f->tw[axis];
  const int64_t nx = b[0], ny = b[1], nz = b[2];
  if (axis == 0) {  // contiguous lines: inner = j, outer = k
    p.li = nx;
    p.lo = nx * ny;
    p.es = 1;
    p.ninner = (int)ny;
    p.nouter = (int)nz;
    if (np) {  // CG's residual sums ride on this (last) pass
      p.sr = sr;
      p.st = st;
      p.parts = ctx->d_partials;
    }
    PB_TRY((launch_dht<1, 0>(ctx, nx, p, skip)));
    if (np) *np = p.nparts_out;
    return PB_OK;
  }
  if (axis == 1) {  // inner = i, outer = k, elements along j
    p.li = 1;
    p.lo = nx * ny;
    p.es = nx;
    p.ninner = (int)nx;
    p.nouter = (int)nz;
    return launch_dht<0, 0>(ctx, ny, p, skip);
  }
  // axis 2 with the scaling: inner = i, outer = j, elements along k
  p.li = 1;
  p.lo = nx;
  p.es = nx * ny;
  p.ninner = (int)nx;
  p.nouter = (int)ny;
  p.tab = f->tab;
  p.nx = (int)f->g->n[0];
  p.ny = (int)f->g->n[1];
  p.j0 = j0;
  p.scale = 1.0 / ((double)f->g->n[0] * (double)f->g->n[1] * (double)f->g->n[2]);
  p.thr = f->thr;
  return launch_dht<0, 1>(ctx, nz, p, skip);
}

int fftpc_apply(FftPc* f, const double* r, double* z, const int* skip, const CgState* sums_st,
                int* nparts) {
  if (nparts) *nparts = 0;
  pb_grid* g = f->g;
  pb_ctx* ctx = g->ctx;
  ScopedTimer tm(ctx, "pc_fft");
  const int64_t b[3] = {g->n[0], g->n[1], g->nzl};
  PB_TRY(dht_axis(ctx, f, b, 0, r, z, skip));
  PB_TRY(dht_axis(ctx, f, b, 1, z, z, skip));
  if (!grid_split(g)) {
    PB_TRY(dht_axis(ctx, f, b, 2, z, z, skip));
  } else {
    YSlabPlan yp;
    double* fy = f->ybuf;
    PB_TRY(yslab_begin(g, fy + yslab_len(g), &yp));
    PB_TRY(yslab_to(g, yp, z, fy));
    const int64_t by[3] = {g->n[0], yp.ny_me, g->n[2]};
    PB_TRY(dht_axis(ctx, f, by, 2, fy, fy, skip, (int)yp.j0[ctx->rank]));
    PB_TRY(yslab_from(g, yp, fy, z));
  }
  PB_TRY(dht_axis(ctx, f, b, 1, z, z, skip));
  // with sums_st: the residual sums of CG (PB_FFT_SUMS, default on) are taken by the last pass
  static const int fused = env_int("PB_FFT_SUMS", 1);
  if (sums_st && nparts && fused) return dht_axis(ctx, f, b, 0, z, z, skip, 0, r, sums_st, nparts);
  return dht_axis(ctx, f, b, 0, z, z, skip);
}

void fftpc_destroy(FftPc* f) {
  if (!f) return;
  (void)wait_stream(f->g->ctx, f->g->ctx->stream, "fftpc_destroy");
  if (f->dev) (void)hipFree(f->dev);
  if (f->ybuf) (void)hipFree(f->ybuf);
  delete f;
}

}  // namespace pb
