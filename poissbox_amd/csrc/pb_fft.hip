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
// Line kernel (r03): a block stages a tile of TL lines in LDS (coalesced rows: TL x-adjacent lines
// give TL*8-byte row pieces on the strided passes, 128 B at TL = 16 -- 64-B pieces cap that pattern
// at ~2.6 TB/s, scripts/zpass_probe.hip), each wave takes two real lines x, y and runs ONE complex
// FFT of z = x + i y in place in LDS as a self-sorting Stockham transform: passes of radix 8
// (then 4, 2, 3, 5) -- every lane reads R elements n/R apart, twiddles them, runs the R-point DFT in
// registers and writes them back at (j / Ns) Ns R + j % Ns + r Ns. The two Hartley spectra follow
// from Z(k) and Z(n - k), read from LDS. Line lengths n = 2^a 3^b 5^c (a >= 1) in 32..1024. The
// element index is XOR-swizzled in LDS (lpad), so the scattered writes of the first pass hit
// distinct banks. Twiddles exp(-2 pi i k / n) come from a per-axis table, copied into LDS
// per block for n <= 512. X passes at 512 / 1024 points run register edges instead
// (dht_reg_x_kernel): no tile staging, the first and last Stockham passes on registers, and the
// first / last X pass also carry CG's x / r update / residual sums. (r02's engine ran the
// 64-point cross-lane part of the transform as six radix-2 stages of DPP / permlane exchanges:
// 2.5x the VALU work, and its Z pass, which runs two transforms, was compute-bound at 1.0-1.1 ms
// at 512^3 whatever the tile width.)
#include <algorithm>
#include <cmath>
#include <vector>

#include "pb_internal.hpp"
#include "pb_device.hpp"

#pragma clang fp contract(fast)

namespace pb {

namespace {

struct DhtPass {
  const double* in;   // tile source (X forward: r), else == out
  double* out;
  int64_t li, lo, es;  // element e of line (outer, inner) at outer*lo + inner*li + e*es
  int64_t lo_out;      // the output's outer stride (Y passes into / out of the padded buffer)
  // blocked elements (decomposed Y passes writing / reading the all-to-all buffer directly):
  // element e of the input at (e >> esh_in) * ebs_in + (e & (2^esh_in - 1)) * es (esh_in = 0:
  // plain e * es); likewise the output with esh_out / ebs_out / es_out (es_out = 0: es)
  int esh_in, esh_out;
  int64_t ebs_in, ebs_out, es_out;
  int ninner, nouter, ntiles_inner;
  const double* w;    // twiddles of the line axis: (re, im) of exp(-2 pi i k / n), k < n
  const double* tab;  // [Lx | Jx | Ly | Jy | Lz | Jz] (SCALE only)
  int nx, ny, j0;     // global x / y sizes, global y of the box's row 0 (SCALE only)
  double scale, thr;  // 1 / (nx ny nz) and the null-mode threshold (SCALE only)
  int remap;          // XCD-aware tile order (on): consecutive tiles share an XCD; Z pass
                      // 1.35-1.36 vs 1.375-1.378 ms without at 512^3 (ab_remap_fft.jsonl)
  // CG's residual sums taken by the last pass (X inverse) as it writes z: t = z - mu, over the
  // tile, against r = sr -> parts[block * 4 + (t, t^2, t r, r)] (cg_pc_sums_kernel's sums)
  const double* sr;
  double* parts;
  const CgState* st;
  int nparts_out;     // (host) partial blocks written
  int ncu;
  // CG's x / r update on the first X pass (register-edge kernel): the line input is
  // r = ru_in + (-alpha) ru_w, also stored to ru_out; ru_x = ru_x + alpha ru_p (ru_first: alpha p)
  const double* ru_in;
  const double* ru_w;
  double* ru_out;
  const double* ru_p;
  double* ru_x;
  int ru_first;
  const CgState* ru_st;
  // the self block of a blocked Y pass (YSlabPlan::self_direct): element block alt_blk is read
  // from in_alt / written to out_alt (the y-slab buffer; the all-to-all does not copy it); -1: none
  const double* in_alt = nullptr;
  double* out_alt = nullptr;
  int alt_blk = -1;
  int ablate;         // timing experiments only (PB_FFT_ABLATE=1): no transforms (tile copy
                      // through LDS); builds with -DPB_FFT_ABLATE_TRAFFIC=1 drop the global loads
                      // and stores instead (transforms on stale LDS)
};
#ifndef PB_FFT_ABLATE_TRAFFIC
#define PB_FFT_ABLATE_TRAFFIC 0
#endif

struct cplx {
  double re, im;
};
typedef double dv2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ cplx cmul(cplx a, cplx b) {
  return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
__device__ __forceinline__ cplx cadd(cplx a, cplx b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cplx csub(cplx a, cplx b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cplx cmi(cplx a) { return {a.im, -a.re}; }  // -i a
__device__ __forceinline__ cplx cpi(cplx a) { return {-a.im, a.re}; }  // +i a
__device__ __forceinline__ cplx cscale(cplx a, double s) { return {a.re * s, a.im * s}; }

// ---- Stockham plans: n = 2^a 3^b 5^c; radix 8 while 8 divides what is left, then 4, 2, 3, 5 ----
__host__ __device__ constexpr int natural_radix_at(int n, int p) {
  int rest = n;
  for (int q = 0; q <= p; ++q) {
    if (rest <= 1) return 0;
    const int r = rest % 8 == 0 ? 8
                  : rest % 4 == 0 ? 4
                  : rest % 2 == 0 ? 2
                  : rest % 3 == 0 ? 3
                  : rest % 5 == 0 ? 5 : 0;
    if (r == 0) return 0;
    if (q == p) return r;
    rest /= r;
  }
  return 0;
}
__host__ __device__ constexpr int natural_len(int n) {
  int rest = n, p = 0;
  for (; rest > 1; ++p) {
    const int r = natural_radix_at(n, p);
    if (r == 0) return 0;
    rest /= r;
  }
  return p;
}
// The plan used everywhere (kernels and the host twiddle tables): the natural order, except that a
// last radix that differs from the first moves to second place when that makes the first and last
// passes equal (1024: 8 8 8 2 -> 8 2 8 8), so the register-edge kernel (dht_reg_kernel) can run
// the first and last passes from registers
__host__ __device__ constexpr int plan_radix_at(int n, int p) {
  const int L = natural_len(n);
  const bool rot = L >= 3 && natural_radix_at(n, L - 1) != natural_radix_at(n, 0) &&
                   natural_radix_at(n, L - 2) == natural_radix_at(n, 0);
  if (!rot || p == 0 || p >= L) return natural_radix_at(n, p);
  return p == 1 ? natural_radix_at(n, L - 1) : natural_radix_at(n, p - 1);
}
__host__ __device__ constexpr int plan_len(int n) { return natural_len(n); }
__host__ __device__ constexpr bool plan_complete(int n) {
  int rest = n;
  for (int p = 0; rest > 1; ++p) {
    const int r = plan_radix_at(n, p);
    if (r == 0) return false;
    rest /= r;
  }
  return true;
}

// LDS index of element e in a line: the low four bits XOR-ed with bits 4..7 -- a permutation
// inside each aligned block of 16 elements, so 32 contiguous lanes still hit 64 distinct banks,
// while the stride-R writes of the first Stockham pass spread over all banks (an LDS bank model
// of the 512-point passes: 72 read cycles against 128 for one pad double every 16 elements, the
// same write cycles, and no padding)
__host__ __device__ constexpr int lpad(int e) { return e ^ ((e >> 4) & 15); }
__host__ __device__ constexpr int lpad_max(int n) {
  int m = 0;
  for (int e = 0; e < n; ++e) m = lpad(e) > m ? lpad(e) : m;
  return m;
}

// ---- R-point DFTs in registers, forward (exp(-2 pi i j k / R)) ----
template <int R>
__device__ __forceinline__ void dft(cplx (&v)[R]) {
  if constexpr (R == 2) {
    const cplx a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
  } else if constexpr (R == 3) {
    constexpr double c1 = -0.5, s1 = -0.86602540378443864676;  // cos, sin(-2 pi / 3)
    const cplx t = cadd(v[1], v[2]), d = csub(v[1], v[2]);
    const cplx m = {v[0].re + c1 * t.re, v[0].im + c1 * t.im};
    v[0] = cadd(v[0], t);
    const cplx sd = cscale(cpi(d), s1);  // i s1 d
    v[1] = cadd(m, sd);
    v[2] = csub(m, sd);
  } else if constexpr (R == 4) {
    const cplx t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
    const cplx t2 = cadd(v[1], v[3]), t3 = csub(v[1], v[3]);
    v[0] = cadd(t0, t2);
    v[2] = csub(t0, t2);
    v[1] = cadd(t1, cmi(t3));
    v[3] = csub(t1, cmi(t3));
  } else if constexpr (R == 5) {
    constexpr double c1 = 0.30901699437494742410, c2 = -0.80901699437494742410;  // cos 2pi/5, 4pi/5
    constexpr double s1 = -0.95105651629515357212, s2 = -0.58778525229247312917;  // -sin 2pi/5, 4pi/5
    const cplx b1 = cadd(v[1], v[4]), b2 = cadd(v[2], v[3]);
    const cplx d1 = csub(v[1], v[4]), d2 = csub(v[2], v[3]);
    const cplx a0 = v[0];
    const cplx m1 = {a0.re + c1 * b1.re + c2 * b2.re, a0.im + c1 * b1.im + c2 * b2.im};
    const cplx m2 = {a0.re + c2 * b1.re + c1 * b2.re, a0.im + c2 * b1.im + c1 * b2.im};
    const cplx e1 = cpi({s1 * d1.re + s2 * d2.re, s1 * d1.im + s2 * d2.im});
    const cplx e2 = cpi({s2 * d1.re - s1 * d2.re, s2 * d1.im - s1 * d2.im});
    v[0] = cadd(a0, cadd(b1, b2));
    v[1] = cadd(m1, e1);
    v[4] = csub(m1, e1);
    v[2] = cadd(m2, e2);
    v[3] = csub(m2, e2);
  } else {
    static_assert(R == 8, "radix 2, 3, 4, 5 or 8");
    constexpr double h = 0.70710678118654752440;
    cplx e[4] = {v[0], v[2], v[4], v[6]}, o[4] = {v[1], v[3], v[5], v[7]};
    dft<4>(e);
    dft<4>(o);
    const cplx w1 = {h * (o[1].re + o[1].im), h * (o[1].im - o[1].re)};   // (1 - i)/sqrt2 o1
    const cplx w2 = cmi(o[2]);                                               // -i o2
    const cplx w3 = {h * (o[3].im - o[3].re), -h * (o[3].re + o[3].im)};  // (-1 - i)/sqrt2 o3
    v[0] = cadd(e[0], o[0]);
    v[4] = csub(e[0], o[0]);
    v[1] = cadd(e[1], w1);
    v[5] = csub(e[1], w1);
    v[2] = cadd(e[2], w2);
    v[6] = csub(e[2], w2);
    v[3] = cadd(e[3], w3);
    v[7] = csub(e[3], w3);
  }
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One Stockham pass of radix R over the wave's two lines (A = re, B = im rows in LDS), after
// NS points of every sub-transform are done. tw: the per-pass twiddle table (fft_twiddles): the
// pass's entries start at complex NS - 1, butterfly k's R - 1 factors exp(-2 pi i r k / (NS R))
// are consecutive (one 16-byte read each; lanes of distinct k hit distinct banks, lanes of the
// same k broadcast -- a plain exp(-2 pi i m / N) table read at m = r k N / (NS R) was 4- to 8-way
// bank-conflicted: 42 % of the Z pass's LDS cycles were conflict cycles).
template <int N, int R, int NS>
__device__ __forceinline__ void stockham_pass(double* A, double* B, const double* tw, int lane) {
  constexpr int NB = N / R, T = (NB + 63) / 64;
  cplx v[T][R];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int j = lane + 64 * t;
    if (NB % 64 == 0 || j < NB) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int e = lpad(j + r * NB);
        v[t][r] = {A[e], B[e]};
      }
      if constexpr (NS > 1) {
        const double* w = tw + 2 * (NS - 1 + (j % NS) * (R - 1));
#pragma unroll
        for (int r = 1; r < R; ++r) {
          const dv2 c = *(const dv2*)(w + 2 * (r - 1));
          v[t][r] = cmul(v[t][r], {c.x, c.y});
        }
      }
      dft<R>(v[t]);
    }
  }
  wave_sync_lds();
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int j = lane + 64 * t;
    if (NB % 64 == 0 || j < NB) {
      const int d = (j / NS) * NS * R + j % NS;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int e = lpad(d + r * NS);
        A[e] = v[t][r].re;
        B[e] = v[t][r].im;
      }
    }
  }
  wave_sync_lds();
}

template <int N, int P, int NS>
__device__ __forceinline__ void fft_passes(double* A, double* B, const double* tw, int lane) {
  constexpr int R = plan_radix_at(N, P);
  if constexpr (R != 0) {
    stockham_pass<N, R, NS>(A, B, tw, lane);
    fft_passes<N, P + 1, NS * R>(A, B, tw, lane);
  }
}

// DHT of the two real lines in rows A, B (in place, natural order): FFT of z = x + i y, then
// H_x(k) = Re X - Im X, H_y(k) = Re Y - Im Y with X, Y from Z(k) and Z(-k). A lane owns the
// pair (k, N - k) (k = 0 owns the two self-paired points 0 and N/2): it reads both and writes
// both, so no wave barrier and no registers are held between the reads and the writes.
template <int N>
__device__ __forceinline__ void dht2(double* A, double* B, const double* tw, int lane) {
  fft_passes<N, 0, 1>(A, B, tw, lane);
  constexpr int H = N / 2, T = (H + 63) / 64;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int k = lane + 64 * t;
    if (H % 64 == 0 || k < H) {
      const int m = k == 0 ? H : N - k;  // k = 0: points 0 and N/2, each its own partner
      const int ek = lpad(k), em = lpad(m);
      const double zr = A[ek], zi = B[ek], mr = A[em], mi = B[em];
      if (k == 0) {
        A[ek] = 0.5 * ((zr + zr) - (zi - zi));
        B[ek] = 0.5 * ((zi + zi) + (zr - zr));
        A[em] = 0.5 * ((mr + mr) - (mi - mi));
        B[em] = 0.5 * ((mi + mi) + (mr - mr));
      } else {
        A[ek] = 0.5 * ((zr + mr) - (zi - mi));
        B[ek] = 0.5 * ((zi + mi) + (zr - mr));
        A[em] = 0.5 * ((mr + zr) - (mi - zi));
        B[em] = 0.5 * ((mi + zi) + (mr - zr));
      }
    }
  }
  wave_sync_lds();
}

// The Z pass as F* diag(s) F per line (for a real symbol even in k, H diag(s) H = F* diag(s) F):
// from Z = F(x + i y), W(k) = s_x(k) X(k) + i s_y(k) Y(k) = ((s_x + s_y)/2) Z(k)
// + ((s_x - s_y)/2) conj Z(-k) with s = 1/(N lambda) of line x (i0) and line y (i0 + 1)
// (1/lambda := 0 on the null modes); conj(W) goes back to A, B, so that a second forward FFT and
// a conjugation on the store give F* W = x' + i y'. One FFT + this step replaces the second
// Hartley split and the separate scaling step of DHT, scale, DHT (80 of 362 LDS operations per
// wave and tile at 512 points).
template <int N>
__device__ __forceinline__ void scale_combine2(double* A, double* B, const DhtPass& p, int lane,
                                               int64_t outer, int i0) {
  const int nx = p.nx, ny = p.ny, j = p.j0 + (int)outer;
  const double* Lx = p.tab;
  const double* Jx = Lx + nx;
  const double* Ly = Jx + nx;
  const double* Jy = Ly + ny;
  const double* Lz = Jy + ny;
  const double* Jz = Lz + N;
  const double ly = Ly[j], jy = Jy[j];
  const double a0 = Lx[i0] * jy + Jx[i0] * ly, c0 = Jx[i0] * jy;
  const double a1 = Lx[i0 + 1] * jy + Jx[i0 + 1] * ly, c1 = Jx[i0 + 1] * jy;
  // the symbol is even in k (the host tables are mirrored exactly): one (hp, hm) per pair
  auto factors = [&](int k, double& hp, double& hm) {
    const double lam0 = a0 * Jz[k] + c0 * Lz[k], lam1 = a1 * Jz[k] + c1 * Lz[k];
    const double sx = fabs(lam0) > p.thr ? p.scale / lam0 : 0.0;
    const double sy = fabs(lam1) > p.thr ? p.scale / lam1 : 0.0;
    hp = 0.5 * (sx + sy);
    hm = 0.5 * (sx - sy);
  };
  constexpr int H = N / 2, T = (H + 63) / 64;
#pragma unroll 2
  for (int t = 0; t < T; ++t) {
    const int k = lane + 64 * t;
    if (H % 64 == 0 || k < H) {
      const int m = k == 0 ? H : N - k;  // k = 0: points 0 and N/2, each its own partner
      const int ek = lpad(k), em = lpad(m);
      const double zr = A[ek], zi = B[ek], mr = A[em], mi = B[em];
      double hp, hm;
      factors(k, hp, hm);
      if (k == 0) {
        double hp2, hm2;
        factors(m, hp2, hm2);
        A[ek] = hp * zr + hm * zr;
        B[ek] = -(hp * zi - hm * zi);
        A[em] = hp2 * mr + hm2 * mr;
        B[em] = -(hp2 * mi - hm2 * mi);
      } else {  // conj(W) with W(k) = hp Z(k) + hm conj Z(N - k), and the same for N - k
        A[ek] = hp * zr + hm * mr;
        B[ek] = -(hp * zi - hm * mi);
        A[em] = hp * mr + hm * zr;
        B[em] = -(hp * mi - hm * zi);
      }
    }
  }
  wave_sync_lds();
}

// ---- register edges (r03): lane l of a wave owns butterflies jb = l + 64 t of the first and of
// the last Stockham pass (plans whose first and last radix agree and N / R is a multiple of 64:
// 512, 1024), whose elements jb + (N / R) r are exactly the ones it would load and store: the first
// pass can run on registers and the last one can leave the natural-order spectrum in registers.
// Each saves one LDS sweep (ds_write_b64 moves 85 B/clk per CU against 256 for ds_read_b64,
// MI355X_MICROARCH.md §LDS). ----
template <int N>
struct RegPlan {
  static constexpr int R = plan_radix_at(N, 0);
  static constexpr int NB = N / R;  // butterflies of the first and of the last pass
  static constexpr int T = NB / 64;
  static constexpr int NP = plan_len(N);
  static constexpr bool OK = NB % 64 == 0 && NP >= 2 && plan_radix_at(N, NP - 1) == R;
};

// first pass (NS = 1) on v, outputs to the wave's LDS rows
template <int N, int R, int T>
__device__ __forceinline__ void first_pass_regs(cplx (&v)[T][R], double* A, double* B, int lane) {
#pragma unroll
  for (int t = 0; t < T; ++t) {
    dft<R>(v[t]);
    const int jb = lane + 64 * t;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int e = lpad(jb * R + r);
      A[e] = v[t][r].re;
      B[e] = v[t][r].im;
    }
  }
  wave_sync_lds();
}

// middle passes P in [1, PL)
template <int N, int P, int PL, int NS>
__device__ __forceinline__ void mid_passes(double* A, double* B, const double* tw, int lane) {
  if constexpr (P < PL) {
    constexpr int R = plan_radix_at(N, P);
    stockham_pass<N, R, NS>(A, B, tw, lane);
    mid_passes<N, P + 1, PL, NS * R>(A, B, tw, lane);
  }
}

// last pass (NS = N / R) from the wave's LDS rows into v: v[t][r] = Z(jb + NB r)
template <int N, int R, int T>
__device__ __forceinline__ void last_pass_regs(cplx (&v)[T][R], const double* A, const double* B,
                                               const double* tw, int lane) {
  constexpr int NB = N / R;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int jb = lane + 64 * t;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int e = lpad(jb + r * NB);
      v[t][r] = {A[e], B[e]};
    }
    const double* w = tw + 2 * (NB - 1 + jb * (R - 1));
#pragma unroll
    for (int r = 1; r < R; ++r) {
      const dv2 c = *(const dv2*)(w + 2 * (r - 1));
      v[t][r] = cmul(v[t][r], {c.x, c.y});
    }
    dft<R>(v[t]);
  }
}

template <int N>
__device__ __forceinline__ void fft_regs(cplx (&v)[RegPlan<N>::T][RegPlan<N>::R], double* A,
                                         double* B, const double* tw, int lane) {
  using RP = RegPlan<N>;
  first_pass_regs<N, RP::R, RP::T>(v, A, B, lane);
  mid_passes<N, 1, RP::NP - 1, RP::R>(A, B, tw, lane);
  last_pass_regs<N, RP::R, RP::T>(v, A, B, tw, lane);
  wave_sync_lds();  // the last pass's reads are done before the rows are written again
}


template <int N, int TL_>
struct DhtTile {
  static constexpr int TL = TL_;              // lines per tile
  static constexpr int NW = TL / 2;           // waves: two lines each
  static constexpr int NT = 64 * NW;
  static constexpr int LP = (lpad_max(N) + 1) | 1;  // line pitch (doubles), odd
  static constexpr bool TWL = N <= 512;       // twiddle table in LDS (else read from L1/L2)
  static constexpr int TWO = TL * LP;         // twiddle table offset (even: TL is)
  static constexpr size_t LDS = (size_t)(TWO + (TWL ? 2 * N : 0)) * sizeof(double);
};

// tile lines per block: 16 (8 waves; 1024-point lines: one block per CU for LDS, which beats two
// blocks of 8-line tiles with 64-B row pieces: 1024^3 Z pass 8.52 -> 6.74 ms, Y 4.42 -> 4.14 ms,
// profiles/r03/fft1024_tl_ab.jsonl), 8 for 768-point lines
template <int N>
constexpr int tile_lines() { return N == 1024 ? 16 : (N > 512 ? 8 : 16); }

// LAYOUT 0: the tile's lines are adjacent (li = 1), elements strided (rows of TL doubles);
// LAYOUT 1: lines contiguous (es = 1), each wave loads / stores its own two lines (no block
// barrier around the transforms). MODE 0: one DHT; MODE 1: DHT, 1/(N lambda), DHT.
// One tile per block, except with PF (the LDS-tile X pass on <= 512 points): persistent
// blocks walk the tiles and fetch the next tile's input into registers while the current one is
// transformed and stored (+32 VGPRs at n = 512; occupancy stays LDS-bound at two blocks per CU).
template <int N, int TL_, int LAYOUT, int MODE, bool SUMS>
__global__ __launch_bounds__(32 * TL_, N <= 512 ? 4 : 1) void dht_lines_kernel(DhtPass p,
                                                                             const int* skip) {
  using T = DhtTile<N, TL_>;
  constexpr int TL = T::TL, NT = T::NT, LP = T::LP;
  if (skip && *skip) return;  // CG's device convergence flag (uniform)
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l0 = 2 * wave;
  const double* tw = p.w;
  if constexpr (T::TWL) {
    double* twl = lds + T::TWO;
    for (int i = threadIdx.x; i < N; i += NT) {
      const dv2 v = *(const dv2*)(p.w + 2 * i);
      twl[2 * i] = v.x;
      twl[2 * i + 1] = v.y;
    }
    tw = twl;
  }
  // tile t: lines [inner0, inner0 + nl) of row `outer`
  const int ntiles = p.ntiles_inner * p.nouter;
  auto tile_of = [&](int t, int64_t& outer, int& inner0, int& nl, int64_t& base) {
    outer = t / p.ntiles_inner;  // consecutive tiles are x-adjacent (same outer row)
    inner0 = (t % p.ntiles_inner) * TL;
    nl = min(TL, p.ninner - inner0);  // even: every extent is
    base = outer * p.lo + (int64_t)inner0 * p.li;
  };
  // 16-byte pairs along the contiguous direction; WAVE (LAYOUT 1): a wave moves its own lines
  constexpr bool WAVE = LAYOUT == 1;
  constexpr int NP = WAVE ? N : TL * N / 2;  // pairs moved by the block (WAVE: by the wave)
  constexpr int NS = WAVE ? 64 : NT;
  constexpr int NR = (NP + NS - 1) / NS;    // pairs per thread (the last round may be partial)
  const int fid = WAVE ? lane : (int)threadIdx.x;
  // element offsets (blocked layouts: the decomposed Y passes, strided LAYOUT 0 only)
  auto eoff_in = [&](int e) -> int64_t {
    if (LAYOUT == 0 && p.esh_in)
      return (int64_t)(e >> p.esh_in) * p.ebs_in + (int64_t)(e & ((1 << p.esh_in) - 1)) * p.es;
    return (int64_t)e * p.es;
  };
  const int64_t es_o = p.es_out ? p.es_out : p.es;
  auto eoff_out = [&](int e) -> int64_t {
    if (LAYOUT == 0 && p.esh_out)
      return (int64_t)(e >> p.esh_out) * p.ebs_out + (int64_t)(e & ((1 << p.esh_out) - 1)) * es_o;
    return (int64_t)e * es_o;
  };
  // (l, e) of the thread's q-th pair; l = TL (no line) past the tile's pairs
  // (the thread index goes through an empty asm per use: recomputing (l, e) costs a few VALU
  // ops, while letting the compiler hoist every pair's coordinates and addresses out of the tile
  // loop held ~50 more VGPRs and halved the resident waves)
  auto coord = [&](int q, int& l, int& e) {
    int fv = fid;
    asm volatile("" : "+v"(fv));
    const int f = fv + q * NS;
    if (NP % NS != 0 && f >= NP) {
      l = TL;
      e = 0;
    } else if (WAVE) {
      l = l0 + f / (N / 2);
      e = (f % (N / 2)) * 2;
    } else {
      l = (f % (TL / 2)) * 2;
      e = f / (TL / 2);
    }
  };
  // PF (persistent blocks, next tile prefetched into registers): the contiguous X pass at <= 512
  // points (512^3: 0.448 -> 0.398 ms). The strided passes run one tile per block and rely on the
  // second resident block for overlap (prefetching there measured slower: Z 0.707 -> 0.808 ms)
  constexpr bool PF = LAYOUT == 1 && N <= 512;
  dv2 pre[PF ? NR : 1];
  // Every tile load is unconditional, from a valid address (pairs past the tile re-read the
  // tile's first pair; put ignores them): a load under a runtime `if` made the compiler wait for
  // each load before issuing the next (s_waitcnt vmcnt(0) after every global_load_dwordx4 in the
  // ISA), one HBM round trip per pair instead of all of them in flight.
  auto load_pair = [&](int64_t base, int nl, int q) -> dv2 {
    int l, e;
    coord(q, l, e);
    const bool ok = l < nl;
    const int lc = ok ? l : 0, ec = ok ? e : 0;  // selects, not a branch around the load
    if (PB_FFT_ABLATE_TRAFFIC) return dv2{0.0, 0.0};
    const double* src = p.in;
    if (LAYOUT == 0 && p.esh_in && (ec >> p.esh_in) == p.alt_blk) src = p.in_alt;  // (a select)
    return __builtin_nontemporal_load((const dv2*)(src + base + lc * p.li + eoff_in(ec)));
  };
  auto fetch = [&](int t) {
    int64_t outer, base;
    int inner0, nl;
    tile_of(t, outer, inner0, nl, base);
    if constexpr (PF) {
#pragma unroll
      for (int q = 0; q < NR; ++q) pre[q] = load_pair(base, nl, q);
    }
  };
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  const double mu = SUMS ? p.st->mu : 0.0;
  // PF: prefetch the next tile into registers (lines of <= 512 points; longer lines have no
  // registers to spare: their tile is loaded where it is needed)
  const int G = PF ? (int)gridDim.x : ntiles;
  int t = PF ? (int)blockIdx.x : xcd_block(p.remap);
  if (PF && t < ntiles) fetch(t);
  for (; t < ntiles; t += G) {
    int64_t outer, base;
    int inner0, nl;
    tile_of(t, outer, inner0, nl, base);

    if (WAVE)
      wave_sync_lds();
    else
      __syncthreads();  // the previous tile's LDS reads are done (and the twiddle table is in)
    auto put = [&](int l, int e, dv2 v) {
      if (LAYOUT == 0) {
        lds[l * LP + lpad(e)] = v.x;
        lds[(l + 1) * LP + lpad(e)] = v.y;
      } else {
        lds[l * LP + lpad(e)] = v.x;
        lds[l * LP + lpad(e + 1)] = v.y;
      }
    };
    if constexpr (PF) {
#pragma unroll
      for (int q = 0; q < NR; ++q) {
        int l, e;
        coord(q, l, e);
        if (l < nl) put(l, e, pre[q]);
      }
    } else {  // QB loads in flight at a time (registers), then their LDS writes
      constexpr int QB = N <= 512 ? (NR < 8 ? NR : 8) : 4;
#pragma unroll
      for (int q0 = 0; q0 < NR; q0 += QB) {
        dv2 v[QB];
#pragma unroll
        for (int q = 0; q < QB; ++q)
          if (q0 + q < NR) v[q] = load_pair(base, nl, q0 + q);
#pragma unroll
        for (int q = 0; q < QB; ++q) {
          int l, e;
          coord(q0 + q, l, e);
          if (q0 + q < NR && l < nl) put(l, e, v[q]);
        }
      }
    }
    if (WAVE && t < G)
      __syncthreads();  // first tile: the twiddle table (written by the whole block) is in
    else if (WAVE)
      wave_sync_lds();
    else
      __syncthreads();
    if (PF && t + G < ntiles) fetch(t + G);  // in flight during the transforms and the stores
    if (l0 < nl && p.ablate != 1) {
      double* A = lds + l0 * LP;
      double* B = A + LP;
      if constexpr (MODE == 1) {  // F* diag(s) F: FFT, scale-combine, FFT, conjugate (store)
        fft_passes<N, 0, 1>(A, B, tw, lane);
        scale_combine2<N>(A, B, p, lane, outer, inner0 + l0);
        fft_passes<N, 0, 1>(A, B, tw, lane);
      } else {
        dht2<N>(A, B, tw, lane);
      }
    }
    if (WAVE)
      wave_sync_lds();
    else
      __syncthreads();
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      int l, e;
      coord(q, l, e);
      if (l < nl) {
        dv2 v;
        if (LAYOUT == 0) {
          v.x = lds[l * LP + lpad(e)];
          v.y = lds[(l + 1) * LP + lpad(e)];
          if (MODE == 1) v.y = -v.y;  // the conjugation of F* W = conj(F conj W)
        } else {
          v.x = lds[l * LP + lpad(e)];
          v.y = lds[l * LP + lpad(e + 1)];
        }
        const int64_t a = base + outer * (p.lo_out - p.lo) + l * p.li + eoff_out(e);
        if (PB_FFT_ABLATE_TRAFFIC) {
          if (v.x == 12345.678) p.out[a] = v.y;  // keeps the LDS reads (never true on real data)
          continue;
        }
        double* dst = p.out;
        if (LAYOUT == 0 && p.esh_out && (e >> p.esh_out) == p.alt_blk) dst = p.out_alt;
        __builtin_nontemporal_store(v, (dv2*)(dst + a));
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

// X passes (contiguous lines) on register edges: wave w of a 512-thread block owns lines
// (2w, 2w+1) of a 16-line tile and loads its elements jb + NB r straight from HBM (two coalesced
// 8-byte rows per element); the first pass runs on them, the last leaves Z(k) in registers, one
// partner exchange gives Z(N - k) for the Hartley split, and the spectra go straight back to HBM.
// No tile staging in LDS and no block barrier after the twiddle table (the waves run
// independently): 512^3 X pass 0.42 -> 0.365 ms (profiles/r03/fft_reg_ab.jsonl). On the strided
// passes the same per-lane rows (one 16-byte piece of each row per wave instruction) stream at
// 0.58 TB/s (scripts/zpass_probe.hip, wave_direct), so those keep the LDS tile.
template <int N, bool SUMS, bool RUPD>
__global__ __launch_bounds__(512, N <= 512 ? 4 : 2) void dht_reg_x_kernel(DhtPass p,
                                                                          const int* skip) {
  static_assert(!(SUMS && RUPD), "sums on the last pass, the r update on the first");
  using RP = RegPlan<N>;
  static_assert(RP::OK, "register-edge plan");
  constexpr int R = RP::R, NB = RP::NB, T = RP::T;
  constexpr int TL = 16, LP = (lpad_max(N) + 1) | 1;
  constexpr bool TWL = N <= 512;
  if (skip && *skip) {  // CG's device convergence flag (uniform)
    if (RUPD && p.ru_first) {  // a breakdown before the first update leaves x = x0 = 0
      const int tile = blockIdx.x;
      const int64_t outer = tile / p.ntiles_inner;
      const int inner0 = (tile % p.ntiles_inner) * TL;
      const int nl = min(TL, p.ninner - inner0);
      for (int i = threadIdx.x; i < nl * N; i += 512)
        p.ru_x[outer * p.lo + (int64_t)(inner0 + i / N) * p.li + i % N] = 0.0;
    }
    return;
  }
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const double* tw = p.w;
  if constexpr (TWL) {
    double* twl = lds + TL * LP;
    for (int i = threadIdx.x; i < N; i += 512) {
      const dv2 c = *(const dv2*)(p.w + 2 * i);
      twl[2 * i] = c.x;
      twl[2 * i + 1] = c.y;
    }
    tw = twl;
    __syncthreads();
  }
  const int l0 = 2 * wave;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  // one tile per block; with the sums, a resident grid walks the tiles (fewer partial blocks for
  // the finalize to reduce: 512 instead of 16384 at 512^3)
  auto do_tile = [&](int tile) {
  const int64_t outer = tile / p.ntiles_inner;
  const int inner0 = (tile % p.ntiles_inner) * TL;
  const int nl = min(TL, p.ninner - inner0);
  wave_sync_lds();  // the wave's LDS reads of its previous tile are done
  if (l0 < nl) {
    const int64_t base = outer * p.lo + (int64_t)(inner0 + l0) * p.li;  // es == 1
    cplx v[T][R];
    if constexpr (RUPD) {  // cg_pc_xr_kernel's arithmetic, rounded as there (no contraction)
      const double a = p.ru_st->alpha, ma = -a;
      const bool first = p.ru_first;
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int64_t e0 = base + lane + 64 * t + NB * r, e1 = e0 + p.li;
          const double r0 = __dadd_rn(__builtin_nontemporal_load(p.ru_in + e0),
                                      __dmul_rn(ma, __builtin_nontemporal_load(p.ru_w + e0)));
          const double r1 = __dadd_rn(__builtin_nontemporal_load(p.ru_in + e1),
                                      __dmul_rn(ma, __builtin_nontemporal_load(p.ru_w + e1)));
          __builtin_nontemporal_store(r0, p.ru_out + e0);
          __builtin_nontemporal_store(r1, p.ru_out + e1);
          v[t][r] = {r0, r1};
          const double ap0 = __dmul_rn(a, __builtin_nontemporal_load(p.ru_p + e0));
          const double ap1 = __dmul_rn(a, __builtin_nontemporal_load(p.ru_p + e1));
          const double x0 = first ? ap0 : __dadd_rn(__builtin_nontemporal_load(p.ru_x + e0), ap0);
          const double x1 = first ? ap1 : __dadd_rn(__builtin_nontemporal_load(p.ru_x + e1), ap1);
          __builtin_nontemporal_store(x0, p.ru_x + e0);
          __builtin_nontemporal_store(x1, p.ru_x + e1);
        }
    } else {
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int e = lane + 64 * t + NB * r;
          v[t][r] = {__builtin_nontemporal_load(p.in + base + e),
                     __builtin_nontemporal_load(p.in + base + p.li + e)};
        }
    }
    double* A = lds + l0 * LP;
    double* B = A + LP;
    fft_regs<N>(v, A, B, tw, lane);
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int e = lpad(lane + 64 * t + NB * r);
        A[e] = v[t][r].re;
        B[e] = v[t][r].im;
      }
    wave_sync_lds();
    const double mu = SUMS ? p.st->mu : 0.0;
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = lane + 64 * t + NB * r;
        const int em = lpad(k == 0 ? 0 : N - k);
        const double zr = v[t][r].re, zi = v[t][r].im, mr = A[em], mi = B[em];
        const double hx = 0.5 * ((zr + mr) - (zi - mi));  // dht2's split
        const double hy = 0.5 * ((zi + mi) + (zr - mr));
        __builtin_nontemporal_store(hx, p.out + base + k);
        __builtin_nontemporal_store(hy, p.out + base + p.li + k);
        if (SUMS) {  // CG's residual sums (t, t^2, t r, r), t = z - mu
          const double rx = __builtin_nontemporal_load(p.sr + base + k);
          const double ry = __builtin_nontemporal_load(p.sr + base + p.li + k);
          const double t0 = hx - mu, t1 = hy - mu;
          acc[0] += t0;
          acc[1] += t0 * t0;
          acc[2] += t0 * rx;
          acc[3] += rx;
          acc[0] += t1;
          acc[1] += t1 * t1;
          acc[2] += t1 * ry;
          acc[3] += ry;
        }
      }
  }
  };
  if constexpr (SUMS) {
    const int ntiles = p.ntiles_inner * p.nouter;
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) do_tile(tile);
  } else {
    do_tile(xcd_block(p.remap));
  }
  if constexpr (SUMS) {  // fixed-order block reduction: wave butterflies, then waves in order
    __syncthreads();     // every wave's LDS rows are done
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      double sv = acc[q];
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) sv += __shfl_xor(sv, off, 64);
      if (lane == 0) lds[wave * 4 + q] = sv;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
      double sv = lds[threadIdx.x];
      for (int w = 1; w < 8; ++w) sv += lds[w * 4 + threadIdx.x];
      p.parts[(int64_t)blockIdx.x * 4 + threadIdx.x] = sv;
    }
  }
}

template <int N>
int launch_dht_reg_x(pb_ctx* ctx, DhtPass& p, const int* skip) {
  constexpr int TL = 16, LP = (lpad_max(N) + 1) | 1;
  constexpr size_t LDS = (size_t)(TL * LP + (N <= 512 ? 2 * N : 0)) * sizeof(double);
  p.ntiles_inner = (p.ninner + TL - 1) / TL;
  const int64_t ntiles = (int64_t)p.ntiles_inner * p.nouter;
  auto kern = dht_reg_x_kernel<N, false, false>;
  auto kern_s = dht_reg_x_kernel<N, true, false>;
  auto kern_r = dht_reg_x_kernel<N, false, true>;
  static bool attr = false;
  if (!attr) {
    for (auto k : {kern, kern_s, kern_r})
      PB_HIP(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)LDS));
    attr = true;
  }
  if (p.ru_st) {
    if (p.parts) return set_error(PB_ERR_STATE, "fft pc: r update and sums on one pass");
    kern = kern_r;
  }
  if (ntiles > INT32_MAX) return set_error(PB_ERR_UNSUPPORTED, "fft pc: too many tiles");
  int64_t nblocks = ntiles;
  if (p.parts) {
    static int occ = 0;
    if (!occ) {
      PB_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern_s, 512, LDS));
      if (occ < 1) occ = 1;
    }
    nblocks = std::min<int64_t>(ntiles, (int64_t)occ * ctx->num_cus);
    if (nblocks * 4 > ctx->partials_cap)
      return set_error(PB_ERR_UNSUPPORTED, "fft pc: %lld blocks exceed the partials capacity",
                       (long long)nblocks);
    p.nparts_out = (int)nblocks;
    kern = kern_s;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)nblocks), dim3(512), LDS, ctx->stream, p, skip);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

// TL lines per tile
template <int N, int TL, int LAYOUT, int MODE>
int launch_dht_k(pb_ctx* ctx, DhtPass& p, const int* skip) {
  using T = DhtTile<N, TL>;
  p.ntiles_inner = (p.ninner + T::TL - 1) / T::TL;
  const int64_t ntiles = (int64_t)p.ntiles_inner * p.nouter;
  constexpr bool SUMS = LAYOUT == 1 && MODE == 0;
  auto kern = dht_lines_kernel<N, TL, LAYOUT, MODE, false>;
  auto kern_s = dht_lines_kernel<N, TL, LAYOUT, MODE, SUMS>;
  static int occ = 0;
  if (!occ) {
    PB_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)T::LDS));
    PB_HIP(hipFuncSetAttribute((const void*)kern_s, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)T::LDS));
    PB_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern_s, T::NT, T::LDS));
    if (occ < 1) occ = 1;
  }
  // persistent passes: one resident round of blocks; the others one tile per block
  int64_t nblocks = (int64_t)occ * ctx->num_cus;
  const bool persist = N <= 512 && LAYOUT == 1;
  if (!persist || nblocks > ntiles) nblocks = ntiles;
  if (p.parts) {
    if (!SUMS) return set_error(PB_ERR_STATE, "fft pc: residual sums on the X pass only");
    if (nblocks * 4 > ctx->partials_cap)
      return set_error(PB_ERR_UNSUPPORTED, "fft pc: %lld blocks exceed the partials capacity",
                       (long long)nblocks);
    p.nparts_out = (int)nblocks;
    kern = kern_s;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)nblocks), dim3(T::NT), T::LDS, ctx->stream, p, skip);
  PB_HIP(hipGetLastError());
  return PB_OK;
}

// Launch shapes (512^3, profiles/r03/fft_ab*.jsonl, lines_ab.jsonl): the strided passes stage
// 16-line tiles (128-B row pieces), one tile per block -- with unconditional tile loads that
// beats persistent blocks with register prefetch (Y 0.389 vs 0.452 ms, Z 0.646 vs 0.651);
// 32-line Z tiles (256-B pieces, one block per CU) measured no faster. The contiguous X passes run
// the register-edge kernel (launch_dht_reg_x) where it has a plan.
template <int N, int LAYOUT, int MODE>
int launch_dht_n(pb_ctx* ctx, DhtPass& p, const int* skip) {
  if (p.ninner % 2)
    return set_error(PB_ERR_UNSUPPORTED, "fft pc: %d lines (even counts only)", p.ninner);
  if constexpr (RegPlan<N>::OK && LAYOUT == 1) return launch_dht_reg_x<N>(ctx, p, skip);
  if (p.ru_st) return set_error(PB_ERR_STATE, "fft pc: r update on the register-edge X pass only");
  return launch_dht_k<N, tile_lines<N>(), LAYOUT, MODE>(ctx, p, skip);
}

// the line lengths with a compiled transform: 2^a (32..1024), 3 * 2^a (48..768), 5 * 2^a (40..640)
#define PB_FFT_LENGTHS(X) \
  X(32) X(64) X(128) X(256) X(512) X(1024) X(48) X(96) X(192) X(384) X(768) X(40) X(80) \
  X(160) X(320) X(640)

template <int LAYOUT, int MODE>
int launch_dht(pb_ctx* ctx, int64_t n, DhtPass& p, const int* skip) {
  switch (n) {
#define PB_FFT_CASE(L)                                                 \
  case L:                                                              \
    static_assert(plan_complete(L), "length without a Stockham plan"); \
    return launch_dht_n<L, LAYOUT, MODE>(ctx, p, skip);
    PB_FFT_LENGTHS(PB_FFT_CASE)
#undef PB_FFT_CASE
  }
  return set_error(PB_ERR_UNSUPPORTED,
                   "fft pc: line length %lld (2^a 32..1024, 3*2^a 48..768, 5*2^a 40..640)",
                   (long long)n);
}

bool dht_length_ok(int64_t n) {
  switch (n) {
#define PB_FFT_OK(L) case L:
    PB_FFT_LENGTHS(PB_FFT_OK)
#undef PB_FFT_OK
    return true;
  }
  return false;
}

}  // namespace

struct FftPc {
  pb_grid* g = nullptr;
  double* dev = nullptr;  // twiddles (2 nx | 2 ny | 2 nz) then symbol tables (2 nx | 2 ny | 2 nz)
  double* tw[3] = {nullptr, nullptr, nullptr};
  double* tab = nullptr;
  double* ybuf = nullptr;  // split grids: one y-slab field + the transpose aux space
  // one rank: the Y forward pass writes into zbuf, whose planes are `zplane` = nx ny + PB_FFT_ZPAD
  // (default 32) doubles apart, the Z pass runs there and the Y inverse pass reads it back: the Z
  // pass's elements are then not 2^k bytes apart (512^3: 2 MiB), which measured 13-23 % slower per
  // DoF than 1.5 / 2.5 MiB (profiles/r03/fft_plane_stride.jsonl). Z pass 0.649 -> 0.502 ms at
  // 512^3, 6.75 -> 6.21 ms at 1024^3 (fft_zpad.jsonl; a 16 KiB pad measured 0.99 ms: not every
  // pad breaks the aliasing)
  double* zbuf = nullptr;
  int64_t zplane = 0;
  double thr = 0.0;
};

// per-axis symbol factors (L, J) of the operator kind at wavenumber t = 2 pi k / n
static void axis_symbols(int compact, int64_t n, double h, double* L, double* J) {
  const double a_d = 63.0 / 62.0 / h, b_d = 17.0 / 62.0 / (3.0 * h), al_d = 9.0 / 62.0;
  const double a_i = 0.75, b_i = 1.0 / 20.0, al_i = 3.0 / 10.0;
  // k <= n/2 evaluated, the rest mirrored: the tables are exactly even (L[n-k] = L[k]), which the
  // Z pass's pairwise scale step relies on
  for (int64_t k = 0; k <= n / 2; ++k) {
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
  for (int64_t k = n / 2 + 1; k < n; ++k) {
    L[k] = L[n - k];
    J[k] = J[n - k];
  }
}

int fftpc_create(pb_grid* g, const double deltas[3], int compact, FftPc** out) {
  for (int d = 0; d < 3; ++d)
    if (!dht_length_ok(g->n[d]))
      return set_error(PB_ERR_UNSUPPORTED,
                       "-pc_type fft: every grid extent must be 2^a (32..1024), 3*2^a (48..768) "
                       "or 5*2^a (40..640) (got %lld x %lld x %lld)",
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
    // per-pass twiddles of the Stockham plan (stockham_pass): pass p (after NS points) holds
    // exp(-2 pi i r k / (NS R)) at complex NS - 1 + k (R - 1) + r - 1; N - 1 entries in all
    int64_t ns = 1;
    for (int pass = 0; ns < n; ++pass) {
      const int R = plan_radix_at((int)n, pass);
      for (int64_t k = 0; k < ns; ++k)
        for (int r = 1; r < R; ++r) {
          const long double t = -2.0L * 3.14159265358979323846264338327950288L * (long double)(r * k) /
                                (long double)(ns * R);
          const int64_t idx = ns - 1 + k * (R - 1) + (r - 1);
          ht[2 * (off + idx)] = (double)cosl(t);
          ht[2 * (off + idx) + 1] = (double)sinl(t);
        }
      ns *= R;
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
  } else if (const int64_t pad = tune("fft_zpad", 32);
             pad > 0 && g->plane >= tune("fft_zpad_min_plane", 512 * 512)) {
    // (256^3, 512 KiB planes: no gain, 0.079 -> 0.083 ms; so only from 2 MiB planes up)
    // the padded buffer is a speed choice (a whole extra field): without the memory for it the
    // Y / Z / Y passes run in place in z
    f->zplane = g->plane + pad;
    if (hipMalloc(&f->zbuf, (size_t)(f->zplane * g->nzl) * sizeof(double)) != hipSuccess) {
      (void)hipGetLastError();  // clear the allocation error
      f->zbuf = nullptr;
      f->zplane = 0;
    }
  }
  *out = f;
  return PB_OK;
}

// one DHT along an axis of the box b (b[2] = planes), in place or from `in`
// blk (Y passes of a decomposed grid): the output (blk_dir 1) or the input (blk_dir 2) is the
// y-slab all-to-all buffer, rank blocks [kl][jl][i] in rank order (yslab_blocked)
static int dht_axis(pb_ctx* ctx, const FftPc* f, const int64_t b[3], int axis, const double* in,
                    double* out, const int* skip, int j0 = 0, const double* sr = nullptr,
                    const CgState* st = nullptr, int* np = nullptr,
                    const RUpdate* ru = nullptr, int64_t pl_in = 0, int64_t pl_out = 0,
                    const YSlabPlan* blk = nullptr, int blk_dir = 0) {
  // pl_in / pl_out: plane strides of in / out (0: nx ny; the Y and Z passes of the padded buffer)
  static const char* names[3] = {"pc_fft_x", "pc_fft_y", "pc_fft_z"};
  ScopedTimer tm(ctx, names[axis]);
  DhtPass p{};
  p.remap = 1;
  p.ablate = PB_ABLATE_FFT;
  p.ncu = ctx->num_cus;
  p.in = in;
  p.out = out;
  p.w = f->tw[axis];
  const int64_t nx = b[0], ny = b[1], nz = b[2];
  if (axis == 0) {  // contiguous lines: inner = j, outer = k
    p.li = nx;
    p.lo = nx * ny;
    p.lo_out = p.lo;
    p.es = 1;
    p.ninner = (int)ny;
    p.nouter = (int)nz;
    if (np) {  // CG's residual sums ride on this (last) pass
      p.sr = sr;
      p.st = st;
      p.parts = ctx->d_partials;
    }
    if (ru) {  // CG's x / r update rides on this (first) pass
      p.ru_in = ru->r_in;
      p.ru_w = ru->w;
      p.ru_out = ru->r_out;
      p.ru_p = ru->p;
      p.ru_x = ru->x;
      p.ru_first = ru->first;
      p.ru_st = ru->st;
    }
    PB_TRY((launch_dht<1, 0>(ctx, nx, p, skip)));
    if (np) *np = p.nparts_out;
    return PB_OK;
  }
  if (axis == 1) {  // inner = i, outer = k, elements along j
    p.li = 1;
    p.lo = pl_in ? pl_in : nx * ny;
    p.lo_out = pl_out ? pl_out : nx * ny;
    p.es = nx;
    p.ninner = (int)nx;
    p.nouter = (int)nz;
    if (blk) {  // row (kl, j) of the z-slab lives at block j / nyl, row kl * nyl + j % nyl
      const int64_t nyl = blk->nyl[0];
      int sh = 0;
      while (((int64_t)1 << sh) < nyl) ++sh;
      if (blk_dir == 1) {
        p.lo_out = nyl * nx;
        p.esh_out = sh;
        p.ebs_out = nz * nyl * nx;
      } else {
        p.lo = nyl * nx;
        p.esh_in = sh;
        p.ebs_in = nz * nyl * nx;
      }
      if (blk->self_direct) {  // the self block goes straight to / comes from the y-slab
        p.alt_blk = blk->me;
        p.out_alt = blk->alt_out;
        p.in_alt = blk->alt_out;
      }
    }
    return launch_dht<0, 0>(ctx, ny, p, skip);
  }
  // axis 2 with the scaling: inner = i, outer = j, elements along k
  p.li = 1;
  p.lo = nx;
  p.lo_out = nx;
  p.es = pl_in ? pl_in : nx * ny;  // in place: pl_out == pl_in
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

bool fftpc_fuses_r_update(const FftPc* f) {
  return (f->g->n[0] == 512 || f->g->n[0] == 1024) && f->g->n[1] % 2 == 0;
}

int fftpc_apply(FftPc* f, const double* r, double* z, const int* skip, const CgState* sums_st,
                int* nparts, const RUpdate* ru) {
  if (nparts) *nparts = 0;
  pb_grid* g = f->g;
  pb_ctx* ctx = g->ctx;
  if (ru && !fftpc_fuses_r_update(f))
    return set_error(PB_ERR_STATE, "fft pc: r update needs the register-edge X pass");
  ScopedTimer tm(ctx, "pc_fft");
  const int64_t b[3] = {g->n[0], g->n[1], g->nzl};
  PB_TRY(dht_axis(ctx, f, b, 0, r, z, skip, 0, nullptr, nullptr, nullptr, ru));
  if (f->zbuf) {  // Y forward into the padded buffer, Z there, Y inverse back into z
    PB_TRY(dht_axis(ctx, f, b, 1, z, f->zbuf, skip, 0, nullptr, nullptr, nullptr, nullptr, 0,
                    f->zplane));
    PB_TRY(dht_axis(ctx, f, b, 2, f->zbuf, f->zbuf, skip, 0, nullptr, nullptr, nullptr, nullptr,
                    f->zplane, f->zplane));
    PB_TRY(dht_axis(ctx, f, b, 1, f->zbuf, z, skip, 0, nullptr, nullptr, nullptr, nullptr,
                    f->zplane, 0));
  } else if (!grid_split(g)) {
    PB_TRY(dht_axis(ctx, f, b, 1, z, z, skip));
    PB_TRY(dht_axis(ctx, f, b, 2, z, z, skip));
    PB_TRY(dht_axis(ctx, f, b, 1, z, z, skip));
  } else {
    YSlabPlan yp;
    double* fy = f->ybuf;
    PB_TRY(yslab_begin(g, fy + yslab_len(g), &yp));
    const int64_t by[3] = {g->n[0], yp.ny_me, g->n[2]};
    if (yslab_blocked(yp)) {
      // the Y passes write / read the all-to-all buffer in its blocked layout: no pack / unpack
      // pass (two field copies per apply)
      yp.alt_out = fy + yp.self_shift;  // (used when yp.self_direct)
      PB_TRY(dht_axis(ctx, f, b, 1, z, yp.stage, skip, 0, nullptr, nullptr, nullptr, nullptr, 0,
                      0, &yp, 1));
      PB_TRY(alltoallv_device(ctx, yp.stage, yp.zc.data(), fy, yp.yc.data(), yp.self_direct));
      PB_TRY(dht_axis(ctx, f, by, 2, fy, fy, skip, (int)yp.j0[ctx->rank]));
      PB_TRY(alltoallv_device(ctx, fy, yp.yc.data(), yp.stage, yp.zc.data(), yp.self_direct));
      PB_TRY(dht_axis(ctx, f, b, 1, yp.stage, z, skip, 0, nullptr, nullptr, nullptr, nullptr, 0,
                      0, &yp, 2));
    } else {
      PB_TRY(dht_axis(ctx, f, b, 1, z, z, skip));
      PB_TRY(yslab_to(g, yp, z, fy));
      PB_TRY(dht_axis(ctx, f, by, 2, fy, fy, skip, (int)yp.j0[ctx->rank]));
      PB_TRY(yslab_from(g, yp, fy, z));
      PB_TRY(dht_axis(ctx, f, b, 1, z, z, skip));
    }
  }
  // with sums_st: the residual sums of CG are taken by the last pass
  if (sums_st && nparts) return dht_axis(ctx, f, b, 0, z, z, skip, 0, r, sums_st, nparts);
  return dht_axis(ctx, f, b, 0, z, z, skip);
}

void fftpc_destroy(FftPc* f) {
  if (!f) return;
  (void)wait_stream(f->g->ctx, f->g->ctx->stream, "fftpc_destroy");
  if (f->dev) (void)hipFree(f->dev);
  if (f->ybuf) (void)hipFree(f->ybuf);
  if (f->zbuf) (void)hipFree(f->zbuf);
  delete f;
}

}  // namespace pb
