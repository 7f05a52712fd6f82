// rw_mix_probe.hip -- streaming rates of the CG passes' access patterns at 512^3 fp64, in the
// stencil engine's order (waves marching in z over 128-wide x-segments of TY rows, 4 waves per
// block, z-chunks, one plane prefetched) and flat: two arrays read and NW = 0 / 1 / 2 written.
// Question it answers: would moving pass A's p store into pass B (pass A read-only 16 B/DoF,
// pass B read-2/write-2 32 B/DoF; same 48 B/DoF per iteration) be faster than the current
// read-2/write-1 + read-2/write-1 split?
// Build: hipcc -O3 --offload-arch=gfx950 -o rw_mix_probe rw_mix_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr int NX = 512, NY = 512, NZ = 512;
constexpr long PLANE = (long)NX * NY;

// ROWS = 1: the 4 waves of a block take the 4 x-segments of the same TY rows (a block reads whole
// 4 KiB rows) instead of 4 consecutive y-tiles of one segment
template <int TY, int NW, int ROWS = 0, int NTL = 0>
__global__ __launch_bounds__(256) void zm_rw(const double* __restrict__ a, const double* __restrict__ b,
                                             double* __restrict__ y0, double* __restrict__ y1,
                                             double* __restrict__ sink, int nchunk) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int bb = blockIdx.x;
  const int nb = gridDim.x, q = nb / 8, r = nb % 8, xcd = bb % 8, slot = bb / 8;
  bb = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  const int nseg = NX / 128, ntile = NY / (4 * TY);
  int seg, tile, chunk, j0;
  if (ROWS) {  // block = TY rows x all 4 segments (NX = 512)
    const int nrow = NY / TY;
    seg = wid;
    tile = bb % nrow;
    chunk = bb / nrow;
    j0 = tile * TY;
  } else {
    seg = bb % nseg;
    bb /= nseg;
    tile = bb % ntile;
    chunk = bb / ntile;
    j0 = (tile * 4 + wid) * TY;
  }
  const int kc = (NZ + nchunk - 1) / nchunk;
  const int kb = chunk * kc, ke = min(kb + kc, NZ);
  const int i0 = seg * 128 + 2 * lane;
  dv2 va[TY], vb[TY];
  dv2 acc = {0.0, 0.0};
  auto ld = [&](int k) {
    const long base = k * PLANE;
#pragma unroll
    for (int t = 0; t < TY; ++t) {
      if (NTL) {  // non-temporal loads
        va[t] = __builtin_nontemporal_load((const dv2*)(a + base + (long)(j0 + t) * NX + i0));
        vb[t] = __builtin_nontemporal_load((const dv2*)(b + base + (long)(j0 + t) * NX + i0));
      } else {
        va[t] = *(const dv2*)(a + base + (long)(j0 + t) * NX + i0);
        vb[t] = *(const dv2*)(b + base + (long)(j0 + t) * NX + i0);
      }
    }
  };
  ld(kb);
  for (int k = kb; k < ke; ++k) {
    dv2 ca[TY], cb[TY];
#pragma unroll
    for (int t = 0; t < TY; ++t) ca[t] = va[t], cb[t] = vb[t];
    ld(k + 1 < ke ? k + 1 : k);
    const long base = k * PLANE;
#pragma unroll
    for (int t = 0; t < TY; ++t) {
      const dv2 p = ca[t] + 0.5 * cb[t];
      if constexpr (NW == 0) acc += p * cb[t];
      if constexpr (NW >= 1) __builtin_nontemporal_store(p, (dv2*)(y0 + base + (long)(j0 + t) * NX + i0));
      if constexpr (NW >= 2)
        __builtin_nontemporal_store(ca[t] - 0.25 * cb[t], (dv2*)(y1 + base + (long)(j0 + t) * NX + i0));
    }
  }
  if constexpr (NW == 0) sink[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y;
}

// Pass A's read pattern with its y-halo rows (rows j0-1 and j0+TY of both arrays, cached loads)
// and, for ROWS = 0, the two x-edge loads per row (cached): own rows cached (NTL = 0), or
// interior rows non-temporal and the block-boundary rows cached (NTL = 1; ROWS = 1 only: the 4
// waves of a block take the 4 x-segments of the same rows, so the x-edges stay inside the block)
template <int TY, int ROWS, int NTL>
__global__ __launch_bounds__(256) void zm_halo(const double* __restrict__ a,
                                               const double* __restrict__ b,
                                               double* __restrict__ sink, int nchunk) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int bb = blockIdx.x;
  const int nb = gridDim.x, q = nb / 8, r = nb % 8, xcd = bb % 8, slot = bb / 8;
  bb = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  const int nseg = NX / 128, ntile = NY / (4 * TY);
  int seg, chunk, j0;
  if (ROWS) {
    const int nrow = NY / TY;
    seg = wid;
    chunk = bb / nrow;
    j0 = (bb % nrow) * TY;
  } else {
    seg = bb % nseg;
    bb /= nseg;
    chunk = bb / ntile;
    j0 = ((bb % ntile) * 4 + wid) * TY;
  }
  const int kc = (NZ + nchunk - 1) / nchunk;
  const int kb = chunk * kc, ke = min(kb + kc, NZ);
  const int i0 = seg * 128 + 2 * lane;
  const int jd = (j0 + NY - 1) % NY, ju = (j0 + TY) % NY;
  const int eix = lane < 32 ? (seg * 128 + NX - 1) % NX : (seg * 128 + 128) % NX;
  dv2 acc = {0.0, 0.0};
  dv2 va[TY], vb[TY], ha[2], hb[2];
  double ea = 0.0, eb = 0.0;
  auto ld = [&](int k) {
    const long base = k * PLANE;
#pragma unroll
    for (int t = 0; t < TY; ++t) {
      const long o = base + (long)(j0 + t) * NX + i0;
      if (NTL && t > 0 && t < TY - 1) {
        va[t] = __builtin_nontemporal_load((const dv2*)(a + o));
        vb[t] = __builtin_nontemporal_load((const dv2*)(b + o));
      } else {
        va[t] = *(const dv2*)(a + o);
        vb[t] = *(const dv2*)(b + o);
      }
    }
    ha[0] = *(const dv2*)(a + base + (long)jd * NX + i0);
    hb[0] = *(const dv2*)(b + base + (long)jd * NX + i0);
    ha[1] = *(const dv2*)(a + base + (long)ju * NX + i0);
    hb[1] = *(const dv2*)(b + base + (long)ju * NX + i0);
    if (!ROWS) {
      const long eo = base + (long)(j0 + ((lane & 31) < TY ? (lane & 31) : 0)) * NX + eix;
      ea = a[eo];
      eb = b[eo];
    }
  };
  ld(kb);
  for (int k = kb; k < ke; ++k) {
    dv2 s = ha[0] * hb[0] + ha[1] * hb[1] + ea * eb;
#pragma unroll
    for (int t = 0; t < TY; ++t) s += va[t] * vb[t];
    ld(k + 1 < ke ? k + 1 : k);
    acc += s;
  }
  sink[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y;
}

template <int NW>
__global__ __launch_bounds__(256) void flat_rw(const dv2* __restrict__ a, const dv2* __restrict__ b,
                                               dv2* __restrict__ y0, dv2* __restrict__ y1,
                                               double* __restrict__ sink, long n) {
  dv2 acc = {0.0, 0.0};
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const dv2 av = a[i], bv = b[i];
    const dv2 p = av + 0.5 * bv;
    if constexpr (NW == 0) acc += p * bv;
    if constexpr (NW >= 1) __builtin_nontemporal_store(p, y0 + i);
    if constexpr (NW >= 2) __builtin_nontemporal_store(av - 0.25 * bv, y1 + i);
  }
  if constexpr (NW == 0) sink[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y;
}

int main() {
  const long N = PLANE * NZ;
  double *a, *b, *y0, *y1, *sink;
  CK(hipMalloc(&a, N * 8));
  CK(hipMalloc(&b, N * 8));
  CK(hipMalloc(&y0, N * 8));
  CK(hipMalloc(&y1, N * 8));
  CK(hipMalloc(&sink, 4096L * 256 * 8));
  CK(hipMemset(a, 0, N * 8));
  CK(hipMemset(b, 0, N * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, int nw, int p1, int p2, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f, tot = 0;
    const int reps = 20;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      tot += ms;
    }
    const double bytes = (16.0 + 8.0 * nw) * N;
    printf("{\"kernel\":\"%s\",\"nw\":%d,\"p1\":%d,\"p2\":%d,\"best_ms\":%.4f,\"avg_ms\":%.4f,"
           "\"GBps_avg\":%.1f}\n",
           name, nw, p1, p2, best, tot / reps, bytes / (tot / reps) / 1e6);
    fflush(stdout);
  };
  for (int g : {1024, 2048, 4096}) {
    run("flat", 0, g, 0, [&] { flat_rw<0><<<g, 256>>>((const dv2*)a, (const dv2*)b, (dv2*)y0, (dv2*)y1, sink, N / 2); });
    run("flat", 1, g, 0, [&] { flat_rw<1><<<g, 256>>>((const dv2*)a, (const dv2*)b, (dv2*)y0, (dv2*)y1, sink, N / 2); });
    run("flat", 2, g, 0, [&] { flat_rw<2><<<g, 256>>>((const dv2*)a, (const dv2*)b, (dv2*)y0, (dv2*)y1, sink, N / 2); });
  }
  for (int nc : {2, 4, 8, 16}) {
    const int nb4 = (NX / 128) * (NY / 16) * nc, nb8 = (NX / 128) * (NY / 32) * nc;
    run("seg_ty4", 0, 4, nc, [&] { zm_rw<4, 0><<<nb4, 256>>>(a, b, y0, y1, sink, nc); });
    run("seg_ty4", 1, 4, nc, [&] { zm_rw<4, 1><<<nb4, 256>>>(a, b, y0, y1, sink, nc); });
    run("seg_ty4", 2, 4, nc, [&] { zm_rw<4, 2><<<nb4, 256>>>(a, b, y0, y1, sink, nc); });
    run("seg_ty8", 0, 8, nc, [&] { zm_rw<8, 0><<<nb8, 256>>>(a, b, y0, y1, sink, nc); });
    run("seg_ty8", 1, 8, nc, [&] { zm_rw<8, 1><<<nb8, 256>>>(a, b, y0, y1, sink, nc); });
    run("seg_ty8", 2, 8, nc, [&] { zm_rw<8, 2><<<nb8, 256>>>(a, b, y0, y1, sink, nc); });
  }
  for (int nc : {2, 4}) {  // pass A's read pattern with halos (16 B/DoF algorithmic)
    const int nb4 = (NX / 128) * (NY / 16) * nc, nb8 = (NX / 128) * (NY / 32) * nc;
    run("halo_seg_ty4", 0, 4, nc, [&] { zm_halo<4, 0, 0><<<nb4, 256>>>(a, b, sink, nc); });
    run("halo_seg_ty8", 0, 8, nc, [&] { zm_halo<8, 0, 0><<<nb8, 256>>>(a, b, sink, nc); });
    run("halo_rows_ty8", 0, 8, nc, [&] { zm_halo<8, 1, 0><<<(NY / 8) * nc, 256>>>(a, b, sink, nc); });
    run("halo_rows_ty8_ntl", 0, 8, nc, [&] { zm_halo<8, 1, 1><<<(NY / 8) * nc, 256>>>(a, b, sink, nc); });
    run("halo_rows_ty4_ntl", 0, 4, nc, [&] { zm_halo<4, 1, 1><<<(NY / 4) * nc, 256>>>(a, b, sink, nc); });
  }
  for (int nc : {2, 4}) {
    const int nb4 = (NX / 128) * (NY / 16) * nc;
    run("seg_ty4_ntl", 0, 4, nc, [&] { zm_rw<4, 0, 0, 1><<<nb4, 256>>>(a, b, y0, y1, sink, nc); });
    run("seg_ty4_ntl", 1, 4, nc, [&] { zm_rw<4, 1, 0, 1><<<nb4, 256>>>(a, b, y0, y1, sink, nc); });
    run("seg_ty4_ntl", 2, 4, nc, [&] { zm_rw<4, 2, 0, 1><<<nb4, 256>>>(a, b, y0, y1, sink, nc); });
    run("seg_ty4", 0, 4, nc, [&] { zm_rw<4, 0><<<nb4, 256>>>(a, b, y0, y1, sink, nc); });
    run("seg_ty4", 2, 4, nc, [&] { zm_rw<4, 2><<<nb4, 256>>>(a, b, y0, y1, sink, nc); });
  }
  for (int nc : {2, 4, 8}) {
    const int nb4 = (NY / 4) * nc, nb8 = (NY / 8) * nc;
    run("rows_ty4", 0, 4, nc, [&] { zm_rw<4, 0, 1><<<nb4, 256>>>(a, b, y0, y1, sink, nc); });
    run("rows_ty4", 1, 4, nc, [&] { zm_rw<4, 1, 1><<<nb4, 256>>>(a, b, y0, y1, sink, nc); });
    run("rows_ty4", 2, 4, nc, [&] { zm_rw<4, 2, 1><<<nb4, 256>>>(a, b, y0, y1, sink, nc); });
    run("rows_ty8", 0, 8, nc, [&] { zm_rw<8, 0, 1><<<nb8, 256>>>(a, b, y0, y1, sink, nc); });
    run("rows_ty8", 1, 8, nc, [&] { zm_rw<8, 1, 1><<<nb8, 256>>>(a, b, y0, y1, sink, nc); });
    run("rows_ty8", 2, 8, nc, [&] { zm_rw<8, 2, 1><<<nb8, 256>>>(a, b, y0, y1, sink, nc); });
  }
  return 0;
}
