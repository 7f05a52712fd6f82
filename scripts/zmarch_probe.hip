// zmarch_probe.hip -- does the stencil engine's ACCESS PATTERN (waves marching in z over
// 128-wide x-segments of TY rows, 512^3 fp64) stream as fast as a flat copy? Pure copies in that
// order, with and without the halo-row / edge loads, against full-row (512-wide) waves.
// Build: hipcc -O3 --offload-arch=gfx950 -o zmarch_probe zmarch_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);  \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int NX = 512, NY = 512, NZ = 512;
constexpr long PLANE = (long)NX * NY;

// 128-wide segments, TY rows per wave, 4 waves per block stacked in y, z-chunks
template <int TY, int HALO, int EDGE>
__global__ __launch_bounds__(256) void zm_seg(const double* __restrict__ x, double* __restrict__ y,
                                              int nchunk) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int b = blockIdx.x;
  const int nb = gridDim.x, q = nb / 8, r = nb % 8, xcd = b % 8, slot = b / 8;
  b = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  const int nseg = NX / 128, ntile = NY / (4 * TY);
  const int seg = b % nseg;
  b /= nseg;
  const int tile = b % ntile, chunk = b / ntile;
  const int kc = (NZ + nchunk - 1) / nchunk;
  const int kb = chunk * kc, ke = min(kb + kc, NZ);
  const int j0 = (tile * 4 + wid) * TY;
  const int i0 = seg * 128 + 2 * lane;
  const int jd = j0 == 0 ? NY - 1 : j0 - 1, ju = j0 + TY >= NY ? 0 : j0 + TY;
  const int ei = lane < 32 ? (seg == 0 ? NX - 1 : seg * 128 - 1) : ((seg + 1) * 128 % NX);
  const int er = lane < 32 ? lane : lane - 32;
  for (int k = kb; k < ke; ++k) {
    const long base = k * PLANE;
    dv2 v[TY];
#pragma unroll
    for (int t = 0; t < TY; ++t) v[t] = *(const dv2*)(x + base + (long)(j0 + t) * NX + i0);
    double extra = 0.0;
    if (HALO) {
      const dv2 a = *(const dv2*)(x + base + (long)jd * NX + i0);
      const dv2 c = *(const dv2*)(x + base + (long)ju * NX + i0);
      extra += a.x + c.y;
    }
    if (EDGE && er < TY) extra += x[base + (long)(j0 + er) * NX + ei];
#pragma unroll
    for (int t = 0; t < TY; ++t) {
      dv2 o = v[t];
      o.x += 1e-300 * extra;
      __builtin_nontemporal_store(o, (dv2*)(y + base + (long)(j0 + t) * NX + i0));
    }
  }
}

// full 512-wide rows per wave (4 x 16-B loads per row), TY rows per wave, 4 waves per block
template <int TY, int HALO>
__global__ __launch_bounds__(256) void zm_full(const double* __restrict__ x, double* __restrict__ y,
                                               int nchunk) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int b = blockIdx.x;
  const int nb = gridDim.x, q = nb / 8, r = nb % 8, xcd = b % 8, slot = b / 8;
  b = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  const int ntile = NY / (4 * TY);
  const int tile = b % ntile, chunk = b / ntile;
  const int kc = (NZ + nchunk - 1) / nchunk;
  const int kb = chunk * kc, ke = min(kb + kc, NZ);
  const int j0 = (tile * 4 + wid) * TY;
  const int jd = j0 == 0 ? NY - 1 : j0 - 1, ju = j0 + TY >= NY ? 0 : j0 + TY;
  for (int k = kb; k < ke; ++k) {
    const long base = k * PLANE;
    dv2 v[TY][4];
#pragma unroll
    for (int t = 0; t < TY; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s)
        v[t][s] = *(const dv2*)(x + base + (long)(j0 + t) * NX + 128 * s + 2 * lane);
    double extra = 0.0;
    if (HALO) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const dv2 a = *(const dv2*)(x + base + (long)jd * NX + 128 * s + 2 * lane);
        const dv2 c = *(const dv2*)(x + base + (long)ju * NX + 128 * s + 2 * lane);
        extra += a.x + c.y;
      }
    }
#pragma unroll
    for (int t = 0; t < TY; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        dv2 o = v[t][s];
        o.x += 1e-300 * extra;
        __builtin_nontemporal_store(o, (dv2*)(y + base + (long)(j0 + t) * NX + 128 * s + 2 * lane));
      }
  }
}

__global__ __launch_bounds__(256) void flat_copy(const dv2* __restrict__ x, dv2* __restrict__ y, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    __builtin_nontemporal_store(x[i], y + i);
}

int main() {
  const long N = PLANE * NZ;
  double *x, *y;
  CK(hipMalloc(&x, N * 8));
  CK(hipMalloc(&y, N * 8));
  CK(hipMemset(x, 0, N * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, int param, auto launch) {
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
    printf("{\"kernel\":\"%s\",\"param\":%d,\"best_ms\":%.4f,\"avg_ms\":%.4f,\"GBps_avg\":%.1f}\n", name,
           param, best, tot / reps, 16.0 * N / (tot / reps) / 1e6);
  };
  for (int g : {1024, 2048})
    run("flat_copy", g, [&] { flat_copy<<<g, 256>>>((const dv2*)x, (dv2*)y, N / 2); });
  for (int nc : {4, 6, 8, 12}) {
    const int nb4 = (NX / 128) * (NY / 16) * nc;
    run("seg_ty4", nc, [&] { zm_seg<4, 0, 0><<<nb4, 256>>>(x, y, nc); });
    run("seg_ty4_halo", nc, [&] { zm_seg<4, 1, 0><<<nb4, 256>>>(x, y, nc); });
    run("seg_ty4_halo_edge", nc, [&] { zm_seg<4, 1, 1><<<nb4, 256>>>(x, y, nc); });
    const int nbf1 = (NY / 4) * nc;
    run("full_ty1", nc, [&] { zm_full<1, 0><<<nbf1, 256>>>(x, y, nc); });
    run("full_ty1_halo", nc, [&] { zm_full<1, 1><<<nbf1, 256>>>(x, y, nc); });
  }
  for (int nc : {8, 12, 16}) {
    const int nbf2 = (NY / 8) * nc;
    run("full_ty2", nc, [&] { zm_full<2, 0><<<nbf2, 256>>>(x, y, nc); });
    run("full_ty2_halo", nc, [&] { zm_full<2, 1><<<nbf2, 256>>>(x, y, nc); });
  }
  return 0;
}
