// r2w1_probe.hip -- the access pattern of CG pass A (two arrays read, one written, fp64, 512^3)
// in the stencil engine's order (waves marching in z over 128-wide x-segments of TY rows, 4 waves
// per block, z-chunks) against a flat grid-stride stream of the same bytes: is pass A's rate the
// pattern's ceiling? Variants: prefetch depth 0/1 (plane k+1 loaded while k is stored), TY 4/8,
// chunk counts (blocks per CU).
// Build: hipcc -O3 --offload-arch=gfx950 -o r2w1_probe r2w1_probe.hip
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

template <int TY, int PF>
__global__ __launch_bounds__(256) void zm_r2w1(const double* __restrict__ a,
                                               const double* __restrict__ b,
                                               double* __restrict__ y, int nchunk) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int bb = blockIdx.x;
  const int nb = gridDim.x, q = nb / 8, r = nb % 8, xcd = bb % 8, slot = bb / 8;
  bb = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  const int nseg = NX / 128, ntile = NY / (4 * TY);
  const int seg = bb % nseg;
  bb /= nseg;
  const int tile = bb % ntile, chunk = bb / ntile;
  const int kc = (NZ + nchunk - 1) / nchunk;
  const int kb = chunk * kc, ke = min(kb + kc, NZ);
  const int j0 = (tile * 4 + wid) * TY;
  const int i0 = seg * 128 + 2 * lane;
  dv2 va[TY], vb[TY];
  auto ld = [&](int k) {
    const long base = k * PLANE;
#pragma unroll
    for (int t = 0; t < TY; ++t) {
      va[t] = *(const dv2*)(a + base + (long)(j0 + t) * NX + i0);
      vb[t] = *(const dv2*)(b + base + (long)(j0 + t) * NX + i0);
    }
  };
  if (PF) ld(kb);
  for (int k = kb; k < ke; ++k) {
    dv2 ca[TY], cb[TY];
    if (PF) {
#pragma unroll
      for (int t = 0; t < TY; ++t) ca[t] = va[t], cb[t] = vb[t];
      ld(k + 1 < ke ? k + 1 : k);
    } else {
      ld(k);
#pragma unroll
      for (int t = 0; t < TY; ++t) ca[t] = va[t], cb[t] = vb[t];
    }
    const long base = k * PLANE;
#pragma unroll
    for (int t = 0; t < TY; ++t)
      __builtin_nontemporal_store(ca[t] + 0.5 * cb[t], (dv2*)(y + base + (long)(j0 + t) * NX + i0));
  }
}

__global__ __launch_bounds__(256) void flat_r2w1(const dv2* __restrict__ a, const dv2* __restrict__ b,
                                                 dv2* __restrict__ y, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    __builtin_nontemporal_store(a[i] + 0.5 * b[i], y + i);
}

int main() {
  const long N = PLANE * NZ;
  double *a, *b, *y;
  CK(hipMalloc(&a, N * 8));
  CK(hipMalloc(&b, N * 8));
  CK(hipMalloc(&y, N * 8));
  CK(hipMemset(a, 0, N * 8));
  CK(hipMemset(b, 0, N * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, int p1, int p2, auto launch) {
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
    printf("{\"kernel\":\"%s\",\"p1\":%d,\"p2\":%d,\"best_ms\":%.4f,\"avg_ms\":%.4f,\"GBps_avg\":%.1f}\n",
           name, p1, p2, best, tot / reps, 24.0 * N / (tot / reps) / 1e6);
    fflush(stdout);
  };
  for (int g : {1024, 2048, 4096})
    run("flat_r2w1", g, 0, [&] { flat_r2w1<<<g, 256>>>((const dv2*)a, (const dv2*)b, (dv2*)y, N / 2); });
  for (int nc : {2, 4, 8, 16}) {
    const int nb4 = (NX / 128) * (NY / 16) * nc, nb8 = (NX / 128) * (NY / 32) * nc;
    run("seg_ty4_pf0", 4, nc, [&] { zm_r2w1<4, 0><<<nb4, 256>>>(a, b, y, nc); });
    run("seg_ty4_pf1", 4, nc, [&] { zm_r2w1<4, 1><<<nb4, 256>>>(a, b, y, nc); });
    run("seg_ty8_pf0", 8, nc, [&] { zm_r2w1<8, 0><<<nb8, 256>>>(a, b, y, nc); });
    run("seg_ty8_pf1", 8, nc, [&] { zm_r2w1<8, 1><<<nb8, 256>>>(a, b, y, nc); });
  }
  return 0;
}
