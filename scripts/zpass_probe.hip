// zpass_probe.hip -- the HBM access pattern of the spectral preconditioner's Z pass (pb_fft.hip):
// tiles of TL x-adjacent z-lines of a 512^3 fp64 grid, i.e. TL*8-byte row pieces 2 MiB apart,
// read and written back with no arithmetic. How fast can that pattern stream, by piece width
// (TL) and by loads in flight per thread (NREG)? Against a flat grid-stride copy of the same
// bytes. Variant "lds": the tile goes through LDS as in the real kernel (TL <= 16).
// Build: hipcc -O3 --offload-arch=gfx950 -o zpass_probe zpass_probe.hip
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

// registers only: a block owns TL lines (x-adjacent) x KB planes; each thread moves NREG pairs
// per round (all loads issued before the stores)
template <int TL, int NREG, int KB>
__global__ __launch_bounds__(256) void tile_regs(const double* __restrict__ in,
                                                 double* __restrict__ out) {
  constexpr int PPR = TL / 2;             // pairs per row piece
  constexpr int NP = PPR * KB;            // pairs per block
  static_assert(NP % (256 * NREG) == 0, "whole rounds only (no out-of-range pairs)");
  static_assert(TL <= NX && NX % TL == 0 && NZ % KB == 0, "tiling");
  const int ntx = NX / TL;
  const int b = blockIdx.x;
  const int tx = b % ntx, rest = b / ntx;
  const int j = rest % NY, kb = (rest / NY) * KB;
  const long base = (long)kb * PLANE + (long)j * NX + tx * TL;
  for (int f0 = 0; f0 < NP; f0 += 256 * NREG) {
    dv2 v[NREG];
#pragma unroll
    for (int q = 0; q < NREG; ++q) {
      const int f = f0 + q * 256 + threadIdx.x;
      const int e = f / PPR, l = (f % PPR) * 2;
      v[q] = __builtin_nontemporal_load((const dv2*)(in + base + e * PLANE + l));
    }
#pragma unroll
    for (int q = 0; q < NREG; ++q) {
      const int f = f0 + q * 256 + threadIdx.x;
      const int e = f / PPR, l = (f % PPR) * 2;
      __builtin_nontemporal_store(v[q], (dv2*)(out + base + e * PLANE + l));
    }
  }
}

// through LDS as dht_lines_kernel<C=8, TL, LAYOUT 0> stages its tile (whole 512-long lines)
template <int TL>
__global__ __launch_bounds__(32 * TL) void tile_lds(const double* __restrict__ in,
                                                    double* __restrict__ out) {
  constexpr int n = NZ, LP = n + 1, NT = 32 * TL, NP = TL * n / 2;
  static_assert(NP % NT == 0 && NX % TL == 0, "tiling");
  extern __shared__ double lds[];
  const int ntx = NX / TL;
  const int tx = blockIdx.x % ntx, j = blockIdx.x / ntx;
  const long base = (long)j * NX + tx * TL;
#pragma unroll 4
  for (int f = threadIdx.x; f < NP; f += NT) {
    const int l = (f % (TL / 2)) * 2, e = f / (TL / 2);
    const dv2 v = __builtin_nontemporal_load((const dv2*)(in + base + e * PLANE + l));
    lds[l * LP + e] = v.x;
    lds[(l + 1) * LP + e] = v.y;
  }
  __syncthreads();
#pragma unroll 4
  for (int f = threadIdx.x; f < NP; f += NT) {
    const int l = (f % (TL / 2)) * 2, e = f / (TL / 2);
    dv2 v;
    v.x = lds[l * LP + e];
    v.y = lds[(l + 1) * LP + e];
    __builtin_nontemporal_store(v, (dv2*)(out + base + e * PLANE + l));
  }
}

// wave-direct: a block of NW waves owns 2 NW x-adjacent lines of one row j; wave w moves lines
// (2w, 2w+1) itself, lane l the elements e = l + 64 r (r < NZ / 64), one 16-B pair per element --
// the access of a Z-pass whose first and last Stockham passes run from registers (every wave
// instruction touches 64 rows; the NW waves of the block together cover each 2NW*8-byte piece)
template <int NW>
__global__ __launch_bounds__(64 * NW) void wave_direct(const double* __restrict__ in,
                                                      double* __restrict__ out) {
  constexpr int TL = 2 * NW, NR = NZ / 64;
  const int ntx = NX / TL;
  const int tx = blockIdx.x % ntx, j = blockIdx.x / ntx;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long base = (long)j * NX + tx * TL + 2 * w;
  dv2 v[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r)
    v[r] = __builtin_nontemporal_load((const dv2*)(in + base + (long)(lane + 64 * r) * PLANE));
#pragma unroll
  for (int r = 0; r < NR; ++r)
    __builtin_nontemporal_store(v[r], (dv2*)(out + base + (long)(lane + 64 * r) * PLANE));
}

__global__ __launch_bounds__(256) void flat_copy(const dv2* __restrict__ in, dv2* __restrict__ out,
                                                 long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load(in + i), out + i);
}

static double* g_in;
static double* g_out;

template <class F>
static void run(const char* name, int p1, int p2, F launch) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) launch();
  CK(hipDeviceSynchronize());
  float best = 1e30f, tot = 0.f;
  const int R = 10;
  for (int r = 0; r < R; ++r) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
    tot += ms;
  }
  CK(hipGetLastError());
  const double bytes = 16.0 * NX * NY * NZ;
  printf("{\"kernel\":\"%s\",\"p1\":%d,\"p2\":%d,\"best_ms\":%.4f,\"avg_ms\":%.4f,"
         "\"GBps_avg\":%.1f}\n", name, p1, p2, best, tot / R, bytes / (tot / R * 1e-3) / 1e9);
  fflush(stdout);
}

template <int TL, int NREG, int KB>
static void regs() {
  const int nb = (NX / TL) * NY * (NZ / KB);
  run("tile_regs", TL, NREG * 1000 + KB, [=] {
    hipLaunchKernelGGL((tile_regs<TL, NREG, KB>), dim3(nb), dim3(256), 0, 0, g_in, g_out);
  });
}

template <int TL>
static void run_lds() {
  const size_t sh = (size_t)TL * (NZ + 1) * 8;
  CK(hipFuncSetAttribute((const void*)tile_lds<TL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                         (int)sh));
  run("tile_lds", TL, 0, [=] {
    hipLaunchKernelGGL(tile_lds<TL>, dim3((NX / TL) * NY), dim3(32 * TL), sh, 0, g_in, g_out);
  });
}

template <int NW>
static void run_direct() {
  run("wave_direct", 2 * NW, 0, [=] {
    hipLaunchKernelGGL(wave_direct<NW>, dim3((NX / (2 * NW)) * NY), dim3(64 * NW), 0, 0, g_in,
                       g_out);
  });
}

int main() {
  const size_t n = (size_t)NX * NY * NZ;
  CK(hipMalloc(&g_in, n * 8));
  CK(hipMalloc(&g_out, n * 8));
  CK(hipMemset(g_in, 0, n * 8));
  run("flat_copy", 0, 0, [=] {
    hipLaunchKernelGGL(flat_copy, dim3(256 * 32), dim3(256), 0, 0, (const dv2*)g_in, (dv2*)g_out,
                       (long)(n / 2));
  });
  run_lds<16>();
  run_direct<4>();
  run_direct<8>();
  run_direct<16>();
  run_lds<16>();
  regs<16, 4, 512>();
  regs<64, 8, 64>();
  return 0;
}
