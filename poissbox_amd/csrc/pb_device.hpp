// pb_device.hpp -- device-side helpers shared by the stencil engine (pb_stencil.hip) and the
// fused multigrid sweeps (pb_mg_sweep.hip): 16-byte row loads/stores, DPP wave shifts, the
// deterministic block reduction of partial sums, the XCD-aware block order.
#pragma once
#include "pb_internal.hpp"

namespace pb {

typedef double dv2 __attribute__((ext_vector_type(2)));

#ifndef PB_KWAVES
#define PB_KWAVES 4  // waves per workgroup (stacked in y)
#endif
static constexpr int kWaves = PB_KWAVES;
static constexpr int kThreads = 64 * kWaves;

template <int V>
__device__ __forceinline__ void load_row(const double* __restrict__ p, int64_t idx, double (&v)[V]) {
  if constexpr (V == 2) {
    const dv2 t = *reinterpret_cast<const dv2*>(p + idx);
    v[0] = t.x;
    v[1] = t.y;
  } else {
    v[0] = p[idx];
  }
}
// point-local rows read exactly once (epilogue operands): non-temporal loads, so they do not
// displace the halo rows neighbouring waves re-read from L2 (measured: CG pass B 3-7 % faster;
// the same on the z-queue rows, which ARE re-read as halos, made pass A 25 % slower)
template <int V>
__device__ __forceinline__ void load_row_nt(const double* __restrict__ p, int64_t idx,
                                            double (&v)[V]) {
  if constexpr (V == 2) {
    const dv2 t = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(p + idx));
    v[0] = t.x;
    v[1] = t.y;
  } else {
    v[0] = __builtin_nontemporal_load(p + idx);
  }
}
template <int V>
__device__ __forceinline__ void store_row(double* p, int64_t idx, const double (&v)[V], int nt) {
  if constexpr (V == 2) {
    dv2 t;
    t.x = v[0];
    t.y = v[1];
    if (nt) __builtin_nontemporal_store(t, reinterpret_cast<dv2*>(p + idx));
    else *reinterpret_cast<dv2*>(p + idx) = t;
  } else {
    if (nt) __builtin_nontemporal_store(v[0], p + idx);
    else p[idx] = v[0];
  }
}

// Row-element address split into a wave-uniform row offset (elements) and the lane's byte
// offset inside the row (32-bit): the loads/stores then take an SGPR base and ONE shared VGPR
// offset instead of a 64-bit VGPR address per row (fewer VGPRs, no spills in the tall kernels).
struct RowIx {
  int64_t row;    // uniform
  unsigned boff;  // lane byte offset
};
template <int V>
__device__ __forceinline__ void load_row(const double* __restrict__ p, RowIx ix, double (&v)[V]) {
  const char* q = reinterpret_cast<const char*>(p + ix.row) + ix.boff;
  if constexpr (V == 2) {
    const dv2 t = *reinterpret_cast<const dv2*>(q);
    v[0] = t.x;
    v[1] = t.y;
  } else {
    v[0] = *reinterpret_cast<const double*>(q);
  }
}
template <int V>
__device__ __forceinline__ void load_row_nt(const double* __restrict__ p, RowIx ix,
                                            double (&v)[V]) {
  const char* q = reinterpret_cast<const char*>(p + ix.row) + ix.boff;
  if constexpr (V == 2) {
    const dv2 t = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(q));
    v[0] = t.x;
    v[1] = t.y;
  } else {
    v[0] = __builtin_nontemporal_load(reinterpret_cast<const double*>(q));
  }
}
template <int V>
__device__ __forceinline__ void store_row(double* p, RowIx ix, const double (&v)[V], int nt) {
  char* q = reinterpret_cast<char*>(p + ix.row) + ix.boff;
  if constexpr (V == 2) {
    dv2 t;
    t.x = v[0];
    t.y = v[1];
    if (nt) __builtin_nontemporal_store(t, reinterpret_cast<dv2*>(q));
    else *reinterpret_cast<dv2*>(q) = t;
  } else {
    if (nt) __builtin_nontemporal_store(v[0], reinterpret_cast<double*>(q));
    else *reinterpret_cast<double*>(q) = v[0];
  }
}

// Stores through a buffer descriptor of one plane (base and size wave-uniform): an offset at or
// past the size is dropped by the range check, so a masked store needs no branch -- control flow
// in a z-march step makes the compiler merge its wait counts at the join (vmcnt(0): the prefetch
// drains; gfx9 counts stores in vmcnt too)
static constexpr unsigned kOob = 0x80000000u;  // a store offset past every plane: dropped
typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, int bytes) {
  // (inputs readfirstlane'd: a descriptor the compiler cannot prove uniform is waterfall'd)
  const uint64_t a = (uint64_t)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a),
                 hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  void* pa = (void*)(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(pa, (short)0, __builtin_amdgcn_readfirstlane(bytes),
                                           0x00020000);
}
// V consecutive doubles of a lane (V = 2: one 16-B store, V = 1: 8 B); AUX 2: non-temporal
template <int V, int AUX = 0>
__device__ __forceinline__ void store_pts(__amdgpu_buffer_rsrc_t rs, unsigned off,
                                          const double (&v)[V]) {
  if constexpr (V == 2) {
    const dv2 d{v[0], v[1]};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, d), rs, (int)off, 0, AUX);
  } else {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v[0]), rs, (int)off, 0, AUX);
  }
}

// ---------------------------------------------------------------------------------------------
// Cross-lane helpers (DPP wave shifts: VALU only, no LDS traffic; bound_ctrl: the end lane
// with no source reads 0, no old-value operand to initialise)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double dpp_from_lower(double v) {  // lane l <- lane l-1 (wave_shr:1)
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, 0x138, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x138, 0xf, 0xf, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double dpp_from_upper(double v) {  // lane l <- lane l+1 (wave_shl:1)
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, 0x130, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x130, 0xf, 0xf, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// ---------------------------------------------------------------------------------------------
// Block-level deterministic reduction of NS partial sums -> parts[block*NS + s]
// ---------------------------------------------------------------------------------------------
template <int NS>
__device__ __forceinline__ void block_partials(double* acc, double* parts) {
  if constexpr (NS > 0) {
    // any block size up to 16 waves (the engine's kWaves, 256-thread elementwise kernels)
    __shared__ double red[16][NS];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      double v = acc[s];
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
      acc[s] = v;
    }
    if (lane == 0) {
#pragma unroll
      for (int s = 0; s < NS; ++s) red[wid][s] = acc[s];
    }
    __syncthreads();
    if (threadIdx.x < NS) {
      double v = 0.0;
#pragma unroll
      for (int w = 0; w < nw; ++w) v += red[w][threadIdx.x];
      parts[(int64_t)blockIdx.x * NS + threadIdx.x] = v;
    }
  }
}

// XCD-aware block order (speed only, bijective): the dispatcher deals blocks round-robin over the
// 8 XCDs, so each XCD gets a contiguous range of logical blocks -- neighbouring tiles then share
// the XCD's L2 and their halo rows hit there.
__device__ __forceinline__ int xcd_block(int remap) {
  int b = blockIdx.x;
  if (remap) {
    const int nb = gridDim.x, q = nb / 8, r = nb % 8;
    const int xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
    b = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  return b;
}

}  // namespace pb
