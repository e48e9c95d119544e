// Shared device-side definitions for the TRPO update engine (gfx950 / CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>

namespace trpo {

// trpo_inksci.py:16
constexpr float kEps = 1e-6f;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Number of blocks used by every grid-stride reduction that produces per-block
// partial sums.  Fixed, so that the final (ordered) sum is deterministic and
// every rank evaluates it identically.
constexpr int kRedBlocks = 256;
constexpr int kRedThreads = 256;

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// wave_sum_d's butterfly (partners l ^ 32, 16, 8, 4, 2, 1 in that order) on lane-crossing moves instead of
// ds_bpermute pairs: bit-identical on every lane.  Before the ^8 step every value depends on l mod 16 only, so a
// rotate by 8 inside the 16-lane row reaches an equal partner; likewise l mod 8 for ^4 (rotate by 4).
__device__ __forceinline__ double wave_sum_d_fast(double v);

// Block-wide sum in a fixed order (wave shuffles, then waves in index order).
// Every thread returns the total.  `scratch` must hold blockDim.x/64 doubles.
__device__ __forceinline__ double block_sum_d(double v, double* scratch) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_sum_d(v);
  __syncthreads();
  if (lane == 0) scratch[wave] = v;
  __syncthreads();
  double t = 0.0;
  for (int w = 0; w < nw; ++w) t += scratch[w];
  __syncthreads();
  return t;
}

// Sum of kRedBlocks per-block partials, evaluated identically by any caller.
__device__ __forceinline__ double sum_partials(const double* partials, int n, double* scratch) {
  double v = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) v += partials[i];
  return block_sum_d(v, scratch);
}


// ---- lane reductions on DPP moves (no LDS round trips) --------------------------------------
// Inside a 16-lane row: quad xor 1, quad xor 2, half-row mirror, row mirror.  After each step every
// lane of a 2^k group holds the group's value, so the mirror partner sits in the other group; every
// lane ends with the same value (both partners add the same two operands).  Across the two rows of a
// 32-lane half: v_permlane16_swap (below).
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u(unsigned v) {
  return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) { return __uint_as_float(dpp_u<CTRL>(__float_as_uint(v))); }
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = dpp_u<CTRL>((unsigned)b), hi = dpp_u<CTRL>((unsigned)(b >> 32));
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// v_permlane16_swap / v_permlane32_swap with both operands = v: the pair holds, in some order, this
// lane's value and that of lane l ^ 16 (resp. l ^ 32), so their sum / max is the same on both partners.
template <bool X32>
__device__ __forceinline__ void pair_u(unsigned v, unsigned& a, unsigned& b) {
  if constexpr (X32) {
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    a = p[0];
    b = p[1];
  } else {
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    a = p[0];
    b = p[1];
  }
}
template <bool X32>
__device__ __forceinline__ float xadd_f(float v) {
  unsigned a, b;
  pair_u<X32>(__float_as_uint(v), a, b);
  return __uint_as_float(a) + __uint_as_float(b);
}
template <bool X32>
__device__ __forceinline__ float xmax_f(float v) {
  unsigned a, b;
  pair_u<X32>(__float_as_uint(v), a, b);
  return fmaxf(__uint_as_float(a), __uint_as_float(b));
}
template <bool X32>
__device__ __forceinline__ double xadd_d(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  unsigned la, lb, ha, hb;
  pair_u<X32>((unsigned)u, la, lb);
  pair_u<X32>((unsigned)(u >> 32), ha, hb);
  return __builtin_bit_cast(double, ((unsigned long long)ha << 32) | la) +
         __builtin_bit_cast(double, ((unsigned long long)hb << 32) | lb);
}
constexpr int kDppX1 = 0xB1, kDppX2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;
constexpr int kDppRor4 = 0x124, kDppRor8 = 0x128;   // row_ror:4 / row_ror:8 (rotate within a 16-lane row)
__device__ __forceinline__ float sum16_dpp(float v) {
  v += dpp_f<kDppX1>(v);
  v += dpp_f<kDppX2>(v);
  v += dpp_f<kDppHalfMirror>(v);
  return v + dpp_f<kDppMirror>(v);
}
__device__ __forceinline__ double sum16_dpp(double v) {
  v += dpp_d<kDppX1>(v);
  v += dpp_d<kDppX2>(v);
  v += dpp_d<kDppHalfMirror>(v);
  return v + dpp_d<kDppMirror>(v);
}
__device__ __forceinline__ float sum32_dpp(float v) { return xadd_f<false>(sum16_dpp(v)); }
__device__ __forceinline__ double sum32_dpp(double v) { return xadd_d<false>(sum16_dpp(v)); }
__device__ __forceinline__ float max32_dpp(float v) {
  v = fmaxf(v, dpp_f<kDppX1>(v));
  v = fmaxf(v, dpp_f<kDppX2>(v));
  v = fmaxf(v, dpp_f<kDppHalfMirror>(v));
  v = fmaxf(v, dpp_f<kDppMirror>(v));
  return xmax_f<false>(v);
}

__device__ __forceinline__ double wave_sum_d_fast(double v) {
  v = xadd_d<true>(v);
  v = xadd_d<false>(v);
  v += dpp_d<0x128>(v);   // row_ror:8
  v += dpp_d<0x124>(v);   // row_ror:4
  v += dpp_d<0x4E>(v);    // quad xor 2
  return v + dpp_d<0xB1>(v);   // quad xor 1
}

// Workgroup barrier for an LDS hand-off only: waits for this wave's LDS operations,
// not for its outstanding global loads.  __syncthreads() also emits vmcnt(0), which
// would drain a register prefetch that is meant to stay in flight across the barrier.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

}  // namespace trpo
