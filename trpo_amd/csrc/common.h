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


// Workgroup barrier for an LDS hand-off only: waits for this wave's LDS operations,
// not for its outstanding global loads.  __syncthreads() also emits vmcnt(0), which
// would drain a register prefetch that is meant to stay in flight across the barrier.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

}  // namespace trpo
