// Backward through the softmax head's layer for the prepare pass and the policy gradient in one read of
// H_{L-1} (gfx950).  Both are row GEMMs with K = n_actions (<= 32) into the last hidden layer:
//   D_{L-2}  = (D_{L-1}  W^T) (1 - H^2)     KL_ff plain delta   (trpo_inksci.py:56-57 through flatgrad, :69)
//   DS_{L-2} = (DS_{L-1} W^T) (1 - H^2)     surr delta          (trpo_inksci.py:54)
// (SURVEY.md Appendix A).  At K <= 32 the product is a few FMAs per output: the kernel is bound by its
// HBM streams (H in, two outputs), so it reads H once for both instead of once per backward.  It can also
// write D_{L-2}'s scaled f16 hi plane (the fused R-backward's one-product D_1 V_1^T segment, rbwd0.hip)
// with one power-of-two scale per 32-row tile, which replaces the separate split_planes pass over D_{L-2}.
//
// Layout: one thread per hidden column, a workgroup walks 32-row tiles (grid stride); the tile's head
// deltas are staged in LDS and broadcast.  Sums run k = 0 .. A-1 as f32 fmaf chains (exact f32, as the
// f32 MFMA row GEMM they replace; the order differs, the rounding level does not).
#include "common.h"
#include "kernels.h"

#include <stdexcept>

namespace trpo {
namespace {

constexpr int kHbRows = 32;     // rows per tile
constexpr int kHbThreads = 256; // one hidden column per thread (Npad <= 256)
constexpr int kHbA = 32;        // max actions

// AT: actions rounded up to a multiple of 4 (the register image of W^T's column)
template <int AT>
__global__ void __launch_bounds__(kHbThreads) head_bwd2_kernel(const HeadBwd2Args a) {
  __shared__ __attribute__((aligned(16))) float sd[2][kHbRows][AT];
  __shared__ float sv[kHbRows][kHbThreads];   // the tile's D values, kept for the hi plane's tile scale
  __shared__ float sred[3][kHbThreads / 64];
  const int c = threadIdx.x, lane = c & 63, wv = c >> 6;
  const bool cv = c < a.Npad;
  float w[AT];
#pragma unroll
  for (int j = 0; j < AT; ++j) w[j] = (cv && j < a.A) ? a.WB[(size_t)j * a.Npad + c] : 0.0f;
  float mx1 = 0.0f, mx2 = 0.0f;
  // the policy gradient's last-layer weight gradient over this split's rows (slab != NULL): gw[j] = sum_r H[r][c]
  // DS2[r][j], column c's row of the W block, and the bias column sum of DS2 (thread j < A)
  const bool wg = a.slab != nullptr;
  float gw[AT];
#pragma unroll
  for (int j = 0; j < AT; ++j) gw[j] = 0.0f;
  float gb = 0.0f;
  // workgroup s walks split s's rows (the weight-gradient slabs' partition, engine set_splits)
  const int r0 = blockIdx.x * a.rows_per_split;
  const int r1 = min(a.rows, r0 + a.rows_per_split);
  for (int t0 = r0; t0 < r1; t0 += kHbRows) {
    const int tile = t0 / kHbRows;
    const int nr = min(kHbRows, r1 - t0);
    __syncthreads();   // the previous tile's deltas and values are consumed
    for (int i = c; i < 2 * kHbRows * AT; i += kHbThreads) {
      const int m = i / (kHbRows * AT), r = (i / AT) % kHbRows, j = i % AT;
      const float* src = m ? a.DS2 : a.D2;
      sd[m][r][j] = (r < nr && j < a.A) ? src[(size_t)(t0 + r) * a.Apad + j] : 0.0f;
    }
    __syncthreads();
    float tm = 0.0f;
#pragma unroll 4
    for (int r = 0; r < kHbRows; ++r) {
      float d = 0.0f, s = 0.0f;
#pragma unroll
      for (int j = 0; j < AT; j += 4) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(&sd[0][r][j]);
        const f32x4 y = *reinterpret_cast<const f32x4*>(&sd[1][r][j]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          d = fmaf(x[q], w[j + q], d);
          s = fmaf(y[q], w[j + q], s);
        }
      }
      float o1 = 0.0f;
      if (r < nr && cv) {
        const size_t idx = (size_t)(t0 + r) * a.Npad + c;
        const float h = a.H[idx];
        if (wg) {
#pragma unroll
          for (int j = 0; j < AT; j += 4) {
            const f32x4 y = *reinterpret_cast<const f32x4*>(&sd[1][r][j]);
#pragma unroll
            for (int q = 0; q < 4; ++q) gw[j + q] = fmaf(h, y[q], gw[j + q]);
          }
        }
        const float om = (1.0f - h) * (1.0f + h);
        o1 = d * om;
        const float o2 = s * om;
        a.D1[idx] = o1;
        a.DS1[idx] = o2;
        mx1 = fmaxf(mx1, fabsf(o1));
        mx2 = fmaxf(mx2, fabsf(o2));
        tm = fmaxf(tm, fabsf(o1));
      }
      sv[r][c] = o1;
      if (wg && c < a.A && r < nr) gb += sd[1][r][c];
    }
    if (a.D1h) {
      // the tile's scale: max |D| over its rows and every column
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) tm = fmaxf(tm, __shfl_xor(tm, off, 64));
      if (lane == 0) sred[2][wv] = tm;
      __syncthreads();
      float m = 0.0f;
#pragma unroll
      for (int u = 0; u < kHbThreads / 64; ++u) m = fmaxf(m, sred[2][u]);
      const int e = f16_scale_exp(m);
      const float sc = __builtin_ldexpf(1.0f, e);
      if (c == 0) a.eD1t[tile] = e;
      if (cv) {
        uint16_t* dst = a.D1h + ((size_t)(c >> 5) * a.d1_mpad + t0) * 32 + (c & 31);
        for (int r = 0; r < nr; ++r) dst[(size_t)r * 32] = __builtin_bit_cast(unsigned short, (_Float16)(sv[r][c] * sc));
      }
    }
  }
  if (wg) {
    float* out = a.slab + (size_t)blockIdx.x * a.slab_stride;
    if (c < a.N) {
#pragma unroll
      for (int j = 0; j < AT; ++j)
        if (j < a.A) out[a.off_w + (int64_t)c * a.A + j] = gw[j];
    }
    if (c < a.A) out[a.off_b + c] = gb;
  }
  // running maxima of both outputs (the f16 split scales of their consumers): one atomicMax per workgroup
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mx1 = fmaxf(mx1, __shfl_xor(mx1, off, 64));
    mx2 = fmaxf(mx2, __shfl_xor(mx2, off, 64));
  }
  __syncthreads();
  if (lane == 0) {
    sred[0][wv] = mx1;
    sred[1][wv] = mx2;
  }
  __syncthreads();
  if (c < 2) {
    unsigned* slot = c == 0 ? a.am_d1 : a.am_ds1;
    if (slot) {
      float m = 0.0f;
#pragma unroll
      for (int u = 0; u < kHbThreads / 64; ++u) m = fmaxf(m, sred[c][u]);
      if (m > 0.0f) atomicMax(slot + (blockIdx.x % kAmaxSub) * kAmaxStride, __float_as_uint(m));
    }
  }
}

}  // namespace

bool head_bwd2_eligible(int A, int Npad) { return A <= kHbA && Npad <= kHbThreads && Npad % 4 == 0; }

void launch_head_bwd2(const HeadBwd2Args& a, int num_cus, hipStream_t s) {
  if (a.rows <= 0) return;
  if (!head_bwd2_eligible(a.A, a.Npad) || a.Apad < a.A || !a.WB || !a.D2 || !a.DS2 || !a.H || !a.D1 || !a.DS1)
    throw std::runtime_error("head_bwd2: unsupported shape or missing operand");
  if (a.D1h && (!a.eD1t || a.d1_mpad < a.rows || a.Npad % 32))
    throw std::runtime_error("head_bwd2: hi plane without its exponents or stride");
  (void)num_cus;
  if (a.splits <= 0 || a.rows_per_split % kHbRows || (int64_t)a.splits * a.rows_per_split < a.rows)
    throw std::runtime_error("head_bwd2: splits do not cover the rows in 32-row tiles");
  const int grid = a.splits;
  switch ((a.A + 3) / 4) {
    case 1: hipLaunchKernelGGL(head_bwd2_kernel<4>, dim3(grid), dim3(kHbThreads), 0, s, a); break;
    case 2: hipLaunchKernelGGL(head_bwd2_kernel<8>, dim3(grid), dim3(kHbThreads), 0, s, a); break;
    case 3: hipLaunchKernelGGL(head_bwd2_kernel<12>, dim3(grid), dim3(kHbThreads), 0, s, a); break;
    case 4: hipLaunchKernelGGL(head_bwd2_kernel<16>, dim3(grid), dim3(kHbThreads), 0, s, a); break;
    case 5: hipLaunchKernelGGL(head_bwd2_kernel<20>, dim3(grid), dim3(kHbThreads), 0, s, a); break;
    case 6: hipLaunchKernelGGL(head_bwd2_kernel<24>, dim3(grid), dim3(kHbThreads), 0, s, a); break;
    case 7: hipLaunchKernelGGL(head_bwd2_kernel<28>, dim3(grid), dim3(kHbThreads), 0, s, a); break;
    default: hipLaunchKernelGGL(head_bwd2_kernel<32>, dim3(grid), dim3(kHbThreads), 0, s, a); break;
  }
}

}  // namespace trpo
