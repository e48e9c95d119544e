// Backward through the softmax head's layer for the prepare pass and the policy gradient in one read of
// H_{L-1} (gfx950).  Both are row GEMMs with K = n_actions (<= 32) into the last hidden layer:
//   D_{L-2}  = (D_{L-1}  W^T) (1 - H^2)     KL_ff plain delta   (trpo_inksci.py:56-57 through flatgrad, :69)
//   DS_{L-2} = (DS_{L-1} W^T) (1 - H^2)     surr delta          (trpo_inksci.py:54)
// (SURVEY.md Appendix A).  At K <= 32 the product is a few FMAs per output: the kernel is bound by its
// HBM streams (H in, two outputs), so it reads H once for both instead of once per backward.  It can also
// write D_{L-2}'s scaled f16 hi plane (the fused R-backward's one-product D_1 V_1^T segment, rbwd0.hip)
// with one power-of-two scale per 32-row tile, which replaces the separate split_planes pass over D_{L-2}.
//
// Layout: one thread per hidden column, a workgroup walks its split's 32-row tiles; the tile's head deltas
// are staged in LDS and broadcast, and the next tile's H and deltas are loaded while the current one computes.
// Sums run k = 0 .. A-1 as f32 fmaf chains (exact f32, as the f32 MFMA row GEMM they replace; the order
// differs, the rounding level does not).
#include "common.h"
#include "kernels.h"

#include <algorithm>
#include <stdexcept>

namespace trpo {
namespace {

constexpr int kHbRows = 32;     // rows per tile
constexpr int kHbThreads = 256; // one hidden column per thread (Npad <= 256)
constexpr int kHbA = 32;        // max actions

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

// AT: actions rounded up to a multiple of 4 (the register image of W^T's column)
template <int AT>
__global__ void __launch_bounds__(kHbThreads) head_bwd2_kernel(const HeadBwd2Args a) {
  __shared__ __attribute__((aligned(16))) float sd[2][kHbRows][AT];
  // the tile's H values (column c is thread c's own), then in place the D values kept for the hi plane's tile scale
  __shared__ float sv[kHbRows][kHbThreads];
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
  // one tile ahead in registers: column c of the tile's 32 H rows, and this thread's share of the head deltas
  // (2 x 32 x AT floats over 256 threads); they move to LDS at the top of the tile, so the next tile's loads
  // are in flight during this tile's FMAs
  constexpr int kSt = 2 * kHbRows * AT / kHbThreads;
  float hc[kHbRows], pc[kSt];
  auto load = [&](int t0, float (&hv)[kHbRows], float (&pv)[kSt]) {
    const int nr = min(kHbRows, r1 - t0);
#pragma unroll
    for (int r = 0; r < kHbRows; ++r) hv[r] = (r < nr && cv) ? a.H[(size_t)(t0 + r) * a.Npad + c] : 0.0f;
#pragma unroll
    for (int u = 0; u < kSt; ++u) {
      const int i = c + u * kHbThreads;
      const int m = i / (kHbRows * AT), r = (i / AT) % kHbRows, j = i % AT;
      const float* src = m ? a.DS2 : a.D2;
      pv[u] = (r < nr && j < a.A) ? src[(size_t)(t0 + r) * a.Apad + j] : 0.0f;
    }
  };
  if (r0 < r1) load(r0, hc, pc);
  for (int t0 = r0; t0 < r1; t0 += kHbRows) {
    const int tile = t0 / kHbRows;
    const int nr = min(kHbRows, r1 - t0);
    __syncthreads();   // the previous tile's deltas and values are consumed
#pragma unroll
    for (int u = 0; u < kSt; ++u) (&sd[0][0][0])[c + u * kHbThreads] = pc[u];
#pragma unroll
    for (int r = 0; r < kHbRows; ++r) sv[r][c] = hc[r];
    __syncthreads();
    if (t0 + kHbRows < r1) load(t0 + kHbRows, hc, pc);   // in flight during this tile's FMAs
    // the tile's own weight-gradient partials, added to the split's sums once per tile: a split is ~15k rows
    // at C4, and one f32 running sum over all of them would carry ~sqrt(n) roundings
    float tw[AT];
#pragma unroll
    for (int j = 0; j < AT; ++j) tw[j] = 0.0f;
    float tb = 0.0f;
    float tm = 0.0f;
#pragma unroll 2
    for (int r = 0; r < kHbRows; ++r) {
      float d = 0.0f, s = 0.0f;
      const float h = sv[r][c];
#pragma unroll
      for (int j = 0; j < AT; j += 4) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(&sd[0][r][j]);
        const f32x4 y = *reinterpret_cast<const f32x4*>(&sd[1][r][j]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          d = fmaf(x[q], w[j + q], d);
          s = fmaf(y[q], w[j + q], s);
          // rows past the end have h = 0; without a slab tw is computed and dropped (under a branch on the
          // uniform slab pointer the compiler issued a select after every FMA: 20 VALU per row at 18 actions)
          tw[j + q] = fmaf(h, y[q], tw[j + q]);
        }
      }
      const float om = (1.0f - h) * (1.0f + h);
      const float o1 = d * om;
      const float o2 = s * om;
      if (r < nr && cv) {
        const size_t idx = (size_t)(t0 + r) * a.Npad + c;
        a.D1[idx] = o1;
        a.DS1[idx] = o2;
        if (a.E1) a.E1[idx] = -2.0f * d * h;
        mx1 = fmaxf(mx1, fabsf(o1));
        mx2 = fmaxf(mx2, fabsf(o2));
        tm = fmaxf(tm, fabsf(o1));
      }
      sv[r][c] = o1;
      if (wg && c < a.A) tb += sd[1][r][c];   // rows past the end were staged as 0
    }
    if (wg) {
#pragma unroll
      for (int j = 0; j < AT; ++j) gw[j] += tw[j];
      gb += tb;
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

// ---------------------------------------------------------------------------------------------------------
// The same three contractions on f32 MFMA (option hbwd2 = 2): v_mfma_f32_32x32x2_f32 is exact f32, the fmaf
// chains' own arithmetic (MI355X_MICROARCH.md), but one instruction does 2 x 32 x 32 of them with operands
// in registers, where the kernel above spends one LDS broadcast and three VALU FMAs per action, row and
// column (2.55e9 VALU instructions per C4 launch, VALU-issue bound: profiles/r4ao).
//   * 8 waves; wave w owns hidden columns [32w, 32w + 32); 32-row tiles of the workgroup's split.
//   * D / DS: C[row][col] = sum_j D2[row][j] W[col][j]: A = the tile's D2 / DS2 rows from LDS (lane = row,
//     k = j), B = W^T held in registers for the launch (lane = column, k = j): k-step s takes actions 2s, 2s+1,
//     so each output is the fmaf chain j = 0, 1, .. of the VALU kernel.
//   * the outputs come out in C layout (lane = column, registers = rows), the layout H is loaded in for
//     (1 - H^2) and the row-coalesced stores.
//   * weight gradient H^T DS2 (K = rows): A = H's C-layout registers themselves (k-step s = register s: lane
//     half h supplies row (s&3) + 8(s>>2) + 4h), B = DS2 from LDS at the same rows (lane = action).
// ---------------------------------------------------------------------------------------------------------
constexpr int kHmW = 8;   // waves

__device__ __forceinline__ float ldbf(__amdgpu_buffer_rsrc_t r, int vo, int so) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
}

template <int K2>   // k-steps of the action contraction: ceil(A / 2)
__global__ void __launch_bounds__(kHmW * 64, 2) head_bwd2m_kernel(const HeadBwd2Args a) {
  __shared__ float sd[2][kHbRows][kHbA + 1];   // the tile's D2 / DS2 rows, zero past A (pad: conflict-free reads)
  __shared__ float sred[3][kHmW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, lr = lane & 31, lh = lane >> 5;
  const int col = 32 * w + lr;
  const bool cv = col < a.Npad;
  constexpr int kOob = 0x40000000;
  const int vo = cv ? ((4 * lh) * a.Npad + col) * 4 : kOob;   // C layout: lane = column, register i = row r(i)
  auto roff = [](int i) { return (i & 3) + 8 * (i >> 2); };
  // W^T in registers: k-step s, lane half h -> action 2s + h
  float wf[K2];
#pragma unroll
  for (int s = 0; s < K2; ++s) {
    const int j = 2 * s + lh;
    wf[s] = (cv && j < a.A) ? a.WB[(size_t)j * a.Npad + col] : 0.0f;
  }
  const bool wg = a.slab != nullptr;
  f32x16 gw = f32x16{};   // H^T DS2 over the split: lane = action, registers = columns 32w + r(i) + 4h
  float gb = 0.0f;        // DS2 column sums (thread j < A)
  float mx1 = 0.0f, mx2 = 0.0f;
  const int r0 = blockIdx.x * a.rows_per_split;
  const int r1 = min(a.rows, r0 + a.rows_per_split);
  auto desc = [&](const void* p, int t0, int ld, int esz) {
    const int nr = max(0, min(kHbRows, r1 - t0));
    return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p + (size_t)t0 * ld * esz), 0, nr * ld * esz,
                                             0x00020000);
  };
  // one tile ahead in registers: the H column block and this thread's share of the head deltas
  constexpr int kSt = 2 * kHbRows * kHbA / (kHmW * 64);   // 4
  float hc[16], pc[kSt];
  auto load = [&](int t0, float (&hv)[16], float (&pv)[kSt]) {
    const __amdgpu_buffer_rsrc_t rH = desc(a.H, t0, a.Npad, 4);
#pragma unroll
    for (int i = 0; i < 16; ++i) hv[i] = ldbf(rH, vo, roff(i) * a.Npad * 4);
    const __amdgpu_buffer_rsrc_t rD = desc(a.D2, t0, a.Apad, 4), rS = desc(a.DS2, t0, a.Apad, 4);
#pragma unroll
    for (int u = 0; u < kSt; ++u) {
      const int i = tid + u * kHmW * 64;
      const int m = i / (kHbRows * kHbA), r = (i / kHbA) % kHbRows, j = i % kHbA;
      const int v = j < a.A ? (r * a.Apad + j) * 4 : kOob;
      pv[u] = ldbf(m ? rS : rD, v, 0);
    }
  };
  if (r0 < r1) load(r0, hc, pc);
  for (int t0 = r0; t0 < r1; t0 += kHbRows) {
    const int tile = t0 / kHbRows;
    __syncthreads();   // the previous tile's deltas are consumed
#pragma unroll
    for (int u = 0; u < kSt; ++u) {
      const int i = tid + u * kHmW * 64;
      const int m = i / (kHbRows * kHbA), r = (i / kHbA) % kHbRows, j = i % kHbA;
      sd[m][r][j] = pc[u];
    }
    float h[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) h[i] = hc[i];
    __syncthreads();
    if (t0 + kHbRows < r1) load(t0 + kHbRows, hc, pc);   // in flight during this tile's MFMAs
    // D / DS: the fmaf chains over the actions, two per MFMA
    f32x16 ad = f32x16{}, as = f32x16{};
#pragma unroll
    for (int s = 0; s < K2; ++s) {
      ad = __builtin_amdgcn_mfma_f32_32x32x2f32(sd[0][lr][2 * s + lh], wf[s], ad, 0, 0, 0);
      as = __builtin_amdgcn_mfma_f32_32x32x2f32(sd[1][lr][2 * s + lh], wf[s], as, 0, 0, 0);
    }
    // the policy gradient's last-layer weight gradient: this tile's partial (one f32 chain per tile, added to
    // the split's sums once: a split is thousands of rows)
    if (wg) {
      f32x16 g = f32x16{};
#pragma unroll
      for (int s = 0; s < 16; ++s)
        g = __builtin_amdgcn_mfma_f32_32x32x2f32(h[s], sd[1][roff(s) + 4 * lh][lr], g, 0, 0, 0);
      gw += g;
      if (tid < a.A) {
        float tb = 0.0f;
#pragma unroll 8
        for (int r = 0; r < kHbRows; ++r) tb += sd[1][r][tid];   // rows past the end were staged as 0
        gb += tb;
      }
    }
    const __amdgpu_buffer_rsrc_t rD1 = desc(a.D1, t0, a.Npad, 4), rS1 = desc(a.DS1, t0, a.Npad, 4);
    const __amdgpu_buffer_rsrc_t rE1 = desc(a.E1 ? a.E1 : a.D1, t0, a.Npad, 4);
    float tm = 0.0f;
    float o1[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float hh = h[i];
      const float om = (1.0f - hh) * (1.0f + hh);
      o1[i] = ad[i] * om;
      const float o2 = as[i] * om;
      const int so = roff(i) * a.Npad * 4;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o1[i]), rD1, vo, so, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o2), rS1, vo, so, 0);
      if (a.E1)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, -2.0f * ad[i] * hh), rE1, vo, so, 0);
      mx1 = fmaxf(mx1, fabsf(o1[i]));   // rows past the end: H = 0 and D2 = 0 -> 0
      mx2 = fmaxf(mx2, fabsf(o2));
      tm = fmaxf(tm, fabsf(o1[i]));
    }
    if (a.D1h) {
      // D_1's hi plane with the tile's scale: max |D| over its rows and every column
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) tm = fmaxf(tm, __shfl_xor(tm, off, 64));
      if (lane == 0) sred[2][w] = tm;
      __syncthreads();
      float m = 0.0f;
#pragma unroll
      for (int u = 0; u < kHmW; ++u) m = fmaxf(m, sred[2][u]);
      const int e = f16_scale_exp(m);
      const float sc = __builtin_ldexpf(1.0f, e);
      if (tid == 0) a.eD1t[tile] = e;
      // k-blocked [column / 32][row][32]: this wave's block, rows t0 .. (past the end: dropped)
      const int nr = max(0, min(kHbRows, r1 - t0));
      const __amdgpu_buffer_rsrc_t rP = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.D1h + ((size_t)w * a.d1_mpad + t0) * 32), 0, cv ? nr * 64 : 0, 0x00020000);
#pragma unroll
      for (int i = 0; i < 16; ++i)
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)(o1[i] * sc)), rP,
                                              ((roff(i) + 4 * lh) * 32 + lr) * 2, 0, 0);
    }
  }
  if (wg) {
    float* out = a.slab + (size_t)blockIdx.x * a.slab_stride;
    if (lr < a.A) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = 32 * w + roff(i) + 4 * lh;
        if (c < a.N) out[a.off_w + (int64_t)c * a.A + lr] = gw[i];
      }
    }
    if (tid < a.A) out[a.off_b + tid] = gb;
  }
  // running maxima of both outputs (the f16 split scales of their consumers): one atomicMax per workgroup
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mx1 = fmaxf(mx1, __shfl_xor(mx1, off, 64));
    mx2 = fmaxf(mx2, __shfl_xor(mx2, off, 64));
  }
  __syncthreads();
  if (lane == 0) {
    sred[0][w] = mx1;
    sred[1][w] = mx2;
  }
  __syncthreads();
  if (tid < 2) {
    unsigned* slot = tid == 0 ? a.am_d1 : a.am_ds1;
    if (slot) {
      float m = 0.0f;
#pragma unroll
      for (int u = 0; u < kHmW; ++u) m = fmaxf(m, sred[tid][u]);
      if (m > 0.0f) atomicMax(slot + (blockIdx.x % kAmaxSub) * kAmaxStride, __float_as_uint(m));
    }
  }
}

}  // namespace

bool head_bwd2_eligible(int A, int Npad) { return A <= kHbA && Npad <= kHbThreads && Npad % 4 == 0; }

void launch_head_bwd2(const HeadBwd2Args& a, int num_cus, hipStream_t s) {
  if (a.rows <= 0) return;
  if (!head_bwd2_eligible(a.A, a.Npad) || a.Apad != (a.A + 3) / 4 * 4 || !a.WB || !a.D2 || !a.DS2 || !a.H || !a.D1 || !a.DS1)
    throw std::runtime_error("head_bwd2: unsupported shape or missing operand");
  if (a.D1h && (!a.eD1t || a.d1_mpad < a.rows || a.Npad % 32))
    throw std::runtime_error("head_bwd2: hi plane without its exponents or stride");
  (void)num_cus;
  if (a.splits <= 0 || a.rows_per_split % kHbRows || (int64_t)a.splits * a.rows_per_split < a.rows)
    throw std::runtime_error("head_bwd2: splits do not cover the rows in 32-row tiles");
  const int grid = a.splits;
  if (g_options.hbwd2 == 2) {
    switch ((a.A + 1) / 2) {
#define HBM_CASE(k) case k: hipLaunchKernelGGL(head_bwd2m_kernel<k>, dim3(grid), dim3(kHmW * 64), 0, s, a); break;
      HBM_CASE(1) HBM_CASE(2) HBM_CASE(3) HBM_CASE(4) HBM_CASE(5) HBM_CASE(6) HBM_CASE(7) HBM_CASE(8)
      HBM_CASE(9) HBM_CASE(10) HBM_CASE(11) HBM_CASE(12) HBM_CASE(13) HBM_CASE(14) HBM_CASE(15)
      default: hipLaunchKernelGGL(head_bwd2m_kernel<16>, dim3(grid), dim3(kHmW * 64), 0, s, a); break;
#undef HBM_CASE
    }
    return;
  }
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

// =============================================================================================================
// Softmax head forward, one state per lane (gfx950): z = H_{L-1} W_L + b_L (K = last hidden width, N = n_actions
// <= 32), p = softmax(z) and the row terms of surr / kl / ent (trpo_inksci.py:38-53), plus for the prepare pass
// the KL_ff plain logit delta D_L and the surr logit delta DS_L (cancellation-free forms, as gemm.hip's kPrepHead
// row epilogue).  K <= 256 and N <= 32 make the product a few thousand FMAs per state: the launch is bound by its
// read of H, so it runs on f32 VALU FMAs with the state's whole softmax row in one lane (no cross-lane sums), the
// H tile staged through LDS in 32-column chunks (the next chunk's loads in flight during the current one's FMAs).
// =============================================================================================================
namespace trpo {
namespace {

constexpr int kHfRows = 256;   // states per tile (one per thread)
constexpr int kHfK = 32;       // columns of H per chunk
constexpr int kHfLd = kHfK + 1;

template <int AT, bool PREP>
__global__ void __launch_bounds__(kHfRows, PREP ? (AT <= 20 ? 3 : 2) : (AT <= 28 ? 4 : 3)) head_fwd_kernel(const HeadFwdArgs a) {
  __shared__ float sH[kHfRows * kHfLd];
  __shared__ __attribute__((aligned(16))) float sW[kHfK][AT];
  __shared__ float sred[2][kHfRows / 64];
  const int t = threadIdx.x;
  const int nchunk = (a.K + kHfK - 1) / kHfK;
  float mD = 0.0f, mS = 0.0f;
  for (int64_t t0 = (int64_t)blockIdx.x * kHfRows; t0 < a.rows; t0 += (int64_t)gridDim.x * kHfRows) {
    const int nr = (int)min<int64_t>(kHfRows, a.rows - t0);
    // chunk loads: thread t moves float4 q of rows t / 8 + 32 q, columns 4 (t % 8) .. + 3 of the chunk
    f32x4 nx[8];
    auto load_chunk = [&](int c) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = t / 8 + 32 * q, col = kHfK * c + 4 * (t % 8);
        nx[q] = (r < nr && col < a.Kpad) ? *reinterpret_cast<const f32x4*>(a.H + (t0 + r) * a.Kpad + col)
                                         : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      }
    };
    f32x2 acc2[AT / 2];   // output pairs: one packed FMA per pair
#pragma unroll
    for (int j = 0; j < AT / 2; ++j) acc2[j] = f32x2{0.0f, 0.0f};
    load_chunk(0);
    for (int c = 0; c < nchunk; ++c) {
      __syncthreads();   // the previous chunk's reads are done
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = t / 8 + 32 * q, col = 4 * (t % 8);
#pragma unroll
        for (int e = 0; e < 4; ++e) sH[r * kHfLd + col + e] = nx[q][e];
      }
      for (int i = t; i < kHfK * AT; i += kHfRows) {
        const int k = i / AT, j = i % AT, kk = kHfK * c + k;
        sW[k][j] = (kk < a.K && j < a.A) ? a.W[(size_t)kk * a.Apad + j] : 0.0f;
      }
      __syncthreads();
      if (c + 1 < nchunk) load_chunk(c + 1);
#pragma unroll 8
      for (int k = 0; k < kHfK; ++k) {
        const float h = sH[t * kHfLd + k];
#pragma unroll
        for (int j = 0; j < AT; j += 4) {
          const f32x4 w4 = *reinterpret_cast<const f32x4*>(&sW[k][j]);
          acc2[j / 2] = pk_fma(f32x2{h, h}, f32x2{w4[0], w4[1]}, acc2[j / 2]);
          acc2[j / 2 + 1] = pk_fma(f32x2{h, h}, f32x2{w4[2], w4[3]}, acc2[j / 2 + 1]);
        }
      }
    }
    constexpr int ldo = AT + 1;   // [row][AT + 1] images in sH (free after the chunk loop)
    static_assert(ldo <= kHfLd, "head_fwd row images");
    // the row's softmax, loss terms and (PREP) the values its P / D / DS rows are made of; threads past the tile's
    // rows keep zeros
    float p[AT];
    float spB = 0.0f, rest = 0.0f, coef = 0.0f;
    int av = -1;
#pragma unroll
    for (int j = 0; j < AT; ++j) p[j] = 0.0f;
    if (t < nr) {
      const int64_t row = t0 + t;
      const float* oldr = a.old + row * a.Apad;
      float z[AT];
      float zm = -INFINITY;
#pragma unroll
      for (int j = 0; j < AT; ++j) {
        z[j] = j < a.A ? acc2[j / 2][j % 2] + a.bias[j] : -INFINITY;
        zm = fmaxf(zm, z[j]);
      }
      float es = 0.0f;
#pragma unroll
      for (int j = 0; j < AT; ++j) {
        p[j] = j < a.A ? expf(z[j] - zm) : 0.0f;
        es += p[j];
      }
#pragma unroll
      for (int j = 0; j < AT; ++j) p[j] = p[j] / es;
      av = a.act[row];
      const float adv = a.adv[row];
      float pa = 0.0f, olda = 0.0f;
      float klp = 0.0f, enp = 0.0f;
#pragma unroll
      for (int j = 0; j < AT; ++j) {
        if (j < a.A) {
          const float oj = oldr[j];
          if (j == av) {
            pa = p[j];
            olda = oj;
          }
          // the reference's own precision (f32 tensors, trpo_inksci.py:50-51): f32 logs and row sums (gemm.hip's
          // row heads alike); the sums over rows are f64
          klp += oj * logf((oj + kEps) / (p[j] + kEps));
          enp += -p[j] * logf(p[j] + kEps);
        }
      }
      double* rt = a.rowterms + 4 * row;
      rt[0] = (double)pa / (double)olda * (double)adv;
      rt[1] = klp;
      rt[2] = enp;
      rt[3] = 0.0;
      if constexpr (PREP) {
        // KL_ff plain logit delta d_j = (p_j/N)(B_j - sum_k p_k B_k), B = eps/(p+eps); surr logit delta
        // -(adv/(N old_a)) p_a (1[j=a] - p_j)  (gemm.hip kPrepHead), in f32 as there
#pragma unroll
        for (int j = 0; j < AT; ++j) {
          const float Bj = j < a.A ? kEps * __builtin_amdgcn_rcpf(p[j] + kEps) : 0.0f;   // O(eps) term: 1-ulp rcp
          spB += p[j] * Bj;
          rest += (j < a.A && j != av) ? p[j] : 0.0f;
        }
        coef = -adv * (float)a.invN / olda * pa;
      }
    }
    if constexpr (PREP) {
      // P, D_L, DS_L through LDS (sH is free after the chunk loop): each thread's row into a [row][AT + 1] image,
      // then the tile's rows -- contiguous in HBM -- stored by consecutive threads.  A row per lane written
      // directly is 64 scattered 80-B pieces per store instruction (round 4: 5.2 vs 3.9 ms for the row GEMM head).
      float* so = sH;
      const float invN = (float)a.invN;
#pragma unroll
      for (int kind = 0; kind < 3; ++kind) {
        __syncthreads();   // the chunk loop's (or the previous kind's) reads of sH are done
#pragma unroll
        for (int j = 0; j < AT; ++j) {
          const bool real = j < a.A;
          const float pd = p[j];
          float v;
          if (kind == 0) {
            v = real ? pd : 0.0f;
          } else if (kind == 1) {
            const float Bj = real ? kEps * __builtin_amdgcn_rcpf(pd + kEps) : 0.0f;
            v = real ? pd * invN * (Bj - spB) : 0.0f;
            mD = fmaxf(mD, fabsf(v));
          } else {
            v = real ? coef * (j == av ? rest : -pd) : 0.0f;
            mS = fmaxf(mS, fabsf(v));
          }
          so[t * ldo + j] = v;
        }
        __syncthreads();
        float* dst = (kind == 0 ? a.P : kind == 1 ? a.D : a.DS) + t0 * AT;   // Apad == AT
        for (int i = t; i < nr * AT; i += kHfRows) {
          const int r = i / AT, c = i - r * AT;
          dst[i] = so[r * ldo + c];
        }
      }
    }
  }
  if constexpr (PREP) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      mD = fmaxf(mD, __shfl_xor(mD, off, 64));
      mS = fmaxf(mS, __shfl_xor(mS, off, 64));
    }
    __syncthreads();
    if ((t & 63) == 0) {
      sred[0][t >> 6] = mD;
      sred[1][t >> 6] = mS;
    }
    __syncthreads();
    if (t < 2) {
      unsigned* slot = t == 0 ? a.am_d : a.am_ds;
      if (slot) {
        float m = 0.0f;
#pragma unroll
        for (int u = 0; u < kHfRows / 64; ++u) m = fmaxf(m, sred[t][u]);
        if (m > 0.0f) atomicMax(slot + (blockIdx.x % kAmaxSub) * kAmaxStride, __float_as_uint(m));
      }
    }
  }
}

template <bool PREP>
void launch_head_fwd_t(const HeadFwdArgs& a, int grid, hipStream_t s) {
  switch ((a.A + 3) / 4) {
    case 1: hipLaunchKernelGGL((head_fwd_kernel<4, PREP>), dim3(grid), dim3(kHfRows), 0, s, a); break;
    case 2: hipLaunchKernelGGL((head_fwd_kernel<8, PREP>), dim3(grid), dim3(kHfRows), 0, s, a); break;
    case 3: hipLaunchKernelGGL((head_fwd_kernel<12, PREP>), dim3(grid), dim3(kHfRows), 0, s, a); break;
    case 4: hipLaunchKernelGGL((head_fwd_kernel<16, PREP>), dim3(grid), dim3(kHfRows), 0, s, a); break;
    case 5: hipLaunchKernelGGL((head_fwd_kernel<20, PREP>), dim3(grid), dim3(kHfRows), 0, s, a); break;
    case 6: hipLaunchKernelGGL((head_fwd_kernel<24, PREP>), dim3(grid), dim3(kHfRows), 0, s, a); break;
    case 7: hipLaunchKernelGGL((head_fwd_kernel<28, PREP>), dim3(grid), dim3(kHfRows), 0, s, a); break;
    default: hipLaunchKernelGGL((head_fwd_kernel<32, PREP>), dim3(grid), dim3(kHfRows), 0, s, a); break;
  }
}

}  // namespace

bool head_fwd_eligible(int A, int K) { return A <= 32 && K >= 1 && K <= 4096; }

void launch_head_fwd(const HeadFwdArgs& a, int num_cus, hipStream_t s) {
  if (a.rows <= 0) return;
  if (!head_fwd_eligible(a.A, a.K) || a.Apad != (a.A + 3) / 4 * 4 || a.Kpad < a.K || a.Kpad % 4 || !a.H || !a.W || !a.bias ||
      !a.old || !a.act || !a.adv || !a.rowterms || (a.prep && (!a.P || !a.D || !a.DS)))
    throw std::runtime_error("head_fwd: unsupported shape or missing operand");
  const int64_t tiles = (a.rows + kHfRows - 1) / kHfRows;
  const int grid = (int)std::min<int64_t>(tiles, (int64_t)4 * num_cus);
  if (a.prep) launch_head_fwd_t<true>(a, grid, s);
  else launch_head_fwd_t<false>(a, grid, s);
}

}  // namespace trpo
