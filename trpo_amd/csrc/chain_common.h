// Device helpers shared by the fused FVP chain (chain.hip) and the fused small-width FVPs
// (fused.hip, fused16.hip): the exact bf16 three-way split, the layout of the chain's weight images
// and of the gradient-pass images.
#pragma once
#include "common.h"

namespace trpo {

typedef __bf16 cbf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short cu16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short cu16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int cu32x4 __attribute__((ext_vector_type(4)));
typedef short fs4 __attribute__((ext_vector_type(4)));   // ds_read_b64_tr_b16 results
typedef short fs8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned short cb_bits(float x) { return __builtin_bit_cast(unsigned short, (__bf16)x); }
__device__ __forceinline__ float cb_val(unsigned short b) { return __builtin_bit_cast(float, (unsigned)b << 16); }

// x = hi + mid + lo exactly (each a bf16), as gemm.hip's split3
__device__ __forceinline__ void csplit(float x, unsigned short& h, unsigned short& m, unsigned short& l) {
  h = cb_bits(x);
  const float r1 = x - cb_val(h);
  m = cb_bits(r1);
  const float r2 = r1 - cb_val(m);
  l = cb_bits(r2);
}

// Gradient-pass images of the fused FVPs (fused.hip, fused16.hip): [state][kFI features] 16-bit planes.
constexpr int kFI = 64;   // features per image row (one pass operand: up to 4 tiles of 16)

// 32-B chunk (one 16-feature tile) of image row r: tile ^ fswz(r).  The 8 rows a half-wave's
// transposed read touches (r0 + {0..3, 8..11}) then cover all 64 banks once.  Within the chunk, the 8-B unit
// of features 4u..4u+3 sits at u ^ fsub(r): fswz takes row bits 1 and 3, fsub bits 0 and 2, so the 16
// consecutive rows of an image store (lane = row, one unit each: ds_write_b64) land on 16 distinct units of
// the 128-B bank window (round 5: 4-way conflicts before, 34 % of the fused FVP's LDS cycles), while a
// transposed read still takes one whole chunk per row.
__device__ __forceinline__ int fswz(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 1); }
__device__ __forceinline__ int fsub(int r) { return (r & 1) | (((r >> 2) & 1) << 1); }
__device__ __forceinline__ int fimg(int r, int f) {
  return r * kFI + ((((f >> 4) ^ fswz(r))) << 4) + (((((f >> 2) & 3) ^ fsub(r))) << 2) + (f & 3);
}

// 16-B chunk position of k-group g in image row o: g ^ chain_hsw(o).  Makes the
// 16-lane groups of a ds_read_b128 (MI355X_MICROARCH.md, LDS table) hit 16
// distinct 4-bank sets for 64-B rows.
__host__ __device__ constexpr int chain_hsw(int o) { return (((o >> 2) & 1) * 2) ^ (((o >> 3) & 1) * 3); }

// MFMA k index kk (0..31) of a chunk -> feature offset within the chunk (acc-layout pairing)
__host__ __device__ constexpr int chain_perm(int kk) {
  return (kk & 7) < 4 ? 4 * (kk >> 3) + (kk & 7) : 16 + 4 * (kk >> 3) + (kk & 7) - 4;
}

__device__ __forceinline__ float c_one_minus_sq(float h) { return (1.0f - h) * (1.0f + h); }

__device__ __forceinline__ double sum4lanes(double v) {   // lanes s, s+16, s+32, s+48 (common.h swaps)
  return xadd_d<true>(xadd_d<false>(v));
}

// B operand (3 bf16 planes) of v_mfma_f32_16x16x32_bf16 from two acc-layout tiles: lane (g, s)
// holds features 4g..4g+3 of each tile for state s (the k order chain_perm describes)
__device__ __forceinline__ void chain_mkb(const f32x4& x0, const f32x4& x1, cbf16x8 (&b)[3]) {
  cu16x8 h, m, l;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    unsigned short hh, mm, ll;
    csplit(x0[j], hh, mm, ll);
    h[j] = hh;
    m[j] = mm;
    l[j] = ll;
    csplit(x1[j], hh, mm, ll);
    h[4 + j] = hh;
    m[4 + j] = mm;
    l[4 + j] = ll;
  }
  b[0] = __builtin_bit_cast(cbf16x8, h);
  b[1] = __builtin_bit_cast(cbf16x8, m);
  b[2] = __builtin_bit_cast(cbf16x8, l);
}

// c += a * b over the split planes, smallest terms first (6 products: every pair with
// plane(a) + plane(b) <= 2; the dropped ones are below f32 rounding)
__device__ __forceinline__ f32x4 chain_mfma6(const cbf16x8 (&a)[3], const cbf16x8 (&b)[3], f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], c, 0, 0, 0);
  return c;
}

}  // namespace trpo
