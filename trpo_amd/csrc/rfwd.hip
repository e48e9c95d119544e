// The FVP's R-forward through the first two layers in one launch (gfx950 / CDNA4): trpo_inksci.py:56-70 (the
// R-operator of the policy forward, trpo_inksci.py:38-40; SURVEY.md Appendix A "R-forward"), at the C4 shape
// (two hidden layers of 256, obs <= 128, the fused tail on the head layer):
//
//   RZ1 = X V0 + c0 ;  RH1 = (1 - H1^2) RZ1 ;  RZ2 = RH1 W1 + H1 V1 + c1
//
// It replaces fvp_rfwd_l0 (plane.hip, writes RH1) + fvp_rfwd_l1 (gemm.hip rowgemm3, reads RH1 and H1 back):
// RH1 is still written (the layer-1 R-backward's E_0 RH1 term and the layer-1 weight gradient read it), but it
// is not read back, and H1 is read once.  Bytes per state: X's f16 planes 512 + H1 1024 + RH1 1024 + RZ2 1024 =
// 3584 (the two launches: 5632).
//
// Layout: one workgroup of 4 waves per CU (persistent over 128-state tiles, 512 registers per wave: the 128
// accumulators in AGPRs, X of the wave's states in VGPRs for the whole tile); wave w owns 32 states of the tile
// and all 256 output columns.  For each 32-feature slice t of layer 1:
//  * phase A: RZ1^T[32 features x 32 states] = V0^T X^T on v_mfma_f32_32x32x16_f16 (V0^T from LDS as the A
//    operand, X's pre-split f16 planes as the B operand, loaded once per tile), 3 products;
//  * epilogue: the accumulator lane holds one state and features 8j + 4h + i (j, i = 0..3, h = lane / 32): RH1
//    and H1 in that layout are exactly the A operand of the next product with its k order permuted (k-step u
//    takes registers 8u..8u+7), so RH1 never leaves registers on its way to the second GEMM;
//  * phase B: RZ2[32 states x 256] += RH1_t W1_t + H1_t V1_t (W1 / V1 rows of slice t, k-permuted the same way,
//    from LDS as B operands), 3 products per segment.
// Weights and H1 stream through a 4-slot LDS ring by LDS-DMA (24 chunks per tile: V0^T slice t + H1 slice t, then
// W1 / V1 rows of slice t for output columns 0-127 and 128-255, 32 KB each; the weight chunks from an image built
// once per FVP in that order by rfwd01_img_kernel, pre-swizzled, so the DMA is a straight copy), each DMA'd three
// chunks ahead; no other loads in the loop but X once per tile, so the DMA waits are counted exactly (arrive()).
// Measured: 10.46 ms at C4 against 3.93 + 7.99 for the two launches (profiles/r6o); ablations: without the
// phase-B MFMAs 6.6 ms, without any MFMA 6.0: the 5 KB per state of weights the 128-state tiles re-stream by DMA
// (50 GB per FVP with H1, ~8 TB/s) and the MFMAs do not overlap (one wave per SIMD).  Then, same box each
// (profiles/r6s-r6v): the DMA pieces one per k-step among the MFMAs 10.12 -> 9.94; X loaded outside the slice
// loop, where hipcc no longer drains every DMA in flight before X's first use (its vmcnt(15) ... vmcnt(0) series)
// 10.22 -> 9.90; the bound-based exponent 9.90 -> 9.25 ms.
//
// Scales (f16 hi + lo split, kernels.h f16_scale_exp): X from its plane exponent, V0 / W1 / V1 from their
// running-max slots; RH1 (made in the launch) per state (an A-operand row is one state, so each state has its own
// exponent) from a bound fixed at the tile's start, |RH1_sj| <= |RZ1_sj| <= |X_s|_2 max_j |V0_j|_2 + max |c0|
// (RF_CSB); H1 fixed (|h| <= 1).  Both phase-B segments share a state's product exponent, the smaller of the two,
// so no slice ever re-scales the accumulators, and the rows are unscaled at the end.  Power-of-two scales change
// no split and no product: a loose bound costs precision only once a split's low half would fall below f16's
// normal range, 2^14 below the bound.  (RF_CSB 0: the exponent from each slice's own max, the accumulator rows
// stepped down by exact powers of two when a later slice needs it: 0.65 ms slower at C4, the re-scaling branch
// keeping 128 accumulator copies in VGPRs.)
#include "chain_common.h"
#include "rowepi.h"

#include <stdexcept>
#include <type_traits>

namespace trpo {
namespace {

typedef __fp16 rf_h2 __attribute__((ext_vector_type(2)));

#ifndef RF_SGB
#define RF_SGB 1   // 1: each k-step region issues its next fragments' LDS reads before its MFMAs (sched_group_barrier)
#endif
#ifndef RF_ILV
#define RF_ILV 1   // 1: a chunk's 8 DMA instructions issued one per k-step among its MFMAs, not as a burst before them
#endif
#ifndef RF_HOIST
#define RF_HOIST 0  // 1: the slice's H1 and c0 values read from LDS before the phase-A MFMAs, not after them
#endif
#ifndef RF_HEAD
#define RF_HEAD 3   // (RF_CSB 0) a later slice re-scales its state only when it needs an exponent more than RF_HEAD
                    // below the state's current one (its scaled max then stays < 2^(12 + RF_HEAD) <= 2^15, in f16)
#endif
#ifndef RF_CSB
#define RF_CSB 1    // 1: a state's product exponent from a bound fixed at the tile's start, |RH1| <= |X_s| max_j |V0_j| +
                    // max |c0| (Cauchy-Schwarz per state): no per-slice exponent, no re-scaling of the accumulators
#endif
#ifndef RF_ABL
#define RF_ABL 0   // timing ablations only (tools/variant.sh), bits: 1 = no phase-B MFMAs, 2 = no phase-B LDS reads,
                   // 4 = no weight DMA, 8 = no RH1 / RZ2 stores, 16 = no H1 / X loads, 32 = no phase-A MFMAs,
                   // 64 = a minimal phase-A epilogue (no tangent, no per-state max: a fixed exponent)
#endif

constexpr int kRfUnits = 2048;                 // 16-B units of a ring slot / image chunk (32 KB)
constexpr int kRfChunks = 24;                  // chunks per tile
constexpr int kRfLd = 256;                     // row stride of H1 / RH1 / RZ2 (floats; launch_rfwd01 checks)
constexpr int kRfTile = 128, kRfWaves = 4;   // 4 waves of 32 states: 512 registers per wave

// 8 values times s -> f16 hi and lo (round toward zero; x - hi is exact): fused16.hip split2 per pair
__device__ __forceinline__ void rf_split8(const float* x, float s, f16x8& hi, f16x8& lo) {
  cu32x4 H, L;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float a = x[2 * q] * s, b = x[2 * q + 1] * s;
    const rf_h2 hp = __builtin_amdgcn_cvt_pkrtz(a, b);
    const rf_h2 lp = __builtin_amdgcn_cvt_pkrtz(a - (float)hp[0], b - (float)hp[1]);
    H[q] = __builtin_bit_cast(unsigned, hp);
    L[q] = __builtin_bit_cast(unsigned, lp);
  }
  hi = __builtin_bit_cast(f16x8, H);
  lo = __builtin_bit_cast(f16x8, L);
}

// c += a b on the split, smallest terms first
__device__ __forceinline__ f32x16 rf_mfma3(const f16x8& ah, const f16x8& al, const f16x8& bh, const f16x8& bl,
                                           f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
  return c;
}

// ---- the chunk image (one per FVP: V0 and V1 change, W1 does not within an update) --------------------------
// chunk 3t (A_t, 16 KB): [plane][feature f 0..31][unit u ^ (f & 15)] with unit u = 2 ks + h holding V0[obs 16 ks
//   + 8 h + q][32 t + f], q = 0..7 (obs >= the real obs: 0);
// chunk 3t + 1 + nh (B_t,nh, 32 KB): [matrix W1, V1][plane][column r 0..127][unit u ^ ((r >> 2) & 3)] with unit
//   u = 2 uu + h holding M[32 t + 16 uu + 4 h + 8 (q >> 2) + (q & 3)][128 nh + r], q = 0..7 (the phase-B k order).
__global__ void __launch_bounds__(256) rfwd01_img_kernel(const float* __restrict__ theta, const float* __restrict__ v,
                                                         int64_t offV0, int64_t offW1, int obs,
                                                         const unsigned* am_v0, const unsigned* am_w1,
                                                         const unsigned* am_v1, uint16_t* __restrict__ img,
                                                         const int* skip) {
  if (skip && *skip) return;
  const int eV0 = amax_exp(am_v0), eW = amax_exp(am_w1), eV = amax_exp(am_v1);
  const int gid = blockIdx.x * 256 + threadIdx.x;   // 8 slices x (512 A units + 2 x 1024 B units)
  const int t = gid / 2560, rem = gid % 2560;
  if (t >= 8) return;
  float x[8];
  cu32x4* dst;
  int plane_units;
  float sc;
  if (rem < 512) {   // A_t: feature f, unit u
    const int f = rem >> 4, u = rem & 15, ks = u >> 1, h = u & 1;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = 16 * ks + 8 * h + q;
      x[q] = k < obs ? v[offV0 + (int64_t)k * 256 + 32 * t + f] : 0.0f;
    }
    sc = __builtin_ldexpf(1.0f, eV0);
    dst = reinterpret_cast<cu32x4*>(img) + (size_t)(3 * t) * kRfUnits + f * 16 + (u ^ (f & 15));
    plane_units = 512;
  } else {   // B_t,nh: matrix m, column r, unit u
    const int b = rem - 512, nh = b >> 10, m = (b >> 9) & 1, r = (b >> 2) & 127, u = b & 3, uu = u >> 1, h = u & 1;
    const float* src = m ? v : theta;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = 32 * t + 16 * uu + 4 * h + 8 * (q >> 2) + (q & 3);
      x[q] = src[offW1 + (int64_t)k * 256 + 128 * nh + r];
    }
    sc = __builtin_ldexpf(1.0f, m ? eV : eW);
    dst = reinterpret_cast<cu32x4*>(img) + (size_t)(3 * t + 1 + nh) * kRfUnits + m * 1024 + r * 4 +
          (u ^ ((r >> 2) & 3));
    plane_units = 512;
  }
  f16x8 hi, lo;
  rf_split8(x, sc, hi, lo);
  dst[0] = __builtin_bit_cast(cu32x4, hi);
  dst[plane_units] = __builtin_bit_cast(cu32x4, lo);
}

// One LDS-DMA instruction (buffer_load_dwordx4 ... lds): 16 B per lane from the buffer at voff + soff into LDS at the
// wave-uniform byte address lds + 16 * lane (soff is added to the lane offset: an soffset operand must be an SGPR,
// and a constant one would reach the assembler as a literal).  Inline asm, opaque to hipcc's s_waitcnt bookkeeping: the kernel counts
// the completions itself (arrive()).  M0 is saved and restored around it (the compiler owns M0).
__device__ __forceinline__ void rf_dma16(__amdgpu_buffer_rsrc_t rsrc, unsigned voff, unsigned soff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff + soff), "s"(rsrc), "s"(lds));
}

template <int KS0>   // 16-deep k-steps over obs (obs <= 16 KS0)
__global__ void __launch_bounds__(kRfWaves * 64, 1) rfwd01_kernel(const Rfwd01Args a) {
  static_assert(!RF_ILV || KS0 == 8, "interleaved DMA: one instruction per k-step of phase A");
  // the ring: chunk c in slot c % 4.  An A chunk holds V0^T slice t (image units 0..1023) and H1 slice t of the
  // tile's 128 states (units 1024..2047, 256 per wave: row r, column unit cu at r * 8 + (cu ^ ((r >> 1) & 7)), so the
  // epilogue's reads of one column unit over 16 rows hit 16 distinct bank slots); a B chunk the W1 / V1 rows.
  __shared__ cu32x4 q0[kRfUnits], q1[kRfUnits], q2[kRfUnits], q3[kRfUnits];
  __shared__ float cvec[2][256];      // the tangent biases c0, c1
  __shared__ float red[3][16];
  __shared__ int pex[kRfWaves][32];   // per-state exponents, from the A-operand lanes to the accumulator lanes
  if (a.skip && *a.skip) return;
  const int tid = threadIdx.x, lane = tid & 63, s = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int eX = __builtin_amdgcn_readfirstlane(*a.eX);
  const int eV0 = __builtin_amdgcn_readfirstlane(amax_exp(a.am_v0));
  const int eW = __builtin_amdgcn_readfirstlane(amax_exp(a.am_w1));
  const int eV = __builtin_amdgcn_readfirstlane(amax_exp(a.am_v1));
  const float uA = __builtin_ldexpf(1.0f, -(eX + eV0));
  const int64_t ntiles = (a.n + kRfTile - 1) / kRfTile;
  const __amdgpu_buffer_rsrc_t rimg =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.img, 0, kRfChunks * kRfUnits * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t rxh = __builtin_amdgcn_make_buffer_rsrc((void*)a.Xh, 0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rxl = __builtin_amdgcn_make_buffer_rsrc((void*)a.Xl, 0, 0x7ffffff0, 0x00020000);
  for (int i = tid; i < 256; i += kRfWaves * 64) {
    cvec[0][i] = a.c0[i];
    cvec[1][i] = a.c1[i];
  }
  // RF_CSB: nv0 = max_j |V0[:, j]|_2 and mc0 = max_j |c0_j| (uniform; thread j takes column j)
  float nv0 = 0.0f, mc0 = 0.0f;
  if constexpr (RF_CSB) {
    float q = 0.0f;
    for (int k = 0; k < a.obs; ++k) {
      const float x = a.V0[(int64_t)k * 256 + tid];
      q = fmaf(x, x, q);
    }
    float m1 = max32_dpp(sqrtf(q)), m2 = max32_dpp(fabsf(a.c0[tid]));
    m1 = fmaxf(m1, __shfl_xor(m1, 32));
    m2 = fmaxf(m2, __shfl_xor(m2, 32));
    if (lane == 0) {
      red[0][wv] = m1;
      red[1][wv] = m2;
    }
    __syncthreads();
    nv0 = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
    mc0 = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
    __syncthreads();   // red is reused by amax_commit3 at the end
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // ordinary loads retired before the first DMA
  auto slot = [&](int k) -> cu32x4* { return k == 0 ? q0 : k == 1 ? q1 : k == 2 ? q2 : q3; };
  auto rows_of = [&](int64_t r0w) { return (int)(a.n - r0w < 32 ? (a.n - r0w > 0 ? a.n - r0w : 0) : 32); };
  // chunk c (0..23) into slot sl (= c % 4), 8 DMA instructions per wave: a B chunk from the image; an A chunk half
  // from the image, half this wave's 32 H1 rows of slice t = c / 3 (r0w: the wave's first state of the chunk's tile;
  // rows past n land as zeros)
  // instruction i (0..7) of that: a B chunk's image piece i; an A chunk's image piece i (i < 4) or H1 piece i - 4
  // (A: chunk c is an A chunk, c % 3 == 0, known at every call site)
  auto dma_one = [&](auto A, int c, int sl, int64_t r0w, int i) __attribute__((always_inline)) {
    if constexpr ((RF_ABL & 4) != 0) return;
    const unsigned lds0 = (unsigned)(uintptr_t)slot(sl);
    if (!decltype(A)::value || i < 4) {
      const int base = wv * 64 + i * kRfWaves * 64;   // units
      rf_dma16(rimg, (unsigned)(base + lane) * 16u, (unsigned)c * kRfUnits * 16u, lds0 + (unsigned)base * 16u);
    } else {
      const int t = c / 3, ih = i - 4;
      const __amdgpu_buffer_rsrc_t rh =
          __builtin_amdgcn_make_buffer_rsrc((void*)(a.H1 + r0w * kRfLd), 0, rows_of(r0w) * kRfLd * 4, 0x00020000);
      const int r = 8 * ih + (lane >> 3), cu = (lane & 7) ^ ((r >> 1) & 7);
      rf_dma16(rh, (unsigned)(r * kRfLd + 4 * cu) * 4u, (unsigned)(32 * t) * 4u,
               lds0 + (unsigned)(1024 + wv * 256 + 64 * ih) * 16u);
    }
  };
  auto dma = [&](auto A, int c, int sl, int64_t r0w) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; ++i) dma_one(A, c, sl, r0w, i);
  };
  using kA = std::true_type;
  using kB = std::false_type;
  // Begin chunk c: this wave's DMA into the chunk's slot has landed, then every wave's (the barrier: the chunk is
  // visible, and every wave is past chunk c - 1, whose slot takes chunk c + 3's DMA next).  Completions retire in
  // issue order, so the wait is "at most the number of VMEM operations this wave issued after chunk c's DMA":
  // chunks c + 1 and c + 2's DMAs (8 + 8) and the 4 RH1 stores of the A chunk among c .. c + 2 = 20 (the first
  // tile's A_0: only the two DMAs, 16).  Across a tile boundary more than 63 sit behind it (the X loads, the 128
  // RZ2 stores): vmcnt(63) there, which also covers the next tile's X loads (128 stores were issued after them).
  // A smaller count than the true one only waits longer; none is larger.
  auto arrive = [&](bool far, bool first_a0) __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    if (far) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
    else if (first_a0 || (RF_ABL & 8) != 0) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    lds_barrier();
  };
  // X's f16 planes, all k-steps, of one state (B operand: lane (state s, half h) holds obs 16 ks + 8 h .. + 7)
  // (row0 = the wave's first state: uniform, so every load is one lane offset + one scalar offset)
  const unsigned xlane = (unsigned)(s * 32 + 8 * h) * 2u;
  auto xload = [&](int64_t row0, f16x8 (&x)[KS0][2]) __attribute__((always_inline)) {
    if constexpr ((RF_ABL & 16) != 0) {
#pragma unroll
      for (int ks = 0; ks < KS0; ++ks) {
        unsigned u = (unsigned)row0 + ks;
        asm volatile("" : "+v"(u));
        x[ks][0] = x[ks][1] = __builtin_bit_cast(f16x8, cu32x4{u, u, u, u});
      }
      return;
    }
#pragma unroll
    for (int ks = 0; ks < KS0; ++ks) {
      const int so = (int)((((unsigned)(ks >> 1) * (unsigned)a.x_mpad + (unsigned)row0) * 32u + 16u * (ks & 1)) * 2u);
      x[ks][0] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rxh, xlane, so, 0));
      x[ks][1] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rxl, xlane, so, 0));
    }
  };
  const unsigned hlane = (unsigned)(s * kRfLd + 4 * h) * 4u;   // RH1 rows: lane part of the offset

  f16x8 xt[KS0][2];   // X of this wave's 32 states, the whole tile
  xload((int64_t)blockIdx.x * kRfTile + wv * 32, xt);   // (grid <= tiles: a real tile)
  // the first tile's X waited for here, where hipcc's own s_waitcnt bookkeeping sees it: the later tiles' X loads
  // are followed by the 128 RZ2 stores (more than vmcnt's 63), so hipcc puts no wait in front of X's uses
  __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0) (gfx9 encoding: expcnt 7, lgkmcnt 15)
  {
    const int64_t r0f = (int64_t)blockIdx.x * kRfTile + wv * 32;
    dma(kA{}, 0, 0, r0f);
    dma(kB{}, 1, 1, r0f);
    dma(kB{}, 2, 2, r0f);
  }

  float mR = 0.0f, mZ = 0.0f;   // running max |RH1|, |RZ2| of this lane
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const bool first = tile == (int64_t)blockIdx.x;
    const int64_t r0 = tile * kRfTile + wv * 32;   // this wave's first state (wave-uniform: the buffer bases)
    const int64_t r0n = r0 + (int64_t)gridDim.x * kRfTile;     // ... in the next tile
    const int rows = rows_of(r0);
    const __amdgpu_buffer_rsrc_t rrh =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.RH1 + r0 * kRfLd), 0, rows * kRfLd * 4, 0x00020000);
    f32x16 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = f32x16{};
    int Ps = 0;   // this lane's state's product exponent (set by slice 0, lowered when a later slice needs it)
    if constexpr (RF_CSB) {
      // |RH1_sj| <= |RZ1_sj| <= |X_s|_2 |V0_j|_2 + |c0_j|; |X_s| from the hi plane (|x| <= |hi| (1 + 2^-10)),
      // 1 % over for that and for the split products' rounding
      float q = 0.0f;
#pragma unroll
      for (int ks = 0; ks < KS0; ++ks) {
        const f16x8 x8 = xt[ks][0];
        q = __builtin_amdgcn_fdot2(__builtin_shufflevector(x8, x8, 0, 1), __builtin_shufflevector(x8, x8, 0, 1), q, false);
        q = __builtin_amdgcn_fdot2(__builtin_shufflevector(x8, x8, 2, 3), __builtin_shufflevector(x8, x8, 2, 3), q, false);
        q = __builtin_amdgcn_fdot2(__builtin_shufflevector(x8, x8, 4, 5), __builtin_shufflevector(x8, x8, 4, 5), q, false);
        q = __builtin_amdgcn_fdot2(__builtin_shufflevector(x8, x8, 6, 7), __builtin_shufflevector(x8, x8, 6, 7), q, false);
      }
      q = xadd_f<true>(q);   // the state's other 8 obs of each 16 (lane s + 32)
      const float bnd = __builtin_ldexpf(sqrtf(q), -eX) * nv0 * 1.01f + mc0;
      Ps = min(bnd > 0.0f ? f16_scale_exp(bnd) + eW : 1000, f16_scale_exp(1.0f) + eV);
    }
    // accumulator register r of this lane holds state 8 (r >> 2) + 4 h + (r & 3): its exponent comes through LDS
    int* px = pex[wv];
#pragma unroll 1
    for (int tq = 0; tq < 2; ++tq) {
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const int t = 4 * tq + tt;
        const int cA = 3 * t, sA = (3 * tt) % 4;   // 12 chunks per tq: the slots are static
        const bool far = t == 0 && !first;
        // ---- phase A: RZ1^T slice t ----
        arrive(far, t == 0 && first);
        const int cA3 = cA + 3 < kRfChunks ? cA + 3 : cA + 3 - kRfChunks;
        const int64_t rA3 = cA + 3 < kRfChunks ? r0 : r0n;
        if (!RF_ILV) dma(kA{}, cA3, (sA + 3) % 4, rA3);
        const cu32x4* S = slot(sA);
        float hv[16], cb[16];
        auto ldh = [&]() __attribute__((always_inline)) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int cu = 2 * j + h;
            const f32x4 v4 = __builtin_bit_cast(f32x4, S[1024 + wv * 256 + s * 8 + (cu ^ ((s >> 1) & 7))]);
#pragma unroll
            for (int i = 0; i < 4; ++i) hv[4 * j + i] = v4[i];
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) cb[r] = cvec[0][32 * t + 8 * (r >> 2) + 4 * h + (r & 3)];
        };
        if (RF_HOIST) ldh();
        f32x16 accA = f32x16{};
        // fragments one k-step ahead of the MFMAs (sched barriers keep the compiler from hoisting them all)
        f16x8 fa[2][2];
        auto lda = [&](int ks, f16x8 (&f)[2]) __attribute__((always_inline)) {
          const int au = s * 16 + ((2 * ks + h) ^ (s & 15));
          f[0] = __builtin_bit_cast(f16x8, S[au]);
          f[1] = __builtin_bit_cast(f16x8, S[512 + au]);
        };
        lda(0, fa[0]);
#pragma unroll
        for (int ks = 0; ks < KS0; ++ks) {
          __builtin_amdgcn_sched_barrier(0);
          if (RF_ILV) dma_one(kA{}, cA3, (sA + 3) % 4, rA3, ks);
          if (ks + 1 < KS0) lda(ks + 1, fa[(ks + 1) & 1]);
          if constexpr ((RF_ABL & 32) == 0) accA = rf_mfma3(fa[ks & 1][0], fa[ks & 1][1], xt[ks][0], xt[ks][1], accA);
          if (RF_SGB && ks + 1 < KS0) {
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- epilogue: RH1 slice t (stored), the state's max -> its phase-B product exponent ----
        if (!RF_HOIST) ldh();
        float rh[16];
        float mt = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if constexpr ((RF_ABL & 64) != 0) {
            rh[r] = accA[r] * uA;
          } else {
            rh[r] = one_minus_sq(hv[r]) * (accA[r] * uA + cb[r]);
            mt = fmaxf(mt, fabsf(rh[r]));
          }
        }
#pragma unroll
        for (int j = 0; j < 4 && (RF_ABL & 8) == 0; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(
              __builtin_bit_cast(cu32x4, f32x4{rh[4 * j], rh[4 * j + 1], rh[4 * j + 2], rh[4 * j + 3]}), rrh, hlane,
              (32 * t + 8 * j) * 4, 0);
        mR = fmaxf(mR, mt);
        if constexpr ((RF_ABL & 64) == 0 && !RF_CSB) mt = xmax_f<true>(mt);   // the state's max over the slice
        const int Pt = (RF_ABL & 64) ? 2 : min(mt > 0.0f ? f16_scale_exp(mt) + eW : 1000, f16_scale_exp(1.0f) + eV);
        if constexpr (RF_CSB) {
          // Ps fixed for the tile
        } else if (t == 0) {
          Ps = Pt;
        } else if (__builtin_amdgcn_ballot_w64(Pt < Ps - RF_HEAD) != 0) {
          // rare: a state whose slice is more than 2^RF_HEAD larger than its exponent allows; its accumulator rows
          // step down by an exact power of two (the other states' by 2^0).  Power-of-two scales change no split and
          // no product, so the headroom only bounds f16's range (the per-slice rule, RF_HEAD = 0, re-scaled in most
          // slices of random data: 1.1 ms of the launch's 10)
          if (h == 0) px[s] = Pt < Ps - RF_HEAD ? Pt - Ps : 0;
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          float f[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) f[r] = __builtin_ldexpf(1.0f, px[8 * (r >> 2) + 4 * h + (r & 3)]);
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][r] *= f[r];
          Ps = Pt < Ps - RF_HEAD ? Pt : Ps;
          __builtin_amdgcn_wave_barrier();
        }
        const float sR = __builtin_ldexpf(1.0f, Ps - eW), sH = __builtin_ldexpf(1.0f, Ps - eV);
        f16x8 aR[2][2], aH[2][2];   // k-step uu: registers 8 uu .. 8 uu + 7 (the permuted k order)
#pragma unroll
        for (int uu = 0; uu < 2; ++uu) {
          rf_split8(rh + 8 * uu, sR, aR[uu][0], aR[uu][1]);
          rf_split8(hv + 8 * uu, sH, aH[uu][0], aH[uu][1]);
        }
        // ---- phase B: RZ2 += RH1_t W1_t + H1_t V1_t, output columns 128 nh .. 128 nh + 127 ----
#pragma unroll
        for (int nh = 0; nh < 2; ++nh) {
          const int cB = cA + 1 + nh, sB = (3 * tt + 1 + nh) % 4;
          arrive(far, false);
          const int cB3 = cB + 3 < kRfChunks ? cB + 3 : cB + 3 - kRfChunks;
          const int64_t rB3 = cB + 3 < kRfChunks ? r0 : r0n;
          if (!RF_ILV) dma(kB{}, cB3, (sB + 3) % 4, rB3);
          const cu32x4* B = slot(sB);
          // step k = 4 uu + tn; its W / V fragments loaded one step ahead
          f16x8 fb[2][4];
          auto ldb = [&](int k, f16x8 (&f)[4]) __attribute__((always_inline)) {
            const int col = 32 * (k & 3) + s;
            const int bu = col * 4 + ((2 * (k >> 2) + h) ^ ((col >> 2) & 3));
            f[0] = __builtin_bit_cast(f16x8, B[bu]);
            f[1] = __builtin_bit_cast(f16x8, B[512 + bu]);
            f[2] = __builtin_bit_cast(f16x8, B[1024 + bu]);
            f[3] = __builtin_bit_cast(f16x8, B[1536 + bu]);
          };
          ldb(0, fb[0]);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            __builtin_amdgcn_sched_barrier(0);
            if (RF_ILV) dma_one(kB{}, cB3, (sB + 3) % 4, rB3, k);
            if (k + 1 < 8 && (RF_ABL & 2) == 0) ldb(k + 1, fb[(k + 1) & 1]);
            const int uu = k >> 2, tn = k & 3;
            const f16x8(&f)[4] = fb[k & 1];
            if ((RF_ABL & 1) == 0) {
              f32x16 c = acc[4 * nh + tn];
              c = rf_mfma3(aR[uu][0], aR[uu][1], f[0], f[1], c);
              c = rf_mfma3(aH[uu][0], aH[uu][1], f[2], f[3], c);
              acc[4 * nh + tn] = c;
            }
            if (RF_SGB && (RF_ABL & 3) == 0 && k + 1 < 8) {
              __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
              __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    xload(r0n < a.x_mpad ? r0n : 0, xt);   // the next tile's X (none: any valid rows), ahead of the RZ2 stores
    // ---- RZ2 = acc 2^-P + c1: lane (column 32 tn + s, states 8 j + 4 h + i) ----
    if (h == 0) px[s] = Ps;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    float un[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) un[r] = __builtin_ldexpf(1.0f, -px[8 * (r >> 2) + 4 * h + (r & 3)]);
    __builtin_amdgcn_wave_barrier();
    const __amdgpu_buffer_rsrc_t rz =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.RZ2 + r0 * kRfLd), 0, rows * kRfLd * 4, 0x00020000);
    const unsigned zlane = (unsigned)(4 * h * kRfLd + s) * 4u;   // lane part: state 4 h, column s
#pragma unroll
    for (int tn = 0; tn < 8; ++tn) {
      const float cn = cvec[1][32 * tn + s];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float o = acc[tn][r] * un[r] + cn;
        mZ = fmaxf(mZ, fabsf(o));
        if constexpr ((RF_ABL & 8) == 0)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), rz, zlane,
                                                ((8 * (r >> 2) + (r & 3)) * kRfLd + 32 * tn) * 4, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may land after the workgroup has left the CU
  amax_commit3<true>(a.am_rh1, mR, a.am_rz2, mZ, nullptr, 0.0f, red);
}


// ---- the policy forward through layers 0 and 1 in one launch (option fwd01): trpo_inksci.py:38-40 ----------------
//   H1 = tanh(X W0 + b0) (stored by the prepare pass only) ;  H2 = tanh(H1 W1 + b1) (stored)
// rfwd01's structure with one phase-B segment and no H1 input: per slice t an A chunk (W0^T slice t, 16 KB, the
// layout of rfwd01's V0^T chunk) and a B chunk (W1 rows of slice t, all 256 columns, 32 KB: [plane][column r
// 0..255][unit u ^ ((r >> 2) & 3)], u = 2 uu + h holding W1[32 t + 16 uu + 4 h + 8 (q >> 2) + (q & 3)][r]), 16
// chunks per tile through the same 4-slot ring.  |h| <= 1, so H1's scale is fixed (2^11) and no exponent is
// tracked per state.
constexpr int kFwChunks = 16;

__global__ void __launch_bounds__(256) fwd01_img_kernel(const float* __restrict__ th, int64_t offW0, int64_t offW1,
                                                        int obs, const unsigned* am_w0, const unsigned* am_w1,
                                                        uint16_t* __restrict__ img) {
  const int eW0 = amax_exp(am_w0), eW1 = amax_exp(am_w1);
  const int gid = blockIdx.x * 256 + threadIdx.x;   // 8 slices x (512 A units + 1024 B units)
  const int t = gid / 1536, rem = gid % 1536;
  if (t >= 8) return;
  float x[8];
  cu32x4* dst;
  int plane_units;
  float sc;
  if (rem < 512) {   // A_t: feature f, unit u
    const int f = rem >> 4, u = rem & 15, ks = u >> 1, h = u & 1;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = 16 * ks + 8 * h + q;
      x[q] = k < obs ? th[offW0 + (int64_t)k * 256 + 32 * t + f] : 0.0f;
    }
    sc = __builtin_ldexpf(1.0f, eW0);
    dst = reinterpret_cast<cu32x4*>(img) + (size_t)(2 * t) * kRfUnits + f * 16 + (u ^ (f & 15));
    plane_units = 512;
  } else {   // B_t: column r, unit u
    const int b = rem - 512, r = b >> 2, u = b & 3, uu = u >> 1, h = u & 1;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = 32 * t + 16 * uu + 4 * h + 8 * (q >> 2) + (q & 3);
      x[q] = th[offW1 + (int64_t)k * 256 + r];
    }
    sc = __builtin_ldexpf(1.0f, eW1);
    dst = reinterpret_cast<cu32x4*>(img) + (size_t)(2 * t + 1) * kRfUnits + r * 4 + (u ^ ((r >> 2) & 3));
    plane_units = 1024;
  }
  f16x8 hi, lo;
  rf_split8(x, sc, hi, lo);
  dst[0] = __builtin_bit_cast(cu32x4, hi);
  dst[plane_units] = __builtin_bit_cast(cu32x4, lo);
}

template <int KS0, bool PREP>
__global__ void __launch_bounds__(kRfWaves * 64, 1) fwd01_kernel(const Fwd01Args a) {
  __shared__ cu32x4 q0[kRfUnits], q1[kRfUnits], q2[kRfUnits], q3[kRfUnits];
  __shared__ float cvec[2][256];      // the biases b0, b1
  const int tid = threadIdx.x, lane = tid & 63, s = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int eX = __builtin_amdgcn_readfirstlane(*a.eX);
  const int eW0 = __builtin_amdgcn_readfirstlane(amax_exp(a.am_w0));
  const int eW1 = __builtin_amdgcn_readfirstlane(amax_exp(a.am_w1));
  const float uA = __builtin_ldexpf(1.0f, -(eX + eW0));
  const int P = f16_scale_exp(1.0f) + eW1;   // products of H1 (scaled 2^(P - eW1) = 2^11) and W1 (2^eW1)
  const float sH = __builtin_ldexpf(1.0f, P - eW1), uP = __builtin_ldexpf(1.0f, -P);
  const int64_t ntiles = (a.n + kRfTile - 1) / kRfTile;
  const __amdgpu_buffer_rsrc_t rimg =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.img, 0, kFwChunks * kRfUnits * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t rxh = __builtin_amdgcn_make_buffer_rsrc((void*)a.Xh, 0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rxl = __builtin_amdgcn_make_buffer_rsrc((void*)a.Xl, 0, 0x7ffffff0, 0x00020000);
  for (int i = tid; i < 256; i += kRfWaves * 64) {
    cvec[0][i] = a.b0[i];
    cvec[1][i] = a.b1[i];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // ordinary loads retired before the first DMA
  auto slot = [&](int k) -> cu32x4* { return k == 0 ? q0 : k == 1 ? q1 : k == 2 ? q2 : q3; };
  auto rows_of = [&](int64_t r0w) { return (int)(a.n - r0w < 32 ? (a.n - r0w > 0 ? a.n - r0w : 0) : 32); };
  // piece i of chunk c's DMA into slot sl: an A chunk has 4 pieces per wave (16 KB), a B chunk 8 (32 KB)
  auto dma_one = [&](int c, int sl, int i) __attribute__((always_inline)) {
    const unsigned lds0 = (unsigned)(uintptr_t)slot(sl);
    const int base = wv * 64 + i * kRfWaves * 64;   // units
    rf_dma16(rimg, (unsigned)(base + lane) * 16u, (unsigned)c * kRfUnits * 16u, lds0 + (unsigned)base * 16u);
  };
  // Begin chunk c (see rfwd01_kernel's arrive()).  Operations behind chunk c's DMA, S = 4 H1 stores per A chunk
  // (prepare) or 0: an A chunk 8 + S (chunk c - 2: the next B chunk's DMA and its stores) + 4 (chunk c - 1: an A
  // chunk's DMA) = 12 + S; a B chunk S + 4 + 8 + S = 12 + 2 S.  The first tile's chunk 0: 12, chunk 1: 12 + S.
  // Across a tile boundary (chunks 0, 1, 2 of a later tile) the X loads and the 128 H2 stores: vmcnt(63).
  // (A count below the true one only waits longer: 12 + S and 12 + 2 S are 16 / 20 or 12 / 12.)
  constexpr int S = PREP ? 4 : 0;
  auto arrive = [&](int cnt) __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    if (cnt >= 63) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
    else if (PREP && cnt == 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else if (PREP && cnt == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    lds_barrier();
  };
  const unsigned xlane = (unsigned)(s * 32 + 8 * h) * 2u;
  auto xload = [&](int64_t row0, f16x8 (&x)[KS0][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < KS0; ++ks) {
      const int so = (int)((((unsigned)(ks >> 1) * (unsigned)a.x_mpad + (unsigned)row0) * 32u + 16u * (ks & 1)) * 2u);
      x[ks][0] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rxh, xlane, so, 0));
      x[ks][1] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rxl, xlane, so, 0));
    }
  };
  const unsigned hlane = (unsigned)(s * kRfLd + 4 * h) * 4u;   // H1 rows: lane part of the offset

  f16x8 xt[KS0][2];
  xload((int64_t)blockIdx.x * kRfTile + wv * 32, xt);
  __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): the first tile's X, where hipcc's bookkeeping sees it
#pragma unroll
  for (int i = 0; i < 4; ++i) dma_one(0, 0, i);
#pragma unroll
  for (int i = 0; i < 8; ++i) dma_one(1, 1, i);
#pragma unroll
  for (int i = 0; i < 4; ++i) dma_one(2, 2, i);

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const bool first = tile == (int64_t)blockIdx.x;
    const int64_t r0 = tile * kRfTile + wv * 32;
    const int64_t r0n = r0 + (int64_t)gridDim.x * kRfTile;
    const int rows = rows_of(r0);
    f32x16 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = f32x16{};
#pragma unroll 1
    for (int tq = 0; tq < 2; ++tq) {
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const int t = 4 * tq + tt;
        const int cA = 2 * t, sA = (2 * tt) % 4, cB = cA + 1, sB = (2 * tt + 1) % 4;
        // ---- phase A: Z0^T slice t; chunk cA + 3 (a B chunk) DMA'd one piece per k-step ----
        arrive(!first && t <= 1 ? 63 : (first && t == 0 ? 12 : 12 + S));
        const int cA3 = cA + 3 < kFwChunks ? cA + 3 : cA + 3 - kFwChunks;
        const cu32x4* SA = slot(sA);
        f32x16 accA = f32x16{};
        f16x8 fa[2][2];
        auto lda = [&](int ks, f16x8 (&f)[2]) __attribute__((always_inline)) {
          const int au = s * 16 + ((2 * ks + h) ^ (s & 15));
          f[0] = __builtin_bit_cast(f16x8, SA[au]);
          f[1] = __builtin_bit_cast(f16x8, SA[512 + au]);
        };
        lda(0, fa[0]);
#pragma unroll
        for (int ks = 0; ks < KS0; ++ks) {
          __builtin_amdgcn_sched_barrier(0);
          dma_one(cA3, (sA + 3) % 4, ks);
          if (ks + 1 < KS0) lda(ks + 1, fa[(ks + 1) & 1]);
          accA = rf_mfma3(fa[ks & 1][0], fa[ks & 1][1], xt[ks][0], xt[ks][1], accA);
          if (RF_SGB && ks + 1 < KS0) {
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- epilogue: H1 slice t (lane: state s, features 8 (r >> 2) + 4 h + (r & 3)), the phase-B A operand ----
        float hv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r)
          hv[r] = tanh_fast(accA[r] * uA + cvec[0][32 * t + 8 * (r >> 2) + 4 * h + (r & 3)]);
        if constexpr (PREP) {
          const __amdgpu_buffer_rsrc_t rh1 =
              __builtin_amdgcn_make_buffer_rsrc((void*)(a.H1 + r0 * kRfLd), 0, rows * kRfLd * 4, 0x00020000);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(cu32x4, f32x4{hv[4 * j], hv[4 * j + 1], hv[4 * j + 2], hv[4 * j + 3]}), rh1,
                hlane, (32 * t + 8 * j) * 4, 0);
        }
        f16x8 aH[2][2];
#pragma unroll
        for (int uu = 0; uu < 2; ++uu) rf_split8(hv + 8 * uu, sH, aH[uu][0], aH[uu][1]);
        // ---- phase B: Z1 += H1_t W1_t, all 256 columns; chunk cB + 3 (an A chunk) DMA'd over the first 4 steps ----
        arrive(!first && t == 0 ? 63 : (first && t == 0 ? 12 + S : 12 + 2 * S));
        const int cB3 = cB + 3 < kFwChunks ? cB + 3 : cB + 3 - kFwChunks;
        const cu32x4* B = slot(sB);
        f16x8 fb[2][2];
        auto ldb = [&](int k, f16x8 (&f)[2]) __attribute__((always_inline)) {   // k = 8 nh + 4 uu + tn
          const int col = 128 * (k >> 3) + 32 * (k & 3) + s;
          const int bu = col * 4 + ((2 * ((k >> 2) & 1) + h) ^ ((col >> 2) & 3));
          f[0] = __builtin_bit_cast(f16x8, B[bu]);
          f[1] = __builtin_bit_cast(f16x8, B[1024 + bu]);
        };
        ldb(0, fb[0]);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          __builtin_amdgcn_sched_barrier(0);
          if (k < 4) dma_one(cB3, (sB + 3) % 4, k);
          if (k + 1 < 16) ldb(k + 1, fb[(k + 1) & 1]);
          const int uu = (k >> 2) & 1, tn = k & 3, nh = k >> 3;
          acc[4 * nh + tn] = rf_mfma3(aH[uu][0], aH[uu][1], fb[k & 1][0], fb[k & 1][1], acc[4 * nh + tn]);
          if (RF_SGB && k + 1 < 16) {
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    xload(r0n < a.x_mpad ? r0n : 0, xt);   // the next tile's X, ahead of the H2 stores (see rfwd01_kernel)
    // ---- H2 = tanh(acc 2^-P + b1): lane (column 32 tn + s, states 8 j + 4 h + i) ----
    const __amdgpu_buffer_rsrc_t rz =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.H2 + r0 * kRfLd), 0, rows * kRfLd * 4, 0x00020000);
    const unsigned zlane = (unsigned)(4 * h * kRfLd + s) * 4u;
#pragma unroll
    for (int tn = 0; tn < 8; ++tn) {
      const float bn = cvec[1][32 * tn + s];
#pragma unroll
      for (int r = 0; r < 16; ++r)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, tanh_fast(acc[tn][r] * uP + bn)), rz,
                                              zlane, ((8 * (r >> 2) + (r & 3)) * kRfLd + 32 * tn) * 4, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may land after the workgroup has left the CU
}

}  // namespace

bool rfwd01_eligible(int L, const int* w, const int* wp) {
  return L == 3 && w[0] >= 1 && w[0] <= 128 && w[1] == 256 && w[2] == 256 && wp[1] == 256 && wp[2] == 256;
}

size_t rfwd01_img_bytes() { return (size_t)kRfChunks * kRfUnits * 16; }

void launch_rfwd01_img(const float* theta, const float* v, int64_t offV0, int64_t offW1, int obs,
                       const unsigned* am_v0, const unsigned* am_w1, const unsigned* am_v1, uint16_t* img,
                       const int* skip, hipStream_t s) {
  hipLaunchKernelGGL(rfwd01_img_kernel, dim3(8 * 2560 / 256), dim3(256), 0, s, theta, v, offV0, offW1, obs, am_v0,
                     am_w1, am_v1, img, skip);
}

void launch_rfwd01(const Rfwd01Args& a, int num_cus, hipStream_t s) {
  if (a.n <= 0) return;
  if (a.obs < 1 || a.obs > 128 || a.ldh != 256 || a.ldz != 256)
    throw std::runtime_error("rfwd01: unsupported shape");
  if ((int64_t)4 * a.x_mpad * 64 >= ((int64_t)1 << 31) || a.x_mpad < (a.n + kRfTile - 1) / kRfTile * kRfTile)
    throw std::runtime_error("rfwd01: X plane geometry");
  const int64_t ntiles = (a.n + kRfTile - 1) / kRfTile;
  const int grid = (int)std::min<int64_t>(ntiles, (int64_t)num_cus);
  hipLaunchKernelGGL(rfwd01_kernel<8>, dim3(grid), dim3(kRfWaves * 64), 0, s, a);
}

bool fwd01_eligible(int L, const int* w, const int* wp) { return rfwd01_eligible(L, w, wp); }

size_t fwd01_img_bytes() { return (size_t)kFwChunks * kRfUnits * 16; }

void launch_fwd01_img(const float* th, int64_t offW0, int64_t offW1, int obs, const unsigned* am_w0,
                      const unsigned* am_w1, uint16_t* img, hipStream_t s) {
  hipLaunchKernelGGL(fwd01_img_kernel, dim3(8 * 1536 / 256), dim3(256), 0, s, th, offW0, offW1, obs, am_w0, am_w1,
                     img);
}

void launch_fwd01(const Fwd01Args& a, int num_cus, hipStream_t s) {
  if (a.n <= 0) return;
  if (a.obs < 1 || a.obs > 128) throw std::runtime_error("fwd01: unsupported shape");
  if ((int64_t)4 * a.x_mpad * 64 >= ((int64_t)1 << 31) || a.x_mpad < (a.n + kRfTile - 1) / kRfTile * kRfTile)
    throw std::runtime_error("fwd01: X plane geometry");
  const int64_t ntiles = (a.n + kRfTile - 1) / kRfTile;
  const int grid = (int)std::min<int64_t>(ntiles, (int64_t)num_cus);
  if (a.H1) hipLaunchKernelGGL((fwd01_kernel<8, true>), dim3(grid), dim3(kRfWaves * 64), 0, s, a);
  else hipLaunchKernelGGL((fwd01_kernel<8, false>), dim3(grid), dim3(kRfWaves * 64), 0, s, a);
}

}  // namespace trpo
