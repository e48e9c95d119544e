// Fused last-layer tail of the FVP (gfx950): the R-softmax head, the R-backward into the last
// hidden layer and that layer's weight R-gradient in one persistent launch.
//
// For the last layer l = L-1 (hidden width a <= 256, n_actions b <= 32) and a 32-row tile the
// reference graph (trpo_inksci.py:56-70) needs, per row:
//   RZ    = RH W + H V + c                                  head R-forward   (K = a, N = b)
//   RD_L  = R-softmax-reverse(RZ)                           row-wise, f64   (gemm.hip kRHead)
//   RDH   = RD_L W^T + D_L V^T ,  DH = D_L W^T              R-backward       (K = b, N = a)
//   RD    = RDH (1 - H^2) - 2 DH H RH                       -> RD_{L-2}, the next R-backward's input
//   G    += RH^T D_L + H^T RD_L ;  g_b += colsum RD_L        weight R-gradient (K = rows)
// The per-layer kernels stream RH and H four times and materialise RZ / RD_L / E; here RH and H
// are read once from HBM, E = -2 DH H is recomputed from D_L (K = b), and only RD_{L-2} is written.
//
// Arithmetic: every product on v_mfma_f32_32x32x16_f16 with each fp32 operand scaled by a power of
// two and split into f16 hi + lo (3 products, 2^-22 relative; gemm.hip rowgemm3_kernel).  Scales:
// RH / D_L / W / V from the engine's running-max slots, H fixed (|tanh| <= 1), RD_L per tile
// (it is produced here).  Every accumulator is unscaled to true f32 values before it is combined.
//
// Layouts (32x32x16: lane l, r = l&31, h = l>>5; C: col = r, row = (i&3) + 8(i>>2) + 4h):
//   * RH / H are loaded in C layout (lane = hidden column, registers = rows): they are the
//     element-wise operands of RD and, unchanged, the A operands of the row-reduced G products
//     (k-step s takes registers 8s..8s+7; row of element j = 16s + 8(j>>2) + 4h + (j&3)).
//   * the head R-forward sums over the hidden columns: its A operands (lane = row, 8 consecutive
//     columns) come from the same registers through an LDS image read with ds_read_b64_tr_b16.
//   * RD_L / D_L cross the 4 waves through LDS once per tile, read back in A layout (R-backward)
//     and in C layout (G products).
// Block = 8 waves (two per SIMD), wave w owns hidden columns [32w, 32w + 32); one block per
// split-K slab.
#include "common.h"
#include "kernels.h"

#include <stdexcept>

namespace trpo {
namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

constexpr int TR = 32;       // rows per tile
constexpr int NW = 8;        // waves per block; wave w owns hidden columns [32w, 32w + 32)
constexpr int SLD = 36;      // row stride (floats) of the [row][action] LDS tiles

__device__ __forceinline__ float omsq(float h) { return (1.0f - h) * (1.0f + h); }

#ifndef TRPO_TAIL_DPP
#define TRPO_TAIL_DPP 1    // 0: R-softmax row sums by ds_bpermute shuffles (A/B builds only)
#endif
template <class T>
__device__ __forceinline__ T hsum32t(T v) {
#if TRPO_TAIL_DPP
  return sum32_dpp(v);   // common.h: DPP moves + one ds_swizzle
#else
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off, 32);
  return v;
#endif
}
#ifndef TRPO_TAIL_HEAD64
#define TRPO_TAIL_HEAD64 0
#endif

// the max of a running-max slot (kAmaxSub counters) -> power-of-two scale exponent; whole wave
__device__ __forceinline__ int slot_exp(const unsigned* amax) {
  if (!amax) return f16_scale_exp(1.0f);
  const int lane = threadIdx.x & 63;
  float v = 0.0f;
#pragma unroll
  for (int i = 0; i < kAmaxSub / 64; ++i) v = fmaxf(v, __uint_as_float(amax[(lane + 64 * i) * kAmaxStride]));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return f16_scale_exp(v);
}

// x * 2^e -> f16 hi + lo, two elements per packed conversion (v_cvt_pkrtz_f16_f32).  Round toward
// zero: x - hi is exact in f32 and |x - hi| < ulp16(x), so lo keeps hi + lo within 2^-21 |x|.
typedef __fp16 fp16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split8(const float* x, float s, h8& hi, h8& lo) {
  u32x4 H, L;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = x[2 * i] * s, b = x[2 * i + 1] * s;
    const fp16x2 hp = __builtin_amdgcn_cvt_pkrtz(a, b);
    const fp16x2 lp = __builtin_amdgcn_cvt_pkrtz(a - (float)hp[0], b - (float)hp[1]);
    H[i] = __builtin_bit_cast(unsigned, hp);
    L[i] = __builtin_bit_cast(unsigned, lp);
  }
  hi = __builtin_bit_cast(h8, H);
  lo = __builtin_bit_cast(h8, L);
}



// a*b ~= ah bh + ah bl + al bh, smallest terms first
__device__ __forceinline__ f32x16 mfma3(const h8& ah, const h8& al, const h8& bh, const h8& bl, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
  return c;
}

__device__ __forceinline__ float ldb(__amdgpu_buffer_rsrc_t r, int vo, int so) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
}

// head planes in LDS: [mat][plane][j][k] u16, the 16-B chunk c of row j stored at c ^ (j & 15)
__device__ __forceinline__ int sw_off(int mat, int plane, int j, int k) {
  return ((mat * 2 + plane) * 32 + j) * kTailK + (((k >> 3) ^ (j & 15)) << 3) + (k & 7);
}

__global__ void __launch_bounds__(NW * 64, 1) fvp_tail_kernel(const TailArgs A) {
  __shared__ __attribute__((aligned(16))) unsigned short sW[2 * 2 * 32 * kTailK];   // 64 KB
  // per wave 8 KB: the tile's RH / H f16 planes as [mat][plane][k][m] images for the transposed
  // reads of the head R-forward, then (same bytes) the wave's RZ partial [16][64] f32
  __shared__ __attribute__((aligned(16))) unsigned short sX[NW][2 * 2 * 32 * 32];
  __shared__ __attribute__((aligned(16))) float sRD[2][TR][SLD];
  __shared__ __attribute__((aligned(16))) float sD[2][TR][SLD];
  // f16 planes of the tile's [RD_L ; D_L] (mat 0 / 1) as [row][action], converted once per tile
  // (4 rows per wave) and read back as A fragments (ds_read_b128) and transposed (tr16)
  __shared__ __attribute__((aligned(16))) unsigned short sP[2 * 2 * TR * 32];
  __shared__ float sMax[2][NW];
  __shared__ float sBias[NW][64];
  __shared__ float sOut[NW];
  if (A.skip && *A.skip) return;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int apad = A.apad, bpad = A.bpad, b = A.b;
  const int r0 = blockIdx.x * A.rows_per_split;
  const int r1 = min(A.rows, r0 + A.rows_per_split);
  const int col0 = 32 * w;                    // this wave's hidden columns [col0, col0 + 32)
  const bool wv = col0 < apad;

  const int eRH = slot_exp(A.am_rh), eD = slot_exp(A.am_d), eW = slot_exp(A.am_w), eV = slot_exp(A.am_v);
  const int eH = f16_scale_exp(1.0f);
  const float sRHf = __builtin_ldexpf(1.0f, eRH), sDf = __builtin_ldexpf(1.0f, eD), sHf = __builtin_ldexpf(1.0f, eH);

  // ---- head planes -> LDS (swizzled) ----
  for (int i = tid; i < 2 * 2 * 32 * (kTailK / 8); i += NW * 64) {
    const int c = i % (kTailK / 8), row = i / (kTailK / 8);   // row = (mat*2 + plane)*32 + j
    const int j = row & 31;
    *reinterpret_cast<u16x8*>(sW + row * kTailK + ((c ^ (j & 15)) << 3)) =
        *reinterpret_cast<const u16x8*>(A.WV16 + (size_t)row * kTailK + 8 * c);
  }

  // ---- R-backward B fragments (constant): [W^T ; V^T] planes [n][k], n = col0 + lr, k = 16s + 8lh ----
  h8 wt[2][2], vt[2][2];   // [s][plane]
  {
    const int n = col0 + lr;
    const bool nv = n < apad;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const size_t o = (size_t)p * A.bplane + (size_t)(nv ? n : 0) * 32 + 16 * s + 8 * lh;
        const u16x8 x = *reinterpret_cast<const u16x8*>(A.WT16 + o);
        const u16x8 y = *reinterpret_cast<const u16x8*>(A.VT16 + o);
        wt[s][p] = nv ? __builtin_bit_cast(h8, x) : h8{};
        vt[s][p] = nv ? __builtin_bit_cast(h8, y) : h8{};
      }
  }
  __syncthreads();

  f32x16 G = f32x16{};   // weight R-gradient, true f32 values: [hidden col0 + ..][action]
  float bsum = 0.0f;     // colsum of RD_L, lane = action (lr), this wave's rows
  float mxo = 0.0f;      // max |RD_out|

  // tile loads (rows past r1 fall outside the per-tile buffer descriptors: read 0, store dropped)
  auto desc = [&](const float* p, int t0, int ld) {
    const int nr = max(0, min(TR, r1 - t0));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(p + (size_t)t0 * ld), 0, nr * ld * 4, 0x00020000);
  };
  const int vo_c = wv ? ((4 * lh) * apad + col0 + lr) * 4 : 0x40000000;   // C layout
  // head rows of this wave: C registers i = 2w + q (q = 0, 1) -> rows (i&3) + 8(i>>2) + 4lh
  const int hrow0 = ((2 * w) & 3) + 8 * ((2 * w) >> 2) + 4 * lh;           // rows hrow0, hrow0 + 1
  const int vo_h = lr < bpad ? (hrow0 * bpad + lr) * 4 : 0x40000000;
  auto load_c = [&](int t0, float (&rh)[16], float (&h)[16], float (&pp)[2], float (&dd)[2]) {
    const __amdgpu_buffer_rsrc_t rRH = desc(A.RH, t0, apad), rH = desc(A.H, t0, apad);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int so = ((i & 3) + 8 * (i >> 2)) * apad * 4;
      rh[i] = ldb(rRH, vo_c, so);
      h[i] = ldb(rH, vo_c, so);
    }
    const __amdgpu_buffer_rsrc_t rP = desc(A.P, t0, bpad), rDL = desc(A.DL, t0, bpad);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      pp[q] = ldb(rP, vo_h, q * bpad * 4);
      dd[q] = ldb(rDL, vo_h, q * bpad * 4);
    }
  };

  float cRH[16], cH[16], cP[2], cD[2];
  if (r0 < r1) load_c(r0, cRH, cH, cP, cD);
  int par = 0;
  for (int t0 = r0; t0 < r1; t0 += TR, par ^= 1) {
    float nRH[16], nH[16], nP[2], nD[2];
    if (t0 + TR < r1) load_c(t0 + TR, nRH, nH, nP, nD);
    // RZ in, R{h} = (1 - H^2) RZ formed here: the R-forward that feeds the tail then never reads H
    // (RowEpi::kRZ); the same f32 operations as its kRHidden epilogue, so R{h} is bit-identical
    if (A.rz) {
#pragma unroll
      for (int i = 0; i < 16; ++i) cRH[i] = omsq(cH[i]) * cRH[i];
    }

    // ---- head R-forward partial over this wave's 32 columns: RZ = RH W + H V.  The tile's C layout
    //      (lane = column k, registers = rows m) goes to LDS as f16 planes [k][m], each lane storing
    //      registers 4g..4g+3 (rows 8g + 4lh ..) as 8 bytes, and comes back transposed (lane = row m,
    //      8 consecutive k) through ds_read_b64_tr_b16.  8-byte unit u = m/4 of row k sits at
    //      u ^ ((k >> 1) & 7): conflict-free stores and transposed reads. ----
    unsigned short* xw = sX[w];
    auto xoff = [](int mat, int plane, int k, int m) {
      return ((mat * 2 + plane) * 32 + k) * 32 + ((((m >> 2) ^ ((k >> 1) & 7))) << 2) + (m & 3);
    };
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      h8 hi, lo;
#pragma unroll
      for (int mat = 0; mat < 2; ++mat) {
        split8(mat == 0 ? &cRH[8 * s2] : &cH[8 * s2], mat == 0 ? sRHf : sHf, hi, lo);
        typedef short s4 __attribute__((ext_vector_type(4)));
        const s4* hp = reinterpret_cast<const s4*>(&hi);
        const s4* lp = reinterpret_cast<const s4*>(&lo);
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int m = 16 * s2 + 8 * half + 4 * lh;
          *reinterpret_cast<s4*>(xw + xoff(mat, 0, lr, m)) = hp[half];
          *reinterpret_cast<s4*>(xw + xoff(mat, 1, lr, m)) = lp[half];
        }
      }
    }
    {
      typedef short s4 __attribute__((ext_vector_type(4)));
      typedef short s8 __attribute__((ext_vector_type(8)));
      const int g4 = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
      const int mrow = 16 * (g4 & 1) + 4 * pp;             // the 4 columns (rows m) this lane addresses
      f32x16 acc = f32x16{}, accv = f32x16{};
      auto tr8 = [&](int mat, int pl, int s2) {
        s8 v;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int k = 16 * s2 + 8 * (g4 >> 1) + 4 * t + q;
          const s4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s4*)(xw + xoff(mat, pl, k, mrow)));
#pragma unroll
          for (int e = 0; e < 4; ++e) v[4 * t + e] = r[e];
        }
        return __builtin_bit_cast(h8, v);
      };
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int k = col0 + 16 * s2 + 8 * lh;
        acc = mfma3(tr8(0, 0, s2), tr8(0, 1, s2), *reinterpret_cast<const h8*>(sW + sw_off(0, 0, lr, k)),
                    *reinterpret_cast<const h8*>(sW + sw_off(0, 1, lr, k)), acc);
        accv = mfma3(tr8(1, 0, s2), tr8(1, 1, s2), *reinterpret_cast<const h8*>(sW + sw_off(1, 0, lr, k)),
                     *reinterpret_cast<const h8*>(sW + sw_off(1, 1, lr, k)), accv);
      }
      const float f0 = __builtin_ldexpf(1.0f, -(eRH + eW)), f1 = __builtin_ldexpf(1.0f, -(eH + eV));
      float* rzw = reinterpret_cast<float*>(xw);            // the planes are consumed: reuse the bytes
#pragma unroll
      for (int i = 0; i < 16; ++i) rzw[i * 64 + lane] = acc[i] * f0 + accv[i] * f1;
    }
    lds_barrier();

    // ---- R-softmax head on this wave's two rows (gemm.hip kRHead, same cancellation-free form):
    //      RD_j = (1/N)[Rp_j (B_j - sum p B) + Rp_j A_j^2 + p_j sum_k Rp_k A_k B_k],
    //      Rp = p (Rz - <p, Rz>), A = p/(p+eps), B = eps/(p+eps); f32 here (TRPO_TAIL_HEAD64: f64) ----
    float m = 0.0f;
    {
      const int j = lr;
      const bool real = j < b;
      const float cj = A.c[real ? j : 0];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = 2 * w + q;
        float zs = 0.0f;
#pragma unroll
        for (int u = 0; u < NW; ++u) zs += reinterpret_cast<const float*>(sX[u])[i * 64 + lane];
        const float z = zs + cj;
#if TRPO_TAIL_HEAD64
        typedef double T;
#else
        typedef float T;
#endif
        const T rz = real ? (T)z : T(0);
        const T pd = real ? (T)cP[q] : T(0);    // rows past the split: P = 0 -> RD = 0
        const T prz = hsum32t(pd * rz);
        const T Rp = pd * (rz - prz);
        const T inv = T(1) / (pd + (T)kEps);
        const T Aa = real ? pd * inv : T(0);
        const T B = real ? (T)kEps * inv : T(0);
        const T spB = hsum32t(pd * B);
        const T sRAB = hsum32t(Rp * Aa * B);
        const T rd = (T)A.invN * (Rp * (B - spB) + Rp * Aa * Aa + pd * sRAB);
        const float rdf = real ? (float)rd : 0.0f;
        const int row = hrow0 + q;
        sRD[par][row][j] = rdf;
        sD[par][row][j] = real ? cD[q] : 0.0f;
        m = fmaxf(m, fabsf(rdf));
        bsum += rdf;
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    if (lane == 0) sMax[par][w] = m;
    lds_barrier();
    float mt = 0.0f;
#pragma unroll
    for (int u = 0; u < NW; ++u) mt = fmaxf(mt, sMax[par][u]);
    const int eRD = f16_scale_exp(mt);
    const float sRDf = __builtin_ldexpf(1.0f, eRD);

    // ---- [RD_L ; D_L] -> f16 planes, rows 4w..4w+3 by wave w; the 16-B chunk c of row r sits at
    //      c ^ ((r >> 2) & 3) (conflict-free A-fragment reads; tr16 reads of 4 consecutive rows) ----
    typedef short s4 __attribute__((ext_vector_type(4)));
    auto pof = [](int mat, int pl, int row, int col) {
      return ((mat * 2 + pl) * TR + row) * 32 + ((((col >> 3) ^ ((row >> 2) & 3))) << 3) + (col & 7);
    };
    {
      const int row = 4 * w + (lane >> 4), col = 2 * (lane & 15);
#pragma unroll
      for (int mat = 0; mat < 2; ++mat) {
        const float sc = mat == 0 ? sRDf : sDf;
        const float a = (mat == 0 ? sRD[par][row][col] : sD[par][row][col]) * sc;
        const float bb = (mat == 0 ? sRD[par][row][col + 1] : sD[par][row][col + 1]) * sc;
        const fp16x2 hp = __builtin_amdgcn_cvt_pkrtz(a, bb);
        const fp16x2 lp = __builtin_amdgcn_cvt_pkrtz(a - (float)hp[0], bb - (float)hp[1]);
        *reinterpret_cast<fp16x2*>(sP + pof(mat, 0, row, col)) = hp;
        *reinterpret_cast<fp16x2*>(sP + pof(mat, 1, row, col)) = lp;
      }
    }
    lds_barrier();

    // ---- R-backward: RDH = RD_L W^T + D_L V^T, DH = D_L W^T (K = actions); A fragments: lane =
    //      row lr, actions 16s + 8lh .. ----
    f32x16 aRW = f32x16{}, aDV = f32x16{}, aDW = f32x16{};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int col = 16 * s + 8 * lh;
      const h8 rh_ = *reinterpret_cast<const h8*>(sP + pof(0, 0, lr, col));
      const h8 rl_ = *reinterpret_cast<const h8*>(sP + pof(0, 1, lr, col));
      const h8 dh_ = *reinterpret_cast<const h8*>(sP + pof(1, 0, lr, col));
      const h8 dl_ = *reinterpret_cast<const h8*>(sP + pof(1, 1, lr, col));
      aRW = mfma3(rh_, rl_, wt[s][0], wt[s][1], aRW);
      aDV = mfma3(dh_, dl_, vt[s][0], vt[s][1], aDV);
      aDW = mfma3(dh_, dl_, wt[s][0], wt[s][1], aDW);
    }
    // ---- RD = RDH (1 - H^2) + E RH, E = -2 DH H (gemm.hip kPrepBwd / kRBwd) ----
    {
      const float fRW = __builtin_ldexpf(1.0f, -(eRD + eW)), fDV = __builtin_ldexpf(1.0f, -(eD + eV));
      const float fDW = __builtin_ldexpf(1.0f, -(eD + eW));
      const __amdgpu_buffer_rsrc_t rOut = desc(A.RDout, t0, apad);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float rdh = aRW[i] * fRW + aDV[i] * fDV;
        const float dh = aDW[i] * fDW;
        const float h = cH[i], rh = cRH[i];
        const float e = -2.0f * dh * h;
        const float o = fmaf(e, rh, rdh * omsq(h));
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), rOut, vo_c,
                                              ((i & 3) + 8 * (i >> 2)) * apad * 4, 0);
        mxo = fmaxf(mxo, fabsf(o));
      }
    }
    // ---- weight R-gradient: G += RH^T D_L + H^T RD_L (rows are the MFMA k).  B fragments (lane =
    //      action, element e of k-step s = row 16s + 8(e>>2) + 4lh + (e&3)) by transposed reads of
    //      the planes: lane 4q+p of a 16-lane group addresses row r0 + q, actions 4p .. 4p+3 ----
    {
      typedef short s8 __attribute__((ext_vector_type(8)));
      const int g4 = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
      auto trb = [&](int mat, int pl, int s2) {
        s8 v;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int row = 16 * s2 + 4 * (g4 >> 1) + 8 * t + q;
          const s4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s4*)(sP + pof(mat, pl, row, 16 * (g4 & 1) + 4 * pp)));
#pragma unroll
          for (int e = 0; e < 4; ++e) v[4 * t + e] = r[e];
        }
        return __builtin_bit_cast(h8, v);
      };
      f32x16 g0 = f32x16{}, g1 = f32x16{};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        h8 ah, al;
        split8(&cRH[8 * s], sRHf, ah, al);
        g0 = mfma3(ah, al, trb(1, 0, s), trb(1, 1, s), g0);
        split8(&cH[8 * s], sHf, ah, al);
        g1 = mfma3(ah, al, trb(0, 0, s), trb(0, 1, s), g1);
      }
      const float fG0 = __builtin_ldexpf(1.0f, -(eRH + eD)), fG1 = __builtin_ldexpf(1.0f, -(eH + eRD));
#pragma unroll
      for (int i = 0; i < 16; ++i) G[i] += g0[i] * fG0 + g1[i] * fG1;
    }

    if (t0 + TR < r1) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        cRH[i] = nRH[i];
        cH[i] = nH[i];
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        cP[q] = nP[q];
        cD[q] = nD[q];
      }
    }
  }

  // ---- this split's slab: W part [a][b] and the bias colsum ----
  float* out = A.slab + (size_t)blockIdx.x * A.slab_stride;
  if (lr < b) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int mrow = col0 + (i & 3) + 8 * (i >> 2) + 4 * lh;
      if (mrow < A.a) out[A.off_w + (int64_t)mrow * b + lr] = G[i];
    }
  }
  sBias[w][lane] = bsum;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mxo = fmaxf(mxo, __shfl_xor(mxo, off, 64));
  if (lane == 0) sOut[w] = mxo;
  __syncthreads();
  if (tid < b) {
    float t = 0.0f;
#pragma unroll
    for (int q = 0; q < NW; ++q) t += sBias[q][tid] + sBias[q][tid + 32];
    out[A.off_b + tid] = t;
  }
  if (tid == 0 && A.am_out) {
    float mm = 0.0f;
#pragma unroll
    for (int q = 0; q < NW; ++q) mm = fmaxf(mm, sOut[q]);
    if (mm > 0.0f) atomicMax(A.am_out + (blockIdx.x % kAmaxSub) * kAmaxStride, __float_as_uint(mm));
  }
}

// head planes [mat][plane][j][k] from the flat theta (mat 0, scale am_w) and tangent (mat 1, am_v)
__global__ void __launch_bounds__(256) tail_pack_kernel(const TailPackArgs P) {
  const int mat = blockIdx.y;
  const float* src = (mat == 0 ? P.theta : P.v) + P.off_w;
  const int e = slot_exp(mat == 0 ? P.am_w : P.am_v);   // whole wave, before any exit
  const float s = __builtin_ldexpf(1.0f, e);
  const int idx = blockIdx.x * 256 + threadIdx.x;       // over 32 j x kTailK k
  if (idx >= 32 * kTailK) return;
  const int j = idx / kTailK, k = idx % kTailK;
  const float x = (j < P.b && k < P.a) ? src[(size_t)k * P.b + j] * s : 0.0f;
  const _Float16 hh = (_Float16)x;
  const _Float16 ll = (_Float16)(x - (float)hh);
  P.out[((size_t)(mat * 2 + 0) * 32 + j) * kTailK + k] = __builtin_bit_cast(unsigned short, hh);
  P.out[((size_t)(mat * 2 + 1) * 32 + j) * kTailK + k] = __builtin_bit_cast(unsigned short, ll);
}

}  // namespace

bool tail_eligible(int apad, int bpad) {
  return apad > 128 && apad <= kTailK && apad % 32 == 0 && bpad > 16 && bpad <= 32;
}

void launch_tail_pack(const TailPackArgs& p, hipStream_t s) {
  hipLaunchKernelGGL(tail_pack_kernel, dim3((32 * kTailK + 255) / 256, 2), dim3(256), 0, s, p);
}

void launch_fvp_tail(const TailArgs& a, hipStream_t s) {
  if (!tail_eligible(a.apad, a.bpad) || a.b > 32 || a.a > a.apad)
    throw std::runtime_error("fvp_tail: unsupported layer shape");
  if (a.splits <= 0) return;
  if (a.rows_per_split % TR) throw std::runtime_error("fvp_tail: rows_per_split % 32");
  hipLaunchKernelGGL(fvp_tail_kernel, dim3(a.splits), dim3(NW * 64), 0, s, a);
}

}  // namespace trpo
