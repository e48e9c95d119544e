// R-backward into the first hidden layer fused with layer 0's weight R-gradient (gfx950).
//
// The per-layer FVP writes RD_0 = ([RD_1 | D_1] [W_1^T ; V_1^T]) (1 - H_1^2) + E_0 RH_1 to HBM in one row GEMM
// and reads it back with X in a weight-gradient GEMM (X^T RD_0 and its column sums: Hv's W_0 / b_0 blocks,
// trpo_inksci.py:56-70 through SURVEY.md Appendix A).  RD_0 has no other reader, so here it never leaves the
// registers: per 128-row tile the row GEMM's accumulators become RD_0 in the epilogue and then, unchanged,
// the B operand of the X^T RD_0 product, whose A operand (X^T) comes from an LDS image of X's pre-split
// f16 planes.  Per row that removes RD_0's write and read (2 x 4 B per hidden column) and the second pass
// over X.  The same kernel with one segment and no E term is the policy gradient's DS_0 = (DS_1 W_1^T)
// (1 - H_1^2) with X^T DS_0 (trpo_inksci.py:54).
//
// Layout (32x32x16 f16 MFMA; lane l, r = l & 31, h = l >> 5; C: col = r, row = (i & 3) + 8 (i >> 2) + 4h):
//   * 8 waves, one workgroup per split-K slab; wave w owns RD_0's columns [32w, 32w + 32) and all 128 rows of
//     a tile (4 accumulator tiles), so its accumulator registers hold, for k-step s of the row-reduced
//     product, rows 16s + 8(j >> 2) + 4h + (j & 3) of its 32 columns in registers 8(s & 1) + j of tile s >> 1:
//     exactly a B operand (lane = column, 8 k-values) once split into f16 hi + lo.
//   * X's tile image in LDS is [row][obs] per plane, 8-row x 32-column subtiles of 512 B with the 16-B chunks
//     XOR-swizzled (cdna_hip_programming.md T10, image (a)); ds_read_b64_tr_b16 returns lane (obs m, h) the
//     4 rows 16s + 8t + 4h .. +3 of column m, the matching A operand.  The image arrives by LDS-DMA
//     (buffer_load ... lds) at the start of each tile, overlapped with the k-loop.
//   * k-loop: the register-staged f16 split of rowgemm3_kernel (A split on the way to LDS, B from the
//     engine's pre-split weight planes), BK = 32 (R0_BK), two k-tiles of loads in flight.
//   * Scales: when segment 1 (D_1 V_1^T) sits >= low_seg binades under segment 0 (rbwd0_sw, the C4 case) its
//     tiles run first on one product from D_1's f16 hi plane at the plane's own scale, and the accumulator
//     then steps down by an exact power of two to segment 0's; otherwise the two segments share one product
//     scale (the smaller of their running-max ones) on three products.  X from its planes' exponent; RD_0 per
//     tile (workgroup max), the weight-gradient accumulator rescaled (exactly, by a power of two) whenever a
//     tile needs a smaller exponent than the running one, and unscaled once at the end.
#include "rowepi.h"
#include <stdexcept>
#include <type_traits>

namespace trpo {
namespace {

#ifndef R0_ROWS
#define R0_ROWS 128  // rows per tile
#endif
#ifndef R0_EC
#define R0_EC 4      // epilogue chunk: accumulator registers per load batch
#endif
#ifndef R0_ELA
#define R0_ELA 2     // epilogue chunks of loads in flight ahead of the one being applied (two segments: H, E, RH;
                     // 3 spill 25 VGPRs). C4 A/B (profiles/r5ela): 1 -> 2 10.58 -> 10.49 ms
#endif
#ifndef R0_ELA1
#define R0_ELA1 6    // the same for one segment (policy gradient: H only): 2 -> 6 6.76 -> 6.67 ms (profiles/r5pgla)
#endif
#ifndef R0_NW
#define R0_NW 8      // waves per workgroup
#endif
#ifndef R0_BK
#define R0_BK 32     // k per staged k-tile: 16 (32-B LDS rows) or 32 (64-B rows; the X image then reuses the
                     // staging buffers after the k-loop). C4 A/B (profiles/r3j): 12.04 ms at 32 / PF 2 against
                     // 12.83 at 16 / PF 4
#endif
#ifndef R0_PF
#if R0_BK == 32
#define R0_PF 2      // k-tiles of A / B loads in flight (register stages): 2 or 4
#else
#define R0_PF 4
#endif
#endif
constexpr int kR0Rows = R0_ROWS;              // rows per tile
constexpr int kR0NW = R0_NW;                  // waves
constexpr int kR0CT = 8 / kR0NW;              // 32-column tiles per wave: wave w owns RD_0 columns [32 CT w, ..)
constexpr int kR0NT = kR0NW * 64;             // threads
constexpr int kR0BK = R0_BK;
constexpr int kR0TM = kR0Rows / 32;           // accumulator row tiles per wave (all rows of the tile)
constexpr int kR0XT = 4;                      // 32-column tiles of X (obs <= 128)
constexpr int kR0APL = kR0Rows * kR0BK;       // u16 per A plane per stage
constexpr int kR0BPL = 256 * kR0BK;           // u16 per B plane per stage
constexpr int kR0STG = 2 * (kR0APL + kR0BPL); // u16 per stage (hi + lo planes of A and B)
constexpr int kR0XPL = kR0Rows * 128;         // u16 per X plane image
constexpr int kR0AI = kR0APL / 4 / kR0NT;     // f32x4 A staging items per thread
constexpr int kR0BI = 2 * kR0BPL / 8 / kR0NT; // u16x8 B staging items per thread
constexpr int kR0XP = 2 * kR0XPL * 2 / 1024;  // 1-KB X DMA pieces per tile (both planes)
constexpr int kR0XD = kR0XP / kR0NW;          // ... per wave
constexpr bool kR0XAlias = (2 * kR0STG + 2 * kR0XPL) * 2 + 64 > 160 * 1024;   // X image in the staging bytes
constexpr int kR0LDSU = kR0XAlias ? (2 * kR0STG > 2 * kR0XPL ? 2 * kR0STG : 2 * kR0XPL) : 2 * kR0STG + 2 * kR0XPL;
static_assert(kR0LDSU * 2 <= 160 * 1024, "rbwd0 LDS");
static_assert(kR0BK == 16 || kR0BK == 32, "rbwd0 k-tile");

// u16 offset of the 16-B chunk c (8 k) of row r in a staged [row][kR0BK] f16 image: 32-B rows flip their two
// chunks on row bit 2 ^ bit 3 (swz16), 64-B rows XOR theirs with row bits 2-3 (plane.hip's pl_swz); both keep
// the ds_read_b128 fragment reads of a 16-lane group on 16 distinct bank slots
__device__ __forceinline__ int swzk(int r, int c) {
  if constexpr (kR0BK == 16) return swz16(r, c);
  else return r * 32 + ((c ^ ((r >> 2) & 3)) << 3);
}
static_assert(kR0AI >= 1 && kR0APL % (4 * kR0NT) == 0 && kR0XP % kR0NW == 0, "rbwd0 tile shape");

// byte offset of the 16-B chunk `ch` (8 obs) of `row` in an X plane image: 8-row x 32-column subtiles of
// 512 B, chunks XOR-swizzled by row bits 2-3 (conflict-free ds_read_b64_tr_b16 of 4 rows x 16 columns)
__device__ __forceinline__ int xoff(int row, int ch) {
  return 2048 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}

// one 16-B-per-lane LDS-DMA (buffer_load_dwordx4 ... lds): lane-linear destination at the wave-uniform LDS
// byte address `lds`, per-lane source offset `voff` in the descriptor `rsrc` (M0 saved and restored)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rsrc), "s"(lds), "s"(0u));
}

#ifndef R0_ABL
#define R0_ABL 0   // timing ablations only (A/B builds): 1 no X^T RD_0 phase, 2 no epilogue loads, 3 no k-loop
#endif
typedef short s4 __attribute__((ext_vector_type(4)));
typedef short s8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));

// x * 2^e -> f16 hi + lo for 8 values (round toward zero: x - hi exact, hi + lo within 2^-21 |x|)
__device__ __forceinline__ void split8h(const float* x, float s, f16x8& hi, f16x8& lo) {
  typedef __fp16 fp16x2 __attribute__((ext_vector_type(2)));
  u32x4v H, L;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = x[2 * i] * s, b = x[2 * i + 1] * s;
    const fp16x2 hp = __builtin_amdgcn_cvt_pkrtz(a, b);
    const fp16x2 lp = __builtin_amdgcn_cvt_pkrtz(a - (float)hp[0], b - (float)hp[1]);
    H[i] = __builtin_bit_cast(unsigned, hp);
    L[i] = __builtin_bit_cast(unsigned, lp);
  }
  hi = __builtin_bit_cast(f16x8, H);
  lo = __builtin_bit_cast(f16x8, L);
}

__device__ __forceinline__ f32x16 mfma3h(const f16x8& ah, const f16x8& al, const f16x8& bh, const f16x8& bl,
                                         f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
}

// NSEG = 2: FVP ([RD_1 | D_1], with the E RH term); NSEG = 1: policy gradient (DS_1, no E term)
// SW: segment 1 on one product from D_1's hi plane (decided per launch on the device, rbwd0_sw); the two
// variants are separate instantiations so neither carries the other's live ranges
template <int NSEG, bool SW>
__device__ __forceinline__ void rbwd0_body(const RBwd0Args& A, unsigned short* smem, float* sMax) {
  constexpr bool kE = NSEG == 2;
  constexpr int TM = kR0TM, CT = kR0CT;

  const int tid0 = threadIdx.x;
  const int r0 = blockIdx.x * A.rows_per_split;
  const int r1 = min(A.rows, r0 + A.rows_per_split);
  const int wv = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  const int Npad = A.Npad, lda = A.lda, K = A.K;
  constexpr int kOob = 0x40000000;

  // ---- scales: both segments' products share one power-of-two scale 2^eP, the smaller of their
  //      running-max product scales (rowgemm3_kernel's per-segment eA + eB): the dominant segment's A is
  //      scaled as in rowgemm3_kernel, the other's below its own optimum (the O(eps) D_1 V_1^T segment
  //      sits ~15 binades under, where 3 products keep it at 2^-11 of itself, 2^-26 of the dominant
  //      products).  One k-loop over both segments, no accumulator rescale, never an f16 overflow. ----
  const int eA0 = amax_exp(A.am_a0), eB0 = amax_exp(A.am_b0);
  const int eA1 = NSEG > 1 ? amax_exp(A.am_a1) : 0, eB1 = NSEG > 1 ? amax_exp(A.am_b1) : 0;
  const int eP = NSEG > 1 ? min(eA0 + eB0, eA1 + eB1) : eA0 + eB0;
  const float sA0 = __builtin_ldexpf(1.0f, eP - eB0), sA1 = __builtin_ldexpf(1.0f, eP - eB1);
  // segment 1 (D_1 V_1^T) >= low_seg binades under segment 0 (the per-layer kernels' test, rowgemm3_kernel):
  // its tiles run hi x hi alone on D_1's f16 hi plane (below), the dropped products 2^-11 of the segment,
  // 2^-(11 + low_seg) of the output
  int one1 = 0;
  if (NSEG > 1 && A.low_seg > 0) {
    const int pen0 = (!A.am_a0 || !A.am_b0) ? 4 : 0;
    one1 = __builtin_amdgcn_readfirstlane((eA1 + eB1) - (eA0 + eB0) >= A.low_seg + pen0 ? 1 : 0);
  }
  const int eX = __builtin_amdgcn_readfirstlane(*A.eX);

  const int nk = (K + kR0BK - 1) / kR0BK;     // k-tiles per segment
  const int ntiles = NSEG * nk;
  // sw: segment 1 on one product from the engine's per-update hi plane of D_1 (k-blocked, 64-B rows: one
  // 16-B load per thread and k-tile, half the bytes of f32 D_1). Its tiles run FIRST, at the plane's own
  // product scale 2^(eA1p + eB1); the accumulator then steps down to 2^eP (a power of two: exact) for
  // segment 0. Without the plane (or with a k-tile count the unrolled loop cannot split) both run 3 products.
  (void)one1;
  constexpr int sw = SW ? 1 : 0;   // rbwd0_sw: one1 with the plane and an even split of the k-loop
  // the plane's scale: one exponent (*eA1p) or one per 32-row tile (eA1t, hbwd.hip: row tile tm of a 128-row
  // tile steps down by its own power of two)
  const int eA1p = (sw && !A.eA1t) ? __builtin_amdgcn_readfirstlane(*A.eA1p) : 0;
  const int bbytes = (int)(2 * A.plane * 2);

  const unsigned xbytes = (unsigned)A.x_ldp * (unsigned)A.x_mpad * 2u;
  const __amdgpu_buffer_rsrc_t rXh = __builtin_amdgcn_make_buffer_rsrc((void*)A.Xh, 0, xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rXl = __builtin_amdgcn_make_buffer_rsrc((void*)A.Xl, 0, xbytes, 0x00020000);
  unsigned short* const sX = smem + (kR0XAlias ? 0 : 2 * kR0STG);
  const unsigned lds_x = (unsigned)(uintptr_t)sX;

  // lane-dependent values are recomputed per tile from an opaque copy of the thread id: hoisted out of
  // the tile loop they stayed live across it (hundreds of registers of offsets, spilled)
  auto lane_of = [&]() {
    int t = tid0;
    asm volatile("" : "+v"(t));
    return t;
  };
  f32x16 G[kR0XT][CT];   // X^T RD_0 for this wave's 64 columns; scaled by 2^(eX + Eacc)
#pragma unroll
  for (int i = 0; i < kR0XT; ++i)
#pragma unroll
    for (int j = 0; j < CT; ++j) G[i][j] = f32x16{};
  int Eacc = 1 << 20;   // sentinel: no nonzero tile yet
  float bsum[CT] = {};  // colsum of RD_0 over this lane's rows, columns col0 + 32 tn + lr

  for (int t0 = r0; t0 < r1; t0 += kR0Rows) {
    const int Mt = min(kR0Rows, r1 - t0);
    const int tid = lane_of(), lane = tid & 63, w = tid >> 6;
    const int lr = lane & 31, lh = lane >> 5;
    const int col0 = 32 * CT * w;
    // X image DMA: wave w moves 1-KB pieces kR0XD w .. of the two 32-KB plane images; the source of lane
    // `lane` in piece kb (row 0 of the tile; + 64 B per tile row)
    auto xsrc = [&](int kb) {
      const int o = (kb % (kR0XP / 2)) * 1024 + 16 * lane;   // byte offset in the plane image
      const int row = 8 * (o >> 11) + ((o >> 6) & 7);
      const int ch = 4 * ((o >> 9) & 3) + (((o >> 4) & 3) ^ ((row >> 2) & 3));
      return (unsigned)(((ch >> 2) * A.x_mpad + row) * 32 + 8 * (ch & 3)) * 2u;
    };
    // X tile image (the previous tile's G phase is behind the loop-end barrier), overlapped with the k-loop
    auto x_dma = [&]() {
#pragma unroll
      for (int i = 0; i < kR0XD; ++i) {
        const int kb = kR0XD * wv + i;   // wave-uniform: descriptor and LDS address in SGPRs
        const int pl = kb / (kR0XP / 2);
        dma16(pl ? rXl : rXh, xsrc(kb) + (unsigned)t0 * 64u,
              lds_x + (unsigned)(pl * kR0XPL * 2 + (kb % (kR0XP / 2)) * 1024));
      }
    };
    if (!kR0XAlias) x_dma();

    // ---- k-loop: acc = [A0 | A1] [B0 ; B1] on the f16 split ----
    f32x16 acc[TM][CT];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < CT; ++j) acc[i][j] = f32x16{};
    struct Stage {
      f32x4 ra[kR0AI];
      u16x8 rb[kR0BI];
    };
    // tile t: segment 1 is tiles [0, nk) under sw, [nk, 2 nk) otherwise; pt = a D_1 hi-plane tile
    auto gload = [&](Stage& st, int t) {
      // segment 1 exists only for NSEG == 2 (compile time): a one-segment launch never forms an A1 / B1
      // address, whatever tile index reaches here
      const bool pt = sw && t < nk;
      const bool s1 = NSEG > 1 && (sw ? t < nk : t >= nk);
      const int kt = (NSEG > 1 && t >= nk) ? t - nk : t;
      const int k0 = kt * kR0BK;
      if (pt) {
        // rows past the tile's Mt read 0 (the next split's rows are in the plane)
        const __amdgpu_buffer_rsrc_t rP = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(A.A1h + ((size_t)kt * A.a1_mpad + t0) * 32), 0, Mt * 64, 0x00020000);
        st.ra[0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rP, 16 * tid, 0, 0));
      } else {
        const float* Ap = s1 ? A.A1 : A.A0;
        const __amdgpu_buffer_rsrc_t rA =
            __builtin_amdgcn_make_buffer_rsrc((void*)(Ap + (size_t)t0 * lda), 0, Mt * lda * 4, 0x00020000);
#pragma unroll
        for (int i = 0; i < kR0AI; ++i) {
          const int f = tid + i * kR0NT, r = f / (kR0BK / 4), kq = f % (kR0BK / 4);
          const int vo = (k0 + kR0BK > K && k0 + 4 * kq >= K) ? kOob : (r * lda + 4 * kq) * 4;
          st.ra[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rA, vo, k0 * 4, 0));
        }
      }
      const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)(s1 ? A.B1 : A.B0), 0, bbytes,
                                                                          0x00020000);
#pragma unroll
      for (int i = 0; i < kR0BI; ++i) {
        if (pt && i >= kR0BI / 2) break;   // items [kR0BI / 2, kR0BI): the lo plane, unread on one product
        constexpr int CB = kR0BK / 8;   // 16-B chunks per column and k-tile
        const int f = tid + i * kR0NT, p = f / (256 * CB), rem = f % (256 * CB), n = rem / CB, kh = rem % CB;
        // columns past Npad and k past the planes' ldk (the next column's row) read 0
        const int vo = (n < Npad && k0 + 8 * kh < A.ldk) ? (int)((p * A.plane + (int64_t)n * A.ldk + 8 * kh) * 2) : kOob;
        st.rb[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rB, vo, k0 * 2, 0));
      }
    };
    auto sstore = [&](const Stage& st, int buf, int t) {
      unsigned short* As = smem + buf * kR0STG;
      unsigned short* Bs = As + 2 * kR0APL;
      const bool pt = sw && t < nk;
      const float sa = (NSEG > 1 && (sw ? t < nk : t >= nk)) ? sA1 : sA0;   // segment 1's scale (not read on pt)
      if (pt) *reinterpret_cast<u16x8*>(As + swzk(tid >> 2, tid & 3)) = __builtin_bit_cast(u16x8, st.ra[0]);
      else
#pragma unroll
      for (int i = 0; i < kR0AI; ++i) {
        const int f = tid + i * kR0NT, r = f / (kR0BK / 4), kq = f % (kR0BK / 4);
        u16x4 h, l;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          unsigned short hh, ll;
          split2h(st.ra[i][j] * sa, hh, ll);
          h[j] = hh;
          l[j] = ll;
        }
        unsigned short* dst = As + swzk(r, kq >> 1) + 4 * (kq & 1);
        *reinterpret_cast<u16x4*>(dst) = h;
        *reinterpret_cast<u16x4*>(dst + kR0APL) = l;
      }
#pragma unroll
      for (int i = 0; i < kR0BI; ++i) {
        if (pt && i >= kR0BI / 2) break;
        constexpr int CB = kR0BK / 8;
        const int f = tid + i * kR0NT, p = f / (256 * CB), rem = f % (256 * CB);
        *reinterpret_cast<u16x8*>(Bs + p * kR0BPL + swzk(rem / CB, rem % CB)) = st.rb[i];
      }
    };
    auto compute = [&](int buf, auto one_c) {
      constexpr bool one = decltype(one_c)::value;
      const unsigned short* As = smem + buf * kR0STG;
      const unsigned short* Bs = As + 2 * kR0APL;
#pragma unroll
      for (int ks = 0; ks < kR0BK / 16; ++ks) {   // 16-k MFMA steps of the staged k-tile
        f16x8 bh[CT], bl[CT];
#pragma unroll
        for (int tn = 0; tn < CT; ++tn) {
          const int bo = swzk(col0 + 32 * tn + lr, 2 * ks + lh);
          bh[tn] = *reinterpret_cast<const f16x8*>(Bs + bo);
          if constexpr (!one) bl[tn] = *reinterpret_cast<const f16x8*>(Bs + kR0BPL + bo);
        }
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          const int ao = swzk(32 * tm + lr, 2 * ks + lh);
          const f16x8 ah = *reinterpret_cast<const f16x8*>(As + ao);
          if constexpr (one) {
#pragma unroll
            for (int tn = 0; tn < CT; ++tn)
              acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[tn], acc[tm][tn], 0, 0, 0);
          } else {
            const f16x8 al = *reinterpret_cast<const f16x8*>(As + kR0APL + ao);
#pragma unroll
            for (int tn = 0; tn < CT; ++tn) acc[tm][tn] = mfma3h(ah, al, bh[tn], bl[tn], acc[tm][tn]);
          }
        }
      }
    };
    if (R0_ABL == 3) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < CT; ++j) acc[i][j] = f32x16{} + 1.0f;
    } else {
      // segment 1's one-product tiles [0, t1) and the 3-product tiles [t1, ntiles) as two loops (t1 a multiple
      // of the unroll): their bodies differ in the compute step, and a branch there inside one loop spills
      const int t1 = sw ? nk : 0;
      // the D_1 plane's scale exponent of each 32-row tile (uniform: scalar registers across the k-loop)
      int e1s[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        e1s[i] = (sw && A.eA1t) ? __builtin_amdgcn_readfirstlane(A.eA1t[(t0 >> 5) + i]) : eA1p;
#if R0_PF == 4
      // four k-tiles of loads in flight: stage S_(j % 4) holds k-tile j from its load, issued three steps
      // ahead, until its LDS store
      Stage S0, S1, S2, S3;
      auto cl = [&](int j) { return j < ntiles ? j : ntiles - 1; };   // unconditional loads: exact vmcnt
      gload(S0, 0);
      gload(S1, cl(1));
      gload(S2, cl(2));
      gload(S3, cl(3));
      sstore(S0, 0, 0);
      lds_barrier();
      auto kloop = [&](int tb, int te, auto one_c) {
        for (int t = tb; t < te; t += 4) {
          // steps past the last k-tile (ntiles % 4 != 0) only keep the load pattern (uniform branches)
          gload(S0, cl(t + 4));
          compute(0, one_c);
          if (t + 1 < ntiles) sstore(S1, 1, t + 1);
          lds_barrier();
          gload(S1, cl(t + 5));
          if (t + 1 < ntiles) compute(1, one_c);
          if (t + 2 < ntiles) sstore(S2, 0, t + 2);
          lds_barrier();
          gload(S2, cl(t + 6));
          if (t + 2 < ntiles) compute(0, one_c);
          if (t + 3 < ntiles) sstore(S3, 1, t + 3);
          lds_barrier();
          gload(S3, cl(t + 7));
          if (t + 3 < ntiles) compute(1, one_c);
          if (t + 4 < ntiles) sstore(S0, 0, t + 4);
          lds_barrier();
        }
      };
#else
      // two k-tiles of loads in flight
      Stage S0, S1;
      gload(S0, 0);
      gload(S1, ntiles > 1 ? 1 : 0);
      sstore(S0, 0, 0);
      lds_barrier();
      auto kloop = [&](int tb, int te, auto one_c) {
        for (int t = tb; t < te; t += 2) {
          gload(S0, t + 2 < ntiles ? t + 2 : ntiles - 1);   // unconditional: keeps vmcnt counting exact
          compute(0, one_c);
          if (t + 1 < ntiles) sstore(S1, 1, t + 1);
          lds_barrier();
          gload(S1, t + 3 < ntiles ? t + 3 : ntiles - 1);
          if (t + 1 < ntiles) compute(1, one_c);
          if (t + 2 < ntiles) sstore(S0, 0, t + 2);
          lds_barrier();
        }
      };
#endif
      kloop(0, t1, std::true_type{});
      if (sw) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const float f = __builtin_ldexpf(1.0f, eP - (e1s[i] + eB1));
#pragma unroll
          for (int j = 0; j < CT; ++j) acc[i][j] *= f;
        }
      }
      kloop(t1, ntiles, std::false_type{});
    }
    if (kR0XAlias) {
      // the X image takes the staging buffers' bytes: every wave is past its last fragment read first
      __syncthreads();
      x_dma();
    }
    {
      const float f = __builtin_ldexpf(1.0f, -eP);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < CT; ++j) acc[i][j] *= f;
    }

    // ---- epilogue: RD_0 = acc (1 - H^2) + E RH in place (rows past the split read 0: RD_0 = 0) ----
    {
      const int tb = Mt * Npad * 4;
      auto mk = [&](const float* p) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)(p + (size_t)t0 * Npad), 0, tb, 0x00020000);
      };
      const __amdgpu_buffer_rsrc_t rH = mk(A.H), rE = mk(kE ? A.E : A.H), rRH = mk(kE ? A.RH : A.H);
      // chunks of EC registers of one accumulator tile, the next LA chunks' loads in flight
      constexpr int EC = R0_EC, LA = kE ? R0_ELA : R0_ELA1;
      float pre[LA + 1][3][EC];
      auto load_part = [&](int c, float (&d)[3][EC]) {
        constexpr int PPT = 16 / EC;   // chunks per accumulator tile
        const int tn = c % CT, tm = (c / CT) / PPT, hf = (c / CT) % PPT;
        const int vo = col0 + 32 * tn < Npad ? ((4 * lh) * Npad + col0 + 32 * tn + lr) * 4 : kOob;
#pragma unroll
        for (int j = 0; j < EC; ++j) {
          const int r = EC * hf + j;
          const int so = (32 * tm + (r & 3) + 8 * (r >> 2)) * Npad * 4;
          if constexpr (R0_ABL == 2) {
            d[0][j] = 0.5f;
            d[1][j] = d[2][j] = 0.25f;
            continue;
          }
          d[0][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rH, vo, so, 0));
          if constexpr (kE) {
            d[1][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rE, vo, so, 0));
            d[2][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rRH, vo, so, 0));
          } else {
            d[1][j] = 0.0f;
            d[2][j] = 0.0f;
          }
        }
      };
      constexpr int NC = (16 / EC) * TM * CT;
#pragma unroll
      for (int c = 0; c < LA && c < NC; ++c) load_part(c, pre[c]);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (c + LA < NC) load_part(c + LA, pre[(c + LA) % (LA + 1)]);
        const float (&op)[3][EC] = pre[c % (LA + 1)];
        const int tn = c % CT, tm = (c / CT) / (16 / EC), hf = (c / CT) % (16 / EC);
#pragma unroll
        for (int j = 0; j < EC; ++j) {
          const int r = EC * hf + j;
          acc[tm][tn][r] = fmaf(op[1][j], op[2][j], acc[tm][tn][r] * one_minus_sq(op[0][j]));
        }
        // no stores here to pin the loads: keep the scheduler from hoisting every chunk's loads
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    float mx = 0.0f;
#pragma unroll
    for (int tn = 0; tn < CT; ++tn)
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          bsum[tn] += acc[tm][tn][r];
          mx = fmaxf(mx, fabsf(acc[tm][tn][r]));
        }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
    if (lane == 0) sMax[w] = mx;
    // the X image has landed (this wave's DMAs: vmcnt; every wave's: the barrier)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float mt = 0.0f;
#pragma unroll
    for (int u = 0; u < kR0NW; ++u) mt = fmaxf(mt, sMax[u]);
    if (R0_ABL != 1 && mt > 0.0f) {
      // RD_0's tile exponent; the accumulator follows the smallest one so far (no f16 overflow)
      const int et = f16_scale_exp(mt);
      if (et < Eacc) {
        if (Eacc != (1 << 20)) {
          const float f = __builtin_ldexpf(1.0f, et - Eacc);
#pragma unroll
          for (int i = 0; i < kR0XT; ++i)
#pragma unroll
            for (int j = 0; j < CT; ++j) G[i][j] *= f;
        }
        Eacc = et;
      }
      const float sR = __builtin_ldexpf(1.0f, Eacc);
      // ---- G += X^T RD_0: k-step s = rows 16s .. 16s + 15 of the tile ----
      const int g4 = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
      for (int s = 0; s < 2 * TM; ++s) {
        f16x8 bh[CT], bl[CT];
#pragma unroll
        for (int tn = 0; tn < CT; ++tn) {
          float vals[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) vals[j] = acc[s >> 1][tn][8 * (s & 1) + j];
          split8h(vals, sR, bh[tn], bl[tn]);
        }
#pragma unroll
        for (int ot = 0; ot < kR0XT; ++ot) {
          f16x8 xa[2];
#pragma unroll
          for (int pl = 0; pl < 2; ++pl) {
            s8 v;
#pragma unroll
            for (int t = 0; t < 2; ++t) {
              const int row = 16 * s + 8 * t + 4 * (g4 >> 1) + q;
              const int ch = 4 * ot + 2 * (g4 & 1) + (pp >> 1);
              const s4 rr = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                  (__attribute__((address_space(3))) s4*)(sX + pl * kR0XPL + (xoff(row, ch) >> 1) + 4 * (pp & 1)));
#pragma unroll
              for (int e = 0; e < 4; ++e) v[4 * t + e] = rr[e];
            }
            xa[pl] = __builtin_bit_cast(f16x8, v);
          }
#pragma unroll
          for (int tn = 0; tn < CT; ++tn) G[ot][tn] = mfma3h(xa[0], xa[1], bh[tn], bl[tn], G[ot][tn]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __syncthreads();   // X image and staging buffers free for the next tile
  }

  // ---- this split's slab: W_0 block [obs][N] and the bias colsum ----
  const int lane = tid0 & 63, lr = lane & 31, lh = lane >> 5, col0 = 32 * CT * (tid0 >> 6);
  float* out = A.slab + (size_t)blockIdx.x * A.slab_stride;
  const float fG = Eacc == (1 << 20) ? 0.0f : __builtin_ldexpf(1.0f, -(eX + Eacc));
#pragma unroll
  for (int tn = 0; tn < CT; ++tn) {
    const int j = col0 + 32 * tn + lr;
    if (j < A.N) {
#pragma unroll
      for (int ot = 0; ot < kR0XT; ++ot)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int i = 32 * ot + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (i < A.obs) out[A.off_w + (int64_t)i * A.N + j] = G[ot][tn][r] * fG;
        }
    }
    const float bt = xadd_f<true>(bsum[tn]);   // the two lane halves' rows, same order on both
    if (lh == 0 && j < A.N) out[A.off_b + j] = bt;
  }
}

__device__ __forceinline__ bool rbwd0_sw(const RBwd0Args& A) {
  if (kR0BK != 32 || A.nseg < 2 || !A.A1h || A.low_seg <= 0) return false;
  const int nk = (A.K + kR0BK - 1) / kR0BK;
  if (nk % R0_PF) return false;
  const int q0 = amax_exp(A.am_a0) + amax_exp(A.am_b0), q1 = amax_exp(A.am_a1) + amax_exp(A.am_b1);
  const int pen0 = (!A.am_a0 || !A.am_b0) ? 4 : 0;
  return __builtin_amdgcn_readfirstlane(q1 - q0 >= A.low_seg + pen0 ? 1 : 0) != 0;
}

template <int NSEG>
__global__ void __launch_bounds__(kR0NT, 1) rbwd0_kernel(const RBwd0Args A) {
  __shared__ __attribute__((aligned(16))) unsigned short smem[kR0LDSU];
  __shared__ float sMax[kR0NW];
  if (A.skip && *A.skip) return;
  if constexpr (NSEG > 1) {
    if (rbwd0_sw(A)) {
      rbwd0_body<NSEG, true>(A, smem, sMax);
      return;
    }
  }
  rbwd0_body<NSEG, false>(A, smem, sMax);
}

}  // namespace

bool rbwd0_eligible(int obs_pad, int x_ldp, int hid_pad, int K) {
  return obs_pad <= 128 && x_ldp <= 128 && hid_pad <= 256 && hid_pad % 32 == 0 && K >= 4 && K % 4 == 0;
}

void launch_rbwd0(const RBwd0Args& a, hipStream_t s) {
  if (a.splits <= 0) return;
  if (!rbwd0_eligible(a.obs, a.x_ldp, a.Npad, a.K) || a.obs > 128 || !a.Xh || !a.Xl || !a.eX || !a.H ||
      (a.nseg > 1 && (!a.A1 || !a.B1)) || (a.E && !a.RH) || a.ldk < (a.K + 15) / 16 * 16 || a.lda < a.K)
    throw std::runtime_error("rbwd0: unsupported shape or missing operand");
  if ((int64_t)a.x_ldp * a.x_mpad * 2 >= (int64_t(1) << 32) || (int64_t)kR0Rows * a.lda * 4 >= (int64_t(1) << 31))
    throw std::runtime_error("rbwd0: operand beyond the buffer-descriptor range");
  if ((int64_t)a.splits * a.rows_per_split < a.rows) throw std::runtime_error("rbwd0: splits do not cover the rows");
  if (a.nseg != 1 && a.nseg != 2) throw std::runtime_error("rbwd0: nseg must be 1 or 2");
  if ((a.nseg == 2) != (a.E != nullptr)) throw std::runtime_error("rbwd0: the E RH term goes with two segments");
  RBwd0Args b = a;
  b.low_seg = g_options.low_seg;
  if (b.nseg == 1) {   // no absent operand is ever a null base: segment 1 aliases segment 0 (never read)
    b.A1 = b.A0;
    b.B1 = b.B0;
    b.am_a1 = b.am_a0;
    b.am_b1 = b.am_b0;
  }
  if (a.nseg == 2) hipLaunchKernelGGL(rbwd0_kernel<2>, dim3(a.splits), dim3(kR0NT), 0, s, b);
  else hipLaunchKernelGGL(rbwd0_kernel<1>, dim3(a.splits), dim3(kR0NT), 0, s, b);
}

}  // namespace trpo
