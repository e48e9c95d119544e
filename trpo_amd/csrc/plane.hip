// Pre-split f16 row GEMM (gfx950): the R-forward / R-backward row GEMMs of the FVP (trpo_inksci.py:56-70,
// SURVEY.md Appendix A) on operands whose scaled f16 hi/lo planes were written once by their producer.
#include "rowepi.h"
#include <stdexcept>

namespace trpo {
namespace {

// ---------------------------------------------------------------------------
// Pre-split row GEMM (f16 split, A as planes): C[M x 256-tile] = sum_seg (Ah + Al)_seg B_seg, then the
// row epilogue.  The A operand arrives as the scaled f16 hi/lo planes its producer wrote (GemmSeg::Ah,
// Al, eAp), so the k-loop carries no split arithmetic at all: both operands stream HBM/L2 -> LDS by
// buffer_load ... lds (no VGPR staging), and the waves only read fragments and issue MFMAs.
//  * Planes are stored k-blocked (kernels.h, GemmSeg::Ah): one stage's rows of one plane are a single
//    contiguous run, so every DMA instruction moves one contiguous KB (16 rows x 64 B).
//  * 256 x 256 tile, 8 waves as 4 (rows) x 2 (columns), 2 x 4 accumulators of 32 x 32 per wave.
//  * A stage = 32 KB = two 16-KB k-blocks of 256 rows x 32 k: a three-product segment stages block kb of
//    the hi and of the lo plane (32 k), a one-product segment (low_seg) blocks kb, kb + 1 of the hi plane
//    (64 k).  B stages the same way from its blocked split planes.  A ring of 3 stages (HBM, 2 in flight),
//    B ring of 2 (L2-resident).  One barrier per stage; the counted vmcnt retires stage t's DMA while
//    stage t + 1's A stays in flight.
//  * LDS rows are 64 B; the 16-B chunk c of row r sits at c ^ ((r >> 2) & 3), so the ds_read_b128 fragment
//    reads of 16-lane groups hit 16 distinct bank slots.  The DMA destination is lane-linear, so the
//    permutation is applied to the source offset within the KB each instruction moves.
// ---------------------------------------------------------------------------
constexpr int kPlBM = 256, kPlBN = 256, kPlNW = 8, kPlSA = 3, kPlSB = 2;
constexpr int kPlWM = 4, kPlWN = 2, kPlTM = 2, kPlTN = 4;
constexpr int kPlSub = 16384;                  // bytes per k-block of a stage (256 rows x 64 B)
constexpr int kPlStage = 2 * kPlSub;           // bytes per stage and operand
constexpr int kPlLDS = (kPlSA + kPlSB) * kPlStage;

__device__ __forceinline__ int pl_swz(int r, int c) { return c ^ ((r >> 2) & 3); }

// Fragment reads + MFMAs of one staged k-block pair (A slot As, B slot Bs, byte addresses in LDS) for
// wave (wm, wn).  ONE: one-product (64 k of hi planes in the two sub-blocks); else three products over 32 k
// (sub-block 0 hi, 1 lo).
template <bool ONE>
__device__ __forceinline__ void pl_compute(const unsigned char* As, const unsigned char* Bs,
                                           f32x16 (&acc)[kPlTM][kPlTN], int wm, int wn, int lr, int lh) {
  constexpr int TM = kPlTM, TN = kPlTN;
  if constexpr (ONE) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int sub = (ks >> 1) * kPlSub, ch = 2 * (ks & 1) + lh;
      f16x8 ah[TM];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int r = wm * TM * 32 + tm * 32 + lr;
        ah[tm] = *reinterpret_cast<const f16x8*>(As + sub + r * 64 + 16 * pl_swz(r, ch));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int nn = wn * TN * 32 + tn * 32 + lr;
        const f16x8 bh = *reinterpret_cast<const f16x8*>(Bs + sub + nn * 64 + 16 * pl_swz(nn, ch));
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[tm], bh, acc[tm][tn], 0, 0, 0);
      }
    }
  } else {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = 2 * ks + lh;
      f16x8 ah[TM], al[TM];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int r = wm * TM * 32 + tm * 32 + lr;
        const int off = r * 64 + 16 * pl_swz(r, ch);
        ah[tm] = *reinterpret_cast<const f16x8*>(As + off);
        al[tm] = *reinterpret_cast<const f16x8*>(As + kPlSub + off);
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int nn = wn * TN * 32 + tn * 32 + lr;
        const int off = nn * 64 + 16 * pl_swz(nn, ch);
        const f16x8 bh = *reinterpret_cast<const f16x8*>(Bs + off);
        const f16x8 bl = *reinterpret_cast<const f16x8*>(Bs + kPlSub + off);
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[tm], bh, acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[tm], bl, acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[tm], bh, acc[tm][tn], 0, 0, 0);
        }
      }
    }
  }
}

// The four DMAs of one wave for one operand of one stage, as buffer_load_dwordx4 ... lds: `rsrc` starts at
// this wave's first row (a contiguous 4 KB run of one k-block), instruction i moves the KB at i KB; `voff`
// is the lane's (swizzled) offset within a KB and `lds0` the uniform LDS byte address of the wave's first
// KB of the slot (M0; the destination is lane-linear).
__device__ __forceinline__ void pl_dma4(__amdgpu_buffer_rsrc_t rsrc, unsigned voff, unsigned lds0) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    unsigned keep;
    // M0 is saved and restored around the DMA (the compiler owns it).  No "memory" clobber: the DMA writes
    // a ring slot that no fragment read of this stage touches, __syncthreads's fences order it against the
    // reads of other stages, and a clobber would pin every address-taken local to the stack.
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(rsrc), "s"(lds0 + 1024u * i), "s"(1024 * i));
  }
}

// NSEG: 1 (layer 0's X-only GEMMs: no second-segment loops or one-product variants to keep registers for)
// or 2 (the runtime args.nseg)
template <int EPI, int NSEG>
__global__ void __launch_bounds__(kPlNW * 64, 2)
rowgemm_pl_kernel(const RowGemmArgs args) {
  constexpr bool kTwo = NSEG > 1;
  constexpr int WM = kPlWM, WN = kPlWN, TM = kPlTM, TN = kPlTN, BM = kPlBM, BN = kPlBN;
  constexpr int SA = kPlSA, SB = kPlSB;
  __shared__ __attribute__((aligned(16))) unsigned char sm[kPlLDS];
  if (args.skip && *args.skip) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int lr = lane & 31, lh = lane >> 5;
  int mt, ntile;
  tile_of((args.Npad + BN - 1) / BN, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;

  // per-segment scales and product count (see rowgemm3_kernel); readfirstlane makes the (wave-uniform)
  // values provably uniform, so the per-stage choices below are scalar branches and SGPR selects
  const int eA0 = *args.seg[0].eAp;
  const int eP0 = __builtin_amdgcn_readfirstlane(eA0 + amax_exp(args.seg[0].amaxB));
  int eP1 = 0;
  if (kTwo && args.nseg > 1) eP1 = __builtin_amdgcn_readfirstlane(*args.seg[1].eAp + amax_exp(args.seg[1].amaxB));
  int one0 = 0, one1 = 0;
  if (kTwo && args.low_seg > 0 && args.nseg > 1) {
    const int pen0 = (!args.seg[0].amaxA || !args.seg[0].amaxB) ? 4 : 0;
    const int pen1 = (!args.seg[1].amaxA || !args.seg[1].amaxB) ? 4 : 0;
    const int q0 = amax_exp(args.seg[0].amaxA) + amax_exp(args.seg[0].amaxB);
    const int q1 = amax_exp(args.seg[1].amaxA) + amax_exp(args.seg[1].amaxB);
    one0 = __builtin_amdgcn_readfirstlane(q0 - q1 >= args.low_seg + pen1 ? 1 : 0);
    one1 = __builtin_amdgcn_readfirstlane(q1 - q0 >= args.low_seg + pen0 ? 1 : 0);
  }
  const int ns0 = one0 ? (args.seg[0].K + 63) / 64 : (args.seg[0].K + 31) / 32;
  const int ns1 = kTwo && args.nseg > 1 ? (one1 ? (args.seg[1].K + 63) / 64 : (args.seg[1].K + 31) / 32) : 0;
  const int nst = ns0 + ns1;
  const uint16_t *ah0 = args.seg[0].Ah, *al0 = args.seg[0].Al, *b0 = args.seg[0].Bb;
  const uint16_t *ah1 = args.seg[1].Ah, *al1 = args.seg[1].Al, *b1 = args.seg[1].Bb;
  const int mpad = args.seg[0].mpad, bplane = args.seg[0].plane;
  // every ordinary global load is consumed before the first DMA (hipcc would drain the ring otherwise)
  asm volatile("s_waitcnt vmcnt(0)");

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int sub = wv >> 2;                    // the k-block (sub-block) of a stage this wave moves
  const int rows0 = (wv & 3) * 64;            // its 64 rows of that block (4 KB)
  const unsigned voff = (unsigned)((lane >> 2) * 64 + 16 * ((lane & 3) ^ ((lane >> 4) & 3)));
  const unsigned lds_sm = (unsigned)(uintptr_t)sm;
  // DMA of stage t into its ring slots (A: slot t % SA, B: slot t % SB after the A ring).  Element (r, k) of a
  // blocked plane sits at ((k / 32) * rows + r) * 32 + k % 32 (u16).
#define PL_ISSUE(t, A_SIDE)                                                                                      \
  {                                                                                                              \
    const bool s1_ = (t) >= ns0;                                                                                 \
    const int o_ = s1_ ? one1 : one0;                                                                            \
    const int kb_ = (s1_ ? (t) - ns0 : (t)) * (o_ ? 2 : 1) + (o_ ? sub : 0);   /* k-block of this wave */         \
    if (A_SIDE) {                                                                                                \
      const uint16_t* p_ = (o_ || !sub) ? (s1_ ? ah1 : ah0) : (s1_ ? al1 : al0);                                 \
      p_ += ((size_t)kb_ * mpad + m0 + rows0) * 32;                                                              \
      const __amdgpu_buffer_rsrc_t r_ = __builtin_amdgcn_make_buffer_rsrc((void*)p_, 0, 4096u, 0x00020000);      \
      pl_dma4(r_, voff, lds_sm + (unsigned)(((t) % SA) * kPlStage + wv * 4096));                                \
    } else {                                                                                                     \
      const uint16_t* p_ = (s1_ ? b1 : b0) + (size_t)(o_ ? 0 : sub) * bplane;                                    \
      p_ += ((size_t)kb_ * args.Npad + n0 + rows0) * 32;                                                         \
      const __amdgpu_buffer_rsrc_t r_ = __builtin_amdgcn_make_buffer_rsrc((void*)p_, 0, 4096u, 0x00020000);      \
      pl_dma4(r_, voff, lds_sm + (unsigned)(SA * kPlStage + ((t) % SB) * kPlStage + wv * 4096));                 \
    }                                                                                                            \
  }
  // Issue order per iteration: B(t + 1), then A(t + 2).  At the top of iteration t the DMAs younger than B(t)
  // are A(t + 1)'s 4, so vmcnt(4) retires B(t) and A(t) (both older) and leaves A(t + 1) in flight.  (No
  // "memory" clobbers on the asm: the DMAs are invisible to hipcc, and __syncthreads's workgroup fences order
  // the fragment reads; hipcc knows of no outstanding VMEM op in the loop, so its fence adds only lgkmcnt(0).)
#ifndef PL_ABLATE
#define PL_ABLATE 0   // timing ablations only (tools): 1 = no DMA in the k-loop, 2 = no fragment reads / MFMAs
#endif
#define PL_TOP(t)                                                                                                \
  {                                                                                                              \
    if ((t) + 1 < nst) asm volatile("s_waitcnt vmcnt(4)");                                                       \
    else asm volatile("s_waitcnt vmcnt(0)");                                                                     \
    __syncthreads(); /* stage t visible to every wave; stage t - 1's slots are free */                          \
    if (PL_ABLATE != 1) {                                                                                        \
      if ((t) + 1 < nst) PL_ISSUE((t) + 1, false)                                                                \
      if ((t) + SA - 1 < nst) PL_ISSUE((t) + SA - 1, true)                                                       \
    }                                                                                                            \
  }
  PL_ISSUE(0, false)
  PL_ISSUE(0, true)
  if (1 < nst) PL_ISSUE(1, true)
  // one loop per segment and layout, so the accumulators stay put (no phis across layout branches)
#define PL_LOOP(t0, t1, ONE)                                                                                     \
  for (int t = (t0); t < (t1); ++t) {                                                                            \
    PL_TOP(t)                                                                                                    \
    if (PL_ABLATE != 2)                                                                                          \
      pl_compute<ONE>(sm + (t % SA) * kPlStage, sm + (SA + t % SB) * kPlStage, acc, wm, wn, lr, lh);             \
  }
  if (kTwo && one0) PL_LOOP(0, ns0, true)
  else PL_LOOP(0, ns0, false)
  if (ns1 > 0) {
    scale_acc<TM, TN>(acc, eP1 - eP0);
    if (one1) PL_LOOP(ns0, nst, true)
    else PL_LOOP(ns0, nst, false)
  }
#undef PL_LOOP
#undef PL_TOP
#undef PL_ISSUE
  scale_acc<TM, TN>(acc, -(ns1 > 0 ? eP1 : eP0));
  __syncthreads();   // every wave's last fragment reads are done before the epilogue reuses LDS
  row_epilogue<WM, WN, TM, TN, EPI, true>(args, acc, m0, n0, wm, wn, lr, lh, reinterpret_cast<float(*)[16]>(sm));
}

template <int EPI>
void launch_row_pl(const RowGemmArgs& a, hipStream_t s) {
  if (!a.f16) throw std::runtime_error("pre-split row GEMM: f16 split only");
  for (int i = 0; i < a.nseg; ++i) {
    const GemmSeg& g = a.seg[i];
    if (!g.Ah || !g.Al || !g.eAp || !g.Bb || g.ldp % 64 || g.ldp < (g.K + 63) / 64 * 64 || g.ldk % 64 ||
        g.ldk < (g.K + 63) / 64 * 64 || g.mpad % 256 || g.mpad < a.M || g.plane != (g.ldk / 32) * a.Npad * 32)
      throw std::runtime_error("pre-split row GEMM: segment without blocked planes or with unaligned strides");
  }
  if (a.Npad % 256) throw std::runtime_error("pre-split row GEMM: Npad must be a multiple of 256");
  if (a.nseg > 1 && (a.seg[1].mpad != a.seg[0].mpad || a.seg[1].plane != a.seg[0].plane))
    throw std::runtime_error("pre-split row GEMM: segments with different strides");
  RowGemmArgs b = a;
  b.low_seg = g_options.low_seg;
  const long nblk = (long)((a.M + kPlBM - 1) / kPlBM) * (a.Npad / kPlBN);
  if (a.nseg == 1) hipLaunchKernelGGL((rowgemm_pl_kernel<EPI, 1>), dim3((unsigned)nblk), dim3(kPlNW * 64), 0, s, b);
  else hipLaunchKernelGGL((rowgemm_pl_kernel<EPI, 2>), dim3((unsigned)nblk), dim3(kPlNW * 64), 0, s, b);
}

}  // namespace

void launch_rowgemm_planes(const RowGemmArgs& a, hipStream_t s) {
  switch (a.epi) {
    case RowEpi::kTanh: launch_row_pl<(int)RowEpi::kTanh>(a, s); break;
    case RowEpi::kRHidden: launch_row_pl<(int)RowEpi::kRHidden>(a, s); break;
    case RowEpi::kRZ: launch_row_pl<(int)RowEpi::kRZ>(a, s); break;
    case RowEpi::kPrepBwd: launch_row_pl<(int)RowEpi::kPrepBwd>(a, s); break;
    case RowEpi::kPgBwd: launch_row_pl<(int)RowEpi::kPgBwd>(a, s); break;
    case RowEpi::kPrepBwdE: launch_row_pl<(int)RowEpi::kPrepBwdE>(a, s); break;
    case RowEpi::kRBwd: launch_row_pl<(int)RowEpi::kRBwd>(a, s); break;
    default: throw std::runtime_error("pre-split row GEMM: epilogue not supported");
  }
}

}  // namespace trpo

namespace trpo {
namespace {
// f32 rows -> scaled f16 hi/lo planes, k-blocked (GemmSeg::Ah): one thread per 8 consecutive k of a row;
// k in [K, ldp) and rows in [M, Mpad) are written as zeros.  Scale 2^e with e = f16_scale_exp(max |A|) from
// the running-max slot (or 11, |A| <= 1, without one); block 0 publishes e.
__global__ void __launch_bounds__(256) split_planes_kernel(const float* __restrict__ A, int M, int Mpad, int K, int lda,
                                                           uint16_t* __restrict__ hi, uint16_t* __restrict__ lo, int ldp,
                                                           const unsigned* amax, int* e_out) {
  const int e = amax_exp(amax);   // whole wave, before any exit
  if (blockIdx.x == 0 && threadIdx.x == 0 && e_out) *e_out = e;
  const float s = __builtin_ldexpf(1.0f, e);
  // consecutive threads: consecutive 8-k chunks of one 32-k block of consecutive rows (coalesced stores);
  // a grid-stride loop over the chunks (one running-max read per thread, not per 8 values)
  const int64_t nchunk = (int64_t)Mpad * (ldp / 8);
  const bool vec = (lda & 3) == 0;
  for (int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x; f < nchunk; f += (int64_t)gridDim.x * 256) {
    const int64_t kb = f / ((int64_t)Mpad * 4);
    const int64_t rem = f % ((int64_t)Mpad * 4);
    const int r = (int)(rem / 4), c = (int)(rem % 4);
    const int k0 = (int)kb * 32 + c * 8;
    float x[8];
    if (vec && r < M && k0 + 8 <= K) {
      const float4 a = *reinterpret_cast<const float4*>(A + (int64_t)r * lda + k0);
      const float4 b = *reinterpret_cast<const float4*>(A + (int64_t)r * lda + k0 + 4);
      x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
      x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = (r < M && k0 + j < K) ? A[(int64_t)r * lda + k0 + j] : 0.0f;
    }
    f16x8 h, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = x[j] * s;
      const _Float16 hh = (_Float16)v;
      h[j] = hh;
      l[j] = (_Float16)(v - (float)hh);
    }
    const int64_t o = (kb * Mpad + r) * 32 + c * 8;
    *reinterpret_cast<f16x8*>(hi + o) = h;
    if (lo) *reinterpret_cast<f16x8*>(lo + o) = l;
  }
}

// [P][R][ld] planes (k contiguous, ld a multiple of 32) -> k-blocked [P][ld / 32][R][32]
__global__ void __launch_bounds__(256) block_planes_kernel(const uint16_t* __restrict__ src, int P, int R, int ld,
                                                           uint16_t* __restrict__ dst) {
  const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;   // one 8-element chunk
  const int64_t per = (int64_t)R * (ld / 8);
  if (f >= per * P) return;
  const int p = (int)(f / per);
  const int64_t rem = f % per;
  const int r = (int)(rem / (ld / 8)), c = (int)(rem % (ld / 8));
  const f16x8 v = *reinterpret_cast<const f16x8*>(src + (int64_t)p * R * ld + (int64_t)r * ld + c * 8);
  const int k = c * 8;
  *reinterpret_cast<f16x8*>(dst + (int64_t)p * R * ld + ((int64_t)(k >> 5) * R + r) * 32 + (k & 31)) = v;
}
}  // namespace

void launch_split_planes(const float* A, int M, int Mpad, int K, int lda, uint16_t* hi, uint16_t* lo, int ldp,
                         const unsigned* amax, int* e_out, hipStream_t s) {
  if (ldp % 32 || ldp < K || Mpad < M) throw std::runtime_error("split_planes: bad ldp / Mpad");
  const int64_t n = (int64_t)Mpad * (ldp / 8);
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)blocks), dim3(256), 0, s, A, M, Mpad, K, lda, hi,
                     lo, ldp, amax, e_out);
}

void launch_block_planes(const uint16_t* src, int P, int R, int ld, uint16_t* dst, hipStream_t s) {
  if (ld % 32) throw std::runtime_error("block_planes: ld must be a multiple of 32");
  const int64_t n = (int64_t)P * R * (ld / 8);
  hipLaunchKernelGGL(block_planes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, P, R, ld, dst);
}
}  // namespace trpo
