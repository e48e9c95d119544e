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
// global_load_lds_dwordx4 (no VGPR staging), and the waves only read fragments and issue MFMAs.
//  * 256 x 256 tile, 8 waves as 4 (rows) x 2 (columns), 2 x 4 accumulators of 32 x 32 per wave.
//  * A stage = 32 KB: a three-product segment stages 32 k of both planes, a one-product segment (low_seg)
//    64 k of the hi plane; B stages the same way from its split planes.  A ring of SA stages (HBM, SA - 1
//    in flight), B ring of 2 (L2-resident).  One barrier per stage; the counted vmcnt retires stage t's
//    DMA while stage t + 1's A stays in flight.
//  * LDS rows are 64 B (32 k) or 128 B (64 k); the 16-B chunk c of row r sits at c ^ ((r >> 2) & 3) resp.
//    c ^ ((r >> 1) & 7), so the ds_read_b128 fragment reads of 16-lane groups hit 16 distinct bank slots.
//    The DMA destination is lane-linear, so the permutation is applied to the source addresses.
// ---------------------------------------------------------------------------
// Fragment reads + MFMAs of one staged k-block (A slot As, B slot Bs) for the 256 x 256 tile's wave (wm, wn):
// ONE = one-product layout (64 k of hi planes, 128-B rows), else three products over 32 k of hi/lo planes.
constexpr int kPlPL = 8192;
template <bool ONE, int TM, int TN>
__device__ __forceinline__ void pl_compute(const unsigned short* As, const unsigned short* Bs, f32x16 (&acc)[TM][TN],
                                           int wm, int wn, int lr, int lh) {
  constexpr int PL = kPlPL;
  if constexpr (ONE) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      f16x8 ah[TM];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int r = wm * TM * 32 + tm * 32 + lr;
        ah[tm] = *reinterpret_cast<const f16x8*>(As + r * 64 + 8 * ((2 * ks + lh) ^ ((r >> 1) & 7)));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int nn = wn * TN * 32 + tn * 32 + lr;
        const f16x8 bh = *reinterpret_cast<const f16x8*>(Bs + nn * 64 + 8 * ((2 * ks + lh) ^ ((nn >> 1) & 7)));
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[tm], bh, acc[tm][tn], 0, 0, 0);
      }
    }
  } else {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f16x8 ah[TM], al[TM];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int r = wm * TM * 32 + tm * 32 + lr;
        const int off = r * 32 + 8 * ((2 * ks + lh) ^ ((r >> 2) & 3));
        ah[tm] = *reinterpret_cast<const f16x8*>(As + off);
        al[tm] = *reinterpret_cast<const f16x8*>(As + PL + off);
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int nn = wn * TN * 32 + tn * 32 + lr;
        const int off = nn * 32 + 8 * ((2 * ks + lh) ^ ((nn >> 2) & 3));
        const f16x8 bh = *reinterpret_cast<const f16x8*>(Bs + off);
        const f16x8 bl = *reinterpret_cast<const f16x8*>(Bs + PL + off);
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

// The IPW DMAs of one wave for one operand of one stage (IPW = 32 / waves: a stage is 32 KB per operand),
// as buffer_load_dwordx4 ... lds: `rsrc` covers the operand from the tile's first row, soffset `soff0` is the
// stage's first k (bytes) and instruction i adds the uniform i * rows_per_instr * row stride; v_even / v_odd
// are the lane's byte offsets for the even / odd instructions (the chunk swizzle of the one-product layout
// flips with the parity of the 8-row block, the three-product one does not).  `lds0` = the uniform LDS byte
// address of this wave's first 1-KB block of the stage's slot (M0; lane-linear destination).
// ONE: 8 rows x 128 B per instruction, rows 8 (w IPW + i) + lane / 8; else 16 rows x 64 B, rows
// 16 ((w mod NW/2) IPW + i) + lane / 4 of the plane w / (NW/2) that rsrc addresses.
template <bool ONE, int IPW>
__device__ __forceinline__ void pl_dma(__amdgpu_buffer_rsrc_t rsrc, int soff0, int stride_b, unsigned v_even,
                                       unsigned v_odd, unsigned lds0) {
  constexpr int RPI = ONE ? 8 : 16;
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    unsigned keep;
    // M0 is saved and restored around the DMA (the compiler owns it); no "memory" clobber (see glds16s)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"((i & 1) ? v_odd : v_even), "s"(rsrc), "s"(lds0 + 1024u * i), "s"(soff0 + i * RPI * stride_b));
  }
}
// the lane's offsets of pl_dma for a row stride of stride_b bytes
template <int NW>
__device__ __forceinline__ void pl_dma_offsets(int wave, int lane, int stride_b, unsigned& v3, unsigned& v1e,
                                               unsigned& v1o) {
  constexpr int IPW = 32 / NW;
  const int q = lane >> 4;
  v3 = (unsigned)(((wave % (NW / 2)) * IPW * 16 + (lane >> 2)) * stride_b + 16 * ((lane & 3) ^ (q & 3)));
  const int r1 = wave * IPW * 8 + (lane >> 3);
  v1e = (unsigned)(r1 * stride_b + 16 * ((lane & 7) ^ q));
  v1o = (unsigned)(r1 * stride_b + 16 * ((lane & 7) ^ (q + 4)));
}

template <int N>
__device__ __forceinline__ void pl_wait_vm() {
  if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)");
  else static_assert(N == 4 || N == 2, "vmcnt count");
}

template <int EPI, int SA, int NW>
__global__ void __launch_bounds__(NW * 64, NW / 4)
rowgemm_pl_kernel(const RowGemmArgs args) {
  // NW = 8: waves 4 x 2, 2 x 4 accumulators each (256 VGPRs, 2 waves / SIMD);
  // NW = 16: waves 4 x 4, 2 x 2 accumulators each (128 VGPRs, 4 waves / SIMD)
  constexpr int WM = 4, WN = NW / 4, TM = 2, TN = 8 / WN;
  constexpr int IPW = 32 / NW;   // DMA instructions per wave and operand per stage
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int SB = 2;
  constexpr int ST = 16384;                 // u16 per stage (32 KB)
  constexpr int PL = 8192;                  // u16 per plane within a three-product stage
  __shared__ __attribute__((aligned(16))) unsigned short sm[(SA + SB) * ST];
  if (args.skip && *args.skip) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int lr = lane & 31, lh = lane >> 5;
  int mt, ntile;
  tile_of((args.Npad + BN - 1) / BN, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int M = args.M;

  // per-segment scales and product count (see rowgemm3_kernel); readfirstlane makes the (wave-uniform)
  // values provably uniform, so the per-stage choices below are scalar branches and SGPR selects
  const int eA0 = *args.seg[0].eAp;
  const int eP0 = __builtin_amdgcn_readfirstlane(eA0 + amax_exp(args.seg[0].amaxB));
  int eP1 = 0;
  if (args.nseg > 1) eP1 = __builtin_amdgcn_readfirstlane(*args.seg[1].eAp + amax_exp(args.seg[1].amaxB));
  int one0 = 0, one1 = 0;
  if (args.low_seg > 0 && args.nseg > 1) {
    const int pen0 = (!args.seg[0].amaxA || !args.seg[0].amaxB) ? 4 : 0;
    const int pen1 = (!args.seg[1].amaxA || !args.seg[1].amaxB) ? 4 : 0;
    const int q0 = amax_exp(args.seg[0].amaxA) + amax_exp(args.seg[0].amaxB);
    const int q1 = amax_exp(args.seg[1].amaxA) + amax_exp(args.seg[1].amaxB);
    one0 = __builtin_amdgcn_readfirstlane(q0 - q1 >= args.low_seg + pen1 ? 1 : 0);
    one1 = __builtin_amdgcn_readfirstlane(q1 - q0 >= args.low_seg + pen0 ? 1 : 0);
  }
  const int ns0 = one0 ? (args.seg[0].K + 63) / 64 : (args.seg[0].K + 31) / 32;
  const int ns1 = args.nseg > 1 ? (one1 ? (args.seg[1].K + 63) / 64 : (args.seg[1].K + 31) / 32) : 0;
  const int nst = ns0 + ns1;
  const uint16_t *ah0 = args.seg[0].Ah, *al0 = args.seg[0].Al, *b30 = args.seg[0].B3;
  const uint16_t *ah1 = args.seg[1].Ah, *al1 = args.seg[1].Al, *b31 = args.seg[1].B3;
  const int ldp = args.seg[0].ldp, ldk = args.seg[0].ldk, bplane = args.seg[0].plane;
  // every ordinary global load is consumed before the first DMA (hipcc would drain the ring otherwise)
  asm volatile("s_waitcnt vmcnt(0)");

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  // (no row clamps: plane arrays carry rows up to a multiple of 256 and Npad is a multiple of 256, host check)
  const int hiw = __builtin_amdgcn_readfirstlane(wave) / (NW / 2);   // three-product stages: plane of this wave
  unsigned vA3, vA1e, vA1o, vB3, vB1e, vB1o;
  pl_dma_offsets<NW>(wave, lane, ldp * 2, vA3, vA1e, vA1o);
  pl_dma_offsets<NW>(wave, lane, ldk * 2, vB3, vB1e, vB1o);
  // DMA of stage t into its ring slots (A: slot t % SA, B: slot SA + t % SB)
  const unsigned lds_sm = (unsigned)(uintptr_t)sm;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const unsigned a_bytes = (unsigned)(((int64_t)(args.M + 255) / 256 * 256 - m0) * ldp * 2);   // planes carry rows to 256
#define PL_ISSUE(t, A_SIDE)                                                                                      \
  {                                                                                                              \
    const bool s1_ = (t) >= ns0;                                                                                 \
    const int o_ = s1_ ? one1 : one0;                                                                            \
    const int k0_ = (s1_ ? (t) - ns0 : (t)) * (o_ ? 64 : 32);                                                    \
    if (A_SIDE) {                                                                                                \
      const unsigned dst_ = lds_sm + (unsigned)(((t) % SA) * ST + wv * IPW * 512) * 2u;                          \
      const uint16_t* p_ = (o_ || !hiw) ? (s1_ ? ah1 : ah0) : (s1_ ? al1 : al0);                                 \
      const __amdgpu_buffer_rsrc_t r_ =                                                                          \
          __builtin_amdgcn_make_buffer_rsrc((void*)(p_ + (size_t)m0 * ldp), 0, a_bytes, 0x00020000);             \
      if (o_) pl_dma<true, IPW>(r_, k0_ * 2, ldp * 2, vA1e, vA1o, dst_);                                         \
      else pl_dma<false, IPW>(r_, k0_ * 2, ldp * 2, vA3, vA3, dst_);                                             \
    } else {                                                                                                     \
      const unsigned dst_ = lds_sm + (unsigned)((SA + (t) % SB) * ST + wv * IPW * 512) * 2u;                     \
      const uint16_t* p_ = (s1_ ? b31 : b30) + (size_t)(o_ ? 0 : hiw) * bplane + (size_t)n0 * ldk;             \
      const __amdgpu_buffer_rsrc_t r_ =                                                                          \
          __builtin_amdgcn_make_buffer_rsrc((void*)p_, 0, (unsigned)(256 * ldk * 2), 0x00020000);              \
      if (o_) pl_dma<true, IPW>(r_, k0_ * 2, ldk * 2, vB1e, vB1o, dst_);                                         \
      else pl_dma<false, IPW>(r_, k0_ * 2, ldk * 2, vB3, vB3, dst_);                                             \
    }                                                                                                            \
  }
  // Issue order per iteration: B(t + 1), then A(t + SA - 1).  At the top of iteration t the DMAs younger
  // than B(t) are the A stages t + 1 .. t + SA - 2 (4 instructions each), so vmcnt(4 (SA - 2)) retires B(t)
  // and A(t) (both older) and leaves the rest in flight.  (No "memory" clobbers on the asm: the DMAs are
  // invisible to hipcc, and __syncthreads's workgroup fences order the fragment reads; hipcc knows of no
  // outstanding VMEM op in the loop, so its fence adds only lgkmcnt(0).)
  static_assert(SA == 3, "ring depth: (SA + 2) x 32 KB of LDS");
#define PL_TOP(t)                                                                                                \
  {                                                                                                              \
    if ((t) + 1 < nst) pl_wait_vm<IPW>();                                                                        \
    else asm volatile("s_waitcnt vmcnt(0)");                                                                     \
    __syncthreads(); /* stage t visible to every wave; stage t - 1's slots are free */                          \
    if ((t) + 1 < nst) PL_ISSUE((t) + 1, false)                                                                  \
    if ((t) + SA - 1 < nst) PL_ISSUE((t) + SA - 1, true)                                                         \
  }
  PL_ISSUE(0, false)
  PL_ISSUE(0, true)
  if (1 < nst) PL_ISSUE(1, true)
  // one loop per segment and layout, so the accumulators stay put (no phis across layout branches)
#define PL_LOOP(t0, t1, ONE)                                                                                     \
  for (int t = (t0); t < (t1); ++t) {                                                                            \
    PL_TOP(t)                                                                                                    \
    pl_compute<ONE, TM, TN>(sm + (t % SA) * ST, sm + (SA + t % SB) * ST, acc, wm, wn, lr, lh);                          \
  }
  if (one0) PL_LOOP(0, ns0, true)
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
  row_epilogue<WM, WN, TM, TN, EPI, true>(args, acc, m0, n0, wm, wn, lr, lh,
                                           reinterpret_cast<float(*)[16]>(sm));
}

template <int EPI>
void launch_row_pl(const RowGemmArgs& a, hipStream_t s) {
  if (!a.f16) throw std::runtime_error("pre-split row GEMM: f16 split only");
  for (int i = 0; i < a.nseg; ++i) {
    const GemmSeg& g = a.seg[i];
    if (!g.Ah || !g.Al || !g.eAp || !g.B3 || g.ldp % 64 || g.ldp < (g.K + 63) / 64 * 64 || g.ldk % 64 ||
        g.ldk < (g.K + 63) / 64 * 64)
      throw std::runtime_error("pre-split row GEMM: segment without planes or with unaligned strides");
  }
  if (a.Npad % 256) throw std::runtime_error("pre-split row GEMM: Npad must be a multiple of 256");
  if (a.nseg > 1 && (a.seg[1].ldp != a.seg[0].ldp || a.seg[1].ldk != a.seg[0].ldk || a.seg[1].plane != a.seg[0].plane))
    throw std::runtime_error("pre-split row GEMM: segments with different strides");
  if ((int64_t)256 * a.seg[0].ldp * 2 >= (int64_t(1) << 31) || (int64_t)a.Npad * a.seg[0].ldk * 2 >= (int64_t(1) << 31))
    throw std::runtime_error("pre-split row GEMM: tile beyond the 32-bit DMA offset range");
  const long nblk = (long)((a.M + 255) / 256) * ((a.Npad + 255) / 256);
  RowGemmArgs b = a;
  b.low_seg = g_options.low_seg;
  if (g_options.pl_waves == 16)
    hipLaunchKernelGGL((rowgemm_pl_kernel<EPI, 3, 16>), dim3((unsigned)nblk), dim3(1024), 0, s, b);
  else
    hipLaunchKernelGGL((rowgemm_pl_kernel<EPI, 3, 8>), dim3((unsigned)nblk), dim3(512), 0, s, b);
}


}  // namespace

void launch_rowgemm_planes(const RowGemmArgs& a, hipStream_t s) {
  switch (a.epi) {
    case RowEpi::kTanh: launch_row_pl<(int)RowEpi::kTanh>(a, s); break;
    case RowEpi::kRHidden: launch_row_pl<(int)RowEpi::kRHidden>(a, s); break;
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
// f32 rows -> scaled f16 hi/lo planes (one thread per 8 consecutive k of a row); k in [K, ldp) and rows in
// [M, Mpad) written as zeros.  Scale 2^e with e = f16_scale_exp(max |A|) from the running-max slot (or 11,
// |A| <= 1, without one); block 0 publishes e.
__global__ void __launch_bounds__(256) split_planes_kernel(const float* __restrict__ A, int M, int Mpad, int K, int lda,
                                                           uint16_t* __restrict__ hi, uint16_t* __restrict__ lo, int ldp,
                                                           const unsigned* amax, int* e_out) {
  const int e = amax_exp(amax);   // whole wave, before any exit
  if (blockIdx.x == 0 && threadIdx.x == 0 && e_out) *e_out = e;
  const float s = __builtin_ldexpf(1.0f, e);
  const int cpr = ldp / 8;
  const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (f >= (int64_t)Mpad * cpr) return;
  const int r = (int)(f / cpr), c = (int)(f % cpr);
  f16x8 h, l;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = c * 8 + j;
    const float x = (r < M && k < K) ? A[(int64_t)r * lda + k] * s : 0.0f;
    const _Float16 hh = (_Float16)x;
    h[j] = hh;
    l[j] = (_Float16)(x - (float)hh);
  }
  *reinterpret_cast<f16x8*>(hi + (int64_t)r * ldp + c * 8) = h;
  if (lo) *reinterpret_cast<f16x8*>(lo + (int64_t)r * ldp + c * 8) = l;
}
}  // namespace

void launch_split_planes(const float* A, int M, int Mpad, int K, int lda, uint16_t* hi, uint16_t* lo, int ldp,
                         const unsigned* amax, int* e_out, hipStream_t s) {
  if (ldp % 8 || ldp < K) throw std::runtime_error("split_planes: bad ldp");
  const int64_t n = (int64_t)Mpad * (ldp / 8);
  hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, A, M, Mpad, K, lda, hi,
                     lo, ldp, amax, e_out);
}
}  // namespace trpo
