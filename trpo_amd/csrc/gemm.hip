// fp32 MFMA GEMM kernels of the TRPO update engine (gfx950 / CDNA4).
//
// Two kernel families cover every dense contraction of the policy update
// ("TF ops on the hot path"):
//
//  * rowgemm  - C[M x N] = sum_seg A_seg * B_seg over row tiles of the state
//               batch, with a fused epilogue.  It implements the policy
//               forward (trpo_inksci.py:38-40), the plain KL_ff / surr
//               backward (tf.gradients at :54,:57), the Pearlmutter R-forward
//               and R-backward of the FVP graph (:56-70), and the softmax
//               heads that produce surr/kl/ent row terms (:44-51).
//  * wgrad    - C[a x b] = sum_seg A_seg^T * B_seg reduced over the rows
//               (split-K into per-split slabs, reduced in a fixed order by
//               vec.hip): the weight/bias gradients of flatgrad (utils.py:119-122).
//
// Arithmetic: v_mfma_f32_32x32x2_f32 (exact f32 FMA chains; the f32 MFMA rate
// equals the f32 vector peak on CDNA4, MFMA frees the VALU for epilogues).
// Tiles are staged global -> registers -> LDS with one barrier per 16-deep
// k-tile (two LDS buffers).  A/B fragments for 32x32x2: lane l holds
// A[i = l&31][k] and B[k][j = l&31] with the k of lane half h = l>>5 permuted
// to 4h + s for k-step s, so A fragments come from one ds_read_b128.
#include "common.h"
#include "kernels.h"
#include <cstdlib>
#include <stdexcept>
#include <type_traits>
#include <string>

#include "rowepi.h"

namespace trpo {

static int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}
Options g_options = {env_int("TRPO_SPLIT_MFMA", 5), env_int("TRPO_SPLIT_WG", 1), env_int("TRPO_CHAIN", 1),
                     env_int("TRPO_SPLIT_F16", 1), env_int("TRPO_SPLIT_MIN_K", 0), env_int("TRPO_GRAPHS", 1),
                     env_int("TRPO_TAIL", 1), env_int("TRPO_FUSED", 3), env_int("TRPO_LOW_SEG", 14),
                     env_int("TRPO_PLANES", 1), env_int("TRPO_RBWD0", 1), env_int("TRPO_HBWD2", 2),
                     env_int("TRPO_HEAD_FWD", 1), env_int("TRPO_SPLITS", 0),
                     env_int("TRPO_PG_SPLITS", 0), env_int("TRPO_LS_FUSED", 1),
                     env_int("TRPO_CG_FUSE_REDUCE", 1), env_int("TRPO_CG_P_IMG", 1),
                     env_int("TRPO_RFWD01", 1), env_int("TRPO_FWD01", 1)};

namespace {

template <int WM, int WN, int TM, int TN, int BK, int EPI, int PF = 1>
__global__ void __launch_bounds__(WM* WN * 64, (TM * TN >= 8 || EPI == 2) ? 2 : 4)   // waves / SIMD
rowgemm_kernel(const RowGemmArgs args) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32, NT = WM * WN * 64;
  constexpr int LDA = BK + 4;   // A tile [BM][BK+4]: conflict-free ds_read_b128 column groups
  constexpr int LDB = BN + 4;   // B tile [BK][BN+4]
  constexpr int ASZ = BM * LDA, BSZ = BK * LDB;
  __shared__ __attribute__((aligned(16))) float smem[2 * (ASZ + BSZ)];
  if (args.skip && *args.skip) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int lr = lane & 31, lh = lane >> 5;
  int mt, ntile;
  tile_of((args.Npad + BN - 1) / BN, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int M = args.M;

  const int nt0 = (args.seg[0].K + BK - 1) / BK;
  const int nt1 = args.nseg > 1 ? (args.seg[1].K + BK - 1) / BK : 0;
  const int ntiles = nt0 + nt1;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  constexpr int AF4 = BM * BK / 4, BF4 = BK * BN / 4;
  constexpr int AP = (AF4 + NT - 1) / NT, BP = (BF4 + NT - 1) / NT;
  // One register stage of a k-tile.  The validity of each staged float4 is applied
  // when the registers are written to LDS (after the compute phase), so the prefetch
  // loads are not waited for early.  PF = 2 keeps two stages in flight.
  struct Stage {
    f32x4 ra[AP], rb[BP];
    bool oka[AP], okb[BP];
  };

  auto gload = [&](Stage& st, int t) {
    const bool s1 = t >= nt0;
    const float* Ap = s1 ? args.seg[1].A : args.seg[0].A;
    const float* Bp = s1 ? args.seg[1].B : args.seg[0].B;
    const int lda = s1 ? args.seg[1].lda : args.seg[0].lda;
    const int ldb = s1 ? args.seg[1].ldb : args.seg[0].ldb;
    const int K = s1 ? args.seg[1].K : args.seg[0].K;
    const int k0 = (s1 ? t - nt0 : t) * BK;
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int f = tid + i * NT;
      const int r = f / (BK / 4), kq = f % (BK / 4);
      const int row = m0 + r, k = k0 + 4 * kq;
      // branch-free guard: always load from a clamped (valid) address, select zero
      const bool ok = (AF4 % NT == 0 || f < AF4) && row < M && k < K;
      st.ra[i] = *reinterpret_cast<const f32x4*>(Ap + (size_t)(ok ? row : 0) * lda + (ok ? k : 0));
      st.oka[i] = ok;
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const int f = tid + i * NT;
      const int kr = f / (BN / 4), cq = f % (BN / 4);
      const int k = k0 + kr, col = n0 + 4 * cq;
      const bool ok = (BF4 % NT == 0 || f < BF4) && k < K && col < args.Npad;
      st.rb[i] = *reinterpret_cast<const f32x4*>(Bp + (size_t)(ok ? k : 0) * ldb + (ok ? col : 0));
      st.okb[i] = ok;
    }
  };
  auto sstore = [&](const Stage& st, int buf) {
    float* As = smem + buf * (ASZ + BSZ);
    float* Bs = As + ASZ;
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int f = tid + i * NT;
      if (AF4 % NT == 0 || f < AF4) {
        const int r = f / (BK / 4), kq = f % (BK / 4);
        *reinterpret_cast<f32x4*>(As + r * LDA + 4 * kq) = st.oka[i] ? st.ra[i] : f32x4{};
      }
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const int f = tid + i * NT;
      if (BF4 % NT == 0 || f < BF4) {
        const int kr = f / (BN / 4), cq = f % (BN / 4);
        *reinterpret_cast<f32x4*>(Bs + kr * LDB + 4 * cq) = st.okb[i] ? st.rb[i] : f32x4{};
      }
    }
  };
  auto compute = [&](int buf) {
    const float* As = smem + buf * (ASZ + BSZ);
    const float* Bs = As + ASZ;
#pragma unroll
    for (int kk = 0; kk < BK / 8; ++kk) {
      f32x4 a[TM];
      float b[TN][4];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        a[tm] = *reinterpret_cast<const f32x4*>(As + (wm * TM * 32 + tm * 32 + lr) * LDA + kk * 8 + 4 * lh);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int s = 0; s < 4; ++s)
          b[tn][s] = Bs[(kk * 8 + 4 * lh + s) * LDB + wn * TN * 32 + tn * 32 + lr];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[tm][s], b[tn][s], acc[tm][tn], 0, 0, 0);
    }
  };

  if (ntiles > 0) {
    if constexpr (PF == 1) {
      Stage S;
      gload(S, 0);
      sstore(S, 0);
      lds_barrier();
      for (int t = 0; t < ntiles; ++t) {
        if (t + 1 < ntiles) gload(S, t + 1);
        compute(t & 1);
        if (t + 1 < ntiles) sstore(S, (t + 1) & 1);
        lds_barrier();
      }
    } else {
      // two stages in flight: tile t in LDS buffer t&1, tile t+1 in a register stage,
      // tile t+2 being loaded; unrolled by two so each stage has a static name
      Stage S0, S1;
      gload(S0, 0);
      gload(S1, ntiles > 1 ? 1 : 0);
      sstore(S0, 0);
      lds_barrier();
      int t = 0;
      for (; t + 1 < ntiles; t += 2) {
        gload(S0, t + 2 < ntiles ? t + 2 : ntiles - 1);   // unconditional: keeps vmcnt counting exact
        compute(0);
        sstore(S1, 1);
        lds_barrier();
        gload(S1, t + 3 < ntiles ? t + 3 : ntiles - 1);
        compute(1);
        if (t + 2 < ntiles) sstore(S0, 0);
        lds_barrier();
      }
      if (t < ntiles) compute(0);
    }
  }

  // ---- epilogue -----------------------------------------------------------
  row_epilogue<WM, WN, TM, TN, EPI>(args, acc, m0, n0, wm, wn, lr, lh);
}



template <int WM, int WN, int TM, int TN, int EPI, int OCC, int PF, int NP, int BKT = 16>
__global__ void __launch_bounds__(WM* WN * 64, OCC)   // OCC waves / SIMD
rowgemm3_kernel(const RowGemmArgs args) {
  // NP = 3: bf16 hi/mid/lo planes, 6 products ; NP = 2: scaled f16 hi/lo planes, 3 products
  // BKT = 16: 32-B LDS rows (swz16) ; 32: 64-B rows, chunks XOR-swizzled by row bits 2-3 (plane.hip's pl_swz), two
  // MFMA k-steps per staged tile and half the barriers (B planes' ldk a multiple of 32: launch_row3_cfg)
  constexpr int BK = BKT;
  static_assert(BK == 16 || BK == 32, "rowgemm3 k-tile");
  auto swk = [](int r, int c) { return BK == 16 ? swz16(r, c) : r * 32 + ((c ^ ((r >> 2) & 3)) << 3); };
  constexpr int CB = BK / 8;   // 16-B chunks per row of a staged tile
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32, NT = WM * WN * 64;
  constexpr int APL = BM * BK, BPL = BN * BK;     // one plane
  constexpr int STG = NP * (APL + BPL);
  __shared__ __attribute__((aligned(16))) unsigned short smem[2 * STG];
  if (args.skip && *args.skip) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int lr = lane & 31, lh = lane >> 5;
  int mt, ntile;
  tile_of((args.Npad + BN - 1) / BN, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int M = args.M;

  const int nt0 = (args.seg[0].K + BK - 1) / BK;
  const int nt1 = args.nseg > 1 ? (args.seg[1].K + BK - 1) / BK : 0;
  const int ntiles = nt0 + nt1;
  // f16: per-segment operand scales 2^eA, 2^eB (products scaled by 2^(eA+eB))
  int eA0 = 0, eP0 = 0, eA1 = 0, eP1 = 0;
  if constexpr (NP == 2) {
    eA0 = amax_exp(args.seg[0].amaxA);
    eP0 = eA0 + amax_exp(args.seg[0].amaxB);
    if (args.nseg > 1) {
      eA1 = amax_exp(args.seg[1].amaxA);
      eP1 = eA1 + amax_exp(args.seg[1].amaxB);
    }
  }
  const float sA0 = __builtin_ldexpf(1.0f, eA0), sA1 = __builtin_ldexpf(1.0f, eA1);
  // f16: a segment whose product scale is >= low_seg binades above the other's (its products are at
  // most 2^(2 - low_seg) of the other segment's) runs on hi x hi alone: the dropped ah bl + al bh are
  // 2^-10 of its own magnitude, 2^(-8 - low_seg) of the other segment's -- below the 3-product split's
  // own 2^-22 at the default 14.  (The KL_ff plain-delta segments D_l V_l^T carry O(eps) terms.)
  bool one0 = false, one1 = false;
  if constexpr (NP == 2) {
    if (args.low_seg > 0 && args.nseg > 1) {
      // an operand without a running-max slot is scaled as if its max were 1 (tanh outputs): as the
      // dominant segment's it may be far below that, so the gap must then be 4 binades wider
      const int pen0 = (!args.seg[0].amaxA || !args.seg[0].amaxB) ? 4 : 0;
      const int pen1 = (!args.seg[1].amaxA || !args.seg[1].amaxB) ? 4 : 0;
      one0 = eP0 - eP1 >= args.low_seg + pen1;
      one1 = eP1 - eP0 >= args.low_seg + pen0;
    }
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  constexpr int AF4 = BM * BK / 4;          // f32x4 of A per k-tile
  constexpr int BC = NP * BN * CB;          // 16-B chunks of B planes per k-tile
  constexpr int AP = (AF4 + NT - 1) / NT, BP = (BC + NT - 1) / NT;
  // Staging loads are buffer ops on per-segment descriptors (rows [m0, M) of A; the B planes): rows past
  // M and k past the segment's K read 0 and invalid B columns address past the end, so a load is one
  // instruction with a lane-constant voffset and a scalar k offset (no 64-bit address math, no selects).
  constexpr int kOob = 0x40000000;
  const int Mt = M - m0 < BM ? M - m0 : BM;
  int vAo[AP], vBo[BP];
  const int ldA = args.seg[0].lda;   // equal across segments (host check)
#pragma unroll
  for (int i = 0; i < AP; ++i) {
    const int f = tid + i * NT;
    const int r = f / (BK / 4), kq = f % (BK / 4);
    vAo[i] = (AF4 % NT == 0 || f < AF4) ? (r * ldA + 4 * kq) * 4 : kOob;
  }
  const int ldkB = args.seg[0].ldk, planeB = args.seg[0].plane;   // equal across segments (host check)
#pragma unroll
  for (int i = 0; i < BP; ++i) {
    const int f = tid + i * NT;
    const int p = f / (BN * CB), rem = f % (BN * CB);
    const int n = rem / CB, kh = rem % CB;
    const bool ok = (BC % NT == 0 || f < BC) && n0 + n < args.Npad;
    vBo[i] = ok ? (p * planeB + (n0 + n) * ldkB + 8 * kh) * 2 : kOob;
  }
  struct Stage {
    f32x4 ra[AP];
    u16x8 rb[BP];
    bool s1;
  };
  auto gload = [&](Stage& st, int t) {
    const bool s1 = t >= nt0;
    st.s1 = s1;
    const GemmSeg& sg = s1 ? args.seg[1] : args.seg[0];
    const int K = sg.K;
    const int k0 = (s1 ? t - nt0 : t) * BK;
    const __amdgpu_buffer_rsrc_t rA =
        __builtin_amdgcn_make_buffer_rsrc((void*)(sg.A + (size_t)m0 * ldA), 0, Mt * ldA * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB =
        __builtin_amdgcn_make_buffer_rsrc((void*)sg.B3, 0, NP * planeB * 2, 0x00020000);
    const bool kpart = k0 + BK > K;   // last k-tile of a segment whose K is not a multiple of BK
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int f = tid + i * NT;
      const int kq = f % (BK / 4);
      const int vo = (kpart && k0 + 4 * kq >= K) ? kOob : vAo[i];
      st.ra[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rA, vo, k0 * 4, 0));
    }
#pragma unroll
    for (int i = 0; i < BP; ++i)
      st.rb[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rB, vBo[i], k0 * 2, 0));
  };
  auto sstore = [&](const Stage& st, int buf) {
    unsigned short* As = smem + buf * STG;
    unsigned short* Bs = As + NP * APL;
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int f = tid + i * NT;
      if (AF4 % NT == 0 || f < AF4) {
        const int r = f / (BK / 4), kq = f % (BK / 4);
        const f32x4 x = st.ra[i];
        unsigned short* dst = As + swk(r, kq >> 1) + 4 * (kq & 1);
        if constexpr (NP == 3) {
          u16x4 h, m, l;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            unsigned short hh, mm, ll;
            split3(x[j], hh, mm, ll);
            h[j] = hh;
            m[j] = mm;
            l[j] = ll;
          }
          *reinterpret_cast<u16x4*>(dst) = h;
          *reinterpret_cast<u16x4*>(dst + APL) = m;
          *reinterpret_cast<u16x4*>(dst + 2 * APL) = l;
        } else {
          const float sa = st.s1 ? sA1 : sA0;
          u16x4 h, l;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            unsigned short hh, ll;
            split2h(x[j] * sa, hh, ll);
            h[j] = hh;
            l[j] = ll;
          }
          *reinterpret_cast<u16x4*>(dst) = h;
          *reinterpret_cast<u16x4*>(dst + APL) = l;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const int f = tid + i * NT;
      if (BC % NT == 0 || f < BC) {
        const int p = f / (BN * CB), rem = f % (BN * CB);
        const int n = rem / CB, kh = rem % CB;
        *reinterpret_cast<u16x8*>(Bs + p * BPL + swk(n, kh)) = st.rb[i];
      }
    }
  };
  auto compute_p = [&](int buf, auto one_c) {
    constexpr bool ONE = decltype(one_c)::value;
    const unsigned short* As = smem + buf * STG;
    const unsigned short* Bs = As + NP * APL;
    // fragments streamed per output column tile to keep few registers live
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int bo = swk(wn * TN * 32 + tn * 32 + lr, 2 * ks + lh);
      if constexpr (NP == 2 && ONE) {
        const f16x8 b0 = *reinterpret_cast<const f16x8*>(Bs + bo);
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          const int ao = swk(wm * TM * 32 + tm * 32 + lr, 2 * ks + lh);
          const f16x8 a0 = *reinterpret_cast<const f16x8*>(As + ao);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, acc[tm][tn], 0, 0, 0);
        }
      } else if constexpr (NP == 3) {
        bf16x8 b[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) b[p] = *reinterpret_cast<const bf16x8*>(Bs + p * BPL + bo);
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          bf16x8 a[3];
          const int ao = swk(wm * TM * 32 + tm * 32 + lr, 2 * ks + lh);
#pragma unroll
          for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8*>(As + p * APL + ao);
          // smallest terms first
          f32x16 c = acc[tm][tn];
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
          acc[tm][tn] = c;
        }
      } else {
        f16x8 b[2];
#pragma unroll
        for (int p = 0; p < 2; ++p) b[p] = *reinterpret_cast<const f16x8*>(Bs + p * BPL + bo);
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          f16x8 a[2];
          const int ao = swk(wm * TM * 32 + tm * 32 + lr, 2 * ks + lh);
#pragma unroll
          for (int p = 0; p < 2; ++p) a[p] = *reinterpret_cast<const f16x8*>(As + p * APL + ao);
          f32x16 c = acc[tm][tn];
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], b[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], c, 0, 0, 0);
          acc[tm][tn] = c;
        }
      }
    }
  };
  auto compute = [&](int buf, int t) {
    if (t >= nt0 ? one1 : one0) compute_p(buf, std::true_type{});
    else compute_p(buf, std::false_type{});
  };
  // f16: when the k-tiles move from segment 0 to segment 1, bring the accumulator to segment 1's
  // product scale (powers of two: exact)
  auto seg_switch = [&](int t) {
    if constexpr (NP == 2) {
      if (t == nt0 && nt1 > 0) {
        // a real branch: the volatile asm keeps the compiler from if-converting the rescale into
        // an unconditional multiply of every accumulator on every k-tile
        asm volatile("; segment switch" ::: "memory");
        scale_acc<TM, TN>(acc, eP1 - eP0);
      }
    }
  };

  if (ntiles > 0) {
    if constexpr (PF == 1) {
      Stage S;
      gload(S, 0);
      sstore(S, 0);
      lds_barrier();
      for (int t = 0; t < ntiles; ++t) {
        if (t + 1 < ntiles) gload(S, t + 1);
        seg_switch(t);
        compute(t & 1, t);
        if (t + 1 < ntiles) sstore(S, (t + 1) & 1);
        lds_barrier();
      }
    } else {
      // two k-tiles of loads in flight (see rowgemm_kernel)
      Stage S0, S1;
      gload(S0, 0);
      gload(S1, ntiles > 1 ? 1 : 0);
      sstore(S0, 0);
      lds_barrier();
      int t = 0;
      for (; t + 1 < ntiles; t += 2) {
        gload(S0, t + 2 < ntiles ? t + 2 : ntiles - 1);   // unconditional: keeps vmcnt counting exact
        seg_switch(t);
        compute(0, t);
        sstore(S1, 1);
        lds_barrier();
        gload(S1, t + 3 < ntiles ? t + 3 : ntiles - 1);
        seg_switch(t + 1);
        compute(1, t + 1);
        if (t + 2 < ntiles) sstore(S0, 0);
        lds_barrier();
      }
      if (t < ntiles) {
        seg_switch(t);
        compute(0, t);
      }
    }
  }
  if constexpr (NP == 2) scale_acc<TM, TN>(acc, -(nt1 > 0 ? eP1 : eP0));
  row_epilogue<WM, WN, TM, TN, EPI>(args, acc, m0, n0, wm, wn, lr, lh);
}


// ---------------------------------------------------------------------------
// Split-bf16 weight gradient: C[i][j] = sum_rows A[r][i] B[r][j] with the rows as
// the MFMA k dimension (see rowgemm3_kernel for the split arithmetic).  Both
// operands are row-major activations, so staging transposes: a thread owns one
// column and 8 consecutive rows (8 coalesced dword loads), splits them and
// writes one 16-B k-chunk per plane of the [column][16 rows] LDS image.
// ---------------------------------------------------------------------------
template <int WM, int WN, int TM, int TN, int OCC, int PF, int NP>
__global__ void __launch_bounds__(WM* WN * 64, OCC)
wgrad3_kernel(const WGradArgs args) {
  constexpr int BK = 16;
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32, NT = WM * WN * 64;
  constexpr int APL = BM * BK, BPL = BN * BK;
  constexpr int STG = NP * (APL + BPL);
  __shared__ __attribute__((aligned(16))) unsigned short smem[2 * STG];
  __shared__ float cs_sh[2][BN];
  if (args.skip && *args.skip) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int lr = lane & 31, lh = lane >> 5;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN, split = blockIdx.z;
  const int r0 = split * args.rows_per_split;
  const int r1 = min(args.rows, r0 + args.rows_per_split);
  const int nk = r1 > r0 ? (r1 - r0 + BK - 1) / BK : 0;
  const int ntiles = nk * args.nseg;
  const bool do_colsum = (blockIdx.x == 0);
  // f16: operand scales per segment (see rowgemm3_kernel)
  int eA[2] = {0, 0}, eB[2] = {0, 0};
  if constexpr (NP == 2) {
    for (int g = 0; g < args.nseg && g < 2; ++g) {
      eA[g] = amax_exp(args.seg[g].amaxA);
      eB[g] = amax_exp(args.seg[g].amaxB);
    }
  }
  // f16: one product for a segment >= low_seg binades below the other (see rowgemm3_kernel)
  bool one0 = false, one1 = false;
  if constexpr (NP == 2) {
    if (args.low_seg > 0 && args.nseg > 1) {
      const int d = (eA[1] + eB[1]) - (eA[0] + eB[0]);
      const int pen0 = (!args.seg[0].amaxA || !args.seg[0].amaxB) ? 4 : 0;   // as in rowgemm3_kernel
      const int pen1 = (!args.seg[1].amaxA || !args.seg[1].amaxB) ? 4 : 0;
      one0 = -d >= args.low_seg + pen1;
      one1 = d >= args.low_seg + pen0;
    }
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  constexpr int AI = 2 * BM, BI = 2 * BN;   // (column, 8-row group) items per k-tile
  constexpr int AP = (AI + NT - 1) / NT, BP = (BI + NT - 1) / NT;
  float csum[BP];
#pragma unroll
  for (int i = 0; i < BP; ++i) csum[i] = 0.0f;
  // Per-split buffer descriptors over rows [r0, r1) of each segment operand: rows past r1 read 0 and a
  // lane whose column is out of range addresses past the end (reads 0), so a load is one buffer op with
  // a lane-constant voffset and a scalar row offset -- no per-load 64-bit address math or selects.
  auto desc = [&](const float* p, int ld) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(p + (size_t)r0 * ld), 0, (r1 - r0) * ld * 4, 0x00020000);
  };
  const int lda4 = args.seg[0].lda * 4, ldb4 = args.seg[0].ldb * 4;   // equal across segments (host check)
  constexpr int kOob = 0x40000000;
  int vA[AP], vB[BP];
#pragma unroll
  for (int i = 0; i < AP; ++i) {
    const int f = tid + i * NT;
    const int c = f % BM, g = f / BM;
    const bool okc = (AI % NT == 0 || f < AI) && m0 + c < args.Mpad;
    vA[i] = okc ? 8 * g * lda4 + (m0 + c) * 4 : kOob;
  }
#pragma unroll
  for (int i = 0; i < BP; ++i) {
    const int f = tid + i * NT;
    const int c = f % BN, g = f / BN;
    const bool okc = (BI % NT == 0 || f < BI) && n0 + c < args.Npad;
    vB[i] = okc ? 8 * g * ldb4 + (n0 + c) * 4 : kOob;
  }
  auto ldbuf = [](__amdgpu_buffer_rsrc_t r, int vo, int so) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
  };
  struct Stage {
    float va[AP][8], vb[BP][8];
    bool cs;         // this tile belongs to the column-summed segment
    int sg;          // segment
  };
  auto gload = [&](Stage& st, int t) {
    const int sg = t / nk;
    const int kt = t - sg * nk;
    st.cs = do_colsum && sg == args.colsum_seg;
    st.sg = sg;
    // descriptors from the (wave-uniform) segment's pointers, built here: a select between two
    // prebuilt descriptors came out in VGPRs and put every load in a readfirstlane loop
    const __amdgpu_buffer_rsrc_t ra = desc(sg ? args.seg[1].A : args.seg[0].A, args.seg[0].lda);
    const __amdgpu_buffer_rsrc_t rb = desc(sg ? args.seg[1].B : args.seg[0].B, args.seg[0].ldb);
    const int sa = kt * BK * lda4, sb = kt * BK * ldb4;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < AP; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) st.va[i][q] = ldbuf(ra, vA[i], sa + q * lda4);
#pragma unroll
    for (int i = 0; i < BP; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) st.vb[i][q] = ldbuf(rb, vB[i], sb + q * ldb4);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto put = [&](unsigned short* base, int plane_elems, int c, int g, const float (&v)[8], int e) {
    unsigned short* dst = base + swz16(c, g);
    if constexpr (NP == 2) {
      const float sc = __builtin_ldexpf(1.0f, e);
      u16x8 h, l;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        unsigned short hh, ll;
        split2h(v[q] * sc, hh, ll);
        h[q] = hh;
        l[q] = ll;
      }
      *reinterpret_cast<u16x8*>(dst) = h;
      *reinterpret_cast<u16x8*>(dst + plane_elems) = l;
    } else {
      u16x8 h, m, l;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        unsigned short hh, mm, ll;
        split3(v[q], hh, mm, ll);
        h[q] = hh;
        m[q] = mm;
        l[q] = ll;
      }
      *reinterpret_cast<u16x8*>(dst) = h;
      *reinterpret_cast<u16x8*>(dst + plane_elems) = m;
      *reinterpret_cast<u16x8*>(dst + 2 * plane_elems) = l;
    }
  };
  auto sstore = [&](const Stage& st, int buf) {
    unsigned short* As = smem + buf * STG;
    unsigned short* Bs = As + NP * APL;
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int f = tid + i * NT;
      if (AI % NT == 0 || f < AI) put(As, APL, f % BM, f / BM, st.va[i], eA[st.sg]);
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const int f = tid + i * NT;
      if (BI % NT == 0 || f < BI) {
        put(Bs, BPL, f % BN, f / BN, st.vb[i], eB[st.sg]);
        if (st.cs) {
          float cs = 0.0f;
#pragma unroll
          for (int q = 0; q < 8; ++q) cs += st.vb[i][q];
          csum[i] += cs;
        }
      }
    }
  };
  auto compute_p = [&](int buf, auto one_c) {
    constexpr bool ONE = decltype(one_c)::value;
    const unsigned short* As = smem + buf * STG;
    const unsigned short* Bs = As + NP * APL;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int bo = swz16(wn * TN * 32 + tn * 32 + lr, lh);
      if constexpr (NP == 2 && ONE) {
        const f16x8 b0 = *reinterpret_cast<const f16x8*>(Bs + bo);
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          const int ao = swz16(wm * TM * 32 + tm * 32 + lr, lh);
          const f16x8 a0 = *reinterpret_cast<const f16x8*>(As + ao);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, acc[tm][tn], 0, 0, 0);
        }
      } else if constexpr (NP == 3) {
        bf16x8 b[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) b[p] = *reinterpret_cast<const bf16x8*>(Bs + p * BPL + bo);
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          bf16x8 a[3];
          const int ao = swz16(wm * TM * 32 + tm * 32 + lr, lh);
#pragma unroll
          for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8*>(As + p * APL + ao);
          f32x16 c = acc[tm][tn];
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
          acc[tm][tn] = c;
        }
      } else {
        f16x8 b[2];
#pragma unroll
        for (int p = 0; p < 2; ++p) b[p] = *reinterpret_cast<const f16x8*>(Bs + p * BPL + bo);
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          f16x8 a[2];
          const int ao = swz16(wm * TM * 32 + tm * 32 + lr, lh);
#pragma unroll
          for (int p = 0; p < 2; ++p) a[p] = *reinterpret_cast<const f16x8*>(As + p * APL + ao);
          f32x16 c = acc[tm][tn];
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], b[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], c, 0, 0, 0);
          acc[tm][tn] = c;
        }
      }
    }
  };
  auto compute = [&](int buf, int t) {
    if (t >= nk ? one1 : one0) compute_p(buf, std::true_type{});
    else compute_p(buf, std::false_type{});
  };
  auto seg_switch = [&](int t) {
    if constexpr (NP == 2) {
      if (t == nk && args.nseg > 1) {
        asm volatile("; segment switch" ::: "memory");   // a real branch (see rowgemm3_kernel)
        scale_acc<TM, TN>(acc, (eA[1] + eB[1]) - (eA[0] + eB[0]));
      }
    }
  };

  if (ntiles > 0) {
    if constexpr (PF == 1) {
      Stage S;
      gload(S, 0);
      sstore(S, 0);
      lds_barrier();
      for (int t = 0; t < ntiles; ++t) {
        if (t + 1 < ntiles) gload(S, t + 1);
        seg_switch(t);
        compute(t & 1, t);
        if (t + 1 < ntiles) sstore(S, (t + 1) & 1);
        lds_barrier();
      }
    } else {
      Stage S0, S1;
      gload(S0, 0);
      gload(S1, ntiles > 1 ? 1 : 0);
      sstore(S0, 0);
      lds_barrier();
      int t = 0;
      for (; t + 1 < ntiles; t += 2) {
        gload(S0, t + 2 < ntiles ? t + 2 : ntiles - 1);
        seg_switch(t);
        compute(0, t);
        sstore(S1, 1);
        lds_barrier();
        gload(S1, t + 3 < ntiles ? t + 3 : ntiles - 1);
        seg_switch(t + 1);
        compute(1, t + 1);
        if (t + 2 < ntiles) sstore(S0, 0);
        lds_barrier();
      }
      if (t < ntiles) {
        seg_switch(t);
        compute(0, t);
      }
    }
  }
  if constexpr (NP == 2) {
    const int last = args.nseg > 1 ? 1 : 0;
    scale_acc<TM, TN>(acc, -(eA[last] + eB[last]));
  }

  float* out = args.slab + (size_t)split * args.slab_stride;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int j = n0 + wn * TN * 32 + tn * 32 + lr;
      if (j >= args.Nb) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = m0 + wm * TM * 32 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (i < args.Ma) out[args.off_w + (int64_t)i * args.Nb + j] = acc[tm][tn][r];
      }
    }
  if (do_colsum) {
    // column sums: the two 8-row groups of a column, combined in a fixed order
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const int f = tid + i * NT;
      if (BI % NT == 0 || f < BI) cs_sh[f / BN][f % BN] = csum[i];
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT)
      if (n0 + c < args.Nb) out[args.off_b + n0 + c] = cs_sh[0][c] + cs_sh[1][c];
  }
}

// One block per (64-column group of one job's planes, job); each thread writes one
// 16-B chunk (8 consecutive k) of the three planes of one column.
__global__ void __launch_bounds__(256) split_b_kernel(const SplitArgs a, const int* skip) {
  if (skip && *skip) return;
  const SplitJob& j = a.job[blockIdx.y];
  const int nchunk = j.ldk / 8;
  const int f = blockIdx.x * 256 + threadIdx.x;
  // lanes run over columns first so the f32 reads of one k row coalesce
  const int n = f % j.Npad, c = f / j.Npad;
  const float sb = a.f16 ? __builtin_ldexpf(1.0f, amax_exp(j.amax)) : 1.0f;   // whole wave, before any exit
  if (c >= nchunk) return;
  const size_t plane = (size_t)j.Npad * j.ldk;
  uint16_t* dst = j.B3 + (size_t)n * j.ldk + 8 * c;
  if (a.f16) {
    u16x8 h, l;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = 8 * c + q;
      const float x = k < j.K ? j.B[(size_t)k * j.ldb + n] : 0.0f;
      unsigned short hh, ll;
      split2h(x * sb, hh, ll);
      h[q] = hh;
      l[q] = ll;
    }
    *reinterpret_cast<u16x8*>(dst) = h;
    *reinterpret_cast<u16x8*>(dst + plane) = l;
    return;
  }
  u16x8 h, m, l;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int k = 8 * c + q;
    const float x = k < j.K ? j.B[(size_t)k * j.ldb + n] : 0.0f;
    unsigned short hh, mm, ll;
    split3(x, hh, mm, ll);
    h[q] = hh;
    m[q] = mm;
    l[q] = ll;
  }
  *reinterpret_cast<u16x8*>(dst) = h;
  *reinterpret_cast<u16x8*>(dst + plane) = m;
  *reinterpret_cast<u16x8*>(dst + 2 * plane) = l;
}

// ---------------------------------------------------------------------------
// weight-gradient kernel: k = rows (split-K), tiles [BK][BM] / [BK][BN] k-major
// ---------------------------------------------------------------------------
template <int WM, int WN, int TM, int TN, int BK = 16, int PF = 1>
__global__ void __launch_bounds__(WM* WN * 64)
wgrad_kernel(const WGradArgs args) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32, NT = WM * WN * 64;
  constexpr int LDA = BM + 4, LDB = BN + 4;
  constexpr int ASZ = BK * LDA, BSZ = BK * LDB;
  __shared__ __attribute__((aligned(16))) float smem[2 * (ASZ + BSZ)];
  if (args.skip && *args.skip) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int lr = lane & 31, lh = lane >> 5;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN, split = blockIdx.z;
  const int r0 = split * args.rows_per_split;
  const int r1 = min(args.rows, r0 + args.rows_per_split);
  const int nk = r1 > r0 ? (r1 - r0 + BK - 1) / BK : 0;
  const int ntiles = nk * args.nseg;
  const bool do_colsum = (blockIdx.x == 0);

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
  float csum = 0.0f;   // column sum of the colsum segment's B (thread tid < BN owns column n0+tid)

  constexpr int AF4 = BK * BM / 4, BF4 = BK * BN / 4;
  constexpr int AP = (AF4 + NT - 1) / NT, BP = (BF4 + NT - 1) / NT;
  struct Stage {   // masks applied at the LDS store, after compute (keeps the prefetch in flight)
    f32x4 ra[AP], rb[BP];
    bool oka[AP], okb[BP];
  };

  auto gload = [&](Stage& st, int t) {
    const int sg = t / nk;
    const int kt = t - sg * nk;
    const float* Ap = sg ? args.seg[1].A : args.seg[0].A;
    const float* Bp = sg ? args.seg[1].B : args.seg[0].B;
    const int lda = sg ? args.seg[1].lda : args.seg[0].lda;
    const int ldb = sg ? args.seg[1].ldb : args.seg[0].ldb;
    const int rb0 = r0 + kt * BK;
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int f = tid + i * NT;
      const int kr = f / (BM / 4), cq = f % (BM / 4);
      const int r = rb0 + kr, c = m0 + 4 * cq;
      const bool ok = (AF4 % NT == 0 || f < AF4) && r < r1 && c < args.Mpad;
      const f32x4 v = *reinterpret_cast<const f32x4*>(Ap + (size_t)(ok ? r : r0) * lda + (ok ? c : 0));
      st.ra[i] = v;
      st.oka[i] = ok;
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const int f = tid + i * NT;
      const int kr = f / (BN / 4), cq = f % (BN / 4);
      const int r = rb0 + kr, c = n0 + 4 * cq;
      const bool ok = (BF4 % NT == 0 || f < BF4) && r < r1 && c < args.Npad;
      const f32x4 v = *reinterpret_cast<const f32x4*>(Bp + (size_t)(ok ? r : r0) * ldb + (ok ? c : 0));
      st.rb[i] = v;
      st.okb[i] = ok;
    }
  };
  auto sstore = [&](const Stage& st, int buf) {
    float* As = smem + buf * (ASZ + BSZ);
    float* Bs = As + ASZ;
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int f = tid + i * NT;
      if (AF4 % NT == 0 || f < AF4) {
        const int kr = f / (BM / 4), cq = f % (BM / 4);
        *reinterpret_cast<f32x4*>(As + kr * LDA + 4 * cq) = st.oka[i] ? st.ra[i] : f32x4{};
      }
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const int f = tid + i * NT;
      if (BF4 % NT == 0 || f < BF4) {
        const int kr = f / (BN / 4), cq = f % (BN / 4);
        *reinterpret_cast<f32x4*>(Bs + kr * LDB + 4 * cq) = st.okb[i] ? st.rb[i] : f32x4{};
      }
    }
  };
  auto compute = [&](int buf, bool colsum) {
    const float* As = smem + buf * (ASZ + BSZ);
    const float* Bs = As + ASZ;
#pragma unroll
    for (int kk = 0; kk < BK / 8; ++kk) {
      float a[TM][4], b[TN][4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = kk * 8 + 4 * lh + s;
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) a[tm][s] = As[k * LDA + wm * TM * 32 + tm * 32 + lr];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) b[tn][s] = Bs[k * LDB + wn * TN * 32 + tn * 32 + lr];
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[tm][s], b[tn][s], acc[tm][tn], 0, 0, 0);
    }
    if (colsum && tid < BN) {
      float cs = 0.0f;
#pragma unroll
      for (int k = 0; k < BK; ++k) cs += Bs[k * LDB + tid];
      csum += cs;
    }
  };

  auto cs_of = [&](int t) { return do_colsum && (t / nk) == args.colsum_seg; };
  if (ntiles > 0) {
    if constexpr (PF == 1) {
      Stage S;
      gload(S, 0);
      sstore(S, 0);
      lds_barrier();
      for (int t = 0; t < ntiles; ++t) {
        if (t + 1 < ntiles) gload(S, t + 1);
        compute(t & 1, cs_of(t));
        if (t + 1 < ntiles) sstore(S, (t + 1) & 1);
        lds_barrier();
      }
    } else {
      Stage S0, S1;
      gload(S0, 0);
      gload(S1, ntiles > 1 ? 1 : 0);
      sstore(S0, 0);
      lds_barrier();
      int t = 0;
      for (; t + 1 < ntiles; t += 2) {
        gload(S0, t + 2 < ntiles ? t + 2 : ntiles - 1);   // unconditional: keeps vmcnt counting exact
        compute(0, cs_of(t));
        sstore(S1, 1);
        lds_barrier();
        gload(S1, t + 3 < ntiles ? t + 3 : ntiles - 1);
        compute(1, cs_of(t + 1));
        if (t + 2 < ntiles) sstore(S0, 0);
        lds_barrier();
      }
      if (t < ntiles) compute(0, cs_of(t));
    }
  }

  float* out = args.slab + (size_t)split * args.slab_stride;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int j = n0 + wn * TN * 32 + tn * 32 + lr;
      if (j >= args.Nb) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = m0 + wm * TM * 32 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (i < args.Ma) out[args.off_w + (int64_t)i * args.Nb + j] = acc[tm][tn][r];
      }
    }
  if (do_colsum && tid < BN && n0 + tid < args.Nb) out[args.off_b + n0 + tid] = csum;
}

template <int WM, int WN, int TM, int TN, int BKT, int EPI, int PF = 1>
void launch_row_cfg(const RowGemmArgs& a, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  const long nblk = (long)((a.M + BM - 1) / BM) * ((a.Npad + BN - 1) / BN);
  hipLaunchKernelGGL((rowgemm_kernel<WM, WN, TM, TN, BKT, EPI, PF>), dim3((unsigned)nblk), dim3(WM * WN * 64),
                     0, s, a);
}

template <int WM, int WN, int TM, int TN, int EPI, int OCC = 2, int PF = 1, int BKT = 16>
void launch_row3_cfg(const RowGemmArgs& a, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  for (int i = 0; i < a.nseg; ++i)
    if (!a.seg[i].B3 || a.seg[i].ldk < ((a.seg[i].K + 15) / 16) * 16 || a.seg[i].ldk % 8)
      throw std::runtime_error("split-bf16 row GEMM: segment without B planes");
  if (a.nseg > 1 && (a.seg[1].lda != a.seg[0].lda || a.seg[1].ldk != a.seg[0].ldk || a.seg[1].plane != a.seg[0].plane))
    throw std::runtime_error("split-bf16 row GEMM: segments with different strides");
  if ((int64_t)BM * a.seg[0].lda * 4 >= (int64_t(1) << 30) || (int64_t)(a.f16 ? 2 : 3) * a.seg[0].plane * 2 >= (int64_t(1) << 30))
    throw std::runtime_error("split-bf16 row GEMM: operand beyond the buffer-descriptor range");
  const long nblk = (long)((a.M + BM - 1) / BM) * ((a.Npad + BN - 1) / BN);
  RowGemmArgs b = a;
  b.low_seg = g_options.low_seg;
  if constexpr (BKT == 32) {
    for (int i = 0; i < a.nseg; ++i)
      if (a.seg[i].ldk % 32) throw std::runtime_error("split row GEMM (BK 32): B planes' ldk not a multiple of 32");
  }
  if (a.f16)
    hipLaunchKernelGGL((rowgemm3_kernel<WM, WN, TM, TN, EPI, OCC, PF, 2, BKT>), dim3((unsigned)nblk),
                       dim3(WM * WN * 64), 0, s, b);
  else if constexpr (BKT == 16)   // three bf16 planes at BK 32 exceed the LDS
    hipLaunchKernelGGL((rowgemm3_kernel<WM, WN, TM, TN, EPI, OCC, PF, 3, BKT>), dim3((unsigned)nblk),
                       dim3(WM * WN * 64), 0, s, a);
  else
    throw std::runtime_error("split row GEMM (BK 32): f16 planes only");
}

// A row GEMM whose k-loop is a few MFMA steps (the R-backward out of the softmax head: K = 2 x actions)
// is bound by its epilogue's HBM streams; the 256 x 256 split tile holds 256 VGPRs (one block per
// CU, nothing to overlap the epilogue with), the 128 x 256 f32 tile runs two blocks per CU.
bool small_k_row(const RowGemmArgs& a) {
  if (g_options.split_min_k <= 0) return false;
  for (int i = 0; i < a.nseg; ++i)
    if (a.seg[i].K >= g_options.split_min_k) return false;
  return true;
}

template <int EPI>
void launch_row_epi(const RowGemmArgs& a, hipStream_t s) {
  if constexpr (epi_is_head(EPI)) {
    // one 32-column tile per 32 actions in every lane half (epi_row)
    if (a.N > 32 * kMaxHeadTiles) throw std::runtime_error("softmax head supports at most 128 actions");
    if (a.N > 64) launch_row_cfg<4, 1, 2, 4, 16, EPI>(a, s);
    else if (a.N > 32) launch_row_cfg<4, 1, 2, 2, 16, EPI>(a, s);
    else launch_row_cfg<4, 1, 2, 1, 16, EPI>(a, s);
  } else if (rowgemm_uses_split(a.Npad, a.epi) && !small_k_row(a)) {
    // split_mfma 5 (default): 256 x 256 tile, BK 32 with one k-tile in flight on f16 planes whose ldk is a
    // multiple of 32 (C4 A/B, profiles/r4b: 2.260 -> 2.281 updates/s), else BK 16 with two in flight;
    // 6: 256 x 256 at BK 16 always (the round-3 default); any other non-zero value: 128 x 256
    bool bk32 = a.f16 != 0 && g_options.split_mfma == 5;
    for (int i = 0; i < a.nseg; ++i) bk32 = bk32 && a.seg[i].ldk % 32 == 0;
    if (bk32) launch_row3_cfg<4, 2, 2, 4, EPI, 2, 1, 32>(a, s);
    else if (g_options.split_mfma == 5 || g_options.split_mfma == 6) launch_row3_cfg<4, 2, 2, 4, EPI, 2, 2>(a, s);
    else launch_row3_cfg<2, 4, 2, 2, EPI>(a, s);
  } else {
    if (a.Npad <= 32) launch_row_cfg<4, 1, 2, 1, 16, EPI>(a, s);
    else if (a.Npad <= 64) launch_row_cfg<4, 1, 2, 2, 16, EPI>(a, s);
    else if (a.Npad <= 128) launch_row_cfg<2, 2, 2, 2, 16, EPI>(a, s);
    else launch_row_cfg<2, 4, 2, 2, 16, EPI>(a, s);   // 128 x 256, 8 waves
  }
}

template <int WM, int WN, int TM, int TN, int BKT = 16, int PF = 1>
void launch_wg_cfg(const WGradArgs& a, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  dim3 grid((a.Ma + BM - 1) / BM, (a.Nb + BN - 1) / BN, a.splits);
  hipLaunchKernelGGL((wgrad_kernel<WM, WN, TM, TN, BKT, PF>), grid, dim3(WM * WN * 64), 0, s, a);
}

template <int WM, int WN, int TM, int TN, int OCC, int PF>
void launch_wg3_cfg(const WGradArgs& a, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  if (a.rows_per_split % 16) throw std::runtime_error("split-bf16 wgrad: rows_per_split % 16");
  if (a.nseg > 1 && (a.seg[1].lda != a.seg[0].lda || a.seg[1].ldb != a.seg[0].ldb))
    throw std::runtime_error("split-bf16 wgrad: segments with different leading dimensions");
  if ((int64_t)a.rows_per_split * (a.seg[0].lda > a.seg[0].ldb ? a.seg[0].lda : a.seg[0].ldb) * 4 >= (int64_t(1) << 30))
    throw std::runtime_error("split-bf16 wgrad: a split's rows exceed the 1 GiB buffer-descriptor range");
  dim3 grid((a.Ma + BM - 1) / BM, (a.Nb + BN - 1) / BN, a.splits);
  WGradArgs b = a;
  b.low_seg = g_options.low_seg;
  if (a.f16)
    hipLaunchKernelGGL((wgrad3_kernel<WM, WN, TM, TN, OCC, PF, 2>), grid, dim3(WM * WN * 64), 0, s, b);
  else
    hipLaunchKernelGGL((wgrad3_kernel<WM, WN, TM, TN, OCC, PF, 3>), grid, dim3(WM * WN * 64), 0, s, a);
}

}  // namespace

bool rowgemm_uses_split(int Npad, RowEpi epi) {
  return g_options.split_mfma != 0 && Npad > 128 && !epi_is_head((int)epi);
}

void launch_split_b(const SplitArgs& a, const int* skip, hipStream_t s) {
  if (a.n <= 0) return;
  int maxb = 1;
  for (int i = 0; i < a.n; ++i) {
    const SplitJob& j = a.job[i];
    if (j.ldk % 8 || j.ldk < ((j.K + 15) / 16) * 16) throw std::runtime_error("split_b: bad ldk");
    const int b = (j.Npad * (j.ldk / 8) + 255) / 256;
    maxb = b > maxb ? b : maxb;
  }
  hipLaunchKernelGGL(split_b_kernel, dim3(maxb, a.n), dim3(256), 0, s, a, skip);
}

void launch_rowgemm(const RowGemmArgs& a, hipStream_t s) {
  if (a.M <= 0) return;
  // pre-split k-blocked A and B planes attached (plane.hip), where the register path would take the split
  if (a.seg[0].Ah && g_options.planes != 0 && a.f16 && rowgemm_uses_split(a.Npad, a.epi) && !small_k_row(a) &&
      a.Npad % 256 == 0) {
    launch_rowgemm_planes(a, s);
    return;
  }
  switch (a.epi) {
    case RowEpi::kTanh: launch_row_epi<(int)RowEpi::kTanh>(a, s); break;
    case RowEpi::kRHidden: launch_row_epi<(int)RowEpi::kRHidden>(a, s); break;
    case RowEpi::kRZ: launch_row_epi<(int)RowEpi::kRZ>(a, s); break;
    case RowEpi::kPrepBwd: launch_row_epi<(int)RowEpi::kPrepBwd>(a, s); break;
    case RowEpi::kPgBwd: launch_row_epi<(int)RowEpi::kPgBwd>(a, s); break;
    case RowEpi::kPrepBwdE: launch_row_epi<(int)RowEpi::kPrepBwdE>(a, s); break;
    case RowEpi::kRBwd: launch_row_epi<(int)RowEpi::kRBwd>(a, s); break;
    case RowEpi::kPrepHead: launch_row_epi<(int)RowEpi::kPrepHead>(a, s); break;
    case RowEpi::kLossHead: launch_row_epi<(int)RowEpi::kLossHead>(a, s); break;
    case RowEpi::kRHead: launch_row_epi<(int)RowEpi::kRHead>(a, s); break;
    case RowEpi::kRelu: launch_row_epi<(int)RowEpi::kRelu>(a, s); break;
    case RowEpi::kReluBwd: launch_row_epi<(int)RowEpi::kReluBwd>(a, s); break;
  }
}

void launch_wgrad(const WGradArgs& a, hipStream_t s) {
  if (a.splits <= 0) return;
  const int Mp = a.Ma, Np = a.Nb;
  // output tile by (fan_in, fan_out); every B column set of one split lives in one block row
  if (Np <= 32) {
    if (Mp <= 64) launch_wg_cfg<2, 1, 1, 1>(a, s);          // 64 x 32
    else if (Mp <= 128) launch_wg_cfg<4, 1, 1, 1>(a, s);    // 128 x 32
    else launch_wg_cfg<4, 1, 2, 1>(a, s);                   // 256 x 32
  } else if (Np <= 64) {
    if (Mp <= 64) launch_wg_cfg<2, 2, 1, 1>(a, s);          // 64 x 64
    else if (Mp <= 128) launch_wg_cfg<2, 1, 2, 2>(a, s);    // 128 x 64
    else launch_wg_cfg<4, 1, 2, 2>(a, s);                   // 256 x 64
  } else if (Np <= 128) {
    if (Mp <= 64) launch_wg_cfg<1, 2, 2, 2>(a, s);          // 64 x 128
    else launch_wg_cfg<2, 2, 2, 2>(a, s);                   // 128 x 128
  } else if (g_options.split_wg != 0) {
    // split-bf16 / f16 tiles
    if (Mp <= 128) launch_wg3_cfg<2, 4, 2, 2, 2, 1>(a, s);   // 128 x 256
    else launch_wg3_cfg<4, 2, 2, 4, 2, 1>(a, s);             // 256 x 256
  } else {
    if (Mp <= 128) launch_wg_cfg<2, 4, 2, 2>(a, s);          // 128 x 256
    else launch_wg_cfg<2, 4, 4, 2>(a, s);                    // 256 x 256
  }
}

}  // namespace trpo
