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
Options g_options = {env_int("TRPO_ROWCFG", 0), env_int("TRPO_WGCFG", 0), env_int("TRPO_FUSED_HEAD", 0),
                     env_int("TRPO_HEAD_BWD", 0), env_int("TRPO_NARROW_PF", 1), env_int("TRPO_SPLIT_MFMA", 5),
                     env_int("TRPO_SPLIT_WG", 1), env_int("TRPO_CHAIN", 1), env_int("TRPO_SPLIT_F16", 1),
                     env_int("TRPO_SPLIT_MIN_K", 0), env_int("TRPO_GRAPHS", 1), env_int("TRPO_TAIL", 1),
                     env_int("TRPO_FUSED", 2), env_int("TRPO_LOW_SEG", 14), env_int("TRPO_PLANES", 1),
                     env_int("TRPO_E16", 0), env_int("TRPO_RBWD0", 1),
                     env_int("TRPO_DUAL", 0)};

namespace {

constexpr int BK = 16;

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



template <int WM, int WN, int TM, int TN, int EPI, int OCC, int PF, int NP>
__global__ void __launch_bounds__(WM* WN * 64, OCC)   // OCC waves / SIMD
rowgemm3_kernel(const RowGemmArgs args) {
  // NP = 3: bf16 hi/mid/lo planes, 6 products ; NP = 2: scaled f16 hi/lo planes, 3 products
  constexpr int BK = 16;
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
  constexpr int BC = NP * BN * (BK / 8);    // 16-B chunks of B planes per k-tile
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
    const int p = f / (BN * 2), rem = f % (BN * 2);
    const int n = rem >> 1, kh = rem & 1;
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
        unsigned short* dst = As + swz16(r, kq >> 1) + 4 * (kq & 1);
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
        const int p = f / (BN * 2), rem = f % (BN * 2);
        const int n = rem >> 1, kh = rem & 1;
        *reinterpret_cast<u16x8*>(Bs + p * BPL + swz16(n, kh)) = st.rb[i];
      }
    }
  };
  auto compute_p = [&](int buf, auto one_c) {
    constexpr bool ONE = decltype(one_c)::value;
    const unsigned short* As = smem + buf * STG;
    const unsigned short* Bs = As + NP * APL;
    // fragments streamed per output column tile to keep few registers live
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

int wide_cfg() { return g_options.row_cfg; }


// ---------------------------------------------------------------------------
// LDS-DMA pipelined f16 split row GEMM (split_mfma = 10).  Same tile as config 5
// (256 x 256, 8 waves as 4 x 2, 2 x 4 accumulators per wave) and the same
// arithmetic as rowgemm3_kernel<.., NP = 2>, but the operands stream straight
// into LDS with global_load_lds_dwordx4 (no VGPR staging): A as raw f32 through
// a ring of KA = 6 k-tiles (5 in flight, 80 KB of HBM reads per CU), B as its
// pre-split f16 planes through a ring of KB = 3 (L2-resident).  Each wave splits
// its own A fragments (f32 -> scaled hi/lo f16) right before its MFMAs.
// Swizzles are applied on the source address (the DMA destination is
// lane-linear): A rows are 64 B, chunk c of row r sits at c ^ ((r >> 2) & 3);
// B rows are 32 B, chunk h of row n at h ^ ((n >> 3) & 1) -- both conflict-free
// for the 16-lane ds_read_b128 groups.  One barrier per k-tile: counted
// vmcnt(4) retires tile t's DMA, then the barrier publishes it and frees the
// stages of tile t - 1 for the next DMA.
// ---------------------------------------------------------------------------
template <int EPI>
__global__ void __launch_bounds__(512, 2)
rowgemm_g_kernel(const RowGemmArgs args) {
  constexpr int WM = 4, WN = 2, TM = 2, TN = 4, BK = 16;
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int KA = 6, KB = 3;
  constexpr int A_ST = BM * BK;              // floats per A stage (16 KB)
  constexpr int B_PL = BN * BK;              // u16 per B plane (8 KB)
  constexpr int B_ST = 2 * B_PL;             // u16 per B stage (16 KB)
  __shared__ __attribute__((aligned(16))) float smA[KA * A_ST];
  __shared__ __attribute__((aligned(16))) unsigned short smB[KB * B_ST];
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
  const int eA0 = amax_exp(args.seg[0].amaxA);
  const int eP0 = eA0 + amax_exp(args.seg[0].amaxB);
  int eA1 = 0, eP1 = 0;
  if (args.nseg > 1) {
    eA1 = amax_exp(args.seg[1].amaxA);
    eP1 = eA1 + amax_exp(args.seg[1].amaxB);
  }
  const float sA0 = __builtin_ldexpf(1.0f, eA0), sA1 = __builtin_ldexpf(1.0f, eA1);
  // every ordinary global load is consumed before the first DMA: hipcc would otherwise drain
  // the DMA ring (vmcnt(0)) at the first later use
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
  if (ntiles <= 0) {
    row_epilogue<WM, WN, TM, TN, EPI>(args, acc, m0, n0, wm, wn, lr, lh);
    return;
  }

  // DMA of k-tile t (clamped into range: tail issues are dummies that keep the counts uniform)
  auto issue = [&](int t, bool with_b) {
    t = t < ntiles ? t : ntiles - 1;
    const bool s1 = t >= nt0;
    const GemmSeg& sg = s1 ? args.seg[1] : args.seg[0];
    const int k0 = (s1 ? t - nt0 : t) * BK;
    // A: 16 rows x 64 B per wave-instruction, 2 per wave
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int blk = wave * 2 + i;
      const int row = blk * 16 + (lane >> 2);
      const int c = (lane & 3) ^ ((row >> 2) & 3);
      int gr = m0 + row;
      gr = gr < M ? gr : M - 1;
      int k = k0 + 4 * c;
      k = k < sg.K - 4 ? k : sg.K - 4;
      const float* src = sg.A + (size_t)gr * sg.lda + k;
      glds16(src, smA + (t % KA) * A_ST + blk * 256);
    }
    if (with_b) {
      // B: 32 columns x 32 B per wave-instruction, 2 per wave (planes 0/1 x 8 column blocks)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int blk = wave * 2 + i;
        const int plane = blk >> 3, sub = blk & 7;
        const int n = sub * 32 + (lane >> 1);
        const int h = (lane & 1) ^ ((n >> 3) & 1);
        int gn = n0 + n;
        gn = gn < args.Npad ? gn : args.Npad - 1;
        const uint16_t* src = sg.B3 + (size_t)plane * sg.plane + (size_t)gn * sg.ldk + k0 + 8 * h;
        glds16(src, smB + (t % KB) * B_ST + plane * B_PL + sub * 512);
      }
    }
  };
  auto compute = [&](int t) {
    const float* As = smA + (t % KA) * A_ST;
    const unsigned short* Bs = smB + (t % KB) * B_ST;
    const float sa = t >= nt0 ? sA1 : sA0;
    f16x8 ah[TM], al[TM];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int r = wm * TM * 32 + tm * 32 + lr;
      const int sw = (r >> 2) & 3;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(As + r * 16 + 4 * ((2 * lh) ^ sw));
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(As + r * 16 + 4 * ((2 * lh + 1) ^ sw));
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = (j < 4 ? x0[j] : x1[j - 4]) * sa;
        const _Float16 hh = (_Float16)x;
        ah[tm][j] = hh;
        al[tm][j] = (_Float16)(x - (float)hh);
      }
    }
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int nn = wn * TN * 32 + tn * 32 + lr;
      const int off = nn * 16 + 8 * (lh ^ ((nn >> 3) & 1));
      const f16x8 bh = *reinterpret_cast<const f16x8*>(Bs + off);
      const f16x8 bl = *reinterpret_cast<const f16x8*>(Bs + B_PL + off);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        f32x16 c = acc[tm][tn];
        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[tm], bh, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[tm], bl, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[tm], bh, c, 0, 0, 0);
        acc[tm][tn] = c;
      }
    }
  };

  // prologue: iterations -(KA-1) .. -1 of the issue schedule (A runs KA-1 tiles ahead, B KB-1)
#pragma unroll
  for (int t = -(KA - 1); t < 0; ++t) {
    issue(t + KA - 1, false);
    if (t + KB - 1 >= 0) {
      // B of tile t + KB - 1 (A of that tile went out earlier)
      const int tb = t + KB - 1;
      const int tbc = tb < ntiles ? tb : ntiles - 1;
      const bool s1 = tbc >= nt0;
      const GemmSeg& sg = s1 ? args.seg[1] : args.seg[0];
      const int k0 = (s1 ? tbc - nt0 : tbc) * BK;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int blk = wave * 2 + i;
        const int plane = blk >> 3, sub = blk & 7;
        const int n = sub * 32 + (lane >> 1);
        const int h = (lane & 1) ^ ((n >> 3) & 1);
        int gn = n0 + n;
        gn = gn < args.Npad ? gn : args.Npad - 1;
        const uint16_t* src = sg.B3 + (size_t)plane * sg.plane + (size_t)gn * sg.ldk + k0 + 8 * h;
        glds16(src, smB + (tb % KB) * B_ST + plane * B_PL + sub * 512);
      }
    }
  }
  for (int t = 0; t < ntiles; ++t) {
    // tile t's B went out at iteration t - 2 and only iteration t - 1's 4 DMAs follow it
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // the stages of tile t - 1 are free now: refill them with A(t + KA - 1) and B(t + KB - 1)
    {
      const int ta = t + KA - 1;
      const int tac = ta < ntiles ? ta : ntiles - 1;
      const bool s1 = tac >= nt0;
      const GemmSeg& sg = s1 ? args.seg[1] : args.seg[0];
      const int k0 = (s1 ? tac - nt0 : tac) * BK;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int blk = wave * 2 + i;
        const int row = blk * 16 + (lane >> 2);
        const int c = (lane & 3) ^ ((row >> 2) & 3);
        int gr = m0 + row;
        gr = gr < M ? gr : M - 1;
        int k = k0 + 4 * c;
        k = k < sg.K - 4 ? k : sg.K - 4;
        glds16(sg.A + (size_t)gr * sg.lda + k, smA + (ta % KA) * A_ST + blk * 256);
      }
      const int tb = t + KB - 1;
      const int tbc = tb < ntiles ? tb : ntiles - 1;
      const bool sb1 = tbc >= nt0;
      const GemmSeg& sgb = sb1 ? args.seg[1] : args.seg[0];
      const int kb0 = (sb1 ? tbc - nt0 : tbc) * BK;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int blk = wave * 2 + i;
        const int plane = blk >> 3, sub = blk & 7;
        const int n = sub * 32 + (lane >> 1);
        const int h = (lane & 1) ^ ((n >> 3) & 1);
        int gn = n0 + n;
        gn = gn < args.Npad ? gn : args.Npad - 1;
        glds16(sgb.B3 + (size_t)plane * sgb.plane + (size_t)gn * sgb.ldk + kb0 + 8 * h, smB + (tb % KB) * B_ST + plane * B_PL + sub * 512);
      }
    }
    if (t == nt0 && nt1 > 0) scale_acc<TM, TN>(acc, eP1 - eP0);
    compute(t);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tail's dummy DMAs land before the block retires
  scale_acc<TM, TN>(acc, -(nt1 > 0 ? eP1 : eP0));
  row_epilogue<WM, WN, TM, TN, EPI>(args, acc, m0, n0, wm, wn, lr, lh);
}

// BK = 32 form of rowgemm_g_kernel (split_mfma = 11): two 32-deep k-steps per barrier, A rows of
// 128 B (whole cache lines) and B rows of 64 B per stage, double-buffered (A 2 x 32 KB, B 2 x 32 KB).
// Swizzles: A chunk c of row r at c ^ ((r >> 1) & 7); B chunk c of column n at c ^ ((n >> 2) & 3).
// Needs every B plane's ldk to be a multiple of 32 (zero-filled past K).
template <int EPI>
__global__ void __launch_bounds__(512, 2)
rowgemm_g32_kernel(const RowGemmArgs args) {
  constexpr int WM = 4, WN = 2, TM = 2, TN = 4, BK = 32;
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int A_ST = BM * BK;              // floats per A stage (32 KB)
  constexpr int B_PL = BN * BK;              // u16 per B plane (16 KB)
  constexpr int B_ST = 2 * B_PL;             // u16 per B stage (32 KB)
  __shared__ __attribute__((aligned(16))) float smA[2 * A_ST];
  __shared__ __attribute__((aligned(16))) unsigned short smB[2 * B_ST];
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
  const int eA0 = amax_exp(args.seg[0].amaxA);
  const int eP0 = eA0 + amax_exp(args.seg[0].amaxB);
  int eA1 = 0, eP1 = 0;
  if (args.nseg > 1) {
    eA1 = amax_exp(args.seg[1].amaxA);
    eP1 = eA1 + amax_exp(args.seg[1].amaxB);
  }
  const float sA0 = __builtin_ldexpf(1.0f, eA0), sA1 = __builtin_ldexpf(1.0f, eA1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
  if (ntiles <= 0) {
    row_epilogue<WM, WN, TM, TN, EPI>(args, acc, m0, n0, wm, wn, lr, lh);
    return;
  }

  auto issue = [&](int t) {
    const bool s1 = t >= nt0;
    const GemmSeg& sg = s1 ? args.seg[1] : args.seg[0];
    const int k0 = (s1 ? t - nt0 : t) * BK;
    float* As = smA + (t & 1) * A_ST;
    unsigned short* Bs = smB + (t & 1) * B_ST;
    // A: 8 rows x 128 B per wave-instruction, 4 per wave
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int blk = wave * 4 + i;
      const int row = blk * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      int gr = m0 + row;
      gr = gr < M ? gr : M - 1;
      int k = k0 + 4 * c;
      k = k < sg.K - 4 ? k : sg.K - 4;
      glds16(sg.A + (size_t)gr * sg.lda + k, As + blk * 256);
    }
    // B: 16 columns x 64 B per wave-instruction, 4 per wave (2 planes x 16 column blocks)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int blk = wave * 4 + i;
      const int plane = blk >> 4, sub = blk & 15;
      const int n = sub * 16 + (lane >> 2);
      const int c = (lane & 3) ^ ((n >> 2) & 3);
      int gn = n0 + n;
      gn = gn < args.Npad ? gn : args.Npad - 1;
      glds16(sg.B3 + (size_t)plane * sg.plane + (size_t)gn * sg.ldk + k0 + 8 * c, Bs + plane * B_PL + sub * 512);
    }
  };
  auto compute = [&](int t) {
    const float* As = smA + (t & 1) * A_ST;
    const unsigned short* Bs = smB + (t & 1) * B_ST;
    const float sa = t >= nt0 ? sA1 : sA0;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f16x8 ah[TM], al[TM];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int r = wm * TM * 32 + tm * 32 + lr;
        const int sw = (r >> 1) & 7;
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(As + r * 32 + 4 * ((4 * ks + 2 * lh) ^ sw));
        const f32x4 x1 = *reinterpret_cast<const f32x4*>(As + r * 32 + 4 * ((4 * ks + 2 * lh + 1) ^ sw));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = (j < 4 ? x0[j] : x1[j - 4]) * sa;
          const _Float16 hh = (_Float16)x;
          ah[tm][j] = hh;
          al[tm][j] = (_Float16)(x - (float)hh);
        }
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int nn = wn * TN * 32 + tn * 32 + lr;
        const int off = nn * 32 + 8 * ((2 * ks + lh) ^ ((nn >> 2) & 3));
        const f16x8 bh = *reinterpret_cast<const f16x8*>(Bs + off);
        const f16x8 bl = *reinterpret_cast<const f16x8*>(Bs + B_PL + off);
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          f32x16 c = acc[tm][tn];
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[tm], bh, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[tm], bl, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[tm], bh, c, 0, 0, 0);
          acc[tm][tn] = c;
        }
      }
    }
  };

  issue(0);
  for (int t = 0; t < ntiles; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                 // tile t landed (this wave's part)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // ... everyone's; tile t-1 is consumed
    if (t + 1 < ntiles) issue(t + 1);                                  // into the buffer of tile t - 1
    if (t == nt0 && nt1 > 0) scale_acc<TM, TN>(acc, eP1 - eP0);
    compute(t);
  }
  scale_acc<TM, TN>(acc, -(nt1 > 0 ? eP1 : eP0));
  row_epilogue<WM, WN, TM, TN, EPI>(args, acc, m0, n0, wm, wn, lr, lh);
}

template <int EPI>
void launch_row_g32(const RowGemmArgs& a, hipStream_t s) {
  for (int i = 0; i < a.nseg; ++i)
    if (!a.seg[i].B3 || a.seg[i].ldk % 32 || a.seg[i].ldk < ((a.seg[i].K + 31) / 32) * 32 || a.seg[i].K % 4 ||
        a.seg[i].K < 4 || a.seg[i].lda % 4)
      throw std::runtime_error("LDS-DMA row GEMM (BK 32): bad segment");
  const long nblk = (long)((a.M + 255) / 256) * ((a.Npad + 255) / 256);
  hipLaunchKernelGGL((rowgemm_g32_kernel<EPI>), dim3((unsigned)nblk), dim3(512), 0, s, a);
}

template <int EPI>
void launch_row_g(const RowGemmArgs& a, hipStream_t s) {
  for (int i = 0; i < a.nseg; ++i)
    if (!a.seg[i].B3 || a.seg[i].ldk < ((a.seg[i].K + 15) / 16) * 16 || a.seg[i].ldk % 8 || a.seg[i].K % 4 ||
        a.seg[i].K < 4 || a.seg[i].lda % 4)
      throw std::runtime_error("LDS-DMA row GEMM: bad segment");
  const long nblk = (long)((a.M + 255) / 256) * ((a.Npad + 255) / 256);
  hipLaunchKernelGGL((rowgemm_g_kernel<EPI>), dim3((unsigned)nblk), dim3(512), 0, s, a);
}

template <int WM, int WN, int TM, int TN, int EPI, int OCC = 2, int PF = 1>
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
  if (a.f16)
    hipLaunchKernelGGL((rowgemm3_kernel<WM, WN, TM, TN, EPI, OCC, PF, 2>), dim3((unsigned)nblk), dim3(WM * WN * 64), 0,
                       s, b);
  else
    hipLaunchKernelGGL((rowgemm3_kernel<WM, WN, TM, TN, EPI, OCC, PF, 3>), dim3((unsigned)nblk), dim3(WM * WN * 64), 0,
                       s, a);
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
    else if (g_options.narrow_pf == 2) launch_row_cfg<4, 1, 2, 1, 16, EPI, 2>(a, s);
    else launch_row_cfg<4, 1, 2, 1, 16, EPI>(a, s);
  } else if (rowgemm_uses_split(a.Npad, a.epi) && !small_k_row(a)) {
    switch (g_options.split_mfma) {
      case 2: launch_row3_cfg<4, 2, 2, 4, EPI>(a, s); break;   // 256 x 256
      case 3: launch_row3_cfg<2, 2, 2, 2, EPI>(a, s); break;   // 128 x 128
      case 4: launch_row3_cfg<4, 2, 2, 2, EPI>(a, s); break;   // 256 x 128
      case 5: launch_row3_cfg<4, 2, 2, 4, EPI, 2, 2>(a, s); break;   // 256 x 256, 2 k-tiles in flight
      case 6: launch_row3_cfg<2, 4, 2, 2, EPI, 2, 2>(a, s); break;   // 128 x 256, 2 k-tiles in flight
      case 7: launch_row3_cfg<4, 4, 2, 2, EPI, 4>(a, s); break;      // 256 x 256, 16 waves
      case 8: launch_row3_cfg<2, 4, 2, 2, EPI, 4>(a, s); break;      // 128 x 256, 2 blocks / CU
      case 9: launch_row3_cfg<2, 4, 2, 2, EPI, 4, 2>(a, s); break;   // 128 x 256, 2 blocks / CU, 2 in flight
      case 12: launch_row3_cfg<2, 2, 2, 4, EPI, 2, 2>(a, s); break;  // 128 x 256, 4 waves, 2 blocks / CU
      case 13: launch_row3_cfg<2, 2, 2, 4, EPI, 2, 1>(a, s); break;  // the same, one k-tile in flight
      case 11: {                                                      // 256 x 256, LDS-DMA, BK 32 (f16 only)
        bool ok = a.f16 != 0;
        for (int i = 0; i < a.nseg; ++i) ok = ok && a.seg[i].ldk % 32 == 0;
        if (ok) {
          launch_row_g32<EPI>(a, s);
          break;
        }
        launch_row3_cfg<4, 2, 2, 4, EPI, 2, 2>(a, s);
        break;
      }
      case 10:                                                        // 256 x 256, LDS-DMA ring (f16 only)
        if (a.f16) {
          launch_row_g<EPI>(a, s);
          break;
        }
        launch_row3_cfg<4, 2, 2, 4, EPI, 2, 2>(a, s);
        break;
      default: launch_row3_cfg<2, 4, 2, 2, EPI>(a, s); break;  // 128 x 256
    }
  } else {
    if (a.Npad <= 32) launch_row_cfg<4, 1, 2, 1, 16, EPI>(a, s);
    else if (a.Npad <= 64) launch_row_cfg<4, 1, 2, 2, 16, EPI>(a, s);
    else if (a.Npad <= 128) launch_row_cfg<2, 2, 2, 2, 16, EPI>(a, s);
    else {
      switch (wide_cfg()) {
        case 1: launch_row_cfg<2, 2, 2, 2, 16, EPI>(a, s); break;   // 128 x 128, 4 waves
        case 2: launch_row_cfg<4, 2, 2, 2, 16, EPI>(a, s); break;   // 256 x 128, 8 waves
        case 3: launch_row_cfg<2, 4, 2, 2, 32, EPI>(a, s); break;   // 128 x 256, BK 32
        case 4: launch_row_cfg<1, 4, 2, 2, 16, EPI>(a, s); break;   // 64 x 256, 4 waves
        case 5: launch_row_cfg<2, 4, 4, 2, 16, EPI>(a, s); break;   // 256 x 256, 8 waves, 128 acc/wave
        default: launch_row_cfg<2, 4, 2, 2, 16, EPI>(a, s); break;  // 128 x 256, 8 waves
      }
    }
  }
}

template <int WM, int WN, int TM, int TN, int BKT = 16, int PF = 1>
void launch_wg_cfg(const WGradArgs& a, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  dim3 grid((a.Ma + BM - 1) / BM, (a.Nb + BN - 1) / BN, a.splits);
  hipLaunchKernelGGL((wgrad_kernel<WM, WN, TM, TN, BKT, PF>), grid, dim3(WM * WN * 64), 0, s, a);
}

int wg_cfg() { return g_options.wg_cfg; }

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
    case RowEpi::kPrepBwd16: launch_row_epi<(int)RowEpi::kPrepBwd16>(a, s); break;
    case RowEpi::kPrepBwdE16: launch_row_epi<(int)RowEpi::kPrepBwdE16>(a, s); break;
    case RowEpi::kRBwd16: launch_row_epi<(int)RowEpi::kRBwd16>(a, s); break;
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
    // split-bf16 tiles
    if (Mp <= 128) {
      if (g_options.split_wg == 2) launch_wg3_cfg<2, 4, 2, 2, 2, 2>(a, s);   // 128 x 256, 2 stages
      else launch_wg3_cfg<2, 4, 2, 2, 2, 1>(a, s);                           // 128 x 256
    } else {
      switch (g_options.split_wg) {
        case 2: launch_wg3_cfg<4, 2, 2, 4, 2, 2>(a, s); break;   // 256 x 256, 2 stages
        case 4: launch_wg3_cfg<2, 2, 2, 4, 2, 2>(a, s); break;   // 128 x 256, 4 waves, 2 blocks / CU
        case 5: launch_wg3_cfg<2, 2, 4, 2, 2, 2>(a, s); break;   // 256 x 128, 4 waves, 2 blocks / CU
        case 3: launch_wg3_cfg<2, 4, 2, 2, 2, 1>(a, s); break;   // 128 x 256
        default: launch_wg3_cfg<4, 2, 2, 4, 2, 1>(a, s); break;  // 256 x 256
      }
    }
  } else {
    if (Mp <= 128) {
      if (g_options.narrow_pf == 2) launch_wg_cfg<2, 4, 2, 2, 16, 2>(a, s);   // 128 x 256, 2 stages
      else launch_wg_cfg<2, 4, 2, 2>(a, s);                                 // 128 x 256
    }
    else if (wg_cfg() == 1) launch_wg_cfg<2, 4, 4, 2, 32>(a, s);   // 256 x 256, BK 32
    else launch_wg_cfg<2, 4, 4, 2>(a, s);                   // 256 x 256
  }
}

}  // namespace trpo

// =============================================================================
// Fused FVP head kernel (see kernels.h, HeadArgs)
// =============================================================================
namespace trpo {
namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int HB_M = 64;            // rows per tile
constexpr int HB_AMAX = 256;        // max hidden width held in LDS
constexpr int HB_LDS_ROW = HB_AMAX + 4;
constexpr int HB_DCAT_LD = 65;      // [RD_L | D_L] row stride (odd: conflict-free column reads)
constexpr int HB_THREADS = 512;

__device__ __forceinline__ double hsum16d(double v) {
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) v += __shfl_xor(v, off, 16);
  return v;
}

__global__ void __launch_bounds__(HB_THREADS)
fvp_head_kernel(const HeadArgs args) {
  __shared__ __attribute__((aligned(16))) float sRH[HB_M * HB_LDS_ROW];
  __shared__ __attribute__((aligned(16))) float sH[HB_M * HB_LDS_ROW];
  __shared__ float sD[HB_M * HB_DCAT_LD];        // cols [0,bpad) = RD_L, [bpad,2bpad) = D_L
  __shared__ float sRed[4 * 2 * 4 * 64];         // K-half partials of the head GEMM
  if (args.skip && *args.skip) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int a = args.a, b = args.b, apad = args.apad, bpad = args.bpad;
  const int split = blockIdx.x;
  const int r0 = split * args.rows_per_split;
  const int r1 = min(args.rows, r0 + args.rows_per_split);

  // persistent weight-gradient accumulator: wave w owns hidden rows [32w, 32w+32) x cols [0,32)
  f32x16 gacc = f32x16{};
  float bsum = 0.0f;

  for (int t0 = r0; t0 < r1; t0 += HB_M) {
    const int nrow = min(HB_M, r1 - t0);
    // ---- P0: stage RH, H (64 x apad) and D_L into LDS ----
    {
      const int q4 = apad / 4;                  // float4 per row
      const int tot = HB_M * q4;
      for (int f = tid; f < 2 * tot; f += HB_THREADS) {
        const int which = f >= tot;
        const int g = which ? f - tot : f;
        const int r = g / q4, c4 = g % q4;
        f32x4_t v = f32x4_t{};
        if (r < nrow)
          v = *reinterpret_cast<const f32x4_t*>((which ? args.H : args.RH) + (size_t)(t0 + r) * apad + 4 * c4);
        *reinterpret_cast<f32x4_t*>((which ? sH : sRH) + r * HB_LDS_ROW + 4 * c4) = v;
      }
      for (int f = tid; f < HB_M * 32; f += HB_THREADS) {
        const int r = f >> 5, c = f & 31;
        float dl = 0.0f;
        if (r < nrow && c < bpad) dl = args.DL[(size_t)(t0 + r) * bpad + c];
        if (c < bpad) sD[r * HB_DCAT_LD + bpad + c] = dl;
      }
    }
    __syncthreads();

    // ---- P1: head GEMM RZ[64 x 32] (16x16x4 MFMA; wave = 16-row tile x K-half) ----
    const int rt = wave & 3, kh = wave >> 2;
    const int l15 = lane & 15, grp = lane >> 4;
    f32x4_t hacc[2] = {f32x4_t{}, f32x4_t{}};
    {
      const float* sA = kh ? sH : sRH;
      const float* W = args.WF + (size_t)kh * apad * bpad;
      for (int kq = 0; kq < apad / 16; ++kq) {
        const f32x4_t a4 = *reinterpret_cast<const f32x4_t*>(sA + (rt * 16 + l15) * HB_LDS_ROW + 16 * kq + 4 * grp);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int k = 16 * kq + 4 * grp + s;
#pragma unroll
          for (int tn = 0; tn < 2; ++tn) {
            const int j = 16 * tn + l15;
            const float bv = (j < bpad) ? W[(size_t)k * bpad + j] : 0.0f;
            hacc[tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[s], bv, hacc[tn], 0, 0, 0);
          }
        }
      }
    }
    if (kh == 1) {
#pragma unroll
      for (int tn = 0; tn < 2; ++tn)
#pragma unroll
        for (int r = 0; r < 4; ++r) sRed[((rt * 2 + tn) * 4 + r) * 64 + lane] = hacc[tn][r];
    }
    __syncthreads();
    if (kh == 0) {
      // ---- P2: R-softmax head epilogue -> RD_L into sD[:, 0:bpad) ----
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rt * 16 + grp * 4 + r;
        const bool rv = row < nrow;
        double rz[2], pd[2];
#pragma unroll
        for (int tn = 0; tn < 2; ++tn) {
          const int j = 16 * tn + l15;
          const bool real = j < b;
          const float z = hacc[tn][r] + sRed[((rt * 2 + tn) * 4 + r) * 64 + lane];
          rz[tn] = real ? (double)(z + args.c[j]) : 0.0;
          pd[tn] = (real && rv) ? (double)args.P[(size_t)(t0 + row) * bpad + j] : 0.0;
        }
        const double prz = hsum16d(pd[0] * rz[0] + pd[1] * rz[1]);
        double Rp[2], Aa[2], B[2];
#pragma unroll
        for (int tn = 0; tn < 2; ++tn) {
          const bool real = 16 * tn + l15 < b;
          Rp[tn] = pd[tn] * (rz[tn] - prz);
          const double den = pd[tn] + (double)kEps;
          Aa[tn] = real ? pd[tn] / den : 0.0;
          B[tn] = real ? (double)kEps / den : 0.0;
        }
        const double spB = hsum16d(pd[0] * B[0] + pd[1] * B[1]);
        const double sRAB = hsum16d(Rp[0] * Aa[0] * B[0] + Rp[1] * Aa[1] * B[1]);
#pragma unroll
        for (int tn = 0; tn < 2; ++tn) {
          const int j = 16 * tn + l15;
          const double rd = args.invN * (Rp[tn] * (B[tn] - spB) + Rp[tn] * Aa[tn] * Aa[tn] + pd[tn] * sRAB);
          if (j < bpad) sD[row * HB_DCAT_LD + j] = (j < b && rv) ? (float)rd : 0.0f;
        }
      }
    }
    __syncthreads();

    // ---- P3: R-backward RDH[64 x apad] = [RD_L | D_L] [W^T ; V^T] (32x32x2) + epilogue ----
    {
      const int lr = lane & 31, lh = lane >> 5;
      const int rt2 = wave & 1, ct = wave >> 1;   // 2 row tiles x 4 col groups of 64
      const int colbase = 64 * ct;
      if (colbase < apad) {
        f32x16 racc[2] = {f32x16{}, f32x16{}};
        const int K = 2 * bpad;
        for (int k0 = 0; k0 < K; k0 += 2) {
          const int k = k0 + lh;
          const float av = sD[(rt2 * 32 + lr) * HB_DCAT_LD + k];
#pragma unroll
          for (int tn = 0; tn < 2; ++tn) {
            const int col = colbase + 32 * tn + lr;
            const float bv = col < apad ? args.WB[(size_t)k * apad + col] : 0.0f;
            racc[tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, racc[tn], 0, 0, 0);
          }
        }
#pragma unroll
        for (int tn = 0; tn < 2; ++tn) {
          const int col = colbase + 32 * tn + lr;
          if (col >= apad) continue;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rt2 * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (row >= nrow) continue;
            const float h = sH[row * HB_LDS_ROW + col];
            const float rh = sRH[row * HB_LDS_ROW + col];
            const size_t gi = (size_t)(t0 + row) * apad + col;
            const float e = args.E[gi];
            args.RDout[gi] = (col < a) ? fmaf(e, rh, racc[tn][r] * one_minus_sq(h)) : 0.0f;
          }
        }
      }
    }

    // ---- P4: weight gradient of the head: G[apad x 32] += RH^T D_L + H^T RD_L ----
    {
      const int lr = lane & 31, lh = lane >> 5;
      const int i = 32 * wave + lr;          // hidden row of this lane's A fragment
      if (32 * wave < apad) {
        for (int rr = 0; rr < HB_M; rr += 2) {
          const int row = rr + lh;
          const float aRH = (i < apad) ? sRH[row * HB_LDS_ROW + i] : 0.0f;
          const float aH = (i < apad) ? sH[row * HB_LDS_ROW + i] : 0.0f;
          const float bD = (lr < bpad) ? sD[row * HB_DCAT_LD + bpad + lr] : 0.0f;
          const float bR = (lr < bpad) ? sD[row * HB_DCAT_LD + lr] : 0.0f;
          gacc = __builtin_amdgcn_mfma_f32_32x32x2f32(aRH, bD, gacc, 0, 0, 0);
          gacc = __builtin_amdgcn_mfma_f32_32x32x2f32(aH, bR, gacc, 0, 0, 0);
        }
      }
      if (tid < b) {
        float cs = 0.0f;
        for (int r = 0; r < HB_M; ++r) cs += sD[r * HB_DCAT_LD + tid];
        bsum += cs;
      }
    }
    __syncthreads();
  }

  // ---- write this split's slab: W part (a x b) and bias ----
  float* out = args.slab + (size_t)split * args.slab_stride;
  {
    const int lr = lane & 31, lh = lane >> 5;
    const int j = lr;
    if (32 * wave < apad && j < b) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (i < a) out[args.off_w + (int64_t)i * b + j] = gacc[r];
      }
    }
  }
  if (tid < b) out[args.off_b + tid] = bsum;
}

}  // namespace

void launch_fvp_head(const HeadArgs& a, hipStream_t s) {
  if (a.apad > HB_AMAX || a.bpad > 32) throw std::runtime_error("fvp_head: layer too wide for the fused head");
  if (a.splits <= 0) return;
  hipLaunchKernelGGL(fvp_head_kernel, dim3(a.splits), dim3(HB_THREADS), 0, s, a);
}

}  // namespace trpo

// =============================================================================
// Fused last-layer R-backward + weight gradient (see kernels.h, HeadBwdArgs)
// Block = 4 waves; wave w owns hidden columns [64w, 64w+64) (two 32-col MFMA
// tiles); a tile is 32 rows.  Per tile:
//   1. [RD_L | D_L] (32 x 2bpad) -> LDS
//   2. RDH = [RD_L|D_L] . [W^T;V^T]   (32x32x2 MFMA, K = 2bpad; the W^T/V^T
//      fragments of a wave never change -> held in registers for the launch)
//   3. H, RH, E buffer-loaded in accumulator layout (lane = hidden col,
//      register = row); RD = RDH (1-H^2) + E RH stored
//   4. weight gradient: the same H / RH registers are the A operands of
//      G[hidden][j] += sum_rows RH D_L + H RD_L (register r of lane half h is
//      row (r&3)+8(r>>2)+4h, used as the MFMA k of step r)
// =============================================================================
namespace trpo {
namespace {

constexpr int HBW_ROWS = 32;
constexpr int HBW_WAVES = 4;
constexpr int HBW_DLD = 65;      // LDS row stride of [RD_L | D_L] (odd: conflict-free column reads)

template <int KPAIRS>   // KPAIRS = bpad (2*bpad K values, 2 per MFMA)
__global__ void __launch_bounds__(HBW_WAVES * 64, 2)
head_bwd_kernel(const HeadBwdArgs args) {
  __shared__ float sD[HBW_ROWS * HBW_DLD];
  if (args.skip && *args.skip) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int a = args.a, b = args.b, apad = args.apad, bpad = args.bpad;
  const int split = blockIdx.x;
  const int r0 = split * args.rows_per_split;
  const int r1 = min(args.rows, r0 + args.rows_per_split);
  const int cbase = 64 * wave;                 // this wave's first hidden column
  const bool active = cbase < apad;

  // B operand of the R-backward: WB[k][cbase + 32 tn + lr] for k = 2s + lh
  float wb[KPAIRS][2];
#pragma unroll
  for (int s = 0; s < KPAIRS; ++s)
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) {
      const int col = cbase + 32 * tn + lr;
      const int k = 2 * s + lh;
      wb[s][tn] = (active && col < apad && k < 2 * bpad) ? args.WB[(size_t)k * apad + col] : 0.0f;
    }

  f32x16 gacc[2] = {f32x16{}, f32x16{}};   // weight gradient, hidden rows x 32 cols
  float bsum = 0.0f;

  for (int t0 = r0; t0 < r1; t0 += HBW_ROWS) {
    const int nrow = min(HBW_ROWS, r1 - t0);
    // 1. [RD_L | D_L] tile
    for (int f = tid; f < HBW_ROWS * 64; f += HBW_WAVES * 64) {
      const int r = f >> 6, c = f & 63;
      float v = 0.0f;
      if (r < nrow && c < 2 * bpad) {
        const bool second = c >= bpad;
        const int cc = second ? c - bpad : c;
        v = (second ? args.DL : args.RDL)[(size_t)(t0 + r) * bpad + cc];
      }
      if (c < 2 * bpad) sD[r * HBW_DLD + c] = v;
    }
    __syncthreads();
    if (tid < b) {
      float cs = 0.0f;
      for (int r = 0; r < HBW_ROWS; ++r) cs += sD[r * HBW_DLD + tid];
      bsum += cs;
    }
    if (active) {
      // 2. R-backward GEMM
      f32x16 racc[2] = {f32x16{}, f32x16{}};
#pragma unroll
      for (int s = 0; s < KPAIRS; ++s) {
        const float av = sD[lr * HBW_DLD + 2 * s + lh];
        racc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, wb[s][0], racc[0], 0, 0, 0);
        racc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, wb[s][1], racc[1], 0, 0, 0);
      }
      // 3. epilogue through per-tile buffer descriptors (rows past the tile read 0 / drop)
      const int tile_bytes = nrow * apad * 4;
      auto mk = [&](const float* p) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)(p + (size_t)t0 * apad), 0, tile_bytes, 0x00020000);
      };
      const __amdgpu_buffer_rsrc_t rH = mk(args.H), rRH = mk(args.RH), rE = mk(args.E), rO = mk(args.RDout);
#pragma unroll
      for (int tn = 0; tn < 2; ++tn) {
        const int col = cbase + 32 * tn + lr;
        const bool colv = col < apad;
        const int vo = ((4 * lh) * apad + (colv ? col : 0)) * 4;
        float h[16], rh[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int so = ((r & 3) + 8 * (r >> 2)) * apad * 4;
          h[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rH, vo, so, 0));
          rh[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rRH, vo, so, 0));
          const float e = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rE, vo, so, 0));
          const float rd = fmaf(e, rh[r], racc[tn][r] * one_minus_sq(h[r]));
          if (colv) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, rd), rO, vo, so, 0);
        }
        // 4. weight gradient: rows are the MFMA k (register r <-> row (r&3)+8(r>>2)+4h)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
          const float dl = lr < bpad ? sD[row * HBW_DLD + bpad + lr] : 0.0f;
          const float rdl = lr < bpad ? sD[row * HBW_DLD + lr] : 0.0f;
          gacc[tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(rh[r], dl, gacc[tn], 0, 0, 0);
          gacc[tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(h[r], rdl, gacc[tn], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }

  float* out = args.slab + (size_t)split * args.slab_stride;
  if (active && lr < b) {
#pragma unroll
    for (int tn = 0; tn < 2; ++tn)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = cbase + 32 * tn + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (i < a) out[args.off_w + (int64_t)i * b + lr] = gacc[tn][r];
      }
  }
  if (tid < b) out[args.off_b + tid] = bsum;
}

}  // namespace

void launch_head_bwd(const HeadBwdArgs& a, hipStream_t s) {
  if (a.apad > 64 * HBW_WAVES || a.bpad > 32 || a.bpad % 4) throw std::runtime_error("head_bwd: unsupported layer shape");
  if (a.splits <= 0) return;
  const dim3 grid(a.splits), block(HBW_WAVES * 64);
  switch (a.bpad) {
    case 4: hipLaunchKernelGGL(head_bwd_kernel<4>, grid, block, 0, s, a); break;
    case 8: hipLaunchKernelGGL(head_bwd_kernel<8>, grid, block, 0, s, a); break;
    case 12: hipLaunchKernelGGL(head_bwd_kernel<12>, grid, block, 0, s, a); break;
    case 16: hipLaunchKernelGGL(head_bwd_kernel<16>, grid, block, 0, s, a); break;
    case 20: hipLaunchKernelGGL(head_bwd_kernel<20>, grid, block, 0, s, a); break;
    case 24: hipLaunchKernelGGL(head_bwd_kernel<24>, grid, block, 0, s, a); break;
    case 28: hipLaunchKernelGGL(head_bwd_kernel<28>, grid, block, 0, s, a); break;
    default: hipLaunchKernelGGL(head_bwd_kernel<32>, grid, block, 0, s, a); break;
  }
}

}  // namespace trpo
