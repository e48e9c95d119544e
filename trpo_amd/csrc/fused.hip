// Fused small-width Fisher-vector product (gfx950 / CDNA4).
//
// The whole FVP of trpo_inksci.py:56-70 (Pearlmutter's R-operator) for a
// policy with one or two tanh hidden layers of width <= 64 and <= 32 actions (C1, C2, C3) in ONE
// persistent launch per shard.  For every group of 16*FW states it runs the R-forward, the
// R-softmax head and the R-backward exactly as fvp_chain_kernel does (chain.hip: 16 states per
// wave, activations in MFMA accumulator layout, weights streamed through LDS from the chain's
// pre-split images), and in the same launch the weight R-gradients
//     (Hv)_W_m = RH_m^T D_m + H_m^T RD_m   (H_0 = X, RH_0 = 0) ,   (Hv)_b_m = colsum RD_m
// (engine.cpp fvp(), trpo_inksci.py:69-70 flatgrad).  RH_m and RD_m never reach HBM: the launch
// reads X, H_m, D_m, E_m and P and writes one partial-gradient slab per workgroup; the chain path
// wrote RH / RD and three weight-gradient GEMMs read them back with the activations again.
//
// Weight-gradient products (rows = the MFMA k dimension).  Per pass, the two operands (act = RH_m,
// H_m or X; delta = D_m or RD_m) of all 16*FW states of the group sit in two LDS images of exact
// bf16 hi/mid/lo planes, [state][64 features], 32-B chunks swizzled.  An image is written from
// registers (RH, RD: acc layout, 8 B per lane and plane), captured while the chain splits the
// same values into its own B operands (H_{L-1} in the head step, D_m in the R-backward step m),
// or re-read (X, H_m below the last hidden layer).  Fragments come back with ds_read_b64_tr_b16:
// lane (i, g) gets states 8g..8g+7 of feature i, the v_mfma_f32_16x16x32_bf16 operand layout, for
// both operands.  Wave w owns every FW-th 16x16 tile of every layer's gradient (registers, across
// the whole launch); 6 products per tile pair, as chain.hip.  Bias sums come from the f32 RD
// values by 16-lane shuffles into per-wave LDS rows.  launch_reduce_slab then sums the slabs in
// index order: deterministic.
//
// States past the shard end read zeros (buffer descriptors), which makes their RD_m and D_m zero
// and their contributions exactly 0.
#include "chain_common.h"
#include "kernels.h"

#include <stdexcept>

// Ablation build for profiling only (tools/fused_ablate.sh; never the shipped library): bit 0 = no
// per-state activation loads, bit 1 = no weight-gradient passes, bit 2 = no weight-chunk staging.
#ifndef FUSED_ABL
#define FUSED_ABL 0
#endif

namespace trpo {
namespace {

// NL = layers (2: one hidden layer, 3: two), FW = waves per workgroup, OBC = 64-wide chunks of obs
#ifndef FUSED_LB
#define FUSED_LB 2   // workgroups per CU the register budget is sized for (A/B builds: 1)
#endif
template <int NL, int FW, int OBC>
__global__ void __launch_bounds__(FW * 64, FUSED_LB) fvp_fused_kernel(const FusedArgs fa) {
  constexpr int OTM = 4;                      // 16-feature tiles of a hidden layer
  constexpr int NT = FW * 64;
  constexpr int CHU = 12 * 16 * OTM;          // 16-B units of the largest weight chunk
  constexpr int NLD = (CHU + NT - 1) / NT;
  constexpr int RB = 16 * FW;                 // states per group
  constexpr int PL = RB * kFI;                // u16 per image plane
  constexpr int KS = RB / 32;                 // k-steps of a gradient pass
  constexpr int RING = 2;
  constexpr int TW0 = (OBC * 16 + FW - 1) / FW;   // owned tiles: obs x hidden
  constexpr int TWH = (16 + FW - 1) / FW;         //              hidden x hidden (NL == 3)
  constexpr int TWL = (8 + FW - 1) / FW;          //              hidden x actions
  __shared__ cu32x4 wl[CHU];
  __shared__ __attribute__((aligned(16))) unsigned short simg[2][3 * PL];   // [act | delta] images
  __shared__ float sb[FW][NL][64];                                         // per-wave bias sums
  __shared__ __attribute__((aligned(16))) float sc[NL][64];               // the tangent's biases c_l

  const ChainArgs& a = fa.c;
  if (a.skip && *a.skip) return;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, s = lane & 15;
  const f32x4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
  unsigned short* const sA = &simg[0][0];
  unsigned short* const sD = &simg[1][0];

  for (int i = tid; i < FW * NL * 64; i += NT) (&sb[0][0][0])[i] = 0.0f;
  for (int i = tid; i < NL * 64; i += NT) {   // read once: every step's epilogue adds them
    const int l = i >> 6, j = i & 63;
    sc[l][j] = j < a.w[l + 1] ? a.v[a.offb[l] + j] : 0.0f;
  }

  f32x4 dw0[TW0], dwh[TWH], dwl[TWL];
#pragma unroll
  for (int k = 0; k < TW0; ++k) dw0[k] = z4;
#pragma unroll
  for (int k = 0; k < TWH; ++k) dwh[k] = z4;
#pragma unroll
  for (int k = 0; k < TWL; ++k) dwl[k] = z4;

  f32x4 acc[OTM], S[OTM], PF[OTM], RHk[NL][OTM];
  f32x4 xn0 = z4, xn1 = z4;   // first X chunk of the next group (loaded one group ahead)
  const int ngroups = fa.ngroups;
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int64_t row_b = (int64_t)grp * RB;
    const int rb = (int)((int64_t)a.n - row_b < RB ? (int64_t)a.n - row_b : RB);
    // lane-derived offsets are recomputed per group from an opaque copy of threadIdx.x: hoisted out
    // of the group loop they would stay live (and spill) across the whole launch
    int tid;
    asm volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"((int)threadIdx.x));
    const int lane = tid & 63, g = lane >> 4, s = lane & 15;
    const int lrow = wave * 16 + s;
    const int frag = s * 32 + ((g ^ chain_hsw(s)) << 3);

    // ---- weight-chunk stream (consumption order = a.tab), as chain.hip ----
    const cu32x4* img = reinterpret_cast<const cu32x4*>(a.img);
    cu32x4 wr[NLD];
    int q = 0;
    auto gload = [&](int qq) {
      qq = qq < a.nchunks ? qq : a.nchunks - 1;
      const int off = a.tab[2 * qq], sz = a.tab[2 * qq + 1];
      const cu32x4* src = img + off;
#pragma unroll
      for (int i = 0; i < NLD; ++i) {
        const int idx = tid + i * NT;
        wr[i] = src[idx < sz ? idx : sz - 1];
      }
    };
    auto chunk_begin = [&]() __attribute__((always_inline)) {
      __builtin_amdgcn_sched_barrier(0);
      lds_barrier();   // every wave is done with the previous chunk (and with the previous pass)
      if constexpr ((FUSED_ABL & 4) == 0) {
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
          const int idx = tid + i * NT;
          if (CHU % NT == 0 || idx < CHU) wl[idx] = wr[i];
        }
      }
      lds_barrier();
      if constexpr ((FUSED_ABL & 4) == 0) gload(++q);
    };

    // ---- image helpers ----
    // acc-layout tile t of this lane (features 16t + 4g.., state lrow) -> 3 planes
    auto put4 = [&](unsigned short* slot, int t, const f32x4& x) {
      cu16x4 h, m, l;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        unsigned short hh, mm, ll;
        csplit(x[j], hh, mm, ll);
        h[j] = hh;
        m[j] = mm;
        l[j] = ll;
      }
      const int o = fimg(lrow, 16 * t + 4 * g);
      *reinterpret_cast<cu16x4*>(slot + o) = h;
      *reinterpret_cast<cu16x4*>(slot + PL + o) = m;
      *reinterpret_cast<cu16x4*>(slot + 2 * PL + o) = l;
    };
    // the f32 values of acc-layout tile t of this lane back from the 3 planes (exact: hi + mid + lo)
    auto get4 = [&](const unsigned short* slot, int t) -> f32x4 {
      const int o = fimg(lrow, 16 * t + 4 * g);
      const cu16x4 h = *reinterpret_cast<const cu16x4*>(slot + o);
      const cu16x4 m = *reinterpret_cast<const cu16x4*>(slot + PL + o);
      const cu16x4 l = *reinterpret_cast<const cu16x4*>(slot + 2 * PL + o);
      f32x4 r;
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = (cb_val(h[j]) + cb_val(m[j])) + cb_val(l[j]);
      return r;
    };
    // chain B operand of chunk c (tiles 2c, 2c+1) -> 3 planes
    auto putb = [&](unsigned short* slot, int c, const cbf16x8 (&b)[3]) {
      const int o0 = fimg(lrow, 32 * c + 4 * g), o1 = fimg(lrow, 32 * c + 16 + 4 * g);
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const cu16x8 v = __builtin_bit_cast(cu16x8, b[p]);
        *reinterpret_cast<cu16x4*>(slot + p * PL + o0) = cu16x4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<cu16x4*>(slot + p * PL + o1) = cu16x4{v[4], v[5], v[6], v[7]};
      }
    };
    // 16x16x32 operand of feature tile ft, k-step ks: lane (i = lane&15, g) <- states 32ks + 8g .. +7
    const int tq = (lane >> 2) & 3, tp = lane & 3;
    auto tfrag = [&](const unsigned short* slot, int ft, int ks, cbf16x8 (&f)[3]) {
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        fs8 v;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int r = 32 * ks + 8 * g + 4 * t + tq;
          const fs4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) fs4*)(slot + p * PL + fimg(r, 16 * ft + 4 * tp)));
#pragma unroll
          for (int e = 0; e < 4; ++e) v[4 * t + e] = x[e];
        }
        f[p] = __builtin_bit_cast(cbf16x8, v);
      }
    };
    // gradient products of this wave's tiles of a layer (TI x TJ tiles) whose act tile lies in
    // [ti0, ti0 + 4) against the two images
    auto run = [&](auto& dacc, int TI, int TJ, int ti0) __attribute__((always_inline)) {
      constexpr int TWm = sizeof(dacc) / sizeof(f32x4);
#pragma unroll
      for (int k = 0; k < TWm; ++k) {
        const int u = wave + FW * k;
        const int it = u / TJ, jt = u - (u / TJ) * TJ;
        if (u < TI * TJ && it >= ti0 && it < ti0 + 4) {
          f32x4 c = dacc[k];
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            cbf16x8 fa_[3], fd_[3];
            tfrag(sA, it - ti0, ks, fa_);
            tfrag(sD, jt, ks, fd_);
            c = chain_mfma6(fa_, fd_, c);
            __builtin_amdgcn_sched_barrier(0);
          }
          dacc[k] = c;
        }
      }
    };
    // bias sums of layer m from acc-layout RD tiles: sum over the wave's 16 states
    auto bias_add = [&](int m, int OT, const f32x4 (&R)[OTM]) {
#pragma unroll
      for (int t = 0; t < OTM; ++t) {
        if (t < OT) {
          f32x4 v = R[t];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = sum16_dpp(v[j]);   // the wave's 16 states of lane group g (common.h: DPP moves)
          }
          if (s == 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) sb[wave][m][16 * t + 4 * g + j] += v[j];
          }
        }
      }
    };


    auto rsrc = [&](const float* p, int ld) {
      return __builtin_amdgcn_make_buffer_rsrc((void*)(p + row_b * ld), 0, rb * ld * 4, 0x00020000);
    };
    auto voff = [&](int ld, int t) {
      const int col = 16 * t + 4 * g;
      return col < ld ? (lrow * ld + col) * 4 : rb * ld * 4;
    };
    auto ld4 = [&](__amdgpu_buffer_rsrc_t r, int vo) -> f32x4 {
      if constexpr (FUSED_ABL & 1) return f32x4{0.5f, 0.25f, 0.125f, 0.0625f};
      return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, 0, 0));
    };
    auto bias4 = [&](int l, int t) -> f32x4 { return *reinterpret_cast<const f32x4*>(&sc[l][16 * t + 4 * g]); };

    auto mma_tile = [&](const unsigned short* W, int pl, int ot, const cbf16x8 (&b)[3]) __attribute__((always_inline)) {
      cbf16x8 w3[3];
      w3[0] = *reinterpret_cast<const cbf16x8*>(W + ot * 512);
      w3[1] = *reinterpret_cast<const cbf16x8*>(W + pl + ot * 512);
      w3[2] = *reinterpret_cast<const cbf16x8*>(W + 2 * pl + ot * 512);
      acc[ot] = chain_mfma6(w3, b, acc[ot]);
    };
    auto mma = [&](int OT, const cbf16x8 (&b)[3]) __attribute__((always_inline)) {
      const unsigned short* W = reinterpret_cast<const unsigned short*>(&wl[0]) + frag;
      const int pl = OT * 512;   // u16 per plane
      if (OT == OTM) {
        cbf16x8 f[3], nx[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const cbf16x8*>(W + p * pl);
#pragma unroll
        for (int ot = 0; ot < OTM; ++ot) {
          if (ot + 1 < OTM) {
#pragma unroll
            for (int p = 0; p < 3; ++p) nx[p] = *reinterpret_cast<const cbf16x8*>(W + p * pl + (ot + 1) * 512);
          }
          acc[ot] = chain_mfma6(f, b, acc[ot]);
          if (ot + 1 < OTM) {
#pragma unroll
            for (int p = 0; p < 3; ++p) f[p] = nx[p];
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      } else if (OT == 2) {
        mma_tile(W, pl, 0, b);
        mma_tile(W, pl, 1, b);
      } else if (OT == 1) {
        mma_tile(W, pl, 0, b);
      } else {
#pragma unroll
        for (int ot = 0; ot < OTM; ++ot)
          if (ot < OT) mma_tile(W, pl, ot, b);
      }
    };

    // One chain step: acc = [S (kc0 chunks, registers) | M1 (kc1 chunks, memory)] x images, with
    // the epilogue operand Pre prefetched into PF; cap (optional) receives M1's split planes.
    auto step = [&](int OT, int kc0, const float* M1, int ld1, int kc1, const float* Pre, int ldp, int OTp,
                    unsigned short* cap, bool pre = false) __attribute__((always_inline)) {
      __builtin_amdgcn_sched_barrier(0);   // keep each step's loads inside the step
#pragma unroll
      for (int t = 0; t < OTM; ++t) acc[t] = z4;
      const __amdgpu_buffer_rsrc_t r1 = rsrc(M1, ld1);
      const int oob1 = rb * ld1 * 4;
      auto mld = [&](int cc, int h) { return ld4(r1, cc < kc1 ? voff(ld1, 2 * cc + h) : oob1); };
      f32x4 n0 = z4, n1 = z4, m0 = z4, m1 = z4;
      if (pre) {            // the first chunk was loaded ahead (X of this group, issued by the previous one)
        n0 = xn0;
        n1 = xn1;
      } else if (kc0 < RING) {
        n0 = mld(0, 0);
        n1 = mld(0, 1);
      }
      if (kc0 == 0) {
        m0 = mld(1, 0);
        m1 = mld(1, 1);
      }
      auto seg0_chunk = [&](int c, int kcc) __attribute__((always_inline)) {
        cbf16x8 b[3];
        chain_mkb(S[2 * c], S[2 * c + 1], b);
        chunk_begin();
        if (c == kcc - RING) {
          n0 = mld(0, 0);
          n1 = mld(0, 1);
        }
        if (c == kcc - 1) {
          m0 = mld(1, 0);
          m1 = mld(1, 1);
        }
        mma(OT, b);
      };
      if (kc0 == 2) {
#pragma unroll
        for (int c = 0; c < 2; ++c) seg0_chunk(c, 2);
      } else {
#pragma unroll
        for (int c = 0; c < 2; ++c)
          if (c < kc0) seg0_chunk(c, kc0);
      }
      auto mem_chunk = [&](int c, bool first) __attribute__((always_inline)) {
        const f32x4 x0 = n0, x1 = n1;
        n0 = m0;
        n1 = m1;
        chunk_begin();
        m0 = mld(c + RING, 0);
        m1 = mld(c + RING, 1);
        if (first) {
          const __amdgpu_buffer_rsrc_t rp = rsrc(Pre, ldp);
#pragma unroll
          for (int t = 0; t < OTM; ++t) PF[t] = ld4(rp, t < OTp ? voff(ldp, t) : rb * ldp * 4);
        }
        cbf16x8 b[3];
        chain_mkb(x0, x1, b);
        if (cap && c < 2) putb(cap, c, b);
        mma(OT, b);
      };
      mem_chunk(0, true);
      for (int c = 1; c < kc1; ++c) mem_chunk(c, false);
    };

    // a gradient pass of layer m with the act image holding act tiles [ti0, ti0+4)
    auto pass_run = [&](int m, int ti0) __attribute__((always_inline)) {
      if constexpr ((FUSED_ABL & 2) != 0) return;
      __builtin_amdgcn_sched_barrier(0);
      const int TI = (a.w[m] + 15) >> 4, TJ = (a.w[m + 1] + 15) >> 4;
      if (m == 0) run(dw0, TI, TJ, ti0);
      else if (m == NL - 1) run(dwl, TI, TJ, ti0);
      else run(dwh, TI, TJ, ti0);
    };

    q = 0;
    gload(0);
    if (grp == (int)blockIdx.x) {   // later groups' first X chunk is loaded during the previous group
      const __amdgpu_buffer_rsrc_t rx = rsrc(a.X, a.ld[0]);
      xn0 = ld4(rx, voff(a.ld[0], 0));
      xn1 = ld4(rx, voff(a.ld[0], 1));
    }

    // ---- R-forward through the hidden layers: RH_{l+1} = (1 - H^2)(RH_l W + H_l V + c) ----
#pragma unroll
    for (int l = 0; l < NL - 1; ++l) {
      const int j = l + 1, OT = (a.w[j] + 15) >> 4, kc = (a.w[l] + 31) >> 5, ldj = a.ld[j];
      if (l == 0) step(OT, 0, a.X, a.ld[0], kc, a.H[j], ldj, OT, nullptr, true);
      else step(OT, kc, a.H[l], a.ld[l], kc, a.H[j], ldj, OT, nullptr);
#pragma unroll
      for (int t = 0; t < OTM; ++t) {
        f32x4 r = z4;
        if (t < OT) {
          const f32x4 cb = bias4(l, t);
          const f32x4 h = PF[t];
#pragma unroll
          for (int i = 0; i < 4; ++i) r[i] = c_one_minus_sq(h[i]) * (acc[t][i] + cb[i]);
        }
        S[t] = r;
        RHk[j][t] = r;
      }
    }

    // ---- R-softmax head (layer NL-1), chain.hip / SURVEY.md Appendix A; H_{NL-1} captured ----
    {
      const int l = NL - 1, A = a.w[NL], ldA = a.ld[NL];
      const int OTh = (A + 15) >> 4, kc = (a.w[l] + 31) >> 5;
      step(OTh, kc, a.H[l], a.ld[l], kc, a.P, ldA, 2, sA);
      // f64 as chain.hip, bit for bit; only the f32 inputs stay live (A and B are recomputed)
      float zf[8], pf[8];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const f32x4 cb = bias4(l, t);
        const f32x4 pv = PF[t];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool real = 16 * t + 4 * g + i < A;
          zf[4 * t + i] = real ? acc[t][i] + cb[i] : 0.0f;
          pf[4 * t + i] = real ? pv[i] : 0.0f;
        }
      }
      double prz = 0.0;
#pragma unroll
      for (int k = 0; k < 8; ++k) prz += (double)pf[k] * (double)zf[k];
      prz = sum4lanes(prz);
      double spB = 0.0, sRAB = 0.0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const bool real = 16 * (k >> 2) + 4 * g + (k & 3) < A;
        const double pd = (double)pf[k];
        const double Rp = pd * ((double)zf[k] - prz);
        const double den = pd + (double)kEps;
        const double Aa = real ? pd / den : 0.0;
        const double B = real ? (double)kEps / den : 0.0;
        spB += pd * B;
        sRAB += Rp * Aa * B;
      }
      spB = sum4lanes(spB);
      sRAB = sum4lanes(sRAB);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = 4 * t + i;
          const bool real = 16 * t + 4 * g + i < A;
          const double pd = (double)pf[k];
          const double Rp = pd * ((double)zf[k] - prz);
          const double den = pd + (double)kEps;
          const double Aa = real ? pd / den : 0.0;
          const double B = real ? (double)kEps / den : 0.0;
          const double rd = a.invN * (Rp * (B - spB) + Rp * Aa * Aa + pd * sRAB);
          r[i] = real ? (float)rd : 0.0f;
        }
        S[t] = r;
      }
#pragma unroll
      for (int t = 2; t < OTM; ++t) S[t] = z4;
      // gradient pass: (Hv)_W_{NL-1} += H^T RD_{NL-1}  (act captured in the step)
      lds_barrier();
      put4(sD, 0, S[0]);
      put4(sD, 1, S[1]);
      bias_add(NL - 1, OTh, S);
      lds_barrier();
      pass_run(NL - 1, 0);
    }

    // ---- R-backward: RD_{l-1} = (RD_l W^T + D_l V^T)(1 - H_l^2) + E_{l-1} RH_l; D_l captured ----
#pragma unroll
    for (int l = NL - 1; l >= 1; --l) {
      const int OT = (a.w[l] + 15) >> 4, kc = (a.w[l + 1] + 31) >> 5, ldl = a.ld[l];
      step(OT, kc, a.D[l], a.ld[l + 1], kc, a.E[l - 1], ldl, OT, sD);
      // H_l for (1 - H_l^2) comes from the act image, which holds this wave's own rows of H_l at this
      // point (captured in the head step for l = NL-1, re-read for the previous pass otherwise): the
      // three bf16 planes sum back to the f32 value exactly, and no HBM load sits on the critical path
#pragma unroll
      for (int t = 0; t < OTM; ++t) {
        f32x4 r = z4;
        if (t < OT) {
          const f32x4 h = get4(sA, t), e = PF[t], rh = RHk[l][t];
#pragma unroll
          for (int i = 0; i < 4; ++i) r[i] = fmaf(e[i], rh[i], acc[t][i] * c_one_minus_sq(h[i]));
        }
        S[t] = r;
      }
      // (Hv)_W_l += RH_l^T D_l ; the next pass's act operand (H_{l-1}, or X's first 64 features) is
      // loaded meanwhile
      lds_barrier();
#pragma unroll
      for (int t = 0; t < OTM; ++t) put4(sA, t, RHk[l][t]);
      f32x4 nxt[OTM];
      {
        const int ldn = a.ld[l - 1];
        const __amdgpu_buffer_rsrc_t rn = rsrc(l - 1 >= 1 ? a.H[l - 1] : a.X, ldn);
#pragma unroll
        for (int t = 0; t < OTM; ++t) nxt[t] = ld4(rn, voff(ldn, t));
      }
      lds_barrier();
      pass_run(l, 0);
      // (Hv)_W_{l-1} += H_{l-1}^T RD_{l-1}  (X for l-1 = 0, in 64-feature chunks)
      lds_barrier();
#pragma unroll
      for (int t = 0; t < OTM; ++t) put4(sD, t, S[t]);
      bias_add(l - 1, OT, S);
#pragma unroll
      for (int t = 0; t < OTM; ++t) put4(sA, t, nxt[t]);
      if (l - 1 >= 1) {
        lds_barrier();
        pass_run(l - 1, 0);
      } else {
        const __amdgpu_buffer_rsrc_t rx = rsrc(a.X, a.ld[0]);
#pragma unroll
        for (int ch = 0; ch < OBC; ++ch) {
          if (ch + 1 < OBC) {
#pragma unroll
            for (int t = 0; t < OTM; ++t) nxt[t] = ld4(rx, voff(a.ld[0], 4 * (ch + 1) + t));
          } else {
            // the next group's first X chunk, in flight during this last gradient pass
            const int64_t nb = row_b + (int64_t)gridDim.x * RB;
            const int nrb = (int)((int64_t)a.n - nb < RB ? (int64_t)a.n - nb : RB);
            const __amdgpu_buffer_rsrc_t rxn = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(a.X + (nb < a.n ? nb : 0) * a.ld[0]), 0, nb < a.n ? nrb * a.ld[0] * 4 : 0, 0x00020000);
            xn0 = ld4(rxn, voff(a.ld[0], 0));
            xn1 = ld4(rxn, voff(a.ld[0], 1));
          }
          lds_barrier();
          pass_run(0, 4 * ch);
          if (ch + 1 < OBC) {
            lds_barrier();
#pragma unroll
            for (int t = 0; t < OTM; ++t) put4(sA, t, nxt[t]);
          }
        }
      }
    }
  }

  // ---- this workgroup's slab: owned gradient tiles (C layout: rows 4g + r, column s) and biases ----
  __syncthreads();
  float* out = fa.slab + (size_t)blockIdx.x * fa.slab_stride;
  auto wout = [&](auto& dacc, int m) __attribute__((always_inline)) {
    constexpr int TWm = sizeof(dacc) / sizeof(f32x4);
    const int wi = a.w[m], wj = a.w[m + 1];
    const int TI = (wi + 15) >> 4, TJ = (wj + 15) >> 4;
#pragma unroll
    for (int k = 0; k < TWm; ++k) {
      const int u = wave + FW * k;
      if (u < TI * TJ) {
        const int it = u / TJ, jt = u - (u / TJ) * TJ;
        const int j = 16 * jt + s;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 16 * it + 4 * g + r;
          if (i < wi && j < wj) out[fa.offW[m] + (int64_t)i * wj + j] = dacc[k][r];
        }
      }
    }
  };
  wout(dw0, 0);
  if constexpr (NL == 3) wout(dwh, 1);
  wout(dwl, NL - 1);
  for (int i = tid; i < NL * 64; i += NT) {
    const int m = i >> 6, j = i & 63;
    if (j < a.w[m + 1]) {
      float t = 0.0f;
#pragma unroll
      for (int u = 0; u < FW; ++u) t += sb[u][m][j];
      out[a.offb[m] + j] = t;
    }
  }
}

template <int NL, int FW>
void launch_fused_nl(const FusedArgs& a, int grid, hipStream_t s) {
  const int obc = (a.c.w[0] + 63) / 64;
  switch (obc) {
    case 1: hipLaunchKernelGGL((fvp_fused_kernel<NL, FW, 1>), dim3(grid), dim3(FW * 64), 0, s, a); break;
    case 2: hipLaunchKernelGGL((fvp_fused_kernel<NL, FW, 2>), dim3(grid), dim3(FW * 64), 0, s, a); break;
    default: throw std::runtime_error("fused fvp: obs_dim > 128");
  }
}

}  // namespace

bool fused_fvp_eligible(int L, const int* w) {
  if (L != 2 && L != 3) return false;
  if (w[0] > 128 || w[L] > 32) return false;
  for (int l = 1; l < L; ++l)
    if (w[l] > 64) return false;
  return true;
}

int fused_fvp_states_per_group(int variant) { return variant == 2 ? 64 : 128; }

void launch_fvp_fused(const FusedArgs& a, int grid, int variant, hipStream_t s) {
  if (grid <= 0) return;   // n = 0: the launch still writes the (zero) slab of workgroup 0
  if (!fused_fvp_eligible(a.c.L, a.c.w)) throw std::runtime_error("fused fvp: unsupported shape");
  const int rb = fused_fvp_states_per_group(variant);
  if (a.ngroups != (a.c.n + rb - 1) / rb) throw std::runtime_error("fused fvp: group count does not match");
  if (variant == 2) {
    if (a.c.L == 2) launch_fused_nl<2, 4>(a, grid, s);
    else launch_fused_nl<3, 4>(a, grid, s);
  } else {
    if (a.c.L == 2) launch_fused_nl<2, 8>(a, grid, s);
    else launch_fused_nl<3, 8>(a, grid, s);
  }
}

}  // namespace trpo
