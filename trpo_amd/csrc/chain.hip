// Fused row-local FVP chain (gfx950 / CDNA4).
//
// One launch evaluates, for every state of the shard, the whole row-local part
// of a Fisher-vector product (the FVP graph of trpo_inksci.py:56-70 by
// Pearlmutter's R-operator):
//
//   R-forward   RH_1     = (1-H_1^2)(X V_0 + c_0)
//               RH_{l+1} = (1-H_{l+1}^2)(RH_l W_l + H_l V_l + c_l)
//   R-head      RD_{L-1} = R-softmax-reverse(RH_{L-1} W_{L-1} + H_{L-1} V_{L-1} + c_{L-1})
//   R-backward  RD_{l-1} = (RD_l W_l^T + D_l V_l^T)(1-H_l^2) + E_{l-1} RH_l
//
// and writes RH_l / RD_l for the weight-gradient GEMMs (gemm.hip, wgrad).  The
// per-layer row-GEMM launches it replaces re-read every intermediate from HBM
// and serialise a three-load epilogue behind each main loop.  Here:
//
//  * Each wave owns 16 states.  The products run transposed,
//      out[feature][state] = W^T[feature][k] * in[k][state],
//    on v_mfma_f32_16x16x32_bf16 with the weights as the A operand, so a
//    layer's output tile lands in the accumulator as lane l = 16g + s holding
//    features 4g..4g+3 of state s ("acc layout").  Two such tiles are exactly
//    one 32-deep B operand of the next layer (lane: 8 k-values of state s), so
//    activations go from one layer to the next in registers with no LDS round
//    trip.  The k order this implies (chain_perm) is absorbed into the weight
//    images.
//  * fp32 accuracy on bf16 MFMA: both operands are split exactly into
//    hi + mid + lo bf16 pieces and 6 products are accumulated in f32 (the same
//    scheme as gemm.hip's split path).
//  * Weights stream through LDS in 32-deep k-chunks shared by all waves of the
//    workgroup, from pre-split, pre-permuted, pre-swizzled images (built by
//    chain_img_kernel: theta parts once per prepare, tangent parts per FVP), so
//    staging is a plain 16-B copy and every A-fragment read is one
//    conflict-free ds_read_b128.
//  * Epilogue operands (H, E, RH, P) and the second-segment activations (X, H,
//    D) are read straight into acc layout with per-workgroup buffer
//    descriptors (out-of-range rows / columns read 0 and drop stores).
#include "chain_common.h"
#include "kernels.h"

#include <stdexcept>

// Ablation build for profiling only (tools/chain_ablate.sh; never the shipped library):
// bit 0 = no weight-chunk staging, bit 1 = no chunk barriers, bit 2 = no activation loads.
#ifndef CHAIN_ABL
#define CHAIN_ABL 0
#endif

namespace trpo {
namespace {

// ---------------------------------------------------------------------------
// weight images: one thread per (chunk, row, k-group) writes 8 k-values x 3 planes
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) chain_img_kernel(const ChainImgArgs a, const float* theta, const float* v,
                                                        int which, const int* skip) {
  if (skip && *skip) return;
  const ChainImgJob& j = a.job[blockIdx.y];
  if (j.which != which) return;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= j.kc * j.otp * 4) return;
  const int gg = idx & 3;
  const int o = (idx >> 2) % j.otp;
  const int c = (idx >> 2) / j.otp;
  const float* src = (which ? v : theta) + j.src_off;
  cu16x8 h, m, l;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int k = 32 * c + chain_perm(8 * gg + q);
    float x = 0.0f;
    if (o < j.O && k < j.K) x = j.trans ? src[(size_t)o * j.ldw + k] : src[(size_t)k * j.ldw + o];
    unsigned short hh, mm, ll;
    csplit(x, hh, mm, ll);
    h[q] = hh;
    m[q] = mm;
    l[q] = ll;
  }
  unsigned short* dst = a.img + j.dst_off + (size_t)c * 3 * j.otp * 32 + o * 32 + ((gg ^ chain_hsw(o)) << 3);
  const size_t pl = (size_t)j.otp * 32;
  *reinterpret_cast<cu16x8*>(dst) = h;
  *reinterpret_cast<cu16x8*>(dst + pl) = m;
  *reinterpret_cast<cu16x8*>(dst + 2 * pl) = l;
}

// ---------------------------------------------------------------------------
// the chain kernel
//   OTM   : max 16-feature tiles of a hidden layer (hidden widths <= 16*OTM)
//   WAVES : waves per workgroup (16 states each)
//   OCC   : waves per SIMD the register budget is sized for
//   PIPE  : software-pipelined tile loop also at 16 register tiles (needs registers)
//   RING  : memory-sourced chunks loaded RING chunks ahead of their use (1 or 2)
//   PRE   : prefetch one epilogue operand during the memory segment (else load it at the epilogue)
//
// Issue order.  vmcnt retires vector-memory operations in issue order (loads and
// stores together), so every wait for a weight chunk also waits for whatever
// was issued before it.  Each chunk therefore issues, right after its barrier:
// the next weight chunk, then the deferred stores of the previous epilogue, then
// the activation loads needed two chunks later; epilogue operands are prefetched
// during the memory-sourced segment of their step.
// ---------------------------------------------------------------------------
template <int OTM, int WAVES, int OCC, bool PIPE, int RING, bool PRE>
__global__ void __launch_bounds__(WAVES * 64, OCC) fvp_chain_kernel(const ChainArgs a) {
  constexpr int NT = WAVES * 64;
  constexpr int CHU = 12 * 16 * OTM;   // 16-B units of the largest chunk: 3 planes x 16*OTM rows x 64 B
  constexpr int NLD = (CHU + NT - 1) / NT;
  constexpr int RB = 16 * WAVES;       // states per workgroup
  __shared__ cu32x4 wl[CHU];
  if (a.skip && *a.skip) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, s = lane & 15;
  const int64_t row_b = (int64_t)blockIdx.x * RB;
  const int rb = (int)((int64_t)a.n - row_b < RB ? (int64_t)a.n - row_b : RB);
  const int lrow = wave * 16 + s;
  const int frag = s * 32 + ((g ^ chain_hsw(s)) << 3);   // u16 offset of this lane's A fragment in a tile
  const int L = a.L;
  const f32x4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};

  // ---- operand helpers ----
  auto rsrc = [&](const float* p, int ld) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(p + row_b * ld), 0, rb * ld * 4, 0x00020000);
  };
  // byte offset of this lane's 4 features of tile t (acc layout); past the row end -> out of range
  auto voff = [&](int ld, int t) {
    const int col = 16 * t + 4 * g;
    return col < ld ? (lrow * ld + col) * 4 : rb * ld * 4;
  };
  auto ld4 = [&](__amdgpu_buffer_rsrc_t r, int vo) -> f32x4 {
    if constexpr (CHAIN_ABL & 4) return f32x4{0.5f, 0.25f, 0.125f, 0.0625f};
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, 0, 0));
  };
  auto st4 = [&](f32x4 x, __amdgpu_buffer_rsrc_t r, int vo) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(cu32x4, x), r, vo, 0, 0);
  };
  // tangent bias c_l at this lane's features of tile t
  auto bias4 = [&](int l, int t) -> f32x4 {
    const __amdgpu_buffer_rsrc_t rc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.v + a.offb[l]), 0, a.w[l + 1] * 4, 0x00020000);
    const int o = (16 * t + 4 * g) * 4;
    f32x4 r;
    r[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, o, 0, 0));
    r[1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, o + 4, 0, 0));
    r[2] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, o + 8, 0, 0));
    r[3] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, o + 12, 0, 0));
    return r;
  };
  auto mkb = [&](const f32x4& x0, const f32x4& x1, cbf16x8 (&b)[3]) { chain_mkb(x0, x1, b); };

  f32x4 acc[OTM], S[OTM], PF[OTM];   // S: first-segment source (RH_l / RD_l); PF: prefetched epilogue operand
#pragma unroll
  for (int t = 0; t < OTM; ++t) S[t] = z4;

  // ---- deferred epilogue stores of S ----
  float* pend_out = nullptr;
  int pend_ld = 0, pend_ot = 0;
  auto flush = [&]() __attribute__((always_inline)) {
    if (pend_out) {
      const __amdgpu_buffer_rsrc_t rO = rsrc(pend_out, pend_ld);
#pragma unroll
      for (int t = 0; t < OTM; ++t) st4(S[t], rO, t < pend_ot ? voff(pend_ld, t) : rb * pend_ld * 4);
      pend_out = nullptr;
    }
  };

  // ---- weight-chunk stream (consumption order = a.tab) ----
  const cu32x4* img = reinterpret_cast<const cu32x4*>(a.img);
  cu32x4 wr[NLD];
  int q = 0;
  // branch-free (no exec-masked loads or stores, so vmcnt waits stay counted): past the
  // last chunk the last one is re-read; lanes past a small chunk re-read its last unit
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
  // chunk q -> LDS; chunk q+1 -> registers
  auto chunk_begin = [&]() __attribute__((always_inline)) {
    // keep each chunk's work inside its chunk: hoisting later chunks' operand splits
    // or loads above the barriers only raises register pressure
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (!(CHAIN_ABL & 2)) lds_barrier();   // every wave is done with the previous chunk
    if constexpr (!(CHAIN_ABL & 1)) {
#pragma unroll
      for (int i = 0; i < NLD; ++i) {
        const int idx = tid + i * NT;
        if (CHU % NT == 0 || idx < CHU) wl[idx] = wr[i];
      }
    }
    if constexpr (!(CHAIN_ABL & 2)) lds_barrier();
    if constexpr (!(CHAIN_ABL & 1)) gload(++q);
  };

  // acc[0..OT) += W^T * B over the chunk in LDS.  The tile loop is branch-free
  // for the compile-time counts (all OTM tiles, or a head's 1-2) where registers
  // allow, so the LDS reads of a tile are issued under the MFMAs of the previous.
  auto mma_tile = [&](const unsigned short* W, int pl, int ot, const cbf16x8 (&b)[3]) __attribute__((always_inline)) {
    const cbf16x8 a0 = *reinterpret_cast<const cbf16x8*>(W + ot * 512);
    const cbf16x8 a1 = *reinterpret_cast<const cbf16x8*>(W + pl + ot * 512);
    const cbf16x8 a2 = *reinterpret_cast<const cbf16x8*>(W + 2 * pl + ot * 512);
    f32x4 c = acc[ot];
    // smallest terms first
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b[0], c, 0, 0, 0);
    acc[ot] = c;
  };
  auto mma = [&](int OT, const cbf16x8 (&b)[3]) __attribute__((always_inline)) {
    const unsigned short* W = reinterpret_cast<const unsigned short*>(&wl[0]) + frag;
    const int pl = OT * 512;   // u16 per plane
    if ((PIPE || OTM < 16) && OT == OTM) {
      cbf16x8 f[3], nx[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const cbf16x8*>(W + p * pl);
#pragma unroll
      for (int ot = 0; ot < OTM; ++ot) {
        if (ot + 1 < OTM) {
#pragma unroll
          for (int p = 0; p < 3; ++p) nx[p] = *reinterpret_cast<const cbf16x8*>(W + p * pl + (ot + 1) * 512);
        }
        f32x4 c = acc[ot];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[1], b[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[2], b[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[0], b[2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[1], b[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[0], b[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[0], b[0], c, 0, 0, 0);
        acc[ot] = c;
        if (ot + 1 < OTM) {
#pragma unroll
          for (int p = 0; p < 3; ++p) f[p] = nx[p];
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if ((PIPE || OTM < 16) && OT == 2) {
      mma_tile(W, pl, 0, b);
      mma_tile(W, pl, 1, b);
    } else if ((PIPE || OTM < 16) && OT == 1) {
      mma_tile(W, pl, 0, b);
    } else {
#pragma unroll
      for (int ot = 0; ot < OTM; ++ot)
        if (ot < OT) mma_tile(W, pl, ot, b);
    }
  };

  // One GEMM step: acc = [S (kc0 chunks, registers) | M1 (kc1 chunks, memory)] x images.
  // Memory chunk c is loaded RING chunks before its use; the epilogue operand Pre (OTp
  // tiles) is prefetched into PF at the first memory chunk.  Every chunk of a loop issues
  // the same vector-memory operations (out-of-range ones read 0 or are dropped), so the
  // compiler's vmcnt waits stay counted instead of collapsing to vmcnt(0).
  auto step = [&](int OT, int kc0, const float* M1, int ld1, int kc1, const float* Pre, int ldp, int OTp)
      __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < OTM; ++t) acc[t] = z4;
    const __amdgpu_buffer_rsrc_t r1 = rsrc(M1, ld1);
    const int oob1 = rb * ld1 * 4;
    auto mld = [&](int cc, int h) { return ld4(r1, cc < kc1 ? voff(ld1, 2 * cc + h) : oob1); };
    f32x4 n0 = z4, n1 = z4, m0 = z4, m1 = z4;
    if (kc0 < RING) {
      n0 = mld(0, 0);
      n1 = mld(0, 1);
    }
    if (RING == 2 && kc0 == 0) {
      m0 = mld(1, 0);
      m1 = mld(1, 1);
    }
    auto seg0_chunk = [&](int c, int kcc) __attribute__((always_inline)) {
      cbf16x8 b[3];
      mkb(S[2 * c], 2 * c + 1 < OTM ? S[2 * c + 1] : z4, b);
      chunk_begin();
      // the previous epilogue's stores (S is overwritten only by this step's epilogue;
      // every step after the first has kc0 >= 1)
      if (c == 0) flush();
      if (c == kcc - RING) {
        n0 = mld(0, 0);
        n1 = mld(0, 1);
      }
      if (RING == 2 && c == kcc - 1) {
        m0 = mld(1, 0);
        m1 = mld(1, 1);
      }
      mma(OT, b);
    };
    if (kc0 == (OTM + 1) / 2) {
#pragma unroll
      for (int c = 0; c < (OTM + 1) / 2; ++c) seg0_chunk(c, (OTM + 1) / 2);
    } else {
#pragma unroll
      for (int c = 0; c < (OTM + 1) / 2; ++c)
        if (c < kc0) seg0_chunk(c, kc0);
    }
    // memory chunk c: its operand was loaded RING chunks earlier; loads for chunk c + RING
    // go out right after this chunk's weight load.  Chunk 0 is peeled: it also issues the
    // epilogue prefetch, unconditionally, so that PF carries nothing across steps (a
    // conditional refill would keep it live through the register segment)
    auto mem_chunk = [&](int c, bool first) __attribute__((always_inline)) {
      const f32x4 x0 = n0, x1 = n1;
      if constexpr (RING == 2) {
        n0 = m0;
        n1 = m1;
      }
      chunk_begin();
      const f32x4 y0 = mld(c + RING, 0), y1 = mld(c + RING, 1);
      if constexpr (RING == 2) {
        m0 = y0;
        m1 = y1;
      } else {
        n0 = y0;
        n1 = y1;
      }
      if (PRE && first) {
        const __amdgpu_buffer_rsrc_t rp = rsrc(Pre, ldp);
#pragma unroll
        for (int t = 0; t < OTM; ++t) PF[t] = ld4(rp, t < OTp ? voff(ldp, t) : rb * ldp * 4);
      }
      cbf16x8 b[3];
      mkb(x0, x1, b);
      mma(OT, b);
    };
    mem_chunk(0, true);
    for (int c = 1; c < kc1; ++c) mem_chunk(c, false);
  };

  gload(0);

  // epilogue operand tile t: prefetched, or loaded now
  auto pre = [&](const float* p, int ld, int t) -> f32x4 {
    if constexpr (PRE) return PF[t];
    return ld4(rsrc(p, ld), voff(ld, t));
  };

  // ---- R-forward through the hidden layers ----
  for (int l = 0; l < L - 1; ++l) {
    const int j = l + 1, OT = (a.w[j] + 15) >> 4, kc = (a.w[l] + 31) >> 5, ldj = a.ld[j];
    if (l == 0) step(OT, 0, a.X, a.ld[0], kc, a.H[j], ldj, OT);
    else step(OT, kc, a.H[l], a.ld[l], kc, a.H[j], ldj, OT);
    // RH_j = (1 - H_j^2)(acc + c_l), H_j prefetched in PF
#pragma unroll
    for (int t = 0; t < OTM; ++t) {
      if (t < OT) {
        const f32x4 cb = bias4(l, t);
        f32x4 r;
        const f32x4 h = pre(a.H[j], ldj, t);
#pragma unroll
        for (int i = 0; i < 4; ++i) r[i] = c_one_minus_sq(h[i]) * (acc[t][i] + cb[i]);
        S[t] = r;
      } else {
        S[t] = z4;
      }
    }
    pend_out = a.RH[j];
    pend_ld = ldj;
    pend_ot = OT;
  }

  // ---- R-softmax head (layer L-1), SURVEY.md Appendix A ----
  {
    const int l = L - 1, A = a.w[L], ldA = a.ld[L];
    const int OTh = (A + 15) >> 4, kc = (a.w[l] + 31) >> 5;
    step(OTh, kc, a.H[l], a.ld[l], kc, a.P, ldA, 2);
    double rz[8], pd[8];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f32x4 cb = bias4(l, t);
      const f32x4 pv = pre(a.P, ldA, t);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool real = 16 * t + 4 * g + i < A;
        rz[4 * t + i] = real ? (double)(acc[t][i] + cb[i]) : 0.0;
        pd[4 * t + i] = real ? (double)pv[i] : 0.0;
      }
    }
    double prz = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) prz += pd[k] * rz[k];
    prz = sum4lanes(prz);
    double Rp[8], Aa[8], B[8], spB = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool real = 16 * (k >> 2) + 4 * g + (k & 3) < A;
      Rp[k] = pd[k] * (rz[k] - prz);
      const double den = pd[k] + (double)kEps;
      Aa[k] = real ? pd[k] / den : 0.0;
      B[k] = real ? (double)kEps / den : 0.0;
      spB += pd[k] * B[k];
    }
    spB = sum4lanes(spB);
    double sRAB = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) sRAB += Rp[k] * Aa[k] * B[k];
    sRAB = sum4lanes(sRAB);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x4 r;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = 4 * t + i;
        const bool real = 16 * t + 4 * g + i < A;
        const double rd = a.invN * (Rp[k] * (B[k] - spB) + Rp[k] * Aa[k] * Aa[k] + pd[k] * sRAB);
        r[i] = real ? (float)rd : 0.0f;
      }
      S[t] = r;
    }
#pragma unroll
    for (int t = 2; t < OTM; ++t) S[t] = z4;
    pend_out = a.RD[L - 1];
    pend_ld = ldA;
    pend_ot = 2;
  }

  // ---- R-backward down to the first hidden layer ----
  for (int l = L - 1; l >= 1; --l) {
    const int OT = (a.w[l] + 15) >> 4, kc = (a.w[l + 1] + 31) >> 5, ldl = a.ld[l];
    step(OT, kc, a.D[l], a.ld[l + 1], kc, a.E[l - 1], ldl, OT);
    // RD_{l-1} = acc (1 - H_l^2) + E_{l-1} RH_l, E prefetched in PF
    const __amdgpu_buffer_rsrc_t rH = rsrc(a.H[l], ldl), rR = rsrc(a.RH[l], ldl);
#pragma unroll
    for (int t = 0; t < OTM; ++t) {
      if (t < OT) {
        const int vo = voff(ldl, t);
        const f32x4 h = ld4(rH, vo), rh = ld4(rR, vo), e = pre(a.E[l - 1], ldl, t);
        f32x4 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) r[i] = fmaf(e[i], rh[i], acc[t][i] * c_one_minus_sq(h[i]));
        S[t] = r;
      } else {
        S[t] = z4;
      }
    }
    pend_out = a.RD[l - 1];
    pend_ld = ldl;
    pend_ot = OT;
  }
  flush();
}

template <int OTM, int WAVES, int OCC, bool PIPE = false, int RING = 2, bool PRE = true>
void launch_chain_cfg(const ChainArgs& a, hipStream_t s) {
  const long nblk = (a.n + 16 * WAVES - 1) / (16 * WAVES);
  hipLaunchKernelGGL((fvp_chain_kernel<OTM, WAVES, OCC, PIPE, RING, PRE>), dim3((unsigned)nblk), dim3(WAVES * 64), 0, s, a);
}

template <int OTM>
void launch_chain_otm(const ChainArgs& a, hipStream_t s) {
  // 1 = auto: 64-state workgroups (two per CU) where the 48-VGPR chunk staging fits the
  // register budget (4 register tiles); 128-state workgroups for 8 and 16
  const int v = g_options.chain == 1 ? (OTM >= 8 ? 2 : 3) : g_options.chain;
  if (v == 2) launch_chain_cfg<OTM, 8, 2>(a, s);   // 128 states / WG, one WG per CU
  else launch_chain_cfg<OTM, 4, 2>(a, s);          // 64 states / WG, two WGs per CU
}

}  // namespace

int chain_max_tiles(int max_hidden) {
  if (max_hidden <= 64) return 4;
  if (max_hidden <= 128) return 8;
  if (max_hidden <= 256) return 16;
  return 0;
}

void launch_fvp_chain(const ChainArgs& a, int otm, hipStream_t s) {
  if (a.n <= 0) return;
  if (a.L < 2 || a.L > kMaxLayers || a.w[a.L] > 32) throw std::runtime_error("fvp chain: unsupported shape");
  for (int l = 1; l < a.L; ++l)
    if (a.w[l] > 16 * otm) throw std::runtime_error("fvp chain: hidden layer wider than the register tile");
  switch (otm) {
    case 4: launch_chain_otm<4>(a, s); break;
    case 8: launch_chain_otm<8>(a, s); break;
    case 16: launch_chain_otm<16>(a, s); break;
    default: throw std::runtime_error("fvp chain: bad tile count");
  }
}

void launch_chain_img(const ChainImgArgs& a, const float* theta, const float* v, int which, const int* skip,
                      hipStream_t s) {
  int maxb = 0, nj = 0;
  for (int i = 0; i < a.n; ++i) {
    const ChainImgJob& j = a.job[i];
    if (j.which != which) continue;
    ++nj;
    const int b = (j.kc * j.otp * 4 + 255) / 256;
    maxb = b > maxb ? b : maxb;
  }
  if (!nj) return;
  hipLaunchKernelGGL(chain_img_kernel, dim3(maxb, a.n), dim3(256), 0, s, a, theta, v, which, skip);
}

}  // namespace trpo
