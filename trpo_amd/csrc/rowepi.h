// Device-side pieces shared by the row-GEMM translation units (gemm.hip, plane.hip): the fused
// row epilogues, running-max bookkeeping, split helpers and the LDS-DMA primitive.  Everything is in an
// anonymous namespace (internal linkage per translation unit).
#pragma once
#include "common.h"
#include "kernels.h"

#ifndef TRPO_EPI_PIPE
#define TRPO_EPI_PIPE 1    // 0: epilogue operand loads chunk by chunk (A/B builds only)
#endif
#ifndef TRPO_FAST_TANH
#define TRPO_FAST_TANH 1   // 0: the device library's tanhf in the forward epilogues (A/B builds only)
#endif
#ifndef TRPO_HEAD_DPP
#define TRPO_HEAD_DPP 1    // 0: head row reductions by ds_bpermute shuffles (A/B builds only)
#endif
#ifndef TRPO_EPI_TRACK
#define TRPO_EPI_TRACK 1   // ablation builds only (tools): 0 drops the f16 running-max tracking
#endif
#ifndef TRPO_PREP_HEAD64
#define TRPO_PREP_HEAD64 0 // 1: the prepare head's KL / surr logit deltas in f64 (round-4 form; A/B only)
#endif
#ifndef TRPO_HEAD_LOG64
#define TRPO_HEAD_LOG64 0  // 1: the loss heads' logs in f64 (round-1 form; A/B only)
#endif

namespace trpo {
namespace {


__device__ __forceinline__ float one_minus_sq(float h) { return (1.0f - h) * (1.0f + h); }

// tanh for the forward epilogues (trpo_inksci.py:38 `tanh` layers), branch-free: both forms are
// evaluated and one selected, where the device library's tanhf branches per lane (a wave runs both
// sides under exec masks, ~35 VALU per element, which made the tanh epilogue ~2 ms of a 256-wide
// C4 forward GEMM).  |x| < 0.625: x + x^3 P(x^2), the minimax odd polynomial of the device library's
// own small-argument branch; otherwise (1 - t) / (1 + t) with t = 2^(-2|x| log2 e) from v_exp_f32
// and v_rcp_f32 (a few ulp; t underflows to 0 past |x| ~ 44, giving 1).  Sign restored last.
__device__ __forceinline__ float tanh_fast(float x) {
#if TRPO_FAST_TANH
  const float ax = fabsf(x);
  const float x2 = x * x;
  float p = __builtin_fmaf(-0.005700020585209131f, x2, 0.02063407190144062f);   // 0xbbbac73d, 0x3ca908c9
  p = __builtin_fmaf(p, x2, -0.053737930953502655f);                        // 0xbd5c1c4e
  p = __builtin_fmaf(p, x2, 0.13331416249275208f);                         // 0x3e088382
  p = __builtin_fmaf(p, x2, -0.3333328068256378f);                        // 0xbeaaaa99
  const float small = __builtin_fmaf(x2, ax * p, ax);
  const float t = __builtin_amdgcn_exp2f(ax * -2.8853900817779268f);   // 2^(-2|x| log2 e) = e^(-2|x|)
  const float r = __builtin_amdgcn_rcpf(1.0f + t);
  const float big = __builtin_fmaf(-t, r, r);                          // (1 - t) / (1 + t)
  return __builtin_copysignf(ax < 0.625f ? small : big, x);
#else
  return tanhf(x);
#endif
}

#if TRPO_HEAD_DPP
// 32-lane (wave-half) reductions on DPP moves + one ds_swizzle (common.h)
__device__ __forceinline__ float hsum32(float v) { return sum32_dpp(v); }
__device__ __forceinline__ double hsum32d(double v) { return sum32_dpp(v); }
__device__ __forceinline__ float hmax32(float v) { return max32_dpp(v); }
#else
__device__ __forceinline__ float hsum32(float v) {
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off, 32);
  return v;
}
__device__ __forceinline__ double hsum32d(double v) {
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off, 32);
  return v;
}
__device__ __forceinline__ float hmax32(float v) {
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 32));
  return v;
}
#endif
__device__ __forceinline__ float hsum32t(float v) { return hsum32(v); }
__device__ __forceinline__ double hsum32t(double v) { return hsum32d(v); }

// workgroup max of v[i] >= 0 for the non-NULL slots, one atomicMax per slot per workgroup (float bits
// order as unsigned for v >= 0) into the slot's counter for this block (kernels.h, kAmaxSub).
// Every thread of the block must call it.
// (`ext`, when given, is 48 floats of the caller's LDS to use instead of a static array: kernels whose
// one LDS array already takes the whole 160 KB.)
template <bool EXT = false>
__device__ __forceinline__ void amax_commit3(unsigned* s0, float v0, unsigned* s1, float v1, unsigned* s2, float v2,
                                             float (*ext)[16] = nullptr) {
  if (!s0 && !s1 && !s2) return;
  float(*red)[16];
  if constexpr (EXT) {
    red = ext;
  } else {
    __shared__ float red_own[3][16];
    red = red_own;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    v0 = fmaxf(v0, __shfl_xor(v0, off, 64));
    v1 = fmaxf(v1, __shfl_xor(v1, off, 64));
    v2 = fmaxf(v2, __shfl_xor(v2, off, 64));
  }
  const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wave] = v0;
    red[1][wave] = v1;
    red[2][wave] = v2;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    unsigned* slot = threadIdx.x == 0 ? s0 : (threadIdx.x == 1 ? s1 : s2);
    if (slot) {
      float m = 0.0f;
      for (int w = 0; w < nw; ++w) m = fmaxf(m, red[threadIdx.x][w]);
      const unsigned bid = blockIdx.x + blockIdx.y * 7919u + blockIdx.z * 104729u;
      if (m > 0.0f) atomicMax(slot + (bid % kAmaxSub) * kAmaxStride, __float_as_uint(m));
    }
  }
}

// ---------------------------------------------------------------------------
// element-wise epilogues (one accumulator element at (row, col))
// ---------------------------------------------------------------------------
template <int EPI>
__device__ __forceinline__ void epi_elem(const RowEpiArgs& e, int row, int col, bool real, float v) {
  const size_t idx = (size_t)row * e.ldo + col;
  if constexpr (EPI == (int)RowEpi::kTanh) {
    e.out0[idx] = real ? tanh_fast(v + e.bias[col]) : 0.0f;
  } else if constexpr (EPI == (int)RowEpi::kRHidden) {
    e.out0[idx] = real ? one_minus_sq(e.H[idx]) * (v + e.bias[col]) : 0.0f;
  } else if constexpr (EPI == (int)RowEpi::kRZ) {
    e.out0[idx] = real ? v + e.bias[col] : 0.0f;
  } else if constexpr (EPI == (int)RowEpi::kPrepBwd) {
    if (real) {
      const float h = e.H[idx];
      e.out0[idx] = v * one_minus_sq(h);
      e.out1[idx] = -2.0f * v * h;
    } else {
      e.out0[idx] = 0.0f;
      e.out1[idx] = 0.0f;
    }
  } else if constexpr (EPI == (int)RowEpi::kPrepBwdE) {
    e.out0[idx] = real ? -2.0f * v * e.H[idx] : 0.0f;
  } else if constexpr (EPI == (int)RowEpi::kPgBwd) {
    e.out0[idx] = real ? v * one_minus_sq(e.H[idx]) : 0.0f;
  } else if constexpr (EPI == (int)RowEpi::kRBwd) {
    e.out0[idx] = real ? fmaf(e.E[idx], e.RH[idx], v * one_minus_sq(e.H[idx])) : 0.0f;
  } else if constexpr (EPI == (int)RowEpi::kRelu) {
    e.out0[idx] = real ? fmaxf(v + e.bias[col], 0.0f) : 0.0f;
  } else if constexpr (EPI == (int)RowEpi::kReluBwd) {
    e.out0[idx] = (real && e.H[idx] > 0.0f) ? v : 0.0f;
  }
}

// value part (loads + math) and store part of the element-wise epilogues.
// No column predicate: padding columns (col >= N) have zero accumulators (zero
// weight padding), zero bias and zero H/E/RH padding, so every formula below
// already yields exactly 0 there.  Loads are therefore unconditional and hipcc
// keeps them all in flight (a `cond ? load : 0` becomes a branch per load).
template <int EPI>
__device__ __forceinline__ void epi_elem_v(const RowEpiArgs& e, size_t idx, bool /*real*/, float v, float bv,
                                           float& o0, float& o1) {
  if constexpr (EPI == (int)RowEpi::kTanh) {
    o0 = tanh_fast(v + bv);
  } else if constexpr (EPI == (int)RowEpi::kRHidden) {
    o0 = one_minus_sq(e.H[idx]) * (v + bv);
  } else if constexpr (EPI == (int)RowEpi::kRZ) {
    o0 = v + bv;
  } else if constexpr (EPI == (int)RowEpi::kPrepBwd) {
    const float h = e.H[idx];
    o0 = v * one_minus_sq(h);
    o1 = -2.0f * v * h;
  } else if constexpr (EPI == (int)RowEpi::kPrepBwdE) {
    o0 = -2.0f * v * e.H[idx];
  } else if constexpr (EPI == (int)RowEpi::kPgBwd) {
    o0 = v * one_minus_sq(e.H[idx]);
  } else if constexpr (EPI == (int)RowEpi::kRBwd) {
    o0 = fmaf(e.E[idx], e.RH[idx], v * one_minus_sq(e.H[idx]));
  } else if constexpr (EPI == (int)RowEpi::kRelu) {
    o0 = fmaxf(v + bv, 0.0f);
  } else if constexpr (EPI == (int)RowEpi::kReluBwd) {
    o0 = e.H[idx] > 0.0f ? v : 0.0f;
  }
}
template <int EPI>
__device__ __forceinline__ void epi_store(const RowEpiArgs& e, size_t idx, float o0, float o1) {
  e.out0[idx] = o0;
  if constexpr (EPI == (int)RowEpi::kPrepBwd) e.out1[idx] = o1;
}


// ---------------------------------------------------------------------------
// row-wise softmax-head epilogues.  The row's columns live on the 32 lanes of one wave half, TN
// per lane (col = 32 t + (lane & 31), t < TN): n_actions <= 32 TN.  Row reductions sum the TN
// values of a lane first, then xor-shuffle over the 32 lanes.
// ---------------------------------------------------------------------------
template <int EPI, int TN>
__device__ __forceinline__ void epi_row(const RowEpiArgs& e, int row, bool rowvalid, int lr, int A,
                                        const float (&v)[TN], float& m0, float& m1, float& m2) {
  // `row` is already clamped into [0, M); loads go to clamped (valid) addresses
  // unconditionally and are masked by selects, so hipcc keeps them in flight.
  bool real[TN];
  size_t idx[TN];
  bool st[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    const int col = 32 * t + lr;
    real[t] = col < A;
    const int colc = col < e.ldo ? col : e.ldo - 1;
    idx[t] = (size_t)row * e.ldo + colc;
    st[t] = rowvalid && col < e.ldo;
  }
  if constexpr (EPI == (int)RowEpi::kPrepHead || EPI == (int)RowEpi::kLossHead) {
    const int av = e.act[row];
    const float advv = e.adv[row];
    float z[TN], oldv[TN];
    float zm = -INFINITY;
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const float bias = e.bias[real[t] ? 32 * t + lr : 0];
      oldv[t] = e.old[idx[t]];
      // p = softmax(z)   (trpo_inksci.py:40)
      z[t] = real[t] ? v[t] + bias : -INFINITY;
      zm = fmaxf(zm, z[t]);
    }
    const float m = hmax32(zm);
    float ex[TN], es = 0.0f;
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      ex[t] = real[t] ? expf(z[t] - m) : 0.0f;
      es += ex[t];
    }
    const float ssum = hsum32(es);
    const int a = rowvalid ? av : 0;
    float p[TN], old[TN];
    float pa_l = 0.0f, olda_l = 0.0f;
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      p[t] = ex[t] / ssum;
      old[t] = (rowvalid && real[t]) ? oldv[t] : 0.0f;
      if (t == (a >> 5)) {
        pa_l = p[t];
        olda_l = old[t];
      }
    }
    const float pa = __shfl(pa_l, a & 31, 32);
    const float olda = __shfl(olda_l, a & 31, 32);
    const float adv = rowvalid ? advv : 0.0f;
    // row loss terms (:46-51)
#if TRPO_HEAD_LOG64
    double klp = 0.0, enp = 0.0;
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const double pd = p[t], od = old[t];
      klp += real[t] ? od * log((od + (double)kEps) / (pd + (double)kEps)) : 0.0;
      enp += real[t] ? -pd * log(pd + (double)kEps) : 0.0;
    }
    const double klt = hsum32d(klp);
    const double ent = hsum32d(enp);
#else
    // the reference's own precision (f32 tensors, trpo_inksci.py:50-51): f32 logs and f32 row sums of <= 32 TN
    // terms; the sums over rows are f64 (rowterms)
    float klp = 0.0f, enp = 0.0f;
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const float lk = logf((old[t] + kEps) / (p[t] + kEps)), le = logf(p[t] + kEps);
      klp += real[t] ? old[t] * lk : 0.0f;
      enp += real[t] ? -p[t] * le : 0.0f;
    }
    const double klt = hsum32(klp);
    const double ent = hsum32(enp);
#endif
    const double sur = rowvalid ? (double)pa / (double)olda * (double)adv : 0.0;
    if (rowvalid && lr == 0) {
      e.rowterms[4 * (size_t)row + 0] = sur;
      e.rowterms[4 * (size_t)row + 1] = klt;
      e.rowterms[4 * (size_t)row + 2] = ent;
      e.rowterms[4 * (size_t)row + 3] = 0.0;
    }
    if constexpr (EPI == (int)RowEpi::kPrepHead) {
      // KL_ff plain logit delta (:56-57), cancellation-free, in f32 (f64 took 40 % of this launch at C4; the
      // O(eps) terms it feeds reach Hv only through D and E, far below f32 rounding of Hv):
      //   d_j = (p_j/N) (B_j - sum_k p_k B_k),  B = eps/(p+eps)
#if TRPO_PREP_HEAD64
      typedef double T;
#else
      typedef float T;
#endif
      const T invN = (T)e.invN;
      T B[TN], spBp = 0, restp = 0;
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const T pd = p[t];
#if TRPO_PREP_HEAD64
        B[t] = real[t] ? (T)kEps / (pd + (T)kEps) : T(0);
#else
        B[t] = real[t] ? kEps * __builtin_amdgcn_rcpf(pd + kEps) : 0.0f;   // O(eps) term: 1-ulp v_rcp_f32
#endif
        spBp += pd * B[t];
        restp += (real[t] && 32 * t + lr != a) ? pd : T(0);
      }
      const T spB = hsum32t(spBp);
      const T rest = hsum32t(restp);   // 1 - p_a
      // surr logit delta (:54): -(adv/(N old_a)) p_a (1[j=a] - p_j)
      const T coef = -(T)adv * invN / (T)olda * (T)pa;
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const int col = 32 * t + lr;
        const T pd = p[t];
        const float dl = real[t] ? (float)(pd * invN * (B[t] - spB)) : 0.0f;
        const float ds = real[t] ? (float)(coef * (col == a ? rest : -pd)) : 0.0f;
        if (st[t]) {
          const size_t sidx = (size_t)row * e.ldo + col;
          e.out0[sidx] = real[t] ? p[t] : 0.0f;
          e.out1[sidx] = (float)dl;
          e.out2[sidx] = (float)ds;
          m1 = fmaxf(m1, fabsf((float)dl));
          m2 = fmaxf(m2, fabsf((float)ds));
        }
      }
    }
  } else if constexpr (EPI == (int)RowEpi::kRHead) {
    // R-softmax + R-reverse of the KL_ff head:
    //   Rp   = p (Rz - <p,Rz>)
    //   RD_j = (1/N)[Rp_j (B_j - sum p B) + Rp_j A_j^2 + p_j sum_k Rp_k A_k B_k]
    //   A = p/(p+eps), B = eps/(p+eps)
    double rz[TN], pd[TN], przp = 0.0;
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const float bias = e.bias[real[t] ? 32 * t + lr : 0];
      const float pv = e.P[idx[t]];
      rz[t] = real[t] ? (double)(v[t] + bias) : 0.0;
      pd[t] = (rowvalid && real[t]) ? (double)pv : 0.0;
      przp += pd[t] * rz[t];
    }
    const double prz = hsum32d(przp);
    double Rp[TN], Aa[TN], B[TN], spBp = 0.0, sRABp = 0.0;
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      Rp[t] = pd[t] * (rz[t] - prz);
      const double den = pd[t] + (double)kEps;
      Aa[t] = real[t] ? pd[t] / den : 0.0;
      B[t] = real[t] ? (double)kEps / den : 0.0;
      spBp += pd[t] * B[t];
      sRABp += Rp[t] * Aa[t] * B[t];
    }
    const double spB = hsum32d(spBp);
    const double sRAB = hsum32d(sRABp);
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const double rd = e.invN * (Rp[t] * (B[t] - spB) + Rp[t] * Aa[t] * Aa[t] + pd[t] * sRAB);
      if (st[t]) {
        e.out0[(size_t)row * e.ldo + 32 * t + lr] = real[t] ? (float)rd : 0.0f;
        if (real[t]) m0 = fmaxf(m0, fabsf((float)rd));
      }
    }
  }
}

// Linear block id -> (m-tile, n-tile).  The n-tiles of one row tile are adjacent in
// the swizzled order and land on one XCD (blocks b and b+8 share an XCD under the
// observed round-robin dispatch: speed only, never correctness), so the second
// n-tile re-reads the A rows from that XCD's L2.
__device__ __forceinline__ void tile_of(int ntn, int& mt, int& nt) {
  const int id = blockIdx.x, nwg = gridDim.x;
  int swz = id;
  if ((nwg & 7) == 0) swz = (id & 7) * (nwg >> 3) + (id >> 3);
  mt = swz / ntn;
  nt = swz - mt * ntn;
}

// Full-width tile of the element-wise epilogues: every epilogue operand goes through a per-block buffer
// descriptor (base = row m0, num_records = the rows this tile owns), so a load/store is one buffer op with
// a lane-constant voffset and a per-row SGPR soffset; rows past M fall outside the descriptor (loads read
// 0, stores are dropped) -- no per-element predicate, no 64-bit address math, and all 16 loads of a chunk
// stay in flight.
template <int WM, int WN, int TM, int TN, int EPI>
__device__ __forceinline__ void row_epi_full(const RowGemmArgs& args, f32x16 (&acc)[TM][TN], int m0, int n0, int wm,
                                             int wn, int lr, int lh, float& mx0, float& mx1) {
  constexpr int BM = WM * TM * 32;
  const int M = args.M;
  const RowEpiArgs& e = args.ea;
  const int ldo = e.ldo;
  const int Mt = M - m0 < BM ? M - m0 : BM;
  const int tile_bytes = Mt * ldo * 4;
  auto mk = [&](const float* ptr) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(ptr + (size_t)m0 * ldo), 0, tile_bytes, 0x00020000);
  };
  constexpr bool kUsesH = EPI == (int)RowEpi::kRHidden || EPI == (int)RowEpi::kPrepBwd ||
                          EPI == (int)RowEpi::kPrepBwdE || EPI == (int)RowEpi::kPgBwd ||
                          EPI == (int)RowEpi::kRBwd || EPI == (int)RowEpi::kReluBwd;
  constexpr bool kRB = EPI == (int)RowEpi::kRBwd;
  constexpr bool kPB = EPI == (int)RowEpi::kPrepBwd;
  constexpr bool kPE = EPI == (int)RowEpi::kPrepBwdE;
  // descriptors of operands an epilogue does not use alias out0 and are never touched
  const __amdgpu_buffer_rsrc_t rO0 = mk(e.out0);
  const __amdgpu_buffer_rsrc_t rH = mk(kUsesH ? e.H : e.out0);
  const __amdgpu_buffer_rsrc_t rE = mk(kRB ? e.E : e.out0);
  const __amdgpu_buffer_rsrc_t rRH = mk(kRB ? e.RH : e.out0);
  const __amdgpu_buffer_rsrc_t rO1 = mk(kPB ? e.out1 : e.out0);
  const int vbase = ((wm * TM * 32 + 4 * lh) * ldo + n0 + wn * TN * 32 + lr) * 4;
  auto ld = [&](__amdgpu_buffer_rsrc_t r, int vo, int so) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
  };
  auto st = [&](float v, __amdgpu_buffer_rsrc_t r, int vo, int so) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, vo, so, 0);
  };
  // Operand loads run one (tm, tn) chunk ahead of the chunk being computed and stored: the
  // chunk's loads are issued before the previous chunk's stores in program order (hipcc cannot
  // prove the descriptors disjoint, so it would not hoist them itself), which leaves one chunk
  // of loads in flight behind every chunk of math instead of a full round trip per chunk.
  constexpr int NL = kRB ? 3 : (kUsesH ? 1 : 0);
  constexpr int NCH = TM * TN;
  float pre[2][NL > 0 ? NL : 1][16];
  auto load_chunk = [&](int c, float (&dst)[NL > 0 ? NL : 1][16]) {
    if constexpr (NL > 0) {
      const int tn = c / TM, tm = c % TM;
      const int vo = vbase + tn * 128;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int so = (tm * 32 + (r & 3) + 8 * (r >> 2)) * ldo * 4;
        dst[0][r] = ld(rH, vo, so);
        if constexpr (NL == 3) {
          dst[1][r] = ld(rE, vo, so);
          dst[2][r] = ld(rRH, vo, so);
        }
      }
    }
  };
  if constexpr (TRPO_EPI_PIPE) load_chunk(0, pre[0]);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int tn = c / TM, tm = c % TM;
    const int col = n0 + wn * TN * 32 + tn * 32 + lr;
    float bv = 0.0f;
    if constexpr (EPI == (int)RowEpi::kTanh || EPI == (int)RowEpi::kRHidden || EPI == (int)RowEpi::kRelu ||
                  EPI == (int)RowEpi::kRZ)
      bv = e.bias[col < args.N ? col : 0] * (col < args.N ? 1.0f : 0.0f);
    const int vo = vbase + tn * 128;
    if constexpr (TRPO_EPI_PIPE) {
      if (c + 1 < NCH) load_chunk(c + 1, pre[(c + 1) & 1]);
    } else {
      load_chunk(c, pre[c & 1]);
    }
    const float (&op)[NL > 0 ? NL : 1][16] = pre[c & 1];
    {
      float o0[16], o1[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = acc[tm][tn][r];
        if constexpr (EPI == (int)RowEpi::kTanh) {
          o0[r] = tanh_fast(v + bv);
        } else if constexpr (EPI == (int)RowEpi::kRHidden) {
          o0[r] = one_minus_sq(op[0][r]) * (v + bv);
        } else if constexpr (EPI == (int)RowEpi::kRZ) {
          o0[r] = v + bv;
        } else if constexpr (kPB) {
          const float h = op[0][r];
          o0[r] = v * one_minus_sq(h);
          o1[r] = -2.0f * v * h;
        } else if constexpr (kPE) {
          o0[r] = -2.0f * v * op[0][r];
        } else if constexpr (EPI == (int)RowEpi::kPgBwd) {
          o0[r] = v * one_minus_sq(op[0][r]);
        } else if constexpr (EPI == (int)RowEpi::kRelu) {
          o0[r] = fmaxf(v + bv, 0.0f);
        } else if constexpr (EPI == (int)RowEpi::kReluBwd) {
          o0[r] = op[0][r] > 0.0f ? v : 0.0f;
        } else {
          o0[r] = fmaf(op[1][r], op[2][r], v * one_minus_sq(op[0][r]));
        }
        // running max for the f16 operand scales (rows past M -- dropped stores -- hold 0 or,
        // for kRHidden, the tangent bias: harmless in a max)
        if constexpr (TRPO_EPI_TRACK && EPI != (int)RowEpi::kTanh && EPI != (int)RowEpi::kRelu &&
                      EPI != (int)RowEpi::kReluBwd && EPI != (int)RowEpi::kPrepBwdE) {
          mx0 = fmaxf(mx0, fabsf(o0[r]));
          if constexpr (kPB) mx1 = fmaxf(mx1, fabsf(o1[r]));
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int so = (tm * 32 + (r & 3) + 8 * (r >> 2)) * ldo * 4;
        st(o0[r], rO0, vo, so);
        if constexpr (kPB) st(o1[r], rO1, vo, so);
      }
    }
  }
}

// Fused epilogue of a row-GEMM tile.  The accumulator layout (col = lane&31,
// row = (r&3) + 8(r>>2) + 4(lane>>5)) is the same for the f32 (32x32x2) and the
// bf16 (32x32x16) MFMA, so both row-GEMM kernels share it.
template <int WM, int WN, int TM, int TN, int EPI, bool EXT_RED = false>
__device__ __forceinline__ void row_epilogue(const RowGemmArgs& args, f32x16 (&acc)[TM][TN], int m0, int n0,
                                             int wm, int wn, int lr, int lh, float (*red)[16] = nullptr) {
  constexpr int BN = WN * TN * 32;
  const int M = args.M;
  const RowEpiArgs& e = args.ea;
  float mx0 = 0.0f, mx1 = 0.0f, mx2 = 0.0f;   // max |stored output| for the f16 operand scales
  if constexpr (epi_is_head(EPI)) {
    static_assert(WN == 1, "row-wise head epilogue needs the whole row in one wave half");
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * TM * 32 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        float v[TN];
#pragma unroll
        for (int t = 0; t < TN; ++t) v[t] = acc[tm][t][r];
        epi_row<EPI, TN>(e, row < M ? row : 0, row < M, lr, args.N, v, mx0, mx1, mx2);
      }
  } else {
    const bool fulln = (n0 + BN <= args.Npad);
    if (fulln) {
      row_epi_full<WM, WN, TM, TN, EPI>(args, acc, m0, n0, wm, wn, lr, lh, mx0, mx1);
    } else {
      // partial-width tile (odd layer widths): predicated path
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int col = n0 + wn * TN * 32 + tn * 32 + lr;
        const bool real = col < args.N;
        const bool colv = col < args.Npad;
        const int colc = colv ? col : 0;
        float bv = 0.0f;
        if constexpr (EPI == (int)RowEpi::kTanh || EPI == (int)RowEpi::kRHidden || EPI == (int)RowEpi::kRelu ||
                      EPI == (int)RowEpi::kRZ)
          bv = e.bias[real ? col : 0];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = m0 + wm * TM * 32 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (row < M && colv) {
              float o0, o1 = 0.0f;
              epi_elem_v<EPI>(e, (size_t)row * e.ldo + colc, real, acc[tm][tn][r], real ? bv : 0.0f, o0, o1);
              epi_store<EPI>(e, (size_t)row * e.ldo + col, o0, o1);
              mx0 = fmaxf(mx0, fabsf(o0));
              mx1 = fmaxf(mx1, fabsf(o1));
            }
          }
      }
    }
  }
  amax_commit3<EXT_RED>(e.amax0, mx0, e.amax1, mx1, e.amax2, mx2, red);
}

// ---------------------------------------------------------------------------
// Split-bf16 row GEMM.  CDNA4 has no reduced-precision f32 MFMA, but bf16 MFMA
// runs at 16x the f32 rate.  Each f32 operand x is split exactly into three
// bf16 pieces x = h + m + l + O(2^-27 |x|) (h = bf16(x), m = bf16(x - h),
// l = bf16(x - h - m); both differences are exact in f32) and
//     a*b ~= ah bh + (ah bm + am bh) + (ah bl + al bh + am bm)
// keeps every product term down to 2^-18 relative; the dropped ones (am bl,
// al bm, al bl) are < 2^-26 relative, below the f32 rounding of the sum.  The
// pieces' products are exact in the MFMA's f32 accumulation, so the result
// matches an f32 GEMM to f32 rounding at 16/6 = 2.7x its MFMA peak.
//
// A (activations, f32 in HBM) is split while staging global -> LDS; B (packed
// weights) is pre-split by split_b_kernel into [3][Npad][ldk] planes.
// v_mfma_f32_32x32x16_bf16: lane l (r = l&31, h = l>>5) holds A[r][8h..8h+7]
// and B[8h..8h+7][col r] - one ds_read_b128 per plane from [row][k] images.
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned short bf16_bits(float x) {
  return __builtin_bit_cast(unsigned short, (__bf16)x);
}
__device__ __forceinline__ float bf16_val(unsigned short b) {
  return __builtin_bit_cast(float, (unsigned)b << 16);
}
__device__ __forceinline__ void split3(float x, unsigned short& h, unsigned short& m, unsigned short& l) {
  h = bf16_bits(x);
  const float r1 = x - bf16_val(h);
  m = bf16_bits(r1);
  const float r2 = r1 - bf16_val(m);
  l = bf16_bits(r2);
}

// f16 split (RowGemmArgs::f16): x (already scaled into [2^11, 2^12) by a power of two, see
// f16_scale_exp) = h + l + O(2^-22 |x|) with h = f16(x), l = f16(x - h) (the difference is exact);
// a*b ~= ah bh + (ah bl + al bh), the dropped al bl is ~2^-22 relative.  f16 MFMA runs at the bf16
// rate, so 3 products instead of 6 halve the MFMA work; the scales keep every piece a normal f16
// down to 2^-15 of the operand's max (below that the error is absolute, 2^-36 of the max).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split2h(float x, unsigned short& h, unsigned short& l) {
  const _Float16 hh = (_Float16)x;
  const _Float16 ll = (_Float16)(x - (float)hh);
  h = __builtin_bit_cast(unsigned short, hh);
  l = __builtin_bit_cast(unsigned short, ll);
}
// the slot's max (over its kAmaxSub counters, kAmaxSub / 64 per lane) -> scale exponent; all lanes of
// the wave must call it
__device__ __forceinline__ int amax_exp(const unsigned* amax) {
  if (!amax) return f16_scale_exp(1.0f);
  const int lane = threadIdx.x & 63;
  float v = 0.0f;
#pragma unroll
  for (int i = 0; i < kAmaxSub / 64; ++i) v = fmaxf(v, __uint_as_float(amax[(lane + 64 * i) * kAmaxStride]));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return f16_scale_exp(v);
}
template <int TM, int TN>
__device__ __forceinline__ void scale_acc(f32x16 (&acc)[TM][TN], int e) {
  if (e == 0) return;
  const float f = __builtin_ldexpf(1.0f, e);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] *= f;
}

// LDS images are [row][16 k] bf16 (32-B rows, no padding); the two 16-B k-chunks of
// a row swap places where bit 2 ^ bit 3 of the row is set.
// (The flip bit is bit 2 ^ bit 3 of the row: the ds_read_b128 fragment reads, serviced in the lane groups
// {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32), put their 16 rows on 16 distinct 16-B bank slots, and so do the
// weight-gradient staging stores -- ds_write_b128, 8 lanes per LDS cycle on 32 banks, 8 consecutive rows of one
// chunk -- which a bit-3-only flip left 2-way conflicted, rows r and r+4 on the same banks.)
__device__ __forceinline__ int swz16(int row, int chunk) {
  return row * 16 + ((chunk ^ (((row >> 2) ^ (row >> 3)) & 1)) << 3);
}

// One global_load_lds_dwordx4 as inline asm: 16 B per lane from `src` into LDS at the wave-uniform
// byte address `lds` + 16 * lane.  Opaque to hipcc's s_waitcnt bookkeeping (the builtin form makes
// hipcc drain vmcnt(0) before every later LDS read), so the caller counts completion itself.
__device__ __forceinline__ void glds16(const void* src, const void* lds) {
  unsigned keep;
  const unsigned dst = (unsigned)(uintptr_t)lds;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(dst))
               : "memory");
}

}  // namespace
}  // namespace trpo
