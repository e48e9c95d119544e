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
#include <stdexcept>
#include <string>

namespace trpo {

namespace {

constexpr int BK = 16;

__device__ __forceinline__ float one_minus_sq(float h) { return (1.0f - h) * (1.0f + h); }

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

// ---------------------------------------------------------------------------
// element-wise epilogues (one accumulator element at (row, col))
// ---------------------------------------------------------------------------
template <int EPI>
__device__ __forceinline__ void epi_elem(const RowEpiArgs& e, int row, int col, bool real, float v) {
  const size_t idx = (size_t)row * e.ldo + col;
  if constexpr (EPI == (int)RowEpi::kTanh) {
    e.out0[idx] = real ? tanhf(v + e.bias[col]) : 0.0f;
  } else if constexpr (EPI == (int)RowEpi::kRHidden) {
    e.out0[idx] = real ? one_minus_sq(e.H[idx]) * (v + e.bias[col]) : 0.0f;
  } else if constexpr (EPI == (int)RowEpi::kPrepBwd) {
    if (real) {
      const float h = e.H[idx];
      e.out0[idx] = v * one_minus_sq(h);
      e.out1[idx] = -2.0f * v * h;
    } else {
      e.out0[idx] = 0.0f;
      e.out1[idx] = 0.0f;
    }
  } else if constexpr (EPI == (int)RowEpi::kPgBwd) {
    e.out0[idx] = real ? v * one_minus_sq(e.H[idx]) : 0.0f;
  } else if constexpr (EPI == (int)RowEpi::kRBwd) {
    e.out0[idx] = real ? fmaf(e.E[idx], e.RH[idx], v * one_minus_sq(e.H[idx])) : 0.0f;
  }
}

// ---------------------------------------------------------------------------
// row-wise softmax-head epilogues.  The 32 columns of one row live on the 32
// lanes of one wave half (col = lane & 31); reductions are xor-shuffles of
// width 32.  Requires n_actions <= 32.
// ---------------------------------------------------------------------------
template <int EPI>
__device__ __forceinline__ void epi_row(const RowEpiArgs& e, int row, bool rowvalid, int col, int A,
                                        float v) {
  const bool real = col < A;
  const size_t idx = (size_t)row * e.ldo + col;
  const bool st = rowvalid && col < e.ldo;
  if constexpr (EPI == (int)RowEpi::kPrepHead || EPI == (int)RowEpi::kLossHead) {
    // p = softmax(z)   (trpo_inksci.py:40)
    const float z = real ? v + e.bias[col] : -INFINITY;
    const float m = hmax32(z);
    const float ex = real ? expf(z - m) : 0.0f;
    const float ssum = hsum32(ex);
    const float p = ex / ssum;
    const int a = rowvalid ? e.act[row] : 0;
    const float old = (rowvalid && real) ? e.old[idx] : 0.0f;
    const float pa = __shfl(p, a, 32);
    const float olda = __shfl(old, a, 32);
    const float adv = rowvalid ? e.adv[row] : 0.0f;
    const double pd = p, od = old;
    // row loss terms (:46-51), accumulated in f64
    const double klt = hsum32d(real ? od * log((od + (double)kEps) / (pd + (double)kEps)) : 0.0);
    const double ent = hsum32d(real ? -pd * log(pd + (double)kEps) : 0.0);
    const double sur = rowvalid ? (double)pa / (double)olda * (double)adv : 0.0;
    if (rowvalid && col == 0) {
      e.rowterms[4 * (size_t)row + 0] = sur;
      e.rowterms[4 * (size_t)row + 1] = klt;
      e.rowterms[4 * (size_t)row + 2] = ent;
      e.rowterms[4 * (size_t)row + 3] = 0.0;
    }
    if constexpr (EPI == (int)RowEpi::kPrepHead) {
      if (st) e.out0[idx] = real ? p : 0.0f;
      // KL_ff plain logit delta (:56-57), cancellation-free:
      //   d_j = (p_j/N) (B_j - sum_k p_k B_k),  B = eps/(p+eps)
      const double B = real ? (double)kEps / (pd + (double)kEps) : 0.0;
      const double spB = hsum32d(pd * B);
      const double dl = real ? pd * e.invN * (B - spB) : 0.0;
      // surr logit delta (:54): -(adv/(N old_a)) p_a (1[j=a] - p_j)
      const double rest = hsum32d((real && col != a) ? pd : 0.0);  // 1 - p_a
      const double coef = -(double)adv * e.invN / (double)olda * (double)pa;
      const double ds = real ? coef * (col == a ? rest : -pd) : 0.0;
      if (st) {
        e.out1[idx] = (float)dl;
        e.out2[idx] = (float)ds;
      }
    }
  } else if constexpr (EPI == (int)RowEpi::kRHead) {
    // R-softmax + R-reverse of the KL_ff head:
    //   Rp   = p (Rz - <p,Rz>)
    //   RD_j = (1/N)[Rp_j (B_j - sum p B) + Rp_j A_j^2 + p_j sum_k Rp_k A_k B_k]
    //   A = p/(p+eps), B = eps/(p+eps)
    const double rz = real ? (double)(v + e.bias[col]) : 0.0;
    const double pd = (rowvalid && real) ? (double)e.P[idx] : 0.0;
    const double prz = hsum32d(pd * rz);
    const double Rp = pd * (rz - prz);
    const double den = pd + (double)kEps;
    const double Aa = real ? pd / den : 0.0;
    const double B = real ? (double)kEps / den : 0.0;
    const double spB = hsum32d(pd * B);
    const double sRAB = hsum32d(Rp * Aa * B);
    const double rd = e.invN * (Rp * (B - spB) + Rp * Aa * Aa + pd * sRAB);
    if (st) e.out0[idx] = real ? (float)rd : 0.0f;
  }
}

template <int WM, int WN, int TM, int TN, int EPI>
__global__ void __launch_bounds__(WM* WN * 64)
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
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
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
  f32x4 ra[AP], rb[BP];

  auto gload = [&](int t) {
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
      f32x4 v = f32x4{};
      if ((AF4 % NT == 0 || f < AF4) && row < M && k < K)
        v = *reinterpret_cast<const f32x4*>(Ap + (size_t)row * lda + k);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const int f = tid + i * NT;
      const int kr = f / (BN / 4), cq = f % (BN / 4);
      const int k = k0 + kr, col = n0 + 4 * cq;
      f32x4 v = f32x4{};
      if ((BF4 % NT == 0 || f < BF4) && k < K && col < args.Npad)
        v = *reinterpret_cast<const f32x4*>(Bp + (size_t)k * ldb + col);
      rb[i] = v;
    }
  };
  auto sstore = [&](int buf) {
    float* As = smem + buf * (ASZ + BSZ);
    float* Bs = As + ASZ;
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int f = tid + i * NT;
      if (AF4 % NT == 0 || f < AF4) {
        const int r = f / (BK / 4), kq = f % (BK / 4);
        *reinterpret_cast<f32x4*>(As + r * LDA + 4 * kq) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const int f = tid + i * NT;
      if (BF4 % NT == 0 || f < BF4) {
        const int kr = f / (BN / 4), cq = f % (BN / 4);
        *reinterpret_cast<f32x4*>(Bs + kr * LDB + 4 * cq) = rb[i];
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
    gload(0);
    sstore(0);
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
      if (t + 1 < ntiles) gload(t + 1);
      compute(t & 1);
      if (t + 1 < ntiles) sstore((t + 1) & 1);
      __syncthreads();
    }
  }

  // ---- epilogue -----------------------------------------------------------
  const RowEpiArgs& e = args.ea;
  if constexpr (EPI >= (int)RowEpi::kPrepHead) {
    static_assert(WN == 1 && TN == 1, "row-wise head epilogue needs the whole row in one wave half");
    const int col = n0 + lr;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * TM * 32 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        epi_row<EPI>(e, row < M ? row : 0, row < M, col, args.N, acc[tm][0][r]);
      }
  } else {
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int col = n0 + wn * TN * 32 + tn * 32 + lr;
        if (col >= args.Npad) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * TM * 32 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (row < M) epi_elem<EPI>(e, row, col, col < args.N, acc[tm][tn][r]);
        }
      }
  }
}

// ---------------------------------------------------------------------------
// weight-gradient kernel: k = rows (split-K), tiles [BK][BM] / [BK][BN] k-major
// ---------------------------------------------------------------------------
template <int WM, int WN, int TM, int TN>
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
  f32x4 ra[AP], rb[BP];

  auto gload = [&](int t) {
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
      f32x4 v = f32x4{};
      if ((AF4 % NT == 0 || f < AF4) && r < r1 && c < args.Mpad)
        v = *reinterpret_cast<const f32x4*>(Ap + (size_t)r * lda + c);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const int f = tid + i * NT;
      const int kr = f / (BN / 4), cq = f % (BN / 4);
      const int r = rb0 + kr, c = n0 + 4 * cq;
      f32x4 v = f32x4{};
      if ((BF4 % NT == 0 || f < BF4) && r < r1 && c < args.Npad)
        v = *reinterpret_cast<const f32x4*>(Bp + (size_t)r * ldb + c);
      rb[i] = v;
    }
  };
  auto sstore = [&](int buf) {
    float* As = smem + buf * (ASZ + BSZ);
    float* Bs = As + ASZ;
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int f = tid + i * NT;
      if (AF4 % NT == 0 || f < AF4) {
        const int kr = f / (BM / 4), cq = f % (BM / 4);
        *reinterpret_cast<f32x4*>(As + kr * LDA + 4 * cq) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const int f = tid + i * NT;
      if (BF4 % NT == 0 || f < BF4) {
        const int kr = f / (BN / 4), cq = f % (BN / 4);
        *reinterpret_cast<f32x4*>(Bs + kr * LDB + 4 * cq) = rb[i];
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

  if (ntiles > 0) {
    gload(0);
    sstore(0);
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
      if (t + 1 < ntiles) gload(t + 1);
      compute(t & 1, do_colsum && (t / nk) == args.colsum_seg);
      if (t + 1 < ntiles) sstore((t + 1) & 1);
      __syncthreads();
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

template <int WM, int WN, int TM, int TN, int EPI>
void launch_row_cfg(const RowGemmArgs& a, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  dim3 grid((a.M + BM - 1) / BM, (a.Npad + BN - 1) / BN);
  hipLaunchKernelGGL((rowgemm_kernel<WM, WN, TM, TN, EPI>), grid, dim3(WM * WN * 64), 0, s, a);
}

template <int EPI>
void launch_row_epi(const RowGemmArgs& a, hipStream_t s) {
  if constexpr (EPI >= (int)RowEpi::kPrepHead) {
    if (a.N > 32) throw std::runtime_error("softmax head supports at most 32 actions");
    launch_row_cfg<4, 1, 2, 1, EPI>(a, s);
  } else {
    if (a.Npad <= 32) launch_row_cfg<4, 1, 2, 1, EPI>(a, s);
    else if (a.Npad <= 64) launch_row_cfg<4, 1, 2, 2, EPI>(a, s);
    else if (a.Npad <= 128) launch_row_cfg<2, 2, 2, 2, EPI>(a, s);
    else launch_row_cfg<2, 4, 2, 2, EPI>(a, s);
  }
}

template <int WM, int WN, int TM, int TN>
void launch_wg_cfg(const WGradArgs& a, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  dim3 grid((a.Ma + BM - 1) / BM, (a.Nb + BN - 1) / BN, a.splits);
  hipLaunchKernelGGL((wgrad_kernel<WM, WN, TM, TN>), grid, dim3(WM * WN * 64), 0, s, a);
}

}  // namespace

void launch_rowgemm(const RowGemmArgs& a, hipStream_t s) {
  if (a.M <= 0) return;
  switch (a.epi) {
    case RowEpi::kTanh: launch_row_epi<(int)RowEpi::kTanh>(a, s); break;
    case RowEpi::kRHidden: launch_row_epi<(int)RowEpi::kRHidden>(a, s); break;
    case RowEpi::kPrepBwd: launch_row_epi<(int)RowEpi::kPrepBwd>(a, s); break;
    case RowEpi::kPgBwd: launch_row_epi<(int)RowEpi::kPgBwd>(a, s); break;
    case RowEpi::kRBwd: launch_row_epi<(int)RowEpi::kRBwd>(a, s); break;
    case RowEpi::kPrepHead: launch_row_epi<(int)RowEpi::kPrepHead>(a, s); break;
    case RowEpi::kLossHead: launch_row_epi<(int)RowEpi::kLossHead>(a, s); break;
    case RowEpi::kRHead: launch_row_epi<(int)RowEpi::kRHead>(a, s); break;
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
  } else {
    if (Mp <= 128) launch_wg_cfg<2, 4, 2, 2>(a, s);         // 128 x 256
    else launch_wg_cfg<2, 4, 4, 2>(a, s);                   // 256 x 256
  }
}

}  // namespace trpo
