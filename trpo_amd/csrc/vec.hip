// Vector / scalar kernels of the TRPO update engine: weight packing, slab
// reduction, the device-resident conjugate gradient (utils.py:185-201), step
// scaling (trpo_inksci.py:147-151), loss reduction (trpo_inksci.py:44-53) and
// the backtracking line search (utils.py:170-182 with trpo_inksci.py:127-129,
// 153-158).
//
// All reductions are deterministic: kRedBlocks fixed per-block partials in
// f64, summed in index order by whoever consumes them (every block of the
// consumer recomputes the same sum, so no inter-block hand-off is needed).
// Every scalar the reference keeps in float32 (rdotr, alpha, mu, losses) is
// rounded to float32 at the same point; the float64 scalars of the reference's
// NumPy-1.x promotion rules (shs, lm, expected-improve rate, line-search ratio)
// stay float64.
#include "common.h"
#include "kernels.h"

#include <stdexcept>

#pragma clang fp contract(off)

namespace trpo {

namespace {

// wave max of v >= 0 -> one atomicMax per wave (float bits order as unsigned for v >= 0)
__device__ __forceinline__ void amax_wave_commit(unsigned* slot, float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  const unsigned wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6) + blockIdx.y * 7919u;
  if ((threadIdx.x & 63) == 0 && v > 0.0f) atomicMax(slot + (wid % kAmaxSub) * kAmaxStride, __float_as_uint(v));
  // (few blocks: per-wave atomics are fine here)
}

__global__ void pack_kernel(const PackArgs pa, const float* src, int which, const int* skip) {
  if (skip && *skip) return;
  const LayerPack& L = pa.L[blockIdx.y];
  const int64_t n = (int64_t)L.a * L.b;
  const float* w = src + L.off_w;
  float mx = 0.0f;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / L.b), j = (int)(e % L.b);
    const float v = w[e];
    mx = fmaxf(mx, fabsf(v));
    L.WF[(int64_t)(which ? L.apad + i : i) * L.bpad + j] = v;
    if (L.WB) L.WB[(int64_t)(which ? L.bpad + j : j) * L.apad + i] = v;
  }
  if (L.amax) amax_wave_commit(L.amax, mx);
}

__global__ void amax_kernel(const float* A, int64_t n, int w, int ld, unsigned* out) {
  float mx = 0.0f;
  const int64_t tot = n * w;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / w;
    const int c = (int)(e - r * w);
    mx = fmaxf(mx, fabsf(A[r * ld + c]));
  }
  amax_wave_commit(out, mx);
}

// Sum of the S split-K slabs.  A block owns 64 consecutive parameters (one 256-B row segment per
// wave-load) and spreads the S slabs over 16 wave groups, each with 4 independent accumulators, so a
// launch has P/64 x 1024 threads with several loads in flight each (one thread per parameter and a
// serial S-long chain was latency-bound: 0.2 ms for 512 slabs).
// PZ: the CG's next step fused in (single rank: Hv needs no all-reduce in between): z = Hv + damping p and the
// block's p.z partial (cg_pz_kernel), partials past the last block zeroed so that cg_xr_kernel's fixed-length sum
// holds
constexpr int kRsCols = 64, kRsGroups = 16;
template <bool PZ>
__global__ void __launch_bounds__(kRsCols* kRsGroups)
reduce_slab_kernel(const float* slab, int S, int64_t stride, int64_t P, float* out, const int* skip,
                   const float* pv = nullptr, float* z = nullptr, const UpdScalars* sc = nullptr,
                   double* partials = nullptr) {
  __shared__ float red[kRsGroups][kRsCols + 1];
  if (skip && *skip) return;
  const int c = threadIdx.x % kRsCols, g = threadIdx.x / kRsCols;
  const int64_t p = (int64_t)blockIdx.x * kRsCols + c;
  float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
  if (p < P) {
    constexpr int G = kRsGroups;
    int s = g;
    for (; s + 3 * G < S; s += 4 * G) {
      a0 += slab[(int64_t)s * stride + p];
      a1 += slab[(int64_t)(s + G) * stride + p];
      a2 += slab[(int64_t)(s + 2 * G) * stride + p];
      a3 += slab[(int64_t)(s + 3 * G) * stride + p];
    }
    for (; s < S; s += G) a0 += slab[(int64_t)s * stride + p];
  }
  red[g][c] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (g == 0 && p < P) {
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < kRsGroups; ++i) acc += red[i][c];
    out[p] = acc;
  }
  if constexpr (PZ) {
    if (g == 0) {   // wave 0: the block's 64 parameters
      double v = 0.0;
      if (p < P) {
        const float damp = sc->damping, pi = pv[p], hv = out[p];
        const float zi = damp != 0.0f ? hv + damp * pi : hv;
        z[p] = zi;
        v = (double)pi * (double)zi;
      }
      v = wave_sum_d(v);
      // the fixed-length partial layout holds kRedBlocks blocks (P <= kRedBlocks x 64, engine.cpp
      // cg_fused_reduce_ok): a larger grid would write past it, so its extra blocks drop their partial (and the
      // host refuses such a launch)
      if (c == 0 && blockIdx.x < kRedBlocks) partials[blockIdx.x] = v;
    }
    if (blockIdx.x == 0)
      for (int i = (int)gridDim.x + threadIdx.x; i < kRedBlocks; i += blockDim.x) partials[i] = 0.0;
  }
}

__global__ void dot_partials_kernel(const float* a, const float* b, int64_t n, double* partials,
                                    const int* skip) {
  __shared__ double scratch[kRedThreads / 64];
  if (skip && *skip) return;
  double v = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    v += (double)a[i] * (double)b[i];
  v = block_sum_d(v, scratch);
  if (threadIdx.x == 0) partials[blockIdx.x] = v;
}

// utils.py:186-189
template <class T>
__global__ void cg_init_kernel(const T* b, T* x, T* r, T* p, int64_t n, double* partials) {
  __shared__ double scratch[kRedThreads / 64];
  double v = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const T bi = b[i];
    x[i] = T(0);
    r[i] = bi;
    p[i] = bi;
    v += (double)bi * (double)bi;
  }
  v = block_sum_d(v, scratch);
  if (threadIdx.x == 0) partials[blockIdx.x] = v;
}

template <class T, class S>
__global__ void cg_init_finish_kernel(const double* partials, S* sc, CGFlags* fl, double tol,
                                      double damping) {
  __shared__ double scratch[kRedThreads / 64];
  const double rr = sum_partials(partials, kRedBlocks, scratch);
  for (int i = threadIdx.x; i < kMaxCG + 2; i += blockDim.x) fl->done[i] = 0;
  if (threadIdx.x == 0) {
    sc->rdotr[0] = (T)rr;
    sc->iters = 0;
    sc->tol = (T)tol;
    sc->damping = (T)damping;
  }
}

// z = fvp(p) + cg_damping * p   (trpo_inksci.py:126) ; partials = p.z (utils.py:192)
template <class T, class S>
__global__ void cg_pz_kernel(const T* hv, const T* p, T* z, int64_t n, const S* sc,
                             double* partials, const int* skip) {
  __shared__ double scratch[kRedThreads / 64];
  if (skip && *skip) return;
  const T damp = sc->damping;
  double v = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const T pi = p[i];
    const T zi = damp != T(0) ? hv[i] + damp * pi : hv[i];
    z[i] = zi;
    v += (double)pi * (double)zi;
  }
  v = block_sum_d(v, scratch);
  if (threadIdx.x == 0) partials[blockIdx.x] = v;
}

// utils.py:192-195
template <class T, class S>
__global__ void cg_xr_kernel(T* x, T* r, const T* p, const T* z, int64_t n, S* sc,
                             const double* partials, double* partials2, int it, const int* skip) {
  __shared__ double scratch[kRedThreads / 64];
  if (skip && *skip) return;
  const T pz = (T)sum_partials(partials, kRedBlocks, scratch);
  const T alpha = sc->rdotr[it & 1] / pz;
  double v = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    x[i] = x[i] + alpha * p[i];
    const T ri = r[i] - alpha * z[i];
    r[i] = ri;
    v += (double)ri * (double)ri;
  }
  v = block_sum_d(v, scratch);
  if (threadIdx.x == 0) partials2[blockIdx.x] = v;
  if (blockIdx.x == 0 && threadIdx.x == 0) sc->alpha = alpha;
}

// utils.py:195-200
template <class T, class S>
__global__ void cg_p_kernel(const T* r, T* p, int64_t n, S* sc, const double* partials2, CGFlags* fl,
                            int it) {
  __shared__ double scratch[kRedThreads / 64];
  if (fl->done[it]) {
    if (blockIdx.x == 0 && threadIdx.x == 0) fl->done[it + 1] = 1;
    return;
  }
  const T newrdotr = (T)sum_partials(partials2, kRedBlocks, scratch);
  const T rdotr = sc->rdotr[it & 1];
  const T mu = newrdotr / rdotr;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = r[i] + mu * p[i];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    sc->mu = mu;
    sc->rdotr[(it + 1) & 1] = newrdotr;
    sc->iters = it + 1;
    fl->done[it + 1] = (newrdotr < sc->tol) ? 1 : 0;
  }
}

// trpo_inksci.py:148,151 ingredients
__global__ void shs_partials_kernel(const float* hv, const float* stepdir, const float* g, int64_t n,
                                    const UpdScalars* sc, double* partials, double* partials2) {
  __shared__ double scratch[kRedThreads / 64];
  const float damp = sc->damping;
  double v = 0.0, w = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float si = stepdir[i];
    const float zi = hv[i] + damp * si;
    v += (double)si * (double)zi;
    w += (double)g[i] * (double)si;
  }
  v = block_sum_d(v, scratch);
  w = block_sum_d(w, scratch);
  if (threadIdx.x == 0) {
    partials[blockIdx.x] = v;
    partials2[blockIdx.x] = w;
  }
}

// shs = .5 * stepdir.dot(fvp(stepdir)) ; lm = sqrt(shs/max_kl) ;
// neggdotstepdir = -g.dot(stepdir) ; rate = neggdotstepdir / lm  (trpo_inksci.py:148-153)
__global__ void shs_finish_kernel(const double* partials, const double* partials2, UpdScalars* sc) {
  __shared__ double scratch[kRedThreads / 64];
  const float sdz = (float)sum_partials(partials, kRedBlocks, scratch);
  const float gs = (float)sum_partials(partials2, kRedBlocks, scratch);
  if (threadIdx.x == 0) {
    sc->sdotz = sdz;
    sc->gdots = gs;
    const double shs = 0.5 * (double)sdz;
    const double lm = sqrt(shs / sc->max_kl);
    sc->shs = shs;
    sc->lm = lm;
    const float neg = -gs;
    sc->rate = (double)neg / lm;
    sc->accepted = 0;
    sc->k = -1;
    sc->reverted = 0;
  }
}

// fullstep = stepdir / lm  (float32 loop, lm cast to float32: NumPy-1.x array/scalar rule)
__global__ void fullstep_kernel(const float* stepdir, float* fullstep, int64_t n, const UpdScalars* sc) {
  const float lm = (float)sc->lm;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    fullstep[i] = stepdir[i] / lm;
}

// xnew = x + stepfrac * fullstep  (utils.py:175)
__global__ void ls_trial_kernel(const float* prev, const float* fullstep, float* trial, int64_t n,
                                int k, const UpdScalars* sc) {
  if (sc->accepted) return;
  const float frac = ldexpf(1.0f, -k);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    trial[i] = prev[i] + frac * fullstep[i];
}

__global__ void rowterms_partials_kernel(const double* rt, int64_t n, double* partials3,
                                         const int* skip) {
  __shared__ double scratch[kRedThreads / 64];
  if (skip && *skip) return;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    s0 += rt[4 * i + 0];
    s1 += rt[4 * i + 1];
    s2 += rt[4 * i + 2];
  }
  s0 = block_sum_d(s0, scratch);
  s1 = block_sum_d(s1, scratch);
  s2 = block_sum_d(s2, scratch);
  if (threadIdx.x == 0) {
    partials3[3 * blockIdx.x + 0] = s0;
    partials3[3 * blockIdx.x + 1] = s1;
    partials3[3 * blockIdx.x + 2] = s2;
  }
}

__global__ void rowterms_finish_kernel(const double* partials3, double* local3, const int* skip) {
  __shared__ double scratch[kRedThreads / 64];
  if (skip && *skip) return;
  for (int c = 0; c < 3; ++c) {
    double v = 0.0;
    for (int i = threadIdx.x; i < kRedBlocks; i += blockDim.x) v += partials3[3 * i + c];
    v = block_sum_d(v, scratch);
    if (threadIdx.x == 0) local3[c] = v;
  }
}

// [surr, kl, ent] as session.run(losses) returns them (float32), trpo_inksci.py:48-51
__global__ void losses_store_kernel(const double* g3, double invN, UpdScalars* sc, int which,
                                    const int* skip) {
  if (skip && *skip) return;
  float* out = which == 0 ? sc->loss_before : sc->loss_trial;
  out[0] = (float)(-g3[0] * invN);
  out[1] = (float)(g3[1] * invN);
  out[2] = (float)(g3[2] * invN);
}

// utils.py:176-181
__global__ void ls_decide_kernel(UpdScalars* sc, int k) {
  if (sc->accepted) return;
  const float fval = sc->loss_before[0];
  const float newfval = sc->loss_trial[0];
  const float actual = fval - newfval;
  const double stepfrac = ldexp(1.0, -k);
  const double expected = sc->rate * stepfrac;
  const double ratio = (double)actual / expected;
  if (ratio > 0.1 && actual > 0.0f) {
    sc->accepted = 1;
    sc->k = k;
    sc->loss_after[0] = sc->loss_trial[0];
    sc->loss_after[1] = sc->loss_trial[1];
    sc->loss_after[2] = sc->loss_trial[2];
  }
}

// trpo_inksci.py:153-158
__global__ void ls_finalize_kernel(const float* prev, const float* fullstep, float* theta,
                                   float* theta_ls, int64_t n, UpdScalars* sc) {
  const int acc = sc->accepted;
  const int k = sc->k;
  const float* la = acc ? sc->loss_after : sc->loss_before;
  const bool revert = (double)la[1] > 2.0 * sc->max_kl;
  const float frac = acc ? ldexpf(1.0f, -k) : 0.0f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float pi = prev[i];
    const float t = acc ? pi + frac * fullstep[i] : pi;
    theta_ls[i] = t;
    theta[i] = revert ? pi : t;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (!acc) {
      sc->loss_after[0] = sc->loss_before[0];
      sc->loss_after[1] = sc->loss_before[1];
      sc->loss_after[2] = sc->loss_before[2];
    }
    sc->reverted = revert ? 1 : 0;
  }
}

__global__ void axpby_kernel(float* y, const float* x, float alpha, float beta, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = alpha * x[i] + beta * y[i];
}

__global__ void scale_copy_kernel(const float* x, float* y, float alpha, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = alpha * x[i];
}

__global__ void i64_to_i32_kernel(const int64_t* src, int* dst, int64_t n, int* bad, int hi) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = src[i];
    if (v < 0 || v >= hi) {
      atomicOr(bad, 1);
      dst[i] = 0;
    } else {
      dst[i] = (int)v;
    }
  }
}

__global__ void copy_rows_kernel(const float* src, int64_t n, int w, int ld_src, float* dst, int ld_dst) {
  const int64_t tot = n * ld_dst;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / ld_dst;
    const int c = (int)(e % ld_dst);
    dst[e] = c < w ? src[r * ld_src + c] : 0.0f;
  }
}

__global__ void f64_to_f32_kernel(const double* src, float* dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = (float)src[i];
}

inline int grid_for(int64_t n, int threads = 256, int cap = 4096) {
  int64_t g = (n + threads - 1) / threads;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace

void launch_pack(const PackArgs& pa, const float* src, int which, const int* skip, hipStream_t s) {
  int64_t mx = 1;
  for (int l = 0; l < pa.nl; ++l) mx = std::max<int64_t>(mx, (int64_t)pa.L[l].a * pa.L[l].b);
  dim3 grid(grid_for(mx, 256, 2048), pa.nl);
  hipLaunchKernelGGL(pack_kernel, grid, dim3(256), 0, s, pa, src, which, skip);
}

void launch_reduce_slab(const float* slab, int S, int64_t stride, int64_t P, float* out,
                        const int* skip, hipStream_t s) {
  if (P <= 0) return;
  hipLaunchKernelGGL(reduce_slab_kernel<false>, dim3((unsigned)((P + kRsCols - 1) / kRsCols)), dim3(kRsCols * kRsGroups), 0,
                     s, slab, S, stride, P, out, skip, nullptr, nullptr, nullptr, nullptr);
}

bool cg_fused_reduce_ok(int64_t P) { return (P + kRsCols - 1) / kRsCols <= kRedBlocks; }

void launch_cg_iter_slabs(const float* slab, int S, int64_t stride, float* hv, float* x, float* r, float* p, float* z,
                          int64_t n, UpdScalars* sc, double* partials, double* partials2, CGFlags* fl, int it,
                          hipStream_t s) {
  if (!cg_fused_reduce_ok(n)) throw std::runtime_error("cg_iter_slabs: too many parameters for one partials row");
  const int* skip = &fl->done[it];
  hipLaunchKernelGGL(reduce_slab_kernel<true>, dim3((unsigned)((n + kRsCols - 1) / kRsCols)), dim3(kRsCols * kRsGroups),
                     0, s, slab, S, stride, n, hv, skip, p, z, sc, partials);
  hipLaunchKernelGGL((cg_xr_kernel<float, UpdScalars>), dim3(kRedBlocks), dim3(kRedThreads), 0, s, x, r, p, z, n, sc,
                     partials, partials2, it, skip);
  hipLaunchKernelGGL((cg_p_kernel<float, UpdScalars>), dim3(kRedBlocks), dim3(kRedThreads), 0, s, r, p, n, sc,
                     partials2, fl, it);
}

void launch_dot_partials(const float* a, const float* b, int64_t n, double* partials,
                         const int* skip, hipStream_t s) {
  hipLaunchKernelGGL(dot_partials_kernel, dim3(kRedBlocks), dim3(kRedThreads), 0, s, a, b, n, partials,
                     skip);
}

template <class T, class S>
void cg_init_t(const T* b, T* x, T* r, T* p, int64_t n, double* partials, S* sc, CGFlags* fl,
               double tol, double damping, hipStream_t s) {
  hipLaunchKernelGGL(cg_init_kernel<T>, dim3(kRedBlocks), dim3(kRedThreads), 0, s, b, x, r, p, n, partials);
  hipLaunchKernelGGL((cg_init_finish_kernel<T, S>), dim3(1), dim3(kRedThreads), 0, s, partials, sc, fl,
                     tol, damping);
}
template <class T, class S>
void cg_iter_t(const T* hv, T* x, T* r, T* p, T* z, int64_t n, S* sc, double* pa, double* pb,
               CGFlags* fl, int it, hipStream_t s) {
  const int* skip = &fl->done[it];
  hipLaunchKernelGGL((cg_pz_kernel<T, S>), dim3(kRedBlocks), dim3(kRedThreads), 0, s, hv, p, z, n, sc, pa,
                     skip);
  hipLaunchKernelGGL((cg_xr_kernel<T, S>), dim3(kRedBlocks), dim3(kRedThreads), 0, s, x, r, p, z, n, sc, pa,
                     pb, it, skip);
  hipLaunchKernelGGL((cg_p_kernel<T, S>), dim3(kRedBlocks), dim3(kRedThreads), 0, s, r, p, n, sc, pb, fl,
                     it);
}

void launch_cg_init(const float* b, float* x, float* r, float* p, int64_t n, double* partials,
                    UpdScalars* sc, CGFlags* fl, float tol, float damping, hipStream_t s) {
  cg_init_t<float, UpdScalars>(b, x, r, p, n, partials, sc, fl, tol, damping, s);
}
void launch_cg_iter(const float* hv, float* x, float* r, float* p, float* z, int64_t n, UpdScalars* sc,
                    double* partials, double* partials2, CGFlags* fl, int it, hipStream_t s) {
  cg_iter_t<float, UpdScalars>(hv, x, r, p, z, n, sc, partials, partials2, fl, it, s);
}
void launch_cg_init_d(const double* b, double* x, double* r, double* p, int64_t n, double* partials,
                      CGScalarsD* sc, CGFlags* fl, double tol, hipStream_t s) {
  cg_init_t<double, CGScalarsD>(b, x, r, p, n, partials, sc, fl, tol, 0.0, s);
}
void launch_cg_iter_d(const double* hv, double* x, double* r, double* p, double* z, int64_t n,
                      CGScalarsD* sc, double* partials, double* partials2, CGFlags* fl, int it,
                      hipStream_t s) {
  cg_iter_t<double, CGScalarsD>(hv, x, r, p, z, n, sc, partials, partials2, fl, it, s);
}

void launch_shs_partials(const float* hv, const float* stepdir, const float* g, int64_t n,
                         const UpdScalars* sc, double* partials, double* partials2, hipStream_t s) {
  hipLaunchKernelGGL(shs_partials_kernel, dim3(kRedBlocks), dim3(kRedThreads), 0, s, hv, stepdir, g, n, sc,
                     partials, partials2);
}

void launch_shs_finish(const double* partials, const double* partials2, UpdScalars* sc, hipStream_t s) {
  hipLaunchKernelGGL(shs_finish_kernel, dim3(1), dim3(kRedThreads), 0, s, partials, partials2, sc);
}

void launch_fullstep(const float* stepdir, float* fullstep, int64_t n, const UpdScalars* sc,
                     hipStream_t s) {
  hipLaunchKernelGGL(fullstep_kernel, dim3(grid_for(n)), dim3(256), 0, s, stepdir, fullstep, n, sc);
}

void launch_ls_trial(const float* prev, const float* fullstep, float* trial, int64_t n, int k,
                     const UpdScalars* sc, hipStream_t s) {
  hipLaunchKernelGGL(ls_trial_kernel, dim3(grid_for(n)), dim3(256), 0, s, prev, fullstep, trial, n, k, sc);
}

void launch_rowterms_partials(const double* rowterms, int64_t n, double* partials3, const int* skip,
                              hipStream_t s) {
  hipLaunchKernelGGL(rowterms_partials_kernel, dim3(kRedBlocks), dim3(kRedThreads), 0, s, rowterms, n,
                     partials3, skip);
}

void launch_rowterms_finish(const double* partials3, double* local3, const int* skip, hipStream_t s) {
  hipLaunchKernelGGL(rowterms_finish_kernel, dim3(1), dim3(kRedThreads), 0, s, partials3, local3, skip);
}

void launch_losses_store(const double* global3, double invN, UpdScalars* sc, int which,
                         const int* skip, hipStream_t s) {
  hipLaunchKernelGGL(losses_store_kernel, dim3(1), dim3(1), 0, s, global3, invN, sc, which, skip);
}

void launch_ls_decide(UpdScalars* sc, int k, hipStream_t s) {
  hipLaunchKernelGGL(ls_decide_kernel, dim3(1), dim3(1), 0, s, sc, k);
}

void launch_ls_finalize(const float* prev, const float* fullstep, float* theta, float* theta_ls,
                        int64_t n, UpdScalars* sc, hipStream_t s) {
  hipLaunchKernelGGL(ls_finalize_kernel, dim3(grid_for(n)), dim3(256), 0, s, prev, fullstep, theta,
                     theta_ls, n, sc);
}

void launch_axpby(float* y, const float* x, float alpha, float beta, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(axpby_kernel, dim3(grid_for(n)), dim3(256), 0, s, y, x, alpha, beta, n);
}

void launch_scale_copy(const float* x, float* y, float alpha, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(scale_copy_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, y, alpha, n);
}

void launch_i64_to_i32(const int64_t* src, int* dst, int64_t n, int* bad, int hi, hipStream_t s) {
  hipLaunchKernelGGL(i64_to_i32_kernel, dim3(grid_for(n)), dim3(256), 0, s, src, dst, n, bad, hi);
}

void launch_amax(const float* A, int64_t n, int w, int ld, unsigned* out, hipStream_t s) {
  if (n <= 0 || w <= 0) return;
  hipLaunchKernelGGL(amax_kernel, dim3(grid_for(n * w, 256, 2048)), dim3(256), 0, s, A, n, w, ld, out);
}

void launch_f64_to_f32(const double* src, float* dst, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(f64_to_f32_kernel, dim3(grid_for(n)), dim3(256), 0, s, src, dst, n);
}

void launch_copy_rows(const float* src, int64_t n, int w, int ld_src, float* dst, int ld_dst,
                      hipStream_t s) {
  hipLaunchKernelGGL(copy_rows_kernel, dim3(grid_for(n * ld_dst, 256, 8192)), dim3(256), 0, s, src, n, w,
                     ld_src, dst, ld_dst);
}

}  // namespace trpo
