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
#include "chain_common.h"
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

// The whole CG iteration after the one-launch FVP (single rank, cg_fuse_reduce = 2), in one launch: every block runs
// reduce_slab_kernel<true> on its 64 parameters (Hv, z = Hv + damping p, its p.z partial), then takes a ticket; the
// block that arrives last runs cg_xr_kernel's and cg_p_kernel's arithmetic over all P (utils.py:192-200) and, on the
// fused16 path, builds the next FVP's V images from the new p (fused16_img_kernel's values and exponents), which
// removes three launches per iteration (cg_xr, cg_p, the image build).  The last block replays the 256-thread blocks
// of those kernels wave by wave: each of its waves sums the 64 values one of their waves held with the same
// butterfly, and the virtual blocks' partials and the final sums are added in the same order, so x, r, p, alpha, mu
// and rdotr are bit-identical to cg_fuse_reduce = 1.  Hand-off: plain stores, s_waitcnt vmcnt(0), workgroup barrier,
// lane-0 agent release fence, vmcnt(0), agent-scope ticket add; the last arriver's agent acquire fence, vmcnt(0) and
// a workgroup barrier before its loads (MI355X_MICROARCH.md, inter-workgroup visibility).  It resets the ticket.
constexpr int kCgStepMax = kRedBlocks * kRsCols;        // P limit: the fixed partial layout (cg_fused_reduce_ok)
constexpr int kCgStepPer = kCgStepMax / (kRsCols * kRsGroups);   // parameters per thread of the last block (16)
static_assert(kRsCols * kRsGroups == 1024 && kRedThreads == 256, "cg_step: 16 waves replay 4-wave blocks");

typedef __fp16 fp16x2_t __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(kRsCols* kRsGroups)
cg_step_slabs_kernel(const CgStepArgs a, const ChainImgArgs img, int* img_e) {
  __shared__ float red[kRsGroups][kRsCols + 1];
  __shared__ double ws[kRedBlocks], pb[kRedBlocks], w4[4];
  __shared__ float pl[kCgStepMax];
  __shared__ unsigned jm[kMaxChainJobs];
  __shared__ int last;
  const int it = a.it;
  if (a.fl->done[it]) {   // converged: this iteration is a no-op, and so is every later one (cg_p_kernel)
    if (blockIdx.x == 0 && threadIdx.x == 0) a.fl->done[it + 1] = 1;
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t P = a.P;
  {   // reduce_slab_kernel<true>'s body
    const int c = tid % kRsCols, g = tid / kRsCols;
    const int64_t p = (int64_t)blockIdx.x * kRsCols + c;
    float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
    if (p < P) {
      constexpr int G = kRsGroups;
      int s = g;
      for (; s + 3 * G < a.S; s += 4 * G) {
        a0 += a.slab[(int64_t)s * a.stride + p];
        a1 += a.slab[(int64_t)(s + G) * a.stride + p];
        a2 += a.slab[(int64_t)(s + 2 * G) * a.stride + p];
        a3 += a.slab[(int64_t)(s + 3 * G) * a.stride + p];
      }
      for (; s < a.S; s += G) a0 += a.slab[(int64_t)s * a.stride + p];
    }
    red[g][c] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (g == 0) {
      double v = 0.0;
      if (p < P) {
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < kRsGroups; ++i) acc += red[i][c];
        a.hv[p] = acc;
        const float damp = a.sc->damping, pi = a.p[p];
        const float zi = damp != 0.0f ? acc + damp * pi : acc;
        a.z[p] = zi;
        v = (double)pi * (double)zi;
      }
      v = wave_sum_d_fast(v);
      if (c == 0) a.partials[blockIdx.x] = v;
    }
  }
  // ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int is_last = old + 1 == gridDim.x;
    if (is_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    last = is_last;
  }
  __syncthreads();
  if (!last) return;

  // pz: cg_xr_kernel's sum_partials(partials, kRedBlocks) on a 256-thread block (blocks past the grid: 0)
  const int nb = (int)gridDim.x;
  if (wv < 4) {
    const double v = wave_sum_d_fast(0.0 + (tid < nb ? a.partials[tid] : 0.0));
    if (lane == 0) w4[wv] = v;
  }
  __syncthreads();
  double t = 0.0;
  for (int w = 0; w < 4; ++w) t += w4[w];
  const float pz = (float)t;
  const float rdotr = a.sc->rdotr[it & 1];
  const float alpha = rdotr / pz;
  // x += alpha p ; r -= alpha z ; r.r per virtual wave (element i: virtual wave i / 64, lane i % 64)
  // every load first: x, r, p, z may alias as far as the compiler knows, so a load behind a store would wait for it
  float rv[kCgStepPer], pv[kCgStepPer], xv[kCgStepPer], zv[kCgStepPer];
#pragma unroll
  for (int k = 0; k < kCgStepPer; ++k) {
    const int64_t i = tid + (int64_t)1024 * k;
    const bool in = i < P;
    pv[k] = in ? a.p[i] : 0.0f;
    xv[k] = in ? a.x[i] : 0.0f;
    rv[k] = in ? a.r[i] : 0.0f;
    zv[k] = in ? a.z[i] : 0.0f;
  }
  double vv[kCgStepPer];
#pragma unroll
  for (int k = 0; k < kCgStepPer; ++k) {
    const int64_t i = tid + (int64_t)1024 * k;
    double v = 0.0;
    if (i < P) {
      a.x[i] = xv[k] + alpha * pv[k];
      const float ri = rv[k] - alpha * zv[k];
      a.r[i] = ri;
      rv[k] = ri;
      v += (double)ri * (double)ri;
    }
    vv[k] = v;
  }
#pragma unroll
  for (int k = 0; k < kCgStepPer; ++k) vv[k] = wave_sum_d_fast(vv[k]);   // 16 independent butterflies
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < kCgStepPer; ++k) ws[16 * k + wv] = vv[k];
  }
  __syncthreads();
  if (tid < kRedBlocks) {   // virtual block tid's partial (block_sum_d: its 4 wave sums in order; past P: 0)
    double s = 0.0;
    if (tid < kCgStepMax / kRedThreads)
      for (int w = 0; w < 4; ++w) s += ws[4 * tid + w];
    pb[tid] = s;
  }
  __syncthreads();
  if (wv < 4) {   // cg_p_kernel's sum_partials(partials2, kRedBlocks)
    const double v = wave_sum_d_fast(0.0 + pb[tid]);
    if (lane == 0) w4[wv] = v;
  }
  if (tid < kMaxChainJobs) jm[tid] = 0u;
  __syncthreads();
  t = 0.0;
  for (int w = 0; w < 4; ++w) t += w4[w];
  const float newrdotr = (float)t;
  const float mu = newrdotr / rdotr;
  // p = r + mu p, kept in LDS for the image
#pragma unroll
  for (int k = 0; k < kCgStepPer; ++k) {
    const int64_t i = tid + (int64_t)1024 * k;
    if (i < P) {
      const float pn = rv[k] + mu * pv[k];
      a.p[i] = pn;
      pl[i] = pn;
    }
  }
  if (tid == 0) {
    a.sc->alpha = alpha;
    a.sc->mu = mu;
    a.sc->rdotr[(it + 1) & 1] = newrdotr;
    a.sc->iters = it + 1;
    a.fl->done[it + 1] = (newrdotr < a.sc->tol) ? 1 : 0;
  }
  if (img.n == 0) return;
  __syncthreads();
  for (int j = 0; j < img.n; ++j) {   // the V jobs' max |p| (fused16_img_kernel: over the whole K x O source)
    const ChainImgJob& jb = img.job[j];
    if (jb.which != 1) continue;
    float m = 0.0f;
    for (int e = tid; e < jb.K * jb.O; e += 1024) m = fmaxf(m, fabsf(pl[jb.src_off + e]));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    if (lane == 0 && m > 0.0f) atomicMax(&jm[j], __float_as_uint(m));
  }
  __syncthreads();
  // the next FVP's V images (fused16_img_kernel: 8 values per unit, scaled by 2^e, split hi / lo, 16-B stores)
  for (int j = 0; j < img.n; ++j) {
    const ChainImgJob& jb = img.job[j];
    if (jb.which != 1) continue;
    const int e = f16_scale_exp(__uint_as_float(jm[j]));
    if (tid == 0) img_e[j] = e;
    const float sc = __builtin_ldexpf(1.0f, e);
    const float* src = pl + jb.src_off;
    const int units = jb.kc * jb.otp * 4;
    for (int idx = tid; idx < units; idx += 1024) {
      const int gg = idx & 3, o = (idx >> 2) % jb.otp, c = (idx >> 2) / jb.otp;
      float x[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int k = 32 * c + chain_perm(8 * gg + q);
        const bool in = o < jb.O && k < jb.K;
        x[q] = in ? src[jb.trans ? o * jb.ldw + k : k * jb.ldw + o] * sc : 0.0f;
      }
      cu32x4 H, L;
#pragma unroll
      for (int q = 0; q < 4; ++q) {   // fused16.hip split2.  (Routing hi through the cu32x4 and back by bit_cast
        // made hipcc subtract pair 0's hi from every pair: kept in fp16x2 registers here)
        const fp16x2_t hp = __builtin_amdgcn_cvt_pkrtz(x[2 * q], x[2 * q + 1]);
        const fp16x2_t lp = __builtin_amdgcn_cvt_pkrtz(x[2 * q] - (float)hp[0], x[2 * q + 1] - (float)hp[1]);
        H[q] = __builtin_bit_cast(unsigned, hp);
        L[q] = __builtin_bit_cast(unsigned, lp);
      }
      unsigned short* dst = img.img + jb.dst_off + (size_t)c * 2 * jb.otp * 32 + o * 32 + ((gg ^ chain_hsw(o)) << 3);
      *reinterpret_cast<cu32x4*>(dst) = H;
      *reinterpret_cast<cu32x4*>(dst + (size_t)jb.otp * 32) = L;
    }
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
                          hipStream_t s, bool p_update) {
  if (!cg_fused_reduce_ok(n)) throw std::runtime_error("cg_iter_slabs: too many parameters for one partials row");
  const int* skip = &fl->done[it];
  hipLaunchKernelGGL(reduce_slab_kernel<true>, dim3((unsigned)((n + kRsCols - 1) / kRsCols)), dim3(kRsCols * kRsGroups),
                     0, s, slab, S, stride, n, hv, skip, p, z, sc, partials);
  hipLaunchKernelGGL((cg_xr_kernel<float, UpdScalars>), dim3(kRedBlocks), dim3(kRedThreads), 0, s, x, r, p, z, n, sc,
                     partials, partials2, it, skip);
  if (p_update)
    hipLaunchKernelGGL((cg_p_kernel<float, UpdScalars>), dim3(kRedBlocks), dim3(kRedThreads), 0, s, r, p, n, sc,
                       partials2, fl, it);
}

void launch_cg_step_slabs(const CgStepArgs& a, const ChainImgArgs* img, int* img_e, hipStream_t s) {
  if (!cg_fused_reduce_ok(a.P)) throw std::runtime_error("cg_step_slabs: too many parameters for one partials row");
  ChainImgArgs none{};
  const ChainImgArgs& ia = img ? *img : none;
  if (img) {   // the V jobs' sources must sit inside P (the last block gathers them from its LDS copy of p)
    for (int j = 0; j < ia.n; ++j)
      if (ia.job[j].which == 1 && ia.job[j].src_off + (int64_t)ia.job[j].K * ia.job[j].O > a.P)
        throw std::runtime_error("cg_step_slabs: image job outside the parameter vector");
  }
  hipLaunchKernelGGL(cg_step_slabs_kernel, dim3((unsigned)((a.P + kRsCols - 1) / kRsCols)), dim3(kRsCols * kRsGroups), 0,
                     s, a, ia, img_e);
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
