// Value-function baseline kernels (gfx950): the VF of utils.py:48-92, a
// [obs | action_dist | t/10] -> 64 ReLU -> 64 ReLU -> 1 MLP fitted by 50
// full-batch Adam steps on sum((net - y)^2) (utils.py:60-66,84-85).
//
// The two hidden layers and their backward run on the row GEMM (gemm.hip,
// RowEpi::kRelu / kReluBwd) and the weight gradients on the split-K wgrad
// GEMM; this file holds the row-wise pieces around them: feature assembly,
// the 64 -> 1 output layer fused with the loss gradient, weight packing and
// TF's Adam update.
#include "common.h"
#include "kernels.h"

#pragma clang fp contract(off)

namespace trpo {
namespace {

constexpr int kPosItems = 16;                       // rows per thread in the position scan
constexpr int kPosBlock = 256 * kPosItems;          // rows per block

__device__ __forceinline__ int64_t wave_incl_max(int64_t v, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t o = __shfl_up(v, off, 64);
    if (lane >= off) v = v > o ? v : o;
  }
  return v;
}

// lastpos[r] = max{ s <= r : starts[s] } within this block (-1 if none); blockmax[b] = block total
__global__ void __launch_bounds__(256) pos_local_kernel(const uint8_t* starts, int64_t n, int64_t* lastpos,
                                                        int64_t* blockmax) {
  __shared__ int64_t wtot[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t base = (int64_t)blockIdx.x * kPosBlock + (int64_t)tid * kPosItems;
  int64_t run = -1;
  int64_t loc[kPosItems];
#pragma unroll
  for (int i = 0; i < kPosItems; ++i) {
    const int64_t r = base + i;
    if (r < n && starts[r]) run = r;
    loc[i] = run;
  }
  // exclusive max over earlier threads of the block
  int64_t incl = wave_incl_max(run, lane);
  int64_t excl = __shfl_up(incl, 1, 64);
  if (lane == 0) excl = -1;
  if (lane == 63) wtot[wave] = incl;
  __syncthreads();
  for (int w = 0; w < wave; ++w) excl = excl > wtot[w] ? excl : wtot[w];
#pragma unroll
  for (int i = 0; i < kPosItems; ++i) {
    const int64_t r = base + i;
    if (r < n) lastpos[r] = loc[i] > excl ? loc[i] : excl;
  }
  if (tid == 255) blockmax[blockIdx.x] = incl > excl ? incl : excl;
}

// blockmax -> exclusive prefix max (one block, sequential over chunks of 256)
__global__ void __launch_bounds__(256) pos_blocks_kernel(int64_t* blockmax, int nb) {
  __shared__ int64_t wtot[4];
  __shared__ int64_t carry_s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) carry_s = -1;
  __syncthreads();
  for (int c0 = 0; c0 < nb; c0 += 256) {
    const int i = c0 + tid;
    const int64_t v = i < nb ? blockmax[i] : -1;
    int64_t incl = wave_incl_max(v, lane);
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    int64_t pre = carry_s;
    for (int w = 0; w < wave; ++w) pre = pre > wtot[w] ? pre : wtot[w];
    int64_t ex = __shfl_up(incl, 1, 64);
    if (lane == 0) ex = -1;
    const int64_t excl = pre > ex ? pre : ex;
    __syncthreads();
    if (i < nb) blockmax[i] = excl;
    if (tid == 255) carry_s = incl > excl ? incl : excl;
    __syncthreads();
  }
}

// feat[r] = [obs[r] | dist[r] | f32(t/10.0)], t = r - (start of r's path); padding zero
__global__ void __launch_bounds__(256) features_kernel(const float* obs, int obs_dim, int ld_obs, const float* dist,
                                                       int A, int ld_dist, const int64_t* lastpos,
                                                       const int64_t* blockpre, int64_t n, float* feat, int Fp) {
  const int64_t total = n * Fp;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / Fp;
    const int c = (int)(e - r * Fp);
    float v = 0.0f;
    if (c < obs_dim) {
      v = obs[r * ld_obs + c];
    } else if (c < obs_dim + A) {
      v = dist[r * ld_dist + (c - obs_dim)];
    } else if (c == obs_dim + A) {
      int64_t s = -1;
      if (lastpos) {
        s = lastpos[r];
        const int64_t bp = blockpre[r / kPosBlock];
        s = s > bp ? s : bp;
      }
      const int64_t t = r - (s < 0 ? 0 : s);
      v = (float)((double)t / 10.0);   // np.arange(l)/10.0 (f64) fed to a float32 placeholder (utils.py:76-77)
    }
    feat[e] = v;
  }
}

__global__ void __launch_bounds__(256) vf_pack_kernel(const VFPackArgs a, const float* theta) {
  const int64_t n1 = (int64_t)a.F * a.H1, n2 = (int64_t)a.H1 * a.H2;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n1 + n2;
       e += (int64_t)gridDim.x * blockDim.x) {
    if (e < n1) {
      const int i = (int)(e / a.H1), j = (int)(e % a.H1);
      a.W1p[(int64_t)i * a.H1p + j] = theta[a.offW1 + e];
    } else {
      const int64_t f = e - n1;
      const int i = (int)(f / a.H2), j = (int)(f % a.H2);
      const float v = theta[a.offW2 + f];
      a.W2p[(int64_t)i * a.H2p + j] = v;
      a.W2T[(int64_t)j * a.H1p + i] = v;
    }
  }
}

// Output layer + loss gradient, 16 lanes per row (4 columns per lane per 64-column chunk):
//   out = Z2 w3 + b3 ;  train: d = out - y, dout = d + d (grad of (net-y)*(net-y), utils.py:64),
//   dZ2 = (dout w3^T) * (Z2 > 0) (ReluGrad) ;  predict: out -> f32 / f64
__global__ void __launch_bounds__(256) vf_head_kernel(const VFHeadArgs a) {
  const int tid = threadIdx.x;
  const int q = tid & 15;
  const int64_t r = (int64_t)blockIdx.x * 16 + (tid >> 4);
  const bool valid = r < a.n;
  const int64_t rr = valid ? r : 0;
  const float* z = a.Z2 + rr * a.H2p;
  float part = 0.0f;
  for (int c0 = 0; c0 < a.H2p; c0 += 64) {
    const int c = c0 + 4 * q;
    if (c < a.H2p) {
      const f32x4 zv = *reinterpret_cast<const f32x4*>(z + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) part += (c + j < a.H2 ? zv[j] * a.w3[c + j] : 0.0f);
    }
  }
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) part += __shfl_xor(part, off, 16);
  const float out = part + a.b3[0];
  if (!a.train) {
    if (valid && q == 0) {
      if (a.out64) a.out64[r] = (double)out;
      else a.out32[r] = out;
    }
    return;
  }
  const float d = out - (valid ? a.y[rr] : 0.0f);
  const float dout = valid ? d + d : 0.0f;
  if (valid && q == 0) {
    a.dout[rr * 4 + 0] = dout;
    a.loss_rows[rr] = (double)d * (double)d;
  }
  if (!valid) return;
  float* dz = a.dZ2 + rr * a.H2p;
  for (int c0 = 0; c0 < a.H2p; c0 += 64) {
    const int c = c0 + 4 * q;
    if (c < a.H2p) {
      const f32x4 zv = *reinterpret_cast<const f32x4*>(z + c);
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (c + j < a.H2 && zv[j] > 0.0f) ? dout * a.w3[c + j] : 0.0f;
      *reinterpret_cast<f32x4*>(dz + c) = o;
    }
  }
}

// TF 1.x ApplyAdam (training_ops.cc), float32:
//   m += (g - m)(1 - b1) ; v += (g^2 - v)(1 - b2) ; var -= (m alpha) / (sqrt(v) + eps)
// alpha = lr sqrt(1 - b2^t)/(1 - b1^t) is computed on the host in float32.
__global__ void __launch_bounds__(256) adam_kernel(float* var, const float* g, float* m, float* v, int64_t n,
                                                   float alpha, float b1, float b2, float eps) {
  const float c1 = 1.0f - b1, c2 = 1.0f - b2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i];
    const float mi = m[i] + (gi - m[i]) * c1;
    const float vi = v[i] + (gi * gi - v[i]) * c2;
    m[i] = mi;
    v[i] = vi;
    var[i] = var[i] - (mi * alpha) / (sqrtf(vi) + eps);
  }
}

inline int grid_of(int64_t n, int cap = 4096) {
  const int64_t b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

}  // namespace

size_t vf_pos_workspace_bytes(int64_t n) { return (size_t)((n + kPosBlock - 1) / kPosBlock + 1) * sizeof(int64_t); }

void launch_vf_features(const float* obs, int obs_dim, int ld_obs, const float* dist, int A, int ld_dist,
                        const uint8_t* starts, int64_t n, int64_t* lastpos, void* ws, float* feat, int Fp,
                        hipStream_t s) {
  if (n <= 0) return;
  int64_t* blockpre = static_cast<int64_t*>(ws);
  if (starts) {
    const int nb = (int)((n + kPosBlock - 1) / kPosBlock);
    hipLaunchKernelGGL(pos_local_kernel, dim3(nb), dim3(256), 0, s, starts, n, lastpos, blockpre);
    hipLaunchKernelGGL(pos_blocks_kernel, dim3(1), dim3(256), 0, s, blockpre, nb);
  }
  hipLaunchKernelGGL(features_kernel, dim3(grid_of(n * Fp)), dim3(256), 0, s, obs, obs_dim, ld_obs, dist, A, ld_dist,
                     starts ? lastpos : nullptr, blockpre, n, feat, Fp);
}

void launch_vf_pack(const VFPackArgs& a, const float* theta, hipStream_t s) {
  hipLaunchKernelGGL(vf_pack_kernel, dim3(grid_of((int64_t)a.F * a.H1 + (int64_t)a.H1 * a.H2, 1024)), dim3(256), 0,
                     s, a, theta);
}

void launch_vf_head(const VFHeadArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(vf_head_kernel, dim3((unsigned)((a.n + 15) / 16)), dim3(256), 0, s, a);
}

void launch_adam(float* var, const float* g, float* m, float* v, int64_t n, float alpha, float b1, float b2, float eps,
                 hipStream_t s) {
  hipLaunchKernelGGL(adam_kernel, dim3(grid_of(n, 1024)), dim3(256), 0, s, var, g, m, v, n, alpha, b1, b2, eps);
}

}  // namespace trpo
