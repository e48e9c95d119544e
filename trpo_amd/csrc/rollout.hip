// Batched policy sampling and CartPole-v0 rollouts on the GPU (gfx950).
//
// Restates, data-parallel over environments:
//   * agent.act (trpo_inksci.py:76-87): the policy forward on one state, then
//     cat_sample (utils.py:95-105) -- inverse CDF over the float32 cumsum of the
//     action distribution against a float64 uniform, first k with csprob > r,
//     else 0 -- or argmax when not training;
//   * rollout (utils.py:18-45): episodes of up to max_pathlength steps, each
//     recording (obs, action, action_dist, reward), until the collected steps
//     reach n_timesteps;
//   * the CartPole-v0 environment the reference runs (gym.make("CartPole-v0"),
//     trpo_inksci.py:179): Euler-integrated cart-pole, reset to U(-0.05, 0.05)^4,
//     done past |x| > 2.4 or |theta| > 12 degrees, reward 1 per step, and the
//     v0 TimeLimit of 200 steps.  gym is not vendored in the reference; this is
//     its published classic_control/cartpole.py restated in float64 (Python floats).
//
// One wave simulates one environment for its whole share of the rollout: the
// policy forward is wave-parallel over output units (activations in a per-wave
// LDS slice), the physics and sampling are computed redundantly by all 64
// lanes so every lane holds the state in registers.  Each environment collects
// episodes until its own step count reaches ceil(n_timesteps / n_envs) -- the
// reference's stopping rule applied per environment, so with n_envs = 1 it is
// exactly utils.py:23-44 and for any n_envs every started episode completes.
// Episodes land in a per-environment region; a compaction kernel concatenates
// the regions in environment order (deterministic for a given seed).
#include "common.h"
#include "kernels.h"

#include <algorithm>

#pragma clang fp contract(off)

namespace trpo {
namespace {

// ---- Philox4x32-10 (counter-based; key = seed, counter = (env, stream, draw)) -------------------
__device__ __forceinline__ void philox_round(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
  const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  c[0] = hi1 ^ c[1] ^ k0;
  c[1] = lo1;
  c[2] = hi0 ^ c[3] ^ k1;
  c[3] = lo0;
}
__device__ __forceinline__ void philox(uint32_t (&c)[4], uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    philox_round(c, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
// uniform double in [0, 1) with 53 random bits, numpy's random_sample recipe ((a>>5)*2^26 + (b>>6)) / 2^53
__device__ __forceinline__ double uniform53(uint64_t seed, uint32_t env, uint32_t stream, uint64_t draw) {
  uint32_t c[4] = {env, stream, (uint32_t)draw, (uint32_t)(draw >> 32)};
  philox(c, seed);
  const uint32_t a = c[0] >> 5, b = c[1] >> 6;
  return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

// ---- CartPole-v0 (gym classic_control/cartpole.py), float64 ------------------------------------
constexpr double kGravity = 9.8, kMassCart = 1.0, kMassPole = 0.1;
constexpr double kTotalMass = kMassPole + kMassCart;
constexpr double kLength = 0.5;                          // half the pole's length
constexpr double kPoleMassLength = kMassPole * kLength;
constexpr double kForceMag = 10.0, kTau = 0.02;
constexpr double kThetaThreshold = 12 * 2 * 3.141592653589793 / 360;
constexpr double kXThreshold = 2.4;

__device__ __forceinline__ bool cartpole_step(double (&s)[4], int action) {
  const double x = s[0], x_dot = s[1], theta = s[2], theta_dot = s[3];
  const double force = action == 1 ? kForceMag : -kForceMag;
  const double costheta = cos(theta), sintheta = sin(theta);
  const double temp = (force + kPoleMassLength * (theta_dot * theta_dot) * sintheta) / kTotalMass;
  const double thetaacc =
      (kGravity * sintheta - costheta * temp) / (kLength * (4.0 / 3.0 - kMassPole * (costheta * costheta) / kTotalMass));
  const double xacc = temp - kPoleMassLength * thetaacc * costheta / kTotalMass;
  s[0] = x + kTau * x_dot;
  s[1] = x_dot + kTau * xacc;
  s[2] = theta + kTau * theta_dot;
  s[3] = theta_dot + kTau * thetaacc;
  return s[0] < -kXThreshold || s[0] > kXThreshold || s[2] < -kThetaThreshold || s[2] > kThetaThreshold;
}

// ---- wave-level policy forward ---------------------------------------------------------------
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}
__device__ __forceinline__ float wave_sumf(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// h_{l} = tanh(h_{l-1} W_l + b_l) ... p = softmax(z_L) (trpo_inksci.py:38-40); `in` holds the
// obs (w[0] floats) on entry; returns this lane's p (lanes >= A: 0).  All lanes must call.
__device__ float wave_policy(const PolicyShape& ps, const float* theta, float* in, float* out, int lane) {
  for (int l = 0; l < ps.L; ++l) {
    const int a = ps.w[l], b = ps.w[l + 1];
    const float* W = theta + ps.offW[l];
    const float* bias = theta + ps.offb[l];
    const bool last = l == ps.L - 1;
    for (int j = lane; j < b; j += 64) {
      float acc = 0.0f;
      for (int k = 0; k < a; ++k) acc = acc + in[k] * W[(int64_t)k * b + j];
      const float z = acc + bias[j];
      out[j] = last ? z : tanhf(z);
    }
    wave_sync();
    float* t = in;
    in = out;
    out = t;
  }
  // softmax over A <= 64 logits, now in `in`
  const int A = ps.w[ps.L];
  const float z = lane < A ? in[lane] : -INFINITY;
  const float m = wave_max(z);
  const float ex = lane < A ? expf(z - m) : 0.0f;
  const float s = wave_sumf(ex);
  return lane < A ? ex / s : 0.0f;
}

// cat_sample (utils.py:95-105) on the wave's distribution: csprob = float32 cumsum, first k with
// csprob > r (float64 comparison), 0 if none.  train = 0: argmax (trpo_inksci.py:82), first max.
__device__ __forceinline__ int wave_choose(float p, int A, double r, int train, int lane) {
  int out = 0;
  if (train) {
    float cs = 0.0f;
    for (int k = 0; k < A; ++k) {
      cs = cs + __shfl(p, k, 64);
      if ((double)cs > r) {
        out = k;
        break;
      }
    }
  } else {
    float best = __shfl(p, 0, 64);
    for (int k = 1; k < A; ++k) {
      const float pk = __shfl(p, k, 64);
      if (pk > best) {
        best = pk;
        out = k;
      }
    }
  }
  (void)lane;
  return out;
}

constexpr int kRollWaves = 4;

__global__ void __launch_bounds__(kRollWaves * 64) rollout_kernel(const RolloutArgs a) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int env = blockIdx.x * kRollWaves + wv;
  if (env >= a.n_envs) return;
  float* buf0 = lds + (size_t)wv * 2 * a.maxw;
  float* buf1 = buf0 + a.maxw;
  const int obs_dim = a.ps.w[0], A = a.ps.w[a.ps.L];
  const int64_t base = (int64_t)env * a.env_cap;
  int64_t count = 0;
  int episode = 0;
  uint64_t adraw = 0;
  while (count < a.budget) {
    // env.reset(): np_random.uniform(-0.05, 0.05, size=(4,))
    double s[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const double u = a.reset_u ? a.reset_u[((int64_t)env * a.max_episodes + episode) * 4 + i]
                                 : uniform53(a.seed, (uint32_t)env, 1u, (uint64_t)episode * 4 + i);
      s[i] = -0.05 + (0.05 - -0.05) * u;
    }
    ++episode;
    for (int t = 0; t < a.max_pathlength; ++t) {
      const int64_t row = base + count;
      // act(ob): the obs fed to the float32 state placeholder, recorded as the float64 ob
      if (lane < obs_dim) {
        buf0[lane] = (float)s[lane];
        a.obs[row * obs_dim + lane] = s[lane];
      }
      wave_sync();
      const float p = wave_policy(a.ps, a.theta, buf0, buf1, lane);
      const double r = a.act_u ? a.act_u[row] : uniform53(a.seed, (uint32_t)env, 0u, adraw);
      ++adraw;
      const int action = wave_choose(p, A, r, a.train, lane);
      if (lane < A) a.dist[row * A + lane] = p;
      const bool done = cartpole_step(s, action);
      if (lane == 0) {
        a.actions[row] = action;
        a.rewards[row] = 1.0;
        a.starts[row] = t == 0 ? 1 : 0;
        if (a.uniforms_out) a.uniforms_out[row] = r;
      }
      ++count;
      // CartPole-v0's TimeLimit(max_episode_steps=200) reports done at step 200
      if (done || t + 1 >= a.time_limit) break;
      wave_sync();
    }
    wave_sync();
  }
  if (lane == 0) {
    a.counts[env] = count;
    a.episodes[env] = episode;
  }
}

// concatenate the per-environment regions in environment order
__global__ void __launch_bounds__(256) rollout_compact_kernel(const RolloutArgs a, const int64_t* offsets,
                                                              RolloutOut o) {
  const int obs_dim = a.ps.w[0], A = a.ps.w[a.ps.L];
  const int env = blockIdx.y;
  const int64_t cnt = a.counts[env], dst0 = offsets[env], src0 = (int64_t)env * a.env_cap;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = src0 + i, d = dst0 + i;
    for (int c = 0; c < obs_dim; ++c) {
      const double v = a.obs[s * obs_dim + c];
      if (o.obs64) o.obs64[d * obs_dim + c] = v;
      if (o.X) o.X[d * o.ldx + c] = (float)v;
    }
    for (int c = 0; c < A; ++c) {
      const float v = a.dist[s * A + c];
      if (o.dist) o.dist[d * A + c] = v;
      if (o.old) o.old[d * o.ld_old + c] = v;
    }
    if (o.actions64) o.actions64[d] = a.actions[s];
    if (o.act32) o.act32[d] = a.actions[s];
    if (o.rewards) o.rewards[d] = a.rewards[s];
    if (o.starts) o.starts[d] = a.starts[s];
    if (o.uniforms && a.uniforms_out) o.uniforms[d] = a.uniforms_out[s];
  }
}

// act on a batch of given states (one wave per state)
__global__ void __launch_bounds__(kRollWaves * 64) act_kernel(const PolicyShape ps, const float* theta, int maxw,
                                                              const float* states, int64_t n, const double* r,
                                                              int train, int64_t* actions, float* dists) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t row = (int64_t)blockIdx.x * kRollWaves + wv;
  if (row >= n) return;
  float* buf0 = lds + (size_t)wv * 2 * maxw;
  float* buf1 = buf0 + maxw;
  const int obs_dim = ps.w[0], A = ps.w[ps.L];
  for (int c = lane; c < obs_dim; c += 64) buf0[c] = states[row * obs_dim + c];
  wave_sync();
  const float p = wave_policy(ps, theta, buf0, buf1, lane);
  const int action = wave_choose(p, A, r ? r[row] : 0.0, train, lane);
  if (lane < A && dists) dists[row * A + lane] = p;
  if (lane == 0 && actions) actions[row] = action;
}

__global__ void __launch_bounds__(256) cat_sample_kernel(const float* prob, int64_t n, int k, const double* r,
                                                         int64_t* out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float cs = 0.0f;
    int64_t o = 0;
    for (int j = 0; j < k; ++j) {
      cs = cs + prob[i * k + j];
      if ((double)cs > r[i]) {
        o = j;
        break;
      }
    }
    out[i] = o;
  }
}

__global__ void __launch_bounds__(256) cartpole_step_kernel(const double* state, const int64_t* action, int64_t n,
                                                            double* state_out, double* reward, uint8_t* done) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double s[4] = {state[4 * i], state[4 * i + 1], state[4 * i + 2], state[4 * i + 3]};
    const bool d = cartpole_step(s, (int)action[i]);
#pragma unroll
    for (int j = 0; j < 4; ++j) state_out[4 * i + j] = s[j];
    if (reward) reward[i] = 1.0;
    if (done) done[i] = d ? 1 : 0;
  }
}

inline unsigned grid1(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

}  // namespace

size_t rollout_lds_bytes(int maxw) { return (size_t)kRollWaves * 2 * maxw * sizeof(float); }

void launch_rollout(const RolloutArgs& a, hipStream_t s) {
  const unsigned blocks = (unsigned)((a.n_envs + kRollWaves - 1) / kRollWaves);
  hipLaunchKernelGGL(rollout_kernel, dim3(blocks), dim3(kRollWaves * 64), rollout_lds_bytes(a.maxw), s, a);
}

void launch_rollout_compact(const RolloutArgs& a, const int64_t* offsets, const RolloutOut& o, int64_t max_count,
                            hipStream_t s) {
  const unsigned bx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((max_count + 255) / 256, 64));
  hipLaunchKernelGGL(rollout_compact_kernel, dim3(bx, a.n_envs), dim3(256), 0, s, a, offsets, o);
}

void launch_act(const PolicyShape& ps, const float* theta, int maxw, const float* states, int64_t n, const double* r,
                int train, int64_t* actions, float* dists, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(act_kernel, dim3((unsigned)((n + kRollWaves - 1) / kRollWaves)), dim3(kRollWaves * 64),
                     rollout_lds_bytes(maxw), s, ps, theta, maxw, states, n, r, train, actions, dists);
}

void launch_cat_sample(const float* prob, int64_t n, int k, const double* r, int64_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(cat_sample_kernel, dim3(grid1(n)), dim3(256), 0, s, prob, n, k, r, out);
}

void launch_cartpole_step(const double* state, const int64_t* action, int64_t n, double* state_out, double* reward,
                          uint8_t* done, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(cartpole_step_kernel, dim3(grid1(n)), dim3(256), 0, s, state, action, n, state_out, reward, done);
}

}  // namespace trpo
