// Standalone check of rowepi.h tanh_fast against a packed-f32 form of the same arithmetic (two values per
// v_pk_fma_f32 / v_pk_mul_f32): max |difference| over a sweep of inputs.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#include "rowepi.h"

using trpo::tanh_fast;
typedef float tf2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ tf2 tanh_fast2(tf2 x) {
  const tf2 ax = {fabsf(x.x), fabsf(x.y)};
  const tf2 x2 = x * x;
  tf2 p = __builtin_elementwise_fma(tf2{-0.005700020585209131f, -0.005700020585209131f}, x2,
                                    tf2{0.02063407190144062f, 0.02063407190144062f});
  p = __builtin_elementwise_fma(p, x2, tf2{-0.053737930953502655f, -0.053737930953502655f});
  p = __builtin_elementwise_fma(p, x2, tf2{0.13331416249275208f, 0.13331416249275208f});
  p = __builtin_elementwise_fma(p, x2, tf2{-0.3333328068256378f, -0.3333328068256378f});
  const tf2 small = __builtin_elementwise_fma(x2, ax * p, ax);
  const tf2 e = ax * tf2{-2.8853900817779268f, -2.8853900817779268f};
  const tf2 t = {__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
  const tf2 d = t + tf2{1.0f, 1.0f};
  const tf2 r = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  const tf2 big = __builtin_elementwise_fma(-t, r, r);
  return tf2{__builtin_copysignf(ax.x < 0.625f ? small.x : big.x, x.x),
             __builtin_copysignf(ax.y < 0.625f ? small.y : big.y, x.y)};
}

__global__ void k(const float* in, float* a, float* b, int n) {
  const int i = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (i + 1 >= n) return;
  const tf2 x = {in[i], in[i + 1]};
  const tf2 y = tanh_fast2(x);
  a[i] = tanh_fast(x.x);
  a[i + 1] = tanh_fast(x.y);
  b[i] = y.x;
  b[i + 1] = y.y;
}

int main() {
  const int n = 1 << 20;
  std::vector<float> h(n), ra(n), rb(n);
  for (int i = 0; i < n; ++i) h[i] = -12.0f + 24.0f * (float)i / (float)n;
  float *din, *da, *db;
  if (hipMalloc(&din, n * 4) || hipMalloc(&da, n * 4) || hipMalloc(&db, n * 4)) return 1;
  hipMemcpy(din, h.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 512), dim3(256), 0, 0, din, da, db, n);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  hipMemcpy(ra.data(), da, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(rb.data(), db, n * 4, hipMemcpyDeviceToHost);
  double md = 0, me = 0;
  int bad = 0, first = -1;
  for (int i = 0; i < n; ++i) {
    const double d = std::fabs((double)ra[i] - (double)rb[i]);
    const double e = std::fabs((double)ra[i] - std::tanh((double)h[i]));
    if (d > 0 && first < 0) first = i;
    bad += d > 0;
    md = d > md ? d : md;
    me = e > me ? e : me;
  }
  std::printf("scalar vs packed: %d of %d differ, max |diff| %.3e (first at x = %.6f: %.8f vs %.8f); scalar vs "
              "tanh: max |err| %.3e\n", bad, n, md, first >= 0 ? h[first] : 0.0, first >= 0 ? ra[first] : 0.0,
              first >= 0 ? rb[first] : 0.0, me);
  return 0;
}
