// Price of a grid-wide barrier on the fused16 grid (two 256-thread workgroups per CU) against the dependent kernel
// boundary it would replace in a persistent CG loop (verdict item "CG as a persistent-kernel loop").
//
//   hipcc -O3 --offload-arch=gfx950 tools/grid_barrier_bench.hip -o tools/bin/grid_barrier_bench
//   tools/bin/grid_barrier_bench [grid] [barriers]
//
// Three timings, each the median of 5 runs (HIP events on one stream):
//  * `graph`: `barriers` empty dependent launches of `grid` workgroups replayed from one hipGraph (the CG's launches);
//  * `counter`: one launch of `grid` workgroups passing `barriers` grid barriers on one monotonic counter (leader
//    lane: agent release fence, relaxed atomic add, relaxed poll with s_sleep, agent acquire fence);
//  * `xcd`: the same with the arrivals first gathered per workgroup group (blockIdx % 8) and one arrival per group
//    on the top counter (MI355X_MICROARCH.md row barrier-xcd).
// Every spin is bounded: a barrier that is not reached within ~2^22 polls sets a timeout word and the kernel ends.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      std::exit(1);                                                                         \
    }                                                                                       \
  } while (0)

constexpr unsigned kSpinLimit = 1u << 22;

__device__ __forceinline__ unsigned ld_relaxed(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool spin_until(unsigned* p, unsigned target, unsigned* tmo) {
  unsigned spins = 0;
  while (ld_relaxed(p) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > kSpinLimit) {
      __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  return true;
}

// per-workgroup work between barriers: a 16-B store per thread, the kind of vector phase a CG step has
__device__ __forceinline__ void touch(float* buf, int it) {
  buf[(size_t)blockIdx.x * blockDim.x + threadIdx.x] += (float)it;
}

__global__ void __launch_bounds__(256) counter_kernel(unsigned* ctr, unsigned* tmo, float* buf, int nbar) {
  bool ok = true;
  for (int it = 0; it < nbar && ok; ++it) {
    touch(buf, it);
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ok = spin_until(ctr, (unsigned)(it + 1) * gridDim.x, tmo);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    ok = __syncthreads_and(ok) != 0;
  }
}

// ctr[0]: top counter (one arrival per group per barrier); ctr[64 * (1 + grp)]: the group's own counter and
// ctr[64 * (9 + grp)] its release generation, each on its own line
__global__ void __launch_bounds__(256) xcd_kernel(unsigned* ctr, unsigned* tmo, float* buf, int nbar) {
  const int grp = blockIdx.x % 8;
  const unsigned members = (gridDim.x - grp + 7) / 8;
  unsigned* gcnt = ctr + 64 * (1 + grp);
  unsigned* ggen = ctr + 64 * (9 + grp);
  const unsigned ngroups = gridDim.x < 8 ? gridDim.x : 8;
  bool ok = true;
  for (int it = 0; it < nbar && ok; ++it) {
    touch(buf, it);
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned prev = __hip_atomic_fetch_add(gcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev + 1 == (unsigned)(it + 1) * members) {   // the group's last arrival carries it to the top
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = spin_until(ctr, (unsigned)(it + 1) * ngroups, tmo);
        __hip_atomic_store(ggen, (unsigned)(it + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        ok = spin_until(ggen, (unsigned)(it + 1), tmo);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    ok = __syncthreads_and(ok) != 0;
  }
}

__global__ void __launch_bounds__(256) step_kernel(float* buf, int it) { touch(buf, it); }

int main(int argc, char** argv) {
  int dev = 0;
  CK(hipSetDevice(dev));
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, dev));
  const int grid = argc > 1 ? std::atoi(argv[1]) : 2 * pr.multiProcessorCount;
  const int nbar = argc > 2 ? std::atoi(argv[2]) : 400;
  if (grid < 1 || grid > 4 * pr.multiProcessorCount || nbar < 1) {
    std::fprintf(stderr, "grid must be 1..%d (co-resident 256-thread workgroups)\n", 4 * pr.multiProcessorCount);
    return 2;
  }
  unsigned *ctr, *tmo;
  float* buf;
  CK(hipMalloc(&ctr, 64 * 17 * sizeof(unsigned)));
  CK(hipMalloc(&tmo, sizeof(unsigned)));
  CK(hipMalloc(&buf, (size_t)grid * 256 * sizeof(float)));
  CK(hipMemset(buf, 0, (size_t)grid * 256 * sizeof(float)));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < nbar; ++i) hipLaunchKernelGGL(step_kernel, dim3(grid), dim3(256), 0, s, buf, i);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));

  auto med = [](std::vector<float> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  auto run = [&](int which) {
    std::vector<float> t;
    for (int r = 0; r < 6; ++r) {
      CK(hipMemsetAsync(ctr, 0, 64 * 17 * sizeof(unsigned), s));
      CK(hipMemsetAsync(tmo, 0, sizeof(unsigned), s));
      CK(hipEventRecord(e0, s));
      if (which == 0) CK(hipGraphLaunch(ge, s));
      else if (which == 1) hipLaunchKernelGGL(counter_kernel, dim3(grid), dim3(256), 0, s, ctr, tmo, buf, nbar);
      else hipLaunchKernelGGL(xcd_kernel, dim3(grid), dim3(256), 0, s, ctr, tmo, buf, nbar);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      unsigned to = 0;
      CK(hipMemcpy(&to, tmo, sizeof to, hipMemcpyDeviceToHost));
      if (to) {
        std::fprintf(stderr, "barrier timed out (grid %d not co-resident?)\n", grid);
        std::exit(3);
      }
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r) t.push_back(ms);   // the first run warms up
    }
    return med(t) * 1000.0f / nbar;
  };
  const float tg = run(0), tc = run(1), tx = run(2);
  std::printf("{\"grid\": %d, \"cus\": %d, \"barriers\": %d, \"us_per_graph_boundary\": %.3f, "
              "\"us_per_counter_barrier\": %.3f, \"us_per_xcd_barrier\": %.3f}\n",
              grid, pr.multiProcessorCount, nbar, tg, tc, tx);
  return 0;
}
