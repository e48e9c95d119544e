// Standalone timing harness for the row/weight-gradient GEMMs (not part of the product).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Itrpo_amd/csrc tools/gemm_bench.cpp \
//        trpo_amd/csrc/gemm.hip -o tools/gemm_bench
// run:   tools/gemm_bench [M] [reps]
// Operands are random (zero data lets the clock run high and overstates throughput).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "kernels.h"
using namespace trpo;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__global__ void fill_kernel(float* p, size_t n, unsigned seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = scale * ((float)(x & 0xffffff) / 16777216.0f * 2.0f - 1.0f);
  }
}
static float* dalloc(size_t n, unsigned seed = 0, float scale = 1.0f) {
  float* p; CK(hipMalloc(&p, n * 4));
  if (seed) hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, p, n, seed, scale);
  else CK(hipMemset(p, 0, n * 4));
  return p;
}

int main(int argc, char** argv) {
  const long M = argc > 1 ? atol(argv[1]) : 8000000;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int K = getenv("GB_K") ? atoi(getenv("GB_K")) : 256, N = 256;   // GB_K: per-segment depth (main-loop length)
  float *RH = dalloc((size_t)M * K, 11), *H = dalloc((size_t)M * K, 12), *Hz = dalloc((size_t)M * N);
  float *out = dalloc((size_t)M * N), *E = dalloc((size_t)M * N, 13), *RH2 = dalloc((size_t)M * N, 14);
  float *W = dalloc(2 * K * N, 15, 0.0625f), *bias = dalloc(N);
  uint16_t* W3; CK(hipMalloc(&W3, (size_t)2 * 3 * N * K * 2));
  auto split = [&](int f16) {
    SplitArgs sa{};
    sa.n = 2;
    sa.f16 = f16;
    sa.job[0] = SplitJob{W, W3, K, N, N, K};
    sa.job[1] = SplitJob{W + K * N, W3 + (size_t)3 * N * K, K, N, N, K};
    launch_split_b(sa, nullptr, 0);
    CK(hipDeviceSynchronize());
  };
  int f16 = 0;
  split(0);
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto mkargs = [&](RowEpi epi, int nseg, const float* Haux) {
    RowGemmArgs g{};
    g.M = (int)M; g.N = N; g.Npad = N; g.nseg = nseg;
    const int lda = getenv("GB_LDA0") ? 0 : K;   // 0: every row re-reads row 0 (L2-resident A: main loop without HBM)
    g.seg[0] = GemmSeg{RH, W, lda, N, K, W3, K, N * K};
    g.seg[1] = GemmSeg{H, W + K * N, lda, N, K, W3 + (size_t)3 * N * K, K, N * K};
    g.epi = epi;
    g.f16 = f16;
    g.ea.bias = bias; g.ea.H = Haux; g.ea.E = E; g.ea.RH = RH2; g.ea.out0 = out; g.ea.out1 = E; g.ea.ldo = N;
    return g;
  };
  auto run = [&](const char* name, RowEpi epi, int nseg) {
    RowGemmArgs g = mkargs(epi, nseg, RH2);
    launch_rowgemm(g, 0); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) launch_rowgemm(g, 0);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= reps;
    const double fl = 2.0 * M * N * K * nseg;
    printf("split=%d f16=%d %-24s M=%-9ld %8.3f ms  %6.1f TF/s\n", g_options.split_mfma, f16, name, M, ms,
           fl / ms / 1e9);
  };
  // accuracy: out = acc (PgBwd with H = 0), sampled rows vs an fp64 host product
  auto accuracy = [&]() {
    RowGemmArgs g = mkargs(RowEpi::kPgBwd, 2, Hz);
    launch_rowgemm(g, 0); CK(hipDeviceSynchronize());
    const int rows = 64;
    std::vector<float> hA((size_t)rows * K), hB((size_t)rows * K), hW(2 * K * N), hO((size_t)rows * N);
    double maxrel = 0, sumsq = 0, refsq = 0;
    for (int t = 0; t < 4; ++t) {
      const size_t r0 = (size_t)(M - rows) * t / 3;
      CK(hipMemcpy(hA.data(), RH + r0 * K, hA.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hB.data(), H + r0 * K, hB.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hW.data(), W, hW.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hO.data(), out + r0 * N, hO.size() * 4, hipMemcpyDeviceToHost));
      for (int i = 0; i < rows; ++i)
        for (int j = 0; j < N; ++j) {
          double s = 0, sa2 = 0;
          for (int k = 0; k < K; ++k) {
            const double p0 = (double)hA[i * K + k] * hW[k * N + j], p1 = (double)hB[i * K + k] * hW[K * N + k * N + j];
            s += p0 + p1;
            sa2 += fabs(p0) + fabs(p1);
          }
          const double err = fabs(hO[i * N + j] - s);
          maxrel = fmax(maxrel, err / sa2);
          sumsq += err * err;
          refsq += s * s;
        }
    }
    printf("split=%d f16=%d accuracy: max |err|/sum|a b| = %.3e   rel-l2 = %.3e\n", g_options.split_mfma, f16, maxrel,
           sqrt(sumsq / refsq));
  };
  // modes: split tile config (0 = f32 MFMA), +100 = f16 planes
  std::vector<int> modes = {105, 110, 111};
  if (argc > 3) modes = {atoi(argv[3])};   // one split mode only (profiling)
  for (int mode : modes) {
    g_options.split_mfma = mode % 100;
    if (f16 != mode / 100) {
      f16 = mode / 100;
      split(f16);
    }
    accuracy();
    run("rfwd (2seg, RHidden)", RowEpi::kRHidden, 2);
    run("rbwd (2seg, RBwd)", RowEpi::kRBwd, 2);
    run("tanh (2seg)", RowEpi::kTanh, 2);
  }
  g_options.split_mfma = 0;
  if (argc > 3) return 0;
  // weight gradient 256x256 over M rows, two segments, 512 splits
  {
    const int S = 512;
    long rps = (M + S - 1) / S;
    rps = (rps + 31) / 32 * 32;
    float* slab = dalloc((size_t)S * (N * K + N));
    WGradArgs w{};
    w.rows = (int)M; w.Ma = K; w.Nb = N; w.Mpad = K; w.Npad = N; w.nseg = 2;
    w.seg[0] = WSeg{RH, RH2, K, N}; w.seg[1] = WSeg{H, E, K, N}; w.colsum_seg = 1;
    w.splits = (int)((M + rps - 1) / rps); w.rows_per_split = (int)rps; w.slab = slab;
    w.slab_stride = N * K + N; w.off_w = 0; w.off_b = N * K;
    for (int mode : {0, 1, 2, 3, 101, 102, 103}) {
      g_options.split_wg = mode % 100;
      w.f16 = mode / 100;
      launch_wgrad(w, 0); CK(hipDeviceSynchronize());
      CK(hipEventRecord(a));
      for (int i = 0; i < reps; ++i) launch_wgrad(w, 0);
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= reps;
      const double fl = 2.0 * M * N * K * 2;
      printf("split_wg=%d %-22s M=%-9ld %8.3f ms  %6.1f TF/s\n", mode, "wgrad (2seg 256x256)", M, ms, fl / ms / 1e9);
    }
  }
  return 0;
}
