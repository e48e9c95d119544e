// Standalone timing harness for the row/weight-gradient GEMMs (not part of the product).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Itrpo_amd/csrc tools/gemm_bench.cpp \
//        trpo_amd/csrc/gemm.hip -o tools/gemm_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "kernels.h"
using namespace trpo;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

static float* dalloc(size_t n) { float* p; CK(hipMalloc(&p, n * 4)); CK(hipMemset(p, 0, n * 4)); return p; }

int main(int argc, char** argv) {
  const long M = argc > 1 ? atol(argv[1]) : 8000000;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int K = 256, N = 256;
  float *RH = dalloc((size_t)M * K), *H = dalloc((size_t)M * K), *H2 = dalloc((size_t)M * N), *out = dalloc((size_t)M * N);
  float *E = dalloc((size_t)M * N), *RH2 = dalloc((size_t)M * N);
  float *W = dalloc(2 * K * N), *bias = dalloc(N);
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto run = [&](const char* name, RowEpi epi, int nseg) {
    RowGemmArgs g{};
    g.M = (int)M; g.N = N; g.Npad = N; g.nseg = nseg;
    g.seg[0] = GemmSeg{RH, W, K, N, K};
    g.seg[1] = GemmSeg{H, W + K * N, K, N, K};
    g.epi = epi;
    g.ea.bias = bias; g.ea.H = H2; g.ea.E = E; g.ea.RH = RH2; g.ea.out0 = out; g.ea.out1 = E; g.ea.ldo = N;
    launch_rowgemm(g, 0); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) launch_rowgemm(g, 0);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= reps;
    const double fl = 2.0 * M * N * K * nseg;
    printf("%-28s M=%-9ld %8.3f ms  %6.1f TF/s  %6.3f ms/Mrow\n", name, M, ms, fl / ms / 1e9, ms / (M / 1e6));
  };
  run("rfwd (2seg, RHidden)", RowEpi::kRHidden, 2);
  run("tanh (2seg, no aux load)", RowEpi::kTanh, 2);
  run("rbwd (2seg, RBwd)", RowEpi::kRBwd, 2);
  run("rfwd (1seg, RHidden)", RowEpi::kRHidden, 1);
  // weight gradient 256x256 over M rows, two segments, 512 splits
  {
    const int S = 512;
    long rps = (M + S - 1) / S;
    rps = (rps + 31) / 32 * 32;
    float* slab = dalloc((size_t)S * (N * K + N));
    WGradArgs w{};
    w.rows = (int)M; w.Ma = K; w.Nb = N; w.Mpad = K; w.Npad = N; w.nseg = 2;
    w.seg[0] = WSeg{RH, H2, K, N}; w.seg[1] = WSeg{H, E, K, N}; w.colsum_seg = 1;
    w.splits = (int)((M + rps - 1) / rps); w.rows_per_split = (int)rps; w.slab = slab;
    w.slab_stride = N * K + N; w.off_w = 0; w.off_b = N * K;
    launch_wgrad(w, 0); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) launch_wgrad(w, 0);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= reps;
    const double fl = 2.0 * M * N * K * 2;
    printf("%-28s M=%-9ld %8.3f ms  %6.1f TF/s\n", "wgrad (2seg 256x256)", M, ms, fl / ms / 1e9);
  }
  return 0;
}
