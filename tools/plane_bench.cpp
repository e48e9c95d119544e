// Standalone A/B of the pre-split-plane row GEMM (plane.hip) against the register-staged split row GEMM
// (gemm.hip rowgemm3, config 5) on the C4 FVP shapes (not part of the product).
// build (after `make -C trpo_amd/csrc`):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Itrpo_amd/csrc tools/plane_bench.cpp \
//     build/csrc/gemm.hip.o build/csrc/plane.hip.o build/csrc/vec.hip.o -o tools/plane_bench
// run: tools/plane_bench [M] [reps]
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
template <class T> static T* dalloc(size_t n) { T* p; CK(hipMalloc(&p, n * sizeof(T))); CK(hipMemset(p, 0, n * sizeof(T))); return p; }
static float* frand(size_t n, unsigned seed, float scale = 1.0f) {
  float* p = dalloc<float>(n);
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, p, n, seed, scale);
  return p;
}

int main(int argc, char** argv) {
  const long M = argc > 1 ? atol(argv[1]) : 8000000;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int K = 256, N = 256;
  const long Mp = (M + 255) / 256 * 256;
  float *RH = frand((size_t)M * K, 11), *H = frand((size_t)M * K, 12), *Dsm = frand((size_t)M * K, 17, 1.0f / 1048576.0f);
  float *Haux = frand((size_t)M * N, 14, 0.9f), *E = frand((size_t)M * N, 13, 1e-6f), *RH2 = frand((size_t)M * N, 15);
  float *out0 = dalloc<float>((size_t)M * N), *out1 = dalloc<float>((size_t)M * N);
  float *W = frand(2 * K * N, 16, 0.0625f), *bias = frand(N, 18, 0.1f);
  unsigned* am = dalloc<unsigned>((size_t)8 * kAmaxSlot);
  unsigned *amRH = am, *amH = am + kAmaxSlot, *amD = am + 2 * kAmaxSlot, *amW0 = am + 3 * kAmaxSlot,
           *amW1 = am + 4 * kAmaxSlot, *amOut = am + 5 * kAmaxSlot;
  launch_amax(RH, M, K, K, amRH, 0);
  launch_amax(H, M, K, K, amH, 0);
  launch_amax(Dsm, M, K, K, amD, 0);
  launch_amax(W, K, N, N, amW0, 0);
  launch_amax(W + K * N, K, N, N, amW1, 0);
  uint16_t* W3 = dalloc<uint16_t>((size_t)2 * 2 * N * K);
  {
    SplitArgs sa{};
    sa.n = 2;
    sa.f16 = 1;
    sa.job[0] = SplitJob{W, W3, K, N, N, K, amW0};
    sa.job[1] = SplitJob{W + K * N, W3 + (size_t)2 * N * K, K, N, N, K, amW1};
    launch_split_b(sa, nullptr, 0);
  }
  uint16_t* W3b = dalloc<uint16_t>((size_t)2 * 2 * N * K);   // k-blocked copies for the planes path
  launch_block_planes(W3, 2, N, K, W3b, 0);
  launch_block_planes(W3 + (size_t)2 * N * K, 2, N, K, W3b + (size_t)2 * N * K, 0);
  uint16_t *RHh = dalloc<uint16_t>((size_t)Mp * K), *RHl = dalloc<uint16_t>((size_t)Mp * K);
  uint16_t *Hh = dalloc<uint16_t>((size_t)Mp * K), *Hl = dalloc<uint16_t>((size_t)Mp * K);
  uint16_t *Dh = dalloc<uint16_t>((size_t)Mp * K), *Dl = dalloc<uint16_t>((size_t)Mp * K);
  int* es = dalloc<int>(8);
  launch_split_planes(RH, (int)M, (int)Mp, K, K, RHh, RHl, K, amRH, es + 0, 0);
  launch_split_planes(H, (int)M, (int)Mp, K, K, Hh, Hl, K, amH, es + 1, 0);
  launch_split_planes(Dsm, (int)M, (int)Mp, K, K, Dh, Dl, K, amD, es + 2, 0);
  CK(hipDeviceSynchronize());

  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  // case: 0 = rfwd (RH W0 + H W1, kRHidden), 1 = rbwd (RH W0 + Dsm W1, kRBwd; low segment on one product),
  //       2 = rfwd_l0-like (one segment, K = 128, kRHidden); decomposition: 3 = case 0's k-loop with a
  //       store-only epilogue (kTanh), 4 = case 1's k-loop, store-only, 5 = case 1's epilogue behind a
  //       64-deep k-loop, 6 = case 0's epilogue behind a 64-deep k-loop
  auto mk = [&](int cs, bool planes) {
    RowGemmArgs g{};
    g.M = (int)M; g.N = N; g.Npad = N; g.f16 = 1;
    const bool low = cs == 1 || cs == 4;
    const float* A1 = low ? Dsm : H;
    const unsigned* am1 = low ? amD : amH;
    g.nseg = (cs == 2 || cs >= 5) ? 1 : 2;
    g.seg[0] = GemmSeg{RH, W, K, N, cs == 2 ? 128 : (cs >= 5 ? 64 : K), W3, K, N * K, amRH, amW0};
    g.seg[1] = GemmSeg{A1, W + K * N, K, N, K, W3 + (size_t)2 * N * K, K, N * K, am1, amW1};
    if (planes) {
      g.seg[0].Ah = RHh; g.seg[0].Al = RHl; g.seg[0].ldp = K; g.seg[0].mpad = (int)Mp; g.seg[0].eAp = es + 0;
      g.seg[0].Bb = W3b;
      g.seg[1].Ah = low ? Dh : Hh; g.seg[1].Al = low ? Dl : Hl; g.seg[1].ldp = K; g.seg[1].mpad = (int)Mp;
      g.seg[1].eAp = es + (low ? 2 : 1);
      g.seg[1].Bb = W3b + (size_t)2 * N * K;
    }
    g.epi = (cs == 1 || cs == 5) ? RowEpi::kRBwd : ((cs == 3 || cs == 4) ? RowEpi::kTanh : RowEpi::kRHidden);
    g.ea.bias = bias; g.ea.H = Haux; g.ea.E = E; g.ea.RH = RH2; g.ea.ldo = N;
    g.ea.out0 = planes ? out1 : out0;
    g.ea.amax0 = amOut;
    return g;
  };
  const char* names[7] = {"rfwd_l1 (2seg K=2x256, RHidden)", "rbwd_l1 (2seg, low seg, RBwd)", "rfwd_l0 (1seg K=128)",
                          "rfwd_l1 k-loop + store", "rbwd_l1 k-loop + store", "rbwd_l1 epilogue (K=64)",
                          "rfwd_l1 epilogue (K=64)"};
  const int c0 = argc > 3 ? atoi(argv[3]) : 0, c1 = argc > 4 ? atoi(argv[4]) : 7;
  for (int cs = c0; cs < c1; ++cs) {
    double tm[2] = {0, 0};
    for (int pl = 0; pl < 2; ++pl) {
      RowGemmArgs g = mk(cs, pl == 1);
      launch_rowgemm(g, 0);
      CK(hipDeviceSynchronize());
    }
    // accuracy: new vs old output, sampled
    {
      const size_t n = (size_t)M * N;
      std::vector<float> o0(1 << 20), o1(1 << 20);
      double md = 0, mx = 0;
      for (int part = 0; part < 4; ++part) {
        const size_t off = (n - o0.size()) / 3 * part;
        CK(hipMemcpy(o0.data(), out0 + off, o0.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(o1.data(), out1 + off, o1.size() * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < o0.size(); ++i) {
          md = fmax(md, fabs((double)o0[i] - o1[i]));
          mx = fmax(mx, fabs((double)o0[i]));
        }
      }
      printf("%-34s planes vs register path: max |diff| / max |out| = %.3e\n", names[cs], md / mx);
    }
    // interleaved timing rounds (same process: rule 24)
    for (int round = 0; round < 3; ++round)
      for (int pl = 0; pl < 2; ++pl) {
        RowGemmArgs g = mk(cs, pl == 1);
        CK(hipEventRecord(a));
        for (int i = 0; i < reps; ++i) launch_rowgemm(g, 0);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        tm[pl] += ms / reps / 3;
      }
    printf("%-34s M=%ld  register-staged %7.3f ms   planes %7.3f ms   (%.2fx)\n", names[cs], M, tm[0], tm[1],
           tm[0] / tm[1]);
    fflush(stdout);
  }
  return 0;
}
