// Discounted-return segmented reverse scan and advantage standardisation.
//
// discount (utils.py:14-16; called per path at trpo_inksci.py:102-104):
//   y[t] = x[t] + gamma * y[t+1]      inside an episode (float64, as scipy's lfilter).
// The whole concatenated batch is scanned at once; starts[t] = 1 marks the
// first step of an episode, which cuts the carry.  Each element is the affine
// map f_t(c) = x_t + a_t c with a_t = gamma (0 when t+1 starts an episode or
// is past the end); maps compose associatively, (A1,B1)o(A2,B2) = (A1 A2, B1 + A1 B2).
//
// Three passes: (1) per-thread chunks of kChunk elements -> thread maps ->
// block map; (2) one block scans the block maps (reverse, exclusive);
// (3) each thread re-walks its chunk sequentially from its carry-in, i.e.
// inside a chunk the arithmetic is exactly the reference's recurrence.
//
// standardisation (trpo_inksci.py:105,115-117): adv = returns - baseline;
// adv -= mean; adv /= std + 1e-8 (population std, float64), then cast to
// float32 as the TF placeholder does (:34,:121).
#include "common.h"
#include "kernels.h"

#pragma clang fp contract(off)

namespace trpo {

namespace {

constexpr int kChunk = 16;
constexpr int kScanThreads = 256;
constexpr int kTile = kChunk * kScanThreads;

struct Aff {
  double A, B;
};

// F covers earlier elements, G later ones: (F o G)(c) = F(G(c))
__device__ __forceinline__ Aff compose(Aff F, Aff G) { return Aff{F.A * G.A, F.B + F.A * G.B}; }

__device__ __forceinline__ double coef(const uint8_t* starts, int64_t t, int64_t n, double gamma) {
  return (t + 1 < n && !starts[t + 1]) ? gamma : 0.0;
}

// The block's tile of x goes through LDS: loaded and stored by consecutive threads (coalesced), walked by each
// thread over its own kChunk elements.  A pad double every kChunk keeps the walk conflict-free (thread j's chunk
// starts at 8 (kChunk + 1) j bytes: the 32 lanes of a ds_read_b64 group cover the 64 banks once).  The strided
// global walk it replaces read 8 B per 128-B line per instruction (C4: 0.38 ms for pass 3).
constexpr int kPadT = kTile + kTile / kChunk;
__device__ __forceinline__ int sidx(int i) { return i + i / kChunk; }
__device__ void tile_load(const double* x, int64_t T0, int64_t n, double* sx) {
  for (int i = threadIdx.x; i < kTile; i += blockDim.x) sx[sidx(i)] = T0 + i < n ? x[T0 + i] : 0.0;
  __syncthreads();
}

// thread map of elements [t0, t1) (x's tile in LDS from T0)
__device__ Aff chunk_map(const double* sx, int64_t T0, const uint8_t* starts, int64_t t0, int64_t t1, int64_t n,
                         double gamma) {
  Aff m{1.0, 0.0};
  for (int64_t t = t1 - 1; t >= t0; --t) {
    const double a = coef(starts, t, n, gamma);
    m = Aff{a * m.A, sx[sidx((int)(t - T0))] + a * m.B};
  }
  return m;
}

// Block-wide reverse exclusive scan of maps: returns S_j = G_{j+1} o ... o G_{T-1}
// (identity for the last thread) and the block total G_0 o ... o G_{T-1}.
__device__ void block_rscan(Aff g, Aff& excl, Aff& total) {
  __shared__ Aff wtot[kScanThreads / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  // inclusive suffix within the wave: lane's map composed with all later lanes
  Aff inc = g;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const double oA = __shfl_down(inc.A, off, 64);
    const double oB = __shfl_down(inc.B, off, 64);
    if (lane + off < 64) inc = compose(inc, Aff{oA, oB});
  }
  Aff ex{__shfl_down(inc.A, 1, 64), __shfl_down(inc.B, 1, 64)};
  if (lane == 63) ex = Aff{1.0, 0.0};
  if (lane == 0) wtot[wave] = inc;
  __syncthreads();
  // suffix of the later waves
  Aff later{1.0, 0.0};
  for (int w = nw - 1; w > wave; --w) later = compose(wtot[w], later);
  excl = compose(ex, later);
  Aff tot{1.0, 0.0};
  for (int w = nw - 1; w >= 0; --w) tot = compose(wtot[w], tot);
  total = tot;
  __syncthreads();
}

__global__ void __launch_bounds__(kScanThreads)
scan_pass1(const double* x, const uint8_t* starts, int64_t n, double gamma, Aff* blockmaps) {
  __shared__ double sx[kPadT];
  const int64_t T0 = (int64_t)blockIdx.x * kTile;
  tile_load(x, T0, n, sx);
  const int64_t t0 = T0 + (int64_t)threadIdx.x * kChunk;
  const int64_t t1 = t0 + kChunk < n ? t0 + kChunk : n;
  Aff g = t0 < n ? chunk_map(sx, T0, starts, t0, t1, n, gamma) : Aff{1.0, 0.0};
  Aff ex, tot;
  block_rscan(g, ex, tot);
  if (threadIdx.x == 0) blockmaps[blockIdx.x] = tot;
}

// one block: carry[b] = (G_{b+1} o ... o G_{nb-1})(0)
__global__ void __launch_bounds__(kScanThreads)
scan_pass2(const Aff* blockmaps, int64_t nb, double* carry) {
  const int64_t per = (nb + blockDim.x - 1) / blockDim.x;
  const int64_t b0 = (int64_t)threadIdx.x * per;
  const int64_t b1 = b0 + per < nb ? b0 + per : nb;
  Aff g{1.0, 0.0};
  for (int64_t b = b1 - 1; b >= b0; --b) g = compose(blockmaps[b], g);
  Aff ex, tot;
  block_rscan(g, ex, tot);
  // walk this thread's blocks from its carry-in
  double c = ex.B;   // (suffix)(0)
  for (int64_t b = b1 - 1; b >= b0; --b) {
    carry[b] = c;
    c = blockmaps[b].B + blockmaps[b].A * c;
  }
}

__global__ void __launch_bounds__(kScanThreads)
scan_pass3(const double* x, const uint8_t* starts, int64_t n, double gamma, const double* carry,
           double* y) {
  __shared__ double sx[kPadT];
  const int64_t T0 = (int64_t)blockIdx.x * kTile;
  tile_load(x, T0, n, sx);
  const int64_t t0 = T0 + (int64_t)threadIdx.x * kChunk;
  const int64_t t1 = t0 + kChunk < n ? t0 + kChunk : n;
  Aff g = t0 < n ? chunk_map(sx, T0, starts, t0, t1, n, gamma) : Aff{1.0, 0.0};
  Aff ex, tot;
  block_rscan(g, ex, tot);
  double c = ex.B + ex.A * carry[blockIdx.x];
  for (int64_t t = t1 - 1; t >= t0; --t) {
    // carry across t -> t+1 is cut when t+1 starts an episode; y replaces x in this thread's own LDS slots
    const double a = coef(starts, t, n, gamma);
    c = sx[sidx((int)(t - T0))] + a * c;
    sx[sidx((int)(t - T0))] = c;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kTile && T0 + i < n; i += blockDim.x) y[T0 + i] = sx[sidx(i)];
}

__global__ void adv_center_partials_kernel(const double* returns, const double* baseline, double* adv,
                                           int64_t n, double* partials) {
  __shared__ double scratch[kRedThreads / 64];
  double v = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double a = baseline ? returns[i] - baseline[i] : returns[i];
    adv[i] = a;
    v += a;
  }
  v = block_sum_d(v, scratch);
  if (threadIdx.x == 0) partials[blockIdx.x] = v;
}

__global__ void sum_finish_kernel(const double* partials, double* out) {
  __shared__ double scratch[kRedThreads / 64];
  const double v = sum_partials(partials, kRedBlocks, scratch);
  if (threadIdx.x == 0) out[0] = v;
}

__global__ void adv_sq_partials_kernel(const double* adv, int64_t n, const double* gsum, double inv_n,
                                       double* partials) {
  __shared__ double scratch[kRedThreads / 64];
  const double mean = gsum[0] * inv_n;
  double v = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double d = adv[i] - mean;
    v += d * d;
  }
  v = block_sum_d(v, scratch);
  if (threadIdx.x == 0) partials[blockIdx.x] = v;
}

__global__ void adv_normalize_kernel(double* adv, float* adv32, int64_t n, const double* gsum,
                                     const double* gsq, double inv_n) {
  const double mean = gsum[0] * inv_n;
  const double denom = sqrt(gsq[0] * inv_n) + 1e-8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double a = (adv[i] - mean) / denom;
    adv[i] = a;
    if (adv32) adv32[i] = (float)a;
  }
}

}  // namespace

size_t discount_workspace_bytes(int64_t n) {
  const int64_t nb = (n + kTile - 1) / kTile;
  return (size_t)(nb > 0 ? nb : 1) * (sizeof(Aff) + sizeof(double)) + 256;
}

void launch_discount(const double* x, const uint8_t* starts, int64_t n, double gamma, double* out,
                     void* workspace, hipStream_t s) {
  if (n <= 0) return;
  const int64_t nb = (n + kTile - 1) / kTile;
  Aff* maps = reinterpret_cast<Aff*>(workspace);
  double* carry = reinterpret_cast<double*>(maps + nb);
  hipLaunchKernelGGL(scan_pass1, dim3((unsigned)nb), dim3(kScanThreads), 0, s, x, starts, n, gamma, maps);
  hipLaunchKernelGGL(scan_pass2, dim3(1), dim3(kScanThreads), 0, s, maps, nb, carry);
  hipLaunchKernelGGL(scan_pass3, dim3((unsigned)nb), dim3(kScanThreads), 0, s, x, starts, n, gamma, carry,
                     out);
}

void launch_adv_center_partials(const double* returns, const double* baseline, double* adv, int64_t n,
                                double* partials, hipStream_t s) {
  hipLaunchKernelGGL(adv_center_partials_kernel, dim3(kRedBlocks), dim3(kRedThreads), 0, s, returns,
                     baseline, adv, n, partials);
}

void launch_sum_finish(const double* partials, double* out, hipStream_t s) {
  hipLaunchKernelGGL(sum_finish_kernel, dim3(1), dim3(kRedThreads), 0, s, partials, out);
}

void launch_adv_sq_partials(const double* adv, int64_t n, const double* global_sum, double inv_n,
                            double* partials, hipStream_t s) {
  hipLaunchKernelGGL(adv_sq_partials_kernel, dim3(kRedBlocks), dim3(kRedThreads), 0, s, adv, n, global_sum,
                     inv_n, partials);
}

void launch_adv_normalize(double* adv, float* adv32, int64_t n, const double* global_sum,
                          const double* global_sq, double inv_n, hipStream_t s) {
  int64_t g = (n + 255) / 256;
  if (g < 1) g = 1;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(adv_normalize_kernel, dim3((unsigned)g), dim3(256), 0, s, adv, adv32, n, global_sum,
                     global_sq, inv_n);
}

}  // namespace trpo
