// Fused small-width Fisher-vector product on the f16 split (gfx950 / CDNA4).
//
// The whole FVP of trpo_inksci.py:56-70 (Pearlmutter's R-operator) for a policy
// with one or two tanh hidden layers of width <= 64 (NH = 1: the reference's own [64] policy, trpo_inksci.py:38-40;
// NH = 2: C2, C3), obs <= 128 and <= 32 actions in one persistent launch per shard.  Hidden widths below 64 run on
// images padded to 64 features with zero weights (the image builder; padded features are tanh(0) = 0 with zero
// tangents and deltas, so they add exact zeros), structured structured as fused.hip (16 states per wave through the R-forward, the R-softmax head
// and the R-backward in MFMA accumulator layout; per-group weight-gradient passes over two LDS images;
// one slab per workgroup) with three differences:
//
//  * Arithmetic.  Every product runs on v_mfma_f32_16x16x32_f16 with each f32 operand scaled by a power of
//    two and split into f16 hi + lo (3 products, 2^-21 relative per operand; gemm.hip rowgemm3 / tail.hip),
//    where fused.hip takes 6 bf16 products.  Half the MFMAs, 2/3 of the image and weight-chunk bytes.
//  * Scales.  Weights: one exponent per image job, set by the image builder from the job's max |w|.
//    X, D_1, D_2: the engine's running-max slots.  H: fixed (|tanh| <= 1).  Values produced in the launch
//    (RH_1, RH_2, the head's RD, RD_1, RD_0) take a per-state exponent as B operands of the chain steps (the
//    max over the state's features: 4 lanes) and a per-group exponent in the gradient-pass images, whose
//    k dimension runs over states (the wave maxima meet in LDS behind a barrier the pass has anyway).
//    A chain step's two segments carry different scales: the accumulator is rescaled by the power of two
//    between them, and every accumulator is unscaled to true f32 values before it is used or summed.
//  * Shapes are compile-time (hidden tiles 4, obs tiles TI0, head tiles OTA): no runtime-width branches.
//    Weight chunks stream through two LDS buffers (one barrier per chunk); the next group's first chunk
//    and first X chunk are loaded during the current group's last pass.
//
// States past the shard end read zeros (buffer descriptors): their D / RD and contributions are exactly 0.
#include "chain_common.h"
#include "rowepi.h"

#include <algorithm>
#include <stdexcept>
#include <type_traits>

#ifndef FUSED16_FW
#define FUSED16_FW 4   // waves per workgroup (16 states each)
#endif
#ifndef FUSED16_LB
#define FUSED16_LB 2   // workgroups per CU the register budget is sized for
#endif
// Ablation builds for profiling only (tools/variant.sh; never the shipped library): bit 0 = no per-state
// activation loads, 1 = no gradient passes, 2 = no weight-chunk loads, 3 = no chunk barriers, 4 = no weight-chunk
// loads with the chunks' LDS stores kept
#ifndef FUSED16_ABL
#define FUSED16_ABL 0
#endif
#ifndef FUSED16_RING
#define FUSED16_RING 2   // memory-sourced B chunks loaded this many chunks ahead
#endif
#ifndef FUSED16_WSETS
#define FUSED16_WSETS 2   // weight chunks in flight (register sets)
#endif
#ifndef FUSED16_REUSE
#define FUSED16_REUSE 1   // H_1 / H_2 tiles loaded once per group and reused as later steps' memory segments (1), and
                          // H_1 also for the layer-1 pass and R-backward epilogue (2); 0: each step loads its own
#endif
#ifndef FUSED16_PFEARLY
#define FUSED16_PFEARLY 1   // 1: a step's epilogue operand is loaded before its register segment, not its memory one
#endif
#ifndef FUSED16_DMA
#define FUSED16_DMA 1   // 1: weight chunks stream by LDS-DMA into a 3-slot ring; 0: through two register sets
#endif


namespace trpo {
namespace {

typedef _Float16 fh8 __attribute__((ext_vector_type(8)));
typedef __fp16 fp16x2 __attribute__((ext_vector_type(2)));
typedef unsigned cu32x2 __attribute__((ext_vector_type(2)));

// (a, b) * 1 -> packed f16 hi pair and lo pair, round toward zero: a - hi is exact in f32 and below
// ulp16(a), so hi + lo is within 2^-21 |a| (tail.hip split8)
// (returned as {hi pair, lo pair})
__device__ __forceinline__ cu32x2 split2(float a, float b) {
  const fp16x2 hp = __builtin_amdgcn_cvt_pkrtz(a, b);
  const fp16x2 lp = __builtin_amdgcn_cvt_pkrtz(a - (float)hp[0], b - (float)hp[1]);
  return cu32x2{__builtin_bit_cast(unsigned, hp), __builtin_bit_cast(unsigned, lp)};
}

// B operand (hi, lo) of v_mfma_f32_16x16x32_f16 from two acc-layout tiles times s (chain_mkb's k order)
__device__ __forceinline__ void mkb16(const f32x4& x0, const f32x4& x1, float s, fh8 (&b)[2]) {
  const cu32x2 p0 = split2(x0[0] * s, x0[1] * s), p1 = split2(x0[2] * s, x0[3] * s);
  const cu32x2 p2 = split2(x1[0] * s, x1[1] * s), p3 = split2(x1[2] * s, x1[3] * s);
  const cu32x4 H = {p0[0], p1[0], p2[0], p3[0]}, L = {p0[1], p1[1], p2[1], p3[1]};
  b[0] = __builtin_bit_cast(fh8, H);
  b[1] = __builtin_bit_cast(fh8, L);
}

// c += a b over the split: al bh + ah bl + ah bh, smallest terms first
__device__ __forceinline__ f32x4 mfma3(const fh8 (&a)[2], const fh8 (&b)[2], f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[0], c, 0, 0, 0);
  return c;
}

__device__ __forceinline__ f32x4 ldexp4(const f32x4& x, int e) {
  f32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = __builtin_amdgcn_ldexpf(x[i], e);
  return r;
}

// max |x| over the first N acc-layout tiles of this lane, then over the 4 lanes of the same state
// (l, l^16, l^32, l^48): the state's max over all its features, on every one of its lanes
template <int N>
__device__ __forceinline__ float state_max(const f32x4 (&x)[4]) {
  float m = 0.0f;
#pragma unroll
  for (int t = 0; t < N; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) m = fmaxf(m, fabsf(x[t][j]));
  return xmax_f<false>(xmax_f<true>(m));
}

// max over the 16 lanes of a row (DPP; every lane of the row ends with it)
__device__ __forceinline__ float max16_dpp(float v) {
  v = fmaxf(v, dpp_f<kDppX1>(v));
  v = fmaxf(v, dpp_f<kDppX2>(v));
  v = fmaxf(v, dpp_f<kDppHalfMirror>(v));
  return fmaxf(v, dpp_f<kDppMirror>(v));
}

// ---------------------------------------------------------------------------------------------------------
// weight images: the chain's layout (chain.hip chain_img_kernel) with 2 f16 planes, scaled per job.  Every
// block of a job takes the job's max |w| itself (<= 128 x 64 values), so one launch does it all.
// ---------------------------------------------------------------------------------------------------------
constexpr int kImgMax = 128 * 64;   // the largest weight matrix of an eligible shape
__global__ void __launch_bounds__(256) fused16_img_kernel(const ChainImgArgs a, const float* theta, const float* v,
                                                          int which, const int* skip, int* img_e) {
  __shared__ float red[4];
  if (skip && *skip) return;
  const ChainImgJob& j = a.job[blockIdx.y];
  if (j.which != which) return;
  const float* src = (which ? v : theta) + j.src_off;
  // this thread's 8 image values, loaded with the max's loads (one round trip to memory, not two)
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const bool live = idx < j.kc * j.otp * 4;
  const int gg = idx & 3;
  const int o = (idx >> 2) % j.otp;
  const int c = (idx >> 2) / j.otp;
  float x[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int k = 32 * c + chain_perm(8 * gg + q);
    const bool in = live && o < j.O && k < j.K;
    const float val = src[in ? (j.trans ? o * j.ldw + k : k * j.ldw + o) : 0];
    x[q] = in ? val : 0.0f;
  }
  float m = 0.0f;
  const int last = j.K * j.O - 1;   // W_l is K x O or O x K, dense, at most 128 x 64: 32 loads in flight per lane
#pragma unroll
  for (int u = 0; u < kImgMax / 256; ++u) m = fmaxf(m, fabsf(src[min((int)threadIdx.x + 256 * u, last)]));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const int e = f16_scale_exp(m);
  if (blockIdx.x == 0 && threadIdx.x == 0) img_e[blockIdx.y] = e;
  if (!live) return;
  const float sc = __builtin_ldexpf(1.0f, e);
#pragma unroll
  for (int q = 0; q < 8; ++q) x[q] *= sc;
  cu32x4 H, L;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const cu32x2 p = split2(x[2 * i], x[2 * i + 1]);
    H[i] = p[0];
    L[i] = p[1];
  }
  unsigned short* dst = a.img + j.dst_off + (size_t)c * 2 * j.otp * 32 + o * 32 + ((gg ^ chain_hsw(o)) << 3);
  *reinterpret_cast<cu32x4*>(dst) = H;
  *reinterpret_cast<cu32x4*>(dst + (size_t)j.otp * 32) = L;
}

// The CG's p update (utils.py:196-198, vec.hip cg_p_kernel) fused with the next FVP's V images (fused16_img_kernel,
// which = 1) in one launch: p_new = r + mu p_old goes to a second buffer (the image blocks read p_old and r while the
// writer blocks write p_new), and every image block forms the p_new values of its job itself (the job's max too).
// blockIdx.y < jobs: image blocks; blockIdx.y == jobs: the writer blocks (grid-stride over P).  mu and the scalars
// as cg_p_kernel (256-thread blocks, the same fixed-order sum of the r.r partials): bit-identical.
__global__ void __launch_bounds__(256) cg_p_img16_kernel(const ChainImgArgs a, const float* r, const float* p_old,
                                                         float* p_new, int64_t n, UpdScalars* sc,
                                                         const double* partials2, CGFlags* fl, int it, int* img_e) {
#pragma clang fp contract(off)
  __shared__ double scratch[kRedThreads / 64];
  __shared__ float red[4];
  const bool writer = (int)blockIdx.y == a.n;
  if (fl->done[it]) {   // converged: a no-op, and so is every later iteration (cg_p_kernel)
    if (writer && blockIdx.x == 0 && threadIdx.x == 0) fl->done[it + 1] = 1;
    return;
  }
  if (!writer && a.job[blockIdx.y].which != 1) return;
  const float newrdotr = (float)sum_partials(partials2, kRedBlocks, scratch);
  const float rdotr = sc->rdotr[it & 1];
  const float mu = newrdotr / rdotr;
  if (writer) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
      p_new[i] = r[i] + mu * p_old[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      sc->mu = mu;
      sc->rdotr[(it + 1) & 1] = newrdotr;
      sc->iters = it + 1;
      fl->done[it + 1] = (newrdotr < sc->tol) ? 1 : 0;
    }
    return;
  }
  const ChainImgJob& j = a.job[blockIdx.y];
  const float* rs = r + j.src_off;
  const float* ps = p_old + j.src_off;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const bool live = idx < j.kc * j.otp * 4;
  const int gg = idx & 3;
  const int o = (idx >> 2) % j.otp;
  const int c = (idx >> 2) / j.otp;
  float x[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int k = 32 * c + chain_perm(8 * gg + q);
    const bool in = live && o < j.O && k < j.K;
    const int e = in ? (j.trans ? o * j.ldw + k : k * j.ldw + o) : 0;
    const float val = rs[e] + mu * ps[e];
    x[q] = in ? val : 0.0f;
  }
  float m = 0.0f;
  const int last = j.K * j.O - 1;
#pragma unroll
  for (int u = 0; u < kImgMax / 256; ++u) {
    const int e = min((int)threadIdx.x + 256 * u, last);
    m = fmaxf(m, fabsf(rs[e] + mu * ps[e]));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const int e = f16_scale_exp(m);
  if (blockIdx.x == 0 && threadIdx.x == 0) img_e[blockIdx.y] = e;
  if (!live) return;
  const float sc2 = __builtin_ldexpf(1.0f, e);
#pragma unroll
  for (int q = 0; q < 8; ++q) x[q] *= sc2;
  cu32x4 H, L;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const cu32x2 pp = split2(x[2 * i], x[2 * i + 1]);
    H[i] = pp[0];
    L[i] = pp[1];
  }
  unsigned short* dst = a.img + j.dst_off + (size_t)c * 2 * j.otp * 32 + o * 32 + ((gg ^ chain_hsw(o)) << 3);
  *reinterpret_cast<cu32x4*>(dst) = H;
  *reinterpret_cast<cu32x4*>(dst + (size_t)j.otp * 32) = L;
}

// image jobs (kernels.h, kFused16Jobs): NH = 2: V_0 | W_1 V_1 | W_2 V_2 | W_2^T V_2^T | W_1^T V_1^T;
// NH = 1: V_0 | W_1 V_1 | W_1^T V_1^T
enum { jV0 = 0, jW1, jV1, jW2, jV2, jW2t, jV2t, jW1t, jV1t };
template <int NH> constexpr int fused16_jobs() { return NH == 2 ? 9 : 5; }
template <int NH> constexpr int job_w1t() { return NH == 2 ? jW1t : 3; }

// FW = waves per workgroup, TI0 = 16-feature tiles of obs (1, 2, 4, 8), OTA = 16-action tiles of the head;
// MODE: 0 the FVP; 1 the policy gradient instead (the same machinery on the backward chain alone); 2 the policy
// gradient and, on the same weight chunks, the prepare pass's backward below the head (NH = 2: D_1, E_1, E_0;
// NH = 1: E_0); NH = hidden layers (1 or 2)
template <int FW, int LB, int TI0, int OTA, int MODE, int NH>
__global__ void __launch_bounds__(FW * 64, LB) fvp_fused16_kernel(const Fused16Args fa) {
  constexpr bool PG = MODE >= 1, PREP = MODE == 2;
  static_assert(NH == 1 || NH == 2, "fused16: one or two hidden layers");
  constexpr int LH = NH + 1;                   // index of the action width in w[] / ld[]
  constexpr int NJ = fused16_jobs<NH>();
  constexpr int JW1T = job_w1t<NH>();
  constexpr int OTM = 4;                       // 16-feature tiles of a hidden layer
  constexpr int NT = FW * 64;
  constexpr int CHU = 8 * 16 * OTM;            // 16-B units of a 64-row chunk: 2 planes x 64 rows x 64 B
  constexpr int NLD = (CHU + NT - 1) / NT;
  constexpr int RB = 16 * FW;                  // states per group
  constexpr int PL = RB * kFI;                 // u16 per image plane
  constexpr int KS = RB / 32;                  // k-steps of a gradient pass
  constexpr int KX = (TI0 + 1) / 2;            // 32-deep chunks of obs
  constexpr int OBC = (TI0 + 3) / 4;           // 64-feature X passes
  constexpr int TW0 = (TI0 * OTM + FW - 1) / FW;   // owned gradient tiles: obs x hidden
  constexpr int TWH = (OTM * OTM + FW - 1) / FW;   //                       hidden x hidden
  constexpr int TWL = (OTM * OTA + FW - 1) / FW;   //                       hidden x actions
  constexpr int RING = FUSED16_RING;
  // weight-chunk ring: FUSED16_DMA: three slots, chunk q of a group in slot q % 3 (three distinct objects, so the
  // compiler's LDS-DMA wait before a slot's first read counts only the DMA into that slot); else two buffers
  __shared__ cu32x4 wl0[CHU], wl1[CHU], wl2[FUSED16_DMA ? CHU : 1];
  __shared__ __attribute__((aligned(16))) unsigned short simg[2][2 * PL];   // [act | delta] images, hi / lo planes
  __shared__ float sb[FW][3][64];                                          // per-wave bias sums
  __shared__ __attribute__((aligned(16))) float sc[3][64];                // the tangent's biases c_l
  __shared__ float sred[5][FW];                                            // wave maxima: RH1 RH2 RDh RD1 RD0
  __shared__ int stab[64];   // the chunk table (offset, size), read per chunk from LDS, not by a vector load

  const ChainArgs& a = fa.f.c;
  if (a.skip && *a.skip) return;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const f32x4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
  unsigned short* const sA = &simg[0][0];
  unsigned short* const sD = &simg[1][0];

  for (int i = threadIdx.x; i < FW * 3 * 64; i += NT) (&sb[0][0][0])[i] = 0.0f;
  for (int i = threadIdx.x; i < 2 * a.nchunks && i < 64; i += NT) stab[i] = a.tab[i];   // (first read after a barrier)
  for (int i = threadIdx.x; i < 3 * 64; i += NT) {   // (no tangent in the policy gradient)
    const int l = i >> 6, j = i & 63;
    sc[l][j] = !PG && l <= NH && j < a.w[l + 1] ? a.v[a.offb[l] + j] : 0.0f;
  }

  // scale exponents (wave-uniform)
  const int eX = __builtin_amdgcn_readfirstlane(amax_exp(fa.am_x));
  const int eD1 = __builtin_amdgcn_readfirstlane(amax_exp(fa.am_d1));
  const int eD2 = __builtin_amdgcn_readfirstlane(amax_exp(fa.am_d2));
  const int eDS = PG ? __builtin_amdgcn_readfirstlane(amax_exp(fa.am_ds2)) : 0;
  const int eH = f16_scale_exp(1.0f);
  int ej[NJ];
#pragma unroll
  for (int i = 0; i < NJ; ++i) ej[i] = __builtin_amdgcn_readfirstlane(fa.img_e[i]);
  const float sX = __builtin_ldexpf(1.0f, eX), sH = __builtin_ldexpf(1.0f, eH);
  const float sD1 = __builtin_ldexpf(1.0f, eD1), sD2 = __builtin_ldexpf(1.0f, eD2);

  f32x4 dw0[TW0], dwh[TWH], dwl[TWL];
#pragma unroll
  for (int k = 0; k < TW0; ++k) dw0[k] = z4;
#pragma unroll
  for (int k = 0; k < TWH; ++k) dwh[k] = z4;
#pragma unroll
  for (int k = 0; k < TWL; ++k) dwl[k] = z4;

  f32x4 acc[OTM], S[OTM], PF[OTM], RH1[OTM], RH2[OTM];
  // H_2 and H_1 in f32 for the R-backward epilogues' (1 - H^2): the images' hi + lo (22 bits) is not exact, and
  // near saturation 1 - H^2 is as small as H's own rounding
  f32x4 H2f[OTM], H1f[OTM];
  f32x4 xn0 = z4, xn1 = z4;   // first X chunk of the next group (loaded one group ahead)
  float mD1 = 0.0f;           // PREP: running max |D_1| of this lane
  const __amdgpu_buffer_rsrc_t rimg = __builtin_amdgcn_make_buffer_rsrc((void*)a.img, 0, 0x7ffffff0, 0x00020000);
  // weight chunks in flight WS ahead, in WS register sets: chunk c of a group sits in set c % WS (the group's
  // chunk count NCH need not be a multiple of WS: the next group's chunk k < WS is loaded into set k by whichever
  // of the last WS chunks frees that set)
  constexpr int NCH = PG ? (NH == 2 ? 3 : 1) : KX + (NH == 2 ? 14 : 6);   // chunks per group
  // image chunk (table index) of the group's chunk q: the FVP streams the whole image, the policy gradient
  // W_2^T (one chunk) and W_1^T (two); with one hidden layer W_1^T (one chunk: K = actions)
  auto chunk_of = [&](int q) { return PG ? (NH == 1 ? KX + 4 : q == 0 ? KX + 8 : KX + 9 + q) : q; };
  constexpr int WS = FUSED16_DMA ? 1 : FUSED16_WSETS;
  cu32x4 wr[WS][NLD];
  // ---- LDS-DMA weight stream (FUSED16_DMA): chunk q of a group is DMA'd into slot q % 3 at chunk q - 2's begin
  // (after its barrier: every wave is past chunk q - 3, the slot's last reader).  The next group's chunk j (0, 1)
  // goes to slot j when one of the current group's last two chunks frees it (both do when NCH % 3 == 0: C2, C3),
  // else at its group's start.  Each wave-instruction moves 1 KB: lanes -> consecutive 16-B units, the image's
  // own layout. ----
  auto slot = [&](int k) -> cu32x4* { return k % 3 == 0 ? wl0 : k % 3 == 1 ? wl1 : wl2; };
  auto dma = [&](int sl, int qq, bool from_lds = true) __attribute__((always_inline)) {
    if constexpr ((FUSED16_ABL & 4) != 0) return;   // ablation: no weight-chunk loads
    const int off = __builtin_amdgcn_readfirstlane(from_lds ? stab[2 * qq] : a.tab[2 * qq]);
    const int sz = __builtin_amdgcn_readfirstlane(from_lds ? stab[2 * qq + 1] : a.tab[2 * qq + 1]);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int base = wv * 64 + i * NT;   // this wave-instruction's first unit
      if (CHU % NT != 0 && base >= CHU) break;
      const int idx = base + (int)(threadIdx.x & 63);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rimg, (__attribute__((address_space(3))) void*)(slot(sl) + base), 16, (idx < sz ? idx : sz - 1) * 16,
          off * 16, 0, 0);
    }
  };
  auto gload = [&](int set, int qq) {
    if constexpr (FUSED16_DMA) return;
    if constexpr ((FUSED16_ABL & 4) != 0) return;
    if constexpr ((FUSED16_ABL & 16) != 0) {   // no weight loads, but the chunk's LDS stores kept (opaque values)
#pragma unroll
      for (int i = 0; i < NLD; ++i) {
        unsigned u = qq + i;
        asm volatile("" : "+v"(u));
        wr[set][i] = cu32x4{u, u, u, u};
      }
      return;
    }
    const int off = __builtin_amdgcn_readfirstlane(a.tab[2 * qq]);
    const int sz = __builtin_amdgcn_readfirstlane(a.tab[2 * qq + 1]);
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int idx = threadIdx.x + i * NT;
      wr[set][i] = __builtin_bit_cast(
          cu32x4, __builtin_amdgcn_raw_buffer_load_b128(rimg, (idx < sz ? idx : sz - 1) * 16, off * 16, 0));
    }
  };
  if constexpr (FUSED16_DMA) {   // (the table's LDS copy is not visible before the first barrier)
    dma(0, chunk_of(0), false);
    if constexpr (NCH > 1) dma(1, chunk_of(1), false);
  } else {
#pragma unroll
    for (int k = 0; k < WS; ++k) gload(k, chunk_of(k));
  }

  const int ngroups = fa.f.ngroups;
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int64_t row_b = (int64_t)grp * RB;
    const int rb = (int)((int64_t)a.n - row_b < RB ? (int64_t)a.n - row_b : RB);
    // lane-derived offsets are recomputed per group from an opaque copy of threadIdx.x (hoisted out of the
    // group loop they would stay live across the whole launch)
    int tid;
    asm volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"((int)threadIdx.x));
    const int lane = tid & 63, g = lane >> 4, s = lane & 15;
    const int lrow = wave * 16 + s;
    const int frag = s * 32 + ((g ^ chain_hsw(s)) << 3);

    // ---- weight-chunk stream: one barrier per chunk ----
    int q = 0;
    const unsigned short* W = nullptr;   // this lane's A fragment in the current chunk
    if constexpr (FUSED16_DMA) {
      // the next group's first chunks that the previous group's last chunks could not prefetch
      if (grp != (int)blockIdx.x) {
        if constexpr (NCH % 3 == 1) dma(0, chunk_of(0));
        if constexpr (NCH % 3 == 2) dma(1, chunk_of(1));
      }
    }
    const bool more = grp + (int)gridDim.x < ngroups;   // a next group (uniform)
    auto chunk_begin_dma = [&]() __attribute__((always_inline)) {
      __builtin_amdgcn_sched_barrier(0);
      cu32x4* buf = slot(q);
      // this wave's DMA into the slot has landed (the compiler's LDS-DMA wait, placed before this read) ...
      cu32x4 probe = buf[threadIdx.x];
      asm volatile("" ::"v"(probe));
      // ... and every wave's: chunk q visible; every wave is past chunk q - 1 (slot (q + 2) % 3's last reader)
      lds_barrier();
      if (q + 2 < NCH) {
        dma(q + 2, chunk_of(q + 2));
      } else if ((q + 2) % 3 <= 1 && (q + 2) % 3 < NCH) {   // the next group's chunk (q + 2) % 3, into its slot
        if (more) dma((q + 2) % 3, chunk_of((q + 2) % 3));
      }
      W = reinterpret_cast<const unsigned short*>(buf) + frag;
      ++q;
    };
    auto chunk_begin = [&]() __attribute__((always_inline)) {
      if constexpr (FUSED16_DMA) {
        chunk_begin_dma();
        return;
      }
      __builtin_amdgcn_sched_barrier(0);
      cu32x4* buf = slot(q & 1);
#pragma unroll
      for (int i = 0; i < NLD; ++i) {
        const int idx = threadIdx.x + i * NT;
        if (CHU % NT == 0 || idx < CHU) buf[idx] = wr[q % WS][i];
      }
      if constexpr ((FUSED16_ABL & 8) == 0) lds_barrier();   // chunk q visible; every wave is past chunk q - 1
      gload(q % WS, chunk_of(q + WS < NCH ? q + WS : q % WS));
      W = reinterpret_cast<const unsigned short*>(buf) + frag;
      ++q;
    };

    // ---- image helpers (planes hi, lo; each image holds values times one power of two) ----
    auto put4 = [&](unsigned short* slot, int t, const f32x4& x, float m) {
      const cu32x2 p0 = split2(x[0] * m, x[1] * m), p1 = split2(x[2] * m, x[3] * m);
      const int o = fimg(lrow, 16 * t + 4 * g);
      *reinterpret_cast<cu32x2*>(slot + o) = cu32x2{p0[0], p1[0]};
      *reinterpret_cast<cu32x2*>(slot + PL + o) = cu32x2{p0[1], p1[1]};
    };
    auto putb = [&](unsigned short* slot, int c, const fh8 (&b)[2]) {   // a B operand of chunk c
      const int o0 = fimg(lrow, 32 * c + 4 * g), o1 = fimg(lrow, 32 * c + 16 + 4 * g);
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const cu32x4 v = __builtin_bit_cast(cu32x4, b[p]);
        *reinterpret_cast<cu32x2*>(slot + p * PL + o0) = cu32x2{v[0], v[1]};
        *reinterpret_cast<cu32x2*>(slot + p * PL + o1) = cu32x2{v[2], v[3]};
      }
    };
    // 16x16x32 operand of feature tile ft, k-step ks: lane (i = lane & 15, g) <- states 32ks + 8g .. +7
    const int tq = (lane >> 2) & 3, tp = lane & 3;
    auto tfrag = [&](const unsigned short* slot, int ft, int ks, fh8 (&f)[2]) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        fs8 v;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int r = 32 * ks + 8 * g + 4 * t + tq;
          const fs4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) fs4*)(slot + p * PL + fimg(r, 16 * ft + 4 * tp)));
#pragma unroll
          for (int e = 0; e < 4; ++e) v[4 * t + e] = x[e];
        }
        f[p] = __builtin_bit_cast(fh8, v);
      }
    };
    // gradient products of this wave's tiles of a TI x TJ layer whose act tile lies in [ti0, ti0 + 4),
    // unscaled by 2^-e into the launch-long accumulators
    auto run = [&](auto& dacc, auto TI_, auto TJ_, int ti0, int e) __attribute__((always_inline)) {
      constexpr int TI = decltype(TI_)::value, TJ = decltype(TJ_)::value;
      constexpr int TWm = sizeof(dacc) / sizeof(f32x4);
      if constexpr ((FUSED16_ABL & 2) != 0) return;
#pragma unroll
      for (int k = 0; k < TWm; ++k) {
        const int u = wave + FW * k;
        const int it = u / TJ, jt = u % TJ;
        if (u < TI * TJ && it >= ti0 && it < ti0 + 4) {
          f32x4 c = z4;
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            fh8 fa_[2], fd_[2];
            tfrag(sA, it - ti0, ks, fa_);
            tfrag(sD, jt, ks, fd_);
            c = mfma3(fa_, fd_, c);
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) dacc[k][i] = __builtin_fmaf(c[i], __builtin_amdgcn_ldexpf(1.0f, -e), dacc[k][i]);
        }
      }
    };
    // bias sums of layer m from acc-layout RD tiles: the sum over the wave's 16 states (the lanes s of a row)
    // of the lane's 4 features, transposed on the way so that the 4 values become 1: partner s^1 takes one
    // pair, s^2 one value, then rotations by 4 and 8 within the row; lane s < 4 ends with feature
    // 4g + 2(s & 1) + (s >> 1 & 1)
    auto bias_add = [&](int m, auto OT_, const f32x4 (&R)[OTM]) {
      constexpr int OT = decltype(OT_)::value;
      const bool o1 = s & 1, o2 = (s >> 1) & 1;
#pragma unroll
      for (int t = 0; t < OT; ++t) {
        const f32x4 v = R[t];
        float k0 = o1 ? v[2] : v[0], k1 = o1 ? v[3] : v[1];
        const float t0 = o1 ? v[0] : v[2], t1 = o1 ? v[1] : v[3];
        k0 += dpp_f<kDppX1>(t0);
        k1 += dpp_f<kDppX1>(t1);
        float k = o2 ? k1 : k0;
        k += dpp_f<kDppX2>(o2 ? k0 : k1);
        k += dpp_f<kDppRor4>(k);
        k += dpp_f<kDppRor8>(k);
        if (s < 4) sb[wave][m][16 * t + 4 * g + 2 * o1 + o2] += k;
      }
    };
    // this wave's max of a tensor whose per-state maxima are m -> sred[k][wave]; its group exponent
    auto wave_max = [&](int k, float m) {
      m = max16_dpp(m);
      if (lane == 0) sred[k][wave] = m;
    };
    auto group_exp = [&](int k) {
      float m = sred[k][0];
#pragma unroll
      for (int w = 1; w < FW; ++w) m = fmaxf(m, sred[k][w]);
      return __builtin_amdgcn_readfirstlane(f16_scale_exp(m));
    };

    auto rsrc = [&](const float* p, int ld) {
      return __builtin_amdgcn_make_buffer_rsrc((void*)(p + row_b * ld), 0, rb * ld * 4, 0x00020000);
    };
    auto voff = [&](int ld, int t) {   // columns past the width read zeros (offset past the buffer); branch-free
      const int col = 16 * t + 4 * g;
      const int bad = -(int)(col >= ld);
      return (((lrow * ld + col) * 4) & ~bad) | ((rb * ld * 4) & bad);
    };
    auto ld4 = [&](__amdgpu_buffer_rsrc_t r, int vo) -> f32x4 {
      if constexpr ((FUSED16_ABL & 1) != 0) return f32x4{0.5f, 0.25f, 0.125f, 0.0625f};
      return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, 0, 0));
    };
    auto st4 = [&](float* p, int ld, int t, const f32x4& x) {   // acc-layout tile t of this lane's state row
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(cu32x4, x), rsrc(p, ld), voff(ld, t), 0, 0);
    };
    auto bias4 = [&](int l, int t) -> f32x4 { return *reinterpret_cast<const f32x4*>(&sc[l][16 * t + 4 * g]); };

    auto mma_to = [&](auto OT_, const fh8 (&b)[2], f32x4 (&ac)[OTM]) __attribute__((always_inline)) {
      constexpr int OT = decltype(OT_)::value;
      constexpr int pl = OT * 512;   // u16 per plane of the chunk
      fh8 f[2], nx[2];
#pragma unroll
      for (int p = 0; p < 2; ++p) f[p] = *reinterpret_cast<const fh8*>(W + p * pl);
#pragma unroll
      for (int ot = 0; ot < OT; ++ot) {
        if (ot + 1 < OT) {
#pragma unroll
          for (int p = 0; p < 2; ++p) nx[p] = *reinterpret_cast<const fh8*>(W + p * pl + (ot + 1) * 512);
        }
        ac[ot] = mfma3(f, b, ac[ot]);
        if (ot + 1 < OT) {
#pragma unroll
          for (int p = 0; p < 2; ++p) f[p] = nx[p];
        }
      }
    };

    auto mma = [&](auto OT_, const fh8 (&b)[2]) __attribute__((always_inline)) { mma_to(OT_, b, acc); };
    auto no_extra = [](int) {};

    // One chain step: acc = [S (KC0 chunks, registers, times 2^eS per state) x job jS |
    //                        M1 (KC1 chunks, memory, times sM) x job jS + 1 (jS when KC0 = 0)];
    // acc * su is the f32 value;
    // the epilogue operand Pre is prefetched into PF; cap (optional) receives M1's split planes; extra(c) runs
    // with chunk c of the step in LDS (more products on the same weights).
    float su = 1.0f;
    auto step = [&](auto OT_, auto KC0_, auto KC1_, int jS, int eS, const float* M1, int ld1, float sM, int eM,
                    const float* Pre, int ldp, int OTp, unsigned short* cap, bool pre, auto&& extra,
                    const f32x4* Mreg = nullptr) __attribute__((always_inline)) {
      constexpr int OT = decltype(OT_)::value, KC0 = decltype(KC0_)::value, KC1 = decltype(KC1_)::value;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < OTM; ++t) acc[t] = z4;
      const __amdgpu_buffer_rsrc_t r1 = rsrc(M1, ld1);
      // memory chunk j (step chunk KC0 + j) is loaded RING chunks ahead of its use, or at the step's start
      f32x4 mb[KC1 > 0 ? KC1 : 1][2];
      auto issue = [&](int j) {
        if (Mreg) {            // M1 already in registers (acc-layout tiles 2j, 2j + 1)
          mb[j][0] = Mreg[2 * j];
          mb[j][1] = Mreg[2 * j + 1];
        } else if (j == 0 && pre) {   // X's first chunk, loaded during the previous group
          mb[0][0] = xn0;
          mb[0][1] = xn1;
        } else {
          mb[j][0] = ld4(r1, voff(ld1, 2 * j));
          mb[j][1] = ld4(r1, voff(ld1, 2 * j + 1));
        }
      };
      auto pf_load = [&]() {
        const __amdgpu_buffer_rsrc_t rp = rsrc(Pre, ldp);
#pragma unroll
        for (int t = 0; t < OTM; ++t) PF[t] = ld4(rp, t < OTp ? voff(ldp, t) : rb * ldp * 4);
      };
      if constexpr (FUSED16_PFEARLY) pf_load();
#pragma unroll
      for (int j = 0; j < KC1; ++j)
        if (KC0 + j < RING) issue(j);
      if constexpr (KC0 > 0) {
        const float sS = __builtin_amdgcn_ldexpf(1.0f, eS);
#pragma unroll
        for (int c = 0; c < KC0; ++c) {
          fh8 b[2];
          mkb16(S[2 * c], S[2 * c + 1], sS, b);
          chunk_begin();
#pragma unroll
          for (int j = 0; j < KC1; ++j)
            if (KC0 + j >= RING && KC0 + j - RING == c) issue(j);
          mma(OT_, b);
          extra(c);
        }
        if constexpr (KC1 > 0) {   // segment scales: 2^(ej[jS] + eS) -> 2^(ej[jS + 1] + eM)
          const int d = ej[jS + 1] + eM - ej[jS] - eS;
#pragma unroll
          for (int t = 0; t < OT; ++t) acc[t] = ldexp4(acc[t], d);
        }
      }
      const int jM = KC0 > 0 ? jS + 1 : jS;
#pragma unroll
      for (int c = 0; c < KC1; ++c) {
        chunk_begin();
        if (c + RING < KC1 && KC0 + c + RING >= RING) issue(c + RING);
        if (!FUSED16_PFEARLY && c == 0) pf_load();
        fh8 b[2];
        mkb16(mb[c][0], mb[c][1], sM, b);
        if (cap) putb(cap, c, b);
        mma(OT_, b);
        extra(KC0 + c);
      }
      // (a register-only step leaves its per-state scale: su is then per lane)
      su = KC1 > 0 ? __builtin_ldexpf(1.0f, -(ej[jM] + eM)) : __builtin_amdgcn_ldexpf(1.0f, -(ej[jS] + eS));
    };

    using C1 = std::integral_constant<int, 1>;
    using C2 = std::integral_constant<int, 2>;
    using C4 = std::integral_constant<int, OTM>;
    using COTA = std::integral_constant<int, OTA>;
    using CKX = std::integral_constant<int, KX>;
    using C0 = std::integral_constant<int, 0>;

    if constexpr (PG) {
      // ---- policy gradient (trpo_inksci.py:54), the surr backward from the head's logit delta DS_h
      //      (the prepare pass's): NH = 2: DS_1 = (DS_2 W_2^T)(1 - H_2^2), DS_0 = (DS_1 W_1^T)(1 - H_1^2);
      //      NH = 1: DS_0 = (DS_1 W_1^T)(1 - H_1^2); g_W_l = H_l^T DS_l (H_0 = X), g_b_l = colsum DS_l. ----
      const float sDS = __builtin_ldexpf(1.0f, eDS);
      // PREP: the KL_ff plain backward on the same chunks from the head's delta D_h:
      //   NH = 2: DH_1 = D_2 W_2^T, D_1 = DH_1 (1 - H_2^2), E_1 = -2 DH_1 H_2, E_0 = -2 (D_1 W_1^T) H_1;
      //   NH = 1: E_0 = -2 (D_1 W_1^T) H_1 (engine.cpp prepare(); D_0 has no reader)
      const float sDh = NH == 2 ? sD2 : sD1;
      const int eDh = NH == 2 ? eD2 : eD1;
      f32x4 accD[OTM], D1v[OTM];
      f32x4 d2c0 = z4, d2c1 = z4;
      if constexpr (PREP) {
        const __amdgpu_buffer_rsrc_t rd2 = rsrc(a.D[NH], a.ld[LH]);
        d2c0 = ld4(rd2, voff(a.ld[LH], 0));
        d2c1 = ld4(rd2, voff(a.ld[LH], 1));
#pragma unroll
        for (int t = 0; t < OTM; ++t) accD[t] = z4;
      }
      auto extra1 = [&](int) {
        if constexpr (PREP) {
          fh8 b[2];
          mkb16(d2c0, d2c1, sDh, b);
          mma_to(C4{}, b, accD);
        }
      };
      // the head layer's backward step: its memory segment DS_h is captured into sD (the head pass's delta image)
      step(C4{}, C0{}, C1{}, NH == 2 ? jW2t : JW1T, 0, fa.DS, a.ld[LH], sDS, eDS, a.H[NH], a.ld[NH], OTM, sD, false,
           extra1);
      const float suD = __builtin_ldexpf(1.0f, -(ej[NH == 2 ? jW2t : JW1T] + eDh));
      f32x4 DS1[OTM];   // NH = 2: DS_1; NH = 1: DS_0 (also in S)
#pragma unroll
      for (int t = 0; t < OTM; ++t) {
        const f32x4 h = PF[t];
        if constexpr (NH == 1) H1f[t] = h;
#pragma unroll
        for (int i = 0; i < 4; ++i) DS1[t][i] = acc[t][i] * (su * c_one_minus_sq(h[i]));
        put4(sA, t, h, sH);   // H_NH, the head layer's pass operand (sA is free: past this step's chunk barrier)
        if constexpr (PREP) {
          f32x4 e1;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float dh = accD[t][i] * suD;
            D1v[t][i] = dh * c_one_minus_sq(h[i]);
            e1[i] = -2.0f * dh * h[i];
          }
          if constexpr (NH == 2) {
            st4(fa.D1out, a.ld[2], t, D1v[t]);
            st4(fa.E1out, a.ld[2], t, e1);
          } else {
            st4(fa.E0out, a.ld[1], t, e1);
          }
        }
      }
      if constexpr (NH == 2) {
        float mst = state_max<OTM>(DS1);
        wave_max(3, mst);
        float mstD = 0.0f;
        if constexpr (PREP) {
          mstD = state_max<OTM>(D1v);
          mD1 = fmaxf(mD1, mstD);
#pragma unroll
          for (int t = 0; t < OTM; ++t) accD[t] = z4;
        }
        const float sD1s = __builtin_ldexpf(1.0f, f16_scale_exp(mstD));
        auto extra2 = [&](int c) {
          if constexpr (PREP) {
            fh8 b[2];
            mkb16(D1v[2 * c], D1v[2 * c + 1], sD1s, b);
            mma_to(C4{}, b, accD);
          }
        };
#pragma unroll
        for (int t = 0; t < OTM; ++t) S[t] = DS1[t];
        step(C4{}, C2{}, C0{}, jW1t, f16_scale_exp(mst), a.H[1], 0, 1.0f, 0, a.H[1], a.ld[1], OTM, nullptr, false,
             extra2);
        const float suD0 = __builtin_amdgcn_ldexpf(1.0f, -(ej[jW1t] + f16_scale_exp(mstD)));
#pragma unroll
        for (int t = 0; t < OTM; ++t) {
          const f32x4 h = PF[t];
          H1f[t] = h;
#pragma unroll
          for (int i = 0; i < 4; ++i) S[t][i] = acc[t][i] * (su * c_one_minus_sq(h[i]));   // DS_0
          if constexpr (PREP) {
            f32x4 e0;
#pragma unroll
            for (int i = 0; i < 4; ++i) e0[i] = -2.0f * (accD[t][i] * suD0) * h[i];
            st4(fa.E0out, a.ld[1], t, e0);
          }
        }
      } else {
#pragma unroll
        for (int t = 0; t < OTM; ++t) S[t] = DS1[t];
      }
      wave_max(4, state_max<OTM>(S));
      const __amdgpu_buffer_rsrc_t rx = rsrc(a.X, a.ld[0]);
      f32x4 nxt[OTM];
#pragma unroll
      for (int t = 0; t < OTM; ++t) nxt[t] = ld4(rx, voff(a.ld[0], t));
      {
        // g_W_NH += H_NH^T DS_h (both images written above); g_b_NH from DS_h's f32 tiles
        f32x4 d2[OTM];
        const __amdgpu_buffer_rsrc_t rd = rsrc(fa.DS, a.ld[LH]);
#pragma unroll
        for (int t = 0; t < OTM; ++t) d2[t] = t < OTA ? ld4(rd, voff(a.ld[LH], t)) : z4;
        lds_barrier();
        bias_add(NH, COTA{}, d2);
        run(dwl, C4{}, COTA{}, 0, eH + eDS);
      }
      if constexpr (NH == 2) {
        // g_W_1 += H_1^T DS_1
        lds_barrier();
        const int eg = group_exp(3);
        const float sg = __builtin_ldexpf(1.0f, eg);
#pragma unroll
        for (int t = 0; t < OTM; ++t) {
          put4(sD, t, DS1[t], sg);
          put4(sA, t, H1f[t], sH);
        }
        bias_add(1, C4{}, DS1);
        lds_barrier();
        run(dwh, C4{}, C4{}, 0, eH + eg);
      }
      {
        // g_W_0 += X^T DS_0 in 64-feature chunks of X
        lds_barrier();
        const int eg = group_exp(4);
        const float sg = __builtin_ldexpf(1.0f, eg);
#pragma unroll
        for (int t = 0; t < OTM; ++t) {
          put4(sD, t, S[t], sg);
          put4(sA, t, nxt[t], sX);
        }
        bias_add(0, C4{}, S);
#pragma unroll
        for (int ch = 0; ch < OBC; ++ch) {
          if (ch + 1 < OBC) {
#pragma unroll
            for (int t = 0; t < OTM; ++t) nxt[t] = ld4(rx, voff(a.ld[0], 4 * (ch + 1) + t));
          }
          lds_barrier();
          run(dw0, std::integral_constant<int, TI0>{}, C4{}, 4 * ch, eX + eg);
          if (ch + 1 < OBC) {
            lds_barrier();
#pragma unroll
            for (int t = 0; t < OTM; ++t) put4(sA, t, nxt[t], sX);
          }
        }
      }
      continue;
    }

    if (grp == (int)blockIdx.x) {   // later groups' first X chunk is loaded during the previous group
      const __amdgpu_buffer_rsrc_t rx = rsrc(a.X, a.ld[0]);
      xn0 = ld4(rx, voff(a.ld[0], 0));
      xn1 = ld4(rx, voff(a.ld[0], 1));
    }

    // ---- R-forward: RH_1 = (1 - H_1^2)(X V_0 + c_0) ----
    step(C4{}, C0{}, CKX{}, jV0, 0, a.X, a.ld[0], sX, eX, a.H[1], a.ld[1], OTM, nullptr, true, no_extra);
#pragma unroll
    for (int t = 0; t < OTM; ++t) {
      const f32x4 cb = bias4(0, t), h = PF[t];
#pragma unroll
      for (int i = 0; i < 4; ++i) RH1[t][i] = c_one_minus_sq(h[i]) * __builtin_fmaf(acc[t][i], su, cb[i]);
      H1f[t] = h;   // H_1: the next step's memory segment (FUSED16_REUSE)
    }
    float mst = state_max<OTM>(RH1);
    wave_max(0, mst);
    if constexpr (NH == 2) {
      // ---- RH_2 = (1 - H_2^2)(RH_1 W_1 + H_1 V_1 + c_1) ----
#pragma unroll
      for (int t = 0; t < OTM; ++t) S[t] = RH1[t];
      step(C4{}, C2{}, C2{}, jW1, f16_scale_exp(mst), a.H[1], a.ld[1], sH, eH, a.H[2], a.ld[2], OTM, nullptr, false,
           no_extra, FUSED16_REUSE ? H1f : nullptr);
#pragma unroll
      for (int t = 0; t < OTM; ++t) {
        const f32x4 cb = bias4(1, t), h = PF[t];
#pragma unroll
        for (int i = 0; i < 4; ++i) RH2[t][i] = c_one_minus_sq(h[i]) * __builtin_fmaf(acc[t][i], su, cb[i]);
        H2f[t] = h;
      }
      mst = state_max<OTM>(RH2);
      wave_max(1, mst);
    }
    // the last hidden layer's R-activations and activations: NH = 2: RH_2, H_2; NH = 1: RH_1, H_1
    f32x4(&RHt)[OTM] = NH == 2 ? RH2 : RH1;
    f32x4(&Htf)[OTM] = NH == 2 ? H2f : H1f;

    // ---- R-softmax head; H_NH captured into the act image ----
    {
      const int A = a.w[LH];
#pragma unroll
      for (int t = 0; t < OTM; ++t) S[t] = RHt[t];
      step(COTA{}, C2{}, C2{}, NH == 2 ? jW2 : jW1, f16_scale_exp(mst), a.H[NH], a.ld[NH], sH, eH, a.P, a.ld[LH], 2, sA,
           false, no_extra, FUSED16_REUSE ? Htf : nullptr);
      // R-softmax in f32 on the cancellation-free form of tail.hip / gemm.hip kRHead:
      //   RD_j = (1/N)[Rp_j (B_j - sum p B) + Rp_j A_j^2 + p_j sum_k Rp_k A_k B_k],
      //   Rp = p (Rz - <p, Rz>), A = p / (p + eps), B = eps / (p + eps); the 4 lanes of a state hold 8 actions each
      float zf[8], pf[8], inv[8];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const f32x4 cb = bias4(NH, t);
        const f32x4 pv = PF[t];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool real = 16 * t + 4 * g + i < A;
          zf[4 * t + i] = real ? __builtin_fmaf(acc[t][i], su, cb[i]) : 0.0f;
          pf[4 * t + i] = real ? pv[i] : 0.0f;
        }
      }
      float prz = 0.0f;
#pragma unroll
      for (int k = 0; k < 8; ++k) prz = __builtin_fmaf(pf[k], zf[k], prz);
      prz = xadd_f<true>(xadd_f<false>(prz));
      float spB = 0.0f, sRAB = 0.0f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        inv[k] = __builtin_amdgcn_rcpf(pf[k] + kEps);   // v_rcp_f32 (1 ulp): A and B need no IEEE quotient
        const float Rp = pf[k] * (zf[k] - prz);
        const float Aa = pf[k] * inv[k], B = kEps * inv[k];
        spB += pf[k] * B;
        sRAB += Rp * Aa * B;
      }
      spB = xadd_f<true>(xadd_f<false>(spB));
      sRAB = xadd_f<true>(xadd_f<false>(sRAB));
      const float invN = (float)a.invN;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = 4 * t + i;
          const bool real = 16 * t + 4 * g + i < A;
          const float Rp = pf[k] * (zf[k] - prz);
          const float Aa = pf[k] * inv[k], B = kEps * inv[k];
          const float rd = invN * (Rp * (B - spB) + Rp * Aa * Aa + pf[k] * sRAB);
          r[i] = real ? rd : 0.0f;
        }
        S[t] = r;
      }
#pragma unroll
      for (int t = 2; t < OTM; ++t) S[t] = z4;
      mst = state_max<2>(S);
      wave_max(2, mst);
      // gradient pass: (Hv)_W_NH += H_NH^T RD_h  (act captured in the step)
      lds_barrier();
      const int eg = group_exp(2);
      const float sg = __builtin_ldexpf(1.0f, eg);
#pragma unroll
      for (int t = 0; t < OTA; ++t) put4(sD, t, S[t], sg);
      bias_add(NH, COTA{}, S);
      lds_barrier();
      run(dwl, C4{}, COTA{}, 0, eH + eg);
    }

    // ---- R-backward into the head layer's input: RD_{NH-1} = (RD_h W_NH^T + D_h V_NH^T)(1 - H_NH^2) + E_{NH-1} RH_NH;
    //      D_h captured ----
    step(C4{}, C1{}, C1{}, NH == 2 ? jW2t : JW1T, f16_scale_exp(mst), a.D[NH], a.ld[LH], NH == 2 ? sD2 : sD1,
         NH == 2 ? eD2 : eD1, a.E[NH - 1], a.ld[NH], OTM, sD, false, no_extra);
#pragma unroll
    for (int t = 0; t < OTM; ++t) {
      const f32x4 h = Htf[t], e = PF[t];
#pragma unroll
      for (int i = 0; i < 4; ++i) S[t][i] = __builtin_fmaf(e[i], RHt[t][i], acc[t][i] * (su * c_one_minus_sq(h[i])));
    }
    mst = state_max<OTM>(S);
    wave_max(NH == 2 ? 3 : 4, mst);
    if constexpr (NH == 2) {
      // (Hv)_W_2 += RH_2^T D_2 ; H_1 for the next pass is loaded meanwhile
      lds_barrier();
      const int eg = group_exp(1);
      const float sg = __builtin_ldexpf(1.0f, eg);
#pragma unroll
      for (int t = 0; t < OTM; ++t) put4(sA, t, RH2[t], sg);
      const __amdgpu_buffer_rsrc_t rn = rsrc(a.H[1], a.ld[1]);
#pragma unroll
      for (int t = 0; t < OTM; ++t)
        if (FUSED16_REUSE < 2) H1f[t] = ld4(rn, voff(a.ld[1], t));
      lds_barrier();
      run(dwl, C4{}, COTA{}, 0, eg + eD2);
      // (Hv)_W_1 += H_1^T RD_1
      lds_barrier();
      const int eg1 = group_exp(3);
      const float sg1 = __builtin_ldexpf(1.0f, eg1);
#pragma unroll
      for (int t = 0; t < OTM; ++t) put4(sD, t, S[t], sg1);
      bias_add(1, C4{}, S);
#pragma unroll
      for (int t = 0; t < OTM; ++t) put4(sA, t, H1f[t], sH);
      lds_barrier();
      run(dwh, C4{}, C4{}, 0, eH + eg1);
    }

    if constexpr (NH == 2) {
      // ---- R-backward into layer 1's input: RD_0 = (RD_1 W_1^T + D_1 V_1^T)(1 - H_1^2) + E_0 RH_1; D_1 captured ----
      step(C4{}, C2{}, C2{}, jW1t, f16_scale_exp(mst), a.D[1], a.ld[2], sD1, eD1, a.E[0], a.ld[1], OTM, sD, false,
           no_extra);
#pragma unroll
      for (int t = 0; t < OTM; ++t) {
        const f32x4 h = H1f[t], e = PF[t];
#pragma unroll
        for (int i = 0; i < 4; ++i) S[t][i] = __builtin_fmaf(e[i], RH1[t][i], acc[t][i] * (su * c_one_minus_sq(h[i])));
      }
      mst = state_max<OTM>(S);
      wave_max(4, mst);
    }
    {
      // (Hv)_W_1 += RH_1^T D_1 (NH = 1: the head layer's, D_1 = D_h) ; X's first 64 features are loaded meanwhile
      lds_barrier();
      const int eg = group_exp(0);
      const float sg = __builtin_ldexpf(1.0f, eg);
#pragma unroll
      for (int t = 0; t < OTM; ++t) put4(sA, t, RH1[t], sg);
      f32x4 nxt[OTM];
      const __amdgpu_buffer_rsrc_t rx = rsrc(a.X, a.ld[0]);
#pragma unroll
      for (int t = 0; t < OTM; ++t) nxt[t] = ld4(rx, voff(a.ld[0], t));
      lds_barrier();
      if constexpr (NH == 2) run(dwh, C4{}, C4{}, 0, eg + eD1);
      else run(dwl, C4{}, COTA{}, 0, eg + eD1);
      // (Hv)_W_0 += X^T RD_0 in 64-feature chunks of X
      lds_barrier();
      const int eg0 = group_exp(4);
      const float sg0 = __builtin_ldexpf(1.0f, eg0);
#pragma unroll
      for (int t = 0; t < OTM; ++t) put4(sD, t, S[t], sg0);
      bias_add(0, C4{}, S);
#pragma unroll
      for (int t = 0; t < OTM; ++t) put4(sA, t, nxt[t], sX);
#pragma unroll
      for (int ch = 0; ch < OBC; ++ch) {
        if (ch + 1 < OBC) {
#pragma unroll
          for (int t = 0; t < OTM; ++t) nxt[t] = ld4(rx, voff(a.ld[0], 4 * (ch + 1) + t));
        } else {
          // the next group's first X chunk, in flight during this last gradient pass
          const int64_t nb = row_b + (int64_t)gridDim.x * RB;
          const int nrb = (int)((int64_t)a.n - nb < RB ? (int64_t)a.n - nb : RB);
          const __amdgpu_buffer_rsrc_t rxn = __builtin_amdgcn_make_buffer_rsrc(
              (void*)(a.X + (nb < a.n ? nb : 0) * a.ld[0]), 0, nb < a.n ? nrb * a.ld[0] * 4 : 0, 0x00020000);
          xn0 = ld4(rxn, voff(a.ld[0], 0));
          xn1 = ld4(rxn, voff(a.ld[0], 1));
        }
        lds_barrier();
        run(dw0, std::integral_constant<int, TI0>{}, C4{}, 4 * ch, eX + eg0);
        if (ch + 1 < OBC) {
          lds_barrier();
#pragma unroll
          for (int t = 0; t < OTM; ++t) put4(sA, t, nxt[t], sX);
        }
      }
    }
  }

  // ---- this workgroup's slab: owned gradient tiles (C layout: rows 4g + r, column s) and biases ----
  __syncthreads();
  if constexpr (PREP) {   // D_1's running max (kernels.h slots): workgroup max, one atomicMax per workgroup
    float m = mD1;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    if ((threadIdx.x & 63) == 0) sred[0][wave] = m;
    __syncthreads();
    if (threadIdx.x == 0 && fa.am_d1_out) {
      float mm = 0.0f;
#pragma unroll
      for (int w = 0; w < FW; ++w) mm = fmaxf(mm, sred[0][w]);
      if (mm > 0.0f) atomicMax(fa.am_d1_out + (blockIdx.x % kAmaxSub) * kAmaxStride, __float_as_uint(mm));
    }
  }
  const int lane = threadIdx.x & 63, g = lane >> 4, s = lane & 15;
  float* out = fa.f.slab + (size_t)blockIdx.x * fa.f.slab_stride;
  auto wout = [&](auto& dacc, int m, int TI, int TJ) __attribute__((always_inline)) {
    constexpr int TWm = sizeof(dacc) / sizeof(f32x4);
    const int wi = a.w[m], wj = a.w[m + 1];
#pragma unroll
    for (int k = 0; k < TWm; ++k) {
      const int u = wave + FW * k;
      if (u < TI * TJ) {
        const int it = u / TJ, jt = u - (u / TJ) * TJ;
        const int j = 16 * jt + s;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 16 * it + 4 * g + r;
          if (i < wi && j < wj) out[fa.f.offW[m] + (int64_t)i * wj + j] = dacc[k][r];
        }
      }
    }
  };
  wout(dw0, 0, TI0, OTM);
  if constexpr (NH == 2) wout(dwh, 1, OTM, OTM);
  wout(dwl, NH, OTM, OTA);
  for (int i = threadIdx.x; i < (NH + 1) * 64; i += NT) {
    const int m = i >> 6, j = i & 63;
    if (j < a.w[m + 1]) {
      float t = 0.0f;
#pragma unroll
      for (int u = 0; u < FW; ++u) t += sb[u][m][j];
      out[a.offb[m] + j] = t;
    }
  }
}

// ---------------------------------------------------------------------------------------------------------
// Line-search loss forward (trpo_inksci.py:38-53 at the trial theta, utils.py:170-182 through loss()):
// X -> tanh(X W_0 + b_0) -> tanh(H_1 W_1 + b_1) -> softmax(H_2 W_2 + b_2) -> the row terms (surr, kl, ent)
// that reduce_losses sums, for the fused16 shapes.  No weight stream and no barrier in the loop: the three
// trial weight images (KX + 4 chunks, <= 64 KB) are copied to LDS once per workgroup, and every wave runs its
// own 16 states through the three layers in accumulator layout (the FVP chain's forward steps with W in place
// of V), with the next group's X in flight behind the current group's math.  Products as the FVP: scaled f16
// hi + lo, 3 products; H's scale fixed, X's from its running max, each weight image's from its builder.
// The head: f32 softmax and logs, as the row GEMM's kLossHead (rowepi.h), over the state's 4 lanes.
// PREP: the prepare pass's forward at theta instead (kPrepHead): H_1, H_2, P, the KL_ff logit delta D_2 and the
// surr logit delta DS_2 stored, with D_2's and DS_2's running maxima, and the same row terms (loss_before).
// ---------------------------------------------------------------------------------------------------------
#ifndef FWDL16_NW
#define FWDL16_NW 8   // waves per workgroup (sharing one LDS copy of the weights): C3 0.217 ms at 4, 0.201 at 8
#endif
template <int TI0, int OTA, bool PREP, int NH>
__global__ void __launch_bounds__(64 * FWDL16_NW, 2) fwd_loss16_kernel(const FwdLoss16Args a) {
  constexpr int OTM = 4, KX = (TI0 + 1) / 2, NW = FWDL16_NW, NT = 64 * NW;
  constexpr int LH = NH + 1;                   // index of the action width in w[] / ld[]
  constexpr int NCK = KX + 2 * NH;             // W_0 (KX chunks), W_1 (2)[, W_2 (2)]
  constexpr int CHU = 8 * 16 * OTM;            // 16-B units of a full chunk
  __shared__ cu32x4 wl[NCK][CHU];
  __shared__ __attribute__((aligned(16))) float sbias[3][64];
  if (a.skip && *a.skip) return;

  for (int q = 0; q < NCK; ++q) {
    const int off = a.tab[2 * q], sz = a.tab[2 * q + 1];
    const cu32x4* src = reinterpret_cast<const cu32x4*>(a.img) + off;
    for (int i = threadIdx.x; i < sz; i += NT) wl[q][i] = src[i];
  }
  for (int i = threadIdx.x; i < 3 * 64; i += NT) {
    const int l = i >> 6, j = i & 63;
    sbias[l][j] = l <= NH && j < a.w[l + 1] ? a.theta[a.offb[l] + j] : 0.0f;
  }
  __syncthreads();

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, g = lane >> 4, s = lane & 15;
  const int eX = __builtin_amdgcn_readfirstlane(amax_exp(a.am_x));
  const int eH = f16_scale_exp(1.0f);
  const int e0 = __builtin_amdgcn_readfirstlane(a.img_e[0]), e1 = __builtin_amdgcn_readfirstlane(a.img_e[1]);
  const int e2 = NH == 2 ? __builtin_amdgcn_readfirstlane(a.img_e[2]) : 0;
  const float sX = __builtin_ldexpf(1.0f, eX), sH = __builtin_ldexpf(1.0f, eH);
  const float u0 = __builtin_ldexpf(1.0f, -(e0 + eX)), u1 = __builtin_ldexpf(1.0f, -(e1 + eH));
  const float u2 = __builtin_ldexpf(1.0f, -((NH == 2 ? e2 : e1) + eH));   // the head layer's
  const int A = a.w[LH], ld0 = a.ld[0], ldo = a.ld[LH];
  const f32x4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};

  // acc[0, OT) += chunk (weights in LDS) x b
  // the fragment offset is re-derived per group from an opaque copy: the weight fragments are the same for every
  // group, and hoisted out of the loop they took 200+ registers
  int frag = 0;
  auto mma_chunk = [&](int q, auto OT_, const fh8 (&b)[2], f32x4 (&ac)[OTM]) __attribute__((always_inline)) {
    constexpr int OT = decltype(OT_)::value, pl = OT * 512;
    const unsigned short* W = reinterpret_cast<const unsigned short*>(&wl[q][0]) + frag;
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) {
      fh8 f[2];
#pragma unroll
      for (int p = 0; p < 2; ++p) f[p] = *reinterpret_cast<const fh8*>(W + p * pl + ot * 512);
      ac[ot] = mfma3(f, b, ac[ot]);
    }
  };
  // X tiles of a 16-state group (rows past n read 0)
  f32x4 xb[KX][2];
  auto load_x = [&](int64_t row_b) {
    const int rb = (int)(row_b < a.n ? min<int64_t>(16, a.n - row_b) : 0);
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.X + (row_b < a.n ? row_b : 0) * ld0), 0, rb * ld0 * 4, 0x00020000);
#pragma unroll
    for (int c = 0; c < KX; ++c)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int col = 16 * (2 * c + h) + 4 * g;
        const int vo = col < ld0 ? (s * ld0 + col) * 4 : rb * ld0 * 4;
        xb[c][h] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, vo, 0, 0));
      }
  };
  using C4 = std::integral_constant<int, OTM>;
  using COTA = std::integral_constant<int, OTA>;

  const int64_t ngroups = (a.n + 15) / 16, stride = (int64_t)gridDim.x * NW;
  int64_t grp = (int64_t)blockIdx.x * NW + wave;
  float md = 0.0f, mds = 0.0f;   // PREP: running max |D_2|, |DS_2| of this lane
  if (grp < ngroups) load_x(grp * 16);
  for (; grp < ngroups; grp += stride) {
    {
      int t = threadIdx.x;
      asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(t));
      const int ss = t & 15, gg = (t >> 4) & 3;
      frag = ss * 32 + ((gg ^ chain_hsw(ss)) << 3);
    }
    f32x4 acc[OTM], H[OTM];
#pragma unroll
    for (int t = 0; t < OTM; ++t) acc[t] = z4;
#pragma unroll
    for (int c = 0; c < KX; ++c) {
      fh8 b[2];
      mkb16(xb[c][0], xb[c][1], sX, b);
      mma_chunk(c, C4{}, b, acc);
    }
    if (grp + stride < ngroups) load_x((grp + stride) * 16);   // the next group's X behind this group's math
    // acc-layout tiles of this lane's state row -> a [n][ld] output (rows past n and columns past ld dropped)
    const int64_t row_b = grp * 16;
    const int rb = (int)min<int64_t>(16, a.n - row_b);
    auto st_tiles = [&](float* out, int ld, int nt, const f32x4* x) {
      const __amdgpu_buffer_rsrc_t r =
          __builtin_amdgcn_make_buffer_rsrc((void*)(out + row_b * ld), 0, rb * ld * 4, 0x00020000);
      for (int t = 0; t < nt; ++t) {
        const int col = 16 * t + 4 * g;
        const int vo = col < ld ? (s * ld + col) * 4 : rb * ld * 4;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(cu32x4, x[t]), r, vo, 0, 0);
      }
    };
    // H_1 = tanh(X W_0 + b_0); padding features: zero weights and bias, tanh(0) = 0
#pragma unroll
    for (int t = 0; t < OTM; ++t) {
      const f32x4 bb = *reinterpret_cast<const f32x4*>(&sbias[0][16 * t + 4 * g]);
#pragma unroll
      for (int i = 0; i < 4; ++i) H[t][i] = tanh_fast(__builtin_fmaf(acc[t][i], u0, bb[i]));
      acc[t] = z4;
    }
    if constexpr (PREP) st_tiles(a.H1, a.ld[1], OTM, H);
    if constexpr (NH == 2) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        fh8 b[2];
        mkb16(H[2 * c], H[2 * c + 1], sH, b);
        mma_chunk(KX + c, C4{}, b, acc);
      }
#pragma unroll
      for (int t = 0; t < OTM; ++t) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(&sbias[1][16 * t + 4 * g]);
#pragma unroll
        for (int i = 0; i < 4; ++i) H[t][i] = tanh_fast(__builtin_fmaf(acc[t][i], u1, bb[i]));
        acc[t] = z4;
      }
      if constexpr (PREP) st_tiles(a.H2, a.ld[2], OTM, H);
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      fh8 b[2];
      mkb16(H[2 * c], H[2 * c + 1], sH, b);
      mma_chunk(KX + 2 * (NH - 1) + c, COTA{}, b, acc);
    }

    // ---- softmax and the row terms (rowepi.h kLossHead): lane g holds actions 16t + 4g + i ----
    const int64_t row = grp * 16 + s;
    const bool rowvalid = row < a.n;
    const int64_t rc = rowvalid ? row : a.n - 1;
    const int av = a.act[rc];
    const float advv = a.adv[rc];
    constexpr int NA = 4 * OTA;
    float z[NA], oldv[NA];
    float zm = -INFINITY;
#pragma unroll
    for (int t = 0; t < OTA; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = 16 * t + 4 * g + i;
        const bool real = col < A;
        z[4 * t + i] = real ? __builtin_fmaf(acc[t][i], u2, sbias[NH][col]) : -INFINITY;
        oldv[4 * t + i] = a.old[rc * ldo + (real ? col : 0)];
        zm = fmaxf(zm, z[4 * t + i]);
      }
    const float m = xmax_f<false>(xmax_f<true>(zm));
    float ex[NA], es = 0.0f;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      ex[k] = z[k] == -INFINITY ? 0.0f : expf(z[k] - m);
      es += ex[k];
    }
    const float ssum = xadd_f<false>(xadd_f<true>(es));
    float pa_l = 0.0f, olda_l = 0.0f, klp = 0.0f, enp = 0.0f;
#pragma unroll
    for (int t = 0; t < OTA; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = 4 * t + i, col = 16 * t + 4 * g + i;
        const bool real = col < A;
        const float p = ex[k] / ssum;
        const float old = (rowvalid && real) ? oldv[k] : 0.0f;
        if (col == av) {
          pa_l = p;
          olda_l = old;
        }
        const float lk = logf((old + kEps) / (p + kEps)), le = logf(p + kEps);
        klp += real ? old * lk : 0.0f;
        enp += real ? -p * le : 0.0f;
      }
    const float pa = xadd_f<false>(xadd_f<true>(pa_l)), olda = xadd_f<false>(xadd_f<true>(olda_l));
    const float klt = xadd_f<false>(xadd_f<true>(klp)), ent = xadd_f<false>(xadd_f<true>(enp));
    if constexpr (PREP) {
      // KL_ff plain logit delta d_j = (p_j/N)(B_j - sum_k p_k B_k), B = eps/(p+eps), and the surr logit delta
      // -(adv/(N old_a)) p_a (1[j=a] - p_j) (rowepi.h kPrepHead, f32)
      const float invN = (float)a.invN;
      float pv[NA], B[NA], spBp = 0.0f, restp = 0.0f;
#pragma unroll
      for (int t = 0; t < OTA; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = 4 * t + i, col = 16 * t + 4 * g + i;
          const bool real = col < A;
          pv[k] = real ? ex[k] / ssum : 0.0f;
          B[k] = real ? kEps * __builtin_amdgcn_rcpf(pv[k] + kEps) : 0.0f;
          spBp += pv[k] * B[k];
          restp += (real && col != av) ? pv[k] : 0.0f;
        }
      const float spB = xadd_f<false>(xadd_f<true>(spBp)), rest = xadd_f<false>(xadd_f<true>(restp));
      const float adv = rowvalid ? advv : 0.0f;
      const float coef = -adv * invN / olda * pa;
      f32x4 P4[OTA], D4[OTA], S4[OTA];
#pragma unroll
      for (int t = 0; t < OTA; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = 4 * t + i, col = 16 * t + 4 * g + i;
          const bool real = col < A;
          P4[t][i] = pv[k];
          D4[t][i] = real ? pv[k] * invN * (B[k] - spB) : 0.0f;
          S4[t][i] = real ? coef * (col == av ? rest : -pv[k]) : 0.0f;
          if (rowvalid) {
            md = fmaxf(md, fabsf(D4[t][i]));
            mds = fmaxf(mds, fabsf(S4[t][i]));
          }
        }
      st_tiles(a.P, ldo, OTA, P4);
      st_tiles(a.D, ldo, OTA, D4);
      st_tiles(a.DS, ldo, OTA, S4);
    }
    if (rowvalid && g == 0) {
      const double adv = advv;
      a.rowterms[4 * row + 0] = (double)pa / (double)olda * adv;
      a.rowterms[4 * row + 1] = klt;
      a.rowterms[4 * row + 2] = ent;
      a.rowterms[4 * row + 3] = 0.0;
    }
  }
  if constexpr (PREP) amax_commit3(a.am_d, md, a.am_ds, mds, nullptr, 0.0f);
}

int ti0_of(int obs) { return obs <= 16 ? 1 : obs <= 32 ? 2 : obs <= 64 ? 4 : 8; }

template <int TI0, int MODE, int NH>
void launch_ti0(const Fused16Args& a, int grid, hipStream_t s) {
  constexpr int FW = FUSED16_FW, LB = FUSED16_LB;
  if (a.f.c.w[NH + 1] <= 16)
    hipLaunchKernelGGL((fvp_fused16_kernel<FW, LB, TI0, 1, MODE, NH>), dim3(grid), dim3(FW * 64), 0, s, a);
  else
    hipLaunchKernelGGL((fvp_fused16_kernel<FW, LB, TI0, 2, MODE, NH>), dim3(grid), dim3(FW * 64), 0, s, a);
}

template <int MODE, int NH>
void launch_nh(const Fused16Args& a, int grid, hipStream_t s) {
  switch (ti0_of(a.f.c.w[0])) {
    case 1: launch_ti0<1, MODE, NH>(a, grid, s); break;
    case 2: launch_ti0<2, MODE, NH>(a, grid, s); break;
    case 4: launch_ti0<4, MODE, NH>(a, grid, s); break;
    default: launch_ti0<8, MODE, NH>(a, grid, s); break;
  }
}

template <int MODE>
void launch_fused16(const Fused16Args& a, int grid, hipStream_t s) {
  constexpr bool PG = MODE >= 1;
  if (grid <= 0) return;
  if (!fused16_eligible(a.f.c.L, a.f.c.w)) throw std::runtime_error("fused16: unsupported shape");
  const int nh = a.f.c.L - 1;
  if (a.f.c.nchunks != fused16_obs_chunks(a.f.c.w[0]) + (nh == 2 ? 14 : 6))
    throw std::runtime_error("fused16: chunk table");
  const int rb = fused16_states_per_group();
  if (a.f.ngroups != (a.f.c.n + rb - 1) / rb) throw std::runtime_error("fused16: group count does not match");
  if (PG && !a.DS) throw std::runtime_error("fused16 policy gradient: no head delta");
  if (MODE == 2 && (!a.E0out || (nh == 2 && (!a.D1out || !a.E1out))))
    throw std::runtime_error("fused16 prepare backward: no outputs");
  if (nh == 2) launch_nh<MODE, 2>(a, grid, s);
  else launch_nh<MODE, 1>(a, grid, s);
}

}  // namespace

// one or two tanh hidden layers of width <= 64 (images padded to 64), obs <= 128, <= 32 actions
bool fused16_eligible(int L, const int* w) {
  if (L != 2 && L != 3) return false;
  if (w[0] < 1 || w[0] > 128 || w[L] < 1 || w[L] > 32) return false;
  for (int l = 1; l < L; ++l)
    if (w[l] < 1 || w[l] > 64) return false;
  return true;
}

int fused16_obs_chunks(int obs) { return (ti0_of(obs) + 1) / 2; }
int fused16_states_per_group() { return 16 * FUSED16_FW; }
int fused16_groups_per_cu() { return FUSED16_LB; }

void launch_fused16_img(const ChainImgArgs& a, const float* theta, const float* v, int which, const int* skip,
                        int* img_e, hipStream_t s) {
  int maxb = 1;
  for (int i = 0; i < a.n; ++i) {
    const ChainImgJob& j = a.job[i];
    if (j.K * j.O > kImgMax || j.K * j.O < 1) throw std::runtime_error("fused16 images: matrix size");
    if (j.which == which) maxb = std::max(maxb, (j.kc * j.otp * 4 + 255) / 256);
  }
  hipLaunchKernelGGL(fused16_img_kernel, dim3(maxb, a.n), dim3(256), 0, s, a, theta, v, which, skip, img_e);
}

void launch_cg_p_img16(const ChainImgArgs& a, const float* r, const float* p_old, float* p_new, int64_t n,
                       UpdScalars* sc, const double* partials2, CGFlags* fl, int it, int* img_e, hipStream_t s) {
  int maxb = 1;
  for (int i = 0; i < a.n; ++i) {
    const ChainImgJob& j = a.job[i];
    if (j.K * j.O > kImgMax || j.K * j.O < 1 || j.src_off + (int64_t)j.K * j.O > n)
      throw std::runtime_error("cg_p_img16: image job");
    if (j.which == 1) maxb = std::max(maxb, (j.kc * j.otp * 4 + 255) / 256);
  }
  maxb = std::max<int>(maxb, (int)std::min<int64_t>((n + 255) / 256, 64));   // the writer row's blocks
  hipLaunchKernelGGL(cg_p_img16_kernel, dim3(maxb, a.n + 1), dim3(256), 0, s, a, r, p_old, p_new, n, sc, partials2,
                     fl, it, img_e);
}

void launch_fwd_loss16(const FwdLoss16Args& a, int num_cus, hipStream_t s) {
  if (a.n <= 0) return;
  const bool prep = a.H1 != nullptr;
  const int nh = a.L - 1;
  if (prep && ((nh == 2 && !a.H2) || !a.P || !a.D || !a.DS)) throw std::runtime_error("fwd_loss16 prepare: missing output");
  if (!fused16_eligible(a.L, a.w)) throw std::runtime_error("fwd_loss16: unsupported shape");
  const int ti0 = ti0_of(a.w[0]);
  if (a.nchunks != (ti0 + 1) / 2 + 2 * nh) throw std::runtime_error("fwd_loss16: chunk table");
  const int64_t waves = (a.n + 15) / 16;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((waves + FWDL16_NW - 1) / FWDL16_NW, (int64_t)num_cus * 2));
  const bool two = a.w[a.L] > 16;
#define FWD_LOSS16_NH(T, NH)                                                                                       \
  if (prep) {                                                                                                      \
    if (two) hipLaunchKernelGGL((fwd_loss16_kernel<T, 2, true, NH>), dim3(grid), dim3(64 * FWDL16_NW), 0, s, a);  \
    else hipLaunchKernelGGL((fwd_loss16_kernel<T, 1, true, NH>), dim3(grid), dim3(64 * FWDL16_NW), 0, s, a);      \
  } else {                                                                                                         \
    if (two) hipLaunchKernelGGL((fwd_loss16_kernel<T, 2, false, NH>), dim3(grid), dim3(64 * FWDL16_NW), 0, s, a); \
    else hipLaunchKernelGGL((fwd_loss16_kernel<T, 1, false, NH>), dim3(grid), dim3(64 * FWDL16_NW), 0, s, a);     \
  }
#define FWD_LOSS16(T)       \
  if (nh == 2) {            \
    FWD_LOSS16_NH(T, 2)     \
  } else {                  \
    FWD_LOSS16_NH(T, 1)     \
  }
  switch (ti0) {
    case 1: FWD_LOSS16(1) break;
    case 2: FWD_LOSS16(2) break;
    case 4: FWD_LOSS16(4) break;
    default: FWD_LOSS16(8) break;
  }
#undef FWD_LOSS16
#undef FWD_LOSS16_NH
}

void launch_fvp_fused16(const Fused16Args& a, int grid, hipStream_t s) { launch_fused16<0>(a, grid, s); }
void launch_pg_fused16(const Fused16Args& a, int grid, hipStream_t s) { launch_fused16<1>(a, grid, s); }
void launch_prep_pg_fused16(const Fused16Args& a, int grid, hipStream_t s) { launch_fused16<2>(a, grid, s); }

}  // namespace trpo
