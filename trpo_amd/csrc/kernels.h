// Host-side launch interface of the HIP kernels (gemm.hip, vec.hip, scan.hip).
//
// Everything here is stream-ordered and allocation-free, so a caller may capture
// it into a hipGraph.  Pointers are device pointers.  Row-major activation
// arrays have a leading dimension that is a multiple of 4 floats (16-B rows)
// and zero-filled padding columns.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace trpo {

// Kernel-variant switches (defaults from TRPO_SPLIT_MFMA, TRPO_SPLIT_WG, TRPO_CHAIN, TRPO_SPLIT_F16,
// TRPO_SPLIT_MIN_K, TRPO_GRAPHS, TRPO_TAIL, TRPO_FUSED, TRPO_LOW_SEG, TRPO_PLANES, TRPO_RBWD0, TRPO_HBWD2,
// TRPO_HEAD_FWD, TRPO_SPLITS, TRPO_PG_SPLITS in gemm.hip; runtime-settable through trpo_set_option for A/B
// and parity tests).
struct Options {
  int split_mfma;  // row GEMMs with N > 128 on the split MFMA: 0 off (f32 MFMA), 5 = 256 x 256 tile at
                   // BK 32 on f16 planes (default), 6 = 256 x 256 at BK 16, any other value = 128 x 256
  int split_wg;    // weight gradients with fan_out > 128 on the split MFMA: 0 off (f32 MFMA), 1 on
  int chain;       // FVP R-forward + R-backward as one fused kernel (chain.hip): 0 off, 1 auto, 2..4 variant
  int split_f16;   // split GEMMs on f16 MFMA: operands scaled by powers of two and split hi+lo (3 products)
  int split_min_k; // row GEMMs whose every segment has K < split_min_k stay on f32 MFMA (epilogue-bound)
  int graphs;      // engine: replay the update's sync-free prefix as a captured hipGraph
  int tail;        // engine: fused last-layer FVP tail (tail.hip) where eligible: 0 off, 1 on
  int fused;       // engine: whole small-width FVP in one launch (fused.hip): 0 off, 1 = 8 waves, 2 = 4 waves,
                   // 3 (default) = on the f16 split (fused16.hip) where it applies, else 2
  int low_seg;     // f16 split GEMMs: a segment whose product scale sits >= low_seg binades below the other
                   // segment's runs on one product (hi x hi) instead of three; 0 = off (gemm.hip)
  int planes;      // engine: row GEMMs whose operands have pre-split k-blocked f16 planes take the LDS-DMA
                   // plane kernel (plane.hip): 0 off, 1 on
  int rbwd0;       // engine: layer 1's R-backward (and the policy gradient's backward into layer 0) fused
                   // with layer 0's weight gradient where eligible (rbwd0.hip): 0 off, 1 on
  int hbwd2;       // engine: the prepare pass's and the policy gradient's backward through the head layer in one
                   // launch that reads H once (hbwd.hip), with D_1's hi plane under rbwd0: 0 off, 1 on VALU fmaf
                   // chains, 2 (default) on f32 MFMA
  int head_fwd;    // engine: softmax head forwards with one state per lane on f32 FMAs (hbwd.hip) instead of the
                   // f32 MFMA row GEMM with its 32-lane row epilogue: 0 off, 1 (default) prepare + line search,
                   // 2 line search, and the prepare head when the head has <= 8 actions
  int splits;      // engine: weight-gradient split-K slabs of the FVP launches (0 = auto: 512 at C4)
  int pg_splits;   // engine: the policy gradient's split-K slabs (0 = auto: 4 x splits, at most 2048)
  int ls_fused;    // engine: the policy forwards in one launch (fused16.hip fwd_loss16) where the FVP runs on
                   // fused16: 1 (default) the prepare pass's and the line search's, 2 the line search's only,
                   // 0 neither (per-layer row GEMMs + head_fwd)
  int cg_fuse_reduce;  // engine: single rank with the one-launch FVP: each CG iteration's slab reduction fused with
                       // its z = Hv + damping p (vec.hip reduce_slab_kernel<true>): 1 (default) on, 0 off; the p.z
                       // partials are grouped differently, so 1 and 0 are not bit-identical to each other; 2 the
                       // rest of the iteration and the next V image in the same launch, run by the workgroup that
                       // finishes last (cg_step_slabs_kernel, bit-identical to 1; measured slower: DESIGN.md §6)
  int cg_p_img;        // engine, fused16 path: each CG iteration's p update and the next FVP's V images in one launch
                       // (fused16.hip cg_p_img16_kernel, bit-identical): 1 (default) on, 0 off
  int rfwd01;          // engine: the FVP's R-forward through layers 0 and 1 in one launch (rfwd.hip) where eligible
  int fwd01;           // engine: the prepare / line-search forward through layers 0 and 1 in one launch (rfwd.hip)
                       // (two hidden layers of 256, obs <= 128, the fused tail, X planes): 1 (default) on, 0 off
};

// A running-max slot is kAmaxSub counters, each on its own 128-B line: producers reduce within the
// workgroup and atomicMax into counter (block id mod kAmaxSub), so the device-scope atomics of a
// launch are few and spread; consumers take the max of the kAmaxSub counters (a few loads per lane).
constexpr int kAmaxSub = 256, kAmaxStride = 32, kAmaxSlot = kAmaxSub * kAmaxStride;   // in unsigned

// Power-of-two scale exponent for the f16 split: max|x| * 2^e lands in [2^11, 2^12).
__host__ __device__ inline int f16_scale_exp(float m) {
  if (!(m > 0.0f) || !(m < 3.0e38f)) return 0;
  int q = 0;
  (void)frexpf(m, &q);
  int e = 12 - q;
  return e < -100 ? -100 : (e > 100 ? 100 : e);
}
extern Options g_options;

// ---------------------------------------------------------------------------
// Row GEMM:  C[M x N] = sum_seg A_seg[M x K_seg] * B_seg[K_seg x Npad]  -> epilogue
// ---------------------------------------------------------------------------
struct GemmSeg {
  const float* A;  // [M][lda]
  const float* B;  // [K][ldb]
  int lda, ldb, K; // K multiple of 4
  // split GEMM only: B as bf16 planes (hi, mid, lo) [3][Npad][ldk] or, with RowGemmArgs::f16,
  // scaled f16 planes (hi, lo) [2][Npad][ldk]; k contiguous, zero for k >= K (launch_split_b);
  // plane = elements per plane
  const uint16_t* B3 = nullptr;
  int ldk = 0, plane = 0;
  // f16 split only: running max |A| / max |B| (float bits, atomicMax'd by their producers) that
  // set the power-of-two operand scales; NULL means "bounded by 1"
  const unsigned* amaxA = nullptr;
  const unsigned* amaxB = nullptr;
  // f16 split, pre-split operands (plane.hip): A = (Ah + Al) * 2^-(*eAp), f16 planes written once by their
  // producer, k-blocked: element (r, k) at ((k / 32) * mpad + r) * 32 + k % 32, k padded to ldp (a multiple of
  // 64) and rows to mpad (a multiple of 256), zero-filled; Bb = B's split planes k-blocked the same way,
  // [2][ldk / 32][Npad][32] (plane = ldk * Npad elements).  Ah != NULL selects the planes path.
  const uint16_t* Ah = nullptr;
  const uint16_t* Al = nullptr;
  int ldp = 0, mpad = 0;
  const int* eAp = nullptr;
  const uint16_t* Bb = nullptr;
};

enum class RowEpi : int {
  kTanh = 0,      // out = tanh(acc + bias)                      (policy forward, hidden)
  kRHidden = 1,   // RH = (1-H^2)(acc + bias)                    (R-forward, hidden)
  kPrepBwd = 2,   // D = acc(1-H^2); E = -2 acc H                (KL_ff plain backward)
  kPgBwd = 3,     // DS = acc(1-H^2)                             (surr backward)
  kRBwd = 4,      // RD = acc(1-H^2) + E RH                      (R-backward)
  kPrepHead = 5,  // softmax head: P, D_L, DS_L, row loss terms  (prepare)
  kLossHead = 6,  // softmax head: row loss terms only           (line search)
  kRHead = 7,     // R-softmax head: RD_L                        (FVP)
  kRelu = 8,      // out = max(acc + bias, 0)                    (VF forward, utils.py:60-61)
  kReluBwd = 9,   // out = acc * (H > 0), H = the ReLU output    (VF backward)
  kPrepBwdE = 10, // E = -2 acc H only                           (KL_ff plain backward into the first
                  //                                              hidden layer: D_0 has no reader)
  kRZ = 11,       // RZ = acc + bias                             (R-forward pre-activation of the last
                  //                                              hidden layer: the fused tail applies
                  //                                              (1-H^2) as it loads H, so H is read once)
};
// the row-wise softmax heads (one output row per 32-lane wave half, up to kMaxHeadTiles 32-column tiles)
constexpr int kMaxHeadTiles = 4;
constexpr bool epi_is_head(int e) { return e >= (int)RowEpi::kPrepHead && e <= (int)RowEpi::kRHead; }

struct RowEpiArgs {
  const float* bias;   // [N] (kTanh, kRHidden, heads)
  const float* H;      // [M][ldo] tanh activation at the output position
  const float* E;      // [M][ldo]
  const float* RH;     // [M][ldo]
  float* out0;         // tanh: H ; RHidden: RH ; PrepBwd: D ; PgBwd: DS ; RBwd: RD ; heads: P/RD_L
  float* out1;         // PrepBwd: E ; PrepHead: D_L
  float* out2;         // PrepHead: DS_L
  int ldo;             // leading dim of outputs/aux (multiple of 4)
  // heads
  const float* P;      // kRHead: cached softmax [M][ldo]
  const float* old;    // [M][ldo]
  const int* act;      // [M]
  const float* adv;    // [M]
  double* rowterms;    // [M][4] (surr*N, kl*N, ent*N, -)
  double invN;         // 1 / N_global
  // optional running max |out0| / |out1| / |out2| over the valid rows (float bits, atomicMax), the
  // operand scales of the f16 split GEMMs that consume these outputs
  unsigned* amax0 = nullptr;
  unsigned* amax1 = nullptr;
  unsigned* amax2 = nullptr;
};

struct RowGemmArgs {
  int M, N, Npad;      // rows; real output columns; padded output columns (<= ldb)
  int nseg;
  GemmSeg seg[2];
  const int* skip;     // optional device flag: launch is a no-op when *skip != 0
  RowEpi epi;
  RowEpiArgs ea;
  int f16 = 0;         // split path: 1 = two scaled f16 planes / 3 products, 0 = three bf16 planes / 6
  int low_seg = 0;     // f16: binade gap that puts the smaller segment on one product (0 = off; set at launch)
};

void launch_rowgemm(const RowGemmArgs& a, hipStream_t s);
// the pre-split-plane form (plane.hip); launch_rowgemm dispatches to it when seg[0].Ah is set
void launch_rowgemm_planes(const RowGemmArgs& a, hipStream_t s);
// f32 A [M][lda] -> scaled f16 planes hi/lo, k-blocked (GemmSeg::Ah; lo may be NULL: hi only); scale exponent
// f16_scale_exp(max |A|) from the running-max slot `amax` (NULL: |A| <= 1), written to *e_out
void launch_split_planes(const float* A, int M, int Mpad, int K, int lda, uint16_t* hi, uint16_t* lo, int ldp,
                         const unsigned* amax, int* e_out, hipStream_t s);
// k-block P planes [P][R][ld] (k contiguous) into [P][ld / 32][R][32] (GemmSeg::Bb)
void launch_block_planes(const uint16_t* src, int P, int R, int ld, uint16_t* dst, hipStream_t s);
// true when launch_rowgemm will take the split-bf16 path for this shape (the segments' B3 must be set)
bool rowgemm_uses_split(int Npad, RowEpi epi);

// Split fp32 matrices B [K][ldb] (columns [0, Npad)) into bf16 planes B3 [3][Npad][ldk]
// (hi = bf16(b), mid = bf16(b - hi), lo = bf16(b - hi - mid); k >= K zero-filled).
struct SplitJob {
  const float* B;
  uint16_t* B3;
  int K, Npad, ldb, ldk;
  const unsigned* amax = nullptr;   // f16: max |B| (float bits) that sets the plane scale
};
constexpr int kMaxSplitJobs = 16;
struct SplitArgs {
  int n;
  SplitJob job[kMaxSplitJobs];
  int f16 = 0;
};
void launch_split_b(const SplitArgs& a, const int* skip, hipStream_t s);

// ---------------------------------------------------------------------------
// Weight-gradient GEMM (split-K over rows):
//   slab[split][off_w + i*Nb + j] = sum_seg sum_rows A_seg[r][i] B_seg[r][j]
//   slab[split][off_b + j]        = sum_rows B_{colsum_seg}[r][j]
// ---------------------------------------------------------------------------
struct WSeg {
  const float* A;  // [rows][lda]
  const float* B;  // [rows][ldb]
  int lda, ldb;
  const unsigned* amaxA = nullptr;   // f16 split: max |A|, max |B| (float bits; NULL = bounded by 1)
  const unsigned* amaxB = nullptr;
};

struct WGradArgs {
  int rows;
  int Ma, Nb;          // real output dims (fan_in, fan_out)
  int Mpad, Npad;      // padded widths of A / B rows
  int nseg;
  WSeg seg[2];
  int colsum_seg;      // B of this segment is column-summed into the bias slot
  int splits, rows_per_split;  // rows_per_split multiple of 16
  float* slab;
  int64_t slab_stride; // floats between consecutive splits
  int64_t off_w, off_b;
  const int* skip;
  int f16 = 0;         // split path: scaled f16 (3 products) instead of bf16 (6 products)
  int low_seg = 0;     // f16: as RowGemmArgs::low_seg (set at launch)
};

void launch_wgrad(const WGradArgs& a, hipStream_t s);

// ---------------------------------------------------------------------------
// vector / scalar kernels (vec.hip)
// ---------------------------------------------------------------------------
struct LayerPack {
  int64_t off_w;   // offset of W_l [a x b] in the flat vector
  int a, b, apad, bpad;
  float* WF;       // [2*apad][bpad]: rows [0,a) = W ; rows [apad, apad+a) = V
  float* WB;       // [2*bpad][apad]: rows [0,b) = W^T ; rows [bpad, bpad+b) = V^T
  unsigned* amax = nullptr;   // optional: atomicMax of max |W_l| (float bits)
};
constexpr int kMaxLayers = 8;
struct PackArgs {
  int nl;
  LayerPack L[kMaxLayers];
};
// which = 0: source is theta -> W halves ; which = 1: source is a tangent -> V halves
void launch_pack(const PackArgs& pa, const float* src, int which, const int* skip, hipStream_t s);

// out[p] = sum_{s<S} slab[s*stride + p]
void launch_reduce_slab(const float* slab, int S, int64_t stride, int64_t P, float* out,
                        const int* skip, hipStream_t s);

// Device scalar state of one update (CG, step scaling, line search).
struct UpdScalars {
  float rdotr[2];     // CG ping-pong (utils.py:189,198)
  float alpha, mu;
  int iters;          // CG iterations run
  int pad0;
  float tol;
  float damping;
  // step scaling (trpo_inksci.py:148-151)
  float sdotz;        // stepdir . fvp(stepdir)
  float gdots;        // g . stepdir
  double shs, lm, rate;
  // losses (f32 like session.run)
  float loss_before[3];
  float loss_trial[3];
  float loss_after[3];
  int accepted, k, reverted, pad1;
  double max_kl;
};
constexpr int kMaxCG = 64;
struct CGFlags {
  int done[kMaxCG + 2];  // done[i] is read by iteration i, written by iteration i-1
};

void launch_dot_partials(const float* a, const float* b, int64_t n, double* partials,
                         const int* skip, hipStream_t s);
// CG of utils.py:185-201.  init: x = 0, r = b, p = b, rdotr = f32(b.b), flags cleared.
// iter `it` (no-op once done[it] is set): z = hv + damping p ; alpha = rdotr/(p.z) ;
// x += alpha p ; r -= alpha z ; mu = (r.r)/rdotr ; p = r + mu p ; done[it+1] = r.r < tol.
void launch_cg_init(const float* b, float* x, float* r, float* p, int64_t n, double* partials,
                    UpdScalars* sc, CGFlags* fl, float tol, float damping, hipStream_t s);
void launch_cg_iter(const float* hv, float* x, float* r, float* p, float* z, int64_t n, UpdScalars* sc,
                    double* partials, double* partials2, CGFlags* fl, int it, hipStream_t s);
// single rank, the one-launch FVP: its slab reduction fused with the iteration's z = Hv + damping p and p.z
// (vec.hip), then the x / r and p updates; P up to kRedBlocks x 64 parameters
bool cg_fused_reduce_ok(int64_t P);
// (p_update = false: the caller runs the p update itself, e.g. launch_cg_p_img16)
void launch_cg_iter_slabs(const float* slab, int S, int64_t stride, float* hv, float* x, float* r, float* p, float* z,
                          int64_t n, UpdScalars* sc, double* partials, double* partials2, CGFlags* fl, int it,
                          hipStream_t s, bool p_update = true);
// cg_fuse_reduce = 2: the whole iteration in one launch (vec.hip cg_step_slabs_kernel): the slab reduction and
// z / p.z as above, then, in the workgroup that finishes last (an agent-scope ticket that it resets), the x / r and
// p updates of launch_cg_iter_slabs with bit-identical results, and, when `img` has jobs (the fused16 path), the next
// FVP's V images and exponents (launch_fused16_img(..., which = 1) of the new p)
struct CgStepArgs {
  const float* slab;
  int S, it;
  int64_t stride, P;
  float *hv, *x, *r, *p, *z;
  UpdScalars* sc;
  double* partials;
  CGFlags* fl;
  unsigned* ticket;   // zero between launches
};
struct ChainImgArgs;
void launch_cg_step_slabs(const CgStepArgs& a, const ChainImgArgs* img, int* img_e, hipStream_t s);
struct CGScalarsD {
  double rdotr[2];
  double alpha, mu;
  int iters, pad;
  double tol, damping;
};
void launch_cg_init_d(const double* b, double* x, double* r, double* p, int64_t n, double* partials,
                      CGScalarsD* sc, CGFlags* fl, double tol, hipStream_t s);
void launch_cg_iter_d(const double* hv, double* x, double* r, double* p, double* z, int64_t n,
                      CGScalarsD* sc, double* partials, double* partials2, CGFlags* fl, int it,
                      hipStream_t s);

// z = hv + damping*stepdir; partials = stepdir.z ; partials2 = g.stepdir
void launch_shs_partials(const float* hv, const float* stepdir, const float* g, int64_t n,
                         const UpdScalars* sc, double* partials, double* partials2, hipStream_t s);
// shs, lm, rate (single block)
void launch_shs_finish(const double* partials, const double* partials2, UpdScalars* sc, hipStream_t s);
// fullstep = stepdir / f32(lm)
void launch_fullstep(const float* stepdir, float* fullstep, int64_t n, const UpdScalars* sc, hipStream_t s);
// trial = prev + f32(0.5^k) * fullstep (no-op when accepted)
void launch_ls_trial(const float* prev, const float* fullstep, float* trial, int64_t n, int k,
                     const UpdScalars* sc, hipStream_t s);

// row loss terms -> kRedBlocks partial triples
void launch_rowterms_partials(const double* rowterms, int64_t n, double* partials3,
                              const int* skip, hipStream_t s);
// local[0..2] = ordered sum of the partial triples
void launch_rowterms_finish(const double* partials3, double* local3, const int* skip, hipStream_t s);
// which: 0 -> loss_before, 1 -> loss_trial ; out3 = f32(-sum_surr/N, sum_kl/N, sum_ent/N)
void launch_losses_store(const double* global3, double invN, UpdScalars* sc, int which,
                         const int* skip, hipStream_t s);
// line search decision for backtrack k (utils.py:176-181)
void launch_ls_decide(UpdScalars* sc, int k, hipStream_t s);
// theta = accepted ? prev + 0.5^k fullstep : prev ; revert if kl > 2 max_kl (trpo_inksci.py:153-158)
void launch_ls_finalize(const float* prev, const float* fullstep, float* theta, float* theta_ls,
                        int64_t n, UpdScalars* sc, hipStream_t s);

void launch_axpby(float* y, const float* x, float alpha, float beta, int64_t n, hipStream_t s);  // y = alpha*x + beta*y
void launch_scale_copy(const float* x, float* y, float alpha, int64_t n, hipStream_t s);          // y = alpha*x
void launch_i64_to_i32(const int64_t* src, int* dst, int64_t n, int* bad, int hi, hipStream_t s);
void launch_f64_to_f32(const double* src, float* dst, int64_t n, hipStream_t s);
// out = max(out, max |A[r][c]|) over r < n, c < w (float bits via atomicMax)
void launch_amax(const float* A, int64_t n, int w, int ld, unsigned* out, hipStream_t s);
void launch_copy_rows(const float* src, int64_t n, int w, int ld_src, float* dst, int ld_dst, hipStream_t s);

// ---------------------------------------------------------------------------
// discount scan + standardisation (scan.hip)
// ---------------------------------------------------------------------------
// out[t] = x[t] + gamma*out[t+1] within episodes (starts[t] = 1 begins an episode)
size_t discount_workspace_bytes(int64_t n);
void launch_discount(const double* x, const uint8_t* starts, int64_t n, double gamma, double* out,
                     void* workspace, hipStream_t s);
// adv = returns - baseline ; partials = sum adv
void launch_adv_center_partials(const double* returns, const double* baseline, double* adv,
                                int64_t n, double* partials, hipStream_t s);
void launch_sum_finish(const double* partials, double* out, hipStream_t s);  // out[0] = ordered sum
// partials = sum (adv - mean)^2 with mean = global_sum[0] * inv_n
void launch_adv_sq_partials(const double* adv, int64_t n, const double* global_sum, double inv_n,
                            double* partials, hipStream_t s);
// adv = (adv - mean)/(sqrt(sq*inv_n) + 1e-8) ; adv32 = f32(adv)
void launch_adv_normalize(double* adv, float* adv32, int64_t n, const double* global_sum,
                          const double* global_sq, double inv_n, hipStream_t s);

}  // namespace trpo

namespace trpo {
// ---------------------------------------------------------------------------
// Fused row-local FVP chain (chain.hip): R-forward through every layer, the
// R-softmax head and the R-backward down to layer 1 in one launch, 16 states
// per wave with activations carried in MFMA accumulator layout; writes RH_l and
// RD_l for the weight-gradient GEMMs.  Eligible when hidden widths <= 256 and
// n_actions <= 32.
// ---------------------------------------------------------------------------
struct ChainArgs {
  int n, L;                          // rows of this shard; layers
  int w[kMaxLayers + 1];             // widths [obs, hidden..., A]
  int ld[kMaxLayers + 1];            // row strides pad4(w)
  const float* X;
  const float* H[kMaxLayers];        // H[l], l = 1..L-1
  float* RH[kMaxLayers];             // RH[l], l = 1..L-1 (written)
  const float* P;                    // softmax at theta
  const float* D[kMaxLayers];        // D[l], l = 0..L-1 (width w[l+1])
  const float* E[kMaxLayers];        // E[l], l = 0..L-2 (width w[l+1])
  float* RD[kMaxLayers];             // RD[l], l = 0..L-1 (written)
  const float* v;                    // tangent (flat), for the tangent biases
  int64_t offb[kMaxLayers];          // bias offsets in the flat vector
  const void* img;                   // weight images (16-B units)
  const int* tab;                    // per chunk (offset, size) in 16-B units, consumption order
  int nchunks;
  double invN;                       // 1 / N_global
  const int* skip;
};

// One weight image segment: a K x O block of W_l (trans = 0: W(o,k) = W_l[k][o],
// forward) or W_l^T (trans = 1: W(o,k) = W_l[o][k], backward), split into bf16
// hi/mid/lo planes in 32-deep k-chunks, k permuted to the accumulator pairing,
// rows swizzled for conflict-free ds_read_b128.  which: 0 = from theta, 1 = tangent.
struct ChainImgJob {
  int64_t src_off, dst_off;          // flat-vector offset of W_l; u16 offset in the image
  int K, O, ldw, trans, kc, otp, which, pad;
};
constexpr int kMaxChainJobs = 4 * kMaxLayers;
struct ChainImgArgs {
  int n;
  ChainImgJob job[kMaxChainJobs];
  unsigned short* img;
};
int chain_max_tiles(int max_hidden);   // register tiles for a max hidden width (0: not eligible)
void launch_fvp_chain(const ChainArgs& a, int otm, hipStream_t s);
void launch_chain_img(const ChainImgArgs& a, const float* theta, const float* v, int which, const int* skip,
                      hipStream_t s);

// ---------------------------------------------------------------------------
// Fused small-width FVP (fused.hip): the chain above plus the weight R-gradients in one
// persistent launch, for one or two hidden layers of width <= 64, obs <= 128, <= 32 actions.
// Reads the chain's ChainArgs (the RH / RD pointers are not used) and writes one partial Hv per
// workgroup to slab[blockIdx.x] (all P entries); launch_reduce_slab over `grid` slabs finishes it.
// variant 1: 8 waves, 128 states per group (one workgroup per CU); 2: 4 waves, 64 states.
// ---------------------------------------------------------------------------
struct FusedArgs {
  ChainArgs c;
  float* slab;
  int64_t slab_stride;
  int64_t offW[kMaxLayers];
  int ngroups;                       // ceil(n / states per group)
};
bool fused_fvp_eligible(int L, const int* w);
int fused_fvp_states_per_group(int variant);
void launch_fvp_fused(const FusedArgs& a, int grid, int variant, hipStream_t s);

// The same one-launch FVP on the f16 split (fused16.hip) for one or two hidden layers of width <= 64, obs <= 128
// and <= 32 actions (C1, C2, C3; hidden dimensions padded to 64 in the images).  Weight images: the chain's job list (ChainImgJob; kc = fused16_obs_chunks(obs) for
// V_0) as 32-deep chunks of [2 f16 planes (hi, lo)][otp rows][32], each job scaled by a power of two whose
// exponent launch_fused16_img writes to img_e[job]; jobs in the order V_0 | W_1 V_1 | W_2 V_2 | W_2^T V_2^T |
// W_1^T V_1^T (one hidden layer: V_0 | W_1 V_1 | W_1^T V_1^T; hidden K padded to 2 chunks, hidden O to 64 rows).  X, D_1 and D_2 are scaled from the engine's running-max slots.
constexpr int kFused16Jobs = 9;
struct Fused16Args {
  FusedArgs f;                       // f.c.img / f.c.tab / f.c.nchunks: the f16 images and their chunk table
  const int* img_e;                  // [kFused16Jobs] scale exponents of the images
  const unsigned* am_x;              // running-max slots: X, D_1, D_2
  const unsigned* am_d1;
  const unsigned* am_d2;
  const float* DS;                   // policy gradient only: the head's surr logit delta DS_2 [n][ld 3] and its slot
  const unsigned* am_ds2;
  float* D1out;                      // with the prepare backward (launch_prep_pg_fused16): D_1, E_1 [n][ld 2], E_0
  float* E1out;                      // [n][ld 1] and D_1's running-max slot
  float* E0out;
  unsigned* am_d1_out;
};
bool fused16_eligible(int L, const int* w);
int fused16_obs_chunks(int obs);     // 32-deep k-chunks of V_0's image (obs rounded to 32, 64 or 128)
int fused16_states_per_group();
int fused16_groups_per_cu();
// the CG's p update (cg_p_kernel, bit-identical) into p_new with the V images of p_new (fused16_img_kernel, which = 1)
void launch_cg_p_img16(const ChainImgArgs& a, const float* r, const float* p_old, float* p_new, int64_t n,
                       UpdScalars* sc, const double* partials2, CGFlags* fl, int it, int* img_e, hipStream_t s);
void launch_fused16_img(const ChainImgArgs& a, const float* theta, const float* v, int which, const int* skip,
                        int* img_e, hipStream_t s);
void launch_fvp_fused16(const Fused16Args& a, int grid, hipStream_t s);
// The policy gradient of the same shapes in one launch (fused16.hip, PG form): DS_1, DS_0 by the backward chain
// over W_2^T / W_1^T's image chunks and g's blocks H_l^T DS_l + colsum DS_l into the slabs, as the FVP's.
void launch_pg_fused16(const Fused16Args& a, int grid, hipStream_t s);
// ... and with it, on the same weight chunks, the prepare pass's backward below the head: D_1, E_1, E_0 and D_1's
// running max (engine.cpp prepare())
void launch_prep_pg_fused16(const Fused16Args& a, int grid, hipStream_t s);
// Line-search loss forward for the same shapes (fused16.hip fwd_loss16_kernel): the row terms of
// trpo_inksci.py:46-53 at a trial theta, from that theta's W_0 | W_1 | W_2 images (ChainImgJob, which = 0, the
// order here; img_e per job) resident in LDS, one wave per 16 states, no barrier in the loop.
struct FwdLoss16Args {
  int64_t n;
  int L = 3;                         // layers (2: one hidden layer, w = [obs, h1, A])
  int w[4], ld[4];                   // widths [obs, h1, h2, A]; row strides
  const float* X;
  const float* theta;                // the trial vector (biases)
  int64_t offb[3];
  const void* img;                   // W_0 | W_1 | W_2 images (16-B units)
  const int* tab;                    // per chunk (offset, size) in 16-B units
  int nchunks;
  const int* img_e;                  // [3]
  const unsigned* am_x;
  const float* old;                  // [n][ld[3]]
  const int* act;
  const float* adv;
  double* rowterms;                  // [n][4]
  const int* skip;
  // the prepare pass (H1 != NULL): H_1, H_2 [n][ld[1|2]], P / D_2 / DS_2 [n][ld[3]] and the maxima of D_2, DS_2
  float* H1 = nullptr;
  float* H2 = nullptr;
  float* P = nullptr;
  float* D = nullptr;
  float* DS = nullptr;
  unsigned* am_d = nullptr;
  unsigned* am_ds = nullptr;
  double invN = 0.0;
};
void launch_fwd_loss16(const FwdLoss16Args& a, int num_cus, hipStream_t s);
}  // namespace trpo

namespace trpo {
// ---------------------------------------------------------------------------
// Fused last-layer FVP tail (tail.hip), for the f16-split engine when the last hidden width is
// in (128, 256] (a multiple of 32) and n_actions <= 32.  Per 32-row tile of a split-K slab:
//   RZ = RH W + H V + c ; RD_L = R-softmax-reverse(RZ)             (head R-forward, kRHead)
//   RD_out = (RD_L W^T + D_L V^T)(1-H^2) - 2 (D_L W^T) H RH        (R-backward, E recomputed)
//   slab  += RH^T D_L + H^T RD_L ; bias += colsum RD_L              (weight R-gradient)
// reading RH and H once.  All products on the scaled f16 hi+lo split.
// ---------------------------------------------------------------------------
constexpr int kTailK = 256;   // max hidden width of the tail (head planes are [2][2][32][kTailK])
struct TailArgs {
  int rows, a, b, apad, bpad;
  const float* RH;            // [rows][apad]  R{h} of the last hidden layer, or with rz its pre-activation RZ
  const float* H;             // [rows][apad]  its tanh activations
  int rz = 0;                 // 1: RH holds RZ (kRZ); R{h} = (1-H^2) RZ is formed on load (same f32 ops as kRHidden)
  const float* P;             // [rows][bpad]  softmax at theta
  const float* DL;            // [rows][bpad]  KL_ff plain logit delta D_{L-1}
  const float* c;             // [b]           tangent bias of the last layer
  const uint16_t* WV16;       // head planes [mat W,V][plane hi,lo][32 j][kTailK k] (launch_tail_pack)
  const uint16_t* WT16;       // R-backward planes of W^T: [plane][apad n][32 k], plane stride bplane
  const uint16_t* VT16;       // ... of V^T
  int64_t bplane;
  const unsigned *am_rh, *am_d, *am_w, *am_v;   // running-max slots of RH, D_L, W, V
  unsigned* am_out;           // running max |RD_out|
  float* RDout;               // [rows][apad]  R-delta into the last hidden layer (RD_{L-2})
  double invN;
  int splits, rows_per_split; // rows_per_split % 32 == 0
  float* slab;
  int64_t slab_stride, off_w, off_b;
  const int* skip;
};
struct TailPackArgs {
  const float* theta;
  const float* v;
  int64_t off_w;              // flat offset of W_{L-1} [a][b]
  int a, b;
  const unsigned *am_w, *am_v;
  uint16_t* out;              // [2][2][32][kTailK]
};
bool tail_eligible(int apad, int bpad);   // (128, kTailK] multiple of 32; bpad in (16, 32]

// ---------------------------------------------------------------------------
// R-backward into the first hidden layer fused with layer 0's weight R-gradient (rbwd0.hip).
// Per 128-row tile of a split-K slab (trpo_inksci.py:56-70):
//   RD_0  = ([RD_1 | D_1] [W_1^T ; V_1^T]) (1 - H_1^2) + E_0 RH_1      (kept in registers, never stored)
//   slab += X^T RD_0 ;  bias += colsum RD_0                            (Hv's W_0 / b_0 blocks)
// With nseg = 1, no E and no RH it is the policy gradient's DS_0 = (DS_1 W_1^T)(1 - H_1^2) and X^T DS_0
// (trpo_inksci.py:54).  Hidden width <= 256 (wave w owns output columns [32w, 32w + 32)), obs <= 128 on
// X's pre-split k-blocked f16 planes; products on the scaled f16 hi+lo split.
// ---------------------------------------------------------------------------
struct RBwd0Args {
  int rows;                 // rows of this rank's shard
  int K, lda;               // per-segment K (the layer-1 output width) and A's leading dimension
  int N, Npad;              // layer-1 input width (RD_0's columns), padded (<= 256, multiple of 32)
  int obs;                  // X's real columns (<= 128)
  int nseg;                 // 2: [RD_1 | D_1] ; 1: DS_1 alone
  const float* A0;          // [rows][lda] RD_1 (or DS_1)
  const float* A1;          // [rows][lda] D_1
  const uint16_t* A1h;      // D_1's k-blocked f16 hi plane (GemmSeg::Ah layout, scale 2^(*eA1p)); NULL: none
  const int* eA1t = nullptr;   // ... or, when set, one scale 2^eA1t[r / 32] per 32-row tile (hbwd.hip)
  int a1_mpad;
  const int* eA1p;
  const uint16_t* B0;       // f16 hi/lo planes of W_1^T: [2][Npad][ldk] (plane stride `plane`)
  const uint16_t* B1;       // ... of V_1^T
  int ldk;
  int64_t plane;
  const unsigned *am_a0, *am_b0, *am_a1, *am_b1;   // running-max slots of the segment operands
  const float* H;           // [rows][Npad] H_1
  const float* E;           // [rows][Npad] E_0 (NULL: no E RH term)
  const float* RH;          // [rows][Npad] RH_1
  const uint16_t* Xh;       // X's k-blocked f16 planes (GemmSeg::Ah layout), scale 2^(*eX)
  const uint16_t* Xl;
  int x_mpad, x_ldp;
  const int* eX;
  int splits, rows_per_split;
  float* slab;
  int64_t slab_stride, off_w, off_b;
  const int* skip;
  int low_seg = 0;          // f16: segment 1 on one product when it sits >= low_seg binades under (set at launch)
};
// The prepare pass's and the policy gradient's backward through the head layer in one read of H (hbwd.hip):
//   D1 = (D2 W^T)(1 - H^2), DS1 = (DS2 W^T)(1 - H^2)  (K = n_actions <= 32), the policy gradient's head-layer
// weight gradient H^T DS2 (+ bias colsum) into the slabs, optionally D1's f16 hi plane
// (GemmSeg::Ah layout, row stride d1_mpad, scale 2^eD1t[r / 32] per 32-row tile)
struct HeadBwd2Args {
  int rows;
  int A, Apad;              // actions; leading dimension of D2 / DS2
  int N, Npad;              // last hidden width; leading dimension of H / D1 / DS1
  const float* WB;          // W^T rows [0, A) of the packed backward operand, [.][Npad]
  const float* D2;
  const float* DS2;
  const float* H;
  float* D1;
  float* DS1;
  unsigned* am_d1;
  unsigned* am_ds1;
  uint16_t* D1h = nullptr;
  int d1_mpad = 0;
  int* eD1t = nullptr;
  float* E1 = nullptr;       // E_{L-2} = -2 (D_{L-1} W^T) H (the kPrepBwd epilogue's second output), when read
  // workgroup s takes the rows of split s (the weight-gradient slab partition); slab != NULL: it also writes the
  // policy gradient's last-layer weight gradient (H^T DS2, W block [N][A] at off_w, bias colsum DS2 at off_b) of
  // its rows into slab s
  int splits = 0, rows_per_split = 0;
  float* slab = nullptr;
  int64_t slab_stride = 0, off_w = 0, off_b = 0;
};
bool head_bwd2_eligible(int A, int Npad);
// The softmax head forward with one state per lane (hbwd.hip): z = H W + b (K = last hidden width, A <= 32 actions),
// p = softmax(z), the surr / kl / ent row terms, and with prep also P, D_L, DS_L (gemm.hip kPrepHead semantics)
struct HeadFwdArgs {
  int64_t rows;
  int A, Apad;              // actions; leading dimension of old / P / D / DS and of W's rows
  int K, Kpad;              // last hidden width; leading dimension of H
  const float* H;
  const float* W;           // [K][Apad] (the packed forward operand's W half)
  const float* bias;        // [A]
  const float* old;
  const int* act;
  const float* adv;
  double* rowterms;         // [rows][4]
  double invN;
  int prep = 0;
  float* P = nullptr;
  float* D = nullptr;
  float* DS = nullptr;
  unsigned* am_d = nullptr;
  unsigned* am_ds = nullptr;
};
bool head_fwd_eligible(int A, int K);
void launch_head_fwd(const HeadFwdArgs& a, int num_cus, hipStream_t s);
void launch_head_bwd2(const HeadBwd2Args& a, int num_cus, hipStream_t s);
// The R-forward through layers 0 and 1 in one launch (rfwd.hip, option rfwd01): RH1 = (1 - H1^2)(X V0 + c0)
// (stored) and RZ2 = RH1 W1 + H1 V1 + c1 (stored, the fused tail's pre-activation) for two hidden layers of 256
// and obs <= 128, X from its pre-split planes, V0 / W1 / V1 from a per-FVP chunk image (launch_rfwd01_img).
struct Rfwd01Args {
  int64_t n;
  int obs, ldh, ldz;                 // obs; row strides of H1 / RH1 and of RZ2 (floats)
  const uint16_t *Xh, *Xl;           // X's k-blocked f16 planes (GemmSeg::Ah), x_mpad rows per 32-k block
  int x_mpad;
  const int* eX;                     // their scale exponent
  const float *H1, *c0, *c1;         // H1; the tangent biases of layers 0 and 1 (v + offb[l])
  const float* V0;                   // the direction's layer-0 block, [obs][256] (v + offW[0])
  float *RH1, *RZ2;
  const uint16_t* img;               // rfwd01_img_bytes()
  const unsigned *am_v0, *am_w1, *am_v1;   // the images' running-max slots
  unsigned *am_rh1, *am_rz2;         // running max |RH1|, |RZ2| (atomicMax'd)
  const int* skip;
};
// The policy forward through layers 0 and 1 in one launch (rfwd.hip, option fwd01): H1 = tanh(X W0 + b0) (stored
// when H1 is set: the prepare pass) and H2 = tanh(H1 W1 + b1), same shapes as rfwd01, W0 / W1 from a per-forward
// chunk image (launch_fwd01_img).
struct Fwd01Args {
  int64_t n;
  int obs;
  const uint16_t *Xh, *Xl;           // X's k-blocked f16 planes, x_mpad rows per 32-k block
  int x_mpad;
  const int* eX;
  const float *b0, *b1;              // th + offb[0], th + offb[1]
  float *H1, *H2;                    // H1: NULL = not stored (the line search)
  const uint16_t* img;               // fwd01_img_bytes()
  const unsigned *am_w0, *am_w1;     // the weights' running-max slots (the image's scales)
};
bool fwd01_eligible(int L, const int* w, const int* wp);
size_t fwd01_img_bytes();
void launch_fwd01_img(const float* th, int64_t offW0, int64_t offW1, int obs, const unsigned* am_w0,
                      const unsigned* am_w1, uint16_t* img, hipStream_t s);
void launch_fwd01(const Fwd01Args& a, int num_cus, hipStream_t s);
bool rfwd01_eligible(int L, const int* w, const int* wp);
size_t rfwd01_img_bytes();
void launch_rfwd01_img(const float* theta, const float* v, int64_t offV0, int64_t offW1, int obs,
                       const unsigned* am_v0, const unsigned* am_w1, const unsigned* am_v1, uint16_t* img,
                       const int* skip, hipStream_t s);
void launch_rfwd01(const Rfwd01Args& a, int num_cus, hipStream_t s);
bool rbwd0_eligible(int obs_pad, int x_ldp, int hid_pad, int K);
void launch_rbwd0(const RBwd0Args& a, hipStream_t s);
void launch_tail_pack(const TailPackArgs& p, hipStream_t s);
void launch_fvp_tail(const TailArgs& a, hipStream_t s);
}  // namespace trpo

namespace trpo {
// ---------------------------------------------------------------------------
// Value-function baseline (vf.hip), utils.py:48-92
// ---------------------------------------------------------------------------
size_t vf_pos_workspace_bytes(int64_t n);
// feat [n][Fp] = [obs | dist | f32(t/10)] with t the step index within each path
// (starts[r] = 1 opens a path; starts may be NULL: one path); lastpos [n] scratch
void launch_vf_features(const float* obs, int obs_dim, int ld_obs, const float* dist, int A, int ld_dist,
                        const uint8_t* starts, int64_t n, int64_t* lastpos, void* ws, float* feat, int Fp,
                        hipStream_t s);
struct VFPackArgs {
  int F, H1, H2, H1p, H2p;
  int64_t offW1, offW2;   // flat offsets of W1 [F][H1], W2 [H1][H2]
  float* W1p;             // [Fp][H1p]
  float* W2p;             // [H1p][H2p]
  float* W2T;             // [H2p][H1p]
};
void launch_vf_pack(const VFPackArgs& a, const float* theta, hipStream_t s);
struct VFHeadArgs {
  int64_t n;
  int H2, H2p;
  const float* Z2;        // [n][H2p]
  const float* w3;        // [H2]
  const float* b3;        // [1]
  int train;
  const float* y;         // [n]            train
  float* dout;            // [n][4]         train: col 0 = d(loss)/d(net)
  float* dZ2;             // [n][H2p]       train
  double* loss_rows;      // [n]            train: (net - y)^2
  float* out32;           // [n]            predict (if out64 == NULL)
  double* out64;          // [n]            predict
};
void launch_vf_head(const VFHeadArgs& a, hipStream_t s);
void launch_adam(float* var, const float* g, float* m, float* v, int64_t n, float alpha, float b1, float b2, float eps,
                 hipStream_t s);
}  // namespace trpo

namespace trpo {
// ---------------------------------------------------------------------------
// Batched sampling and CartPole-v0 rollouts (rollout.hip): agent.act
// (trpo_inksci.py:76-87), cat_sample (utils.py:95-105), rollout (utils.py:18-45)
// ---------------------------------------------------------------------------
struct PolicyShape {
  int L;
  int w[kMaxLayers + 1];
  int64_t offW[kMaxLayers], offb[kMaxLayers];
};
struct RolloutArgs {
  PolicyShape ps;
  const float* theta;
  int maxw;                 // max layer width (LDS slice per wave: 2 * maxw floats)
  int n_envs, max_pathlength, time_limit, train;
  int64_t budget;           // steps per environment: ceil(n_timesteps / n_envs)
  int64_t env_cap;          // rows per environment region: budget + max episode length - 1
  int max_episodes;         // second dim of reset_u
  uint64_t seed;
  const double* reset_u;    // optional [n_envs][max_episodes][4] uniforms for env.reset
  const double* act_u;      // optional [n_envs][env_cap] uniforms for cat_sample
  // per-environment regions (row = env * env_cap + i)
  double* obs;              // [.][obs_dim]
  int64_t* actions;
  float* dist;              // [.][A]
  double* rewards;
  uint8_t* starts;
  double* uniforms_out;     // optional: the cat_sample uniform of every step
  int64_t* counts;          // [n_envs] steps collected
  int64_t* episodes;        // [n_envs] episodes collected
};
struct RolloutOut {         // concatenated outputs; any pointer may be NULL
  double* obs64;            // [N][obs_dim]
  float* X;                 // [N][ldx]   (engine batch: f32 states)
  int ldx;
  float* dist;              // [N][A]
  float* old;               // [N][ld_old] (engine batch: oldaction_dist)
  int ld_old;
  int64_t* actions64;
  int* act32;
  double* rewards;
  uint8_t* starts;
  double* uniforms;
};
size_t rollout_lds_bytes(int maxw);
void launch_rollout(const RolloutArgs& a, hipStream_t s);
void launch_rollout_compact(const RolloutArgs& a, const int64_t* offsets, const RolloutOut& o, int64_t max_count,
                            hipStream_t s);
void launch_act(const PolicyShape& ps, const float* theta, int maxw, const float* states, int64_t n, const double* r,
                int train, int64_t* actions, float* dists, hipStream_t s);
void launch_cat_sample(const float* prob, int64_t n, int k, const double* r, int64_t* out, hipStream_t s);
void launch_cartpole_step(const double* state, const int64_t* action, int64_t n, double* state_out, double* reward,
                          uint8_t* done, hipStream_t s);
}  // namespace trpo
