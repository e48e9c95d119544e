// Runtime of the TRPO update engine behind the C-ABI of include/trpo_engine.h.
//
// One engine = one GPU = one shard of the state batch.  It owns every device
// buffer of the update (HBM layout in DESIGN.md), one HIP stream, and an
// optional RCCL communicator.  The reference's session.run calls
// (trpo_inksci.py:126,129,146,156) become kernel sequences on that stream:
//
//   prepare()      policy forward at theta + the KL_ff plain backward; caches
//                  H_l, P, D_l, E_l (fixed while theta is fixed, i.e. over the
//                  whole CG solve — the reference recomputes them per call)
//   policy_grad()  surr backward + weight-gradient GEMMs (flatgrad, :54)
//   fvp()          R-forward + R-backward + weight gradients (:56-70)
//   cg()           utils.py:185-201 with scalars on device and an early-exit flag
//   update()       trpo_inksci.py:144-158
#include "../../include/trpo_engine.h"
#include "abi_util.h"
#include "common.h"
#include "kernels.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

using namespace trpo;

using namespace trpo_abi;

struct trpo_engine {
  int device = 0;
  int num_cus = 256;               // compute units of `device` (hipDeviceAttributeMultiprocessorCount)
  hipStream_t stream = nullptr;
  // policy shape
  int L = 0;                       // layers
  std::vector<int> w, wp;          // widths [obs, hidden..., A] and padded
  int64_t P = 0;
  std::vector<int64_t> offW, offb;
  int64_t cap = 0, n = 0, n_global = 0;
  // multi-GPU
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
  trpo_allreduce_cb host_ar = nullptr;   // test transport (trpo_comm_set_host_allreduce)
  void* host_ar_ctx = nullptr;
  std::vector<uint8_t> host_ar_buf;

  // ---- device buffers ----
  std::vector<void*> allocs;
  float *theta = nullptr, *theta_prev = nullptr, *theta_trial = nullptr, *theta_ls = nullptr;
  float *g = nullptr, *bneg = nullptr, *x = nullptr, *r = nullptr, *p = nullptr, *z = nullptr;
  float* p2 = nullptr;   // the CG's second direction buffer (p ping-pongs when the p update writes a new buffer)
  float *hv = nullptr, *stepdir = nullptr, *fullstep = nullptr, *vin = nullptr, *vout = nullptr;
  std::vector<float*> WF, WB, WFt;   // packed [W;V], [W^T;V^T], trial forward weights
  float* WBt_scratch = nullptr;
  // bf16 (hi, mid, lo) planes of the packed matrices for the split-bf16 row GEMM:
  // [part][3][Npad][r16(K)], part 0 = W half, 1 = V half (WF3t: W half only)
  std::vector<uint16_t*> WF3, WB3, WFt3;
  bool w3_valid = false;   // W halves of WF3/WB3 match WF/WB
  float* X = nullptr;
  float* stage = nullptr;   // staging for host inputs / compact outputs: cap rows of max(pad4(obs), pad4(A), 2) floats
  int* act = nullptr;
  float *adv32 = nullptr, *old = nullptr;
  double *rewards = nullptr, *returns = nullptr, *adv64 = nullptr, *baseline = nullptr;
  uint8_t* starts = nullptr;
  bool have_baseline = false, have_rewards = false, have_returns = false;
  double* ev_tmp = nullptr;   // explained_variance scratch
  std::vector<float*> H, D, E, RH, RD;   // indexed as in DESIGN.md
  float *Pm = nullptr, *DSL = nullptr;
  double* rowterms = nullptr;
  float* slab = nullptr;
  int S = 1, rows_per_split = 16;
  int S_pg = 1, S_cur = 1;
  int64_t slab_stride = 0;
  double *partA = nullptr, *partB = nullptr, *part3 = nullptr, *local3 = nullptr, *dscal = nullptr;
  void* scan_ws = nullptr;
  UpdScalars* sc = nullptr;
  CGFlags* fl = nullptr;
  int* dbad = nullptr;
  UpdScalars* hsc = nullptr;   // pinned host mirror

  bool prepared = false;
  // f16 split GEMMs: running max |operand| slots (float bits) that set the power-of-two scales,
  // grouped by kind, kMaxLayers slots per group (see am_*)
  bool f16 = false;
  unsigned* amax = nullptr;
  unsigned* am(int group, int l) const {
    return f16 ? amax + (size_t)(1 + group * kMaxLayers + l) * kAmaxSlot : nullptr;
  }
  unsigned* am_x() const { return f16 ? amax : nullptr; }
  unsigned* am_w(int l) const { return am(0, l); }
  unsigned* am_v(int l) const { return am(1, l); }
  unsigned* am_wt(int l) const { return am(2, l); }
  unsigned* am_d(int l) const { return am(3, l); }
  unsigned* am_ds(int l) const { return am(4, l); }
  unsigned* am_rh(int l) const { return am(5, l); }
  unsigned* am_rd(int l) const { return am(6, l); }
  void am_reset(unsigned* first, int count) {
    if (first && count > 0)
      HIPCHECK(hipMemsetAsync(first, 0, (size_t)count * kAmaxSlot * sizeof(unsigned), stream));
  }
  // pre-split k-blocked f16 planes for the plane row GEMM (plane.hip): X's hi/lo planes, refreshed with X's
  // running max whenever X changes (layout stride x_mpad = round256(n)), and blocked copies of layer 0's
  // W / V weight planes, re-blocked from WF3 / WFt3 before each use
  uint16_t *Xh = nullptr, *Xl = nullptr, *W0b = nullptr, *V0b = nullptr;
  int* pl_e = nullptr;   // scale exponents published by the plane producers: [0] = X, [1] = D_1
  // D_1's f16 hi plane (k-blocked like Xh, stride d1_mpad = round256(n)), written by prepare() for the fused
  // R-backward's one-product D_1 V_1^T segment (rbwd0.hip)
  uint16_t* D1h = nullptr;
  int d1_mpad = 0, d1_ldp = 0;
  bool d1_plane = false;   // D1h holds the current D_1
  bool d1_tiled = false;   // ... with one scale per 32-row tile (eD1t, hbwd.hip) instead of pl_e[1]
  int* eD1t = nullptr;
  // the prepare pass also produced the policy gradient's DS_{L-2} (hbwd.hip, in RD[L-2]); any launch that
  // writes RD clears it
  bool ds_ready = false;
  // fused16.hip's prepare launch also left the policy gradient's blocks in the first pg_grid slabs; any slab writer
  // clears it
  bool pg_ready = false;
  int pg_grid = 0;
  bool use_hbwd2() const {
    // a hidden layer below the head layer, wider than 128 (one thread per column: at 64 columns three
    // quarters of its lanes idle, and C3 ran 3 % slower than on the row GEMMs); E_{L-2} is written too
    // where the FVP path reads it (no fused tail)
    return g_options.hbwd2 != 0 && L >= 3 && wp[L - 1] > 128 && head_bwd2_eligible(w[L], wp[L - 1]);
  }
  int x_mpad = 0, x_ldp = 0;
  bool x_planes = false;   // Xh/Xl hold the current X
  bool planes_geom_l0() const {   // layer 0's row GEMMs fit the plane kernel
    return L >= 2 && wp[1] % 256 == 0 && r16(wp[0]) % 64 == 0;
  }
  bool planes_l0() const {
    return x_planes && planes_geom_l0() && g_options.planes != 0 && split_on() &&
           rowgemm_uses_split(wp[1], RowEpi::kTanh);
  }
  // X's planes also feed the fused layer-1 R-backward + layer-0 weight gradient (rbwd0.hip)
  bool rbwd0_geom() const { return L >= 2 && rbwd0_eligible(wp[0], (wp[0] + 63) / 64 * 64, wp[1], wp[2]); }
  // attach X's planes and the blocked copy (into `dst`) of the 2 weight planes at `w3` to a layer-0 segment
  void attach_x_planes(GemmSeg& sg, const uint16_t* w3, uint16_t* dst) {
    launch_block_planes(w3, 2, wp[1], r16(wp[0]), dst, stream);
    sg.Ah = Xh;
    sg.Al = Xl;
    sg.ldp = x_ldp;
    sg.mpad = x_mpad;
    sg.eAp = pl_e;
    sg.Bb = dst;
  }
  uint16_t* tail_planes = nullptr;   // head planes of the fused FVP tail (tail.hip), [2][2][32][kTailK]
  // the fused last-layer tail: f16 split, last hidden width in (128, 256], 17..32 actions
  bool use_tail() const {
    return g_options.tail != 0 && f16 && split_on() && L >= 2 &&
           tail_eligible(wp[L - 1], wp[L]) && w[L] <= 32;
  }
  // whether the FVP path reads E_{L-2} (the plain tanh'' term under the last hidden layer): every path
  // but the fused tail, which recomputes it (tail.hip)
  bool e_top_needed() const { return L < 2 || !use_tail() || use_fused() || use_chain(); }
  bool prep_e_top = true;    // prepare() wrote E_{L-2}
  bool prep_fused16 = false; // prepare() took the fused16 branch (D_1 / E_1 / E_0 and the pg slabs from bwd_pg)
  // prepare()'s outputs belong to the other kernel path when option fused / split_f16 changed after it ran
  void reprepare_if_path_changed() {
    if (prepared && ((e_top_needed() && !prep_e_top) || prep_fused16 != use_fused16())) prepared = false;
  }

  // fused FVP chain (chain.hip): weight images in consumption order + chunk table
  int chain_otm = 0;         // register tiles per hidden layer; 0 = shape not eligible
  uint16_t* chain_img = nullptr;
  int* chain_tab = nullptr;
  int chain_nchunks = 0;
  bool chain_w_valid = false;   // theta parts of the images match theta
  ChainImgArgs chain_jobs{};
  // auto (option 1) takes the chain up to 8 register tiles (hidden widths <= 128), where it
  // beats the per-layer row GEMMs; at 16 tiles its per-128-state weight re-streaming
  // (~2 MB of bf16 planes per workgroup tile) costs more than the fusion saves
  // whole FVP (R-forward, head, R-backward and weight gradients) in one launch (fused.hip): one or
  // two hidden layers of width <= 64, obs <= 128, <= 32 actions; reuses the chain's weight images
  bool use_fused() const { return g_options.fused != 0 && chain_otm > 0 && fused_fvp_eligible(L, w.data()); }
  // the same launch on the f16 split (fused16.hip, option fused = 3): two hidden layers of width 49..64; its
  // own weight images (2 f16 planes, one scale exponent per job in f16_e) and chunk table
  uint16_t* f16_img = nullptr;
  int* f16_tab = nullptr;
  int* f16_e = nullptr;
  bool f16_v_img_ready = false;   // cg(): the V images of the next fvp_fused16 were built by the CG step launch
  unsigned* cg_ticket = nullptr;  // cg_step_slabs_kernel's arrival ticket (zero between launches)
  int f16_nchunks = 0;
  bool f16_w_valid = false;     // theta parts of the f16 images match theta
  ChainImgArgs f16_jobs{};
  // the line-search loss forward's images (W_0 | W_1 | W_2 of the trial vector, fwd_loss16)
  uint16_t* f16_limg = nullptr;
  int* f16_ltab = nullptr;
  int* f16_le = nullptr;
  int f16_lnchunks = 0;
  ChainImgArgs f16_ljobs{};
  bool use_fused16() const { return g_options.fused == 3 && f16 && f16_img && fused16_eligible(L, w.data()); }
  // layer 1's R-backward (and the policy gradient's backward into layer 0) fused with layer 0's weight
  // gradient (rbwd0.hip): f16 split with X's planes, obs <= 128, first hidden width <= 256
  uint16_t* rf_img = nullptr;   // rfwd.hip's chunk image (V0^T, W1, V1 in the kernel's LDS order), per FVP
  uint16_t* fw_img = nullptr;   // rfwd.hip's forward image (W0^T, W1), per forward
  // the R-forward through layers 0 and 1 in one launch: X's planes, the fused tail (RZ2 is its pre-activation)
  bool use_rfwd01() const {
    return g_options.rfwd01 != 0 && rf_img && f16 && split_on() && use_tail() && planes_l0() &&
           rfwd01_eligible(L, w.data(), wp.data()) && (int64_t)x_mpad <= ((int64_t)1 << 23);
  }
  // the forward's layers 0 and 1 in one launch (rfwd.hip fwd01_kernel): tanh layers of 256, X on its planes
  bool use_fwd01() const {
    return g_options.fwd01 != 0 && fw_img && f16 && split_on() && planes_l0() && fwd01_eligible(L, w.data(), wp.data()) &&
           (int64_t)x_mpad <= ((int64_t)1 << 23);
  }
  bool use_rbwd0() const {
    return g_options.rbwd0 != 0 && f16 && x_planes && rbwd0_geom() && g_options.planes != 0 && split_on() &&
           rowgemm_uses_split(wp[1], RowEpi::kRBwd);
  }
  RBwd0Args rbwd0_args(const int* skip) const {
    RBwd0Args a{};
    a.rows = (int)n;
    a.K = wp[2];
    a.lda = wp[2];
    a.N = w[1];
    a.Npad = wp[1];
    a.obs = w[0];
    a.B0 = WB3[1];
    a.B1 = WB3[1] + 3 * plane3_b(1);
    a.ldk = r16(wp[2]);
    a.plane = (int64_t)plane3_b(1);
    a.am_b0 = am_w(1);
    a.am_b1 = am_v(1);
    a.H = H[1];
    a.Xh = Xh;
    a.Xl = Xl;
    a.x_mpad = x_mpad;
    a.x_ldp = x_ldp;
    a.eX = pl_e;
    a.splits = active_splits;
    a.rows_per_split = rows_per_split;
    a.slab = slab;
    a.slab_stride = slab_stride;
    a.off_w = offW[0];
    a.off_b = offb[0];
    a.skip = skip;
    return a;
  }
  bool use_chain() const {
    return chain_otm > 0 && (g_options.chain >= 2 || (g_options.chain == 1 && chain_otm <= 8));
  }

  // rollout (rollout.hip): per-environment regions, reallocated when a rollout needs more
  struct RollBufs {
    std::vector<void*> mem;
    int64_t rows = 0;      // capacity in region rows
    int envs = 0;
    double* obs = nullptr;
    int64_t* actions = nullptr;
    float* dist = nullptr;
    double* rewards = nullptr;
    uint8_t* starts = nullptr;
    double* uniforms = nullptr;
    int64_t *counts = nullptr, *episodes = nullptr, *offsets = nullptr;
    double *reset_u = nullptr, *act_u = nullptr;
    int64_t reset_u_n = 0, act_u_n = 0;
  } roll;
  RolloutArgs roll_args{};
  int64_t roll_n = 0, roll_paths = 0, roll_maxcount = 0;
  bool roll_valid = false;

  // profiling
  bool prof = false;
  struct Ev {
    std::string tag;
    hipEvent_t a, b;
  };
  std::vector<Ev> ev_live;
  std::vector<hipEvent_t> ev_pool;
  std::map<std::string, std::pair<long, double>> prof_acc;

  // ------------------------------------------------------------------------
  template <class T>
  T* dalloc(size_t count) {
    void* ptr = nullptr;
    const size_t bytes = std::max<size_t>(count * sizeof(T), 16);
    HIPCHECK(hipMalloc(&ptr, bytes));
    HIPCHECK(hipMemsetAsync(ptr, 0, bytes, stream));
    allocs.push_back(ptr);
    return static_cast<T*>(ptr);
  }

  void use() {
    HIPCHECK(hipSetDevice(device));
    if (!har_slots.empty()) rewind_har();
  }

  const float* act_in(int l) const { return l == 0 ? X : H[l]; }

  hipEvent_t take_event() {
    if (!ev_pool.empty()) {
      hipEvent_t e = ev_pool.back();
      ev_pool.pop_back();
      return e;
    }
    hipEvent_t e;
    HIPCHECK(hipEventCreate(&e));
    return e;
  }
  struct Scope {
    trpo_engine* e;
    int idx = -1;
    Scope(trpo_engine* eng, const char* tag) : e(eng) {
      if (!e->prof) return;
      Ev ev{tag, e->take_event(), e->take_event()};
      HIPCHECK(hipEventRecord(ev.a, e->stream));
      e->ev_live.push_back(ev);
      idx = (int)e->ev_live.size() - 1;
    }
    ~Scope() {
      if (idx >= 0) (void)hipEventRecord(e->ev_live[idx].b, e->stream);
    }
  };
  void prof_collect() {
    if (ev_live.empty()) return;
    HIPCHECK(hipStreamSynchronize(stream));
    for (auto& ev : ev_live) {
      float ms = 0.f;
      HIPCHECK(hipEventElapsedTime(&ms, ev.a, ev.b));
      auto& acc = prof_acc[ev.tag];
      acc.first += 1;
      acc.second += ms;
      ev_pool.push_back(ev.a);
      ev_pool.push_back(ev.b);
    }
    ev_live.clear();
  }

  // ------------------------------------------------------------------------
  void init(int obs, const int* hidden, int nh, int A, int64_t max_rows, int dev) {
    REQUIRE(obs > 0 && A > 0 && nh >= 0 && max_rows > 0, "invalid policy dimensions");
    REQUIRE(nh + 1 <= kMaxLayers, "too many layers");
    REQUIRE(A <= 32 * kMaxHeadTiles, "n_actions must be <= 128 (softmax rows of up to 4 x 32 lanes)");
    REQUIRE(max_rows < (int64_t(1) << 31), "max_rows must fit in int32 row indices");
    for (int i = 0; i < nh; ++i) REQUIRE(hidden[i] > 0, "hidden widths must be positive");
    device = dev;
    use();
    HIPCHECK(hipDeviceGetAttribute(&num_cus, hipDeviceAttributeMultiprocessorCount, device));
    HIPCHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    w.push_back(obs);
    for (int i = 0; i < nh; ++i) w.push_back(hidden[i]);
    w.push_back(A);
    L = (int)w.size() - 1;
    for (int v : w) wp.push_back(pad4(v));
    P = 0;
    for (int l = 0; l < L; ++l) {
      offW.push_back(P);
      P += (int64_t)w[l] * w[l + 1];
      offb.push_back(P);
      P += w[l + 1];
    }
    cap = max_rows;

    for (float** v : {&theta, &theta_prev, &theta_trial, &theta_ls, &g, &bneg, &x, &r, &p, &p2, &z, &hv,
                      &stepdir, &fullstep, &vin, &vout})
      *v = dalloc<float>(P);
    int maxpad = 4;
    for (int l = 0; l < L; ++l) {
      WF.push_back(dalloc<float>((size_t)2 * wp[l] * wp[l + 1]));
      WB.push_back(dalloc<float>((size_t)2 * wp[l + 1] * wp[l]));
      WFt.push_back(dalloc<float>((size_t)2 * wp[l] * wp[l + 1]));
      maxpad = std::max<int>(maxpad, 2 * wp[l] * wp[l + 1]);
    }
    WBt_scratch = dalloc<float>(maxpad);
    for (int l = 0; l < L; ++l) {
      WF3.push_back(dalloc<uint16_t>(2 * plane3_f(l) * 3));
      WB3.push_back(dalloc<uint16_t>(2 * plane3_b(l) * 3));
      WFt3.push_back(dalloc<uint16_t>(plane3_f(l) * 3));
    }
    X = dalloc<float>((size_t)cap * wp[0]);
    act = dalloc<int>(cap);
    adv32 = dalloc<float>(cap);
    old = dalloc<float>((size_t)cap * wp[L]);
    rewards = dalloc<double>(cap);
    returns = dalloc<double>(cap);
    adv64 = dalloc<double>(cap);
    baseline = dalloc<double>(cap);
    starts = dalloc<uint8_t>(cap);
    H.assign(L + 1, nullptr);
    RH.assign(L + 1, nullptr);
    D.assign(L, nullptr);
    RD.assign(L, nullptr);
    E.assign(L, nullptr);
    for (int l = 1; l < L; ++l) {
      H[l] = dalloc<float>((size_t)cap * wp[l]);
      RH[l] = dalloc<float>((size_t)cap * wp[l]);
    }
    for (int l = 0; l < L; ++l) {
      D[l] = dalloc<float>((size_t)cap * wp[l + 1]);
      RD[l] = dalloc<float>((size_t)cap * wp[l + 1]);
      if (l < L - 1) E[l] = dalloc<float>((size_t)cap * wp[l + 1]);
    }
    Pm = dalloc<float>((size_t)cap * wp[L]);
    DSL = dalloc<float>((size_t)cap * wp[L]);
    rowterms = dalloc<double>((size_t)cap * 4);
    // split-K slabs for the weight gradients
    int tiles_max = 1;
    for (int l = 0; l < L; ++l)
      tiles_max = std::max(tiles_max, ((w[l] + 255) / 256) * ((w[l + 1] + 255) / 256));
    slab_stride = (P + 63) / 64 * 64;
    int s_target = std::max(1, std::min(512, 1024 / tiles_max));
    // narrow layers (one output tile each): a 512-split launch is 1-4 waves per CU, too few to stream
    // the activations at HBM rate; small policies take up to 2048 splits while the slabs fit 128 MB
    if (tiles_max == 1)
      s_target = (int)std::max<int64_t>(s_target, std::min<int64_t>(2048, (int64_t(128) << 20) / (slab_stride * 4)));
    // a split accumulates its rows in f32 MFMA accumulators, whose error grows with the rows per split (DESIGN.md
    // §6, numerics at full size): at least one FVP split per 16k rows (wide layers: C5 64 -> 245), and for the
    // policy gradient (once per update; its layer-0/1 blocks are sums of adv_n s_n with mean-zero advantages) 4x
    // that and one per 4k rows, up to 2048; slabs within 2 GB / 8 GB
    const int64_t slab_bytes = (int64_t)slab_stride * 4;
    auto fit = [&](int64_t bytes) { return std::max<int64_t>(1, bytes / slab_bytes); };
    s_target = (int)std::max<int64_t>(s_target, std::min<int64_t>(fit(int64_t(2) << 30), (cap + 16383) / 16384));
    // wide single-tile layers (C4) with few rows (a rank of a 2-8 GPU run): one split per CU when the rows allow it,
    // i.e. one round of the one-workgroup-per-CU split kernels and half the slab reduction (1M rows: 58.3 -> 57.2
    // ms per update, 2M: 111.1 -> 110.4; 128 splits lose half the CUs, profiles/r5u)
    if (tiles_max == 1 && s_target == 512 && num_cus < 512 && (cap + 16383) / 16384 <= num_cus) s_target = num_cus;
    if (g_options.splits > 0) s_target = std::min(g_options.splits, 8192);
    int s_pg = (int)std::max<int64_t>(
        s_target, std::min<int64_t>({2048, std::max<int64_t>(4 * (int64_t)s_target, (cap + 4095) / 4096),
                                     fit(int64_t(8) << 30)}));
    if (g_options.pg_splits > 0) s_pg = std::min(g_options.pg_splits, 8192);
    slab = dalloc<float>((size_t)std::max(s_target, s_pg) * slab_stride);
    S = s_target;
    S_pg = s_pg;
    S_cur = S;
    partA = dalloc<double>(kRedBlocks * 3);
    partB = dalloc<double>(kRedBlocks * 3);
    part3 = dalloc<double>(kRedBlocks * 3);
    local3 = dalloc<double>(4);
    dscal = dalloc<double>(8);
    scan_ws = dalloc<uint8_t>(discount_workspace_bytes(cap));
    sc = dalloc<UpdScalars>(1);
    fl = dalloc<CGFlags>(1);
    cg_ticket = dalloc<unsigned>(1);
    dbad = dalloc<int>(1);
    f16 = g_options.split_f16 != 0;
    amax = dalloc<unsigned>((size_t)(1 + 8 * kMaxLayers) * kAmaxSlot);
    if (L >= 2 && tail_eligible(wp[L - 1], wp[L])) tail_planes = dalloc<uint16_t>((size_t)2 * 2 * 32 * kTailK);
    if (rfwd01_eligible(L, w.data(), wp.data())) rf_img = dalloc<uint16_t>(rfwd01_img_bytes() / 2);
    if (fwd01_eligible(L, w.data(), wp.data())) fw_img = dalloc<uint16_t>(fwd01_img_bytes() / 2);
    // allocated last: the big activation buffers keep the placement the kernels were tuned on
    stage = dalloc<float>((size_t)cap * std::max(std::max(wp[0], wp[L]), 2));
    if (f16 && (planes_geom_l0() || rbwd0_geom())) {
      x_ldp = (wp[0] + 63) / 64 * 64;
      const size_t xp = (size_t)((cap + 255) / 256 * 256) * x_ldp;
      Xh = dalloc<uint16_t>(xp);
      Xl = dalloc<uint16_t>(xp);
      W0b = dalloc<uint16_t>(2 * plane3_f(0));
      V0b = dalloc<uint16_t>(2 * plane3_f(0));
      pl_e = dalloc<int>(8);
    }
    if (f16 && L >= 2 && rbwd0_geom()) {
      d1_ldp = (wp[2] + 31) / 32 * 32;
      D1h = dalloc<uint16_t>((size_t)((cap + 255) / 256 * 256) * d1_ldp);
      eD1t = dalloc<int>((size_t)(cap + 31) / 32 + 8);
    }
    HIPCHECK(hipHostMalloc((void**)&hsc, sizeof(UpdScalars), hipHostMallocDefault));
    std::memset(hsc, 0, sizeof(UpdScalars));
    setup_chain();
    setup_fused16();
    HIPCHECK(hipStreamSynchronize(stream));
  }

  // Weight-image layout of the fused FVP chain, in the order the kernel consumes
  // chunks: R-forward F_0 (V_0), F_l (W_l, V_l) for l = 1..L-1, then R-backward
  // B_l (W_l^T, V_l^T) for l = L-1..1.  Each segment is ceil(K/32) chunks of
  // [3 planes][16*ceil(O/16) rows][32] bf16.
  void setup_chain() {
    if (L < 2 || w[L] > 32) return;
    int hmax = 0;
    for (int l = 1; l < L; ++l) hmax = std::max(hmax, w[l]);
    const int otm = chain_max_tiles(hmax);
    if (!otm) return;
    std::vector<int> tab;
    int64_t off16 = 0;
    int nj = 0;
    auto seg = [&](int l, int trans, int which) {
      const int K = trans ? w[l + 1] : w[l], O = trans ? w[l] : w[l + 1];
      const int kc = (K + 31) / 32, otp = (O + 15) / 16 * 16, csz = otp * 12;   // 16-B units per chunk
      ChainImgJob& j = chain_jobs.job[nj++];
      j.src_off = offW[l];
      j.dst_off = off16 * 8;
      j.K = K;
      j.O = O;
      j.ldw = w[l + 1];
      j.trans = trans;
      j.kc = kc;
      j.otp = otp;
      j.which = which;
      j.pad = 0;
      for (int c = 0; c < kc; ++c) {
        tab.push_back((int)(off16 + (int64_t)c * csz));
        tab.push_back(csz);
      }
      off16 += (int64_t)kc * csz;
    };
    seg(0, 0, 1);
    for (int l = 1; l < L; ++l) {
      seg(l, 0, 0);
      seg(l, 0, 1);
    }
    for (int l = L - 1; l >= 1; --l) {
      seg(l, 1, 0);
      seg(l, 1, 1);
    }
    REQUIRE(nj <= kMaxChainJobs && off16 < (int64_t(1) << 31), "fvp chain: layout too large");
    chain_jobs.n = nj;
    chain_img = dalloc<uint16_t>((size_t)off16 * 8);
    chain_tab = dalloc<int>(tab.size());
    chain_jobs.img = chain_img;
    HIPCHECK(hipMemcpyAsync(chain_tab, tab.data(), tab.size() * sizeof(int), hipMemcpyHostToDevice, stream));
    HIPCHECK(hipStreamSynchronize(stream));   // `tab` is a local vector
    chain_nchunks = (int)(tab.size() / 2);
    chain_otm = otm;
  }

  // fused16.hip's images: the chain's job order with 2 f16 planes per chunk, V_0 padded to
  // fused16_obs_chunks(obs) chunks and every hidden dimension to 64 (2 chunks of K, 64 rows of O: the kernel's
  // hidden layers are 4 tiles of 16 whatever the width, the padding zeros)
  void setup_fused16() {
    if (!fused16_eligible(L, w.data())) return;
    std::vector<int> tab;
    int64_t off16 = 0;
    int nj = 0;
    ChainImgArgs* jobs = &f16_jobs;
    auto seg = [&](int l, int trans, int which) {
      const int K = trans ? w[l + 1] : w[l], O = trans ? w[l] : w[l + 1];
      const bool k_hidden = trans ? l + 1 < L : l > 0, o_hidden = trans ? true : l + 1 < L;
      const int kc = l == 0 && !trans ? fused16_obs_chunks(w[0]) : k_hidden ? 2 : (K + 31) / 32;
      const int otp = o_hidden ? 64 : (O + 15) / 16 * 16, csz = otp * 8;
      ChainImgJob& j = jobs->job[nj++];
      j.src_off = offW[l];
      j.dst_off = off16 * 8;
      j.K = K;
      j.O = O;
      j.ldw = w[l + 1];
      j.trans = trans;
      j.kc = kc;
      j.otp = otp;
      j.which = which;
      j.pad = 0;
      for (int c = 0; c < kc; ++c) {
        tab.push_back((int)(off16 + (int64_t)c * csz));
        tab.push_back(csz);
      }
      off16 += (int64_t)kc * csz;
    };
    seg(0, 0, 1);
    for (int l = 1; l < L; ++l) {
      seg(l, 0, 0);
      seg(l, 0, 1);
    }
    for (int l = L - 1; l >= 1; --l) {
      seg(l, 1, 0);
      seg(l, 1, 1);
    }
    REQUIRE(nj == (L == 3 ? kFused16Jobs : 5), "fused16: job count");
    f16_jobs.n = nj;
    f16_img = dalloc<uint16_t>((size_t)off16 * 8);
    f16_tab = dalloc<int>(tab.size());
    f16_e = dalloc<int>(kFused16Jobs);
    f16_jobs.img = f16_img;
    HIPCHECK(hipMemcpyAsync(f16_tab, tab.data(), tab.size() * sizeof(int), hipMemcpyHostToDevice, stream));
    HIPCHECK(hipStreamSynchronize(stream));   // `tab` is a local vector
    f16_nchunks = (int)(tab.size() / 2);
    // the loss forward's W_0 | W_1 | W_2 (from the trial vector: which = 0, built per line-search trial)
    tab.clear();
    off16 = 0;
    nj = 0;
    jobs = &f16_ljobs;
    for (int l = 0; l < L; ++l) seg(l, 0, 0);
    f16_ljobs.n = nj;
    f16_limg = dalloc<uint16_t>((size_t)off16 * 8);
    f16_ltab = dalloc<int>(tab.size());
    f16_le = dalloc<int>(nj);
    f16_ljobs.img = f16_limg;
    HIPCHECK(hipMemcpyAsync(f16_ltab, tab.data(), tab.size() * sizeof(int), hipMemcpyHostToDevice, stream));
    HIPCHECK(hipStreamSynchronize(stream));
    f16_lnchunks = (int)(tab.size() / 2);
  }

  PolicyShape policy_shape() const {
    PolicyShape ps{};
    ps.L = L;
    for (int l = 0; l <= L; ++l) ps.w[l] = w[l];
    for (int l = 0; l < L; ++l) {
      ps.offW[l] = offW[l];
      ps.offb[l] = offb[l];
    }
    return ps;
  }
  int max_width() const {
    int m = 1;
    for (int l = 0; l <= L; ++l) m = std::max(m, w[l]);
    return m;
  }

  template <class T>
  T* ralloc(size_t count) {
    void* ptr = nullptr;
    HIPCHECK(hipMalloc(&ptr, std::max<size_t>(count * sizeof(T), 16)));
    roll.mem.push_back(ptr);
    return static_cast<T*>(ptr);
  }

  // rollout (utils.py:18-45) of n_envs CartPole-v0 instances under the current policy
  void rollout(const trpo_rollout_params& p) {
    REQUIRE(p.n_envs >= 1 && p.n_envs <= (1 << 20), "n_envs out of range");
    REQUIRE(p.n_timesteps >= 1 && p.max_pathlength >= 1 && p.time_limit >= 1, "bad rollout lengths");
    REQUIRE(w[0] == 4 && w[L] == 2, "CartPole-v0 needs obs_dim 4 and 2 actions");
    const int ep_max = std::min(p.max_pathlength, p.time_limit);
    const int64_t budget = (p.n_timesteps + p.n_envs - 1) / p.n_envs;
    const int64_t env_cap = budget + ep_max - 1;
    const int64_t rows = env_cap * p.n_envs;
    REQUIRE(rows <= (int64_t(1) << 34), "rollout too large");
    if (rows > roll.rows || p.n_envs > roll.envs) {
      for (void* ptr : roll.mem) HIPCHECK(hipFree(ptr));
      roll = RollBufs{};
      roll.rows = rows;
      roll.envs = p.n_envs;
      roll.obs = ralloc<double>((size_t)rows * 4);
      roll.actions = ralloc<int64_t>(rows);
      roll.dist = ralloc<float>((size_t)rows * 2);
      roll.rewards = ralloc<double>(rows);
      roll.starts = ralloc<uint8_t>(rows);
      roll.uniforms = ralloc<double>(rows);
      roll.counts = ralloc<int64_t>(p.n_envs);
      roll.episodes = ralloc<int64_t>(p.n_envs);
      roll.offsets = ralloc<int64_t>(p.n_envs);
    }
    RolloutArgs a{};
    a.ps = policy_shape();
    a.theta = theta;
    a.maxw = max_width();
    a.n_envs = p.n_envs;
    a.max_pathlength = p.max_pathlength;
    a.time_limit = p.time_limit;
    a.train = p.train;
    a.budget = budget;
    a.env_cap = env_cap;
    a.max_episodes = p.max_episodes_per_env;
    a.seed = p.seed;
    // optional injected uniforms (tests): reset [n_envs][max_episodes][4], act [n_envs][env_cap]
    auto stage_u = [&](const double* src, int64_t count, double*& buf, int64_t& cap_n) -> const double* {
      if (!src) return nullptr;
      if (p.mem == TRPO_MEM_DEVICE) return src;
      if (count > cap_n) {
        buf = ralloc<double>(count);
        cap_n = count;
      }
      copy_in(buf, src, (size_t)count * sizeof(double), TRPO_MEM_HOST);
      return buf;
    };
    if (p.reset_uniforms) REQUIRE(p.max_episodes_per_env >= 1, "max_episodes_per_env required with reset_uniforms");
    a.reset_u = stage_u(p.reset_uniforms, (int64_t)p.n_envs * std::max(1, p.max_episodes_per_env) * 4, roll.reset_u,
                        roll.reset_u_n);
    a.act_u = stage_u(p.action_uniforms, rows, roll.act_u, roll.act_u_n);
    if (a.reset_u) {
      // every episode an environment can start must have its uniforms
      REQUIRE((int64_t)p.max_episodes_per_env >= budget, "max_episodes_per_env must be >= ceil(n_timesteps/n_envs)");
    }
    a.obs = roll.obs;
    a.actions = roll.actions;
    a.dist = roll.dist;
    a.rewards = roll.rewards;
    a.starts = roll.starts;
    a.uniforms_out = roll.uniforms;
    a.counts = roll.counts;
    a.episodes = roll.episodes;
    launch_rollout(a, stream);
    check_launch();
    std::vector<int64_t> counts(p.n_envs), offs(p.n_envs);
    copy_out(counts.data(), roll.counts, counts.size() * sizeof(int64_t), TRPO_MEM_HOST);
    int64_t tot = 0, mx = 0;
    for (int i = 0; i < p.n_envs; ++i) {
      offs[i] = tot;
      tot += counts[i];
      mx = std::max(mx, counts[i]);
    }
    copy_in(roll.offsets, offs.data(), offs.size() * sizeof(int64_t), TRPO_MEM_HOST);
    std::vector<int64_t> eps(p.n_envs);
    copy_out(eps.data(), roll.episodes, eps.size() * sizeof(int64_t), TRPO_MEM_HOST);
    roll_args = a;
    roll_n = tot;
    roll_maxcount = mx;
    roll_paths = 0;
    for (int64_t x : eps) roll_paths += x;
    roll_valid = true;
  }

  void rollout_compact(const RolloutOut& o) {
    REQUIRE(roll_valid, "no rollout to fetch");
    launch_rollout_compact(roll_args, roll.offsets, o, roll_maxcount, stream);
    check_launch();
  }

  void release() {
    if (device >= 0) (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    for (auto& ev : ev_live) {
      (void)hipEventDestroy(ev.a);
      (void)hipEventDestroy(ev.b);
    }
    for (auto e : ev_pool) (void)hipEventDestroy(e);
    for (void* ptr : allocs) (void)hipFree(ptr);
    allocs.clear();
    for (void* ptr : roll.mem) (void)hipFree(ptr);
    roll.mem.clear();
    drop_graph();
    free_har_slots();
    if (hsc) (void)hipHostFree(hsc);
    if (comm) (void)ncclCommDestroy(comm);
    if (stream) (void)hipStreamDestroy(stream);
  }

  // the split geometry of the launches that follow: S (FVP weight gradients) or S_pg (policy gradient)
  void use_splits(int s) {
    if (s == S_cur) return;
    S_cur = s;
    set_splits();
  }
  // the policy gradient's split geometry for one scope; the FVP's comes back on every exit, a throwing launch
  // included
  struct PgSplits {
    trpo_engine* e;
    explicit PgSplits(trpo_engine* en) : e(en) { e->use_splits(e->S_pg); }
    ~PgSplits() { e->use_splits(e->S); }
  };
  void set_splits() {
    // rows per split: a multiple of the 16-row k-tile, >= 64 rows
    const int smax = S_cur;
    int64_t rps = (n + smax - 1) / smax;
    rps = std::max<int64_t>(64, (rps + 31) / 32 * 32);   // multiple of the largest wgrad k-tile
    rows_per_split = (int)rps;
    active_splits = (int)std::max<int64_t>(1, (n + rps - 1) / rps);
  }
  int active_splits = 1;

  void copy_in(void* dst, const void* src, size_t bytes, int mem) {
    if (bytes == 0) return;
    HIPCHECK(hipMemcpyAsync(dst, src, bytes, mem == TRPO_MEM_DEVICE ? hipMemcpyDeviceToDevice
                                                                     : hipMemcpyHostToDevice,
                            stream));
    if (mem != TRPO_MEM_DEVICE) HIPCHECK(hipStreamSynchronize(stream));
  }
  void copy_out(void* dst, const void* src, size_t bytes, int mem) {
    if (bytes == 0) return;
    HIPCHECK(hipMemcpyAsync(dst, src, bytes, mem == TRPO_MEM_DEVICE ? hipMemcpyDeviceToDevice
                                                                     : hipMemcpyDeviceToHost,
                            stream));
    HIPCHECK(hipStreamSynchronize(stream));
    har_pending = false;
    check_har();
  }

  // Host test transport, stream-ordered: D2H into a pinned slot, a host node that calls the
  // caller's all-reduce (e.g. gloo) on it, H2D back.  No host synchronisation, so it is captured
  // into the update hipGraph like an RCCL call.  Each call site owns its own slot (a replayed graph
  // keeps the pointers it captured); a callback failure is latched and raised at the next sync.
  struct HostArSlot {
    trpo_engine* e;
    void* host;
    size_t bytes;
    int64_t count;
    int dtype;
  };
  std::vector<HostArSlot*> har_slots;
  size_t har_next = 0;          // slot cursor, rewound by every update / standalone call
  int har_failed = 0;           // written by the host node, read after a stream sync
  static void host_ar_node(void* arg) {
    HostArSlot* s = static_cast<HostArSlot*>(arg);
    if (s->e->host_ar(s->host, s->count, s->dtype, s->e->host_ar_ctx) != 0) s->e->har_failed = 1;
  }
  HostArSlot* har_slot(size_t bytes, int64_t count, int dtype) {
    if (har_next == har_slots.size()) {
      auto* s = new HostArSlot{this, nullptr, 0, 0, 0};
      har_slots.push_back(s);
    }
    HostArSlot* s = har_slots[har_next++];
    if (s->bytes < bytes) {
      if (s->host) HIPCHECK(hipHostFree(s->host));
      s->host = nullptr;
      HIPCHECK(hipHostMalloc(&s->host, bytes, hipHostMallocDefault));
      s->bytes = bytes;
    }
    s->count = count;
    s->dtype = dtype;
    return s;
  }
  void free_har_slots() {
    for (HostArSlot* s : har_slots) {
      if (s->host) (void)hipHostFree(s->host);
      delete s;
    }
    har_slots.clear();
    har_next = 0;
  }
  void check_har() {
    if (har_failed) {
      har_failed = 0;
      throw std::runtime_error("host all-reduce callback failed");
    }
  }
  void host_allreduce(void* buf, size_t bytes, size_t count, int dtype) {
    HostArSlot* s = har_slot(bytes, (int64_t)count, dtype);
    HIPCHECK(hipMemcpyAsync(s->host, buf, bytes, hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipLaunchHostFunc(stream, host_ar_node, s));
    HIPCHECK(hipMemcpyAsync(buf, s->host, bytes, hipMemcpyHostToDevice, stream));
    har_pending = true;
  }
  bool har_pending = false;     // a host node may still read its slot
  size_t har_graph_end = 0;     // slots [0, har_graph_end) belong to the captured update graph
  // every C-ABI entry: slots are reused from the first one the update graph does not own, once no
  // enqueued host node can still read them
  void rewind_har() {
    if (har_pending) {
      HIPCHECK(hipStreamSynchronize(stream));
      har_pending = false;
    }
    check_har();
    har_next = har_graph_end;
  }
  bool multi_rank() const { return comm != nullptr || (host_ar && world > 1); }
  // RCCL when a communicator exists (any world size, world = 1 included: trpo_comm_init always
  // creates one), else the host transport for world > 1, else nothing to reduce
  void allreduce_f32(float* buf, size_t count) {
    if (!multi_rank()) return;
    Scope sp(this, "allreduce");
    if (!comm) return host_allreduce(buf, count * sizeof(float), count, TRPO_F32);
    NCCLCHECK(ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, comm, stream));
  }
  void allreduce_f64(double* buf, size_t count) {
    if (!multi_rank()) return;
    if (!comm) return host_allreduce(buf, count * sizeof(double), count, TRPO_F64);
    NCCLCHECK(ncclAllReduce(buf, buf, count, ncclFloat64, ncclSum, comm, stream));
  }

  // ------------------------------------------------------------------------
  PackArgs pack_args(const std::vector<float*>& wf, const std::vector<float*>* wb, int am_group = -1) {
    PackArgs pa{};
    pa.nl = L;
    if (am_group >= 0) am_reset(am(am_group, 0), L);
    for (int l = 0; l < L; ++l) {
      pa.L[l].amax = am_group >= 0 ? am(am_group, l) : nullptr;
      pa.L[l].off_w = offW[l];
      pa.L[l].a = w[l];
      pa.L[l].b = w[l + 1];
      pa.L[l].apad = wp[l];
      pa.L[l].bpad = wp[l + 1];
      pa.L[l].WF = wf[l];
      pa.L[l].WB = wb ? (*wb)[l] : nullptr;
    }
    return pa;
  }

  // ---- split-bf16 planes ----
  static int r16(int k) { return (k + 15) / 16 * 16; }
  size_t plane3_f(int l) const { return (size_t)wp[l + 1] * r16(wp[l]); }   // WF part: K = wp[l], N = wp[l+1]
  size_t plane3_b(int l) const { return (size_t)wp[l] * r16(wp[l + 1]); }   // WB part: K = wp[l+1], N = wp[l]
  SplitJob job_f(const std::vector<float*>& wf, const std::vector<uint16_t*>& wf3, int l, int part) const {
    return SplitJob{wf[l] + (size_t)part * wp[l] * wp[l + 1], wf3[l] + part * 3 * plane3_f(l), wp[l], wp[l + 1],
                    wp[l + 1], r16(wp[l]), part ? am_v(l) : (&wf == &WFt ? am_wt(l) : am_w(l))};
  }
  SplitJob job_b(int l, int part) const {
    return SplitJob{WB[l] + (size_t)part * wp[l + 1] * wp[l], WB3[l] + part * 3 * plane3_b(l), wp[l + 1], wp[l],
                    wp[l], r16(wp[l + 1]), part ? am_v(l) : am_w(l)};
  }
  // attach the planes of a packed matrix part to a row-GEMM segment
  static void seg3(GemmSeg& sg, uint16_t* base, size_t plane, int part, int K) {
    sg.B3 = base + part * 3 * plane;
    sg.ldk = r16(K);
    sg.plane = (int)plane;
  }
  bool split_on() const { return g_options.split_mfma != 0; }
  // split the given packed-matrix parts; only layers whose GEMM takes the split path
  void split_parts(bool fwd_w, bool fwd_v, bool bwd_w, bool bwd_v, const std::vector<float*>& wf,
                   const std::vector<uint16_t*>& wf3, const int* skip, const char* tag) {
    if (!split_on()) return;
    SplitArgs sa{};
    sa.f16 = f16;
    for (int l = 0; l < L; ++l) {
      const bool f = rowgemm_uses_split(wp[l + 1], RowEpi::kTanh);   // layer l's forward output
      const bool b = l >= 1 && rowgemm_uses_split(wp[l], RowEpi::kRBwd);   // backward into layer l's input
      if (f && fwd_w) sa.job[sa.n++] = job_f(wf, wf3, l, 0);
      if (f && fwd_v) sa.job[sa.n++] = job_f(wf, wf3, l, 1);
      if (b && bwd_w) sa.job[sa.n++] = job_b(l, 0);
      if (b && bwd_v) sa.job[sa.n++] = job_b(l, 1);
      if (sa.n > kMaxSplitJobs - 4 || (l == L - 1 && sa.n)) {
        Scope sp(this, tag);
        launch_split_b(sa, skip, stream);
        sa.n = 0;
      }
    }
    check_launch();
  }
  void ensure_w3() {
    if (split_on() && !w3_valid) {
      split_parts(true, false, true, false, WF, WF3, nullptr, "split_w");
      w3_valid = true;
    }
  }

  RowGemmArgs row_args(int l_out_width, int l_out_pad) {
    RowGemmArgs a{};
    a.f16 = f16;
    a.M = (int)n;
    a.N = l_out_width;
    a.Npad = l_out_pad;
    return a;
  }

  // forward through layers 0..L-1 with weights packed in wf (W half); the head
  // epilogue is `head`; hidden activations go to `hout`
  void forward(const std::vector<float*>& wf, const std::vector<uint16_t*>& wf3, const float* th,
               const std::vector<float*>& hout, RowEpi head, const char* tag) {
    int l_first = 0;
    if (use_fwd01()) {   // layers 0 and 1 in one launch; H1 stored by the prepare pass only (the FVP reads it)
      const bool wt = &wf == &WFt;
      char t[32];
      std::snprintf(t, sizeof t, "%s_img", tag);
      {
        Scope sp(this, t);
        launch_fwd01_img(th, offW[0], offW[1], w[0], wt ? am_wt(0) : am_w(0), wt ? am_wt(1) : am_w(1), fw_img, stream);
        check_launch();
      }
      Fwd01Args fa{};
      fa.n = n;
      fa.obs = w[0];
      fa.Xh = Xh;
      fa.Xl = Xl;
      fa.x_mpad = x_mpad;
      fa.eX = pl_e;
      fa.b0 = th + offb[0];
      fa.b1 = th + offb[1];
      fa.H1 = head == RowEpi::kPrepHead ? hout[1] : nullptr;
      fa.H2 = hout[2];
      fa.img = fw_img;
      fa.am_w0 = wt ? am_wt(0) : am_w(0);
      fa.am_w1 = wt ? am_wt(1) : am_w(1);
      std::snprintf(t, sizeof t, "%s_l01", tag);
      Scope sp(this, t);
      launch_fwd01(fa, num_cus, stream);
      check_launch();
      l_first = 2;
    }
    for (int l = l_first; l < L; ++l) {
      RowGemmArgs a = row_args(w[l + 1], wp[l + 1]);
      a.nseg = 1;
      a.seg[0] = GemmSeg{l == 0 ? X : hout[l], wf[l], wp[l], wp[l + 1], wp[l]};
      seg3(a.seg[0], wf3[l], plane3_f(l), 0, wp[l]);
      a.seg[0].amaxA = l == 0 ? am_x() : nullptr;   // hidden activations are tanh outputs, |h| <= 1
      a.seg[0].amaxB = &wf == &WFt ? am_wt(l) : am_w(l);
      if (l == 0 && planes_l0()) attach_x_planes(a.seg[0], wf3[0], W0b);
      // head_fwd 1 (default): the prepare and the loss heads (the prepare outputs leave through LDS as coalesced
      // rows: C4 3.6 -> 3.1 ms); 2: the loss heads, and the prepare head for <= 8 actions
      const int hfo = g_options.head_fwd;
      const bool prep_hf = hfo == 1 || (hfo == 2 && w[L] <= 8);
      if (l == L - 1 && (hfo == 1 || hfo == 2) && head_fwd_eligible(w[L], w[L - 1]) &&
          ((head == RowEpi::kPrepHead && prep_hf) || head == RowEpi::kLossHead)) {
        // the softmax head with one state per lane (hbwd.hip): bound by its read of H_{L-1}
        HeadFwdArgs hf{};
        hf.rows = n;
        hf.A = w[L];
        hf.Apad = wp[L];
        hf.K = w[l];
        hf.Kpad = wp[l];
        hf.H = l == 0 ? X : hout[l];
        hf.W = wf[l];
        hf.bias = th + offb[l];
        hf.old = old;
        hf.act = act;
        hf.adv = adv32;
        hf.rowterms = rowterms;
        hf.invN = 1.0 / (double)n_global;
        if (head == RowEpi::kPrepHead) {
          hf.prep = 1;
          hf.P = Pm;
          hf.D = D[L - 1];
          hf.DS = DSL;
          hf.am_d = am_d(L - 1);
          hf.am_ds = am_ds(L - 1);
        }
        char t[32];
        std::snprintf(t, sizeof t, "%s_l%d", tag, l);
        Scope sp(this, t);
        launch_head_fwd(hf, num_cus, stream);
        check_launch();
        continue;
      }
      a.ea.bias = th + offb[l];
      a.ea.ldo = wp[l + 1];
      if (l < L - 1) {
        a.epi = RowEpi::kTanh;
        a.ea.out0 = hout[l + 1];
      } else {
        a.epi = head;
        a.ea.out0 = Pm;
        a.ea.out1 = D[L - 1];
        a.ea.out2 = DSL;
        a.ea.old = old;
        a.ea.act = act;
        a.ea.adv = adv32;
        a.ea.rowterms = rowterms;
        a.ea.invN = 1.0 / (double)n_global;
        if (head == RowEpi::kPrepHead) {
          a.ea.amax1 = am_d(L - 1);
          a.ea.amax2 = am_ds(L - 1);
        }
      }
      char t[32];
      std::snprintf(t, sizeof t, "%s_l%d", tag, l);
      Scope sp(this, t);
      launch_rowgemm(a, stream);
      check_launch();
    }
  }

  // rowterms -> [surr, kl, ent] into sc->loss_before (which=0) or loss_trial (which=1)
  void reduce_losses(int which, const int* skip) {
    launch_rowterms_partials(rowterms, n, part3, skip, stream);
    launch_rowterms_finish(part3, local3, skip, stream);
    allreduce_f64(local3, 3);
    launch_losses_store(local3, 1.0 / (double)n_global, sc, which, skip, stream);
    check_launch();
  }

  void require_batch() { REQUIRE(n > 0, "no batch: call trpo_set_batch first"); }

  void update_x_amax() {
    if (!f16) return;
    am_reset(am_x(), 1);
    launch_amax(X, n, w[0], wp[0], am_x(), stream);
    x_planes = false;
    if (Xh && g_options.planes != 0 && n > 0) {
      x_mpad = (int)((n + 255) / 256 * 256);
      Scope sp(this, "split_x");
      launch_split_planes(X, (int)n, x_mpad, w[0], wp[0], Xh, Xl, x_ldp, am_x(), pl_e, stream);
      x_planes = true;
    }
    check_launch();
  }

  // policy forward + KL_ff plain backward at theta (cached over CG)
  void prepare() {
    require_batch();
    if (prepared) return;
    PackArgs pa = pack_args(WF, &WB, 0);
    launch_pack(pa, theta, 0, nullptr, stream);
    w3_valid = false;
    chain_w_valid = false;
    f16_w_valid = false;
    ensure_w3();
    am_reset(am_d(0), L);
    am_reset(am_ds(L - 1), 1);
    if (use_fused16() && g_options.ls_fused == 1) fused16_forward(theta, true);   // fwd_loss16's prepare form
    else forward(WF, WF3, theta, H, RowEpi::kPrepHead, "fwd");
    // KL_ff plain backward: DH_l = D_l W_l^T ; D_{l-1} = DH (1-H^2) ; E_{l-1} = -2 DH H.
    // Only what the FVP path will read is written (prep_e_top records it; fvp() re-prepares if the
    // path changes): D_0 never (the R-backward stops at RD_0), E_{L-2} not under the fused tail, which
    // recomputes it from H and D_{L-1}.
    prep_e_top = e_top_needed();
    prep_fused16 = use_fused16();
    ds_ready = false;
    pg_ready = false;
    d1_plane = false;
    d1_tiled = false;
    const bool hb2 = use_hbwd2();
    if (use_fused16()) {
      // D_1, E_1, E_0 and the policy gradient's slabs in one launch on the f16 weight images (fused16.hip)
      fused16_w_images();
      Fused16Args fa = fused16_args(nullptr, nullptr, pg_grid);
      fa.D1out = L == 3 ? D[1] : nullptr;   // one hidden layer: E_0 only (D_1 is the head's delta)
      fa.E1out = L == 3 ? E[1] : nullptr;
      fa.E0out = E[0];
      fa.am_d1_out = L == 3 ? am_d(1) : nullptr;
      {
        Scope sp(this, "bwd_pg");
        launch_prep_pg_fused16(fa, pg_grid, stream);
        check_launch();
      }
      pg_ready = true;
      reduce_losses(0, nullptr);
      prepared = true;
      return;
    }
    for (int l = L - 1; l >= 1; --l) {
      const bool need_d = l > 1, need_e = l < L - 1 || prep_e_top;
      if (!need_d && !need_e) continue;
      if (l == L - 1 && hb2) {
        // D_{L-2} and the policy gradient's DS_{L-2} in one read of H_{L-1} (hbwd.hip), with D_1's hi plane for
        // the fused R-backward where it runs (two hidden layers), scaled per 32-row tile
        am_reset(am_ds(L - 2), 1);
        HeadBwd2Args hb{};
        hb.rows = (int)n;
        hb.A = w[L];
        hb.Apad = wp[L];
        hb.N = w[L - 1];
        hb.Npad = wp[L - 1];
        hb.WB = WB[L - 1];
        hb.D2 = D[L - 1];
        hb.DS2 = DSL;
        hb.H = H[L - 1];
        hb.D1 = D[L - 2];
        hb.DS1 = RD[L - 2];
        hb.E1 = prep_e_top ? E[L - 2] : nullptr;
        hb.am_d1 = am_d(L - 2);
        hb.am_ds1 = am_ds(L - 2);
        PgSplits pgs(this);   // the slab block it writes is reduced with the policy gradient's
        hb.splits = active_splits;
        hb.rows_per_split = rows_per_split;
        hb.slab = slab;   // the policy gradient's W_{L-1} / b_{L-1} block, reduced by policy_grad()
        hb.slab_stride = slab_stride;
        hb.off_w = offW[L - 1];
        hb.off_b = offb[L - 1];
        if (L == 3 && D1h && eD1t && use_rbwd0() && wp[2] % 32 == 0 && n > 0) {
          d1_mpad = (int)((n + 255) / 256 * 256);
          hb.D1h = D1h;
          hb.d1_mpad = d1_mpad;
          hb.eD1t = eD1t;
        }
        Scope sp(this, "bwd2_l2");
        launch_head_bwd2(hb, num_cus, stream);
        check_launch();
        ds_ready = true;
        if (hb.D1h) {
          d1_plane = true;
          d1_tiled = true;
        }
        continue;
      }
      RowGemmArgs a = row_args(w[l], wp[l]);
      a.nseg = 1;
      a.seg[0] = GemmSeg{D[l], WB[l], wp[l + 1], wp[l], wp[l + 1]};
      seg3(a.seg[0], WB3[l], plane3_b(l), 0, wp[l + 1]);
      a.seg[0].amaxA = am_d(l);
      a.seg[0].amaxB = am_w(l);
      // both: kPrepBwd ; E only (D_0): kPrepBwdE ; D only: kPgBwd, whose epilogue is DH (1-H^2)
      a.epi = need_d ? (need_e ? RowEpi::kPrepBwd : RowEpi::kPgBwd) : RowEpi::kPrepBwdE;
      a.ea.H = H[l];
      a.ea.out0 = need_d ? D[l - 1] : E[l - 1];
      a.ea.amax0 = need_d ? am_d(l - 1) : nullptr;
      a.ea.out1 = need_d && need_e ? E[l - 1] : nullptr;
      a.ea.ldo = wp[l];
      char t[32];
      std::snprintf(t, sizeof t, "bwd_l%d", l);
      Scope sp(this, t);
      launch_rowgemm(a, stream);
      check_launch();
    }
    // D_1's hi plane for the fused R-backward (per update; the FVPs' D_1 V_1^T segment reads half the bytes)
    if (!d1_plane && D1h && use_rbwd0() && n > 0) {
      d1_mpad = (int)((n + 255) / 256 * 256);
      Scope sp(this, "split_d1");
      launch_split_planes(D[1], (int)n, d1_mpad, wp[2], wp[2], D1h, nullptr, d1_ldp, am_d(1), pl_e + 1, stream);
      check_launch();
      d1_plane = true;
    }
    reduce_losses(0, nullptr);
    prepared = true;
  }

  // sum over splits -> out (local partial) ; all-reduce
  void reduce_grad(float* out, const int* skip, int slabs = 0) {
    {
      Scope sp(this, "reduce");
      launch_reduce_slab(slab, slabs > 0 ? slabs : active_splits, slab_stride, P, out, skip, stream);
      check_launch();
    }
    allreduce_f32(out, (size_t)P);
  }

  // every slab writer other than the policy gradient's own layers clears ds_ready: the head-layer block and
  // DS_{L-2} that prepare() leaves for policy_grad() (hbwd.hip) are then recomputed instead of trusted
  void wgrad_layer(int l, int nseg, WSeg s0, WSeg s1, int colsum_seg, const int* skip, const char* tag,
                   bool keeps_pg_head = false) {
    if (!keeps_pg_head) ds_ready = false;
    pg_ready = false;
    WGradArgs a{};
    a.rows = (int)n;
    a.Ma = w[l];
    a.Nb = w[l + 1];
    a.Mpad = wp[l];
    a.Npad = wp[l + 1];
    a.nseg = nseg;
    a.seg[0] = s0;
    a.seg[1] = s1;
    a.colsum_seg = colsum_seg;
    a.splits = active_splits;
    a.rows_per_split = rows_per_split;
    a.slab = slab;
    a.slab_stride = slab_stride;
    a.off_w = offW[l];
    a.off_b = offb[l];
    a.skip = skip;
    a.f16 = f16;
    Scope sp(this, tag);
    launch_wgrad(a, stream);
    check_launch();
  }

  // flatgrad(surr) (trpo_inksci.py:54) -> g (all ranks)
  void policy_grad() {
    reprepare_if_path_changed();
    prepare();
    if (use_fused16()) {
      if (!pg_ready) pg_fused16();
      ds_ready = false;
      reduce_grad(g, nullptr, pg_grid);
      return;
    }
    ensure_w3();
    PgSplits pgs(this);
    // surr backward: DS_{l-1} = (DS_l W_l^T)(1-H_l^2) ; DS of hidden layers lives in RD scratch
    std::vector<float*> DS(L);
    DS[L - 1] = DSL;
    for (int l = 0; l < L - 1; ++l) DS[l] = RD[l];
    const bool have_ds = ds_ready;   // DS_{L-2} (and its running max) from the prepare pass (hbwd.hip)
    am_reset(am_ds(0), have_ds ? L - 2 : L - 1);
    const bool r0f = use_rbwd0();
    for (int l = have_ds ? L - 2 : L - 1; l >= 1; --l) {
      if (l == 1 && r0f) {
        // DS_0 stays in registers: X^T DS_0 and its column sums go straight to the slab (rbwd0.hip)
        RBwd0Args a = rbwd0_args(nullptr);
        a.nseg = 1;
        a.A0 = DS[1];
        a.am_a0 = am_ds(1);
        Scope sp(this, "pg_bwdwg_l1");
        launch_rbwd0(a, stream);
        check_launch();
        continue;
      }
      RowGemmArgs a = row_args(w[l], wp[l]);
      a.nseg = 1;
      a.seg[0] = GemmSeg{DS[l], WB[l], wp[l + 1], wp[l], wp[l + 1]};
      seg3(a.seg[0], WB3[l], plane3_b(l), 0, wp[l + 1]);
      a.seg[0].amaxA = am_ds(l);
      a.seg[0].amaxB = am_w(l);
      a.epi = RowEpi::kPgBwd;
      a.ea.H = H[l];
      a.ea.out0 = DS[l - 1];
      a.ea.amax0 = am_ds(l - 1);
      a.ea.ldo = wp[l];
      char t[32];
      std::snprintf(t, sizeof t, "pg_bwd_l%d", l);
      Scope sp(this, t);
      launch_rowgemm(a, stream);
      check_launch();
    }
    // with DS_{L-2} from the prepare pass the head layer's weight gradient is already in the slabs
    for (int l = r0f ? 1 : 0; l < (have_ds ? L - 1 : L); ++l) {
      char t[32];
      std::snprintf(t, sizeof t, "pg_wgrad_l%d", l);
      wgrad_layer(l, 1, WSeg{act_in(l), DS[l], wp[l], wp[l + 1], l == 0 ? am_x() : nullptr, am_ds(l)}, WSeg{}, 0,
                  nullptr, t, /*keeps_pg_head=*/true);
    }
    reduce_grad(g, nullptr);
  }

  // Hv (undamped, all ranks) for device vector v -> out ; no-op when *skip
  // defer (single rank, the one-launch FVP): the slab reduction is left to the caller (the CG iteration fuses it),
  // *defer receives the slab count; 0 when this FVP reduced into out itself
  void fvp(const float* v, float* out, const int* skip, int* defer = nullptr) {
    if (defer) *defer = 0;
    // the path changed since prepare(): E_{L-2} needed but not written, or the other side of the fused16 switch
    reprepare_if_path_changed();
    prepare();
    ds_ready = false;   // the FVP's R-backward writes RD (DS_{L-2}'s scratch)
    pg_ready = false;   // ... and every FVP path the slabs
    if (use_fused16()) {
      fvp_fused16(v, out, skip, defer && !multi_rank() && cg_fused_reduce_ok(P) ? defer : nullptr);
      return;
    }
    if (use_fused()) {
      fvp_fused(v, out, skip);
      return;
    }
    if (use_chain()) {
      fvp_chain(v, out, skip);
      return;
    }
    {
      PackArgs pa = pack_args(WF, &WB, 1);
      launch_pack(pa, v, 1, skip, stream);
      check_launch();
    }
    ensure_w3();
    split_parts(false, true, false, true, WF, WF3, skip, "split_v");
    am_reset(am_rh(0), L);
    am_reset(am_rd(0), L);
    // R-forward (the fused tail takes the last layer's)
    const bool tail = use_tail();
    const int Lf = tail ? L - 1 : L;
    int l_first = 0;
    if (use_rfwd01()) {   // layers 0 and 1 in one launch (rfwd.hip): RH1 and the tail's RZ2
      {
        Scope sp(this, "fvp_rfwd_img");
        launch_rfwd01_img(theta, v, offW[0], offW[1], w[0], am_v(0), am_w(1), am_v(1), rf_img, skip, stream);
        check_launch();
      }
      Rfwd01Args ra{};
      ra.n = n;
      ra.obs = w[0];
      ra.ldh = wp[1];
      ra.ldz = wp[2];
      ra.Xh = Xh;
      ra.Xl = Xl;
      ra.x_mpad = x_mpad;
      ra.eX = pl_e;
      ra.H1 = H[1];
      ra.c0 = v + offb[0];
      ra.c1 = v + offb[1];
      ra.V0 = v + offW[0];
      ra.RH1 = RH[1];
      ra.RZ2 = RH[2];
      ra.img = rf_img;
      ra.am_v0 = am_v(0);
      ra.am_w1 = am_w(1);
      ra.am_v1 = am_v(1);
      ra.am_rh1 = am_rh(1);
      ra.am_rz2 = am_rh(2);
      ra.skip = skip;
      Scope sp(this, "fvp_rfwd01");
      launch_rfwd01(ra, num_cus, stream);
      check_launch();
      l_first = 2;
    }
    for (int l = l_first; l < Lf; ++l) {
      RowGemmArgs a = row_args(w[l + 1], wp[l + 1]);
      float* Vpart = WF[l] + (size_t)wp[l] * wp[l + 1];
      if (l == 0) {
        a.nseg = 1;
        a.seg[0] = GemmSeg{X, Vpart, wp[0], wp[1], wp[0]};
        seg3(a.seg[0], WF3[l], plane3_f(l), 1, wp[l]);
        a.seg[0].amaxA = am_x();
        a.seg[0].amaxB = am_v(0);
        if (planes_l0()) attach_x_planes(a.seg[0], WF3[0] + 3 * plane3_f(0), V0b);
      } else {
        a.nseg = 2;
        a.seg[0] = GemmSeg{RH[l], WF[l], wp[l], wp[l + 1], wp[l]};
        a.seg[1] = GemmSeg{H[l], Vpart, wp[l], wp[l + 1], wp[l]};
        seg3(a.seg[0], WF3[l], plane3_f(l), 0, wp[l]);
        seg3(a.seg[1], WF3[l], plane3_f(l), 1, wp[l]);
        a.seg[0].amaxA = am_rh(l);
        a.seg[0].amaxB = am_w(l);
        a.seg[1].amaxB = am_v(l);
      }
      a.skip = skip;
      a.ea.bias = v + offb[l];
      a.ea.ldo = wp[l + 1];
      if (l < L - 1) {
        // the fused tail is the only reader of RH_{L-1}: it gets the pre-activation and applies (1-H^2)
        // itself, so H_{L-1} is read once per FVP instead of twice (its max bounds max |RH_{L-1}|)
        a.epi = (tail && l == L - 2) ? RowEpi::kRZ : RowEpi::kRHidden;
        a.ea.H = H[l + 1];
        a.ea.out0 = RH[l + 1];
        a.ea.amax0 = am_rh(l + 1);
      } else {
        a.epi = RowEpi::kRHead;
        a.ea.P = Pm;
        a.ea.out0 = RD[L - 1];
        a.ea.amax0 = am_rd(L - 1);
        a.ea.invN = 1.0 / (double)n_global;
      }
      char tag[32];
      std::snprintf(tag, sizeof tag, "fvp_rfwd_l%d", l);
      Scope sp(this, tag);
      launch_rowgemm(a, stream);
      check_launch();
    }
    if (tail) {
      const int l = L - 1;
      TailPackArgs tp{};
      tp.theta = theta;
      tp.v = v;
      tp.off_w = offW[l];
      tp.a = w[l];
      tp.b = w[l + 1];
      tp.am_w = am_w(l);
      tp.am_v = am_v(l);
      tp.out = tail_planes;
      TailArgs ta{};
      ta.rows = (int)n;
      ta.a = w[l];
      ta.b = w[l + 1];
      ta.apad = wp[l];
      ta.bpad = wp[l + 1];
      ta.RH = RH[l];
      ta.rz = 1;
      ta.H = H[l];
      ta.P = Pm;
      ta.DL = D[l];
      ta.c = v + offb[l];
      ta.WV16 = tail_planes;
      ta.WT16 = WB3[l];
      ta.VT16 = WB3[l] + 3 * plane3_b(l);
      ta.bplane = (int64_t)plane3_b(l);
      ta.am_rh = am_rh(l);
      ta.am_d = am_d(l);
      ta.am_w = am_w(l);
      ta.am_v = am_v(l);
      ta.am_out = am_rd(l - 1);
      ta.RDout = RD[l - 1];
      ta.invN = 1.0 / (double)n_global;
      ta.splits = active_splits;
      ta.rows_per_split = rows_per_split;
      ta.slab = slab;
      ta.slab_stride = slab_stride;
      ta.off_w = offW[l];
      ta.off_b = offb[l];
      ta.skip = skip;
      char tag[32];
      std::snprintf(tag, sizeof tag, "fvp_tail_l%d", l);
      Scope sp(this, tag);
      ds_ready = false;   // slab and RD writer
      launch_tail_pack(tp, stream);
      launch_fvp_tail(ta, stream);
      check_launch();
    }
    const bool tail_fused = tail;
    // layer 1's R-backward fused with layer 0's weight gradient when layer 1 is not inside the tail
    const bool r0f = use_rbwd0() && (tail_fused ? L - 2 : L - 1) >= 1;
    auto r_backward = [&]() {
      // R-backward: RDH_l = RD_l W_l^T + D_l V_l^T ; RD_{l-1} = RDH (1-H_l^2) + E_{l-1} RH_l
      for (int l = tail_fused ? L - 2 : L - 1; l >= 1; --l) {
        if (l == 1 && r0f) {
          RBwd0Args a = rbwd0_args(skip);
          a.nseg = 2;
          a.A0 = RD[1];
          a.A1 = D[1];
          if (d1_plane) {
            a.A1h = D1h;
            a.a1_mpad = d1_mpad;
            a.eA1p = pl_e + 1;
            if (d1_tiled) a.eA1t = eD1t;
          }
          a.am_a0 = am_rd(1);
          a.am_a1 = am_d(1);
          a.E = E[0];
          a.RH = RH[1];
          ds_ready = false;   // slab writer
          Scope sp(this, "fvp_rbwdwg_l1");
          launch_rbwd0(a, stream);
          check_launch();
          continue;
        }
        RowGemmArgs a = row_args(w[l], wp[l]);
        a.nseg = 2;
        a.seg[0] = GemmSeg{RD[l], WB[l], wp[l + 1], wp[l], wp[l + 1]};
        a.seg[1] = GemmSeg{D[l], WB[l] + (size_t)wp[l + 1] * wp[l], wp[l + 1], wp[l], wp[l + 1]};
        seg3(a.seg[0], WB3[l], plane3_b(l), 0, wp[l + 1]);
        seg3(a.seg[1], WB3[l], plane3_b(l), 1, wp[l + 1]);
        a.seg[0].amaxA = am_rd(l);
        a.seg[0].amaxB = am_w(l);
        a.seg[1].amaxA = am_d(l);
        a.seg[1].amaxB = am_v(l);
        a.skip = skip;
        a.epi = RowEpi::kRBwd;
        a.ea.H = H[l];
        a.ea.E = E[l - 1];
        a.ea.RH = RH[l];
        a.ea.out0 = RD[l - 1];
        a.ea.amax0 = am_rd(l - 1);
        a.ea.ldo = wp[l];
        char tag[32];
        std::snprintf(tag, sizeof tag, "fvp_rbwd_l%d", l);
        Scope sp(this, tag);
        launch_rowgemm(a, stream);
        check_launch();
      }
    };
    auto weight_grads = [&]() {
      // weight gradients: (Hv)_W_l = RH_l^T D_l + H_l^T RD_l ; (Hv)_b_l = colsum RD_l
      for (int l = r0f ? 1 : 0; l < (tail_fused ? L - 1 : L); ++l) {
        char tag[32];
        std::snprintf(tag, sizeof tag, "fvp_wgrad_l%d", l);
        if (l == 0)
          wgrad_layer(0, 1, WSeg{X, RD[0], wp[0], wp[1], am_x(), am_rd(0)}, WSeg{}, 0, skip, tag);
        else
          wgrad_layer(l, 2, WSeg{RH[l], D[l], wp[l], wp[l + 1], am_rh(l), am_d(l)},
                      WSeg{H[l], RD[l], wp[l], wp[l + 1], nullptr, am_rd(l)}, 1, skip, tag);
      }
    };
    r_backward();
    weight_grads();
    reduce_grad(out, skip);
  }

  ChainArgs chain_args(const float* v, const int* skip) const {
    ChainArgs ca{};
    ca.n = (int)n;
    ca.L = L;
    for (int l = 0; l <= L; ++l) {
      ca.w[l] = w[l];
      ca.ld[l] = wp[l];
    }
    ca.X = X;
    for (int l = 0; l < L; ++l) {
      ca.H[l] = H[l];
      ca.RH[l] = RH[l];
      ca.D[l] = D[l];
      ca.E[l] = E[l];
      ca.RD[l] = RD[l];
      ca.offb[l] = offb[l];
    }
    ca.P = Pm;
    ca.v = v;
    ca.img = chain_img;
    ca.tab = chain_tab;
    ca.nchunks = chain_nchunks;
    ca.invN = 1.0 / (double)n_global;
    ca.skip = skip;
    return ca;
  }

  // the whole Hv in one launch (fused.hip) + the slab reduction
  void fvp_fused(const float* v, float* out, const int* skip) {
    if (!chain_w_valid) {
      Scope sp(this, "fvp_img_w");
      launch_chain_img(chain_jobs, theta, v, 0, nullptr, stream);
      check_launch();
      chain_w_valid = true;
    }
    {
      Scope sp(this, "fvp_img_v");
      launch_chain_img(chain_jobs, theta, v, 1, skip, stream);
      check_launch();
    }
    const int variant = g_options.fused == 1 ? 1 : 2;   // 3 (f16) where fused16.hip does not apply: 4 waves
    const int rb = fused_fvp_states_per_group(variant);
    FusedArgs fa{};
    fa.c = chain_args(v, skip);
    fa.slab = slab;
    fa.slab_stride = slab_stride;
    for (int l = 0; l < L; ++l) fa.offW[l] = offW[l];
    fa.ngroups = (int)((n + rb - 1) / rb);
    // one persistent workgroup per CU (8 waves) or two (4 waves), at most one per slab
    const int per_cu = variant == 2 ? 2 : 1;
    const int grid =
        (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)fa.ngroups, (int64_t)S, (int64_t)num_cus * per_cu}));
    {
      Scope sp(this, "fvp_fused");
      launch_fvp_fused(fa, grid, variant, stream);
      check_launch();
    }
    {
      Scope sp(this, "reduce");
      launch_reduce_slab(slab, grid, slab_stride, P, out, skip, stream);
      check_launch();
    }
    allreduce_f32(out, (size_t)P);
  }

  // fused16.hip's arguments for the tangent v (the FVP) or none (the policy gradient), and its grid: persistent
  // workgroups, at most one per slab, as few as take the same number of group rounds (fewer slabs to reduce)
  Fused16Args fused16_args(const float* v, const int* skip, int& grid) {
    const int rb = fused16_states_per_group();
    Fused16Args fa{};
    fa.f.c = chain_args(v, skip);
    fa.f.c.img = f16_img;
    fa.f.c.tab = f16_tab;
    fa.f.c.nchunks = f16_nchunks;
    fa.f.slab = slab;
    fa.f.slab_stride = slab_stride;
    for (int l = 0; l < L; ++l) fa.f.offW[l] = offW[l];
    fa.f.ngroups = (int)((n + rb - 1) / rb);
    fa.img_e = f16_e;
    fa.am_x = am_x();
    fa.am_d1 = am_d(1);
    fa.am_d2 = L == 3 ? am_d(2) : nullptr;
    fa.DS = DSL;
    fa.am_ds2 = am_ds(L - 1);
    const int64_t slots = std::max<int64_t>(
        1, std::min<int64_t>({(int64_t)fa.f.ngroups, (int64_t)S, (int64_t)num_cus * fused16_groups_per_cu()}));
    const int64_t rounds = (fa.f.ngroups + slots - 1) / slots;
    grid = (int)std::max<int64_t>(1, (fa.f.ngroups + rounds - 1) / rounds);
    return fa;
  }
  void fused16_w_images() {
    if (f16_w_valid) return;
    Scope sp(this, "fvp_img_w");
    launch_fused16_img(f16_jobs, theta, nullptr, 0, nullptr, f16_e, stream);
    check_launch();
    f16_w_valid = true;
  }

  // the whole Hv in one launch on the f16 split (fused16.hip) + the slab reduction
  void fvp_fused16(const float* v, float* out, const int* skip, int* defer = nullptr) {
    fused16_w_images();
    if (!f16_v_img_ready) {   // else the previous CG step's launch built v's images (cg())
      Scope sp(this, "fvp_img_v");
      launch_fused16_img(f16_jobs, theta, v, 1, skip, f16_e, stream);
      check_launch();
    }
    f16_v_img_ready = false;
    int grid = 1;
    const Fused16Args fa = fused16_args(v, skip, grid);
    {
      Scope sp(this, "fvp_fused");
      launch_fvp_fused16(fa, grid, stream);
      check_launch();
    }
    if (defer) {
      *defer = grid;
      return;
    }
    {
      Scope sp(this, "reduce");
      launch_reduce_slab(slab, grid, slab_stride, P, out, skip, stream);
      check_launch();
    }
    allreduce_f32(out, (size_t)P);
  }

  // g's slabs in one launch on the same machinery (fused16.hip, PG form): the surr backward from DS_2 and every
  // block of g (when the prepare launch's are gone)
  void pg_fused16() {
    fused16_w_images();
    const Fused16Args fa = fused16_args(nullptr, nullptr, pg_grid);
    {
      Scope sp(this, "pg_fused");
      launch_pg_fused16(fa, pg_grid, stream);
      check_launch();
    }
    pg_ready = true;
  }

  // the same Hv with the row-local part (R-forward, R-head, R-backward) in one fused launch
  void fvp_chain(const float* v, float* out, const int* skip) {
    if (!chain_w_valid) {
      Scope sp(this, "fvp_img_w");
      launch_chain_img(chain_jobs, theta, v, 0, nullptr, stream);
      check_launch();
      chain_w_valid = true;
    }
    {
      Scope sp(this, "fvp_img_v");
      launch_chain_img(chain_jobs, theta, v, 1, skip, stream);
      check_launch();
    }
    const ChainArgs ca = chain_args(v, skip);
    {
      Scope sp(this, "fvp_chain");
      launch_fvp_chain(ca, chain_otm, stream);
      check_launch();
    }
    bool split_wg_used = false;   // a weight gradient on the split path reads RH / RD scales
    for (int l = 0; l < L; ++l) split_wg_used |= g_options.split_wg != 0 && w[l + 1] > 128;
    if (f16 && split_wg_used) {
      // the chain writes RH / RD without running maxima; the split weight gradients need them
      am_reset(am_rh(0), L);
      am_reset(am_rd(0), L);
      for (int l = 0; l < L; ++l) {
        if (l >= 1) launch_amax(RH[l], n, w[l], wp[l], am_rh(l), stream);
        launch_amax(RD[l], n, w[l + 1], wp[l + 1], am_rd(l), stream);
      }
      check_launch();
    }
    // weight gradients: (Hv)_W_l = RH_l^T D_l + H_l^T RD_l ; (Hv)_b_l = colsum RD_l
    for (int l = 0; l < L; ++l) {
      char tag[32];
      std::snprintf(tag, sizeof tag, "fvp_wgrad_l%d", l);
      if (l == 0)
        wgrad_layer(0, 1, WSeg{X, RD[0], wp[0], wp[1], am_x(), am_rd(0)}, WSeg{}, 0, skip, tag);
      else
        wgrad_layer(l, 2, WSeg{RH[l], D[l], wp[l], wp[l + 1], am_rh(l), am_d(l)},
                    WSeg{H[l], RD[l], wp[l], wp[l + 1], nullptr, am_rd(l)}, 1, skip, tag);
    }
    reduce_grad(out, skip);
  }

  // conjugate_gradient(fvp, b) (utils.py:185-201): b, x device vectors
  void cg(const float* b, float* xo, int iters, float tol, float damping) {
    REQUIRE(iters >= 0 && iters <= kMaxCG, "cg_iters out of range");
    prepare();
    launch_cg_init(b, xo, r, p, P, partA, sc, fl, tol, damping, stream);
    check_launch();
    f16_v_img_ready = false;
    float* pc = p;    // this iteration's direction; cg_p_img16 writes the next one into the other buffer
    float* pn = p2;
    for (int it = 0; it < iters; ++it) {
      int slabs = 0;
      fvp(pc, hv, &fl->done[it], g_options.cg_fuse_reduce ? &slabs : nullptr);
      Scope sp(this, "cg_vec");
      if (slabs > 0 && g_options.cg_fuse_reduce == 2) {
        // the rest of the iteration in the slab reduction's launch; on the fused16 path it also builds the next
        // iteration's V image, which that FVP then does not launch (fvp_fused16)
        const CgStepArgs ca{slab, slabs, it, slab_stride, P, hv, xo, r, pc, z, sc, partA, fl, cg_ticket};
        const bool img = use_fused16() && it + 1 < iters;
        launch_cg_step_slabs(ca, img ? &f16_jobs : nullptr, f16_e, stream);
        f16_v_img_ready = img;
      } else if (slabs > 0 && g_options.cg_p_img != 0 && use_fused16() && it + 1 < iters) {
        // the p update and the next FVP's V images in one launch (the next p in the other buffer)
        launch_cg_iter_slabs(slab, slabs, slab_stride, hv, xo, r, pc, z, P, sc, partA, partB, fl, it, stream, false);
        launch_cg_p_img16(f16_jobs, r, pc, pn, P, sc, partB, fl, it, f16_e, stream);
        f16_v_img_ready = true;
        std::swap(pc, pn);
      } else if (slabs > 0) {
        launch_cg_iter_slabs(slab, slabs, slab_stride, hv, xo, r, pc, z, P, sc, partA, partB, fl, it, stream);
      } else {
        launch_cg_iter(hv, xo, r, pc, z, P, sc, partA, partB, fl, it, stream);
      }
      check_launch();
    }
    f16_v_img_ready = false;
  }

  void fetch_scalars() {
    HIPCHECK(hipMemcpyAsync(hsc, sc, sizeof(UpdScalars), hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipStreamSynchronize(stream));
    har_pending = false;
    check_har();
  }

  // loss(th) at a device parameter vector, without touching the prepared cache
  // the policy forward in one launch from th's f16 weight images (fused16.hip fwd_loss16_kernel): the line search's
  // row loss terms, or (prep) the prepare pass's H_1, H_2, P, D_2, DS_2, their maxima and the row terms
  void fused16_forward(const float* th, bool prep) {
    {
      Scope sp(this, prep ? "fwd_img" : "ls_img");
      launch_fused16_img(f16_ljobs, th, nullptr, 0, nullptr, f16_le, stream);
      check_launch();
    }
    FwdLoss16Args la{};
    la.n = n;
    la.L = L;
    for (int l = 0; l <= L; ++l) {
      la.w[l] = w[l];
      la.ld[l] = wp[l];
    }
    la.X = X;
    la.theta = th;
    for (int l = 0; l < L; ++l) la.offb[l] = offb[l];
    la.img = f16_limg;
    la.tab = f16_ltab;
    la.nchunks = f16_lnchunks;
    la.img_e = f16_le;
    la.am_x = am_x();
    la.old = old;
    la.act = act;
    la.adv = adv32;
    la.rowterms = rowterms;
    if (prep) {
      la.H1 = H[1];
      la.H2 = L == 3 ? H[2] : nullptr;
      la.P = Pm;
      la.D = D[L - 1];
      la.DS = DSL;
      la.am_d = am_d(L - 1);
      la.am_ds = am_ds(L - 1);
      la.invN = 1.0 / (double)n_global;
    }
    Scope sp(this, prep ? "fwd" : "ls_fwd");
    launch_fwd_loss16(la, num_cus, stream);
    check_launch();
  }

  void eval_losses_dev(const float* th) {
    require_batch();
    if (use_fused16() && g_options.ls_fused != 0) {
      fused16_forward(th, false);
      reduce_losses(1, nullptr);
      return;
    }
    PackArgs pa = pack_args(WFt, nullptr, 2);
    launch_pack(pa, th, 0, nullptr, stream);
    split_parts(true, false, false, false, WFt, WFt3, nullptr, "split_t");
    forward(WFt, WFt3, th, RH, RowEpi::kLossHead, "ls_fwd");
    reduce_losses(1, nullptr);
  }

  void compute_advantages(double gamma) {
    REQUIRE(have_rewards, "no rewards: call trpo_set_rewards first");
    launch_discount(rewards, starts, n, gamma, returns, scan_ws, stream);
    launch_adv_center_partials(returns, have_baseline ? baseline : nullptr, adv64, n, partA, stream);
    launch_sum_finish(partA, dscal, stream);
    allreduce_f64(dscal, 1);
    const double inv_n = 1.0 / (double)n_global;
    launch_adv_sq_partials(adv64, n, dscal, inv_n, partA, stream);
    launch_sum_finish(partA, dscal + 1, stream);
    allreduce_f64(dscal + 1, 1);
    launch_adv_normalize(adv64, adv32, n, dscal, dscal + 1, inv_n, stream);
    check_launch();
    prepared = false;
    have_returns = true;
  }

  // adv = (adv - mean)/(std + 1e-8) over all ranks (trpo_inksci.py:115-117), device arrays on this
  // engine's stream; the same kernels and sums as compute_advantages
  void standardize(double* adv, float* adv32, int64_t cnt, int64_t cnt_global) {
    const double inv_n = 1.0 / (double)cnt_global;
    launch_adv_center_partials(adv, nullptr, adv, cnt, partA, stream);
    launch_sum_finish(partA, dscal + 6, stream);
    allreduce_f64(dscal + 6, 1);
    launch_adv_sq_partials(adv, cnt, dscal + 6, inv_n, partA, stream);
    launch_sum_finish(partA, dscal + 7, stream);
    allreduce_f64(dscal + 7, 1);
    launch_adv_normalize(adv, adv32, cnt, dscal + 6, dscal + 7, inv_n, stream);
    check_launch();
  }

  // 1 - var(y - ypred)/var(y) with y = returns, ypred = baseline (utils.py:208-211), f64 over all ranks
  double explained_variance() {
    REQUIRE(have_returns, "no returns: compute the advantages first");
    if (!ev_tmp) ev_tmp = dalloc<double>(cap);
    const double inv_n = 1.0 / (double)n_global;
    auto var = [&](const double* ypred, int slot) {
      launch_adv_center_partials(returns, ypred, ev_tmp, n, partA, stream);
      launch_sum_finish(partA, dscal + slot, stream);
      allreduce_f64(dscal + slot, 1);
      launch_adv_sq_partials(ev_tmp, n, dscal + slot, inv_n, partA, stream);
      launch_sum_finish(partA, dscal + slot + 1, stream);
      allreduce_f64(dscal + slot + 1, 1);
      check_launch();
    };
    var(nullptr, 2);
    var(have_baseline ? baseline : nullptr, 4);
    double h[6];
    copy_out(h, dscal, sizeof h, TRPO_MEM_HOST);
    const double vary = h[3] * inv_n, vard = h[5] * inv_n;
    return vary == 0.0 ? std::nan("") : 1.0 - vard / vary;
  }

  // The update's sync-free prefix: advantages .. CG .. step scaling .. the first line-search trial
  // (trpo_inksci.py:102-153 up to the first `loss(xnew)` of utils.py:176).  Nothing in it waits on
  // the host, so it is replayed as one captured hipGraph (update()).
  void update_prefix(const trpo_update_params& prm) {
    if (prm.compute_advantages) {
      Scope sp(this, "advantages");
      compute_advantages(prm.gamma);
    }
    prepare();
    // thprev = self.gf()  (:144)
    HIPCHECK(hipMemcpyAsync(theta_prev, theta, P * sizeof(float), hipMemcpyDeviceToDevice, stream));
    // g = session.run(pg)  (:146)
    policy_grad();
    // stepdir = conjugate_gradient(fisher_vector_product, -g)  (:147)
    launch_scale_copy(g, bneg, -1.0f, P, stream);
    cg(bneg, stepdir, prm.cg_iters, prm.residual_tol, prm.cg_damping);
    // shs = .5 * stepdir.dot(fisher_vector_product(stepdir)) ; lm ; fullstep ; rate  (:148-151)
    fvp(stepdir, hv, nullptr);
    {
      Scope sp(this, "step_scale");
      launch_shs_partials(hv, stepdir, g, P, sc, partA, partB, stream);
      launch_shs_finish(partA, partB, sc, stream);
      launch_fullstep(stepdir, fullstep, P, sc, stream);
      check_launch();
    }
    // theta = linesearch(loss, thprev, fullstep, neggdotstepdir / lm)  (:153): trial k = 0
    launch_ls_trial(theta_prev, fullstep, theta_trial, P, 0, sc, stream);
    eval_losses_dev(theta_trial);
    launch_ls_decide(sc, 0, stream);
    check_launch();
  }

  // hipGraph of update_prefix: keyed on everything that shapes its launches (rows, the update
  // parameters that become kernel arguments, the baseline switch, the kernel-variant options).
  // The first update with a key runs eagerly (lazy allocations happen there), the second captures
  // and replays, later ones replay.  Host flags the prefix leaves behind are restored after a replay.
  struct GraphKey {
    int64_t n, n_global;
    const void* comm;   // the communicator / host transport the all-reduces were captured with
    const void* host_ar;
    int rank, world;
    int cg_iters, adv, baseline;
    int x_planes;   // X's planes hold the current batch: the captured plane kernels read them (set_batch
                    // writes them outside the graph, so a replay must not outlive a change of this flag)
    float tol, damping;
    double gamma;
    Options opt;
  };
  GraphKey graph_key(const trpo_update_params& prm) const {
    GraphKey k;
    std::memset(&k, 0, sizeof k);
    k.n = n;
    k.n_global = n_global;
    k.comm = comm;
    k.host_ar = (const void*)host_ar;
    k.rank = rank;
    k.world = world;
    k.cg_iters = prm.cg_iters;
    k.adv = prm.compute_advantages != 0;
    k.baseline = have_baseline;
    k.x_planes = x_planes ? 1 : 0;
    k.tol = prm.residual_tol;
    k.damping = prm.cg_damping;
    k.gamma = prm.compute_advantages ? prm.gamma : 0.0;
    k.opt = g_options;
    return k;
  }
  hipGraphExec_t upd_exec = nullptr;
  GraphKey upd_key{};
  bool upd_key_seen = false, graphs_broken = false;
  struct PrefixFlags {
    bool prepared, w3_valid, chain_w_valid, f16_w_valid, have_returns, prep_e_top, prep_fused16, ds_ready, pg_ready,
        d1_plane, d1_tiled;
    int pg_grid;
  } upd_flags{};
  void drop_graph() {
    if (upd_exec) {
      if (har_graph_end) (void)hipStreamSynchronize(stream);   // its host nodes may still be pending
      (void)hipGraphExecDestroy(upd_exec);
    }
    upd_exec = nullptr;
    upd_key_seen = false;
    har_graph_end = 0;
  }
  void run_prefix(const trpo_update_params& prm) {
    // multi-rank engines capture their all-reduces too (RCCL calls or the host transport's nodes)
    const bool graphable = g_options.graphs != 0 && !prof && !graphs_broken;
    if (!graphable) {
      update_prefix(prm);
      return;
    }
    const GraphKey key = graph_key(prm);
    const bool same = upd_key_seen && std::memcmp(&key, &upd_key, sizeof key) == 0;
    if (same && upd_exec) {
      HIPCHECK(hipGraphLaunch(upd_exec, stream));
      if (har_graph_end) har_pending = true;
      prepared = upd_flags.prepared;
      w3_valid = upd_flags.w3_valid;
      chain_w_valid = upd_flags.chain_w_valid;
      f16_w_valid = upd_flags.f16_w_valid;
      have_returns = upd_flags.have_returns;
      prep_e_top = upd_flags.prep_e_top;
      prep_fused16 = upd_flags.prep_fused16;
      ds_ready = upd_flags.ds_ready;
      pg_ready = upd_flags.pg_ready;
      pg_grid = upd_flags.pg_grid;
      d1_plane = upd_flags.d1_plane;
      d1_tiled = upd_flags.d1_tiled;
      return;
    }
    if (!same) {
      drop_graph();
      har_next = 0;
      update_prefix(prm);
      upd_key = key;
      upd_key_seen = true;
      return;
    }
    // capture (the cache is rebuilt inside the graph, so the prefix must not skip prepare())
    prepared = false;
    hipGraph_t graph = nullptr;
    har_next = 0;
    HIPCHECK(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    try {
      update_prefix(prm);
    } catch (...) {
      (void)hipStreamEndCapture(stream, &graph);
      if (graph) (void)hipGraphDestroy(graph);
      graphs_broken = true;
      throw;
    }
    HIPCHECK(hipStreamEndCapture(stream, &graph));
    const hipError_t ie = hipGraphInstantiate(&upd_exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (ie != hipSuccess) {
      upd_exec = nullptr;
      graphs_broken = true;
      (void)hipGetLastError();
      prepared = false;
      update_prefix(prm);
      return;
    }
    upd_flags = PrefixFlags{prepared,   w3_valid, chain_w_valid, f16_w_valid, have_returns, prep_e_top,
                            prep_fused16, ds_ready, pg_ready,    d1_plane,    d1_tiled,     pg_grid};
    har_graph_end = har_next;   // the graph's host nodes own these slots from now on
    HIPCHECK(hipGraphLaunch(upd_exec, stream));
    if (har_graph_end) har_pending = true;
  }

  void update(const trpo_update_params& prm, trpo_update_stats* st) {
    require_batch();
    REQUIRE(prm.cg_iters >= 0 && prm.cg_iters <= kMaxCG, "cg_iters out of range");
    REQUIRE(!prm.compute_advantages || have_rewards, "no rewards: call trpo_set_rewards first");
    // max_kl goes to the scalar block before shs_finish reads it (no prefix kernel writes it)
    HIPCHECK(hipMemcpyAsync(&sc->max_kl, &prm.max_kl, sizeof(double), hipMemcpyHostToDevice, stream));
    run_prefix(prm);
    fetch_scalars();
    for (int k = 1; k < 10 && !hsc->accepted; ++k) {
      launch_ls_trial(theta_prev, fullstep, theta_trial, P, k, sc, stream);
      eval_losses_dev(theta_trial);
      launch_ls_decide(sc, k, stream);
      check_launch();
      fetch_scalars();
    }
    // sff(theta) ; losses ; revert if kl > 2 max_kl  (:154-158)
    launch_ls_finalize(theta_prev, fullstep, theta, theta_ls, P, sc, stream);
    check_launch();
    prepared = false;
    fetch_scalars();
    if (st) {
      st->cg_iters = hsc->iters;
      st->k = hsc->accepted ? hsc->k : -1;
      st->reverted = hsc->reverted;
      st->shs = hsc->shs;
      st->lm = hsc->lm;
      st->rate = hsc->rate;
      st->surr_before = hsc->loss_before[0];
      st->kl_before = hsc->loss_before[1];
      st->ent_before = hsc->loss_before[2];
      st->surr_after = hsc->loss_after[0];
      st->kl_after = hsc->loss_after[1];
      st->ent_after = hsc->loss_after[2];
      st->rdotr = hsc->rdotr[hsc->iters & 1];
      st->gdotstepdir = hsc->gdots;
    }
  }
};

// =============================================================================
// C-ABI
// =============================================================================
extern "C" {

const char* trpo_last_error(void) { return g_last_error.c_str(); }

int trpo_create(trpo_engine** out, int obs_dim, const int* hidden, int n_hidden, int n_actions,
                int64_t max_rows, int device) {
  return guarded([&] {
    REQUIRE(out, "out is NULL");
    REQUIRE(n_hidden == 0 || hidden, "hidden is NULL");
    auto e = std::make_unique<trpo_engine>();
    try {
      e->init(obs_dim, hidden, n_hidden, n_actions, max_rows, device);
    } catch (...) {
      e->release();
      throw;
    }
    *out = e.release();
  });
}

void trpo_destroy(trpo_engine* e) {
  if (!e) return;
  e->release();
  delete e;
}

int64_t trpo_num_params(const trpo_engine* e) { return e ? e->P : -1; }

int trpo_synchronize(trpo_engine* e) {
  return guarded([&] {
    REQUIRE(e, "engine is NULL");
    e->use();
    HIPCHECK(hipStreamSynchronize(e->stream));
    e->har_pending = false;
    e->check_har();
  });
}

void* trpo_stream(trpo_engine* e) { return e ? (void*)e->stream : nullptr; }

int trpo_comm_unique_id(uint8_t out_id[128]) {
  return guarded([&] {
    REQUIRE(out_id, "out_id is NULL");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    NCCLCHECK(ncclGetUniqueId(&id));
    std::memcpy(out_id, &id, sizeof id);
  });
}

int trpo_comm_init(trpo_engine* e, const uint8_t id[128], int rank, int world) {
  return guarded([&] {
    REQUIRE(e && id, "NULL argument");
    REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad rank/world");
    e->use();
    if (e->comm) {
      NCCLCHECK(ncclCommDestroy(e->comm));
      e->comm = nullptr;
    }
    e->drop_graph();
    e->rank = rank;
    e->world = world;
    e->host_ar = nullptr;
    // world = 1 creates a one-rank communicator as well: every all-reduce then runs through RCCL
    // (an identity), which exercises that path on a single GPU
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    NCCLCHECK(ncclCommInitRank(&e->comm, world, uid, rank));
  });
}

int trpo_comm_set_host_allreduce(trpo_engine* e, trpo_allreduce_cb cb, void* ctx, int rank, int world) {
  return guarded([&] {
    REQUIRE(e && cb, "NULL argument");
    REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad rank/world");
    e->use();
    e->drop_graph();
    if (e->comm) {
      NCCLCHECK(ncclCommDestroy(e->comm));
      e->comm = nullptr;
    }
    e->host_ar = cb;
    e->host_ar_ctx = ctx;
    e->rank = rank;
    e->world = world;
  });
}

int trpo_comm_info(trpo_engine* e, trpo_comm_info_t* out) {
  return guarded([&] {
    REQUIRE(e && out, "NULL argument");
    e->use();
    trpo_comm_info_t ci{};
    ci.transport = e->comm ? 1 : (e->host_ar ? 2 : 0);
    ci.rank = e->rank;
    ci.world = e->world;
    ci.comm_count = ci.comm_rank = ci.comm_device = -1;
    if (e->comm) {
      NCCLCHECK(ncclCommCount(e->comm, &ci.comm_count));
      NCCLCHECK(ncclCommUserRank(e->comm, &ci.comm_rank));
      NCCLCHECK(ncclCommCuDevice(e->comm, &ci.comm_device));
    }
    ci.device = e->device;
    HIPCHECK(hipDeviceGetPCIBusId(ci.pci_bus_id, (int)sizeof ci.pci_bus_id, e->device));
    *out = ci;
  });
}

int trpo_set_flat(trpo_engine* e, const float* theta, int mem) {
  return guarded([&] {
    REQUIRE(e && theta, "NULL argument");
    e->use();
    e->copy_in(e->theta, theta, e->P * sizeof(float), mem);
    e->prepared = false;
  });
}

int trpo_get_flat(trpo_engine* e, float* out, int mem) {
  return guarded([&] {
    REQUIRE(e && out, "NULL argument");
    e->use();
    e->copy_out(out, e->theta, e->P * sizeof(float), mem);
  });
}

int trpo_get_vector(trpo_engine* e, int which, float* out, int mem) {
  return guarded([&] {
    REQUIRE(e && out, "NULL argument");
    e->use();
    const float* src = nullptr;
    switch (which) {
      case TRPO_VEC_THETA: src = e->theta; break;
      case TRPO_VEC_THETA_PREV: src = e->theta_prev; break;
      case TRPO_VEC_G: src = e->g; break;
      case TRPO_VEC_STEPDIR: src = e->stepdir; break;
      case TRPO_VEC_FULLSTEP: src = e->fullstep; break;
      case TRPO_VEC_THETA_LS: src = e->theta_ls; break;
      default: throw ArgError("unknown vector id");
    }
    e->copy_out(out, src, e->P * sizeof(float), mem);
  });
}

int trpo_set_batch(trpo_engine* e, int64_t n, int64_t n_global, const float* states,
                   const int64_t* actions, const float* advant, const float* old_dist, int mem) {
  return guarded([&] {
    REQUIRE(e && states && actions && old_dist, "NULL argument");
    REQUIRE(n > 0 && n <= e->cap, "n out of range (0 < n <= max_rows)");
    REQUIRE(n_global >= n, "n_global must be >= n");
    e->use();
    e->n = n;
    e->n_global = n_global;
    const int obs = e->w[0], A = e->w[e->L];
    // states -> [n][pad4(obs)], old_dist -> [n][pad4(A)] (padding zero)
    auto stage = [&](const float* src, int width, int ldp, float* dst) {
      if (width == ldp) {
        e->copy_in(dst, src, (size_t)n * width * sizeof(float), mem);
        return;
      }
      // (a stream-ordered hipMallocAsync temporary here lost the pageable host copy on its first
      // use in the VF runtime; persistent staging avoids the pattern)
      const float* s = src;
      if (mem != TRPO_MEM_DEVICE) {
        e->copy_in(e->stage, src, (size_t)n * width * sizeof(float), mem);
        s = e->stage;
      }
      launch_copy_rows(s, n, width, width, dst, ldp, e->stream);
      check_launch();
      HIPCHECK(hipStreamSynchronize(e->stream));
    };
    stage(states, obs, e->wp[0], e->X);
    stage(old_dist, A, e->wp[e->L], e->old);
    e->update_x_amax();
    const int64_t* acts = actions;
    if (mem != TRPO_MEM_DEVICE) {
      e->copy_in(e->stage, actions, (size_t)n * sizeof(int64_t), mem);
      acts = reinterpret_cast<const int64_t*>(e->stage);
    }
    HIPCHECK(hipMemsetAsync(e->dbad, 0, sizeof(int), e->stream));
    launch_i64_to_i32(acts, e->act, n, e->dbad, A, e->stream);
    check_launch();
    int bad = 0;
    e->copy_out(&bad, e->dbad, sizeof(int), TRPO_MEM_HOST);
    REQUIRE(!bad, "action index out of range [0, n_actions)");
    if (advant) e->copy_in(e->adv32, advant, (size_t)n * sizeof(float), mem);
    e->set_splits();
    e->prepared = false;
    e->have_rewards = false;
    e->have_returns = false;
  });
}

int trpo_set_rewards(trpo_engine* e, const double* rewards, const uint8_t* starts,
                     const double* baseline, int mem) {
  return guarded([&] {
    REQUIRE(e && rewards && starts, "NULL argument");
    e->require_batch();
    e->use();
    e->copy_in(e->rewards, rewards, (size_t)e->n * sizeof(double), mem);
    e->copy_in(e->starts, starts, (size_t)e->n, mem);
    e->have_baseline = baseline != nullptr;
    if (baseline) e->copy_in(e->baseline, baseline, (size_t)e->n * sizeof(double), mem);
    e->have_rewards = true;
    e->have_returns = false;
  });
}

int trpo_compute_advantages(trpo_engine* e, double gamma, double* returns_out, double* advant_out,
                            int mem) {
  return guarded([&] {
    REQUIRE(e, "engine is NULL");
    e->use();
    e->compute_advantages(gamma);
    if (returns_out) e->copy_out(returns_out, e->returns, (size_t)e->n * sizeof(double), mem);
    if (advant_out) e->copy_out(advant_out, e->adv64, (size_t)e->n * sizeof(double), mem);
  });
}

int trpo_standardize(trpo_engine* e, double* adv, int64_t n, int64_t n_global, float* adv32_out, int mem) {
  return guarded([&] {
    REQUIRE(adv, "adv is NULL");
    REQUIRE(n >= 0 && n_global >= n, "need 0 <= n <= n_global");
    REQUIRE(e || n_global == n, "n_global != n needs an engine (its communicator sums the ranks)");
    if (e) e->use();
    if (n_global == 0) return;
    hipStream_t s = e ? e->stream : nullptr;
    std::vector<void*> tmps;
    auto dev = [&](size_t bytes) {
      void* ptr = nullptr;
      HIPCHECK(hipMalloc(&ptr, std::max<size_t>(bytes, 16)));
      tmps.push_back(ptr);
      return ptr;
    };
    try {
      const bool host = mem != TRPO_MEM_DEVICE;
      double* da = adv;
      float* d32 = adv32_out;
      if (host) {
        da = static_cast<double*>(dev((size_t)n * sizeof(double)));
        copy_in(da, adv, (size_t)n * sizeof(double), TRPO_MEM_HOST, s);
        d32 = adv32_out ? static_cast<float*>(dev((size_t)n * sizeof(float))) : nullptr;
      }
      if (e) {
        e->standardize(da, d32, n, n_global);
      } else {
        double* part = static_cast<double*>(dev(kRedBlocks * sizeof(double)));
        double* sums = static_cast<double*>(dev(2 * sizeof(double)));
        const double inv_n = 1.0 / (double)n;
        launch_adv_center_partials(da, nullptr, da, n, part, s);
        launch_sum_finish(part, sums, s);
        launch_adv_sq_partials(da, n, sums, inv_n, part, s);
        launch_sum_finish(part, sums + 1, s);
        launch_adv_normalize(da, d32, n, sums, sums + 1, inv_n, s);
        check_launch();
      }
      if (host) {
        copy_out(adv, da, (size_t)n * sizeof(double), TRPO_MEM_HOST, s);
        if (adv32_out) copy_out(adv32_out, d32, (size_t)n * sizeof(float), TRPO_MEM_HOST, s);
      }
      HIPCHECK(hipStreamSynchronize(s));
      if (e) {
        // the host all-reduce callbacks of the two sums ran during the sync: a failure there means the
        // mean / std were rank-local, so it is this call's error (as fetch_scalars / copy_out report it)
        e->har_pending = false;
        e->check_har();
      }
    } catch (...) {
      (void)hipStreamSynchronize(s);
      for (void* t : tmps) (void)hipFree(t);
      throw;
    }
    for (void* t : tmps) HIPCHECK(hipFree(t));
  });
}

int trpo_losses(trpo_engine* e, float out3[3]) {
  return guarded([&] {
    REQUIRE(e && out3, "NULL argument");
    e->use();
    e->prepare();
    e->fetch_scalars();
    std::memcpy(out3, e->hsc->loss_before, 3 * sizeof(float));
  });
}

int trpo_eval_losses(trpo_engine* e, const float* theta, float out3[3], int mem) {
  return guarded([&] {
    REQUIRE(e && theta && out3, "NULL argument");
    e->use();
    e->copy_in(e->theta, theta, e->P * sizeof(float), mem);   // sff(th), trpo_inksci.py:128
    e->prepared = false;
    e->eval_losses_dev(e->theta);
    e->fetch_scalars();
    std::memcpy(out3, e->hsc->loss_trial, 3 * sizeof(float));
  });
}

int trpo_action_dist(trpo_engine* e, float* out, int mem) {
  return guarded([&] {
    REQUIRE(e && out, "NULL argument");
    e->use();
    e->prepare();
    const int A = e->w[e->L];
    float* dst = mem == TRPO_MEM_DEVICE ? out : e->stage;
    launch_copy_rows(e->Pm, e->n, A, e->wp[e->L], dst, A, e->stream);
    check_launch();
    if (mem != TRPO_MEM_DEVICE) e->copy_out(out, e->stage, (size_t)e->n * A * sizeof(float), mem);
    HIPCHECK(hipStreamSynchronize(e->stream));
  });
}

int trpo_policy_grad(trpo_engine* e, float* g_out, int mem) {
  return guarded([&] {
    REQUIRE(e && g_out, "NULL argument");
    e->use();
    e->policy_grad();
    e->copy_out(g_out, e->g, e->P * sizeof(float), mem);
  });
}

int trpo_fvp(trpo_engine* e, const float* v, float* out, float damping, int mem) {
  return guarded([&] {
    REQUIRE(e && v && out, "NULL argument");
    e->use();
    e->copy_in(e->vin, v, e->P * sizeof(float), mem);
    e->fvp(e->vin, e->hv, nullptr);
    // out = fvp + damping * v  (float32, trpo_inksci.py:126)
    HIPCHECK(hipMemcpyAsync(e->vout, e->hv, e->P * sizeof(float), hipMemcpyDeviceToDevice, e->stream));
    if (damping != 0.0f) {
      float* tmp = e->z;
      launch_scale_copy(e->vin, tmp, damping, e->P, e->stream);
      launch_axpby(e->vout, tmp, 1.0f, 1.0f, e->P, e->stream);
      check_launch();
    }
    e->copy_out(out, e->vout, e->P * sizeof(float), mem);
  });
}

int trpo_cg(trpo_engine* e, const float* b, float* x_out, int cg_iters, float residual_tol,
            float damping, int* iters_out, int mem) {
  return guarded([&] {
    REQUIRE(e && b && x_out, "NULL argument");
    e->use();
    e->copy_in(e->bneg, b, e->P * sizeof(float), mem);
    e->cg(e->bneg, e->stepdir, cg_iters, residual_tol, damping);
    e->copy_out(x_out, e->stepdir, e->P * sizeof(float), mem);
    e->fetch_scalars();
    if (iters_out) *iters_out = e->hsc->iters;
  });
}

int trpo_cg_callback(trpo_fax_cb f_Ax, void* ctx, const void* b, void* x_out, int64_t n, int dtype,
                     int cg_iters, double residual_tol, int* iters_out) {
  return guarded([&] {
    REQUIRE(f_Ax && b && x_out, "NULL argument");
    REQUIRE(n > 0, "n must be positive");
    REQUIRE(dtype == TRPO_F32 || dtype == TRPO_F64, "dtype must be TRPO_F32 or TRPO_F64");
    REQUIRE(cg_iters >= 0 && cg_iters <= kMaxCG, "cg_iters out of range");
    const size_t es = dtype == TRPO_F64 ? 8 : 4;
    const size_t bytes = (size_t)n * es;
    hipStream_t s = nullptr;
    HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<void*> bufs;
    auto alloc = [&](size_t by) {
      void* p = nullptr;
      HIPCHECK(hipMalloc(&p, std::max<size_t>(by, 16)));
      HIPCHECK(hipMemsetAsync(p, 0, std::max<size_t>(by, 16), s));
      bufs.push_back(p);
      return p;
    };
    try {
      void *db = alloc(bytes), *dx = alloc(bytes), *dr = alloc(bytes), *dp = alloc(bytes),
           *dz = alloc(bytes), *dhv = alloc(bytes);
      double* pa = (double*)alloc(kRedBlocks * sizeof(double));
      double* pb = (double*)alloc(kRedBlocks * sizeof(double));
      CGFlags* fl = (CGFlags*)alloc(sizeof(CGFlags));
      void* sc = alloc(std::max(sizeof(UpdScalars), sizeof(CGScalarsD)));
      std::vector<uint8_t> ph(bytes), zh(bytes);
      HIPCHECK(hipMemcpyAsync(db, b, bytes, hipMemcpyHostToDevice, s));
      if (dtype == TRPO_F64)
        launch_cg_init_d((double*)db, (double*)dx, (double*)dr, (double*)dp, n, pa, (CGScalarsD*)sc, fl,
                         residual_tol, s);
      else
        launch_cg_init((float*)db, (float*)dx, (float*)dr, (float*)dp, n, pa, (UpdScalars*)sc, fl,
                       (float)residual_tol, 0.0f, s);
      HIPCHECK(hipGetLastError());
      int iters = 0;
      for (int it = 0; it < cg_iters; ++it) {
        int done = 0;
        HIPCHECK(hipMemcpyAsync(&done, &fl->done[it], sizeof(int), hipMemcpyDeviceToHost, s));
        HIPCHECK(hipMemcpyAsync(ph.data(), dp, bytes, hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
        if (done) break;
        REQUIRE(f_Ax(ph.data(), zh.data(), ctx) == 0, "f_Ax callback failed");
        HIPCHECK(hipMemcpyAsync(dhv, zh.data(), bytes, hipMemcpyHostToDevice, s));
        if (dtype == TRPO_F64)
          launch_cg_iter_d((double*)dhv, (double*)dx, (double*)dr, (double*)dp, (double*)dz, n,
                           (CGScalarsD*)sc, pa, pb, fl, it, s);
        else
          launch_cg_iter((float*)dhv, (float*)dx, (float*)dr, (float*)dp, (float*)dz, n, (UpdScalars*)sc,
                         pa, pb, fl, it, s);
        HIPCHECK(hipGetLastError());
        iters = it + 1;
      }
      HIPCHECK(hipMemcpyAsync(x_out, dx, bytes, hipMemcpyDeviceToHost, s));
      HIPCHECK(hipStreamSynchronize(s));
      if (iters_out) *iters_out = iters;
    } catch (...) {
      (void)hipStreamSynchronize(s);
      for (void* p : bufs) (void)hipFree(p);
      (void)hipStreamDestroy(s);
      throw;
    }
    for (void* p : bufs) (void)hipFree(p);
    HIPCHECK(hipStreamDestroy(s));
  });
}

int trpo_linesearch(trpo_engine* e, const float* x, const float* fullstep, double rate,
                    float* theta_out, int* k_out, int mem) {
  return guarded([&] {
    REQUIRE(e && x && fullstep && theta_out, "NULL argument");
    e->use();
    const int64_t P = e->P;
    e->copy_in(e->theta_prev, x, P * sizeof(float), mem);
    e->copy_in(e->fullstep, fullstep, P * sizeof(float), mem);
    // fval = f(x)  (utils.py:173)
    e->eval_losses_dev(e->theta_prev);
    e->fetch_scalars();
    UpdScalars init = *e->hsc;
    init.loss_before[0] = init.loss_trial[0];
    init.loss_before[1] = init.loss_trial[1];
    init.loss_before[2] = init.loss_trial[2];
    init.rate = rate;
    init.accepted = 0;
    init.k = -1;
    *e->hsc = init;
    HIPCHECK(hipMemcpyAsync(e->sc, e->hsc, sizeof(UpdScalars), hipMemcpyHostToDevice, e->stream));
    int k_acc = -1;
    for (int k = 0; k < 10; ++k) {
      launch_ls_trial(e->theta_prev, e->fullstep, e->theta_trial, P, k, e->sc, e->stream);
      e->eval_losses_dev(e->theta_trial);
      launch_ls_decide(e->sc, k, e->stream);
      check_launch();
      e->fetch_scalars();
      HIPCHECK(hipMemcpyAsync(e->theta, e->theta_trial, P * sizeof(float), hipMemcpyDeviceToDevice,
                              e->stream));   // loss() leaves sff(xnew) behind
      if (e->hsc->accepted) {
        k_acc = k;
        break;
      }
    }
    e->prepared = false;
    e->copy_out(theta_out, k_acc >= 0 ? e->theta_trial : e->theta_prev, P * sizeof(float), mem);
    if (k_out) *k_out = k_acc;
  });
}

void trpo_default_params(trpo_update_params* p) {
  if (!p) return;
  p->cg_iters = 10;
  p->residual_tol = 1e-10f;
  p->cg_damping = 0.1f;
  p->max_kl = 0.01;
  p->compute_advantages = 0;
  p->gamma = 0.95;
}

int trpo_update(trpo_engine* e, const trpo_update_params* p, trpo_update_stats* stats) {
  return guarded([&] {
    REQUIRE(e, "engine is NULL");
    e->use();
    trpo_update_params prm;
    trpo_default_params(&prm);
    if (p) prm = *p;
    e->update(prm, stats);
  });
}

int trpo_device_count(int* out) {
  return guarded([&] {
    REQUIRE(out, "NULL argument");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    (void)hipGetLastError();
    *out = n;
  });
}

void trpo_default_rollout_params(trpo_rollout_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof *p);
  p->n_envs = 1;
  p->max_pathlength = 1000;    // config["max_steps"] (trpo_inksci.py:17)
  p->n_timesteps = 1000;       // config["episodes_per_roll"] (trpo_inksci.py:17, used as a step budget)
  p->train = 1;
  p->time_limit = 200;         // CartPole-v0 TimeLimit
  p->seed = 1;
  p->mem = TRPO_MEM_HOST;
}

int trpo_rollout_cartpole(trpo_engine* e, const trpo_rollout_params* p, int64_t* n_steps_out, int64_t* n_paths_out) {
  return guarded([&] {
    REQUIRE(e && p, "NULL argument");
    e->use();
    e->rollout(*p);
    if (n_steps_out) *n_steps_out = e->roll_n;
    if (n_paths_out) *n_paths_out = e->roll_paths;
  });
}

int trpo_rollout_fetch(trpo_engine* e, double* obs, float* obs32, int64_t* actions, float* action_dists,
                       double* rewards, uint8_t* episode_starts, double* uniforms, int mem) {
  return guarded([&] {
    REQUIRE(e, "NULL argument");
    REQUIRE(e->roll_valid, "no rollout to fetch");
    e->use();
    const int64_t N = e->roll_n;
    const int obs_dim = e->w[0], A = e->w[e->L];
    RolloutOut o{};
    std::vector<void*> tmps;
    auto dst = [&](auto* user, size_t elems) {
      using T = std::remove_pointer_t<decltype(user)>;
      if (!user || mem == TRPO_MEM_DEVICE) return user;
      void* ptr = nullptr;
      HIPCHECK(hipMalloc(&ptr, std::max<size_t>(elems * sizeof(T), 16)));
      tmps.push_back(ptr);
      return static_cast<T*>(ptr);
    };
    o.obs64 = dst(obs, (size_t)N * obs_dim);
    o.X = dst(obs32, (size_t)N * obs_dim);
    o.ldx = obs_dim;
    o.actions64 = dst(actions, (size_t)N);
    o.dist = dst(action_dists, (size_t)N * A);
    o.rewards = dst(rewards, (size_t)N);
    o.starts = dst(episode_starts, (size_t)N);
    o.uniforms = dst(uniforms, (size_t)N);
    try {
      e->rollout_compact(o);
      if (mem != TRPO_MEM_DEVICE) {
        if (obs) e->copy_out(obs, o.obs64, (size_t)N * obs_dim * sizeof(double), mem);
        if (obs32) e->copy_out(obs32, o.X, (size_t)N * obs_dim * sizeof(float), mem);
        if (actions) e->copy_out(actions, o.actions64, (size_t)N * sizeof(int64_t), mem);
        if (action_dists) e->copy_out(action_dists, o.dist, (size_t)N * A * sizeof(float), mem);
        if (rewards) e->copy_out(rewards, o.rewards, (size_t)N * sizeof(double), mem);
        if (episode_starts) e->copy_out(episode_starts, o.starts, (size_t)N, mem);
        if (uniforms) e->copy_out(uniforms, o.uniforms, (size_t)N * sizeof(double), mem);
      }
      HIPCHECK(hipStreamSynchronize(e->stream));
    } catch (...) {
      for (void* t : tmps) (void)hipFree(t);
      throw;
    }
    for (void* t : tmps) HIPCHECK(hipFree(t));
  });
}

int trpo_rollout_to_batch(trpo_engine* e, int64_t n_global) {
  return guarded([&] {
    REQUIRE(e, "NULL argument");
    REQUIRE(e->roll_valid, "no rollout to load");
    const int64_t N = e->roll_n;
    REQUIRE(N <= e->cap, "rollout has more steps than max_rows");
    REQUIRE(n_global >= N, "n_global must be >= the rollout's steps");
    e->use();
    RolloutOut o{};
    o.X = e->X;
    o.ldx = e->wp[0];
    o.old = e->old;
    o.ld_old = e->wp[e->L];
    o.act32 = e->act;
    o.rewards = e->rewards;
    o.starts = e->starts;
    e->rollout_compact(o);
    e->n = N;
    e->n_global = n_global;
    e->update_x_amax();
    e->set_splits();
    e->prepared = false;
    e->have_rewards = true;
    e->have_returns = false;
    e->have_baseline = false;
    HIPCHECK(hipStreamSynchronize(e->stream));
  });
}

int trpo_get_feed_view(trpo_engine* e, trpo_feed_view* v) {
  return guarded([&] {
    REQUIRE(e && v, "NULL argument");
    e->require_batch();
    e->use();
    HIPCHECK(hipStreamSynchronize(e->stream));   // other streams read these buffers next
    v->n = e->n;
    v->n_global = e->n_global;
    v->obs_dim = e->w[0];
    v->n_actions = e->w[e->L];
    v->states = e->X;
    v->ld_states = e->wp[0];
    v->old_dist = e->old;
    v->ld_old = e->wp[e->L];
    v->episode_starts = e->have_rewards ? e->starts : nullptr;
    v->returns = e->have_returns ? e->returns : nullptr;   // stale until the advantages are computed
    v->baseline = e->baseline;
  });
}

int trpo_set_baseline(trpo_engine* e, const double* baseline, int mem) {
  return guarded([&] {
    REQUIRE(e && baseline, "NULL argument");
    e->require_batch();
    e->use();
    if (baseline != e->baseline) e->copy_in(e->baseline, baseline, (size_t)e->n * sizeof(double), mem);
    e->have_baseline = true;
  });
}

int trpo_explained_variance(trpo_engine* e, double* out) {
  return guarded([&] {
    REQUIRE(e && out, "NULL argument");
    e->use();
    *out = e->explained_variance();
  });
}

int trpo_act(trpo_engine* e, const float* states, int64_t n, const double* uniforms, int train, int64_t* actions_out,
             float* dists_out, int mem) {
  return guarded([&] {
    REQUIRE(e && states && n >= 0, "bad argument");
    REQUIRE(!train || uniforms, "train = 1 needs uniforms (cat_sample's np.random.rand)");
    REQUIRE(e->w[e->L] <= 64, "act: n_actions must be <= 64 (one wave per state)");
    e->use();
    if (n == 0) return;
    const int obs = e->w[0], A = e->w[e->L];
    const float* s = states;
    const double* r = uniforms;
    int64_t* ao = actions_out;
    float* dout = dists_out;
    std::vector<void*> tmps;
    auto dev = [&](size_t bytes) {
      void* ptr = nullptr;
      HIPCHECK(hipMalloc(&ptr, std::max<size_t>(bytes, 16)));
      tmps.push_back(ptr);
      return ptr;
    };
    try {
      if (mem != TRPO_MEM_DEVICE) {
        float* ds = static_cast<float*>(dev((size_t)n * obs * sizeof(float)));
        e->copy_in(ds, states, (size_t)n * obs * sizeof(float), mem);
        s = ds;
        if (uniforms) {
          double* dr = static_cast<double*>(dev((size_t)n * sizeof(double)));
          e->copy_in(dr, uniforms, (size_t)n * sizeof(double), mem);
          r = dr;
        }
        if (actions_out) ao = static_cast<int64_t*>(dev((size_t)n * sizeof(int64_t)));
        if (dists_out) dout = static_cast<float*>(dev((size_t)n * A * sizeof(float)));
      }
      launch_act(e->policy_shape(), e->theta, e->max_width(), s, n, r, train, ao, dout, e->stream);
      check_launch();
      if (mem != TRPO_MEM_DEVICE) {
        if (actions_out) e->copy_out(actions_out, ao, (size_t)n * sizeof(int64_t), mem);
        if (dists_out) e->copy_out(dists_out, dout, (size_t)n * A * sizeof(float), mem);
      }
      HIPCHECK(hipStreamSynchronize(e->stream));
    } catch (...) {
      for (void* t : tmps) (void)hipFree(t);
      throw;
    }
    for (void* t : tmps) HIPCHECK(hipFree(t));
  });
}

namespace {
// engine-free kernels on the current device: stage host arrays in plain hipMalloc buffers
struct Scratch {
  std::vector<void*> p;
  void* get(size_t bytes) {
    void* ptr = nullptr;
    HIPCHECK(hipMalloc(&ptr, std::max<size_t>(bytes, 16)));
    p.push_back(ptr);
    return ptr;
  }
  ~Scratch() {
    for (void* x : p) (void)hipFree(x);
  }
};
}  // namespace

int trpo_cat_sample(const float* prob, int64_t n, int k, const double* r, int64_t* out, int mem) {
  return guarded([&] {
    REQUIRE(prob && r && out && n >= 0 && k >= 1, "bad argument");
    if (n == 0) return;
    Scratch sc;
    const float* dp = prob;
    const double* dr = r;
    int64_t* dout = out;
    if (mem != TRPO_MEM_DEVICE) {
      float* a = static_cast<float*>(sc.get((size_t)n * k * sizeof(float)));
      double* b = static_cast<double*>(sc.get((size_t)n * sizeof(double)));
      HIPCHECK(hipMemcpy(a, prob, (size_t)n * k * sizeof(float), hipMemcpyHostToDevice));
      HIPCHECK(hipMemcpy(b, r, (size_t)n * sizeof(double), hipMemcpyHostToDevice));
      dp = a;
      dr = b;
      dout = static_cast<int64_t*>(sc.get((size_t)n * sizeof(int64_t)));
    }
    launch_cat_sample(dp, n, k, dr, dout, nullptr);
    check_launch();
    if (mem != TRPO_MEM_DEVICE) HIPCHECK(hipMemcpy(out, dout, (size_t)n * sizeof(int64_t), hipMemcpyDeviceToHost));
    HIPCHECK(hipDeviceSynchronize());
  });
}

int trpo_cartpole_step(const double* state, const int64_t* action, int64_t n, double* state_out, double* reward,
                       uint8_t* done, int mem) {
  return guarded([&] {
    REQUIRE(state && action && state_out && n >= 0, "bad argument");
    if (n == 0) return;
    Scratch sc;
    const double* ds = state;
    const int64_t* da = action;
    double *dso = state_out, *dr = reward;
    uint8_t* dd = done;
    if (mem != TRPO_MEM_DEVICE) {
      double* a = static_cast<double*>(sc.get((size_t)n * 4 * sizeof(double)));
      int64_t* b = static_cast<int64_t*>(sc.get((size_t)n * sizeof(int64_t)));
      HIPCHECK(hipMemcpy(a, state, (size_t)n * 4 * sizeof(double), hipMemcpyHostToDevice));
      HIPCHECK(hipMemcpy(b, action, (size_t)n * sizeof(int64_t), hipMemcpyHostToDevice));
      ds = a;
      da = b;
      dso = static_cast<double*>(sc.get((size_t)n * 4 * sizeof(double)));
      dr = reward ? static_cast<double*>(sc.get((size_t)n * sizeof(double))) : nullptr;
      dd = done ? static_cast<uint8_t*>(sc.get((size_t)n)) : nullptr;
    }
    launch_cartpole_step(ds, da, n, dso, dr, dd, nullptr);
    check_launch();
    if (mem != TRPO_MEM_DEVICE) {
      HIPCHECK(hipMemcpy(state_out, dso, (size_t)n * 4 * sizeof(double), hipMemcpyDeviceToHost));
      if (reward) HIPCHECK(hipMemcpy(reward, dr, (size_t)n * sizeof(double), hipMemcpyDeviceToHost));
      if (done) HIPCHECK(hipMemcpy(done, dd, (size_t)n, hipMemcpyDeviceToHost));
    }
    HIPCHECK(hipDeviceSynchronize());
  });
}

int trpo_discount(const double* x, const uint8_t* starts, int64_t n, double gamma, double* out, int mem) {
  return guarded([&] {
    REQUIRE(x && out, "NULL argument");
    REQUIRE(n >= 0, "n < 0");
    if (n == 0) return;
    hipStream_t s = nullptr;
    double *dx = nullptr, *dy = nullptr;
    uint8_t* ds = nullptr;
    void* ws = nullptr;
    const bool dev = mem == TRPO_MEM_DEVICE;
    HIPCHECK(hipMalloc(&ws, discount_workspace_bytes(n)));
    if (!dev) {
      HIPCHECK(hipMalloc(&dx, n * sizeof(double)));
      HIPCHECK(hipMalloc(&dy, n * sizeof(double)));
      HIPCHECK(hipMemcpy(dx, x, n * sizeof(double), hipMemcpyHostToDevice));
    }
    HIPCHECK(hipMalloc(&ds, n));
    if (starts)
      HIPCHECK(hipMemcpy(ds, starts, n, dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice));
    else
      HIPCHECK(hipMemset(ds, 0, n));
    launch_discount(dev ? x : dx, ds, n, gamma, dev ? out : dy, ws, s);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipDeviceSynchronize());
    if (!dev) HIPCHECK(hipMemcpy(out, dy, n * sizeof(double), hipMemcpyDeviceToHost));
    (void)hipFree(ws);
    (void)hipFree(ds);
    if (dx) (void)hipFree(dx);
    if (dy) (void)hipFree(dy);
  });
}

static int* option_slot(const std::string& k) {
  if (k == "split_mfma") return &g_options.split_mfma;
  if (k == "split_wg") return &g_options.split_wg;
  if (k == "chain") return &g_options.chain;
  if (k == "split_f16") return &g_options.split_f16;
  if (k == "split_min_k") return &g_options.split_min_k;
  if (k == "graphs") return &g_options.graphs;
  if (k == "tail") return &g_options.tail;
  if (k == "fused") return &g_options.fused;
  if (k == "low_seg") return &g_options.low_seg;
  if (k == "planes") return &g_options.planes;
  if (k == "rbwd0") return &g_options.rbwd0;
  if (k == "hbwd2") return &g_options.hbwd2;
  if (k == "head_fwd") return &g_options.head_fwd;
  if (k == "splits") return &g_options.splits;
  if (k == "pg_splits") return &g_options.pg_splits;
  if (k == "ls_fused") return &g_options.ls_fused;
  if (k == "cg_fuse_reduce") return &g_options.cg_fuse_reduce;
  if (k == "rfwd01") return &g_options.rfwd01;
  if (k == "fwd01") return &g_options.fwd01;
  if (k == "cg_p_img") return &g_options.cg_p_img;
  throw ArgError("unknown option " + k);
}

int trpo_set_option(const char* name, int value) {
  return guarded([&] {
    REQUIRE(name, "NULL argument");
    *option_slot(name) = value;
  });
}

int trpo_get_option(const char* name, int* value) {
  return guarded([&] {
    REQUIRE(name && value, "NULL argument");
    *value = *option_slot(name);
  });
}

int trpo_profile_enable(trpo_engine* e, int enable) {
  return guarded([&] {
    REQUIRE(e, "engine is NULL");
    e->use();
    e->prof_collect();
    e->prof = enable != 0;
  });
}

int trpo_profile_reset(trpo_engine* e) {
  return guarded([&] {
    REQUIRE(e, "engine is NULL");
    e->use();
    e->prof_collect();
    e->prof_acc.clear();
  });
}

int trpo_profile_query(trpo_engine* e, char* buf, int cap) {
  std::string js;
  int rc = guarded([&] {
    REQUIRE(e, "engine is NULL");
    e->use();
    e->prof_collect();
    js = "{";
    bool first = true;
    for (auto& kv : e->prof_acc) {
      char item[256];
      std::snprintf(item, sizeof item, "%s\"%s\": [%ld, %.6f]", first ? "" : ", ", kv.first.c_str(),
                    kv.second.first, kv.second.second);
      js += item;
      first = false;
    }
    js += "}";
  });
  if (rc != TRPO_OK) return rc;
  if (buf && cap > 0) {
    std::strncpy(buf, js.c_str(), (size_t)cap - 1);
    buf[cap - 1] = '\0';
  }
  return (int)js.size();
}

}  // extern "C"
