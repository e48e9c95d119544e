/*
 * trpo_engine.h — C-ABI of the MI355X-native TRPO policy-update engine.
 *
 * The reference (inksci/TRPO) runs its update through a TF-1.3 session and
 * numpy; every entry point below replaces one reference interface, cited as
 * file:line into the reference tree.  Conventions:
 *
 *   - return 0 on success, a negative code on failure; trpo_last_error()
 *     returns the message of the calling thread's last failure;
 *   - `mem` selects where a caller pointer lives: TRPO_MEM_HOST or
 *     TRPO_MEM_DEVICE (a device pointer on the engine's GPU, e.g. a torch-ROCm
 *     tensor's data_ptr()).  Inputs are copied; caller buffers are never
 *     retained (reference: caller-owned numpy in, fresh numpy out);
 *   - one engine is driven from one host thread; calls are ordered on the
 *     engine's HIP stream and synchronise only when they return host data;
 *   - flat parameter vectors use the reference's layout
 *     [W1, b1, W2, b2, ..., WL, bL], W_l row-major [fan_in][fan_out]
 *     (tf.trainable_variables() order, trpo_inksci.py:49; var_shape/numel,
 *     utils.py:108-116).
 *
 * All arithmetic that the reference does in float32 is float32 here; the
 * scalars its NumPy-1.x promotion keeps in float64 (shs, lm, the
 * expected-improve rate, the line-search ratio) are float64.
 */
#ifndef TRPO_ENGINE_H
#define TRPO_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TRPO_MEM_HOST 0
#define TRPO_MEM_DEVICE 1

#define TRPO_OK 0
#define TRPO_ERR_ARG (-1)
#define TRPO_ERR_HIP (-2)
#define TRPO_ERR_RCCL (-3)
#define TRPO_ERR_STATE (-4)

typedef struct trpo_engine trpo_engine;

/* Hyper-parameters of one update; defaults are config/eps of trpo_inksci.py:16-17
 * and the CG/line-search defaults of utils.py:171-172,185. */
typedef struct trpo_update_params {
  int cg_iters;            /* 10          utils.py:185 */
  float residual_tol;      /* 1e-10       utils.py:185 (absolute, on r.r) */
  float cg_damping;        /* 0.1         trpo_inksci.py:17,126 */
  double max_kl;           /* 0.01        trpo_inksci.py:17,149,157 */
  int compute_advantages;  /* 1: discount + standardise the rewards given to trpo_set_rewards first */
  double gamma;            /* 0.95        trpo_inksci.py:17,104 */
} trpo_update_params;

typedef struct trpo_update_stats {
  int cg_iters;            /* CG iterations run (early exit on r.r < residual_tol) */
  int k;                   /* accepted backtrack index (step fraction 0.5^k), -1 if none */
  int reverted;            /* 1 if kl > 2 max_kl restored theta_prev (trpo_inksci.py:157-158) */
  int pad;
  double shs, lm, rate;    /* trpo_inksci.py:148-153 */
  float surr_before, kl_before, ent_before;   /* losses at theta_prev */
  float surr_after, kl_after, ent_after;      /* losses at the line-search result (:156) */
  float rdotr;             /* final CG residual r.r */
  float gdotstepdir;       /* g . stepdir */
} trpo_update_stats;

/* Vectors of the last update, for trpo_get_vector(). */
#define TRPO_VEC_THETA 0       /* current parameters (GetFlat) */
#define TRPO_VEC_THETA_PREV 1  /* thprev, trpo_inksci.py:144 */
#define TRPO_VEC_G 2           /* policy gradient, :146 */
#define TRPO_VEC_STEPDIR 3     /* CG solution, :147 */
#define TRPO_VEC_FULLSTEP 4    /* :150 */
#define TRPO_VEC_THETA_LS 5    /* linesearch result before the revert check, :153 */

/* ---- lifecycle --------------------------------------------------------- */

/* Build an engine for the categorical tanh-MLP policy of trpo_inksci.py:38-40
 * (hidden widths as a list; the reference is the depth-1 case {64}) with room
 * for `max_rows` states on GPU `device`.  n_actions <= 128 for the update (trpo_act: <= 64; the reference's softmax_classifier has
 * no bound; a softmax row spans up to 4 x 32 lanes here). */
int trpo_create(trpo_engine** out, int obs_dim, const int* hidden, int n_hidden, int n_actions,
                int64_t max_rows, int device);
void trpo_destroy(trpo_engine* e);
const char* trpo_last_error(void);
int64_t trpo_num_params(const trpo_engine* e);
int trpo_synchronize(trpo_engine* e);
/* the engine's HIP stream (hipStream_t) as an opaque pointer */
void* trpo_stream(trpo_engine* e);

/* ---- multi-GPU (one process per GPU, RCCL over xGMI) ---------------------
 * The reference is single-process (trpo_inksci.py:23).  Rank 0 creates an id,
 * the launcher broadcasts it, every rank calls trpo_comm_init.  After that the
 * FVP / gradient / loss sums of each rank's shard are all-reduced. */
int trpo_comm_unique_id(uint8_t out_id[128]);
int trpo_comm_init(trpo_engine* e, const uint8_t id[128], int rank, int world);
/* Test transport: instead of RCCL, every all-reduce is stream-ordered and capturable: an async copy of
 * the buffer into a pinned host slot, a hipLaunchHostFunc callback that calls cb(host_buf, count,
 * dtype = TRPO_F32 / TRPO_F64, ctx), which must sum it across ranks in place (e.g. torch.distributed
 * over gloo), and an async copy back.  Lets several ranks share one GPU in tests. */
typedef int (*trpo_allreduce_cb)(void* host_buf, int64_t count, int dtype, void* ctx);
int trpo_comm_set_host_allreduce(trpo_engine* e, trpo_allreduce_cb cb, void* ctx, int rank, int world);
/* What carries this engine's all-reduces, for a launcher to verify (e.g. that N ranks of an RCCL
 * communicator sit on N distinct devices).  transport: 0 none (one process), 1 RCCL, 2 host callback.
 * comm_count / comm_rank / comm_device: ncclCommCount / ncclCommUserRank / ncclCommCuDevice of the RCCL
 * communicator (-1 without one); device: the engine's HIP device; pci_bus_id: hipDeviceGetPCIBusId. */
typedef struct trpo_comm_info_t {
  int transport;
  int rank, world;
  int comm_count, comm_rank, comm_device;
  int device;
  char pci_bus_id[64];
} trpo_comm_info_t;
int trpo_comm_info(trpo_engine* e, trpo_comm_info_t* out);

/* ---- parameters: SetFromFlat / GetFlat (utils.py:125-158) ---------------- */
int trpo_set_flat(trpo_engine* e, const float* theta, int mem);
int trpo_get_flat(trpo_engine* e, float* theta_out, int mem);
int trpo_get_vector(trpo_engine* e, int which, float* out, int mem);

/* ---- the feed (trpo_inksci.py:119-122) ------------------------------------
 * states [n][obs_dim] f32, actions [n] int64 in [0, n_actions), advant [n] f32
 * (may be NULL when trpo_set_rewards + compute_advantages provide it),
 * old_dist [n][n_actions] f32.  n_global = rows over all ranks (the 1/N of
 * reduce_mean, trpo_inksci.py:48-51,56). */
int trpo_set_batch(trpo_engine* e, int64_t n, int64_t n_global, const float* states,
                   const int64_t* actions, const float* advant, const float* old_dist, int mem);
/* rewards [n] f64, episode_starts [n] u8 (1 = first step of a path), baseline [n] f64 or NULL.
 * The paths of trpo_inksci.py:102-112, concatenated; this rank's shard must begin at a path start. */
int trpo_set_rewards(trpo_engine* e, const double* rewards, const uint8_t* episode_starts,
                     const double* baseline, int mem);
/* returns = discount(rewards, gamma) per path; advant = returns - baseline,
 * standardised (trpo_inksci.py:102-117).  Optional host copies (f64). */
int trpo_compute_advantages(trpo_engine* e, double gamma, double* returns_out, double* advant_out,
                            int mem);

/* adv = (adv - adv.mean()) / (adv.std() + 1e-8) in place, float64, population std
 * (trpo_inksci.py:115-117; SURVEY.md §8(b) `standardize(adv, n)`).  adv32_out (may be NULL) receives
 * float32(adv), what the advant placeholder is fed (:121).  With an engine the two sums run over all
 * ranks of its communicator (n = this rank's rows, n_global = all ranks') on its stream; e = NULL
 * runs on the current device for one process (n_global must equal n). */
int trpo_standardize(trpo_engine* e, double* adv, int64_t n, int64_t n_global, float* adv32_out, int mem);

/* ---- the graph outputs ---------------------------------------------------- */
/* session.run(self.losses) -> [surr, kl, ent] at the current parameters (trpo_inksci.py:53,156) */
int trpo_losses(trpo_engine* e, float out3[3]);
/* loss(th): SetFromFlat(th) then session.run(surr) (trpo_inksci.py:127-129); out3 = [surr, kl, ent] */
int trpo_eval_losses(trpo_engine* e, const float* theta, float out3[3], int mem);
/* session.run(self.action_dist) -> [n][n_actions] f32 at the current parameters
 * (trpo_inksci.py:38-40,78; the policy forward) */
int trpo_action_dist(trpo_engine* e, float* out, int mem);
/* session.run(self.pg) = flatgrad(surr, var_list) (trpo_inksci.py:54,146) */
int trpo_policy_grad(trpo_engine* e, float* g_out, int mem);
/* fisher_vector_product(p) = session.run(self.fvp) + cg_damping * p (trpo_inksci.py:56-70,124-126) */
int trpo_fvp(trpo_engine* e, const float* v, float* out, float damping, int mem);

/* ---- the numpy half --------------------------------------------------------- */
/* conjugate_gradient(fisher_vector_product, b, cg_iters, residual_tol) (utils.py:185-201),
 * device-resident: every FVP, dot and axpy stays on the GPU. */
int trpo_cg(trpo_engine* e, const float* b, float* x_out, int cg_iters, float residual_tol,
            float damping, int* iters_out, int mem);
/* conjugate_gradient(f_Ax, b, cg_iters, residual_tol) for an arbitrary host f_Ax
 * (utils.py:185-201, the reference's generic signature).  The CG vectors, dots and axpys run
 * on the current GPU in `dtype` (TRPO_F32 / TRPO_F64, the dtype of the caller's b); for each
 * iteration p is copied out and f_Ax(p, z, ctx) must write z = A p (n elements of dtype) and
 * return 0.  Engine-free. */
#define TRPO_F32 0
#define TRPO_F64 1
typedef int (*trpo_fax_cb)(const void* p, void* z, void* ctx);
int trpo_cg_callback(trpo_fax_cb f_Ax, void* ctx, const void* b, void* x_out, int64_t n, int dtype,
                     int cg_iters, double residual_tol, int* iters_out);
/* linesearch(loss, x, fullstep, expected_improve_rate) (utils.py:170-182) with f = the policy
 * surrogate (trpo_inksci.py:127-129).  theta_out = accepted xnew or x; k_out = accepted index or -1.
 * Leaves the engine's parameters at the last evaluated point, as loss() does. */
int trpo_linesearch(trpo_engine* e, const float* x, const float* fullstep, double expected_improve_rate,
                    float* theta_out, int* k_out, int mem);

/* ---- the update block (trpo_inksci.py:101-158) ---------------------------------- */
void trpo_default_params(trpo_update_params* p);
int trpo_update(trpo_engine* e, const trpo_update_params* p, trpo_update_stats* stats);

/* ---- engine-free helpers ------------------------------------------------------------ */
/* number of visible GPUs (0 when none); never fails on a host without GPUs */
int trpo_device_count(int* out);
/* discount(x, gamma) (utils.py:14-16) over a concatenation of paths on the current device.
 * episode_starts may be NULL (one path). */
int trpo_discount(const double* x, const uint8_t* episode_starts, int64_t n, double gamma,
                  double* out, int mem);

/* ---- kernel-variant switches (for A/B measurements and variant parity tests) ----------
 * "split_mfma" (0 = f32 MFMA row GEMMs; 5 = the 256 x 256 split row-GEMM tile for outputs wider than
 * 128, at BK 32 on f16 planes, the default; 6 = the same tile at BK 16; any other value = 128 x 256),
 * "split_wg" (0 = f32 weight gradients; 1 = split tile for fan_out > 128), "chain" (fused FVP chain: 0 off, 1 auto, 2..4 forced variants),
 * "split_f16" (split GEMMs on scaled f16 hi+lo planes), "split_min_k" (few-k row GEMMs stay on f32
 * MFMA), "graphs" (1 = trpo_update replays its sync-free prefix as a captured hipGraph, all-reduces
 * included; results are bit-identical to eager launches), "tail" (1 = the fused last-layer FVP tail
 * of tail.hip where eligible: f16 split, last hidden width in (128, 256], 17..32 actions), "fused"
 * (whole FVP incl. weight gradients in one launch of fused.hip for one or two hidden layers of
 * width <= 64, obs <= 128, <= 32 actions: 0 off, 1 = 8-wave workgroups, 2 = 4-wave workgroups, 3 = the
 * default: two hidden layers of width 49..64 on the scaled f16 hi+lo split (fused16.hip, needs "split_f16"),
 * other eligible shapes as 2),
 * "low_seg" (f16 split GEMMs with two K-segments: a segment whose running-max product scale lies at
 * least this many binades below the other's -- the O(eps) KL_ff plain-delta terms -- runs on one
 * f16 product instead of three; 4 more binades when the dominant segment has an operand without a
 * running max; 0 = off; default 14), "planes" (1 = row GEMMs whose operands the engine keeps as
 * pre-split k-blocked f16 hi/lo planes run the LDS-DMA plane kernel of plane.hip; bit-identical to
 * the register-staged split; default 1),
 * "rbwd0" (1 = layer 1's R-backward and layer 0's weight gradient run as one launch of rbwd0.hip:
 * RD_0 stays in registers and X^T RD_0 is reduced from the engine's X planes; eligible on the f16
 * split with planes on, obs <= 128, hidden widths <= 256 and multiples of 32; also serves the policy
 * gradient's layer-1 backward; default 1),
 * "hbwd2" (1 = the prepare pass's and the policy gradient's backward through the softmax head's layer
 * run as one launch of hbwd.hip over one read of H_{L-1}, which also writes D_{L-2}'s f16 hi plane for
 * rbwd0 (or E_{L-2} where the FVP path reads it) and the policy gradient's head-layer weight gradient;
 * <= 32 actions, last hidden width 129..256; 2 = on f32 MFMA, the default; 1 = on VALU f32 FMA chains),
 * "head_fwd" (softmax head forwards with one state per lane on f32 FMAs,
 * hbwd.hip: 1 = the prepare and the line-search heads, the default; 2 = the line-search heads, and the
 * prepare head when the head has <= 8 actions; 0 = off), "splits" (split-K slabs of the FVP's weight
 * gradients; 0 = auto: by tile count, at least one per 16k rows; 512 at C4, 245 at C5) and "pg_splits" (the
 * policy gradient's; 0 = auto: 4 x splits or one per 4k rows, up to 2048): both are read when an engine
 * is created; "ls_fused" (where the FVP runs on fused16.hip, the policy forward as one launch from f16 weight
 * images, fwd_loss16: 1 = the prepare pass's and the line search's, the default; 2 = the line search's only;
 * 0 = the per-layer forwards); "cg_fuse_reduce" (single rank with the one-launch FVP: each CG iteration's slab
 * reduction fused with its z = Hv + damping p step; 1 = on, the default; 2 = on, and the rest of the iteration
 * (x, r, p, the next FVP's f16 V image) runs in the same launch, in the workgroup that finishes last,
 * bit-identical to 1 but slower (one CU's serial tail); 0 = off: 0 and 1 group the p.z partials differently, so
 * each is deterministic but their CG scalars are not bit-identical to each other).
 * "cg_p_img" (the fused16 path: each CG iteration's p update and the next FVP's f16 V images in one launch,
 * bit-identical: 1 = on, the default; 0 = two launches).
 * "rfwd01" (the FVP's R-forward through layers 0 and 1 as one launch, rfwd.hip, where two hidden layers of 256
 * with obs <= 128 run the fused tail: 1 = on, the default; 0 = the plane and row GEMM launches).
 * "fwd01" (the prepare and line-search forwards through layers 0 and 1 as one launch, rfwd.hip, at the same
 * shapes: 1 = on, the default; 0 = the plane and row GEMM launches).
 * "ls_fused" = 2 mixes two forwards inside one line search (loss_before from the per-layer forward, the
 * trials' losses from fwd_loss16); it exists for A/B timing and is held to the same parity tests.
 * Rejected variants (other tiles, last-layer fusions, 16-bit E planes, a second stream) were removed
 * from the build in round 4; tools/patches/pruned_variants.patch restores them.
 * Process-wide. */
int trpo_set_option(const char* name, int value);
int trpo_get_option(const char* name, int* value);

/* ---- profiling: per-launch HIP events on the engine stream ------------------------- */
int trpo_profile_enable(trpo_engine* e, int enable);
/* JSON {"tag": [count, total_ms], ...}; returns bytes needed (excluding NUL) or < 0 */
int trpo_profile_query(trpo_engine* e, char* buf, int cap);
int trpo_profile_reset(trpo_engine* e);

/* ==== sampling and rollouts (trpo_inksci.py:76-87, utils.py:18-45,95-105) ======================
 * The reference steps one gym CartPole-v0 env and calls agent.act once per step (a 1-row
 * session.run + cat_sample).  Here n_envs CartPole-v0 instances (gym's classic_control/cartpole.py
 * restated in float64; gym is not vendored) run on the GPU, one wave each, under the engine's
 * current policy.  Every environment collects whole episodes until its own step count reaches
 * ceil(n_timesteps / n_envs) -- utils.py:23-44's stopping rule per environment (n_envs = 1 is the
 * reference's loop) -- and the episodes are concatenated in environment order. */
typedef struct trpo_rollout_params {
  int n_envs;                /* parallel environments (1) */
  int max_pathlength;        /* config["max_steps"] = 1000 (trpo_inksci.py:17; utils.py:28) */
  int64_t n_timesteps;       /* config["episodes_per_roll"] = 1000 (trpo_inksci.py:17; utils.py:23) */
  int train;                 /* 1: cat_sample; 0: argmax (trpo_inksci.py:79-83) */
  int time_limit;            /* CartPole-v0's TimeLimit: 200 steps */
  uint64_t seed;             /* Philox stream: action uniforms and env.reset draws */
  /* optional injected uniforms (tests): reset [n_envs][max_episodes_per_env][4] in [0,1) and
   * cat_sample [n_envs][ceil(n_timesteps/n_envs) + min(max_pathlength, time_limit) - 1] */
  const double* reset_uniforms;
  const double* action_uniforms;
  int max_episodes_per_env;
  int mem;                   /* where the injected arrays live */
} trpo_rollout_params;
void trpo_default_rollout_params(trpo_rollout_params* p);
/* run the rollout; returns the total steps N and the number of paths */
int trpo_rollout_cartpole(trpo_engine* e, const trpo_rollout_params* p, int64_t* n_steps_out, int64_t* n_paths_out);
/* the concatenated paths (utils.py:36-39): obs [N][4] f64 (and/or as the float32 the placeholders
 * receive), actions [N] i64, action_dists [N][A] f32, rewards [N] f64, episode_starts [N] u8, and the
 * cat_sample uniform of every step; any may be NULL */
int trpo_rollout_fetch(trpo_engine* e, double* obs, float* obs32, int64_t* actions, float* action_dists,
                       double* rewards, uint8_t* episode_starts, double* uniforms, int mem);
/* the rollout becomes the feed on the device (trpo_inksci.py:108-112,119-122): states, actions,
 * oldaction_dist, rewards and path starts, with no host round trip; baseline cleared */
int trpo_rollout_to_batch(trpo_engine* e, int64_t n_global);
/* Device pointers into the current feed, for other device-side consumers (the VF) to read in place;
 * synchronises the engine stream first. */
typedef struct trpo_feed_view {
  int64_t n, n_global;
  int obs_dim, n_actions;
  const float* states;       /* [n][ld_states] f32 */
  int ld_states;
  const float* old_dist;     /* [n][ld_old] f32 */
  int ld_old;
  const uint8_t* episode_starts;   /* [n] */
  const double* returns;     /* [n] f64 after the advantages of this feed were computed, else NULL */
  double* baseline;          /* [n] f64; trpo_set_baseline(e, view.baseline, TRPO_MEM_DEVICE) marks it set */
} trpo_feed_view;
int trpo_get_feed_view(trpo_engine* e, trpo_feed_view* out);
/* set only the baseline [n] f64 of the current feed (VF.predict output, trpo_inksci.py:103) */
int trpo_set_baseline(trpo_engine* e, const double* baseline, int mem);
/* explained_variance(baseline, returns) (utils.py:208-211, trpo_inksci.py:167) over the current
 * feed (all ranks), after the returns were computed; NaN when var(returns) == 0 */
int trpo_explained_variance(trpo_engine* e, double* out);
/* agent.act on n states [n][obs_dim] f32 (trpo_inksci.py:76-87): action_dist at the current
 * parameters and cat_sample against `uniforms` [n] (train = 1) or argmax (train = 0).
 * n_actions <= 64 here (one wave per state): an engine created with 65..128 actions updates, but
 * trpo_act returns an error for it (and trpo_rollout_cartpole needs exactly 2 actions). */
int trpo_act(trpo_engine* e, const float* states, int64_t n, const double* uniforms, int train, int64_t* actions_out,
             float* dists_out, int mem);
/* cat_sample(prob_nk) (utils.py:95-105) with the uniforms given: engine-free, current device */
int trpo_cat_sample(const float* prob, int64_t n, int k, const double* uniforms, int64_t* out, int mem);
/* one CartPole-v0 step per row (state [n][4] f64, action [n] i64); done = termination (not the TimeLimit) */
int trpo_cartpole_step(const double* state, const int64_t* action, int64_t n, double* state_out, double* reward,
                       uint8_t* done, int mem);

/* ==== value-function baseline: class VF (utils.py:48-92) ==================================
 * Features [obs | action_dist | t/10] (VF._features, utils.py:70-77) -> fully_connected(64, relu)
 * -> fully_connected(64, relu) -> fully_connected(1) (create_net, utils.py:56-62); fit = 50 steps
 * of tf.train.AdamOptimizer() on sum((net - y)^2) over the whole batch (utils.py:64-66,79-85);
 * predict = the net on one path's features (utils.py:87-92).  Parameters are flat in creation
 * order [W1, b1, W2, b2, W3, b3], W row-major [fan_in][fan_out]. */
typedef struct trpo_vf trpo_vf;
/* feat_dim = obs_dim + n_actions + 1; hidden = {64, 64} (utils.py:60-61) or NULL/0 for that default */
int trpo_vf_create(trpo_vf** out, int feat_dim, const int* hidden, int n_hidden, int64_t max_rows, int device);
void trpo_vf_destroy(trpo_vf* vf);
int64_t trpo_vf_num_params(const trpo_vf* vf);
int trpo_vf_set_params(trpo_vf* vf, const float* flat, int mem);
int trpo_vf_get_params(trpo_vf* vf, float* flat_out, int mem);
/* AdamOptimizer(learning_rate, beta1, beta2, epsilon) (defaults 1e-3, 0.9, 0.999, 1e-8); resets the slots */
int trpo_vf_set_adam(trpo_vf* vf, float lr, float beta1, float beta2, float epsilon);
/* m = v = 0, beta powers = (beta1, beta2): the state tf.initialize_all_variables() gives (utils.py:66) */
int trpo_vf_reset_optimizer(trpo_vf* vf);
/* Adam slots m, v [P] (either may be NULL), beta powers, steps taken */
int trpo_vf_get_optimizer(trpo_vf* vf, float* m_out, float* v_out, float powers_out[2], int64_t* steps_out,
                          int mem);
/* Build the features on the device from a concatenation of paths: obs [n][obs_dim], action_dists
 * [n][n_actions] f32, episode_starts [n] u8 (1 = first step of a path; NULL = one path).  t counts
 * steps from each path start.  n_global = rows over all ranks. */
int trpo_vf_set_features(trpo_vf* vf, int64_t n, int64_t n_global, const float* obs, int obs_dim,
                         const float* action_dists, int n_actions, const uint8_t* episode_starts, int mem);
/* ... or from an engine's feed in place (trpo_get_feed_view), targets = its returns when with_targets */
int trpo_vf_set_features_view(trpo_vf* vf, const trpo_feed_view* view, int with_targets);
/* ... or take a ready feature matrix [n][feat_dim] f32 */
int trpo_vf_set_feature_matrix(trpo_vf* vf, int64_t n, int64_t n_global, const float* feat, int mem);
int trpo_vf_get_feature_matrix(trpo_vf* vf, float* feat_out, int mem);
/* regression targets = the paths' returns [n] (TRPO_F64 as the reference feeds them, or TRPO_F32) */
int trpo_vf_set_targets(trpo_vf* vf, const void* returns, int dtype, int mem);
/* VF.fit's loop body `steps` times (utils.py:84-85; the reference runs 50) */
int trpo_vf_fit(trpo_vf* vf, int steps);
/* gradient of sum((net - y)^2) at the current parameters (all ranks) and, if loss_out, that sum */
int trpo_vf_gradient(trpo_vf* vf, float* grad_out, double* loss_out, int mem);
/* VF.predict: net on the current features -> out [n] (TRPO_F32 / TRPO_F64) */
int trpo_vf_predict(trpo_vf* vf, void* out, int dtype, int mem);
/* multi-GPU: shard rows, all-reduce the [P] gradient (RCCL), or the host test transport */
int trpo_vf_comm_init(trpo_vf* vf, const uint8_t id[128], int rank, int world);
int trpo_vf_comm_set_host_allreduce(trpo_vf* vf, trpo_allreduce_cb cb, void* ctx, int rank, int world);

#ifdef __cplusplus
}
#endif
#endif /* TRPO_ENGINE_H */
