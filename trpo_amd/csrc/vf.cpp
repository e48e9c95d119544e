// Value-function baseline runtime behind the trpo_vf_* C-ABI (include/trpo_engine.h).
//
// The VF of utils.py:48-92: features [obs | action_dist | t/10] (utils.py:70-77),
// a 64-64 ReLU MLP with a linear output (utils.py:58-62), fitted with 50
// full-batch steps of TF's AdamOptimizer on sum((net - y)^2) (utils.py:64-66,84-85)
// and evaluated by predict (utils.py:87-92).  One handle = one GPU = one row
// shard; with a communicator the per-shard gradient sums are all-reduced, which
// is the full-batch gradient of the reference.
//
// One Adam step:
//   Z1  = relu(F W1 + b1)            rowgemm, RowEpi::kRelu
//   Z2  = relu(Z1 W2 + b2)           rowgemm, RowEpi::kRelu
//   net = Z2 w3 + b3 ; dnet = 2(net - y) ; dZ2 = dnet w3^T (Z2 > 0)     vf_head_kernel
//   dZ1 = (dZ2 W2^T)(Z1 > 0)         rowgemm, RowEpi::kReluBwd
//   gW1, gb1 = F^T dZ1, colsum dZ1 ; gW2, gb2 = Z1^T dZ2, colsum dZ2 ; gw3, gb3 = Z2^T dnet, sum dnet
//                                    split-K wgrad slabs, reduced in a fixed order
//   Adam (TF 1.x ApplyAdam)          adam_kernel
#include "../../include/trpo_engine.h"
#include "abi_util.h"
#include "common.h"
#include "kernels.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

using namespace trpo;
using namespace trpo_abi;

struct trpo_vf {
  int device = 0;
  hipStream_t stream = nullptr;
  int F = 0, Fp = 0, H1 = 64, H1p = 64, H2 = 64, H2p = 64;
  int64_t P = 0, offW1 = 0, offb1 = 0, offW2 = 0, offb2 = 0, offW3 = 0, offb3 = 0;
  int64_t cap = 0, n = 0, n_global = 0;
  bool have_feat = false, have_tgt = false;
  // Adam (tf.train.AdamOptimizer() defaults) and its state; beta powers as TF's float32 variables
  float lr = 0.001f, b1 = 0.9f, b2 = 0.999f, eps = 1e-8f;
  float b1p = 0.9f, b2p = 0.999f;
  int64_t steps_done = 0;
  // multi-GPU
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
  trpo_allreduce_cb host_ar = nullptr;
  void* host_ar_ctx = nullptr;

  std::vector<void*> allocs;
  float *theta = nullptr, *grad = nullptr, *m = nullptr, *v = nullptr;
  float *W1p = nullptr, *W2p = nullptr, *W2T = nullptr;
  float *feat = nullptr, *Z1 = nullptr, *Z2 = nullptr, *dZ1 = nullptr, *dZ2 = nullptr, *dout = nullptr, *tgt = nullptr;
  double* loss_rows = nullptr;
  int64_t* lastpos = nullptr;
  void* pos_ws = nullptr;
  // staging for host inputs: cap rows of max(F floats, 1 double) + cap starts
  float* stage = nullptr;
  uint8_t* stage_starts = nullptr;
  float* slab = nullptr;
  int S = 1, active_splits = 1, rows_per_split = 64;
  int64_t slab_stride = 0;
  bool packed = false;

  template <class T>
  T* dalloc(size_t count) {
    void* ptr = nullptr;
    const size_t bytes = std::max<size_t>(count * sizeof(T), 16);
    HIPCHECK(hipMalloc(&ptr, bytes));
    HIPCHECK(hipMemsetAsync(ptr, 0, bytes, stream));
    allocs.push_back(ptr);
    return static_cast<T*>(ptr);
  }
  void use() { HIPCHECK(hipSetDevice(device)); }

  void init(int feat_dim, const int* hidden, int n_hidden, int64_t max_rows, int dev) {
    REQUIRE(feat_dim >= 1, "feat_dim must be >= 1");
    REQUIRE(max_rows >= 1, "max_rows must be >= 1");
    REQUIRE(n_hidden == 0 || n_hidden == 2, "the VF has two hidden layers (utils.py:60-61)");
    if (n_hidden == 2) {
      REQUIRE(hidden && hidden[0] >= 1 && hidden[1] >= 1 && hidden[0] <= 4096 && hidden[1] <= 4096,
              "bad hidden widths");
      H1 = hidden[0];
      H2 = hidden[1];
    }
    int ndev = 0;
    HIPCHECK(hipGetDeviceCount(&ndev));
    REQUIRE(dev >= 0 && dev < ndev, "device id out of range");
    device = dev;
    use();
    HIPCHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    F = feat_dim;
    Fp = pad4(F);
    H1p = pad4(H1);
    H2p = pad4(H2);
    // flat layout [W1, b1, W2, b2, W3, b3] (creation order of pt.fully_connected x3)
    offW1 = 0;
    offb1 = offW1 + (int64_t)F * H1;
    offW2 = offb1 + H1;
    offb2 = offW2 + (int64_t)H1 * H2;
    offW3 = offb2 + H2;
    offb3 = offW3 + H2;
    P = offb3 + 1;
    cap = max_rows;
    theta = dalloc<float>(P);
    grad = dalloc<float>(P);
    m = dalloc<float>(P);
    v = dalloc<float>(P);
    W1p = dalloc<float>((size_t)Fp * H1p);
    W2p = dalloc<float>((size_t)H1p * H2p);
    W2T = dalloc<float>((size_t)H2p * H1p);
    feat = dalloc<float>((size_t)cap * Fp);
    Z1 = dalloc<float>((size_t)cap * H1p);
    Z2 = dalloc<float>((size_t)cap * H2p);
    dZ1 = dalloc<float>((size_t)cap * H1p);
    dZ2 = dalloc<float>((size_t)cap * H2p);
    dout = dalloc<float>((size_t)cap * 4);
    tgt = dalloc<float>(cap);
    loss_rows = dalloc<double>(cap);
    lastpos = dalloc<int64_t>(cap);
    pos_ws = dalloc<uint8_t>(vf_pos_workspace_bytes(cap));
    stage = dalloc<float>((size_t)cap * std::max(Fp, 2));
    stage_starts = dalloc<uint8_t>(cap);
    const int tiles = ((F + 255) / 256) * ((H1 + 255) / 256);
    S = std::max(1, std::min(512, 1024 / std::max(1, tiles)));
    slab_stride = (P + 63) / 64 * 64;
    slab = dalloc<float>((size_t)S * slab_stride);
    HIPCHECK(hipStreamSynchronize(stream));
  }

  void release() {
    if (device >= 0) (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    if (comm) (void)ncclCommDestroy(comm);
    comm = nullptr;
    for (void* p : allocs) (void)hipFree(p);
    allocs.clear();
    if (stream) (void)hipStreamDestroy(stream);
    stream = nullptr;
  }

  void set_rows(int64_t rows, int64_t rows_global) {
    REQUIRE(rows > 0 && rows <= cap, "n out of range (0 < n <= max_rows)");
    REQUIRE(rows_global >= rows, "n_global must be >= n");
    if (have_feat && rows != n) have_tgt = false;
    n = rows;
    n_global = rows_global;
    int64_t rps = (n + S - 1) / S;
    rps = std::max<int64_t>(64, (rps + 31) / 32 * 32);
    rows_per_split = (int)rps;
    active_splits = (int)std::max<int64_t>(1, (n + rps - 1) / rps);
  }

  void pack() {
    if (packed) return;
    VFPackArgs a{F, H1, H2, H1p, H2p, offW1, offW2, W1p, W2p, W2T};
    launch_vf_pack(a, theta, stream);
    check_launch();
    packed = true;
  }

  RowGemmArgs row(const float* A, int lda, int K, const float* B, int ldb, int N, int Npad) {
    RowGemmArgs a{};
    a.M = (int)n;
    a.N = N;
    a.Npad = Npad;
    a.nseg = 1;
    a.seg[0] = GemmSeg{A, B, lda, ldb, K};
    return a;
  }

  void forward() {
    pack();
    RowGemmArgs a = row(feat, Fp, Fp, W1p, H1p, H1, H1p);
    a.epi = RowEpi::kRelu;
    a.ea.bias = theta + offb1;
    a.ea.out0 = Z1;
    a.ea.ldo = H1p;
    launch_rowgemm(a, stream);
    check_launch();
    RowGemmArgs b = row(Z1, H1p, H1p, W2p, H2p, H2, H2p);
    b.epi = RowEpi::kRelu;
    b.ea.bias = theta + offb2;
    b.ea.out0 = Z2;
    b.ea.ldo = H2p;
    launch_rowgemm(b, stream);
    check_launch();
  }

  void wgrad(const float* A, int Ma, int Mpad, const float* B, int Nb, int Npad, int64_t offw, int64_t offb) {
    WGradArgs a{};
    a.rows = (int)n;
    a.Ma = Ma;
    a.Nb = Nb;
    a.Mpad = Mpad;
    a.Npad = Npad;
    a.nseg = 1;
    a.seg[0] = WSeg{A, B, Mpad, Npad};
    a.colsum_seg = 0;
    a.splits = active_splits;
    a.rows_per_split = rows_per_split;
    a.slab = slab;
    a.slab_stride = slab_stride;
    a.off_w = offw;
    a.off_b = offb;
    launch_wgrad(a, stream);
    check_launch();
  }

  void allreduce_grad() {
    if (!comm && !(host_ar && world > 1)) return;
    if (!comm) {
      std::vector<float> h((size_t)P);
      HIPCHECK(hipMemcpyAsync(h.data(), grad, P * sizeof(float), hipMemcpyDeviceToHost, stream));
      HIPCHECK(hipStreamSynchronize(stream));
      REQUIRE(host_ar(h.data(), P, TRPO_F32, host_ar_ctx) == 0, "host all-reduce callback failed");
      HIPCHECK(hipMemcpyAsync(grad, h.data(), P * sizeof(float), hipMemcpyHostToDevice, stream));
      HIPCHECK(hipStreamSynchronize(stream));
      return;
    }
    NCCLCHECK(ncclAllReduce(grad, grad, (size_t)P, ncclFloat32, ncclSum, comm, stream));
  }

  // gradient of sum over all rows (all ranks) of (net - y)^2
  void gradient() {
    REQUIRE(have_feat && have_tgt, "VF: features and targets must be set first");
    forward();
    VFHeadArgs h{};
    h.n = n;
    h.H2 = H2;
    h.H2p = H2p;
    h.Z2 = Z2;
    h.w3 = theta + offW3;
    h.b3 = theta + offb3;
    h.train = 1;
    h.y = tgt;
    h.dout = dout;
    h.dZ2 = dZ2;
    h.loss_rows = loss_rows;
    launch_vf_head(h, stream);
    check_launch();
    RowGemmArgs a = row(dZ2, H2p, H2p, W2T, H1p, H1, H1p);
    a.epi = RowEpi::kReluBwd;
    a.ea.H = Z1;
    a.ea.out0 = dZ1;
    a.ea.ldo = H1p;
    launch_rowgemm(a, stream);
    check_launch();
    wgrad(feat, F, Fp, dZ1, H1, H1p, offW1, offb1);
    wgrad(Z1, H1, H1p, dZ2, H2, H2p, offW2, offb2);
    wgrad(Z2, H2, H2p, dout, 1, 4, offW3, offb3);
    launch_reduce_slab(slab, active_splits, slab_stride, P, grad, nullptr, stream);
    check_launch();
    allreduce_grad();
  }

  // one AdamOptimizer.minimize step (utils.py:65,85)
  void adam_step() {
    gradient();
    // alpha = lr * sqrt(1 - beta2_power) / (1 - beta1_power) in float32 (training_ops.cc ApplyAdam)
    const float alpha = lr * std::sqrt(1.0f - b2p) / (1.0f - b1p);
    launch_adam(theta, grad, m, v, P, alpha, b1, b2, eps, stream);
    check_launch();
    packed = false;
    // the _finish ops: beta1_power *= beta1, beta2_power *= beta2 (float32 variables)
    b1p = b1p * b1;
    b2p = b2p * b2;
    ++steps_done;
  }

  void reset_optimizer() {
    HIPCHECK(hipMemsetAsync(m, 0, P * sizeof(float), stream));
    HIPCHECK(hipMemsetAsync(v, 0, P * sizeof(float), stream));
    b1p = b1;
    b2p = b2;
    steps_done = 0;
  }
};

extern "C" {

int trpo_vf_create(trpo_vf** out, int feat_dim, const int* hidden, int n_hidden, int64_t max_rows, int device) {
  return guarded([&] {
    REQUIRE(out, "out is NULL");
    auto e = std::make_unique<trpo_vf>();
    try {
      e->init(feat_dim, hidden, n_hidden, max_rows, device);
    } catch (...) {
      e->release();
      throw;
    }
    *out = e.release();
  });
}

void trpo_vf_destroy(trpo_vf* e) {
  if (!e) return;
  e->release();
  delete e;
}

int64_t trpo_vf_num_params(const trpo_vf* e) { return e ? e->P : -1; }

int trpo_vf_set_params(trpo_vf* e, const float* flat, int mem) {
  return guarded([&] {
    REQUIRE(e && flat, "NULL argument");
    e->use();
    copy_in(e->theta, flat, e->P * sizeof(float), mem, e->stream);
    e->packed = false;
  });
}

int trpo_vf_get_params(trpo_vf* e, float* out, int mem) {
  return guarded([&] {
    REQUIRE(e && out, "NULL argument");
    e->use();
    copy_out(out, e->theta, e->P * sizeof(float), mem, e->stream);
  });
}

int trpo_vf_set_adam(trpo_vf* e, float lr, float beta1, float beta2, float epsilon) {
  return guarded([&] {
    REQUIRE(e, "NULL argument");
    REQUIRE(lr > 0.0f && beta1 >= 0.0f && beta1 < 1.0f && beta2 >= 0.0f && beta2 < 1.0f && epsilon >= 0.0f,
            "bad Adam hyper-parameters");
    e->lr = lr;
    e->b1 = beta1;
    e->b2 = beta2;
    e->eps = epsilon;
    e->use();
    e->reset_optimizer();
  });
}

int trpo_vf_reset_optimizer(trpo_vf* e) {
  return guarded([&] {
    REQUIRE(e, "NULL argument");
    e->use();
    e->reset_optimizer();
  });
}

int trpo_vf_get_optimizer(trpo_vf* e, float* m_out, float* v_out, float powers_out[2], int64_t* steps_out, int mem) {
  return guarded([&] {
    REQUIRE(e, "NULL argument");
    e->use();
    if (m_out) copy_out(m_out, e->m, e->P * sizeof(float), mem, e->stream);
    if (v_out) copy_out(v_out, e->v, e->P * sizeof(float), mem, e->stream);
    if (powers_out) {
      powers_out[0] = e->b1p;
      powers_out[1] = e->b2p;
    }
    if (steps_out) *steps_out = e->steps_done;
  });
}

int trpo_vf_set_features(trpo_vf* e, int64_t n, int64_t n_global, const float* obs, int obs_dim,
                         const float* action_dists, int n_actions, const uint8_t* episode_starts, int mem) {
  return guarded([&] {
    REQUIRE(e && obs && action_dists, "NULL argument");
    REQUIRE(obs_dim >= 1 && n_actions >= 1 && obs_dim + n_actions + 1 == e->F,
            "feat_dim must equal obs_dim + n_actions + 1 (utils.py:70-77)");
    e->use();
    e->set_rows(n, n_global);
    const float* o = obs;
    const float* d = action_dists;
    const uint8_t* st = episode_starts;
    if (mem != TRPO_MEM_DEVICE) {
      // obs and dists side by side in the staging buffer (n * (obs_dim + A) <= n * F floats)
      float* so = e->stage;
      float* sd = e->stage + (size_t)n * obs_dim;
      copy_in(so, obs, (size_t)n * obs_dim * sizeof(float), mem, e->stream);
      copy_in(sd, action_dists, (size_t)n * n_actions * sizeof(float), mem, e->stream);
      o = so;
      d = sd;
      if (episode_starts) {
        copy_in(e->stage_starts, episode_starts, (size_t)n, mem, e->stream);
        st = e->stage_starts;
      }
    }
    launch_vf_features(o, obs_dim, obs_dim, d, n_actions, n_actions, st, n, e->lastpos, e->pos_ws, e->feat, e->Fp,
                       e->stream);
    check_launch();
    HIPCHECK(hipStreamSynchronize(e->stream));
    e->have_feat = true;
  });
}

int trpo_vf_set_features_view(trpo_vf* e, const trpo_feed_view* v, int with_targets) {
  return guarded([&] {
    REQUIRE(e && v && v->states && v->old_dist, "NULL argument");
    REQUIRE(v->obs_dim + v->n_actions + 1 == e->F, "feat_dim must equal obs_dim + n_actions + 1 (utils.py:70-77)");
    e->use();
    e->set_rows(v->n, v->n_global);
    launch_vf_features(v->states, v->obs_dim, v->ld_states, v->old_dist, v->n_actions, v->ld_old, v->episode_starts,
                       v->n, e->lastpos, e->pos_ws, e->feat, e->Fp, e->stream);
    check_launch();
    if (with_targets) {
      REQUIRE(v->returns, "view has no returns");
      launch_f64_to_f32(v->returns, e->tgt, e->n, e->stream);
      check_launch();
    }
    HIPCHECK(hipStreamSynchronize(e->stream));
    e->have_feat = true;
    if (with_targets) e->have_tgt = true;
  });
}

int trpo_vf_set_feature_matrix(trpo_vf* e, int64_t n, int64_t n_global, const float* feat, int mem) {
  return guarded([&] {
    REQUIRE(e && feat, "NULL argument");
    e->use();
    e->set_rows(n, n_global);
    if (e->Fp == e->F) {
      copy_in(e->feat, feat, (size_t)n * e->F * sizeof(float), mem, e->stream);
    } else {
      const float* src = feat;
      if (mem != TRPO_MEM_DEVICE) {
        copy_in(e->stage, feat, (size_t)n * e->F * sizeof(float), mem, e->stream);
        src = e->stage;
      }
      launch_copy_rows(src, n, e->F, e->F, e->feat, e->Fp, e->stream);
      check_launch();
      HIPCHECK(hipStreamSynchronize(e->stream));
    }
    e->have_feat = true;
  });
}

int trpo_vf_get_feature_matrix(trpo_vf* e, float* out, int mem) {
  return guarded([&] {
    REQUIRE(e && out, "NULL argument");
    REQUIRE(e->have_feat, "no features set");
    e->use();
    HIPCHECK(hipMemcpy2DAsync(out, (size_t)e->F * sizeof(float), e->feat, (size_t)e->Fp * sizeof(float),
                              (size_t)e->F * sizeof(float), (size_t)e->n,
                              mem == TRPO_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, e->stream));
    HIPCHECK(hipStreamSynchronize(e->stream));
  });
}

int trpo_vf_set_targets(trpo_vf* e, const void* returns, int dtype, int mem) {
  return guarded([&] {
    REQUIRE(e && returns, "NULL argument");
    REQUIRE(e->have_feat, "set features first (the row count comes from them)");
    REQUIRE(dtype == TRPO_F32 || dtype == TRPO_F64, "dtype must be TRPO_F32 or TRPO_F64");
    e->use();
    if (dtype == TRPO_F32) {
      copy_in(e->tgt, returns, (size_t)e->n * sizeof(float), mem, e->stream);
    } else {
      // the float64 returns fed to the float32 placeholder y (utils.py:58,85)
      const double* src = static_cast<const double*>(returns);
      if (mem != TRPO_MEM_DEVICE) {
        copy_in(e->stage, returns, (size_t)e->n * sizeof(double), mem, e->stream);
        src = reinterpret_cast<const double*>(e->stage);
      }
      launch_f64_to_f32(src, e->tgt, e->n, e->stream);
      check_launch();
      HIPCHECK(hipStreamSynchronize(e->stream));
    }
    e->have_tgt = true;
  });
}

int trpo_vf_fit(trpo_vf* e, int steps) {
  return guarded([&] {
    REQUIRE(e, "NULL argument");
    REQUIRE(steps >= 0, "steps must be >= 0");
    e->use();
    for (int i = 0; i < steps; ++i) e->adam_step();
    HIPCHECK(hipStreamSynchronize(e->stream));
  });
}

int trpo_vf_gradient(trpo_vf* e, float* grad_out, double* loss_out, int mem) {
  return guarded([&] {
    REQUIRE(e, "NULL argument");
    e->use();
    e->gradient();
    if (grad_out) copy_out(grad_out, e->grad, e->P * sizeof(float), mem, e->stream);
    if (loss_out) {
      std::vector<double> rows((size_t)e->n);
      copy_out(rows.data(), e->loss_rows, (size_t)e->n * sizeof(double), TRPO_MEM_HOST, e->stream);
      double s = 0.0;
      for (double x : rows) s += x;
      *loss_out = s;
    }
    HIPCHECK(hipStreamSynchronize(e->stream));
  });
}

int trpo_vf_predict(trpo_vf* e, void* out, int dtype, int mem) {
  return guarded([&] {
    REQUIRE(e && out, "NULL argument");
    REQUIRE(e->have_feat, "no features set");
    REQUIRE(dtype == TRPO_F32 || dtype == TRPO_F64, "dtype must be TRPO_F32 or TRPO_F64");
    e->use();
    e->forward();
    const size_t bytes = (size_t)e->n * (dtype == TRPO_F64 ? sizeof(double) : sizeof(float));
    void* dst = mem == TRPO_MEM_DEVICE ? out : (void*)e->stage;
    VFHeadArgs h{};
    h.n = e->n;
    h.H2 = e->H2;
    h.H2p = e->H2p;
    h.Z2 = e->Z2;
    h.w3 = e->theta + e->offW3;
    h.b3 = e->theta + e->offb3;
    h.train = 0;
    h.out32 = dtype == TRPO_F32 ? static_cast<float*>(dst) : nullptr;
    h.out64 = dtype == TRPO_F64 ? static_cast<double*>(dst) : nullptr;
    launch_vf_head(h, e->stream);
    check_launch();
    if (mem != TRPO_MEM_DEVICE) copy_out(out, e->stage, bytes, TRPO_MEM_HOST, e->stream);
    HIPCHECK(hipStreamSynchronize(e->stream));
  });
}

int trpo_vf_comm_init(trpo_vf* e, const uint8_t id[128], int rank, int world) {
  return guarded([&] {
    REQUIRE(e && id, "NULL argument");
    REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad rank/world");
    e->use();
    if (e->comm) {
      NCCLCHECK(ncclCommDestroy(e->comm));
      e->comm = nullptr;
    }
    e->rank = rank;
    e->world = world;
    e->host_ar = nullptr;
    // world = 1 creates a one-rank communicator too (the RCCL path on a single GPU)
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    NCCLCHECK(ncclCommInitRank(&e->comm, world, uid, rank));
  });
}

int trpo_vf_comm_set_host_allreduce(trpo_vf* e, trpo_allreduce_cb cb, void* ctx, int rank, int world) {
  return guarded([&] {
    REQUIRE(e && cb, "NULL argument");
    REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad rank/world");
    e->use();
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

}  // extern "C"
