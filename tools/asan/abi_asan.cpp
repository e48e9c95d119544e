// Host AddressSanitizer driver for the C-ABI ("host side: ASan on the C++ runtime
// build").  Built by `make -C trpo_amd/csrc asan` (engine.cpp / vf.cpp host code instrumented with
// -fsanitize=address; device objects unchanged) and run by tests/test_asan.py on a CPU-only host:
// every entry point's argument validation, error reporting and cleanup of a partially
// initialised engine, with no GPU present.  Exit code 0 = all checks passed, ASan clean.
#include "../../include/trpo_engine.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

static int fails = 0;
#define CHECK(cond)                                                          \
  do {                                                                       \
    if (!(cond)) {                                                           \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);   \
      ++fails;                                                               \
    }                                                                        \
  } while (0)
#define CHECK_ERR(call, code)                                                \
  do {                                                                       \
    const int rc_ = (call);                                                  \
    CHECK(rc_ == (code));                                                    \
    CHECK(std::strlen(trpo_last_error()) > 0);                               \
  } while (0)

static int fax(const void*, void*, void*) { return 0; }
static int allreduce(void*, int64_t, int, void*) { return 0; }

int main() {
  // ---- pure host entries ----
  trpo_update_params p;
  trpo_default_params(&p);
  CHECK(p.cg_iters == 10 && p.max_kl == 0.01 && p.gamma == 0.95);
  trpo_default_params(nullptr);
  trpo_rollout_params rp;
  trpo_default_rollout_params(&rp);
  CHECK(rp.n_envs == 1 && rp.max_pathlength == 1000 && rp.time_limit == 200);
  int ndev = -1;
  CHECK(trpo_device_count(&ndev) == TRPO_OK && ndev >= 0);
  CHECK_ERR(trpo_device_count(nullptr), TRPO_ERR_ARG);

  // ---- options ----
  int v = -1;
  CHECK(trpo_get_option("graphs", &v) == TRPO_OK);
  CHECK(trpo_set_option("graphs", v) == TRPO_OK);
  CHECK_ERR(trpo_set_option("no_such_option", 1), TRPO_ERR_ARG);
  CHECK_ERR(trpo_get_option(nullptr, &v), TRPO_ERR_ARG);
  CHECK_ERR(trpo_get_option("tail", nullptr), TRPO_ERR_ARG);

  // ---- engine creation: argument validation, then (no GPU) the HIP failure path ----
  trpo_engine* e = nullptr;
  const int hid[2] = {64, 64};
  CHECK_ERR(trpo_create(nullptr, 4, hid, 2, 2, 100, 0), TRPO_ERR_ARG);
  CHECK_ERR(trpo_create(&e, 4, hid, 2, 200, 100, 0), TRPO_ERR_ARG);     // n_actions > 128
  CHECK_ERR(trpo_create(&e, 0, hid, 2, 2, 100, 0), TRPO_ERR_ARG);
  CHECK_ERR(trpo_create(&e, 4, nullptr, 2, 2, 100, 0), TRPO_ERR_ARG);
  const int badh[2] = {64, -3};
  CHECK_ERR(trpo_create(&e, 4, badh, 2, 2, 100, 0), TRPO_ERR_ARG);
  CHECK_ERR(trpo_create(&e, 4, hid, 9, 2, 100, 0), TRPO_ERR_ARG);      // too many layers
  CHECK_ERR(trpo_create(&e, 4, hid, 2, 2, int64_t(1) << 40, 0), TRPO_ERR_ARG);
  if (ndev == 0) {
    // a well-formed engine on a host without a GPU: hipSetDevice fails inside init, the partially
    // built engine is released (the code path ASan watches)
    CHECK(trpo_create(&e, 4, hid, 2, 2, 100, 0) != TRPO_OK);
    CHECK(e == nullptr);
  }

  // ---- NULL engine handles ----
  float f3[3];
  std::vector<float> buf(16);
  CHECK(trpo_num_params(nullptr) == -1);
  trpo_destroy(nullptr);
  CHECK(trpo_stream(nullptr) == nullptr);
  CHECK_ERR(trpo_synchronize(nullptr), TRPO_ERR_ARG);
  CHECK_ERR(trpo_set_flat(nullptr, buf.data(), TRPO_MEM_HOST), TRPO_ERR_ARG);
  CHECK_ERR(trpo_get_flat(nullptr, buf.data(), TRPO_MEM_HOST), TRPO_ERR_ARG);
  CHECK_ERR(trpo_get_vector(nullptr, 0, buf.data(), TRPO_MEM_HOST), TRPO_ERR_ARG);
  CHECK_ERR(trpo_set_batch(nullptr, 1, 1, buf.data(), nullptr, nullptr, buf.data(), TRPO_MEM_HOST), TRPO_ERR_ARG);
  CHECK_ERR(trpo_losses(nullptr, f3), TRPO_ERR_ARG);
  CHECK_ERR(trpo_eval_losses(nullptr, buf.data(), f3, TRPO_MEM_HOST), TRPO_ERR_ARG);
  CHECK_ERR(trpo_policy_grad(nullptr, buf.data(), TRPO_MEM_HOST), TRPO_ERR_ARG);
  CHECK_ERR(trpo_fvp(nullptr, buf.data(), buf.data(), 0.1f, TRPO_MEM_HOST), TRPO_ERR_ARG);
  CHECK_ERR(trpo_cg(nullptr, buf.data(), buf.data(), 10, 1e-10f, 0.1f, nullptr, TRPO_MEM_HOST), TRPO_ERR_ARG);
  int k = 0;
  CHECK_ERR(trpo_linesearch(nullptr, buf.data(), buf.data(), 1.0, buf.data(), &k, TRPO_MEM_HOST), TRPO_ERR_ARG);
  CHECK_ERR(trpo_update(nullptr, &p, nullptr), TRPO_ERR_ARG);
  CHECK_ERR(trpo_compute_advantages(nullptr, 0.95, nullptr, nullptr, TRPO_MEM_HOST), TRPO_ERR_ARG);
  CHECK_ERR(trpo_profile_enable(nullptr, 1), TRPO_ERR_ARG);
  CHECK(trpo_profile_query(nullptr, nullptr, 0) < 0);
  CHECK_ERR(trpo_profile_reset(nullptr), TRPO_ERR_ARG);
  CHECK_ERR(trpo_comm_init(nullptr, nullptr, 0, 1), TRPO_ERR_ARG);
  CHECK_ERR(trpo_comm_set_host_allreduce(nullptr, allreduce, nullptr, 0, 1), TRPO_ERR_ARG);
  CHECK_ERR(trpo_rollout_cartpole(nullptr, &rp, nullptr, nullptr), TRPO_ERR_ARG);
  CHECK_ERR(trpo_rollout_to_batch(nullptr, 1), TRPO_ERR_ARG);
  trpo_feed_view fv;
  CHECK_ERR(trpo_get_feed_view(nullptr, &fv), TRPO_ERR_ARG);
  double ev = 0.0;
  CHECK_ERR(trpo_explained_variance(nullptr, &ev), TRPO_ERR_ARG);

  // ---- engine-free kernels: argument validation before any device work ----
  std::vector<double> d(8, 1.0);
  CHECK_ERR(trpo_discount(nullptr, nullptr, 8, 0.95, d.data(), TRPO_MEM_HOST), TRPO_ERR_ARG);
  CHECK_ERR(trpo_discount(d.data(), nullptr, -1, 0.95, d.data(), TRPO_MEM_HOST), TRPO_ERR_ARG);
  CHECK(trpo_discount(d.data(), nullptr, 0, 0.95, d.data(), TRPO_MEM_HOST) == TRPO_OK);   // n = 0: no-op
  CHECK_ERR(trpo_standardize(nullptr, nullptr, 8, 8, nullptr, TRPO_MEM_HOST), TRPO_ERR_ARG);
  CHECK_ERR(trpo_standardize(nullptr, d.data(), 8, 16, nullptr, TRPO_MEM_HOST), TRPO_ERR_ARG);
  CHECK_ERR(trpo_standardize(nullptr, d.data(), 9, 8, nullptr, TRPO_MEM_HOST), TRPO_ERR_ARG);
  CHECK(trpo_standardize(nullptr, d.data(), 0, 0, nullptr, TRPO_MEM_HOST) == TRPO_OK);      // empty
  int64_t out[4];
  CHECK_ERR(trpo_cat_sample(nullptr, 4, 2, d.data(), out, TRPO_MEM_HOST), TRPO_ERR_ARG);
  CHECK(trpo_cat_sample(buf.data(), 0, 2, d.data(), out, TRPO_MEM_HOST) == TRPO_OK);
  CHECK_ERR(trpo_cartpole_step(nullptr, out, 1, d.data(), nullptr, nullptr, TRPO_MEM_HOST), TRPO_ERR_ARG);
  int iters = 0;
  CHECK_ERR(trpo_cg_callback(nullptr, nullptr, d.data(), d.data(), 8, TRPO_F64, 10, 0.0, &iters), TRPO_ERR_ARG);
  CHECK_ERR(trpo_cg_callback(fax, nullptr, d.data(), d.data(), 8, 7, 10, 0.0, &iters), TRPO_ERR_ARG);
  CHECK_ERR(trpo_cg_callback(fax, nullptr, d.data(), d.data(), 0, TRPO_F64, 10, 0.0, &iters), TRPO_ERR_ARG);
  CHECK_ERR(trpo_cg_callback(fax, nullptr, d.data(), d.data(), 8, TRPO_F64, 1000, 0.0, &iters), TRPO_ERR_ARG);

  // ---- VF handles ----
  trpo_vf* vf = nullptr;
  CHECK(trpo_vf_num_params(nullptr) == -1);
  trpo_vf_destroy(nullptr);
  CHECK_ERR(trpo_vf_create(nullptr, 7, nullptr, 0, 100, 0), TRPO_ERR_ARG);
  CHECK_ERR(trpo_vf_create(&vf, 0, nullptr, 0, 100, 0), TRPO_ERR_ARG);
  CHECK_ERR(trpo_vf_fit(nullptr, 50), TRPO_ERR_ARG);
  CHECK_ERR(trpo_vf_set_params(nullptr, buf.data(), TRPO_MEM_HOST), TRPO_ERR_ARG);
  if (ndev == 0) {
    CHECK(trpo_vf_create(&vf, 7, nullptr, 0, 100, 0) != TRPO_OK);
    CHECK(vf == nullptr);
  }

  if (fails) {
    std::fprintf(stderr, "%d check(s) failed\n", fails);
    return 1;
  }
  std::printf("ABI ASAN OK (%d GPU(s) visible)\n", ndev);
  return 0;
}
