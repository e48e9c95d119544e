"""GPU parity of the value-function baseline (trpo_vf_* C-ABI, utils.py:48-92) against the VF
oracle (oracle/vf_oracle.py, float64).  Bars: features bit-exact; gradient, predictions and the
parameters after one Adam step norm-relative <= 1e-5; after the reference's 50-step fit the
parameters and predictions norm-relative <= 1e-4 (Adam divides each step by sqrt(v), so fp32
summation-order differences in near-zero gradient entries are amplified over 50 steps)."""
import numpy as np
import pytest

from conftest import assert_vec_close, rel_l2
from oracle import vf_oracle as V

pytestmark = pytest.mark.gpu


def batch(n, obs, A, seed, path_len=37):
    rng = np.random.RandomState(seed)
    o = rng.standard_normal((n, obs)).astype(np.float32)
    d = rng.dirichlet(np.ones(A), n).astype(np.float32)
    starts = np.zeros(n, np.uint8)
    starts[::path_len] = 1
    starts[rng.randint(0, n, 5)] = 1
    y = np.cumsum(rng.uniform(0, 1, n))[::-1].copy() % 20.0
    return o, d, starts, y


def net_for(F, n):
    from trpo_amd.vf import VFNet, vf_xavier_params
    net = VFNet(F, max(n, 16))
    th = vf_xavier_params(F, (64, 64), np.random.RandomState(F))
    th[F * 64:F * 64 + 64] = 0.05        # non-zero biases exercise the bias paths
    net.set_params(th)
    return net, th


@pytest.mark.parametrize("n,obs,A", [(1000, 4, 2), (4099, 128, 18), (70000, 11, 3)])
def test_features_bit_exact(gpu_available, n, obs, A):
    o, d, starts, _ = batch(n, obs, A, n)
    net, _ = net_for(obs + A + 1, n)
    net.set_features(o, d, starts)
    assert np.array_equal(net.feature_matrix(), V.features_concat(o, d, starts))
    net.set_features(o, d, None)     # one path
    assert np.array_equal(net.feature_matrix(), V.features_concat(o, d, np.r_[1, np.zeros(n - 1, np.uint8)]))
    net.close()


@pytest.mark.parametrize("n,obs,A", [(1000, 4, 2), (3001, 128, 18), (513, 376, 17)])
def test_gradient_predict_and_one_step(gpu_available, n, obs, A):
    o, d, starts, y = batch(n, obs, A, 7 * n)
    F = obs + A + 1
    net, th = net_for(F, n)
    net.set_features(o, d, starts)
    net.set_targets(y)
    feat = V.features_concat(o, d, starts)
    g, loss = net.gradient()
    g_ref, loss_ref = V.gradient(th.astype(np.float64), feat, y.astype(np.float32))
    assert_vec_close(g, g_ref, 1e-5, "VF gradient")
    assert loss == pytest.approx(loss_ref, rel=1e-5)
    assert_vec_close(net.predict(), V.predict(th.astype(np.float64), feat), 1e-5, "VF predict")
    net.fit(1)
    adam = V.Adam(th.size)
    th1 = adam.step(th.astype(np.float64), g_ref)
    assert_vec_close(net.get_params(), th1, 1e-5, "VF params after one Adam step")
    st = net.optimizer_state()
    assert st["steps"] == 1 and st["beta1_power"] == adam.b1p and st["beta2_power"] == adam.b2p
    net.close()


def test_fit_50_steps_vs_oracle(gpu_available):
    n, obs, A = 4000, 4, 2
    o, d, starts, y = batch(n, obs, A, 3)
    F = obs + A + 1
    net, th = net_for(F, n)
    net.set_features(o, d, starts)
    net.set_targets(y)
    net.fit(50)
    feat = V.features_concat(o, d, starts)
    th_ref, adam = V.fit(th.astype(np.float64), feat, y.astype(np.float32), steps=50)
    assert rel_l2(net.get_params(), th_ref) < 1e-4
    assert rel_l2(net.predict(), V.predict(th_ref, feat)) < 1e-4
    # Adam state carries over to the next fit (one optimizer per VF, utils.py:65)
    net.fit(50)
    th_ref2, _ = V.fit(th_ref, feat, y.astype(np.float32), steps=50, adam=adam)
    assert rel_l2(net.get_params(), th_ref2) < 1e-4
    net.close()


def test_vf_class_matches_reference_protocol(gpu_available):
    """VF(session): predict -> zeros before the first fit; fit(paths) creates the net, asks the
    session to re-initialise (utils.py:66), runs 50 steps; predict(path) is the net on that path."""
    from trpo_amd.vf import VF, vf_xavier_params
    calls = []

    class S:
        engine = None

        def initialize_all_variables(self):
            calls.append(1)

    rng = np.random.RandomState(0)
    paths = []
    for L in (20, 35, 200):
        paths.append({"obs": rng.standard_normal((L, 4)), "action_dists": rng.dirichlet([1, 1], L),
                      "rewards": np.ones(L), "returns": np.cumsum(np.ones(L))[::-1] * 0.5})
    vf = VF(S(), max_rows=1024)
    assert np.array_equal(vf.predict(paths[0]), np.zeros(20))
    vf.fit(paths)
    assert calls == [1]
    feat = np.concatenate([V.features(p) for p in paths])
    th_init = vf_xavier_params(7, (64, 64), np.random.RandomState(1)).astype(np.float64)   # VF's default rng
    th0 = V.fit(th_init, feat, np.concatenate([p["returns"] for p in paths]).astype(np.float32))[0]
    pred = vf.predict(paths[1])
    assert pred.shape == (35,) and pred.dtype == np.float32
    assert rel_l2(pred, V.predict(th0, V.features(paths[1]))) < 1e-4
    vf.fit(paths)
    assert calls == [1]          # create_net runs once


def test_sharded_gradient_sums_to_full(gpu_available):
    """Two row shards with the host all-reduce transport give the full-batch gradient."""
    n, obs, A = 2000, 11, 3
    o, d, starts, y = batch(n, obs, A, 11)
    F = obs + A + 1
    full, th = net_for(F, n)
    full.set_features(o, d, starts)
    full.set_targets(y)
    g_full, _ = full.gradient()
    cut = 1000
    starts2 = starts.copy()
    starts2[cut] = 1                  # shards begin at a path start
    parts = []
    nets = []
    for lo, hi in ((0, cut), (cut, n)):
        net, _ = net_for(F, n)
        net.set_features(o[lo:hi], d[lo:hi], starts2[lo:hi], n_global=n)
        net.set_targets(y[lo:hi])
        parts.append(net.gradient()[0])
        nets.append(net)
    g_sum = parts[0].astype(np.float64) + parts[1]
    full.set_features(o, d, starts2)
    full.set_targets(y)
    assert_vec_close(g_sum, full.gradient()[0], 1e-5, "sharded VF gradient")
    for x in nets + [full]:
        x.close()
