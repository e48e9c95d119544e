"""The learn() loop of trpo_inksci.py:89-177 on the device (rollout -> VF -> advantages -> update
-> explained variance), and the utils surface added for it."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_explained_variance_matches_numpy(gpu_available):
    from trpo_amd import Engine, utils
    from trpo_amd.agent import xavier_theta
    e = Engine(4, [64], 2, max_rows=1 << 14)
    e.set_flat(xavier_theta(4, [64], 2))
    n, _ = e.rollout_cartpole(n_envs=16, n_timesteps=4000, seed=5)
    e.rollout_to_batch()
    out = e.rollout_fetch()
    base = np.random.RandomState(0).uniform(0, 10, n)
    e.set_baseline(base)
    ret = np.empty(n)
    e.compute_advantages_device(0.95, returns_out=ret)
    # the returns are the reference's discount per path
    from oracle.trpo_oracle import discount_segmented
    assert np.allclose(ret, discount_segmented(out["rewards"], out["starts"], 0.95), rtol=1e-12)
    assert e.explained_variance() == pytest.approx(utils.explained_variance(base, ret), rel=1e-12)
    e.close()


def test_learn_improves_cartpole(gpu_available):
    from trpo_amd import TRPOAgent
    agent = TRPOAgent(4, 2, hidden=(64,), max_rows=4096)
    hist = agent.learn(max_iterations=30, n_envs=4, seed=3, log=None)
    assert len(hist) == 30
    trained = [h for h in hist if h["train"]]
    for h in trained:
        assert np.isfinite(h["entropy"]) and np.isfinite(h["surr"])
        assert h["reverted"] or h["kl"] <= 2 * 0.01
        assert h["steps"] >= 1000
    first = np.mean([h["reward_mean"] for h in hist[:5]])
    last = np.mean([h["reward_mean"] for h in hist[-5:]])
    assert last > first + 20, (first, last)
    assert agent.vf.net is not None


def test_utils_cat_sample_and_rollout_dropins(gpu_available):
    from trpo_amd import utils
    from oracle.cartpole_oracle import CartPoleV0, OracleAgent, cat_sample
    p = np.random.RandomState(1).dirichlet(np.ones(5), 300)
    np.random.seed(4)
    a = utils.cat_sample(p)
    np.random.seed(4)
    r = np.random.rand(300)
    assert a.dtype == np.dtype("i") and np.array_equal(a, cat_sample(p.astype(np.float32), r))
    theta = np.random.RandomState(2).uniform(-0.3, 0.3, 4 * 64 + 64 + 64 * 2 + 2).astype(np.float32)
    agent = OracleAgent(theta, [4, 64, 2], utils.cat_sample)
    paths = utils.rollout(CartPoleV0(seed=1), agent, 1000, 500)
    assert sum(len(p["rewards"]) for p in paths) >= 500
    assert all(p["obs"].shape == (len(p["rewards"]), 4) and p["action_dists"].shape == (len(p["rewards"]), 2)
               for p in paths)
