"""The learn() loop of trpo_inksci.py:89-177 on the device (rollout -> VF -> advantages -> update
-> explained variance), and the utils surface added for it."""
import numpy as np
import pytest

from conftest import rel_l2

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


# ---------------------------------------------------------------------------- learn() vs the oracle loop
N_ITER = 3


def _draws(seed, n_iter, n_timesteps=1000, ep_max=200):
    """Recorded env.reset / cat_sample uniforms per iteration, as the reference's loop draws them
    (one environment: [1][max_episodes][4] and [1][budget + ep_max - 1])."""
    rng = np.random.RandomState(seed)
    ru = [rng.random_sample((1, n_timesteps, 4)) for _ in range(n_iter)]
    au = [rng.random_sample((1, n_timesteps + ep_max - 1)) for _ in range(n_iter)]
    return lambda i: (ru[i], au[i], n_timesteps)


def _oracle_inputs():
    from trpo_amd.agent import xavier_theta
    from trpo_amd.vf import vf_xavier_params
    rng = np.random.RandomState(1)                       # Session.init_rng (utils.py:7-9 seed)
    th0 = xavier_theta(4, [64], 2, rng)                  # TRPOAgent's initial policy
    th1 = xavier_theta(4, [64], 2, rng)                  # tf.initialize_all_variables() at the first VF fit
    return th0, th1, (lambda F: vf_xavier_params(F, (64, 64), np.random.RandomState(1)))


def test_learn_matches_oracle_loop(gpu_available):
    """Three learn() iterations (rollout -> VF predict -> advantages -> VF fit -> update ->
    explained variance, trpo_inksci.py:88-176) on the device against the oracle loop with the same
    recorded draws.  The oracle replays the device's sampled trajectory (its actions follow the
    device's action_dists under the same uniforms), so per-iteration numbers compare on identical
    paths; its own policy on those states must match the device's dists.  Bars: paths, actions,
    starts, rewards exact; returns 1e-12; baselines / advantages 1e-4 (the float32 VF after 50 Adam
    steps, tests/test_gpu_vf.py); k exact; surr / kl / ent / explained variance 1e-5 relative at iteration 0
    (zero baseline, no VF in the loop: north_star's bar), 1e-3 after (the VF's advantage drift)."""
    from trpo_amd import TRPOAgent
    from oracle import learn_oracle
    draws = _draws(11, N_ITER)
    agent = TRPOAgent(4, 2, hidden=(64,), max_rows=4096)
    hist = agent.learn(max_iterations=N_ITER, n_envs=1, log=None, draws=draws, record=True)
    th0, th1, vf_init = _oracle_inputs()
    ref = learn_oracle.learn(th0, [4, 64, 2], N_ITER, draws, th1, vf_init,
                             dists_from=lambda i: hist[i]["rollout"]["action_dists"])
    assert len(hist) == len(ref) == N_ITER
    for i, (h, r) in enumerate(zip(hist, ref)):
        ro_d, ro_o = h["rollout"], r["rollout"]
        assert h["steps"] == r["steps"] and h["paths"] == r["paths"], i
        assert np.array_equal(ro_d["actions"], ro_o["actions"]), i
        assert np.array_equal(ro_d["starts"], ro_o["starts"]) and np.array_equal(ro_d["rewards"], ro_o["rewards"])
        assert np.allclose(ro_d["obs"], ro_o["obs"], rtol=1e-12, atol=1e-14), i
        # the oracle's own policy on the device's states (theta after i updates)
        tol = 1e-6 if i == 0 else 1e-4
        assert np.max(np.abs(ro_d["action_dists"] - r["policy_dists"])) < tol, i
        assert np.allclose(h["returns"], r["returns"], rtol=1e-12), i
        if i == 0:
            assert not np.any(h["baseline"]) and not np.any(r["baseline"])
        else:
            assert rel_l2(h["baseline"], r["baseline"]) < 1e-4, (i, rel_l2(h["baseline"], r["baseline"]))
        assert rel_l2(h["advantages"], r["advantages"]) < 1e-4, (i, rel_l2(h["advantages"], r["advantages"]))
        assert h["k"] == r["k"] and h["reverted"] == r["reverted"], (i, h["k"], r["k"])
        # iteration 0 has no VF in the loop (zero baseline): only the update's own arithmetic separates the two
        rel = 1e-5 if i == 0 else 1e-3
        for key in ("surr", "kl", "ent", "explained_variance"):
            hk = "entropy" if key == "ent" else key
            assert h[hk] == pytest.approx(r[hk], rel=rel, abs=1e-7), (i, key, h[hk], r[hk])
    assert hist[0]["reverted"] == ref[0]["reverted"]


def test_learn_argmax_phase_and_end_count_exit(gpu_available):
    """trpo_inksci.py:137-141,174-175: once the baseline explains > 0.8 of the returns' variance,
    training stops, the rollouts take the argmax action, and the loop ends after end_count passes
    100.  The explained variance is forced above 0.8 at iteration 1 (control-flow test)."""
    from trpo_amd import TRPOAgent
    agent = TRPOAgent(4, 2, hidden=(64,), max_rows=4096)
    real_ev = agent.engine.explained_variance
    calls = []

    def forced_ev():
        calls.append(real_ev())
        return 0.9 if len(calls) >= 2 else calls[-1]
    agent.engine.explained_variance = forced_ev
    hist = agent.learn(max_iterations=200, n_envs=1, seed=5, log=None)
    trained = [h for h in hist if h["train"]]
    frozen = [h for h in hist if not h["train"]]
    assert len(trained) == 2 and len(calls) == 2
    assert len(frozen) == 101 and frozen[-1]["end_count"] == 101
    assert len(hist) == 103 and hist[-1]["iteration"] == 102
    theta = agent.engine.get_flat()
    # argmax rollouts never change the policy; two identical draws give identical paths
    agent.engine.rollout_cartpole(n_envs=1, n_timesteps=1000, train=False, seed=2)
    ro = agent.engine.rollout_fetch()
    from oracle.cartpole_oracle import policy_dist32
    assert np.array_equal(ro["actions"], np.argmax(ro["action_dists"], axis=1))
    assert np.max(np.abs(ro["action_dists"] - policy_dist32(theta, ro["obs"], [4, 64, 2]))) < 1e-6
    assert np.array_equal(agent.engine.get_flat(), theta)


def test_learn_mean_reward_stop_rule(gpu_available):
    """trpo_inksci.py:135-136: a mean episode reward above 1.1*500 stops training (unreachable on
    CartPole-v0's 200-step limit, so the statistics the loop reads are scaled: control flow only)."""
    from trpo_amd import TRPOAgent
    agent = TRPOAgent(4, 2, hidden=(64,), max_rows=4096)
    real = agent.engine.rollout_fetch_stats
    agent.engine.rollout_fetch_stats = lambda: {k: (v * 50.0 if k == "rewards" else v) for k, v in real().items()}
    hist = agent.learn(max_iterations=5, n_envs=1, seed=2, log=None)
    assert all(not h["train"] for h in hist)
    assert [h["end_count"] for h in hist] == [1, 2, 3, 4, 5]
    assert agent.vf.net is None            # never fitted


def test_learn_nan_entropy_exit(gpu_available):
    """trpo_inksci.py:172-173: a NaN entropy ends the loop (the reference calls exit(-1)).  A NaN
    policy parameter after the first update makes every loss NaN on the next one."""
    from trpo_amd import TRPOAgent
    agent = TRPOAgent(4, 2, hidden=(64,), max_rows=4096)
    real_update = agent.engine.update
    n_upd = []

    def update(params):
        n_upd.append(1)
        if len(n_upd) == 2:
            th = agent.engine.get_flat()
            th[3] = np.nan
            agent.engine.set_flat(th)
        return real_update(params)
    agent.engine.update = update
    hist = agent.learn(max_iterations=10, n_envs=1, seed=3, log=None)
    assert len(hist) == 2 and hist[-1].get("nan_exit") and np.isnan(hist[-1]["entropy"])


def test_learn_two_ranks_share_gpu(gpu_available):
    """learn() as two ranks on one GPU (TRPOAgent.set_ranks with the host transport): each rank rolls out
    half of the timestep budget with its own draws; after every iteration both ranks hold bitwise-identical
    policy and VF parameters, the episode count and mean reward are the concatenated rollouts', and
    iteration 0's update equals one engine's update of the concatenated rollouts at 1e-5
    (tools/mrank_learn.py; trpo_inksci.py:89-158)."""
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "tools", "mrank_learn.py"),
           "--host-allreduce", "--iters", "3"]
    res = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stdout[-3000:] + res.stderr[-3000:]
    assert "MRANK LEARN OK" in res.stdout
    print(res.stdout.strip().splitlines()[-2])
