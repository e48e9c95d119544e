"""GPU parity of batched sampling and CartPole-v0 rollouts (rollout.hip via the C-ABI) against
fixtures from the reference's own rollout / cat_sample (tests/golden/rollout.npz) and the oracle
(oracle/cartpole_oracle.py).  Bars: sampled indices, actions, path starts and rewards exact;
float64 states to 1e-12 (gym's math.cos/sin vs the device's differ in the last ulp at most);
float32 action distributions to 1e-6 absolute (summation order of the policy forward)."""
import numpy as np
import pytest

from conftest import golden
from oracle import cartpole_oracle as C

pytestmark = pytest.mark.gpu
D = golden("rollout.npz")


def engine_c1(theta, max_rows=4096):
    from trpo_amd import Engine
    e = Engine(4, [64], 2, max_rows=max_rows)
    e.set_flat(theta)
    return e


def test_cat_sample_bit_exact(gpu_available):
    from trpo_amd.engine import cat_sample_device
    assert np.array_equal(cat_sample_device(D["cat_prob"], D["cat_r"]), D["cat_out"])


def test_cartpole_step_vs_oracle(gpu_available):
    from trpo_amd.engine import cartpole_step_device
    rng = np.random.RandomState(0)
    s = rng.uniform(-0.3, 0.3, (5000, 4)) * np.array([8, 3, 1, 3])
    a = rng.randint(0, 2, 5000)
    so, rw, dn = cartpole_step_device(s, a)
    ref = [C.CartPoleV0.dynamics(s[i], a[i]) for i in range(len(a))]
    ref_s = np.array([r[0] for r in ref])
    ref_d = np.array([r[1] for r in ref])
    assert np.allclose(so, ref_s, rtol=1e-13, atol=1e-15)
    assert np.array_equal(dn, ref_d) and (rw == 1.0).all()


def test_act_matches_policy_and_cat_sample(gpu_available):
    theta = D["a_theta"]
    e = engine_c1(theta)
    rng = np.random.RandomState(1)
    states = rng.uniform(-0.2, 0.2, (3000, 4)).astype(np.float32)
    r = rng.random_sample(3000)
    acts, dists = e.act(states, r, train=True)
    ref = C.policy_dist32(theta, states, [4, 64, 2])
    assert np.max(np.abs(dists - ref)) < 1e-6
    assert np.array_equal(acts, C.cat_sample(dists, r))           # sampling on the device's own dists
    acts0, _ = e.act(states, None, train=False)
    assert np.array_equal(acts0, np.argmax(dists, axis=1))
    e.close()


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_single_env_rollout_vs_reference_rollout(gpu_available, tag):
    """n_envs = 1 with the reference's recorded draws reproduces utils.rollout's paths."""
    theta = D[tag + "_theta"]
    nt = int(D[tag + "_n_timesteps"])
    e = engine_c1(theta)
    n_ref = len(D[tag + "_rewards"])
    ru = D[tag + "_reset_uniforms"].reshape(-1, 4)
    ru = np.concatenate([ru, np.zeros((nt, 4))])[:max(nt, len(ru))]      # >= budget episodes
    au = np.concatenate([D[tag + "_act_uniforms"], np.zeros(nt + 200)])[:nt + 199]
    n, paths = e.rollout_cartpole(n_envs=1, n_timesteps=nt, max_pathlength=1000, train=bool(D[tag + "_train"]),
                                  reset_uniforms=ru.reshape(1, -1, 4), action_uniforms=au,
                                  max_episodes_per_env=len(ru))
    assert n == n_ref and paths == int(D[tag + "_starts"].sum())
    out = e.rollout_fetch()
    for k in ("actions", "rewards", "starts"):
        assert np.array_equal(out[k], D[tag + "_" + k]), k
    assert np.allclose(out["obs"], D[tag + "_obs"], rtol=0, atol=1e-12)
    assert np.max(np.abs(out["action_dists"] - D[tag + "_action_dists"])) < 1e-6
    e.close()


def test_many_env_rollout_replays_and_is_deterministic(gpu_available):
    theta = D["a_theta"]
    e = engine_c1(theta, max_rows=1 << 16)
    n, paths = e.rollout_cartpole(n_envs=256, n_timesteps=20000, seed=7)
    out = e.rollout_fetch()
    n2, paths2 = e.rollout_cartpole(n_envs=256, n_timesteps=20000, seed=7)
    out2 = e.rollout_fetch()
    assert (n, paths) == (n2, paths2)
    for k in out:
        assert np.array_equal(out[k], out2[k]), k
    assert n >= 20000 and out["starts"][0] == 1 and out["starts"].sum() == paths
    # replay every transition on the host
    starts = out["starts"].astype(bool)
    ends = np.r_[starts[1:], True]
    assert np.array_equal(out["actions"], C.cat_sample(out["action_dists"], out["uniforms"]))
    assert np.max(np.abs(out["action_dists"] - C.policy_dist32(theta, out["obs"], [4, 64, 2]))) < 1e-6
    assert (np.abs(out["obs"][starts]) <= 0.05).all()
    lens = np.diff(np.r_[np.flatnonzero(starts), n])
    assert lens.max() <= 200
    for i in np.flatnonzero(~ends)[:5000]:
        s1, d = C.CartPoleV0.dynamics(out["obs"][i], out["actions"][i])
        assert not d
        assert np.allclose(s1, out["obs"][i + 1], rtol=1e-13, atol=1e-15)
    last = np.flatnonzero(ends)
    for i in last[:500]:
        _, d = C.CartPoleV0.dynamics(out["obs"][i], out["actions"][i])
        length = i - np.flatnonzero(starts[:i + 1])[-1] + 1
        assert d or length == 200
    e.close()


def test_rollout_to_batch_feeds_the_update(gpu_available):
    """The device-resident rollout -> feed gives the same update as fetching it to the host and
    calling set_batch / set_rewards."""
    from trpo_amd import UpdateParams
    theta = D["a_theta"]
    e = engine_c1(theta, max_rows=1 << 15)
    n, _ = e.rollout_cartpole(n_envs=64, n_timesteps=10000, seed=3)
    out = e.rollout_fetch()
    e.rollout_to_batch()
    st1 = e.update(UpdateParams(compute_advantages=True, residual_tol=0.0))
    th1 = e.get_flat()
    f = engine_c1(theta, max_rows=1 << 15)
    f.set_batch(out["obs"].astype(np.float32), out["actions"], None, out["action_dists"])
    f.set_rewards(out["rewards"], out["starts"])
    st2 = f.update(UpdateParams(compute_advantages=True, residual_tol=0.0))
    assert np.array_equal(th1, f.get_flat())
    assert st1 == st2
    e.close()
    f.close()
