"""The sampling / CartPole oracle (oracle/cartpole_oracle.py) against fixtures recorded from the
reference's own rollout (utils.py:18-45) and cat_sample (utils.py:95-105). CPU only."""
import numpy as np
import pytest

from conftest import golden
from oracle import cartpole_oracle as C

D = golden("rollout.npz")


def test_cat_sample_matches_reference_fixture():
    assert np.array_equal(C.cat_sample(D["cat_prob"], D["cat_r"]), D["cat_out"])
    # rows whose float32 cumsum never exceeds r fall back to 0, as the reference's zeros-init does
    assert (D["cat_out"][:10] == 0).all()


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_batched_rollout_restatement_equals_reference_rollout(tag):
    """rollout_envs with one environment and the reference's recorded draws reproduces the
    reference's utils.rollout bit for bit (obs, actions, dists, rewards, path starts)."""
    n = len(D[tag + "_rewards"])
    ru = D[tag + "_reset_uniforms"].reshape(1, -1, 4)
    au = D[tag + "_act_uniforms"].reshape(1, -1)
    train = bool(D[tag + "_train"])
    out = C.rollout_envs(D[tag + "_theta"], [4, 64, 2], 1, int(D[tag + "_n_timesteps"]), ru,
                         np.pad(au, ((0, 0), (0, 400))), train=train)
    assert len(out["rewards"]) == n
    for k in ("obs", "actions", "action_dists", "rewards", "starts"):
        assert np.array_equal(out[k], D[tag + "_" + k]), k


def test_cartpole_dynamics_terminates_and_time_limit():
    env = C.CartPoleV0(seed=0)
    env.reset()
    steps = 0
    done = False
    while not done:
        _, r, done, _ = env.step(1)      # always push right: falls quickly
        steps += 1
        assert r == 1.0
    assert steps < 200
    s, d = C.CartPoleV0.dynamics((0.0, 0.0, 0.0, 0.0), 0)     # push left from rest
    assert s[0] == 0.0 and s[1] < 0 and s[2] == 0.0 and s[3] > 0 and not d
