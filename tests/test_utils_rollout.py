"""utils.rollout keeps the reference's path bookkeeping (utils.py:18-45), checked with a scripted
env whose episode lengths are chosen by the test: paths that end with ``done`` are kept, an episode
cut at max_pathlength is dropped and the count advances by the previous path's length, and a cut
episode before any kept path raises (the reference reads an unbound ``path``)."""
import numpy as np
import pytest

from trpo_amd import utils


class ScriptedEnv:
    """Episode i lasts lengths[i] steps (done on its last step); observations count steps."""

    def __init__(self, lengths):
        self.lengths = list(lengths)
        self.ep = -1
        self.t = 0

    def reset(self):
        self.ep += 1
        self.t = 0
        return np.zeros(2, np.float32)

    def step(self, action):
        self.t += 1
        return np.full(2, self.t, np.float32), 1.0, self.t >= self.lengths[self.ep], {}


class ConstAgent:
    def __init__(self):
        self.prev_action = np.zeros((1, 2), np.float32)

    def act(self, ob):
        return 0, np.array([[0.5, 0.5]], np.float32), ob


def test_done_paths_kept():
    paths = utils.rollout(ScriptedEnv([3, 4, 5]), ConstAgent(), 10, 7)
    assert [len(p["rewards"]) for p in paths] == [3, 4]


def test_cut_episode_dropped_and_previous_length_counted():
    # episode 2 runs into max_pathlength = 6 without done: dropped, and the count advances by the
    # length of the last kept path (3), so a 4th episode is collected: 3 + 3 + 5 >= 10
    env = ScriptedEnv([3, 50, 5, 2])
    paths = utils.rollout(env, ConstAgent(), 6, 10)
    assert [len(p["rewards"]) for p in paths] == [3, 5]
    assert env.ep == 2


def test_cut_first_episode_raises_like_reference():
    with pytest.raises(UnboundLocalError):
        utils.rollout(ScriptedEnv([50]), ConstAgent(), 6, 10)
