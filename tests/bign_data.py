"""The synthetic 8M-state C4 batch of test_gpu_bigN.py, shared with its float64 child process
(tests/bign_truth.py), which regenerates it from the same seeds instead of receiving 4 GB of inputs."""
import numpy as np

from oracle import trpo_oracle as O

N = 8_000_000
SPEC = O.PolicySpec(128, [256, 256], 18)
PATH_LEN = 200   # CartPole-v0 path length cap: an episode start every 200 states


def make_batch(n=N):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((n, SPEC.obs_dim), dtype=np.float32)
    actions = rng.integers(0, SPEC.n_actions, n, dtype=np.int64)
    theta = O.init_theta(SPEC, np.random.RandomState(1)).astype(np.float32)
    u = np.random.RandomState(2).standard_normal(SPEC.n_params).astype(np.float32)
    v = np.random.RandomState(3).standard_normal(SPEC.n_params).astype(np.float32)
    return {"X": X, "actions": actions, "theta": theta, "u": u, "v": v}


def make_rewards(n=N):
    rng = np.random.default_rng(5)
    rewards = rng.random(n)
    starts = (np.arange(n) % PATH_LEN == 0).astype(np.uint8)
    return rewards, starts
