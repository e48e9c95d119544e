"""The synthetic full-size batches of the float64 whole-update tests (test_gpu_bigN.py: C4, 8M states;
test_gpu_full_size.py: C2 / C3 / C5), shared with their float64 child process (tests/bign_truth.py), which
regenerates them from the same seeds instead of receiving gigabytes of inputs."""
import numpy as np

from oracle import trpo_oracle as O

N = 8_000_000
SPEC = O.PolicySpec(128, [256, 256], 18)
PATH_LEN = 200   # CartPole-v0 path length cap: an episode start every 200 states
CONFIGS = {"c4": (SPEC, N), "c3": (O.PolicySpec(128, [64, 64], 18), 1_000_000),
           "c2": (O.PolicySpec(11, [64, 64], 3), 50_000), "c5": (O.PolicySpec(376, [1024, 1024], 17), 4_000_000)}


def make_batch(n=N, spec=SPEC):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((n, spec.obs_dim), dtype=np.float32)
    actions = rng.integers(0, spec.n_actions, n, dtype=np.int64)
    theta = O.init_theta(spec, np.random.RandomState(1)).astype(np.float32)
    u = np.random.RandomState(2).standard_normal(spec.n_params).astype(np.float32)
    v = np.random.RandomState(3).standard_normal(spec.n_params).astype(np.float32)
    return {"X": X, "actions": actions, "theta": theta, "u": u, "v": v}


def make_rewards(n=N):
    rng = np.random.default_rng(5)
    rewards = rng.random(n)
    starts = (np.arange(n) % PATH_LEN == 0).astype(np.uint8)
    return rewards, starts
