"""Host-side logic of the product package (no GPU compute). CPU only."""
import numpy as np
import pytest

from oracle import trpo_oracle as O
from trpo_amd.agent import paths_to_batch, xavier_theta
from trpo_amd.dist import shard_bounds


def test_shard_bounds_even():
    assert shard_bounds(10, 1) == [(0, 10)]
    b = shard_bounds(10, 3)
    assert b[0][0] == 0 and b[-1][1] == 10
    assert all(lo <= hi for lo, hi in b)
    assert sum(hi - lo for lo, hi in b) == 10


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_shard_bounds_align_to_episodes(world):
    n = 2000
    starts = np.zeros(n, np.uint8)
    starts[::200] = 1
    starts[1234] = 1
    b = shard_bounds(n, world, starts)
    assert b[0][0] == 0 and b[-1][1] == n
    for lo, hi in b:
        assert lo == hi or starts[lo] == 1 or lo == n
    for (_, h0), (l1, _) in zip(b[:-1], b[1:]):
        assert h0 == l1


def test_xavier_layout_matches_var_list_order():
    th = xavier_theta(4, [64], 2)
    spec = O.PolicySpec(4, [64], 2)
    assert th.shape == (spec.n_params,) and th.dtype == np.float32
    (W1, b1), (W2, b2) = O.unflatten(th, spec)
    assert np.all(b1 == 0) and np.all(b2 == 0)
    assert np.abs(W1).max() <= np.sqrt(6 / 68) and np.abs(W2).max() <= np.sqrt(6 / 66)


def test_paths_to_batch_concatenates_and_marks_starts():
    paths = [{"obs": np.ones((3, 4)), "action_dists": np.full((3, 2), .5), "rewards": np.ones(3),
              "actions": np.array([0, 1, 0])},
             {"obs": np.zeros((2, 4)), "action_dists": np.full((2, 2), .5), "rewards": np.ones(2),
              "actions": np.array([1, 1]), "baseline": np.array([.5, .25])}]
    b = paths_to_batch(paths)
    assert b["state"].shape == (5, 4) and b["action_dist"].shape == (5, 2)
    np.testing.assert_array_equal(b["starts"], [1, 0, 0, 1, 0])
    np.testing.assert_array_equal(b["baseline"], [0, 0, 0, .5, .25])


class _CommRecorder:
    def __init__(self):
        self.calls = []

    def comm_set_host_allreduce(self, fn, rank, world):
        self.calls.append((rank, world))


def test_set_ranks_after_vf_exists_hooks_the_existing_net():
    """set_ranks called once the VF net exists (after a fit) must sum that net's gradient too,
    not only a net created later."""
    from types import SimpleNamespace
    from trpo_amd.agent import TRPOAgent
    net = _CommRecorder()
    fake = SimpleNamespace(engine=_CommRecorder(), vf=SimpleNamespace(net=net, on_create=None))
    TRPOAgent.set_ranks(fake, 1, 2, group=None, host_allreduce=True)
    assert fake.engine.calls == [(1, 2)]
    assert net.calls == [(1, 2)]                 # the existing net, hooked at once
    later = _CommRecorder()
    fake.vf.on_create(later)                     # and any net created afterwards
    assert later.calls == [(1, 2)]


def test_rollout_seeds_never_collide_across_ranks():
    from trpo_amd.agent import rollout_seed
    seen = {rollout_seed(1, i, r) for r in range(8) for i in range(100_000)}
    assert len(seen) == 8 * 100_000
    assert rollout_seed(1, 5, 0) == 1 * 1000003 + 5        # rank 0 keeps the one-rank stream
