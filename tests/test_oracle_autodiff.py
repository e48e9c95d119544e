"""Pins the closed-form R-op oracle against reverse-over-reverse autodiff of the
reference graph, and checks the sharding algebra of the multi-GPU path. CPU only."""
import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from conftest import rel_l2
from oracle import trpo_oracle as O
from oracle.tf_graph_torch import TFGraph

SPECS = [O.PolicySpec(4, [64], 2), O.PolicySpec(11, [64, 64], 3), O.PolicySpec(128, [64, 64], 18),
         O.PolicySpec(9, [20, 13, 7], 5), O.PolicySpec(6, [], 4)]


@pytest.mark.parametrize("spec", SPECS, ids=lambda s: f"{s.obs_dim}-{list(s.hidden)}-{s.n_actions}")
@pytest.mark.parametrize("steady", [True, False])
def test_rop_matches_autodiff(spec, steady):
    d = O.synthetic_batch(spec, 257, seed=5, steady_state=steady, perturb=0.2)
    th = d["theta"].astype(np.float64)
    G = TFGraph(spec, d["X"], d["actions"], d["advant"], d["old_dist"])
    v = np.random.RandomState(6).standard_normal(spec.n_params)
    assert rel_l2(O.fvp_undamped(th, d["X"], v, spec), G.fvp(th, v)) < 1e-13
    assert rel_l2(O.policy_grad(th, d["X"], d["actions"], d["advant"], d["old_dist"], spec), G.pg(th)) < 1e-13
    np.testing.assert_allclose(O.losses(th, d["X"], d["actions"], d["advant"], d["old_dist"], spec),
                               G.losses(th), rtol=1e-12, atol=1e-15)


def test_eps_terms_matter():
    """The eps-exact Hessian differs from the plain Gauss-Newton Fisher by more than the
    1e-5 parity bar, so dropping the O(eps) deltas would be caught."""
    spec = O.PolicySpec(128, [64, 64], 18)
    d = O.synthetic_batch(spec, 500, seed=9)
    th = d["theta"].astype(np.float64)
    v = np.random.RandomState(1).standard_normal(spec.n_params)
    exact = O.fvp_undamped(th, d["X"], v, spec)
    saved = O.EPS
    try:
        O.EPS = 0.0
        no_eps = O.fvp_undamped(th, d["X"], v, spec)
    finally:
        O.EPS = saved
    assert rel_l2(no_eps, exact) > 2e-5


@pytest.mark.parametrize("shards", [2, 4, 8])
def test_shard_partials_sum_to_full(shards):
    """Fake multi-GPU: per-shard partials scaled by 1/N_global, summed (all-reduce)."""
    spec = O.PolicySpec(11, [64, 64], 3)
    n = 1000
    d = O.synthetic_batch(spec, n, seed=3)
    th = d["theta"].astype(np.float64)
    v = np.random.RandomState(4).standard_normal(spec.n_params)
    cuts = np.linspace(0, n, shards + 1).astype(int)
    hv = sum(O.fvp_undamped(th, d["X"][a:b], v, spec, n_global=n) for a, b in zip(cuts[:-1], cuts[1:]))
    g = sum(O.policy_grad(th, d["X"][a:b], d["actions"][a:b], d["advant"][a:b], d["old_dist"][a:b], spec,
                          n_global=n) for a, b in zip(cuts[:-1], cuts[1:]))
    ls = sum(O.losses(th, d["X"][a:b], d["actions"][a:b], d["advant"][a:b], d["old_dist"][a:b], spec,
                      n_global=n) for a, b in zip(cuts[:-1], cuts[1:]))
    assert rel_l2(hv, O.fvp_undamped(th, d["X"], v, spec)) < 1e-13
    assert rel_l2(g, O.policy_grad(th, d["X"], d["actions"], d["advant"], d["old_dist"], spec)) < 1e-13
    np.testing.assert_allclose(ls, O.losses(th, d["X"], d["actions"], d["advant"], d["old_dist"], spec),
                               rtol=1e-12, atol=1e-15)


@settings(max_examples=25, deadline=None)
@given(n=st.integers(2, 40), seed=st.integers(0, 10_000), iters=st.integers(1, 40))
def test_cg_solves_spd(n, seed, iters):
    rng = np.random.RandomState(seed)
    M = rng.standard_normal((n, n))
    A = M @ M.T + n * np.eye(n)
    b = rng.standard_normal(n)
    x, it = O.conjugate_gradient(lambda p: A @ p, b, max(iters, n + 5), 1e-24)
    assert it <= max(iters, n + 5)
    np.testing.assert_allclose(A @ x, b, rtol=1e-6, atol=1e-8)


@settings(max_examples=40, deadline=None)
@given(n=st.integers(1, 300), seed=st.integers(0, 10_000), p_start=st.floats(0.0, 0.3))
def test_segmented_discount_equals_per_episode(n, seed, p_start):
    rng = np.random.RandomState(seed)
    r = rng.uniform(0, 1, n)
    starts = rng.uniform(size=n) < p_start
    starts[0] = True
    y = O.discount_segmented(r, starts, 0.95)
    idx = list(np.flatnonzero(starts)) + [n]
    for a, b in zip(idx[:-1], idx[1:]):
        np.testing.assert_array_equal(y[a:b], O.discount(r[a:b], 0.95))


def test_standardize_population_std():
    x = np.arange(10.0)
    y = O.standardize(x)
    assert abs(y.mean()) < 1e-15
    assert y.std() == pytest.approx(1.0 / (1.0 + 1e-8 / x.std()), rel=1e-12)
