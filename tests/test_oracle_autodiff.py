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


@pytest.mark.parametrize("chunk", [97, 1000])
def test_chunked_f64_graph_matches_oracle(chunk):
    """oracle/chunked_f64.py (the float64 truth of the 8M-state GPU tests) against the numpy oracle: losses,
    pg, FVP and a whole update, the batch cut into row chunks summed with 1/N_global; advantages from the
    equal-path lfilter form against the oracle's segmented recurrence."""
    from oracle.chunked_f64 import ChunkedGraph, advantages_equal_paths
    spec = O.PolicySpec(11, [32, 16], 5)
    n = 600
    d = O.synthetic_batch(spec, n, seed=11, episode_len=200, steady_state=False, perturb=0.1)
    adv = advantages_equal_paths(d["rewards"], 200)
    np.testing.assert_allclose(adv, d["advant"], rtol=1e-12, atol=1e-12)
    th = d["theta"].astype(np.float64)
    G = ChunkedGraph(spec, d["X"], d["actions"], adv, d["old_dist"], chunk=chunk)
    v = np.random.RandomState(12).standard_normal(spec.n_params)
    assert rel_l2(G.fvp(th, v), O.fvp_undamped(th, d["X"], v, spec)) < 1e-13
    assert rel_l2(G.pg(th), O.policy_grad(th, d["X"], d["actions"], adv, d["old_dist"], spec)) < 1e-13
    np.testing.assert_allclose(G.losses(th), O.losses(th, d["X"], d["actions"], adv, d["old_dist"], spec),
                               rtol=1e-12, atol=1e-15)
    ref = O.trpo_update(th, O.Batch(d["X"], d["actions"], adv, d["old_dist"]), spec, residual_tol=0.0)
    got = G.update(th, residual_tol=0.0)
    assert got["k"] == ref.k and got["cg_iters"] == ref.cg_iters and got["reverted"] == ref.reverted
    for key, r in (("g", ref.g), ("stepdir", ref.stepdir), ("fullstep", ref.fullstep), ("theta", ref.theta_new)):
        assert rel_l2(got[key], r) < 1e-11, key
    assert got["shs"] == pytest.approx(ref.shs, rel=1e-11)


def test_chunked_float32_graph_near_oracle():
    """The float32 mode of the chunked graph (the reference-arithmetic floor of the 8M tests) is the float64
    graph to float32 rounding."""
    import torch
    from oracle.chunked_f64 import ChunkedGraph
    spec = O.PolicySpec(11, [32, 16], 5)
    d = O.synthetic_batch(spec, 600, seed=13)
    th = d["theta"].astype(np.float64)
    G32 = ChunkedGraph(spec, d["X"], d["actions"], d["advant"], d["old_dist"], chunk=128, dtype=torch.float32)
    G64 = ChunkedGraph(spec, d["X"], d["actions"], d["advant"], d["old_dist"], chunk=128)
    v = np.random.RandomState(14).standard_normal(spec.n_params)
    assert G32.pg(th).dtype == np.float32
    assert rel_l2(G32.pg(th), G64.pg(th)) < 1e-5
    assert rel_l2(G32.fvp(th, v), G64.fvp(th, v)) < 1e-5
    u32, u64 = G32.update(th, residual_tol=0.0), G64.update(th, residual_tol=0.0)
    assert u32["stepdir"].dtype == np.float32 and u32["k"] == u64["k"]
    assert rel_l2(u32["stepdir"], u64["stepdir"]) < 1e-4
