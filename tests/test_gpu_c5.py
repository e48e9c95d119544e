"""One GPU's share of BASELINE.json configs[4] (C5: 4M states, obs 376, 1024x1024 tanh MLP, 17 actions,
8 GPUs): 500k rows with n_global = 4M, the MFMA-bound shape where every hidden GEMM is 1024 wide on the
scaled f16 hi+lo split (trpo_inksci.py:38-70).

As at 8M (test_gpu_bigN.py) the oracle cannot evaluate the shard, so it is checked by properties of a
Hessian-vector product and a row slice the oracle does evaluate:

* symmetry    u.Hv = v.Hu (relative to |u||Hv|, 1e-5); v.Hv > 0
* linearity   H(2u - 3v) = 2Hu - 3Hv (norm-relative 1e-5)
* arithmetic  f16x3 (+ one-product low segment) vs the exact bf16x6 split on the same shard (1e-5)
* slice       1200 rows at n_global = 4M against the float64 oracle (SURVEY.md §8(d) bar)
"""
import numpy as np
import pytest

from conftest import assert_vec_close, rel_l2
from oracle import trpo_oracle as O

pytestmark = pytest.mark.gpu

N_GLOBAL = 4_000_000
N_RANK = N_GLOBAL // 8
SPEC = O.PolicySpec(376, [1024, 1024], 17)
REL = 1e-5


@pytest.fixture(scope="module")
def shard():
    rng = np.random.default_rng(7)
    X = rng.standard_normal((N_RANK, SPEC.obs_dim), dtype=np.float32)
    actions = rng.integers(0, SPEC.n_actions, N_RANK, dtype=np.int64)
    theta = O.init_theta(SPEC, np.random.RandomState(8)).astype(np.float32)
    u = np.random.RandomState(9).standard_normal(SPEC.n_params).astype(np.float32)
    v = np.random.RandomState(10).standard_normal(SPEC.n_params).astype(np.float32)
    return {"X": X, "actions": actions, "theta": theta, "u": u, "v": v}


def _engine(b, rows):
    from trpo_amd import Engine
    e = Engine(SPEC.obs_dim, SPEC.hidden, SPEC.n_actions, max_rows=rows)
    e.set_flat(b["theta"])
    X, a = b["X"][:rows], b["actions"][:rows]
    uniform = np.full((rows, SPEC.n_actions), 1.0 / SPEC.n_actions, np.float32)
    e.set_batch(X, a, None, uniform, n_global=N_GLOBAL)
    old = e.action_dist()                                  # steady state: pi_old = p(theta)
    e.set_batch(X, a, None, old, n_global=N_GLOBAL)
    return e


@pytest.fixture(scope="module")
def hv(shard):
    e = _engine(shard, N_RANK)
    u, v = shard["u"], shard["v"]
    out = {"Hu": e.fvp(u, 0.0), "Hv": e.fvp(v, 0.0), "H(2u-3v)": e.fvp(2.0 * u - 3.0 * v, 0.0)}
    e.close()
    return out


def test_c5_rank_shard_symmetry_and_curvature(gpu_available, shard, hv):
    u, v = shard["u"].astype(np.float64), shard["v"].astype(np.float64)
    Hu, Hv = hv["Hu"].astype(np.float64), hv["Hv"].astype(np.float64)
    asym = abs(u @ Hv - v @ Hu) / (np.linalg.norm(u) * np.linalg.norm(Hv))
    assert asym < REL, asym
    assert v @ Hv > 0 and u @ Hu > 0


def test_c5_rank_shard_linearity(gpu_available, hv):
    comb = 2.0 * hv["Hu"].astype(np.float64) - 3.0 * hv["Hv"].astype(np.float64)
    assert_vec_close(hv["H(2u-3v)"], comb, REL, "C5 shard: H(2u-3v) vs 2Hu-3Hv")


def test_c5_rank_shard_f16_split_vs_exact_bf16_split(gpu_available, shard, hv):
    from trpo_amd._lib import get_option, set_option
    saved = get_option("split_f16")
    set_option("split_f16", 0)
    try:
        e = _engine(shard, N_RANK)
        hv6 = e.fvp(shard["v"], 0.0)
        e.close()
    finally:
        set_option("split_f16", saved)
    print(f"C5 shard f16x3 vs bf16x6: rel L2 {rel_l2(hv['Hv'], hv6):.2e}")
    assert_vec_close(hv["Hv"], hv6, REL, "C5 shard: f16x3 vs bf16x6 Hv")


def test_c5_slice_at_n_global_4m_vs_oracle(gpu_available, shard):
    n = 1200
    e = _engine(shard, n)
    hv = e.fvp(shard["v"], 0.0)
    e.close()
    ref = O.fvp_undamped(shard["theta"].astype(np.float64), shard["X"][:n], shard["v"].astype(np.float64), SPEC,
                         n_global=N_GLOBAL)
    assert_vec_close(hv, ref, REL, "C5: Hv of a 1200-row slice at n_global = 4M")
