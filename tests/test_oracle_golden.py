"""The CPU oracle against the golden vectors recorded from the reference's own
numpy functions (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from conftest import golden, update_fixtures, spec_of, rel_l2
from oracle import trpo_oracle as O
from oracle.ref_loader import reference_available


def test_discount_matches_reference_bitwise():
    d = golden("discount.npz")
    keys = sorted(k[:-2] for k in d.files if k.endswith("_x"))
    assert len(keys) == 16
    for k in keys:
        gamma = float(k.split("_")[0][1:])
        y = O.discount(d[k + "_x"], gamma)
        np.testing.assert_array_equal(y, d[k + "_y"], err_msg=k)   # lfilter's recurrence, same rounding


def test_cg_matches_reference():
    d = golden("cg.npz")
    for case in d["cases"]:
        base = str(d[case + "_base"])
        A, b = d[base + "_A"], d[base + "_b"]
        x, it = O.conjugate_gradient(lambda p: A @ p, b.copy(), int(d[case + "_maxit"]), float(d[case + "_tol"]))
        assert it == int(d[case + "_iters"]), case
        np.testing.assert_array_equal(x, d[case + "_x"], err_msg=case)
        assert x.dtype == b.dtype


def test_linesearch_matches_reference():
    d = golden("linesearch.npz")
    for case in d["cases"]:
        c = d[case + "_c"]
        f = lambda x: np.float32(0.5 * np.sum((np.asarray(x, np.float32) - c) ** 2, dtype=np.float32))
        res, k = O.linesearch(f, d[case + "_x"], d[case + "_fullstep"], float(d[case + "_rate"]))
        assert k == int(d[case + "_k"]), case
        np.testing.assert_array_equal(np.asarray(res, np.float64), d[case + "_result"], err_msg=case)
    assert {int(d[c + "_k"]) for c in d["cases"]} >= {-1, 0, 1, 3}   # all branches covered


def test_explained_variance():
    d = golden("explained_variance.npz")
    assert O.explained_variance(d["ypred"], d["y"]) == pytest.approx(float(d["ev"]), rel=1e-15)
    assert np.isnan(O.explained_variance(np.zeros(10), d["yconst"]))


@pytest.mark.parametrize("name", update_fixtures())
def test_update_tuple(name):
    d = golden(name)
    spec = spec_of(d)
    th = d["theta"].astype(np.float64)
    X, a, adv, old = d["X"], d["actions"], d["advant"], d["old_dist"]
    # inputs: discount + standardisation reproduce the recorded advantages
    ret = O.discount_segmented(d["rewards"], d["starts"], 0.95)
    np.testing.assert_allclose(ret, d["returns"], rtol=1e-14)
    np.testing.assert_allclose(O.standardize(ret), adv, rtol=1e-12, atol=1e-12)
    # graph outputs
    assert rel_l2(O.fvp_undamped(th, X, d["v"], spec), d["hv"]) < 1e-12
    assert rel_l2(O.policy_grad(th, X, a, adv, old, spec), d["g"]) < 1e-12
    np.testing.assert_allclose(O.losses(th, X, a, adv, old, spec), d["losses_before"], rtol=1e-10, atol=1e-14)
    # the whole update block
    r = O.trpo_update(th, O.Batch(X, a, adv, old), spec, np.float64, 10, float(d["residual_tol"]),
                      float(d["max_kl"]))
    assert r.cg_iters == int(d["cg_iters"])
    assert r.k == int(d["k"])
    assert r.reverted == bool(d["reverted"])
    assert rel_l2(r.stepdir, d["stepdir"]) < 1e-10
    assert r.shs == pytest.approx(float(d["shs"]), rel=1e-10)
    assert r.lm == pytest.approx(float(d["lm"]), rel=1e-10)
    assert rel_l2(r.theta_new, d["theta_new"]) < 1e-10
    np.testing.assert_allclose(r.losses_after, d["losses_after"], rtol=1e-9, atol=1e-14)


@pytest.mark.skipif(not reference_available(), reason="/root/reference not mounted (GPU box)")
def test_oracle_against_live_reference_utils():
    """Where the reference is mounted, re-run its numpy functions on fresh inputs."""
    from oracle.ref_loader import load_reference_utils
    U = load_reference_utils()
    rng = np.random.RandomState(123)
    for n in (1, 3, 57, 400):
        x = rng.uniform(-1, 1, n)
        np.testing.assert_array_equal(O.discount(x, 0.97), U.discount(x, 0.97))
    M = rng.standard_normal((30, 30))
    A = M @ M.T + 30 * np.eye(30)
    b = rng.standard_normal(30).astype(np.float32)
    A32 = A.astype(np.float32)
    x1, _ = O.conjugate_gradient(lambda p: A32 @ p, b.copy(), 10, 1e-10)
    np.testing.assert_array_equal(x1, U.conjugate_gradient(lambda p: A32 @ p, b.copy(), 10, 1e-10))
