"""The oracle follows numpy's IEEE semantics on degenerate inputs, as the reference does
(utils.py:191 divides by p.z unguarded; trpo_inksci.py:149 takes np.sqrt of shs)."""
import numpy as np

from oracle import trpo_oracle as O


def test_cg_zero_operator_gives_nan():
    x, it = O.conjugate_gradient(lambda p: np.zeros_like(p), np.ones(5, np.float32), 10, 1e-10)
    assert it == 10 and np.isnan(x).all()


def test_zero_advantage_update_keeps_theta():
    spec = O.PolicySpec(5, [8], 3)
    d = O.synthetic_batch(spec, 400, seed=1)
    r = O.trpo_update(d["theta"], O.Batch(d["X"], d["actions"], np.zeros(400), d["old_dist"]), spec,
                      dtype=np.float32)
    assert r.k == -1 and np.isnan(r.shs) and np.isnan(r.lm) and not r.reverted
    assert np.array_equal(r.theta_new, d["theta"].astype(np.float32))


def test_negative_shs_is_nan_not_an_error():
    # a non-positive-definite operator: shs < 0, np.sqrt -> nan, every step rejected
    spec = O.PolicySpec(5, [8], 3)
    d = O.synthetic_batch(spec, 400, seed=2)
    r = O.trpo_update(d["theta"], O.Batch(d["X"], d["actions"], d["advant"], d["old_dist"]), spec,
                      dtype=np.float64, cg_damping=-50.0)
    assert r.shs < 0 and np.isnan(r.lm) and r.k == -1
