"""Degenerate inputs the reference runs through numpy's IEEE semantics (no guards):

* CG with p.z = 0 (utils.py:191): ``rdotr / p.dot(z)`` is inf (or nan for 0/0) and the NaNs
  propagate through the remaining iterations -- the device CG must give the same non-finite
  pattern, not stop or clamp.
* A zero-advantage batch: g = 0, so CG runs 0/0 = nan, shs = nan, lm = np.sqrt(nan)
  (trpo_inksci.py:148-149), the line search rejects every step (nan ratios) and the update keeps
  theta (utils.py:182) -- bitwise, with k = -1 and cg_iters = 10, as the oracle gives.
"""
import numpy as np
import pytest

from oracle import trpo_oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("case", ["zero_operator", "zero_rhs"])
def test_cg_p_dot_z_zero(gpu_available, dt, case):
    from trpo_amd.engine import cg_callback
    n = 257
    b = np.zeros(n, dt) if case == "zero_rhs" else np.random.RandomState(0).standard_normal(n).astype(dt)

    def f(p):
        return np.zeros_like(p)

    x, it = cg_callback(f, b, 10, 1e-10)
    xr, itr = O.conjugate_gradient(f, b.copy(), 10, 1e-10)
    assert it == itr == 10
    assert np.array_equal(np.isnan(x), np.isnan(xr)) and np.array_equal(np.isinf(x), np.isinf(xr))
    assert not np.isfinite(x).any()


@pytest.mark.parametrize("dims", [(11, [64, 64], 3), (128, [256, 256], 18)])
def test_zero_advantage_update_keeps_theta(gpu_available, dims):
    from trpo_amd import Engine, UpdateParams
    spec = O.PolicySpec(*dims)
    n = 3000
    d = O.synthetic_batch(spec, n, seed=5)
    adv = np.zeros(n)
    ref = O.trpo_update(d["theta"], O.Batch(d["X"], d["actions"], adv, d["old_dist"]), spec, dtype=np.float32)
    assert ref.k == -1 and np.isnan(ref.shs) and ref.cg_iters == 10
    e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
    e.set_flat(d["theta"])
    e.set_batch(d["X"], d["actions"], adv, d["old_dist"])
    st = e.update(UpdateParams())
    th = e.get_flat()
    e.close()
    assert st["k"] == -1 and st["cg_iters"] == 10, st
    assert np.isnan(st["shs"]), st
    assert np.array_equal(th, d["theta"].astype(np.float32))
    assert np.array_equal(th, ref.theta_new)


def test_negative_shs_update_keeps_theta(gpu_available):
    """A damping that makes the operator indefinite: shs < 0, lm = np.sqrt(<0) = nan, no step."""
    from trpo_amd import Engine, UpdateParams
    spec = O.PolicySpec(11, [64, 64], 3)
    n = 3000
    d = O.synthetic_batch(spec, n, seed=6)
    ref = O.trpo_update(d["theta"], O.Batch(d["X"], d["actions"], d["advant"], d["old_dist"]), spec,
                        dtype=np.float32, cg_damping=-50.0)
    assert ref.shs < 0 and ref.k == -1
    e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
    e.set_flat(d["theta"])
    e.set_batch(d["X"], d["actions"], d["advant"], d["old_dist"])
    st = e.update(UpdateParams(cg_damping=-50.0))
    th = e.get_flat()
    e.close()
    assert st["shs"] < 0 and np.isnan(st["lm"]) and st["k"] == -1, st
    assert np.array_equal(th, ref.theta_new)
