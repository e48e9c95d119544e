"""The communicator paths of the engine on one GPU, and the standalone standardisation entry.

* RCCL at world = 1: trpo_comm_init always creates a communicator, so every all-reduce of the
  update (FVP / gradient [P] f32, loss and standardisation sums f64) goes through ncclAllReduce.
  A one-rank sum is the identity, so the update must be bitwise identical to an engine without a
  communicator -- eager and replayed from the captured hipGraph (RCCL calls inside it).
* trpo_standardize (trpo_inksci.py:115-117; SURVEY.md §8(b) `standardize(adv, n)`) against the
  oracle at rtol 1e-11, host and device memory, engine-free and on an engine.
"""
import numpy as np
import pytest

from oracle import trpo_oracle as O

pytestmark = pytest.mark.gpu


def _engine(spec, d, comm=False):
    from trpo_amd import Engine
    e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=d["X"].shape[0])
    if comm:
        e.comm_init(Engine.comm_unique_id(), 0, 1)
    e.set_flat(d["theta"])
    e.set_batch(d["X"], d["actions"], None, d["old_dist"])
    e.set_rewards(d["rewards"], d["starts"])
    return e


@pytest.mark.parametrize("dims", [((11, [64, 64], 3), 3000), ((128, [256, 256], 18), 4000)])
def test_rccl_world1_update_bitwise(gpu_available, dims):
    from trpo_amd import UpdateParams
    from trpo_amd._lib import get_option, set_option
    (obs, hidden, A), n = dims
    spec = O.PolicySpec(obs, hidden, A)
    d = O.synthetic_batch(spec, n, seed=7)
    prm = UpdateParams(residual_tol=0.0, compute_advantages=True)
    saved = get_option("graphs")
    try:
        set_option("graphs", 0)
        e0 = _engine(spec, d)
        st0 = e0.update(prm)
        th0 = e0.get_flat()
        e0.set_flat(d["theta"])
        g0 = e0.policy_grad()
        e0.close()
        e1 = _engine(spec, d, comm=True)
        runs = []
        for graphs in (0, 1, 1, 1, 1):       # eager; graphs: first-seen eager, capture, replay, replay
            set_option("graphs", graphs)
            e1.set_flat(d["theta"])
            st = e1.update(prm)
            runs.append((st, e1.get_flat()))
        e1.set_flat(d["theta"])
        g1 = e1.policy_grad()
        e1.close()
    finally:
        set_option("graphs", saved)
    assert np.array_equal(g1, g0)
    for i, (st, th) in enumerate(runs):
        assert np.array_equal(th, th0), f"run {i}: theta differs from the no-communicator engine"
        assert st == st0, f"run {i}: {st} vs {st0}"


def test_vf_rccl_world1_fit_bitwise(gpu_available):
    from trpo_amd import Engine
    from trpo_amd.vf import VFNet
    rng = np.random.RandomState(0)
    n, F = 3000, 12
    feat = rng.standard_normal((n, F)).astype(np.float32)
    y = rng.standard_normal(n)
    out = []
    for comm in (False, True):
        vf = VFNet(F, max_rows=n)
        vf.set_params(np.random.RandomState(1).uniform(-0.2, 0.2, vf.num_params).astype(np.float32))
        vf.reset_optimizer()
        if comm:
            vf.comm_init(Engine.comm_unique_id(), 0, 1)
        vf.set_feature_matrix(feat)
        vf.set_targets(y)
        vf.fit(50)
        out.append(vf.get_params())
        vf.close()
    assert np.array_equal(out[0], out[1])


@pytest.mark.parametrize("n", [1, 2, 999, 200_000])
def test_standardize_engine_free(gpu_available, n):
    from trpo_amd.engine import standardize_device
    rng = np.random.RandomState(n)
    adv = rng.standard_normal(n) * 3.0 + 1.5
    ref = O.standardize(adv.copy())
    a = adv.copy()
    a32 = np.empty(n, np.float32)
    out = standardize_device(a, adv32_out=a32)
    assert out is a
    assert np.allclose(a, ref, rtol=1e-11, atol=1e-11)
    assert np.array_equal(a32, a.astype(np.float32))


_DEVICE_SCRIPT = r"""
import sys, numpy as np, torch
torch.cuda.init()                      # torch's HIP runtime first (engine.py: rollout_fetch note)
sys.path.insert(0, sys.argv[1])
from trpo_amd import Engine
from oracle import trpo_oracle as O
n = 50_000
adv = np.random.RandomState(3).gamma(2.0, 2.0, n)
ref = O.standardize(adv.copy())
t = torch.from_numpy(adv.copy()).cuda()
t32 = torch.empty(n, dtype=torch.float32, device="cuda")
e = Engine(4, [8], 2, max_rows=16)
e.standardize(t, adv32_out=t32)
e.synchronize()
assert np.allclose(t.cpu().numpy(), ref, rtol=1e-11, atol=1e-11)
assert np.array_equal(t32.cpu().numpy(), t.cpu().numpy().astype(np.float32))
print("DEVICE STANDARDIZE OK")
"""


def test_standardize_device_tensor(gpu_available):
    """mem = TRPO_MEM_DEVICE on torch-ROCm tensors (own process: torch initialises HIP first)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = subprocess.run([sys.executable, "-c", _DEVICE_SCRIPT, root], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0 and "DEVICE STANDARDIZE OK" in res.stdout, res.stdout[-2000:] + res.stderr[-2000:]


def test_standardize_engine_constant(gpu_available):
    """Constant advantages: std = 0 and the 1e-8 keeps the result finite (zeros), as numpy does."""
    from trpo_amd import Engine
    e = Engine(4, [8], 2, max_rows=16)
    c = np.full(10, 2.5)
    e.standardize(c)
    assert np.array_equal(c, O.standardize(np.full(10, 2.5)))
    e.close()


def test_standardize_matches_compute_advantages(gpu_available):
    """The standalone entry and the fused advantages path run the same sums: bitwise equal."""
    from trpo_amd import Engine
    spec = O.PolicySpec(11, [64, 64], 3)
    d = O.synthetic_batch(spec, 5000, seed=9)
    e = Engine(11, [64, 64], 3, max_rows=5000)
    e.set_flat(d["theta"])
    e.set_batch(d["X"], d["actions"], None, d["old_dist"])
    e.set_rewards(d["rewards"], d["starts"])
    ret, adv = e.compute_advantages(0.95)
    a = ret.copy()
    e.standardize(a)
    assert np.array_equal(a, adv)
    e.close()
