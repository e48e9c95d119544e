"""The whole update at the full sizes of BASELINE's other GPU configs against its float64 evaluation
(oracle/chunked_f64.py in a child process, tests/bign_truth.py): discount + standardise + pg + 10 CG + shs + line
search, trpo_inksci.py:102-158. C2 (50k states, obs 11, 64x64, 3 actions) and C3 (1M states, obs 128, 64x64,
18 actions) run the one-launch FVP on the scaled f16 hi+lo split (fused16.hip); C5 (4M states, obs 376, 1024x1024, 17 actions,
one GPU) the f16x3 split row GEMMs. C4 is tests/test_gpu_bigN.py."""
import os
import subprocess
import sys

import numpy as np
import pytest

from bign_data import CONFIGS, make_batch, make_rewards
from conftest import assert_vec_close, rel_l2

pytestmark = pytest.mark.gpu

REL = 1e-5


@pytest.fixture(scope="module", params=["c2", "c3", "c5"])
def full_run(request, gpu_available, tmp_path_factory):
    from trpo_amd import Engine, UpdateParams
    cfg = request.param
    SPEC, N = CONFIGS[cfg]
    from trpo_amd._lib import VEC_FULLSTEP, VEC_G, VEC_STEPDIR, VEC_THETA
    b = make_batch(N, SPEC)
    rewards, starts = make_rewards(N)
    e = Engine(SPEC.obs_dim, SPEC.hidden, SPEC.n_actions, max_rows=N)
    e.set_flat(b["theta"])
    uniform = np.full((N, SPEC.n_actions), 1.0 / SPEC.n_actions, np.float32)
    e.set_batch(b["X"], b["actions"], None, uniform, n_global=N)
    old = e.action_dist()                                  # steady state: pi_old = p(theta)
    e.set_batch(b["X"], b["actions"], None, old, n_global=N)
    e.set_rewards(rewards, starts)
    st = e.update(UpdateParams(cg_iters=10, residual_tol=0.0, compute_advantages=True))
    got = {"g": e.get_vector(VEC_G), "stepdir": e.get_vector(VEC_STEPDIR), "fullstep": e.get_vector(VEC_FULLSTEP),
           "theta": e.get_vector(VEC_THETA), "stats": st}
    e.close()
    d = tmp_path_factory.mktemp(f"{cfg}full")
    np.save(d / "old.npy", old)
    here = os.path.dirname(os.path.abspath(__file__))
    subprocess.run([sys.executable, os.path.join(here, "bign_truth.py"), str(d / "old.npy"), str(d / "truth.npz"),
                    cfg], check=True, timeout=900)
    with np.load(d / "truth.npz", allow_pickle=False) as t:
        truth = {k: t[k] for k in t.files}
    return cfg, got, truth


def test_full_size_update_vs_float64(full_run):
    """g, stepdir, fullstep and theta_new within 1e-5 of float64 (norm-relative and elementwise); shs, lm and the
    losses after the step within 1e-5 relative; the CG count, the line-search k and the revert decision exact."""
    cfg, a, t = full_run
    sa = a["stats"]
    assert sa["cg_iters"] == int(t["f64_cg_iters"]) == 10
    assert sa["k"] == int(t["f64_k"]) and bool(sa["reverted"]) == bool(t["f64_reverted"])
    for key in ("g", "stepdir", "fullstep", "theta"):
        line = (f"full size {cfg} {key}: rel L2 vs float64 {rel_l2(a[key], t[f'f64_{key}']):.2e} "
                f"(float32 reference {rel_l2(t[f'f32_{key}'], t[f'f64_{key}']):.2e})")
        print(line)
        if os.environ.get("TRPO_MARGIN_LOG"):   # tools/gpu.sh keeps these margins in the evidence log
            with open(os.environ["TRPO_MARGIN_LOG"], "a") as f:
                f.write(line + "\n")
        assert_vec_close(a[key], t[f"f64_{key}"], REL, f"{key}: {cfg} vs float64 at full size")
    for key in ("shs", "lm", "surr_after", "ent_after"):
        assert sa[key] == pytest.approx(float(t[f"f64_{key}"]), rel=REL), key
    assert sa["kl_after"] == pytest.approx(float(t["f64_kl_after"]), rel=REL, abs=1e-9)
