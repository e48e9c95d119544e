"""Test configuration.

Markers:
  gpu  — needs an MI355X (runs the HIP engine through the C-ABI); the driver runs
         ``pytest -m gpu`` on a GPU box and ``pytest -m "not gpu"`` here.
"""
import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD GPU (MI355X) and the built HIP engine")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def update_fixtures():
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "update_*.npz")))


def spec_of(d):
    from oracle.trpo_oracle import PolicySpec
    return PolicySpec(int(d["obs_dim"]), [int(h) for h in d["hidden"]], int(d["n_actions"]))


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def assert_vec_close(a, b, rel=1e-5, what=""):
    """Parity bar of SURVEY.md §8(d): norm-relative <= rel and elementwise
    allclose(rtol=rel, atol=rel*max|b|)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    r = rel_l2(a, b)
    assert r <= rel, f"{what}: rel L2 {r:.3e} > {rel:.1e}"
    atol = rel * float(np.max(np.abs(b))) if b.size else 0.0
    bad = ~np.isclose(a, b, rtol=rel, atol=atol)
    assert not bad.any(), f"{what}: {int(bad.sum())} elements outside rtol/atol (max |d| {np.max(np.abs(a-b)):.3e})"


@pytest.fixture(scope="session")
def gpu_available():
    from trpo_amd import _lib
    if _lib.device_count() < 1:
        pytest.skip("no GPU visible")
    return True
