"""The VF oracle (oracle/vf_oracle.py) pinned against torch autograd and TF's Adam formula. CPU only."""
import numpy as np
import pytest

from conftest import rel_l2
from oracle import vf_oracle as V


def _data(n=300, obs=4, A=2, seed=0):
    rng = np.random.RandomState(seed)
    obs_m = rng.standard_normal((n, obs)).astype(np.float32)
    d = rng.dirichlet(np.ones(A), n).astype(np.float32)
    starts = np.zeros(n, np.uint8)
    starts[[0, 17, 90, 91, 200]] = 1
    feat = V.features_concat(obs_m, d, starts)
    F = feat.shape[1]
    widths = [F, 64, 64, 1]
    theta = np.concatenate([np.concatenate([rng.uniform(-np.sqrt(6 / (a + b)), np.sqrt(6 / (a + b)), a * b),
                                            0.1 * rng.standard_normal(b)]) for a, b in zip(widths[:-1], widths[1:])])
    y = rng.uniform(0, 20, n)
    return feat, theta, y, starts, obs_m, d


def test_features_match_per_path_features():
    feat, _, _, starts, obs_m, d = _data()
    cuts = list(np.flatnonzero(starts)) + [len(starts)]
    per_path = np.concatenate([V.features({"obs": obs_m[a:b], "action_dists": d[a:b], "rewards": np.zeros(b - a)})
                               for a, b in zip(cuts[:-1], cuts[1:])])
    assert np.array_equal(per_path, feat)
    assert feat[17, -1] == np.float32(0.0) and feat[20, -1] == np.float32(0.3)


def test_gradient_matches_torch_autograd():
    torch = pytest.importorskip("torch")
    feat, theta, y, *_ = _data()
    g, loss = V.gradient(theta, feat, y)
    th = torch.tensor(theta, dtype=torch.float64, requires_grad=True)
    (W1, b1), (W2, b2), (W3, b3) = V.unflatten(th, feat.shape[1])
    x = torch.tensor(feat, dtype=torch.float64)
    net = (torch.relu(torch.relu(x @ W1 + b1) @ W2 + b2) @ W3 + b3).reshape(-1)
    l2 = (net - torch.tensor(y)) * (net - torch.tensor(y))
    l2.sum().backward()
    assert rel_l2(g, th.grad.numpy()) < 1e-12
    assert loss == pytest.approx(float(l2.sum()), rel=1e-12)


def test_adam_first_step_is_lr_sign():
    """TF ApplyAdam, t=1: alpha = lr sqrt(1-b2)/(1-b1), m = (1-b1) g, v = (1-b2) g^2 -> step ~ lr sign(g)."""
    a = V.Adam(3)
    g = np.array([2.0, -0.5, 1e-3])
    out = a.step(np.zeros(3), g)
    assert np.allclose(out, -0.001 * np.sign(g), rtol=1e-3)
    assert a.b1p == np.float32(np.float32(0.9) * np.float32(0.9))


def test_fit_reduces_loss():
    feat, theta, y, *_ = _data()
    _, l0 = V.gradient(theta, feat, y)
    th, adam = V.fit(theta, feat, y, steps=50)
    _, l1 = V.gradient(th, feat, y)
    assert adam.t == 50 and l1 < l0
