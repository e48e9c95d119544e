"""CPU oracle for the value-function baseline — TEST INFRASTRUCTURE ONLY.

The checker for ``trpo_amd.vf`` / the ``trpo_vf_*`` C-ABI; never imported by the product.
It restates ``class VF`` of the reference (``utils.py:48-92``) in numpy:

* ``features``      VF._features (``utils.py:70-77``): ``[obs | action_dists | arange(l)/10]``
  per path, the float64 concatenation cast to the float32 placeholder ``x`` (``:58``);
* ``forward``       create_net (``utils.py:56-62``): relu(x W1 + b1) -> relu(. W2 + b2) -> . W3 + b3,
  reshaped to ``[-1]`` (``:63``);
* ``gradient``      d/dtheta of ``sum((net - y)^2)`` — ``minimize(l2)`` on the vector ``l2``
  (``:64-65``) differentiates its sum (``tf.gradients`` seeds ones); ReLU's gradient masks by
  ``output > 0`` (TF ``ReluGrad``);
* ``adam_step``     TF 1.x ``AdamOptimizer`` (``ApplyAdam``, training_ops.cc) with the defaults of
  ``tf.train.AdamOptimizer()``: ``alpha = lr*sqrt(1-b2^t)/(1-b1^t)``, ``m += (g-m)(1-b1)``,
  ``v += (g^2-v)(1-b2)``, ``var -= m*alpha/(sqrt(v)+eps)``; beta powers are float32 variables
  that start at ``(b1, b2)`` and are multiplied after each step;
* ``fit``           50 such steps on the whole batch (``utils.py:84-85``).

Pinning: TF 1.3 is absent, so the VF graph cannot run here; ``gradient`` is checked against
torch autograd of the same network (``tests/test_vf_oracle.py``), the Adam formula is TF's
published kernel restated.  Parity with TF itself is therefore "pinned by an independent
autodiff", like the policy graph.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

ADAM = dict(lr=0.001, beta1=0.9, beta2=0.999, eps=1e-08)   # tf.train.AdamOptimizer() (utils.py:65)
FIT_STEPS = 50                                              # utils.py:84


def features(path: Dict) -> np.ndarray:
    o = np.asarray(path["obs"]).astype("float32")
    o = o.reshape(o.shape[0], -1)
    act = np.asarray(path["action_dists"]).astype("float32").reshape(o.shape[0], -1)
    l = len(path["rewards"])
    al = np.arange(l).reshape(-1, 1) / 10.0
    return np.concatenate([o, act, al], axis=1).astype(np.float32)


def features_concat(obs, dists, starts) -> np.ndarray:
    """features() of every path of a concatenated batch (starts[r] = 1 opens a path)."""
    obs = np.asarray(obs, np.float32).reshape(len(obs), -1)
    dists = np.asarray(dists, np.float32).reshape(len(obs), -1)
    starts = np.asarray(starts).astype(bool)
    t = np.zeros(len(obs), np.int64)
    last = 0
    for r in range(len(obs)):
        if starts[r]:
            last = r
        t[r] = r - last
    return np.concatenate([obs, dists, (t / 10.0).reshape(-1, 1)], axis=1).astype(np.float32)


def unflatten(theta: np.ndarray, F: int, hidden: Sequence[int] = (64, 64)):
    widths = [F, *hidden, 1]
    out, o = [], 0
    for a, b in zip(widths[:-1], widths[1:]):
        out.append((theta[o:o + a * b].reshape(a, b), theta[o + a * b:o + a * b + b]))
        o += a * b + b
    assert o == theta.shape[0]
    return out


def forward(theta, feat, hidden=(64, 64), dtype=np.float64):
    (W1, b1), (W2, b2), (W3, b3) = [(W.astype(dtype), b.astype(dtype))
                                    for W, b in unflatten(np.asarray(theta), feat.shape[1], hidden)]
    x = feat.astype(dtype)
    z1 = np.maximum(x @ W1 + b1, 0)
    z2 = np.maximum(z1 @ W2 + b2, 0)
    net = (z2 @ W3 + b3).reshape(-1)
    return net, (x, z1, z2)


def gradient(theta, feat, y, hidden=(64, 64), dtype=np.float64) -> Tuple[np.ndarray, float]:
    (W1, b1), (W2, b2), (W3, b3) = [(W.astype(dtype), b.astype(dtype))
                                    for W, b in unflatten(np.asarray(theta), feat.shape[1], hidden)]
    net, (x, z1, z2) = forward(theta, feat, hidden, dtype)
    d = net - np.asarray(y).astype(dtype)
    dnet = (d + d).reshape(-1, 1)
    gW3 = z2.T @ dnet
    gb3 = dnet.sum(0)
    dz2 = (dnet @ W3.T) * (z2 > 0)
    gW2 = z1.T @ dz2
    gb2 = dz2.sum(0)
    dz1 = (dz2 @ W2.T) * (z1 > 0)
    gW1 = x.T @ dz1
    gb1 = dz1.sum(0)
    g = np.concatenate([gW1.ravel(), gb1, gW2.ravel(), gb2, gW3.ravel(), gb3])
    return g, float(np.sum(d.astype(np.float64) ** 2))


class Adam:
    """TF 1.x AdamOptimizer state + ApplyAdam."""

    def __init__(self, P: int, lr=ADAM["lr"], beta1=ADAM["beta1"], beta2=ADAM["beta2"], eps=ADAM["eps"],
                 dtype=np.float64):
        self.dtype = dtype
        self.lr, self.b1, self.b2, self.eps = (dtype(lr), dtype(beta1), dtype(beta2), dtype(eps))
        self.m = np.zeros(P, dtype)
        self.v = np.zeros(P, dtype)
        # beta1_power / beta2_power are float32 variables in TF
        self.b1p = np.float32(beta1)
        self.b2p = np.float32(beta2)
        self.t = 0

    def step(self, var: np.ndarray, g: np.ndarray) -> np.ndarray:
        dt = self.dtype
        one = dt(1)
        alpha = dt(self.lr * np.sqrt(one - dt(self.b2p)) / (one - dt(self.b1p)))
        g = g.astype(dt)
        self.m = self.m + (g - self.m) * (one - self.b1)
        self.v = self.v + (g * g - self.v) * (one - self.b2)
        out = var.astype(dt) - (self.m * alpha) / (np.sqrt(self.v) + self.eps)
        self.b1p = np.float32(self.b1p * np.float32(self.b1))
        self.b2p = np.float32(self.b2p * np.float32(self.b2))
        self.t += 1
        return out


def fit(theta, feat, y, steps=FIT_STEPS, hidden=(64, 64), dtype=np.float64, adam: Adam = None):
    """VF.fit's loop (utils.py:84-85); returns (theta, adam)."""
    adam = adam or Adam(theta.size, dtype=dtype)
    th = np.asarray(theta).astype(dtype)
    for _ in range(steps):
        g, _ = gradient(th, feat, y, hidden, dtype)
        th = adam.step(th, g)
    return th, adam


def predict(theta, feat, hidden=(64, 64), dtype=np.float64):
    return forward(theta, feat, hidden, dtype)[0]
