"""CPU oracle for the TRPO policy update — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import it.  The product path (``trpo_amd``) runs the HIP kernels behind the
C-ABI in ``include/trpo_engine.h`` and fails loudly when that library is
missing; it never falls back to anything in this directory.

What it restates (numpy, float64 by default, float32 on request):

* the policy graph of ``trpo_inksci.py:38-40`` (tanh MLP + softmax head; the
  hidden widths are a list, the reference is the depth-1 case ``[64]``),
* ``surr``/``kl``/``ent`` of ``trpo_inksci.py:44-53`` (``slice_2d`` gather of
  ``utils.py:161-167``, ``eps = 1e-6`` of ``trpo_inksci.py:16``),
* ``pg = flatgrad(surr)`` of ``trpo_inksci.py:54`` (``utils.py:119-122``),
* the FVP graph of ``trpo_inksci.py:56-70`` as the closed-form Pearlmutter
  R-op of SURVEY.md Appendix A (eps-exact, including the O(eps) plain
  deltas and the ``-2 h R{h}`` tanh'' term), plus the damping closure of
  ``trpo_inksci.py:124-126``,
* ``conjugate_gradient`` (``utils.py:185-201``), ``linesearch``
  (``utils.py:170-182``), the step scaling of ``trpo_inksci.py:147-151``, the
  post-update revert of ``trpo_inksci.py:154-158``,
* ``discount`` (``utils.py:14-16``; ``scipy.signal.lfilter`` restated as its
  order-1 recurrence) and the advantage standardisation of
  ``trpo_inksci.py:115-117``.

How it is pinned: ``tests/golden/make_golden.py`` imports the reference's own
``utils.py`` (numpy half) in the build container and records its outputs;
the TF-graph half (no TF 1.3 / Python 2 anywhere) is pinned against an
independent reverse-over-reverse autodiff restatement of the same graph in
``oracle/tf_graph_torch.py`` (float64).  See DESIGN.md "Oracle".

Flat parameter layout (``var_shape``/``numel`` ``utils.py:108-116``;
``tf.trainable_variables()`` order ``trpo_inksci.py:49``):
``[W1, b1, W2, b2, ..., WL, bL]`` with every ``W_l`` row-major
``[fan_in, fan_out]``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, List, Sequence

import numpy as np

EPS = 1e-6                                   # trpo_inksci.py:16
CONFIG = {"max_steps": 1000, "episodes_per_roll": 1000, "gamma": 0.95,
          "cg_damping": 0.1, "max_kl": 0.01}  # trpo_inksci.py:17
ACCEPT_RATIO = 0.1                           # utils.py:171
MAX_BACKTRACKS = 10                          # utils.py:172


@dataclass(frozen=True)
class PolicySpec:
    """Shape of the categorical tanh-MLP policy (trpo_inksci.py:38-40)."""
    obs_dim: int
    hidden: Sequence[int]
    n_actions: int

    @property
    def widths(self) -> List[int]:
        return [self.obs_dim, *self.hidden, self.n_actions]

    @property
    def n_layers(self) -> int:
        return len(self.hidden) + 1

    def layer_dims(self):
        w = self.widths
        return [(w[i], w[i + 1]) for i in range(len(w) - 1)]

    def param_shapes(self):
        """var_shape() of tf.trainable_variables(), creation order (utils.py:108)."""
        out = []
        for a, b in self.layer_dims():
            out.append((a, b))
            out.append((b,))
        return out

    @property
    def n_params(self) -> int:
        return int(sum(int(np.prod(s)) for s in self.param_shapes()))


# ----------------------------------------------------------------------------
# flat-parameter plumbing (GetFlat / SetFromFlat, utils.py:125-158)
# ----------------------------------------------------------------------------
def unflatten(theta: np.ndarray, spec: PolicySpec):
    """Split a flat vector into [(W1, b1), ...] views (SetFromFlat, utils.py:125-149)."""
    theta = np.asarray(theta)
    assert theta.ndim == 1 and theta.shape[0] == spec.n_params, (theta.shape, spec.n_params)
    out, off = [], 0
    for a, b in spec.layer_dims():
        W = theta[off:off + a * b].reshape(a, b)
        off += a * b
        bias = theta[off:off + b]
        off += b
        out.append((W, bias))
    return out


def flatten(params) -> np.ndarray:
    """Concatenate [(W, b), ...] row-major (GetFlat, utils.py:151-158)."""
    return np.concatenate([np.concatenate([W.reshape(-1), b.reshape(-1)]) for W, b in params])


def init_theta(spec: PolicySpec, rng: np.random.RandomState, bias_std: float = 0.1,
               dtype=np.float32) -> np.ndarray:
    """Synthetic parameters: W ~ U(+-sqrt(6/(fan_in+fan_out))),
    b ~ N(0, bias_std^2) (non-zero so the bias paths are exercised)."""
    params = []
    for a, b in spec.layer_dims():
        lim = math.sqrt(6.0 / (a + b))
        W = rng.uniform(-lim, lim, size=(a, b))
        bias = rng.normal(0.0, bias_std, size=(b,)) if bias_std > 0 else np.zeros(b)
        params.append((W, bias))
    return flatten(params).astype(dtype)


# ----------------------------------------------------------------------------
# policy forward + losses (trpo_inksci.py:38-53)
# ----------------------------------------------------------------------------
def _softmax(z):
    z = z - z.max(axis=1, keepdims=True)
    e = np.exp(z)
    return e / e.sum(axis=1, keepdims=True)


def forward(theta, X, spec: PolicySpec, dtype=np.float64):
    """Returns (hs, p): hs = [h_0 = X, h_1, ..., h_{L-1}], p = softmax(z_L)."""
    params = unflatten(np.asarray(theta, dtype), spec)
    h = np.asarray(X, dtype)
    hs = [h]
    L = spec.n_layers
    for l, (W, b) in enumerate(params):
        z = h @ W + b
        if l < L - 1:
            h = np.tanh(z)
            hs.append(h)
        else:
            return hs, _softmax(z)
    raise AssertionError("unreachable")


def action_dist(theta, X, spec, dtype=np.float64):
    return forward(theta, X, spec, dtype)[1]


def losses(theta, X, actions, advant, old_dist, spec, n_global=None, dtype=np.float64):
    """[surr, kl, ent] (trpo_inksci.py:44-53).  With ``n_global`` the sums are
    divided by the global batch size (a shard's partial contribution)."""
    _, p = forward(theta, X, spec, dtype)
    old = np.asarray(old_dist, dtype)
    adv = np.asarray(advant, dtype)
    n = X.shape[0]
    N = n if n_global is None else n_global
    idx = np.arange(n)
    a = np.asarray(actions, np.int64)
    p_n = p[idx, a]                       # slice_2d, utils.py:161-167
    oldp_n = old[idx, a]
    ratio_n = p_n / oldp_n                # trpo_inksci.py:46 (no eps)
    surr = -np.sum(ratio_n * adv) / N     # -reduce_mean, :48
    kl = np.sum(old * np.log((old + EPS) / (p + EPS))) / N     # :50
    ent = np.sum(-p * np.log(p + EPS)) / N                      # :51
    return np.array([surr, kl, ent], dtype)


def _backprop(params, hs, delta_L, dtype):
    """Reverse pass from the logit delta; returns flat gradient."""
    L = len(params)
    grads = [None] * L
    d = delta_L
    for l in range(L - 1, -1, -1):
        W, _ = params[l]
        grads[l] = (hs[l].T @ d, d.sum(axis=0))
        if l > 0:
            dh = d @ W.T
            d = dh * (1.0 - hs[l] ** 2)
    return flatten(grads).astype(dtype)


def policy_grad(theta, X, actions, advant, old_dist, spec, n_global=None, dtype=np.float64):
    """pg = flatgrad(surr, var_list) (trpo_inksci.py:54; utils.py:119-122).

    d surr / d z[n, j] = -(adv_n / (N pold[n, a_n])) p[n, a_n] (1[j = a_n] - p[n, j])
    (the TF SoftmaxGrad of the gathered ratio)."""
    params = unflatten(np.asarray(theta, dtype), spec)
    hs, p = forward(theta, X, spec, dtype)
    n = X.shape[0]
    N = n if n_global is None else n_global
    idx = np.arange(n)
    a = np.asarray(actions, np.int64)
    old = np.asarray(old_dist, dtype)
    adv = np.asarray(advant, dtype)
    gp = np.zeros_like(p)
    gp[idx, a] = -adv / (N * old[idx, a])
    delta = p * (gp - np.sum(gp * p, axis=1, keepdims=True))
    return _backprop(params, hs, delta, dtype)


# ----------------------------------------------------------------------------
# Fisher-vector product (trpo_inksci.py:56-70)
# ----------------------------------------------------------------------------
def fvp_undamped(theta, X, v, spec, n_global=None, dtype=np.float64):
    """Hv = grad_theta[(grad_theta KL_ff) . v] with
    KL_ff = (1/N) sum p0 log((p0+eps)/(p+eps)), p0 = stop_gradient(p) at the
    same theta (trpo_inksci.py:56).  Closed-form Pearlmutter R-op."""
    params = unflatten(np.asarray(theta, dtype), spec)
    tang = unflatten(np.asarray(v, dtype), spec)
    hs, p = forward(theta, X, spec, dtype)
    n = X.shape[0]
    N = n if n_global is None else n_global
    L = len(params)
    p0 = p
    # plain reverse pass of KL_ff: deltas are O(eps), not zero
    g_p = -(1.0 / N) * p0 / (p + EPS)
    gpp = np.sum(g_p * p, axis=1, keepdims=True)
    deltas = [None] * L          # delta_l = dKL/dz_l
    dhs = [None] * L             # dh_{l} = delta_{l+1} W_{l+1}^T  (index by l)
    deltas[L - 1] = p * (g_p - gpp)
    for l in range(L - 1, 0, -1):
        dh = deltas[l] @ params[l][0].T
        dhs[l - 1] = dh
        deltas[l - 1] = dh * (1.0 - hs[l] ** 2)
    # R-forward
    Rh = [np.zeros_like(hs[0])]
    Rz_L = None
    for l in range(L):
        W, _ = params[l]
        V, c = tang[l]
        Rz = hs[l] @ V + c
        if l > 0:
            Rz = Rz + Rh[l] @ W
        if l < L - 1:
            Rh.append((1.0 - hs[l + 1] ** 2) * Rz)
        else:
            Rz_L = Rz
    Rp = p * (Rz_L - np.sum(p * Rz_L, axis=1, keepdims=True))
    # R-reverse
    Rg_p = (1.0 / N) * p0 * Rp / (p + EPS) ** 2
    Rdelta = Rp * (g_p - gpp) + p * (Rg_p - np.sum(Rg_p * p, axis=1, keepdims=True)
                                     - np.sum(g_p * Rp, axis=1, keepdims=True))
    out = [None] * L
    for l in range(L - 1, -1, -1):
        W, _ = params[l]
        V, _ = tang[l]
        gW = hs[l].T @ Rdelta
        if l > 0:
            gW = gW + Rh[l].T @ deltas[l]
        out[l] = (gW, Rdelta.sum(axis=0))
        if l > 0:
            Rdh = Rdelta @ W.T + deltas[l] @ V.T
            Rdelta = Rdh * (1.0 - hs[l] ** 2) - 2.0 * dhs[l - 1] * hs[l] * Rh[l]
    return flatten(out).astype(dtype)


def fisher_vector_product(theta, X, v, spec, damping=CONFIG["cg_damping"], dtype=np.float64):
    """session.run(fvp) + cg_damping * p (trpo_inksci.py:124-126)."""
    v = np.asarray(v, dtype)
    return fvp_undamped(theta, X, v, spec, dtype=dtype) + dtype(damping) * v


# ----------------------------------------------------------------------------
# numpy half: CG, line search, discount (utils.py)
# ----------------------------------------------------------------------------
def conjugate_gradient(f_Ax: Callable, b, cg_iters=10, residual_tol=1e-10):
    """utils.py:185-201, returning (x, iterations_run).  Same arithmetic order;
    the array dtype of ``b`` carries through (float32 in the reference)."""
    p = b.copy()
    r = b.copy()
    x = np.zeros_like(b)
    rdotr = r.dot(r)
    it = 0
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):  # p.z = 0: inf / nan, as numpy gives
        for i in range(cg_iters):
            z = f_Ax(p)
            v = rdotr / p.dot(z)
            x += v * p
            r -= v * z
            newrdotr = r.dot(r)
            mu = newrdotr / rdotr
            p = r + mu * p
            rdotr = newrdotr
            it = i + 1
            if rdotr < residual_tol:
                break
    return x, it


def linesearch(f: Callable, x, fullstep, expected_improve_rate):
    """utils.py:170-182, returning (theta, k): k = index of the accepted step
    fraction 0.5**k, or -1 when every backtrack is rejected (then ``x`` itself
    is returned, as utils.py:182 does).  ``xnew`` keeps x's dtype (the
    reference's NumPy-1.x ran this loop in float32)."""
    fval = f(x)
    for k, stepfrac in enumerate(.5 ** np.arange(MAX_BACKTRACKS)):
        xnew = (x + x.dtype.type(stepfrac) * fullstep).astype(x.dtype)
        newfval = f(xnew)
        actual_improve = fval - newfval
        expected_improve = expected_improve_rate * stepfrac
        with np.errstate(divide="ignore", invalid="ignore"):
            ratio = actual_improve / expected_improve
        if ratio > ACCEPT_RATIO and actual_improve > 0:
            return xnew, k
    return x, -1


def discount(x, gamma):
    """utils.py:14-16: lfilter([1], [1, -gamma], x[::-1])[::-1], i.e.
    y[t] = x[t] + gamma * y[t+1] evaluated in that order (the order-1 IIR of
    scipy's direct form II transposed: one rounding for the product, one for
    the sum)."""
    x = np.asarray(x)
    assert x.ndim >= 1
    y = np.empty(x.shape, dtype=np.result_type(x.dtype, np.float64))
    acc = 0.0
    for t in range(x.shape[0] - 1, -1, -1):
        acc = x[t] + gamma * acc
        y[t] = acc
    return y


def discount_segmented(rewards, starts, gamma):
    """Per-episode discount over a concatenated batch (trpo_inksci.py:102-104):
    ``starts[i]`` true where an episode begins."""
    rewards = np.asarray(rewards, np.float64)
    starts = np.asarray(starts, bool).copy()
    if rewards.shape[0]:
        starts[0] = True
    out = np.empty_like(rewards)
    acc = 0.0
    for t in range(rewards.shape[0] - 1, -1, -1):
        acc = rewards[t] + gamma * acc
        out[t] = acc
        if starts[t]:
            acc = 0.0
    return out


def standardize(advant):
    """trpo_inksci.py:116-117 (population std, float64)."""
    adv = np.array(advant, dtype=np.float64, copy=True)
    adv -= adv.mean()
    adv /= (adv.std() + 1e-8)
    return adv


def explained_variance(ypred, y):
    """utils.py:208-211."""
    assert y.ndim == 1 and ypred.ndim == 1
    vary = np.var(y)
    return np.nan if vary == 0 else 1 - np.var(y - ypred) / vary


# ----------------------------------------------------------------------------
# the update block (trpo_inksci.py:101-158)
# ----------------------------------------------------------------------------
@dataclass
class Batch:
    X: np.ndarray              # [N, obs] float32
    actions: np.ndarray        # [N] int64
    advant: np.ndarray         # [N] (already standardised)
    old_dist: np.ndarray       # [N, A] float32


@dataclass
class UpdateResult:
    g: np.ndarray
    stepdir: np.ndarray
    cg_iters: int
    shs: float
    lm: float
    fullstep: np.ndarray
    neggdotstepdir: float
    rate: float
    theta_ls: np.ndarray
    k: int
    losses_after: np.ndarray
    reverted: bool
    theta_new: np.ndarray
    losses_before: np.ndarray = field(default=None)


def trpo_update(theta_prev, batch: Batch, spec: PolicySpec, dtype=np.float64,
                cg_iters=10, residual_tol=1e-10, max_kl=CONFIG["max_kl"],
                cg_damping=CONFIG["cg_damping"]) -> UpdateResult:
    """One policy update, trpo_inksci.py:144-158, evaluated in ``dtype``.

    Scalar dtypes follow the reference's NumPy-1.x rules: ``shs``, ``lm`` and the
    expected-improve rate are float64 (python-float x numpy-scalar promotes),
    vectors stay in ``dtype``."""
    th = np.asarray(theta_prev, dtype).copy()
    X, a, adv, old = batch.X, batch.actions, batch.advant, batch.old_dist

    def fvp(p):
        return fisher_vector_product(th_cur[0], X, p, spec, cg_damping, dtype)

    th_cur = [th]
    thprev = th.copy()
    losses_before = losses(thprev, X, a, adv, old, spec, dtype=dtype)
    g = policy_grad(thprev, X, a, adv, old, spec, dtype=dtype)
    stepdir, iters = conjugate_gradient(fvp, -g, cg_iters, residual_tol)
    shs = 0.5 * float(stepdir.dot(fvp(stepdir)))
    with np.errstate(invalid="ignore"):                    # np.sqrt: shs < 0 gives nan, as in the reference
        lm = float(np.sqrt(np.float64(shs / max_kl)))
    with np.errstate(divide="ignore", invalid="ignore"):
        fullstep = (stepdir / dtype(lm)).astype(dtype)
    neggdotstepdir = -g.dot(stepdir)
    with np.errstate(divide="ignore", invalid="ignore"):
        rate = float(np.float64(neggdotstepdir) / np.float64(lm))

    def loss(x):
        return losses(x, X, a, adv, old, spec, dtype=dtype)[0]

    theta_ls, k = linesearch(loss, thprev, fullstep, rate)
    la = losses(theta_ls, X, a, adv, old, spec, dtype=dtype)
    reverted = bool(la[1] > 2.0 * max_kl)
    theta_new = thprev.copy() if reverted else np.asarray(theta_ls, dtype).copy()
    return UpdateResult(g=g, stepdir=stepdir, cg_iters=iters, shs=shs, lm=lm,
                        fullstep=fullstep, neggdotstepdir=float(neggdotstepdir), rate=rate,
                        theta_ls=np.asarray(theta_ls, dtype), k=k, losses_after=la,
                        reverted=reverted, theta_new=theta_new, losses_before=losses_before)


# ----------------------------------------------------------------------------
# synthetic workload
# ----------------------------------------------------------------------------
def synthetic_batch(spec: PolicySpec, n: int, seed: int = 0, episode_len: int = 200,
                    gamma: float = CONFIG["gamma"], steady_state: bool = True,
                    perturb: float = 0.0):
    """X ~ N(0,1) f32; theta (see init_theta); a ~ U{0..A-1}; rewards ~ U(0,1)
    with an episode start every ``episode_len`` steps -> discount -> standardise;
    old_dist = p(theta) (steady state) or p(theta + perturb * noise)."""
    rng = np.random.RandomState(seed)
    X = rng.standard_normal((n, spec.obs_dim)).astype(np.float32)
    theta = init_theta(spec, rng)
    actions = rng.randint(0, spec.n_actions, size=n).astype(np.int64)
    rewards = rng.uniform(0.0, 1.0, size=n)
    starts = np.zeros(n, bool)
    starts[::episode_len] = True
    returns = discount_segmented(rewards, starts, gamma)
    adv = standardize(returns)
    th_old = theta.astype(np.float64)
    if not steady_state:
        th_old = th_old + perturb * rng.standard_normal(th_old.shape)
    old = action_dist(th_old, X, spec, np.float64).astype(np.float32)
    return dict(X=X, theta=theta, actions=actions, rewards=rewards, starts=starts,
                returns=returns, advant=adv, old_dist=old)
