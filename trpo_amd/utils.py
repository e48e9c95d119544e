"""The reference's ``utils.py`` surface, backed by the HIP engine.

Same names, signatures, defaults and calling conventions as
``/root/reference/utils.py`` so the reference's update block
(``trpo_inksci.py:101-158``) reads unchanged on top of it:

============================  =========================================  ===============================
reference                     here                                       runs on
============================  =========================================  ===============================
discount        :14-16        ``discount(x, gamma)``                     device segmented scan (f64)
flatgrad        :119-122      ``flatgrad(loss, var_list)``               graph node -> engine kernels
SetFromFlat     :125-149      ``SetFromFlat(session, var_list)(theta)``  engine parameter buffer
GetFlat         :151-158      ``GetFlat(session, var_list)()``           engine parameter buffer
linesearch      :170-182      ``linesearch(f, x, fullstep, rate)``       device loop for the engine loss
conjugate_gradient :185-201   ``conjugate_gradient(f_Ax, b, ...)``       device CG (FVP operator: fully
                                                                          device-resident)
var_shape/numel :108-116      same                                       shapes only
explained_variance :208-211   same                                       numpy (statistics print-out)
rollout         :18-45        ``rollout(env, agent, max_pathlength, n)`` host loop over any env; the
                                                                          CartPole-v0 batch runs on the
                                                                          device (``Engine.rollout_cartpole``)
VF              :48-92        ``VF(session)``                            device MLP fit / predict (vf.hip)
cat_sample      :95-105       ``cat_sample(prob_nk)``                    device inverse-CDF sampling
dict2           :203-206      same                                       -
============================  =========================================  ===============================

``session`` here is a :class:`trpo_amd.agent.Session` (or anything with an
``engine`` attribute, or an :class:`~trpo_amd.engine.Engine`).
"""
from __future__ import annotations

import numpy as np

from .engine import Engine, cat_sample_device, cg_callback, discount_device
from .vf import VF  # noqa: F401  (utils.py:48-92)

__all__ = ["discount", "conjugate_gradient", "linesearch", "flatgrad", "GetFlat", "SetFromFlat",
           "var_shape", "numel", "explained_variance", "FisherVectorProduct", "SurrogateLoss", "VF",
           "cat_sample", "rollout", "dict2"]


def _engine_of(session) -> Engine:
    if isinstance(session, Engine):
        return session
    eng = getattr(session, "engine", None)
    if not isinstance(eng, Engine):
        raise TypeError("expected an Engine or a Session wrapping one")
    return eng


# ---------------------------------------------------------------------------- utils.py:14-16
def discount(x, gamma):
    """scipy.signal.lfilter([1], [1, -gamma], x[::-1], axis=0)[::-1] on the GPU."""
    x = np.asarray(x)
    assert x.ndim >= 1
    if x.ndim == 1:
        return discount_device(x.astype(np.float64), gamma)
    flat = x.reshape(x.shape[0], -1).astype(np.float64)
    out = np.empty_like(flat)
    for c in range(flat.shape[1]):
        out[:, c] = discount_device(np.ascontiguousarray(flat[:, c]), gamma)
    return out.reshape(x.shape)


# ---------------------------------------------------------------------------- utils.py:108-116
def var_shape(x):
    out = [int(k) for k in (x.shape if hasattr(x, "shape") else x)]
    assert all(isinstance(a, int) for a in out), "shape function assumes that shape is fully known"
    return out


def numel(x):
    return int(np.prod(var_shape(x)))


# ---------------------------------------------------------------------------- graph nodes
class SurrogateLoss:
    """The ``surr`` tensor of trpo_inksci.py:48 on an engine."""

    def __init__(self, engine: Engine):
        self.engine = engine


class KLFirstFixedGVP:
    """``gvp`` of trpo_inksci.py:56-69 (grad of KL_firstfixed dotted with a tangent)."""

    def __init__(self, engine: Engine):
        self.engine = engine


class PolicyGradient:
    """``flatgrad(surr, var_list)`` (trpo_inksci.py:54)."""

    def __init__(self, engine: Engine):
        self.engine = engine

    def __call__(self):
        return self.engine.policy_grad()


class FisherVectorProduct:
    """``fisher_vector_product(p) = session.run(fvp) + cg_damping * p`` (trpo_inksci.py:124-126)
    as an operator the device CG consumes directly."""

    def __init__(self, engine: Engine, damping: float = 0.1):
        self.engine = engine
        self.damping = float(damping)

    def __call__(self, p):
        return self.engine.fvp(p, self.damping)

    def damped(self, damping: float) -> "FisherVectorProduct":
        """``session.run(fvp) + damping * p`` (trpo_inksci.py:126) as an operator on the same engine."""
        return FisherVectorProduct(self.engine, damping)


def flatgrad(loss, var_list=None):
    """utils.py:119-122: the flat gradient node of ``loss`` w.r.t. the policy parameters."""
    if isinstance(loss, SurrogateLoss):
        return PolicyGradient(loss.engine)
    if isinstance(loss, KLFirstFixedGVP):
        return FisherVectorProduct(loss.engine, damping=0.0)
    raise TypeError("flatgrad: unsupported loss node")


# ---------------------------------------------------------------------------- utils.py:125-158
class SetFromFlat:
    def __init__(self, session, var_list=None):
        self.engine = _engine_of(session)

    def __call__(self, theta):
        self.engine.set_flat(np.asarray(theta, np.float32) if not hasattr(theta, "data_ptr") else theta)


class GetFlat:
    def __init__(self, session, var_list=None):
        self.engine = _engine_of(session)

    def __call__(self):
        return self.engine.get_flat()


# ---------------------------------------------------------------------------- utils.py:170-182
class EngineLoss:
    """``loss(th)`` of trpo_inksci.py:127-129: sff(th); session.run(surr)."""

    def __init__(self, engine: Engine):
        self.engine = engine

    def __call__(self, th):
        return np.float32(self.engine.eval_losses(th)[0])


def linesearch(f, x, fullstep, expected_improve_rate):
    """utils.py:170-182.  With ``f`` an :class:`EngineLoss` the whole search runs on the
    device (one surrogate forward per backtrack); any other callable gets the reference's
    loop verbatim (its arithmetic is on ``f``'s side)."""
    if isinstance(f, EngineLoss):
        theta, k = f.engine.linesearch(np.asarray(x, np.float32), np.asarray(fullstep, np.float32),
                                       float(expected_improve_rate))
        return x if k < 0 else theta
    accept_ratio = .1
    max_backtracks = 10
    fval = f(x)
    for (_n_backtracks, stepfrac) in enumerate(.5 ** np.arange(max_backtracks)):
        xnew = x + x.dtype.type(stepfrac) * fullstep
        newfval = f(xnew)
        actual_improve = fval - newfval
        expected_improve = expected_improve_rate * stepfrac
        ratio = actual_improve / expected_improve
        if ratio > accept_ratio and actual_improve > 0:
            return xnew
    return x


# ---------------------------------------------------------------------------- utils.py:185-201
def conjugate_gradient(f_Ax, b, cg_iters=10, residual_tol=1e-10, return_iters=False):
    """utils.py:185-201.  ``f_Ax`` = :class:`FisherVectorProduct` runs the device-resident CG
    (FVP, dots and axpys all on the GPU); any other callable runs the same CG vector kernels on
    the GPU with a host round trip per ``f_Ax`` call.  ``b`` is not modified."""
    if isinstance(f_Ax, FisherVectorProduct):
        x, it = f_Ax.engine.cg(np.asarray(b, np.float32), cg_iters, residual_tol, f_Ax.damping)
    else:
        x, it = cg_callback(f_Ax, np.asarray(b), cg_iters, residual_tol)
    return (x, it) if return_iters else x


# ---------------------------------------------------------------------------- utils.py:208-211
def explained_variance(ypred, y):
    assert y.ndim == 1 and ypred.ndim == 1
    vary = np.var(y)
    return np.nan if vary == 0 else 1 - np.var(y - ypred) / vary


# ---------------------------------------------------------------------------- utils.py:18-45
def rollout(env, agent, max_pathlength, n_timesteps):
    """utils.py:18-45 for any gym-style env and an agent with act()/prev_action: whole episodes until
    n_timesteps steps are collected.  (For CartPole-v0 the batched device rollout
    ``Engine.rollout_cartpole`` does this for many environments at once.)

    Reference semantics kept as they are: a path is appended only when its episode ends (``done``)
    within max_pathlength steps (utils.py:35-43); an episode cut off at max_pathlength is dropped,
    and the step count then advances by the length of the last appended path (utils.py:44 reads the
    previous ``path``), or raises UnboundLocalError when no path was appended yet, as the reference
    does.  With gym's CartPole-v0 (TimeLimit 200 < max_pathlength 1000) every episode ends with done."""
    paths = []
    timesteps_sofar = 0
    while timesteps_sofar < n_timesteps:
        obs, actions, rewards, action_dists = [], [], [], []
        ob = env.reset()
        agent.prev_action *= 0.0
        for _ in range(max_pathlength):
            action, action_dist, ob = agent.act(ob)
            obs.append(ob)
            actions.append(action)
            action_dists.append(action_dist)
            res = env.step(action)
            ob = res[0]
            rewards.append(res[1])
            if res[2]:
                path = {"obs": np.concatenate(np.expand_dims(obs, 0)), "action_dists": np.concatenate(action_dists),
                        "rewards": np.array(rewards), "actions": np.array(actions)}
                paths.append(path)
                agent.prev_action *= 0.0
                break
        timesteps_sofar += len(path["rewards"])   # noqa: F821  (the reference's stale-path read)
    return paths


# ---------------------------------------------------------------------------- utils.py:95-105
def cat_sample(prob_nk):
    """Inverse-CDF sampling of each row of prob_nk against np.random.rand(N), on the GPU."""
    prob_nk = np.asarray(prob_nk)
    assert prob_nk.ndim == 2
    r = np.random.rand(prob_nk.shape[0])
    return cat_sample_device(prob_nk.astype(np.float32), r).astype("i")


# ---------------------------------------------------------------------------- utils.py:203-206
class dict2(dict):
    def __init__(self, **kwargs):
        dict.__init__(self, kwargs)
        self.__dict__ = self
