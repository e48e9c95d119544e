"""Autodiff restatement of the reference TF graph — TEST INFRASTRUCTURE ONLY.

Two uses, both outside the product path:

1. It pins ``oracle/trpo_oracle.py``'s closed-form R-op.  The reference's
   graph (``trpo_inksci.py:38-70``) is rebuilt op for op with torch autograd
   standing in for ``tf.gradients``: the same ``stop_gradient`` placement
   (``:56``), the same per-variable tangent split (``:58-67``), the same
   ``gvp = [reduce_sum(g * t)]`` (``:69``) and a second ``flatgrad``
   (``:70``; ``utils.py:119-122``).  Reverse-over-reverse autodiff is an
   independent derivation of the Hessian-vector product, so agreement with
   the hand-written R-op (to ~1e-15 in float64) pins the algebra.

2. ``TFFaithfulCPU`` is the CPU baseline ``bench.py`` times: float32, and every
   FVP / gradient / loss call rebuilds the forward and both backward passes,
   exactly as each ``session.run`` of the reference does
   (``trpo_inksci.py:124-129,146,156``).
"""
from __future__ import annotations

import numpy as np
import torch

from .trpo_oracle import EPS, PolicySpec

torch.set_grad_enabled(True)


def _vars_from_flat(theta: torch.Tensor, spec: PolicySpec, requires_grad=True):
    """tf.trainable_variables() as separate leaves (trpo_inksci.py:49)."""
    out, off = [], 0
    for shape in spec.param_shapes():
        n = int(np.prod(shape))
        v = theta[off:off + n].reshape(shape).detach().clone()
        v.requires_grad_(requires_grad)
        out.append(v)
        off += n
    return out


def _flatgrad(ys, var_list, **kw):
    """utils.py:119-122."""
    grads = torch.autograd.grad(ys, var_list, **kw)
    return torch.cat([g.reshape(-1) for g in grads])


class TFGraph:
    """One 'session' over a fixed feed: state/action/advant/oldaction_dist."""

    def __init__(self, spec: PolicySpec, X, actions, advant, old_dist, dtype=torch.float64):
        self.spec = spec
        self.dtype = dtype
        self.X = torch.as_tensor(np.asarray(X), dtype=dtype)
        self.a = torch.as_tensor(np.asarray(actions, np.int64))
        self.adv = torch.as_tensor(np.asarray(advant), dtype=dtype)
        self.old = torch.as_tensor(np.asarray(old_dist), dtype=dtype)
        self.N = self.X.shape[0]

    def _action_dist(self, var_list):
        # pt.wrap(state).fully_connected(64, tanh)...softmax_classifier(A) (:38-40)
        h = self.X
        L = self.spec.n_layers
        for l in range(L):
            z = h @ var_list[2 * l] + var_list[2 * l + 1]
            h = torch.tanh(z) if l < L - 1 else z
        return torch.softmax(h, dim=1)

    def _losses(self, var_list):
        p = self._action_dist(var_list)
        flat = p.reshape(-1)                                   # slice_2d (utils.py:161-167)
        inds = torch.arange(self.N) * p.shape[1] + self.a
        p_n = flat[inds]
        oldp_n = self.old.reshape(-1)[inds]
        ratio_n = p_n / oldp_n                                 # :46
        Nf = float(self.N)
        surr = -torch.mean(ratio_n * self.adv)                 # :48
        kl = torch.sum(self.old * torch.log((self.old + EPS) / (p + EPS))) / Nf   # :50
        ent = torch.sum(-p * torch.log(p + EPS)) / Nf          # :51
        return p, surr, kl, ent

    def losses(self, theta):
        with torch.no_grad():
            vl = _vars_from_flat(torch.as_tensor(theta, dtype=self.dtype), self.spec, False)
            _, surr, kl, ent = self._losses(vl)
        return np.array([surr.item(), kl.item(), ent.item()])

    def pg(self, theta):
        vl = _vars_from_flat(torch.as_tensor(theta, dtype=self.dtype), self.spec)
        _, surr, _, _ = self._losses(vl)
        return _flatgrad(surr, vl).detach().numpy()            # :54

    def fvp(self, theta, tangent):
        """session.run(self.fvp) — undamped (:56-70)."""
        vl = _vars_from_flat(torch.as_tensor(theta, dtype=self.dtype), self.spec)
        p = self._action_dist(vl)
        Nf = float(self.N)
        kl_ff = torch.sum(p.detach() * torch.log((p + EPS).detach() / (p + EPS))) / Nf   # :56
        grads = torch.autograd.grad(kl_ff, vl, create_graph=True)                        # :57
        t = torch.as_tensor(tangent, dtype=self.dtype)
        tangents, start = [], 0
        for shape in self.spec.param_shapes():                                           # :59-67
            size = int(np.prod(shape))
            tangents.append(t[start:start + size].reshape(shape))
            start += size
        gvp = [torch.sum(g * tt) for g, tt in zip(grads, tangents)]                       # :69
        return _flatgrad(gvp, vl).detach().numpy()                                       # :70


class TFFaithfulCPU:
    """float32 CPU mirror of the reference update (bench cpu_baseline leg).

    Every call recomputes the whole graph as ``session.run`` does; CG and the
    line search are the reference's numpy loops (restated in trpo_oracle)."""

    def __init__(self, spec, X, actions, advant, old_dist, theta):
        self.g = TFGraph(spec, X, actions, advant, old_dist, dtype=torch.float32)
        self.theta = np.asarray(theta, np.float32).copy()

    def update(self, cg_iters=10, residual_tol=0.0, max_kl=0.01, cg_damping=0.1):
        from .trpo_oracle import conjugate_gradient, linesearch
        thprev = self.theta.copy()
        g = self.g.pg(thprev)

        def fvp(p):
            return self.g.fvp(self.theta, p) + np.float32(cg_damping) * p

        stepdir, iters = conjugate_gradient(fvp, -g, cg_iters, residual_tol)
        shs = .5 * float(stepdir.dot(fvp(stepdir)))
        lm = np.sqrt(shs / max_kl)
        fullstep = (stepdir / np.float32(lm)).astype(np.float32)
        neg = float(-g.dot(stepdir))

        def loss(th):
            self.theta = np.asarray(th, np.float32)
            return self.g.losses(self.theta)[0]

        theta, k = linesearch(loss, thprev, fullstep, neg / lm)
        self.theta = np.asarray(theta, np.float32)
        la = self.g.losses(self.theta)
        if la[1] > 2.0 * max_kl:
            self.theta = thprev
        return dict(iters=iters, k=k, losses=la)
