"""Float64 restatement of the whole update at sizes the numpy oracle cannot finish — TEST INFRASTRUCTURE ONLY.

``TFGraph`` (``tf_graph_torch.py``) rebuilt for millions of states: the batch is cut into row chunks, each
chunk's surr / KL / entropy sums, policy gradient and Fisher-vector product are evaluated by torch autograd in
float64 (on whatever device the caller names, the GPU in the ``-m gpu`` tests) with ``1/N_global`` scaling, and
the chunk results are summed in float64. Every quantity of the reference is a sum over states
(``trpo_inksci.py:44-70``), so the chunked sum equals the one-batch graph up to float64 rounding.

The update block (``trpo_inksci.py:144-158``: CG, shs, lm, fullstep, line search, revert) runs on float64
numpy vectors through ``trpo_oracle``'s ``conjugate_gradient`` / ``linesearch``, with the same residual_tol,
damping and max_kl as the engine call it checks. Advantages are the reference's discount + standardisation
(``trpo_inksci.py:102-117``) on paths of equal length, where ``scipy.signal.lfilter`` runs along one axis
(``utils.py:14-16``).

``dtype=torch.float32`` evaluates the same graph in float32 throughout (chunk sums, CG and line-search vectors
included), as the reference's TF float32 session and numpy float32 vectors do: its distance to the float64
result is the rounding level float32 arithmetic itself reaches on a batch (the conditioning floor the GPU tests
compare the engine's own error with).

Never imported by the product path.
"""
from __future__ import annotations

import numpy as np
import torch

from .trpo_oracle import CONFIG, EPS, PolicySpec, conjugate_gradient, linesearch


def advantages_equal_paths(rewards, path_len, gamma=CONFIG["gamma"]):
    """discount per path + standardize (trpo_inksci.py:102-117) for a batch of consecutive paths of one
    length: lfilter([1], [1, -gamma], x[::-1])[::-1] along each path (utils.py:14-16), population std."""
    from scipy.signal import lfilter
    r = np.asarray(rewards, np.float64)
    assert r.shape[0] % path_len == 0
    paths = r.reshape(-1, path_len)
    ret = lfilter([1.0], [1.0, -gamma], paths[:, ::-1], axis=1)[:, ::-1].reshape(-1)
    adv = ret - ret.mean()
    return adv / (adv.std() + 1e-8)


class ChunkedGraph:
    """The reference graph over N states held as float32 arrays on the host, evaluated chunk by chunk."""

    def __init__(self, spec: PolicySpec, X, actions, advant, old_dist, device="cpu", chunk=1 << 20,
                 dtype=torch.float64, resident=False):
        self.spec = spec
        self.dt = dtype
        self.np_dt = np.float64 if dtype == torch.float64 else np.float32
        self.X, self.a, self.adv, self.old = X, actions, advant, old_dist
        self.N = int(X.shape[0])
        self.dev = torch.device(device)
        self.chunk = int(chunk)
        self.resident = None
        if resident:   # the batch copied to the device once, in the graph's dtype (timing runs)
            f = lambda x, dt=self.dt: torch.as_tensor(np.ascontiguousarray(x), device=self.dev).to(dt)
            self.resident = (f(X), f(actions, torch.int64), f(advant), f(old_dist))

    def _vars(self, theta, grad):
        out, off = [], 0
        t = torch.as_tensor(np.asarray(theta, self.np_dt), device=self.dev)
        for shape in self.spec.param_shapes():
            n = int(np.prod(shape))
            v = t[off:off + n].reshape(shape).clone()
            v.requires_grad_(grad)
            out.append(v)
            off += n
        return out

    def _chunks(self):
        for lo in range(0, self.N, self.chunk):
            hi = min(self.N, lo + self.chunk)
            if self.resident is not None:
                yield tuple(t[lo:hi] for t in self.resident)
                continue
            f = lambda x, dt=self.dt: torch.as_tensor(np.ascontiguousarray(x[lo:hi]), device=self.dev).to(dt)
            yield f(self.X), f(self.a, torch.int64), f(self.adv), f(self.old)

    def _dist(self, vl, X):
        h = X
        L = self.spec.n_layers
        for l in range(L):
            z = h @ vl[2 * l] + vl[2 * l + 1]
            h = torch.tanh(z) if l < L - 1 else z
        return torch.softmax(h, dim=1)

    def _losses(self, vl, X, a, adv, old):
        p = self._dist(vl, X)
        p_n = p.gather(1, a[:, None])[:, 0]
        oldp_n = old.gather(1, a[:, None])[:, 0]
        surr = -torch.sum(p_n / oldp_n * adv) / self.N                            # :48
        kl = torch.sum(old * torch.log((old + EPS) / (p + EPS))) / self.N         # :50
        ent = torch.sum(-p * torch.log(p + EPS)) / self.N                         # :51
        return surr, kl, ent

    def losses(self, theta):
        tot = torch.zeros(3, dtype=self.dt, device=self.dev)
        with torch.no_grad():
            vl = self._vars(theta, False)
            for X, a, adv, old in self._chunks():
                tot += torch.stack(self._losses(vl, X, a, adv, old))
        return tot.cpu().numpy().astype(np.float64)

    def pg(self, theta):
        tot = None
        for X, a, adv, old in self._chunks():
            vl = self._vars(theta, True)
            surr, _, _ = self._losses(vl, X, a, adv, old)
            g = torch.cat([t.reshape(-1) for t in torch.autograd.grad(surr, vl)])   # :54
            tot = g if tot is None else tot + g
        return tot.cpu().numpy()

    def fvp(self, theta, tangent):
        """Undamped, trpo_inksci.py:56-70, per chunk with 1/N_global."""
        t = torch.as_tensor(np.asarray(tangent, self.np_dt), device=self.dev)
        tot = None
        for X, _, _, _ in self._chunks():
            vl = self._vars(theta, True)
            p = self._dist(vl, X)
            kl_ff = torch.sum(p.detach() * torch.log((p + EPS).detach() / (p + EPS))) / self.N
            grads = torch.autograd.grad(kl_ff, vl, create_graph=True)
            gvp, off = 0.0, 0
            for g, shape in zip(grads, self.spec.param_shapes()):
                n = int(np.prod(shape))
                gvp = gvp + torch.sum(g * t[off:off + n].reshape(shape))
                off += n
            hv = torch.cat([x.reshape(-1) for x in torch.autograd.grad(gvp, vl)])
            tot = hv if tot is None else tot + hv
        return tot.cpu().numpy()

    def update(self, theta, cg_iters=10, residual_tol=0.0, max_kl=CONFIG["max_kl"],
               cg_damping=CONFIG["cg_damping"]):
        """trpo_inksci.py:144-158 in the graph's dtype (scalars shs / lm / rate in float64, as
        trpo_oracle.trpo_update)."""
        dt = self.np_dt
        th = np.asarray(theta, dt).copy()
        g = self.pg(th)

        def fvp(p):
            return (self.fvp(th, p) + dt(cg_damping) * p).astype(dt)

        stepdir, iters = conjugate_gradient(fvp, -g, cg_iters, residual_tol)
        shs = 0.5 * float(stepdir.dot(fvp(stepdir)))
        lm = float(np.sqrt(shs / max_kl))
        fullstep = (stepdir / dt(lm)).astype(dt)
        rate = float(-g.dot(stepdir)) / lm
        theta_ls, k = linesearch(lambda x: self.losses(x)[0], th, fullstep, rate)
        la = self.losses(theta_ls)
        reverted = bool(la[1] > 2.0 * max_kl)
        return {"g": g, "stepdir": stepdir, "fullstep": fullstep, "shs": shs, "lm": lm, "k": k,
                "theta": th.copy() if reverted else theta_ls, "reverted": reverted, "cg_iters": iters,
                "surr_after": la[0], "kl_after": la[1], "ent_after": la[2]}
