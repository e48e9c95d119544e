"""Generate the committed golden fixtures (run in the build container only).

    python tests/golden/make_golden.py

Inputs and expected outputs come from the reference's OWN numpy functions
(``/root/reference/utils.py``: ``discount`` :14-16, ``linesearch`` :170-182,
``conjugate_gradient`` :185-201, ``explained_variance`` :208-211), imported
with stub ``tensorflow``/``prettytensor`` modules by ``oracle/ref_loader.py``.
The TF-graph half of each full-update tuple (``trpo_inksci.py:38-70``: pg and
FVP) cannot run here (TF 1.3 / Python 2 absent); it is evaluated in float64
by the autodiff restatement ``oracle/tf_graph_torch.TFGraph`` and cross-checked
against the closed-form R-op of ``oracle/trpo_oracle.py`` before anything is
written.  The update driver below restates ``trpo_inksci.py:144-158`` line for
line around the reference's ``conjugate_gradient`` / ``linesearch``.

Outputs: ``tests/golden/*.npz`` (data only: inputs and expected outputs).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import trpo_oracle as O                       # noqa: E402
from oracle.ref_loader import load_reference_utils         # noqa: E402
from oracle.tf_graph_torch import TFGraph                  # noqa: E402


def _save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {name}: {os.path.getsize(path) / 1024:.1f} KiB")


def gen_discount(U):
    rng = np.random.RandomState(7)
    out = {}
    for gamma in (0.95, 0.99):
        for n in (1, 2, 200, 1000):
            for kind in ("uniform", "ones"):
                x = rng.uniform(0, 1, n) if kind == "uniform" else np.ones(n)
                key = f"g{gamma}_n{n}_{kind}"
                out[key + "_x"] = x
                out[key + "_y"] = np.asarray(U.discount(x, gamma))
    _save("discount.npz", **out)


class _Counter:
    def __init__(self, f):
        self.f, self.calls = f, 0

    def __call__(self, x):
        self.calls += 1
        return self.f(x)


def gen_cg(U):
    out = {}
    cases = []
    rng = np.random.RandomState(11)
    for dt in (np.float32, np.float64):
        for n, cond in ((50, 10.0), (200, 1e3)):
            Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
            ev = np.geomspace(1.0, cond, n)
            A = (Q * ev) @ Q.T
            A = ((A + A.T) / 2).astype(dt)
            b = rng.standard_normal(n).astype(dt)
            base = f"{np.dtype(dt).name}_n{n}_c{int(cond)}"
            out[base + "_A"] = A
            out[base + "_b"] = b
            for tol_name, tol in (("default", 1e-10), ("zero", 0.0), ("loose", 1e-2)):
                for iters in (10, 25):
                    f = _Counter(lambda p, A=A: A @ p)
                    b_in = b.copy()
                    x = U.conjugate_gradient(f, b_in, iters, tol)
                    assert np.array_equal(b_in, b)           # b not mutated (utils.py:186-187)
                    key = f"{base}_{tol_name}_it{iters}"
                    out[key + "_base"] = np.array(base)
                    out[key + "_x"] = np.asarray(x)
                    out[key + "_iters"] = np.int64(f.calls)
                    out[key + "_tol"] = np.float64(tol)
                    out[key + "_maxit"] = np.int64(iters)
                    cases.append(key)
    out["cases"] = np.array(cases)
    _save("cg.npz", **out)


def gen_linesearch(U):
    """f(x) = 0.5 ||x - c||^2 scaled; cases: accept k=0, accept k>0, reject all."""
    out = {}
    cases = []
    rng = np.random.RandomState(13)
    n = 16
    c = rng.standard_normal(n).astype(np.float32)
    x0 = np.zeros(n, np.float32)
    grad = (x0 - c)
    for name, scale, rate_mul in (("accept0", 1.0, 1.0), ("accept_k3", 12.0, 1.0),
                                  ("accept_k1", 3.0, 1.0), ("reject", -1.0, 1.0),
                                  ("ratio_gate", 1.0, 1e6)):
        fullstep = (-scale * grad).astype(np.float32)
        rate = float(-grad.dot(fullstep)) * rate_mul
        f = _Counter(lambda x: np.float32(0.5 * np.sum((np.asarray(x, np.float32) - c) ** 2, dtype=np.float32)))
        res = U.linesearch(f, x0, fullstep, rate)
        same = res is x0
        k = -1 if same else f.calls - 2
        out[name + "_x"] = x0
        out[name + "_c"] = c
        out[name + "_fullstep"] = fullstep
        out[name + "_rate"] = np.float64(rate)
        out[name + "_result"] = np.asarray(res, np.float64)
        out[name + "_k"] = np.int64(k)
        out[name + "_calls"] = np.int64(f.calls)
        cases.append(name)
        print(f"  linesearch {name}: k={k} calls={f.calls}")
    out["cases"] = np.array(cases)
    _save("linesearch.npz", **out)


def gen_explained_variance(U):
    rng = np.random.RandomState(17)
    y = rng.standard_normal(100)
    out = dict(y=y, ypred=y + 0.3 * rng.standard_normal(100), yconst=np.ones(10))
    out["ev"] = np.float64(U.explained_variance(out["ypred"], y))
    out["ev_const_is_nan"] = np.bool_(np.isnan(U.explained_variance(np.zeros(10), out["yconst"])))
    _save("explained_variance.npz", **out)


def gen_update(U, name, spec, n, seed, max_kl=0.01, steady=True, perturb=0.0,
               residual_tol=1e-10, episode_len=200):
    d = O.synthetic_batch(spec, n, seed=seed, episode_len=episode_len, steady_state=steady,
                          perturb=perturb)
    X, a, adv, old = d["X"], d["actions"], d["advant"], d["old_dist"]
    G = TFGraph(spec, X, a, adv, old, dtype=__import__("torch").float64)
    theta0 = d["theta"].astype(np.float64)
    state = {"theta": theta0.copy()}

    # cross-check the two float64 restatements on this batch before recording
    v = np.random.RandomState(seed + 1).standard_normal(spec.n_params)
    hv_tf = G.fvp(theta0, v)
    hv_cf = O.fvp_undamped(theta0, X, v, spec)
    rel = np.linalg.norm(hv_tf - hv_cf) / np.linalg.norm(hv_tf)
    assert rel < 1e-12, rel
    g_tf = G.pg(theta0)
    assert np.linalg.norm(g_tf - O.policy_grad(theta0, X, a, adv, old, spec)) < 1e-12 * np.linalg.norm(g_tf)

    # ---- trpo_inksci.py:124-129 closures -------------------------------------
    def fisher_vector_product(p):
        return G.fvp(state["theta"], p) + 0.1 * p

    def sff(th):
        state["theta"] = np.array(th, np.float64)

    def loss(th):
        sff(th)
        return G.losses(state["theta"])[0]

    # ---- trpo_inksci.py:144-158 ----------------------------------------------
    thprev = state["theta"].copy()
    losses_before = G.losses(thprev)
    g = G.pg(thprev)
    fvpc = _Counter(fisher_vector_product)
    stepdir = U.conjugate_gradient(fvpc, -g, 10, residual_tol)
    cg_iters = fvpc.calls
    shs = .5 * stepdir.dot(fisher_vector_product(stepdir))
    lm = np.sqrt(shs / max_kl)
    fullstep = stepdir / lm
    neggdotstepdir = -g.dot(stepdir)
    lossc = _Counter(loss)
    theta = U.linesearch(lossc, thprev, fullstep, neggdotstepdir / lm)
    k = -1 if theta is thprev else lossc.calls - 2
    sff(theta)
    losses_after = G.losses(state["theta"])
    reverted = bool(losses_after[1] > 2.0 * max_kl)
    if reverted:
        sff(thprev)
    theta_new = state["theta"].copy()

    # and the closed-form oracle must reproduce the whole tuple
    res = O.trpo_update(thprev, O.Batch(X, a, adv, old), spec, np.float64, 10, residual_tol, max_kl)
    assert res.cg_iters == cg_iters and res.k == k and res.reverted == reverted, (res.cg_iters, cg_iters, res.k, k)
    assert np.linalg.norm(res.theta_new - theta_new) <= 1e-10 * np.linalg.norm(theta_new)

    _save(f"update_{name}.npz",
          obs_dim=np.int64(spec.obs_dim), hidden=np.array(list(spec.hidden), np.int64),
          n_actions=np.int64(spec.n_actions), max_kl=np.float64(max_kl),
          residual_tol=np.float64(residual_tol), episode_len=np.int64(episode_len),
          X=X, actions=a, rewards=d["rewards"], starts=d["starts"], returns=d["returns"],
          advant=adv, old_dist=old, theta=d["theta"],
          v=v, hv=hv_tf, g=g, stepdir=stepdir, cg_iters=np.int64(cg_iters), shs=np.float64(shs),
          lm=np.float64(lm), fullstep=fullstep, rate=np.float64(neggdotstepdir / lm),
          k=np.int64(k), theta_ls=np.asarray(theta, np.float64), losses_before=losses_before,
          losses_after=losses_after, reverted=np.bool_(reverted), theta_new=theta_new)
    print(f"  {name}: P={spec.n_params} iters={cg_iters} k={k} reverted={reverted} "
          f"kl={losses_after[1]:.4g} fvp-crosscheck={rel:.2e}")


def gen_rollout(U):
    """The reference's own ``rollout`` (utils.py:18-45) and ``cat_sample`` (utils.py:95-105) driving
    the CartPole-v0 restatement and a float32 policy agent (oracle/cartpole_oracle.py).  The
    uniforms both RNGs produced are recorded, so the device rollout can be fed the same draws."""
    from oracle.cartpole_oracle import CartPoleV0, OracleAgent
    spec = O.PolicySpec(4, [64], 2)
    out = {}
    for tag, seed, n_timesteps, train in (("a", 11, 1000, True), ("b", 12, 450, True), ("c", 13, 300, False)):
        rng = np.random.RandomState(seed)
        theta = np.concatenate([np.concatenate([rng.uniform(-np.sqrt(6 / (a + b)), np.sqrt(6 / (a + b)), a * b),
                                                0.3 * rng.standard_normal(b)])
                                for a, b in zip(spec.widths[:-1], spec.widths[1:])]).astype(np.float32)
        env = CartPoleV0(seed=100 + seed)
        agent = OracleAgent(theta, spec.widths, U.cat_sample, train=train)
        np.random.seed(200 + seed)
        paths = U.rollout(env, agent, 1000, n_timesteps)
        n = sum(len(p["rewards"]) for p in paths)
        starts = np.concatenate([np.r_[1, np.zeros(len(p["rewards"]) - 1)] for p in paths]).astype(np.uint8)
        out[tag + "_theta"] = theta
        out[tag + "_n_timesteps"] = np.int64(n_timesteps)
        out[tag + "_train"] = np.bool_(train)
        out[tag + "_obs"] = np.concatenate([p["obs"] for p in paths]).astype(np.float64)
        out[tag + "_actions"] = np.concatenate([p["actions"] for p in paths]).astype(np.int64)
        out[tag + "_action_dists"] = np.concatenate([p["action_dists"] for p in paths]).astype(np.float32)
        out[tag + "_rewards"] = np.concatenate([p["rewards"] for p in paths]).astype(np.float64)
        out[tag + "_starts"] = starts
        # the draws: np.random.rand(1) per act() in training, 4 per env.reset()
        out[tag + "_act_uniforms"] = np.random.RandomState(200 + seed).random_sample(n) if train else np.zeros(n)
        out[tag + "_reset_uniforms"] = np.random.RandomState(100 + seed).random_sample(4 * len(paths))
        print(f"  rollout {tag}: {len(paths)} paths, {n} steps")
    rng = np.random.RandomState(5)
    prob = rng.dirichlet(np.ones(7), 400).astype(np.float32)
    prob[:50] = np.float32(1.0 / 7)                       # cumsum can end below r (out stays 0)
    r = np.random.RandomState(9).random_sample(400)
    prob[:10] *= np.float32(0.999)                        # cumsum ends at 0.999 < r = 0.9995:
    r[:10] = 0.9995                                       # the reference's zeros-init fallback
    # cat_sample draws np.random.rand(N) itself: call it per row with np.random.rand
    # temporarily returning r[i]
    vals = []
    orig = U.np.random.rand
    try:
        for i in range(400):
            U.np.random.rand = (lambda *a, _v=r[i]: np.array([_v]))
            vals.append(int(U.cat_sample(prob[i:i + 1])[0]))
    finally:
        U.np.random.rand = orig
    out["cat_prob"] = prob
    out["cat_r"] = r
    out["cat_out"] = np.array(vals, np.int64)
    _save("rollout.npz", **out)


def main(only=None):
    U = load_reference_utils()
    if only == "rollout":
        gen_rollout(U)
        return
    gen_rollout(U)
    gen_discount(U)
    gen_cg(U)
    gen_linesearch(U)
    gen_explained_variance(U)
    gen_update(U, "c1", O.PolicySpec(4, [64], 2), 1000, seed=1)
    gen_update(U, "c2", O.PolicySpec(11, [64, 64], 3), 2000, seed=2)
    gen_update(U, "c3", O.PolicySpec(128, [64, 64], 18), 1500, seed=3)
    gen_update(U, "c3_perturbed", O.PolicySpec(128, [64, 64], 18), 1500, seed=4,
               steady=False, perturb=0.3)
    gen_update(U, "c2_bigkl", O.PolicySpec(11, [64, 64], 3), 2000, seed=5, max_kl=100.0)
    gen_update(U, "deep_odd", O.PolicySpec(7, [40, 24, 33], 5), 777, seed=6, episode_len=50)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
