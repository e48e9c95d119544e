"""CPU oracle of the learn() loop — TEST INFRASTRUCTURE ONLY (never imported by the product).

Restates ``TRPOAgent.learn`` (trpo_inksci.py:88-176) for one CartPole-v0 environment with the
random draws injected, on the other oracles:

* rollout      ``cartpole_oracle.rollout_envs`` with n_envs = 1 (utils.py:18-45's loop; pinned by
               tests/golden/rollout.npz, recorded from the reference's own rollout / cat_sample);
* baseline     ``vf_oracle.predict`` on ``features_concat`` (utils.py:70-77,87-92), zeros before the
               first fit (:88-89);
* advantages   ``discount_segmented`` + ``standardize`` (trpo_inksci.py:102-117);
* VF fit       ``vf_oracle.fit`` with one persistent TF-Adam state (utils.py:79-85); the first fit
               creates the net and re-initialises the policy too (utils.py:67,
               ``tf.initialize_all_variables()``), so iteration 0 updates a re-drawn theta against
               the old rollout's action_dist;
* update       ``trpo_oracle.trpo_update`` (trpo_inksci.py:144-158);
* stop rules   mean reward > 1.1*500 or explained variance > 0.8 -> argmax rollouts, break after
               100 of them; NaN entropy -> exit (:131-141,172-175).
"""
from __future__ import annotations

from typing import Callable, List, Sequence

import numpy as np

from . import cartpole_oracle as C
from . import trpo_oracle as O
from . import vf_oracle as V

CONFIG = {"max_steps": 1000, "episodes_per_roll": 1000, "gamma": 0.95, "cg_damping": 0.1, "max_kl": 0.01}


def learn(theta0, widths: Sequence[int], iterations: int, draws: Callable[[int], tuple],
          reinit_theta, vf_init: Callable[[int], np.ndarray], policy_dtype=np.float64, vf_dtype=np.float32,
          explained_variance_override=None, dists_from: Callable[[int], np.ndarray] = None) -> List[dict]:
    """theta0: the agent's initial parameters; reinit_theta: those tf.initialize_all_variables()
    draws at the first VF fit; vf_init(F): the VF net's initial parameters.  dists_from(i): sample
    iteration i's actions from these recorded action_dists (replay mode: the loop follows a
    recorded trajectory, and rec["policy_dists"] holds this oracle's own policy on its states)."""
    spec = O.PolicySpec(widths[0], list(widths[1:-1]), widths[-1])
    theta = np.asarray(theta0, np.float32)
    vf_theta, adam = None, None
    train, end_count, numeptotal = True, 0, 0
    hist = []
    for i in range(iterations):
        ru, au, _me = draws(i)
        rec_d = dists_from(i) if dists_from is not None else None
        ro = C.rollout_envs(theta, widths, 1, CONFIG["episodes_per_roll"], ru, au,
                            max_pathlength=CONFIG["max_steps"], train=train, dists_from=rec_d)
        n = len(ro["rewards"])
        policy_dists = C.policy_dist32(theta, ro["obs"], widths) if rec_d is not None else ro["action_dists"]
        feat = V.features_concat(ro["obs"].astype(np.float32), ro["action_dists"], ro["starts"])
        baseline = (np.zeros(n) if vf_theta is None else
                    V.predict(vf_theta, feat, dtype=vf_dtype).astype(np.float64))
        returns = O.discount_segmented(ro["rewards"], ro["starts"], CONFIG["gamma"])
        adv = O.standardize(returns - baseline)
        starts_idx = np.flatnonzero(ro["starts"])
        episoderewards = np.add.reduceat(ro["rewards"], starts_idx)
        rec = {"iteration": i, "steps": n, "paths": len(starts_idx), "train": train, "rollout": ro,
               "policy_dists": policy_dists,
               "baseline": baseline, "returns": returns, "advantages": adv,
               "reward_mean": float(episoderewards.mean())}
        if episoderewards.mean() > 1.1 * 500:
            train = False
        if not train:
            end_count += 1
            rec["end_count"] = end_count
            if end_count > 100:
                hist.append(rec)
                break
        if train:
            if vf_theta is None:                      # create_net: VF init + global re-init
                vf_theta = np.asarray(vf_init(feat.shape[1]), np.float32)
                adam = V.Adam(vf_theta.size, dtype=vf_dtype)
                theta = np.asarray(reinit_theta, np.float32)
            vf_theta, adam = V.fit(vf_theta, feat, returns.astype(np.float32), adam=adam, dtype=vf_dtype)
            vf_theta = vf_theta.astype(np.float32)
            r = O.trpo_update(theta.astype(policy_dtype),
                              O.Batch(ro["obs"].astype(np.float32), ro["actions"], adv, ro["action_dists"]),
                              spec, policy_dtype, 10, 1e-10, CONFIG["max_kl"], CONFIG["cg_damping"])
            theta = np.asarray(r.theta_new, np.float32)
            numeptotal += len(episoderewards)
            exp = O.explained_variance(baseline, returns)
            if explained_variance_override is not None:
                exp = explained_variance_override(i, exp)
            surr, kl, ent = (float(x) for x in r.losses_after)
            rec.update({"entropy": ent, "kl": kl, "surr": surr, "explained_variance": float(exp),
                        "reverted": r.reverted, "k": r.k, "cg_iters": r.cg_iters, "shs": r.shs,
                        "episodes": numeptotal, "theta": theta.copy()})
            hist.append(rec)
            if ent != ent:
                rec["nan_exit"] = True
                break
            if exp > 0.8:
                train = False
        else:
            hist.append(rec)
    return hist
