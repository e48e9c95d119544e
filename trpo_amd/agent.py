"""``TRPOAgent`` — the update block of ``trpo_inksci.py:101-158`` on the HIP engine.

Two ways to run one policy update, both on the GPU:

* :meth:`TRPOAgent.update` — the fused path: one ``trpo_update`` C-ABI call does
  discount + standardise + pg + CG + step scaling + line search + revert on
  the device with no host round trip except the line search's accept flag.
* :meth:`TRPOAgent.update_stepwise` — the reference's block written line for
  line over the ``trpo_amd.utils`` surface (``conjugate_gradient``,
  ``linesearch``, ``GetFlat``/``SetFromFlat``), i.e. what
  ``trpo_inksci.py`` looks like once its TF session is replaced.

Rollout and the value-function baseline are outside the hot path (SURVEY.md
§8(f)); paths come in as the reference's dicts (``utils.py:36-39``) with an
optional ``"baseline"`` entry (zeros otherwise, as ``VF.predict`` returns before
its first fit, ``utils.py:88-89``).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np

from .engine import Engine, UpdateParams
from .utils import (EngineLoss, FisherVectorProduct, GetFlat, SetFromFlat, SurrogateLoss,
                    conjugate_gradient, flatgrad, linesearch)

CONFIG = {"max_steps": 1000, "episodes_per_roll": 1000, "gamma": 0.95, "cg_damping": 0.1,
          "max_kl": 0.01}   # trpo_inksci.py:17


class Session:
    """Stands in for the ``tf.Session`` the reference threads through utils (trpo_inksci.py:23)."""

    def __init__(self, engine: Engine):
        self.engine = engine


def xavier_theta(obs_dim: int, hidden: Sequence[int], n_actions: int,
                 rng: Optional[np.random.RandomState] = None) -> np.ndarray:
    """Initial parameters: W ~ U(+-sqrt(6/(fan_in+fan_out))), b = 0 (prettytensor's
    fully_connected defaults, trpo_inksci.py:38-40), flat in var_list order."""
    rng = rng or np.random.RandomState(1)   # utils.py:7-9 seed
    widths = [obs_dim, *hidden, n_actions]
    parts = []
    for a, b in zip(widths[:-1], widths[1:]):
        lim = math.sqrt(6.0 / (a + b))
        parts.append(rng.uniform(-lim, lim, size=a * b))
        parts.append(np.zeros(b))
    return np.concatenate(parts).astype(np.float32)


def paths_to_batch(paths: List[Dict]) -> Dict[str, np.ndarray]:
    """Concatenate rollout paths (trpo_inksci.py:108-115) and mark episode starts."""
    starts = []
    for path in paths:
        s = np.zeros(len(path["rewards"]), np.uint8)
        s[0] = 1
        starts.append(s)
    obs = np.concatenate([np.asarray(p["obs"], np.float32).reshape(len(p["rewards"]), -1) for p in paths])
    out = {
        "state": obs,
        "action_dist": np.concatenate([np.asarray(p["action_dists"], np.float32).reshape(len(p["rewards"]), -1)
                                       for p in paths]),
        "action": np.concatenate([np.asarray(p["actions"], np.int64) for p in paths]),
        "rewards": np.concatenate([np.asarray(p["rewards"], np.float64) for p in paths]),
        "baseline": np.concatenate([np.asarray(p.get("baseline", np.zeros(len(p["rewards"]))), np.float64)
                                    for p in paths]),
        "starts": np.concatenate(starts),
    }
    return out


class TRPOAgent:
    def __init__(self, obs_dim: int, n_actions: int, hidden: Sequence[int] = (64,), max_rows: int = 4096,
                 device: int = 0, theta: Optional[np.ndarray] = None, config: Optional[dict] = None):
        self.config = dict(CONFIG if config is None else config)
        self.engine = Engine(obs_dim, hidden, n_actions, max_rows, device)
        self.session = Session(self.engine)
        self.gf = GetFlat(self.session)                          # trpo_inksci.py:71
        self.sff = SetFromFlat(self.session)                     # :72
        self.pg = flatgrad(SurrogateLoss(self.engine))           # :54
        self.sff(xavier_theta(obs_dim, hidden, n_actions) if theta is None else theta)

    def feed(self, paths_or_batch, n_global: Optional[int] = None):
        """The feed dict of trpo_inksci.py:119-122 (+ rewards for :102-117)."""
        b = paths_to_batch(paths_or_batch) if isinstance(paths_or_batch, list) else paths_or_batch
        self.engine.set_batch(b["state"], b["action"], b.get("advant"), b["action_dist"], n_global)
        if "rewards" in b:
            self.engine.set_rewards(b["rewards"], b["starts"], b.get("baseline"))
        return b

    def update(self, paths_or_batch, n_global: Optional[int] = None, cg_iters: int = 10,
               residual_tol: float = 1e-10) -> dict:
        """trpo_inksci.py:101-158 as one device call."""
        b = self.feed(paths_or_batch, n_global)
        prm = UpdateParams(cg_iters=cg_iters, residual_tol=residual_tol,
                           cg_damping=self.config["cg_damping"], max_kl=self.config["max_kl"],
                           compute_advantages="rewards" in b, gamma=self.config["gamma"])
        return self.engine.update(prm)

    def update_stepwise(self, paths_or_batch, n_global: Optional[int] = None) -> dict:
        """trpo_inksci.py:101-158 line for line over the utils surface."""
        b = self.feed(paths_or_batch, n_global)
        if "rewards" in b:
            self.engine.compute_advantages(self.config["gamma"])      # :102-117
        fisher_vector_product = FisherVectorProduct(self.engine, self.config["cg_damping"])   # :124-126
        loss = EngineLoss(self.engine)                                                        # :127-129
        thprev = self.gf()                                                     # :144
        g = self.pg()                                                          # :146
        stepdir = conjugate_gradient(fisher_vector_product, -g)                # :147
        shs = .5 * float(stepdir.dot(fisher_vector_product(stepdir)))         # :148
        lm = np.sqrt(shs / self.config["max_kl"])                              # :149
        fullstep = (stepdir / np.float32(lm)).astype(np.float32)               # :150
        neggdotstepdir = -g.dot(stepdir)                                       # :151
        theta = linesearch(loss, thprev, fullstep, float(neggdotstepdir) / lm)   # :153
        self.sff(theta)                                                        # :154
        surrafter, kloldnew, entropy = self.engine.losses()                    # :156
        reverted = bool(kloldnew > 2.0 * self.config["max_kl"])
        if reverted:                                                           # :157-158
            self.sff(thprev)
        return {"surr_after": float(surrafter), "kl_after": float(kloldnew), "ent_after": float(entropy),
                "reverted": reverted, "shs": shs, "lm": float(lm)}
