"""``TRPOAgent`` — the update block of ``trpo_inksci.py:101-158`` on the HIP engine.

Two ways to run one policy update, both on the GPU:

* :meth:`TRPOAgent.update` — the fused path: one ``trpo_update`` C-ABI call does
  discount + standardise + pg + CG + step scaling + line search + revert on
  the device with no host round trip except the line search's accept flag.
* :meth:`TRPOAgent.update_stepwise` — the reference's block written line for
  line over the ``trpo_amd.utils`` surface (``conjugate_gradient``,
  ``linesearch``, ``GetFlat``/``SetFromFlat``), i.e. what
  ``trpo_inksci.py`` looks like once its TF session is replaced.

* :meth:`TRPOAgent.learn` — the whole loop of ``trpo_inksci.py:89-177`` on the
  device: CartPole-v0 rollouts (``rollout.hip``), VF baselines and fit
  (``vf.hip``), advantages, the update, explained variance and the reference's
  stop rules; only the print-out statistics come back to the host.

For the update methods, paths come in as the reference's dicts
(``utils.py:36-39``) with an optional ``"baseline"`` entry (zeros otherwise, as
``VF.predict`` returns before its first fit, ``utils.py:88-89``).
"""
from __future__ import annotations

import math
import time
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np

from .engine import Engine, UpdateParams
from .vf import VF
from .utils import (EngineLoss, GetFlat, KLFirstFixedGVP, SetFromFlat, SurrogateLoss, conjugate_gradient,
                    flatgrad, linesearch)

CONFIG = {"max_steps": 1000, "episodes_per_roll": 1000, "gamma": 0.95, "cg_damping": 0.1,
          "max_kl": 0.01}   # trpo_inksci.py:17


class Session:
    """Stands in for the ``tf.Session`` the reference threads through utils (trpo_inksci.py:23)."""

    def __init__(self, engine: Engine, init_rng: Optional[np.random.RandomState] = None,
                 reinit_policy: bool = True):
        self.engine = engine
        self.init_rng = init_rng or np.random.RandomState(1)
        self.reinit_policy = reinit_policy

    def initialize_all_variables(self):
        """tf.initialize_all_variables() re-draws every variable, the policy included; the reference
        runs it again when the VF creates its net (utils.py:66), so its first update starts from a
        fresh initialisation.  reinit_policy=False keeps the current policy instead."""
        if self.reinit_policy:
            e = self.engine
            self.engine.set_flat(xavier_theta(e.obs_dim, e.hidden, e.n_actions, self.init_rng))


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


def rollout_seed(seed: int, iteration: int, rank: int) -> int:
    """The Philox key of one rank's rollout at one iteration: ranks live 2^40 keys apart, so no rank
    ever draws another rank's stream at any reachable iteration count."""
    return (seed * 1000003 + iteration + (rank << 40)) & ((1 << 64) - 1)


class TRPOAgent:
    def __init__(self, obs_dim: int, n_actions: int, hidden: Sequence[int] = (64,), max_rows: int = 4096,
                 device: int = 0, theta: Optional[np.ndarray] = None, config: Optional[dict] = None,
                 reinit_policy: bool = True):
        self.config = dict(CONFIG if config is None else config)
        self.engine = Engine(obs_dim, hidden, n_actions, max_rows, device)
        self.session = Session(self.engine, reinit_policy=reinit_policy)
        self.gf = GetFlat(self.session)                          # trpo_inksci.py:71
        self.sff = SetFromFlat(self.session)                     # :72
        self.pg = flatgrad(SurrogateLoss(self.engine))           # :54
        self.fvp = flatgrad(KLFirstFixedGVP(self.engine))        # :56-70 (flatgrad(gvp))
        self.sff(xavier_theta(obs_dim, hidden, n_actions, self.session.init_rng) if theta is None else theta)
        self.train = True                                        # :28
        self.end_count = 0                                       # :29
        self.vf = VF(self.session, max_rows=max_rows, device=device)   # :73
        self.rank, self.world, self.group = 0, 1, None

    def set_ranks(self, rank: int, world: int, group=None, host_allreduce: bool = False):
        """Run learn() as one of `world` ranks (one process per GPU, torch.distributed initialised by the
        caller; `group` a gloo group for the host-side scalars, None = the default group, which must then
        be gloo). Each rank rolls out its own share of the episode budget; the update's partial sums,
        the advantage standardisation, the explained variance and the VF gradient are summed over the
        ranks (the engine's and the VF's RCCL communicators, or with host_allreduce the stream-ordered
        host transport over gloo, for ranks that share a GPU). Policy and VF parameters start identical
        on every rank and stay so: every rank applies the same all-reduced step."""
        self.rank, self.world, self.group = int(rank), int(world), group
        if self.world <= 1:
            return
        import torch
        import torch.distributed as dist
        from .dist import broadcast_unique_id, init_engine_comm

        def ar(arr):
            dist.all_reduce(torch.from_numpy(arr), group=group)

        if host_allreduce:
            self.engine.comm_set_host_allreduce(ar, self.rank, self.world)
        else:
            init_engine_comm(self.engine, self.rank, self.world, group)

        def vf_comm(net):   # the VF net is created at its first fit (utils.py:83)
            if host_allreduce:
                net.comm_set_host_allreduce(ar, self.rank, self.world)
            else:
                net.comm_init(broadcast_unique_id(Engine.comm_unique_id, self.rank, group), self.rank, self.world)

        self.vf.on_create = vf_comm
        if self.vf.net is not None:   # set_ranks after a fit: the existing net's gradient is summed from now on
            vf_comm(self.vf.net)

    def _host_sum(self, *vals: float) -> np.ndarray:
        """Sum of host scalars over the ranks (gloo), float64; identity for one rank."""
        a = np.array(vals, np.float64)
        if self.world > 1:
            import torch
            import torch.distributed as dist
            t = torch.from_numpy(a)
            dist.all_reduce(t, group=self.group)
        return a

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
        fisher_vector_product = self.fvp.damped(self.config["cg_damping"])                   # :124-126
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

    # ------------------------------------------------------------------ trpo_inksci.py:89-177
    def learn(self, max_iterations: Optional[int] = None, n_envs: int = 1, seed: int = 1,
              log: Optional[Callable[[str], None]] = print,
              draws: Optional[Callable[[int], tuple]] = None, record: bool = False) -> List[dict]:
        """The reference's learn() loop on CartPole-v0, device-resident.  Stop rules as
        trpo_inksci.py:131-141,172-175: training stops when the mean episode reward exceeds
        1.1*500 or the baseline explains > 0.8 of the returns' variance; the loop then keeps
        rolling out the argmax policy and ends after 100 such iterations; a NaN entropy ends it
        (the reference calls exit(-1)).  max_iterations bounds the loop (None: as the reference).
        draws(i) -> (reset_uniforms, action_uniforms, max_episodes_per_env) injects the random draws
        of iteration i's rollout (env.reset and cat_sample; tests), else a Philox stream per iteration.
        record=True also returns each iteration's rollout arrays, baselines, returns and
        standardised advantages (host copies; parity tests).
        Returns one stats dict per iteration."""
        cfg = self.config
        eng = self.engine
        # this rank's share of the timestep budget (trpo_inksci.py:96-100 over `world` ranks)
        n_timesteps = -(-cfg["episodes_per_roll"] // self.world)
        # worst case rows of one rollout: every environment overshoots its budget by one episode
        budget = -(-n_timesteps // n_envs)
        worst = n_envs * (budget + min(cfg["max_steps"], 200) - 1)
        if worst > eng.max_rows:
            raise ValueError(f"learn(): a rollout of {n_envs} environments can reach {worst} steps, more than "
                             f"max_rows={eng.max_rows}; create the agent with max_rows >= {worst}")
        say = log or (lambda _s: None)
        start_time = time.time()
        i = 0
        numeptotal = 0
        history = []
        while max_iterations is None or i < max_iterations:
            say("Rollout")
            inj = {}
            if draws is not None:
                ru, au, me = draws(i)
                inj = {"reset_uniforms": ru, "action_uniforms": au, "max_episodes_per_env": me}
            n, n_paths = eng.rollout_cartpole(n_envs=n_envs, n_timesteps=n_timesteps,
                                              max_pathlength=cfg["max_steps"],
                                              seed=rollout_seed(seed, i, self.rank),
                                              train=self.train, **inj)                   # :96-100
            n_global = int(self._host_sum(n)[0])
            eng.rollout_to_batch(n_global=n_global)                                      # :108-122
            have_base = self.vf.predict_engine(eng)                                      # :103
            if record:
                rb = self.vf.net.predict(np.empty(n, np.float64)) if have_base else np.zeros(n)
                r_ret, r_adv = np.empty(n), np.empty(n)
                eng.compute_advantages_device(cfg["gamma"], returns_out=r_ret, advant_out=r_adv)
            else:
                eng.compute_advantages_device(cfg["gamma"])                              # :104-117
            ep = eng.rollout_fetch_stats()
            episoderewards = np.add.reduceat(ep["rewards"], np.flatnonzero(ep["starts"]))   # :131
            # the mean over every rank's episodes (one rank: episoderewards.mean())
            ep_sum, ep_cnt = self._host_sum(episoderewards.sum(), len(episoderewards))
            reward_mean = ep_sum / ep_cnt if self.world > 1 else float(episoderewards.mean())
            say("\n********** Iteration %i ************" % i)
            rec = {"iteration": i, "steps": n, "paths": n_paths, "train": self.train,
                   "reward_mean": float(reward_mean), "end_count": self.end_count}
            if record:
                rec.update({"rollout": eng.rollout_fetch(), "baseline": rb, "returns": r_ret, "advantages": r_adv})
            if reward_mean > 1.1 * 500:                                                  # :135-136
                self.train = False
            rec["train"] = self.train                    # whether this iteration updates the policy
            if not self.train:                                                           # :137-141
                say("Episode mean: %f" % reward_mean)
                self.end_count += 1
                rec["end_count"] = self.end_count
                if self.end_count > 100:
                    history.append(rec)
                    break
            if self.train:
                self.vf.fit_engine(eng)                                                  # :143
                if record:
                    rec["theta_before"] = eng.get_flat().copy()
                st = eng.update(UpdateParams(cg_iters=10, residual_tol=1e-10, cg_damping=cfg["cg_damping"],
                                             max_kl=cfg["max_kl"], compute_advantages=False))     # :144-158
                if record:
                    rec["theta"] = eng.get_flat().copy()
                    rec["vf_params"] = self.vf.net.get_params().copy()
                numeptotal += int(ep_cnt)
                exp = eng.explained_variance()                                           # :167
                stats = {
                    "Total number of episodes": numeptotal,
                    "Average sum of rewards per episode": reward_mean,
                    "Entropy": st["ent_after"],
                    "Baseline explained": exp,
                    "Time elapsed": "%.2f mins" % ((time.time() - start_time) / 60.0),
                    "KL between old and new distribution": st["kl_after"],
                    "Surrogate loss": st["surr_after"],
                }
                for k, v in stats.items():
                    say(k + ": " + " " * (40 - len(k)) + str(v))
                rec.update({"entropy": float(st["ent_after"]), "kl": float(st["kl_after"]),
                            "surr": float(st["surr_after"]), "explained_variance": float(exp),
                            "reverted": bool(st["reverted"]), "k": int(st["k"]), "episodes": numeptotal,
                            "cg_iters": int(st["cg_iters"]), "shs": float(st["shs"])})
                history.append(rec)
                if st["ent_after"] != st["ent_after"]:                                    # :172-173
                    rec["nan_exit"] = True
                    break
                if exp > 0.8:                                                            # :174-175
                    self.train = False
            else:
                history.append(rec)
            i += 1
        return history
