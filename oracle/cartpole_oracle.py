"""CPU oracle for sampling and rollouts — TEST INFRASTRUCTURE ONLY.

The checker for ``trpo_act`` / ``trpo_cat_sample`` / ``trpo_cartpole_step`` /
``trpo_rollout_cartpole``; never imported by the product.

* ``CartPoleV0`` — the environment ``trpo_inksci.py:179`` makes (``gym.make("CartPole-v0")``).
  gym is not vendored in the reference (and not installed), so this restates its published
  ``classic_control/cartpole.py`` (Euler integration, float64 Python arithmetic, ``reset`` to
  ``U(-0.05, 0.05)^4``, termination past ``|x| > 2.4`` or ``|theta| > 12 deg``, reward 1 per step)
  plus the v0 ``TimeLimit(max_episode_steps=200)``.  Its reset draws come from a numpy
  ``RandomState``: ``uniform(-0.05, 0.05, 4)`` = ``-0.05 + 0.1 * random_sample(4)``.
* ``cat_sample`` — ``utils.py:95-105`` with the uniforms passed in.
* ``OracleAgent`` — ``agent.act`` (``trpo_inksci.py:76-87``): float32 policy forward on one
  state, the reference's ``cat_sample`` draws ``np.random.rand(1)``.
* ``rollout_envs`` — the engine's batched rollout restated: each of ``n_envs`` environments runs
  utils.py:23-44's loop with budget ``ceil(n_timesteps / n_envs)``, concatenated in env order.
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence

import numpy as np


class CartPoleV0:
    gravity = 9.8
    masscart = 1.0
    masspole = 0.1
    total_mass = masspole + masscart
    length = 0.5
    polemass_length = masspole * length
    force_mag = 10.0
    tau = 0.02
    theta_threshold_radians = 12 * 2 * math.pi / 360
    x_threshold = 2.4
    max_episode_steps = 200

    def __init__(self, seed: int = 0, reset_uniforms=None):
        self.np_random = np.random.RandomState(seed)
        self._ru = None if reset_uniforms is None else list(np.asarray(reset_uniforms, np.float64).reshape(-1))
        self.state = None
        self._elapsed = 0

    def reset(self):
        if self._ru is not None:
            u = np.array([self._ru.pop(0) for _ in range(4)])
            self.state = -0.05 + (0.05 - -0.05) * u
        else:
            self.state = self.np_random.uniform(low=-0.05, high=0.05, size=(4,))
        self._elapsed = 0
        return np.array(self.state)

    @classmethod
    def dynamics(cls, state, action):
        x, x_dot, theta, theta_dot = [float(v) for v in state]
        force = cls.force_mag if action == 1 else -cls.force_mag
        costheta = math.cos(theta)
        sintheta = math.sin(theta)
        temp = (force + cls.polemass_length * theta_dot ** 2 * sintheta) / cls.total_mass
        thetaacc = (cls.gravity * sintheta - costheta * temp) / (
            cls.length * (4.0 / 3.0 - cls.masspole * costheta ** 2 / cls.total_mass))
        xacc = temp - cls.polemass_length * thetaacc * costheta / cls.total_mass
        x = x + cls.tau * x_dot
        x_dot = x_dot + cls.tau * xacc
        theta = theta + cls.tau * theta_dot
        theta_dot = theta_dot + cls.tau * thetaacc
        done = x < -cls.x_threshold or x > cls.x_threshold or \
            theta < -cls.theta_threshold_radians or theta > cls.theta_threshold_radians
        return (x, x_dot, theta, theta_dot), bool(done)

    def step(self, action):
        self.state, done = self.dynamics(self.state, action)
        self._elapsed += 1
        if self._elapsed >= self.max_episode_steps:
            done = True
        return np.array(self.state), 1.0, done, {}


def cat_sample(prob_nk, r):
    prob_nk = np.asarray(prob_nk)
    assert prob_nk.ndim == 2
    csprob_nk = np.cumsum(prob_nk, axis=1)
    out = np.zeros(prob_nk.shape[0], dtype=np.int64)
    for n, (csprob_k, rn) in enumerate(zip(csprob_nk, r)):
        for k, csprob in enumerate(csprob_k):
            if csprob > rn:
                out[n] = k
                break
    return out


def policy_dist32(theta, state, widths: Sequence[int]):
    """float32 policy forward (trpo_inksci.py:38-40) on states [n, obs]."""
    h = np.asarray(state, np.float32).reshape(-1, widths[0])
    o = 0
    L = len(widths) - 1
    for l in range(L):
        a, b = widths[l], widths[l + 1]
        W = np.asarray(theta[o:o + a * b], np.float32).reshape(a, b)
        bias = np.asarray(theta[o + a * b:o + a * b + b], np.float32)
        o += a * b + b
        z = h @ W + bias
        h = np.tanh(z) if l < L - 1 else z
    m = h.max(axis=1, keepdims=True)
    ex = np.exp(h - m)
    return (ex / ex.sum(axis=1, keepdims=True)).astype(np.float32)


class OracleAgent:
    """The agent surface utils.rollout touches (act, prev_action); cat_sample is supplied so the
    reference's own function can be used."""

    def __init__(self, theta, widths, cat_sample_fn, train=True):
        self.theta = np.asarray(theta, np.float32)
        self.widths = list(widths)
        self.cat_sample = cat_sample_fn
        self.train = train
        self.prev_action = np.zeros((1, widths[-1]))

    def act(self, state):
        state = np.expand_dims(state, 0)
        action_dist = policy_dist32(self.theta, state, self.widths)
        if self.train:
            action = int(self.cat_sample(action_dist)[0])
        else:
            action = int(np.argmax(action_dist))
        self.prev_action *= 0.0
        self.prev_action[0, action] = 1.0
        return action, action_dist, np.squeeze([state])


def rollout_envs(theta, widths, n_envs, n_timesteps, reset_u, act_u, max_pathlength=1000, time_limit=200,
                 dists_from=None, train=True):
    """The engine's batched rollout with injected uniforms: reset_u [n_envs][max_eps][4],
    act_u [n_envs][env_cap].  dists_from: optional recorded action_dists [N, A] to sample from
    instead of recomputing (replay mode).  Returns the concatenated arrays."""
    budget = -(-n_timesteps // n_envs)
    ep_max = min(max_pathlength, time_limit)
    env_cap = budget + ep_max - 1
    obs, acts, dists, rews, starts, us = [], [], [], [], [], []
    row = 0
    for e in range(n_envs):
        count, ep = 0, 0
        while count < budget:
            s = -0.05 + (0.05 - -0.05) * np.asarray(reset_u[e][ep], np.float64)
            ep += 1
            for t in range(max_pathlength):
                d = dists_from[row:row + 1] if dists_from is not None else policy_dist32(theta, s, widths)
                r = act_u[e][count]
                a = int(cat_sample(d, [r])[0]) if train else int(np.argmax(d[0]))
                obs.append(np.array(s))
                acts.append(a)
                dists.append(d[0])
                rews.append(1.0)
                starts.append(1 if t == 0 else 0)
                us.append(r)
                s, done = CartPoleV0.dynamics(s, a)
                s = np.array(s)
                count += 1
                row += 1
                if done or t + 1 >= time_limit:
                    break
        assert count <= env_cap
    return {"obs": np.array(obs), "actions": np.array(acts, np.int64), "action_dists": np.array(dists, np.float32),
            "rewards": np.array(rews), "starts": np.array(starts, np.uint8), "uniforms": np.array(us)}
