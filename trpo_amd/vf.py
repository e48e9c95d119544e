"""Value-function baseline on the GPU: the reference's ``class VF`` (``utils.py:48-92``).

:class:`VFNet` is the thin handle over the ``trpo_vf_*`` C-ABI (features, targets, Adam fit,
predict, all on the device).  :class:`VF` mirrors the reference class line for line:

=====================  ===========================================================
reference              here
=====================  ===========================================================
``VF(session)``        ``VF(session)``
``create_net(shape)``  lazily at the first ``fit``; calls ``session.initialize_all_variables()``
                       like ``utils.py:66`` (which re-draws the *policy* too)
``_features(path)``    same: ``[obs | action_dists | arange(l)/10]``
``fit(paths)``         50 full-batch Adam steps on ``sum((net - y)^2)`` (``utils.py:79-85``)
``predict(path)``      zeros before the first fit, else the net (``utils.py:87-92``)
=====================  ===========================================================

Initialisation: prettytensor's ``fully_connected`` defaults as SURVEY.md §8(c) records them
(weights Xavier-uniform ``U(+-sqrt(6/(fan_in+fan_out)))``, biases zero); the draws come from a
numpy ``RandomState`` (TF's graph RNG cannot be reproduced).
"""
from __future__ import annotations

import ctypes
import math
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import MEM_DEVICE, MEM_HOST, check, lib
from .engine import _Arg, _is_torch

__all__ = ["VFNet", "VF", "vf_features", "vf_xavier_params"]

ADAM_DEFAULTS = (0.001, 0.9, 0.999, 1e-08)   # tf.train.AdamOptimizer() (utils.py:65)
FIT_STEPS = 50                               # utils.py:84


def vf_xavier_params(feat_dim: int, hidden: Sequence[int] = (64, 64),
                     rng: Optional[np.random.RandomState] = None) -> np.ndarray:
    rng = rng or np.random.RandomState(1)
    widths = [int(feat_dim), *[int(h) for h in hidden], 1]
    parts = []
    for a, b in zip(widths[:-1], widths[1:]):
        lim = math.sqrt(6.0 / (a + b))
        parts.append(rng.uniform(-lim, lim, size=a * b))
        parts.append(np.zeros(b))
    return np.concatenate(parts).astype(np.float32)


def vf_features(path: Dict) -> np.ndarray:
    """VF._features (utils.py:70-77), as the float32 matrix the placeholder receives."""
    o = np.asarray(path["obs"]).astype("float32")
    o = o.reshape(o.shape[0], -1)
    act = np.asarray(path["action_dists"]).astype("float32")
    act = act.reshape(act.shape[0], -1)
    l = len(path["rewards"])
    al = np.arange(l).reshape(-1, 1) / 10.0
    ret = np.concatenate([o, act, al], axis=1)
    return ret.astype(np.float32)


class VFNet:
    """The device-resident VF regressor (``trpo_vf_*``)."""

    def __init__(self, feat_dim: int, max_rows: int, hidden: Sequence[int] = (64, 64), device: int = 0):
        self.feat_dim = int(feat_dim)
        self.hidden = [int(h) for h in hidden]
        self.max_rows = int(max_rows)
        self.device = int(device)
        h = (ctypes.c_int * 2)(*self.hidden)
        handle = ctypes.c_void_p()
        check(lib.trpo_vf_create(ctypes.byref(handle), self.feat_dim, h, 2, self.max_rows, self.device),
              "trpo_vf_create")
        self._h = handle
        self.num_params = int(lib.trpo_vf_num_params(self._h))
        self.n = 0

    def close(self):
        if getattr(self, "_h", None):
            lib.trpo_vf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- parameters / optimizer
    def set_params(self, flat):
        a = _Arg(flat, np.float32, (self.num_params,))
        check(lib.trpo_vf_set_params(self._h, a.ptr, a.mem), "trpo_vf_set_params")

    def get_params(self) -> np.ndarray:
        out = np.empty(self.num_params, np.float32)
        check(lib.trpo_vf_get_params(self._h, out.ctypes.data_as(ctypes.c_void_p), MEM_HOST), "trpo_vf_get_params")
        return out

    def set_adam(self, lr=ADAM_DEFAULTS[0], beta1=ADAM_DEFAULTS[1], beta2=ADAM_DEFAULTS[2], epsilon=ADAM_DEFAULTS[3]):
        check(lib.trpo_vf_set_adam(self._h, float(lr), float(beta1), float(beta2), float(epsilon)), "trpo_vf_set_adam")

    def reset_optimizer(self):
        check(lib.trpo_vf_reset_optimizer(self._h), "trpo_vf_reset_optimizer")

    def optimizer_state(self) -> dict:
        m = np.empty(self.num_params, np.float32)
        v = np.empty(self.num_params, np.float32)
        pw = (ctypes.c_float * 2)()
        steps = ctypes.c_int64(0)
        check(lib.trpo_vf_get_optimizer(self._h, m.ctypes.data_as(ctypes.c_void_p), v.ctypes.data_as(ctypes.c_void_p),
                                        pw, ctypes.byref(steps), MEM_HOST), "trpo_vf_get_optimizer")
        return {"m": m, "v": v, "beta1_power": np.float32(pw[0]), "beta2_power": np.float32(pw[1]),
                "steps": steps.value}

    # ---------------------------------------------------------------- data
    def set_features(self, obs, action_dists, episode_starts=None, n_global: Optional[int] = None):
        """Features built on the device from concatenated paths (utils.py:70-77)."""
        n = int(obs.shape[0])
        obs_dim = int(np.prod(obs.shape[1:])) if len(obs.shape) > 1 else 1
        A = int(action_dists.shape[-1])
        o = _Arg(obs, np.float32, (n, obs_dim))
        d = _Arg(action_dists, np.float32, (n, A))
        if episode_starts is None:
            s = _Arg(None, np.uint8)
        else:
            s = _Arg(episode_starts if _is_torch(episode_starts) else np.asarray(episode_starts).astype(np.uint8),
                     np.uint8, (n,))
        if o.mem != d.mem or (s.ptr is not None and s.mem != o.mem):
            raise ValueError("set_features: pass all host arrays or all device tensors")
        check(lib.trpo_vf_set_features(self._h, n, n if n_global is None else int(n_global), o.ptr, obs_dim, d.ptr,
                                       A, s.ptr, o.mem), "trpo_vf_set_features")
        self.n = n

    def set_features_view(self, view, with_targets: bool = False):
        """Features (and the returns as targets) read in place from an engine feed view."""
        check(lib.trpo_vf_set_features_view(self._h, ctypes.byref(view), int(bool(with_targets))),
              "trpo_vf_set_features_view")
        self.n = int(view.n)

    def predict_to_device(self, ptr: int, dtype=np.float64):
        """predict into a device buffer (raw pointer) of this GPU."""
        check(lib.trpo_vf_predict(self._h, ctypes.c_void_p(ptr), _lib.F64 if dtype == np.float64 else _lib.F32,
                                  MEM_DEVICE), "trpo_vf_predict")

    def set_feature_matrix(self, feat, n_global: Optional[int] = None):
        n = int(feat.shape[0])
        f = _Arg(feat, np.float32, (n, self.feat_dim))
        check(lib.trpo_vf_set_feature_matrix(self._h, n, n if n_global is None else int(n_global), f.ptr, f.mem),
              "trpo_vf_set_feature_matrix")
        self.n = n

    def feature_matrix(self) -> np.ndarray:
        out = np.empty((self.n, self.feat_dim), np.float32)
        check(lib.trpo_vf_get_feature_matrix(self._h, out.ctypes.data_as(ctypes.c_void_p), MEM_HOST),
              "trpo_vf_get_feature_matrix")
        return out

    def set_targets(self, returns):
        dt = np.float32 if (getattr(returns, "dtype", None) in (np.float32,) or
                            (_is_torch(returns) and str(returns.dtype) == "torch.float32")) else np.float64
        r = _Arg(returns, dt, (self.n,))
        check(lib.trpo_vf_set_targets(self._h, r.ptr, _lib.F32 if dt == np.float32 else _lib.F64, r.mem),
              "trpo_vf_set_targets")

    # ---------------------------------------------------------------- compute
    def fit(self, steps: int = FIT_STEPS):
        check(lib.trpo_vf_fit(self._h, int(steps)), "trpo_vf_fit")

    def gradient(self):
        g = np.empty(self.num_params, np.float32)
        loss = ctypes.c_double(0.0)
        check(lib.trpo_vf_gradient(self._h, g.ctypes.data_as(ctypes.c_void_p), ctypes.byref(loss), MEM_HOST),
              "trpo_vf_gradient")
        return g, loss.value

    def predict(self, out=None, dtype=np.float32):
        if out is None:
            out = np.empty(self.n, dtype)
        a = _Arg(out, np.float64 if str(getattr(out, "dtype", "")).endswith("float64") else np.float32,
                 (self.n,), writable=True)
        dt = _lib.F64 if str(out.dtype).endswith("float64") else _lib.F32
        check(lib.trpo_vf_predict(self._h, a.ptr, dt, a.mem), "trpo_vf_predict")
        return out

    # ---------------------------------------------------------------- multi-GPU
    def comm_init(self, uid: bytes, rank: int, world: int):
        buf = (ctypes.c_uint8 * 128)(*uid)
        check(lib.trpo_vf_comm_init(self._h, buf, int(rank), int(world)), "trpo_vf_comm_init")

    def comm_set_host_allreduce(self, fn, rank: int, world: int):
        def cb(ptr, count, dtype, _ctx):
            try:
                ct = ctypes.c_double if dtype == _lib.F64 else ctypes.c_float
                fn(np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ct)), shape=(count,)))
                return 0
            except Exception:   # pragma: no cover
                return 1
        self._host_ar = _lib.ALLREDUCE_CB(cb)
        check(lib.trpo_vf_comm_set_host_allreduce(self._h, self._host_ar, None, int(rank), int(world)),
              "trpo_vf_comm_set_host_allreduce")


class VF(object):
    """utils.py:48-92 on the GPU."""
    coeffs = None
    on_create = None   # callable(VFNet) run when the net is created

    def __init__(self, session, max_rows: Optional[int] = None, device: Optional[int] = None,
                 rng: Optional[np.random.RandomState] = None):
        self.net = None
        self.session = session
        eng = getattr(session, "engine", None)
        self.max_rows = int(max_rows or (eng.max_rows if eng is not None else 1 << 16))
        self.device = int(device if device is not None else (eng.device if eng is not None else 0))
        self.rng = rng or np.random.RandomState(1)

    def create_net(self, shape):
        """utils.py:56-66.  The reference ends with tf.initialize_all_variables(), which also
        re-initialises the policy; a Session that can do that is asked to."""
        self.net = VFNet(int(shape), self.max_rows, (64, 64), self.device)
        self.net.set_params(vf_xavier_params(int(shape), (64, 64), self.rng))
        self.net.reset_optimizer()
        if self.on_create is not None:   # multi-rank learn(): the net's gradient all-reduce (TRPOAgent.set_ranks)
            self.on_create(self.net)
        reinit = getattr(self.session, "initialize_all_variables", None)
        if callable(reinit):
            reinit()

    def _features(self, path):
        return vf_features(path)

    def fit(self, paths: List[Dict]):
        featmat = np.concatenate([self._features(path) for path in paths])
        if self.net is None:
            self.create_net(featmat.shape[1])
        returns = np.concatenate([path["returns"] for path in paths])
        self.net.set_feature_matrix(featmat)
        self.net.set_targets(np.asarray(returns, np.float64))
        self.net.fit(FIT_STEPS)

    def predict(self, path):
        if self.net is None:
            return np.zeros(len(path["rewards"]))
        self.net.set_feature_matrix(self._features(path))
        ret = self.net.predict()
        return np.reshape(ret, (ret.shape[0], ))

    # ---- device-resident forms over an engine's feed (the learn() loop) ----
    def predict_engine(self, engine) -> bool:
        """VF.predict for every path of the engine's feed, written into its baseline in place.
        Before the first fit the reference predicts zeros; the feed then has no baseline."""
        if self.net is None:
            return False
        view = engine.feed_view()
        self.net.set_features_view(view)
        self.net.predict_to_device(view.baseline)
        engine.set_baseline_in_place()
        return True

    def fit_engine(self, engine):
        """VF.fit on the engine's feed: features and returns read in place (advantages computed)."""
        view = engine.feed_view()
        if self.net is None:
            self.create_net(int(view.obs_dim) + int(view.n_actions) + 1)
        self.net.set_features_view(view, with_targets=True)
        self.net.fit(FIT_STEPS)

    # ---- device-resident forms for a concatenated batch ----
    def fit_batch(self, obs, action_dists, episode_starts, returns, n_global: Optional[int] = None):
        if self.net is None:
            self.create_net(int(np.prod(obs.shape[1:])) + int(action_dists.shape[-1]) + 1)
        self.net.set_features(obs, action_dists, episode_starts, n_global)
        self.net.set_targets(returns)
        self.net.fit(FIT_STEPS)

    def predict_batch(self, obs, action_dists, episode_starts, out=None):
        """Baselines for every row of a concatenated batch: float64, zeros before the first fit."""
        n = int(obs.shape[0])
        if self.net is None:
            if out is not None:
                out.zero_() if _is_torch(out) else out.fill(0.0)
                return out
            return np.zeros(n)
        self.net.set_features(obs, action_dists, episode_starts)
        if out is None:
            out = np.empty(n, np.float64)
        return self.net.predict(out)
