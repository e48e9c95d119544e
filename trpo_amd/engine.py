"""Python handle over the HIP TRPO update engine (``include/trpo_engine.h``).

Arrays may be numpy arrays (host; copied in/out) or torch-ROCm tensors on the
engine's GPU (device pointers; no host round trip).  Results come back as fresh
numpy arrays unless an ``out`` tensor is given — the reference's
"caller-owned numpy in, fresh numpy out" convention.
"""
from __future__ import annotations

import ctypes
import json
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import MEM_DEVICE, MEM_HOST, check, lib

__all__ = ["Engine", "UpdateParams"]


def _is_torch(x) -> bool:
    mod = type(x).__module__
    return mod.startswith("torch")


class _Arg:
    """A (pointer, mem-kind) pair that keeps its backing array alive."""

    def __init__(self, x, dtype, shape=None, writable=False):
        if x is None:
            self.ptr, self.mem, self.obj = None, MEM_HOST, None
            return
        if _is_torch(x):
            import torch
            tdt = {np.float32: torch.float32, np.float64: torch.float64, np.int64: torch.int64,
                   np.uint8: torch.uint8}[dtype]
            if x.dtype != tdt or not x.is_contiguous():
                if writable:
                    raise TypeError(f"output tensor must be contiguous {tdt}")
                x = x.to(tdt).contiguous()
            if shape is not None and x.numel() != int(np.prod(shape)):
                raise ValueError(f"expected {int(np.prod(shape))} elements, got {x.numel()}")
            self.obj = x
            if x.is_cuda:
                self.ptr, self.mem = ctypes.c_void_p(x.data_ptr()), MEM_DEVICE
            else:
                self.ptr, self.mem = ctypes.c_void_p(x.data_ptr()), MEM_HOST
            return
        a = np.asarray(x)
        if a.dtype != dtype or not a.flags.c_contiguous:
            if writable:
                raise TypeError(f"output array must be C-contiguous {np.dtype(dtype)}")
            a = np.ascontiguousarray(a, dtype=dtype)
        if shape is not None and a.size != int(np.prod(shape)):
            raise ValueError(f"expected {int(np.prod(shape))} elements, got {a.size}")
        self.obj = a
        self.ptr, self.mem = a.ctypes.data_as(ctypes.c_void_p), MEM_HOST


class UpdateParams:
    """Defaults: trpo_inksci.py:17 config and utils.py:171-172,185."""

    def __init__(self, cg_iters=10, residual_tol=1e-10, cg_damping=0.1, max_kl=0.01,
                 compute_advantages=False, gamma=0.95):
        self.cg_iters = cg_iters
        self.residual_tol = residual_tol
        self.cg_damping = cg_damping
        self.max_kl = max_kl
        self.compute_advantages = compute_advantages
        self.gamma = gamma

    def to_c(self) -> _lib.UpdateParams:
        return _lib.UpdateParams(int(self.cg_iters), float(self.residual_tol), float(self.cg_damping),
                                 float(self.max_kl), int(bool(self.compute_advantages)), float(self.gamma))


class Engine:
    def __init__(self, obs_dim: int, hidden: Sequence[int], n_actions: int, max_rows: int,
                 device: int = 0):
        self.obs_dim = int(obs_dim)
        self.hidden = [int(h) for h in hidden]
        self.n_actions = int(n_actions)
        self.max_rows = int(max_rows)
        self.device = int(device)
        h = (ctypes.c_int * max(1, len(self.hidden)))(*self.hidden)
        handle = ctypes.c_void_p()
        check(lib.trpo_create(ctypes.byref(handle), self.obs_dim, h, len(self.hidden), self.n_actions,
                              self.max_rows, self.device), "trpo_create")
        self._h = handle
        self.num_params = int(lib.trpo_num_params(self._h))
        self.n = 0
        self.n_global = 0

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "_h", None):
            lib.trpo_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def synchronize(self):
        check(lib.trpo_synchronize(self._h), "trpo_synchronize")

    @property
    def stream_handle(self) -> int:
        return int(lib.trpo_stream(self._h) or 0)

    # ------------------------------------------------------------------ comm
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = (ctypes.c_uint8 * 128)()
        check(lib.trpo_comm_unique_id(buf), "trpo_comm_unique_id")
        return bytes(buf)

    def comm_init(self, uid: bytes, rank: int, world: int):
        assert len(uid) == 128
        buf = (ctypes.c_uint8 * 128)(*uid)
        check(lib.trpo_comm_init(self._h, buf, int(rank), int(world)), "trpo_comm_init")

    def comm_set_host_allreduce(self, fn, rank: int, world: int):
        """Test transport: fn(numpy_array) must sum the array across ranks in place."""
        def cb(ptr, count, dtype, _ctx):
            try:
                ct = ctypes.c_double if dtype == _lib.F64 else ctypes.c_float
                arr = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ct)), shape=(count,))
                fn(arr)
                return 0
            except Exception:   # pragma: no cover
                return 1
        self._host_ar = _lib.ALLREDUCE_CB(cb)   # keep alive
        check(lib.trpo_comm_set_host_allreduce(self._h, self._host_ar, None, int(rank), int(world)),
              "trpo_comm_set_host_allreduce")

    def comm_info(self) -> dict:
        """What carries the all-reduces: transport ("none" / "rccl" / "host"), rank, world, the RCCL
        communicator's rank count / user rank / device, this engine's HIP device and its PCI bus id."""
        ci = _lib.CommInfo()
        check(lib.trpo_comm_info(self._h, ctypes.byref(ci)), "trpo_comm_info")
        return {"transport": ("none", "rccl", "host")[ci.transport], "rank": ci.rank, "world": ci.world,
                "comm_count": ci.comm_count, "comm_rank": ci.comm_rank, "comm_device": ci.comm_device,
                "device": ci.device, "pci_bus_id": ci.pci_bus_id.decode()}

    # ------------------------------------------------------------------ params
    def _out(self, out, dtype, n):
        if out is None:
            arr = np.empty(n, dtype)
            return arr, _Arg(arr, dtype, writable=True)
        return out, _Arg(out, dtype, shape=(n,), writable=True)

    def set_flat(self, theta):
        a = _Arg(theta, np.float32, (self.num_params,))
        check(lib.trpo_set_flat(self._h, a.ptr, a.mem), "trpo_set_flat")

    def get_flat(self, out=None):
        res, a = self._out(out, np.float32, self.num_params)
        check(lib.trpo_get_flat(self._h, a.ptr, a.mem), "trpo_get_flat")
        return res

    def get_vector(self, which: int, out=None):
        res, a = self._out(out, np.float32, self.num_params)
        check(lib.trpo_get_vector(self._h, int(which), a.ptr, a.mem), "trpo_get_vector")
        return res

    # ------------------------------------------------------------------ feed
    def set_batch(self, states, actions, advant, old_dist, n_global: Optional[int] = None):
        n = int(states.shape[0])
        n_global = n if n_global is None else int(n_global)
        s = _Arg(states, np.float32, (n, self.obs_dim))
        a = _Arg(actions, np.int64, (n,))
        adv = _Arg(advant, np.float32, (n,)) if advant is not None else _Arg(None, np.float32)
        o = _Arg(old_dist, np.float32, (n, self.n_actions))
        mems = {x.mem for x in (s, a, o) if x.ptr is not None} | ({adv.mem} if adv.ptr is not None else set())
        if len(mems) != 1:
            raise ValueError("set_batch: pass all host arrays or all device tensors")
        check(lib.trpo_set_batch(self._h, n, n_global, s.ptr, a.ptr, adv.ptr, o.ptr, mems.pop()),
              "trpo_set_batch")
        self.n, self.n_global = n, n_global

    def set_rewards(self, rewards, episode_starts, baseline=None):
        n = self.n
        r = _Arg(rewards, np.float64, (n,))
        st = _Arg(np.asarray(episode_starts).astype(np.uint8) if not _is_torch(episode_starts)
                  else episode_starts, np.uint8, (n,))
        b = _Arg(baseline, np.float64, (n,)) if baseline is not None else _Arg(None, np.float64)
        check(lib.trpo_set_rewards(self._h, r.ptr, st.ptr, b.ptr, r.mem), "trpo_set_rewards")

    def set_baseline(self, baseline):
        """The VF.predict baselines of the current feed (trpo_inksci.py:103), f64 [n]."""
        b = _Arg(baseline, np.float64, (self.n,))
        check(lib.trpo_set_baseline(self._h, b.ptr, b.mem), "trpo_set_baseline")

    def feed_view(self) -> "_lib.FeedView":
        """Device pointers into the current feed (synchronises the engine stream)."""
        v = _lib.FeedView()
        check(lib.trpo_get_feed_view(self._h, ctypes.byref(v)), "trpo_get_feed_view")
        return v

    def set_baseline_in_place(self):
        """Mark the feed's own baseline buffer (written through feed_view().baseline) as set."""
        v = self.feed_view()
        check(lib.trpo_set_baseline(self._h, v.baseline, MEM_DEVICE), "trpo_set_baseline")

    def explained_variance(self) -> float:
        """explained_variance(baseline, returns) (utils.py:208-211) over the feed, on the device."""
        out = ctypes.c_double(0.0)
        check(lib.trpo_explained_variance(self._h, ctypes.byref(out)), "trpo_explained_variance")
        return out.value

    def compute_advantages_device(self, gamma: float, returns_out=None, advant_out=None):
        """trpo_inksci.py:102-117 on the device; optional device/host outputs (f64 [n])."""
        r = _Arg(returns_out, np.float64, (self.n,), writable=True) if returns_out is not None else _Arg(None, np.float64)
        a = _Arg(advant_out, np.float64, (self.n,), writable=True) if advant_out is not None else _Arg(None, np.float64)
        mem = r.mem if r.ptr is not None else (a.mem if a.ptr is not None else MEM_HOST)
        check(lib.trpo_compute_advantages(self._h, float(gamma), r.ptr, a.ptr, mem), "trpo_compute_advantages")

    def compute_advantages(self, gamma: float = 0.95):
        ret = np.empty(self.n, np.float64)
        adv = np.empty(self.n, np.float64)
        check(lib.trpo_compute_advantages(self._h, float(gamma), ret.ctypes.data_as(ctypes.c_void_p),
                                          adv.ctypes.data_as(ctypes.c_void_p), MEM_HOST),
              "trpo_compute_advantages")
        return ret, adv

    def standardize(self, adv, n_global: Optional[int] = None, adv32_out=None):
        """trpo_inksci.py:115-117 on the device, summed over the engine's ranks: adv (f64 [n]) is
        standardised in place (a numpy array is updated too); returns adv."""
        return _standardize(self._h, adv, n_global, adv32_out)

    # ------------------------------------------------------------------ graph outputs
    def losses(self):
        out = (ctypes.c_float * 3)()
        check(lib.trpo_losses(self._h, out), "trpo_losses")
        return np.array(out[:], np.float32)

    def eval_losses(self, theta):
        t = _Arg(theta, np.float32, (self.num_params,))
        out = (ctypes.c_float * 3)()
        check(lib.trpo_eval_losses(self._h, t.ptr, out, t.mem), "trpo_eval_losses")
        return np.array(out[:], np.float32)

    def action_dist(self, out=None):
        """session.run(action_dist): the policy's softmax at the current parameters, [n, A]."""
        if out is None:
            res = np.empty((self.n, self.n_actions), np.float32)
            a = _Arg(res, np.float32, writable=True)
        else:
            res, a = out, _Arg(out, np.float32, shape=(self.n, self.n_actions), writable=True)
        check(lib.trpo_action_dist(self._h, a.ptr, a.mem), "trpo_action_dist")
        return res

    def policy_grad(self, out=None):
        res, a = self._out(out, np.float32, self.num_params)
        check(lib.trpo_policy_grad(self._h, a.ptr, a.mem), "trpo_policy_grad")
        return res

    def fvp(self, v, damping: float = 0.1, out=None):
        vi = _Arg(v, np.float32, (self.num_params,))
        res, a = self._out(out, np.float32, self.num_params)
        if vi.mem != a.mem:
            raise ValueError("fvp: v and out must live in the same memory")
        check(lib.trpo_fvp(self._h, vi.ptr, a.ptr, float(damping), vi.mem), "trpo_fvp")
        return res

    def cg(self, b, cg_iters=10, residual_tol=1e-10, damping=0.1, out=None):
        bi = _Arg(b, np.float32, (self.num_params,))
        res, a = self._out(out, np.float32, self.num_params)
        it = ctypes.c_int(0)
        check(lib.trpo_cg(self._h, bi.ptr, a.ptr, int(cg_iters), float(residual_tol), float(damping),
                          ctypes.byref(it), bi.mem), "trpo_cg")
        return res, it.value

    def linesearch(self, x, fullstep, expected_improve_rate: float):
        xi = _Arg(x, np.float32, (self.num_params,))
        fi = _Arg(fullstep, np.float32, (self.num_params,))
        out = np.empty(self.num_params, np.float32)
        k = ctypes.c_int(-1)
        if xi.mem != MEM_HOST or fi.mem != MEM_HOST:
            raise ValueError("linesearch: host arrays expected")
        check(lib.trpo_linesearch(self._h, xi.ptr, fi.ptr, float(expected_improve_rate),
                                  out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(k), MEM_HOST),
              "trpo_linesearch")
        return out, k.value

    # ------------------------------------------------------------------ the update
    def update(self, params: Optional[UpdateParams] = None, **kw) -> dict:
        prm = params or UpdateParams(**kw)
        cp = prm.to_c()
        st = _lib.UpdateStats()
        check(lib.trpo_update(self._h, ctypes.byref(cp), ctypes.byref(st)), "trpo_update")
        return st.as_dict()

    # ------------------------------------------------------------------ sampling / rollouts
    def act(self, states, uniforms=None, train: bool = True):
        """agent.act on a batch (trpo_inksci.py:76-87): (actions int64 [n], action_dist f32 [n, A])."""
        n = int(states.shape[0])
        s = _Arg(states, np.float32, (n, self.obs_dim))
        if s.mem == MEM_DEVICE:
            import torch
            acts = torch.empty(n, dtype=torch.int64, device=s.obj.device)
            dists = torch.empty((n, self.n_actions), dtype=torch.float32, device=s.obj.device)
        else:
            acts = np.empty(n, np.int64)
            dists = np.empty((n, self.n_actions), np.float32)
        u = _Arg(uniforms, np.float64, (n,)) if uniforms is not None else _Arg(None, np.float64)
        a = _Arg(acts, np.int64, writable=True)
        d = _Arg(dists, np.float32, writable=True)
        check(lib.trpo_act(self._h, s.ptr, n, u.ptr, int(bool(train)), a.ptr, d.ptr, s.mem), "trpo_act")
        return acts, dists

    def rollout_cartpole(self, n_envs: int = 1, n_timesteps: int = 1000, max_pathlength: int = 1000,
                         seed: int = 1, train: bool = True, time_limit: int = 200,
                         reset_uniforms=None, action_uniforms=None, max_episodes_per_env: int = 0):
        """rollout(env, agent, max_pathlength, n_timesteps) (utils.py:18-45) over n_envs CartPole-v0
        instances on the GPU.  Returns (total steps, number of paths)."""
        p = _lib.RolloutParams()
        lib.trpo_default_rollout_params(ctypes.byref(p))
        p.n_envs, p.n_timesteps, p.max_pathlength = int(n_envs), int(n_timesteps), int(max_pathlength)
        p.seed, p.train, p.time_limit = int(seed) & ((1 << 64) - 1), int(bool(train)), int(time_limit)
        keep = []
        if reset_uniforms is not None:
            ru = _Arg(reset_uniforms, np.float64)
            keep.append(ru)
            p.reset_uniforms = ru.ptr
            p.max_episodes_per_env = int(max_episodes_per_env)
            p.mem = ru.mem
        if action_uniforms is not None:
            au = _Arg(action_uniforms, np.float64)
            keep.append(au)
            p.action_uniforms = au.ptr
            p.mem = au.mem
        n = ctypes.c_int64(0)
        paths = ctypes.c_int64(0)
        check(lib.trpo_rollout_cartpole(self._h, ctypes.byref(p), ctypes.byref(n), ctypes.byref(paths)),
              "trpo_rollout_cartpole")
        self.rollout_steps = n.value
        return n.value, paths.value

    def rollout_fetch(self, device=None):
        """The concatenated rollout as the reference's arrays: obs f64 [N,4] (and f32), actions i64,
        action_dists f32 [N,A], rewards f64, episode starts u8, cat_sample uniforms f64 (numpy, or torch
        tensors on `device` -- torch must have initialised its GPU context before the first engine was
        created: it bundles its own HIP runtime, which cannot start after ours)."""
        N = self.rollout_steps
        if device is not None:
            import torch
            mk = lambda shape, dt: torch.empty(shape, dtype=dt, device=device)   # noqa: E731
            out = {"obs": mk((N, self.obs_dim), torch.float64), "obs32": mk((N, self.obs_dim), torch.float32),
                   "actions": mk(N, torch.int64),
                   "action_dists": mk((N, self.n_actions), torch.float32), "rewards": mk(N, torch.float64),
                   "starts": mk(N, torch.uint8), "uniforms": mk(N, torch.float64)}
            mem = MEM_DEVICE
            ptr = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731
        else:
            out = {"obs": np.empty((N, self.obs_dim)), "obs32": np.empty((N, self.obs_dim), np.float32),
                   "actions": np.empty(N, np.int64),
                   "action_dists": np.empty((N, self.n_actions), np.float32), "rewards": np.empty(N),
                   "starts": np.empty(N, np.uint8), "uniforms": np.empty(N)}
            mem = MEM_HOST
            ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)   # noqa: E731
        check(lib.trpo_rollout_fetch(self._h, ptr(out["obs"]), ptr(out["obs32"]), ptr(out["actions"]),
                                     ptr(out["action_dists"]),
                                     ptr(out["rewards"]), ptr(out["starts"]), ptr(out["uniforms"]), mem),
              "trpo_rollout_fetch")
        return out

    def rollout_fetch_stats(self):
        """Rewards and path starts of the last rollout (host; for the print-out statistics)."""
        N = self.rollout_steps
        rew, st = np.empty(N), np.empty(N, np.uint8)
        check(lib.trpo_rollout_fetch(self._h, None, None, None, None, rew.ctypes.data_as(ctypes.c_void_p),
                                     st.ctypes.data_as(ctypes.c_void_p), None, MEM_HOST), "trpo_rollout_fetch")
        return {"rewards": rew, "starts": st}

    def rollout_to_batch(self, n_global: Optional[int] = None):
        """Load the rollout as the feed (states, actions, oldaction_dist, rewards, path starts) on the device."""
        N = self.rollout_steps
        check(lib.trpo_rollout_to_batch(self._h, N if n_global is None else int(n_global)), "trpo_rollout_to_batch")
        self.n, self.n_global = N, (N if n_global is None else int(n_global))

    # ------------------------------------------------------------------ profiling
    def profile_enable(self, on: bool = True):
        check(lib.trpo_profile_enable(self._h, int(bool(on))), "trpo_profile_enable")

    def profile_reset(self):
        check(lib.trpo_profile_reset(self._h), "trpo_profile_reset")

    def profile_query(self) -> dict:
        need = lib.trpo_profile_query(self._h, None, 0)
        if need < 0:
            check(need, "trpo_profile_query")
        buf = ctypes.create_string_buffer(need + 1)
        lib.trpo_profile_query(self._h, buf, need + 1)
        return json.loads(buf.value.decode())


def cat_sample_device(prob_nk, uniforms) -> np.ndarray:
    """cat_sample (utils.py:95-105) on the current GPU with the uniforms given."""
    p = np.ascontiguousarray(prob_nk, np.float32)
    r = np.ascontiguousarray(uniforms, np.float64)
    assert p.ndim == 2 and r.shape == (p.shape[0],)
    out = np.empty(p.shape[0], np.int64)
    check(lib.trpo_cat_sample(p.ctypes.data_as(ctypes.c_void_p), p.shape[0], p.shape[1],
                              r.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p), MEM_HOST),
          "trpo_cat_sample")
    return out


def cartpole_step_device(state, action):
    """One CartPole-v0 step per row on the current GPU: (state_out [n,4], reward [n], done [n] bool)."""
    s = np.ascontiguousarray(state, np.float64).reshape(-1, 4)
    a = np.ascontiguousarray(action, np.int64).reshape(-1)
    n = s.shape[0]
    so, rw, dn = np.empty((n, 4)), np.empty(n), np.empty(n, np.uint8)
    check(lib.trpo_cartpole_step(s.ctypes.data_as(ctypes.c_void_p), a.ctypes.data_as(ctypes.c_void_p), n,
                                 so.ctypes.data_as(ctypes.c_void_p), rw.ctypes.data_as(ctypes.c_void_p),
                                 dn.ctypes.data_as(ctypes.c_void_p), MEM_HOST), "trpo_cartpole_step")
    return so, rw, dn.astype(bool)


def discount_device(x, gamma: float, episode_starts=None) -> np.ndarray:
    """Engine-free discounted-return scan (utils.py:14-16) on the current GPU."""
    xa = _Arg(x, np.float64)
    n = int(np.asarray(xa.obj).shape[0]) if xa.mem == MEM_HOST else int(xa.obj.numel())
    st = _Arg(None, np.uint8) if episode_starts is None else _Arg(
        np.asarray(episode_starts).astype(np.uint8) if not _is_torch(episode_starts) else episode_starts,
        np.uint8, (n,))
    if xa.mem == MEM_DEVICE:
        import torch
        out = torch.empty(n, dtype=torch.float64, device=xa.obj.device)
        oa = _Arg(out, np.float64, writable=True)
    else:
        out = np.empty(n, np.float64)
        oa = _Arg(out, np.float64, writable=True)
    check(lib.trpo_discount(xa.ptr, st.ptr, n, float(gamma), oa.ptr, xa.mem), "trpo_discount")
    return out


def _standardize(handle, adv, n_global, adv32_out):
    if not _is_torch(adv):
        if not (isinstance(adv, np.ndarray) and adv.dtype == np.float64 and adv.flags.c_contiguous):
            raise TypeError("standardize: adv must be a C-contiguous float64 array (updated in place)")
    a = _Arg(adv, np.float64, writable=True)
    n = int(adv.numel()) if _is_torch(adv) else int(adv.size)
    o = _Arg(adv32_out, np.float32, (n,), writable=True) if adv32_out is not None else _Arg(None, np.float32)
    if o.ptr is not None and o.mem != a.mem:
        raise ValueError("standardize: adv and adv32_out must live in the same memory")
    check(lib.trpo_standardize(handle, a.ptr, n, n if n_global is None else int(n_global), o.ptr, a.mem),
          "trpo_standardize")
    return adv


def standardize_device(adv, adv32_out=None):
    """adv = (adv - mean)/(std + 1e-8) (trpo_inksci.py:115-117) in place on the current GPU, one
    process (engine-free)."""
    return _standardize(None, adv, None, adv32_out)


def cg_callback(f_Ax, b, cg_iters=10, residual_tol=1e-10):
    """conjugate_gradient(f_Ax, b) for an arbitrary host callable (utils.py:185-201):
    vectors, dots and axpys on the current GPU in b's dtype (float32 or float64).
    Returns (x, iterations)."""
    b = np.asarray(b)
    if b.dtype not in (np.float32, np.float64) or b.ndim != 1:
        raise TypeError("conjugate_gradient: b must be a 1-D float32/float64 array")
    b = np.ascontiguousarray(b)
    n = b.shape[0]
    dt = b.dtype
    err = []

    def cb(p_ptr, z_ptr, _ctx):
        try:
            p = np.ctypeslib.as_array(ctypes.cast(p_ptr, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                      shape=(n,)).copy()
            z = np.asarray(f_Ax(p), dtype=dt).reshape(n)
            np.ctypeslib.as_array(ctypes.cast(z_ptr, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                  shape=(n,))[:] = z
            return 0
        except Exception as exc:  # re-raised after the C call returns
            err.append(exc)
            return 1

    cfn = _lib.FAX_CB(cb)
    x = np.empty(n, dt)
    it = ctypes.c_int(0)
    rc = lib.trpo_cg_callback(cfn, None, b.ctypes.data_as(ctypes.c_void_p),
                              x.ctypes.data_as(ctypes.c_void_p), n,
                              _lib.F64 if dt == np.float64 else _lib.F32, int(cg_iters),
                              float(residual_tol), ctypes.byref(it))
    if err:
        raise err[0]
    check(rc, "trpo_cg_callback")
    return x, it.value
