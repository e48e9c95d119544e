"""ctypes binding of ``libtrpo_engine.so`` (C-ABI: ``include/trpo_engine.h``).

The shared library is built in-tree (``trpo_amd/libtrpo_engine.so``, see
``trpo_amd/build.py``).  There is no fallback: if the library is missing or
fails to load, importing anything that needs it raises ``ImportError``.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (CFUNCTYPE, POINTER, byref, c_char_p, c_double, c_float, c_int, c_int64, c_uint8,
                    c_void_p)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TRPO_ENGINE_LIB", os.path.join(HERE, "libtrpo_engine.so"))

MEM_HOST = 0
MEM_DEVICE = 1

VEC_THETA, VEC_THETA_PREV, VEC_G, VEC_STEPDIR, VEC_FULLSTEP, VEC_THETA_LS = range(6)


class UpdateParams(ctypes.Structure):
    _fields_ = [("cg_iters", c_int), ("residual_tol", c_float), ("cg_damping", c_float),
                ("max_kl", c_double), ("compute_advantages", c_int), ("gamma", c_double)]


class UpdateStats(ctypes.Structure):
    _fields_ = [("cg_iters", c_int), ("k", c_int), ("reverted", c_int), ("pad", c_int),
                ("shs", c_double), ("lm", c_double), ("rate", c_double),
                ("surr_before", c_float), ("kl_before", c_float), ("ent_before", c_float),
                ("surr_after", c_float), ("kl_after", c_float), ("ent_after", c_float),
                ("rdotr", c_float), ("gdotstepdir", c_float)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_ if name != "pad"}


class RolloutParams(ctypes.Structure):
    _fields_ = [("n_envs", c_int), ("max_pathlength", c_int), ("n_timesteps", c_int64), ("train", c_int),
                ("time_limit", c_int), ("seed", ctypes.c_uint64), ("reset_uniforms", c_void_p),
                ("action_uniforms", c_void_p), ("max_episodes_per_env", c_int), ("mem", c_int)]


class CommInfo(ctypes.Structure):
    _fields_ = [("transport", c_int), ("rank", c_int), ("world", c_int), ("comm_count", c_int),
                ("comm_rank", c_int), ("comm_device", c_int), ("device", c_int), ("pci_bus_id", ctypes.c_char * 64)]


class FeedView(ctypes.Structure):
    _fields_ = [("n", c_int64), ("n_global", c_int64), ("obs_dim", c_int), ("n_actions", c_int),
                ("states", c_void_p), ("ld_states", c_int), ("old_dist", c_void_p), ("ld_old", c_int),
                ("episode_starts", c_void_p), ("returns", c_void_p), ("baseline", c_void_p)]


FAX_CB = CFUNCTYPE(c_int, c_void_p, c_void_p, c_void_p)
ALLREDUCE_CB = CFUNCTYPE(c_int, c_void_p, c_int64, c_int, c_void_p)
F32, F64 = 0, 1

# name -> (restype, argtypes); every symbol include/trpo_engine.h declares
SIGNATURES = {
    "trpo_create": (c_int, [POINTER(c_void_p), c_int, POINTER(c_int), c_int, c_int, c_int64, c_int]),
    "trpo_destroy": (None, [c_void_p]),
    "trpo_last_error": (c_char_p, []),
    "trpo_num_params": (c_int64, [c_void_p]),
    "trpo_synchronize": (c_int, [c_void_p]),
    "trpo_stream": (c_void_p, [c_void_p]),
    "trpo_comm_unique_id": (c_int, [POINTER(c_uint8)]),
    "trpo_comm_init": (c_int, [c_void_p, POINTER(c_uint8), c_int, c_int]),
    "trpo_comm_set_host_allreduce": (c_int, [c_void_p, ALLREDUCE_CB, c_void_p, c_int, c_int]),
    "trpo_comm_info": (c_int, [c_void_p, ctypes.POINTER(CommInfo)]),
    "trpo_set_flat": (c_int, [c_void_p, c_void_p, c_int]),
    "trpo_get_flat": (c_int, [c_void_p, c_void_p, c_int]),
    "trpo_get_vector": (c_int, [c_void_p, c_int, c_void_p, c_int]),
    "trpo_set_batch": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_int]),
    "trpo_set_rewards": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int]),
    "trpo_compute_advantages": (c_int, [c_void_p, c_double, c_void_p, c_void_p, c_int]),
    "trpo_standardize": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_int]),
    "trpo_losses": (c_int, [c_void_p, POINTER(c_float)]),
    "trpo_eval_losses": (c_int, [c_void_p, c_void_p, POINTER(c_float), c_int]),
    "trpo_action_dist": (c_int, [c_void_p, c_void_p, c_int]),
    "trpo_policy_grad": (c_int, [c_void_p, c_void_p, c_int]),
    "trpo_fvp": (c_int, [c_void_p, c_void_p, c_void_p, c_float, c_int]),
    "trpo_cg": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_float, c_float, POINTER(c_int), c_int]),
    "trpo_cg_callback": (c_int, [FAX_CB, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_double,
                                 POINTER(c_int)]),
    "trpo_linesearch": (c_int, [c_void_p, c_void_p, c_void_p, c_double, c_void_p, POINTER(c_int), c_int]),
    "trpo_default_params": (None, [POINTER(UpdateParams)]),
    "trpo_update": (c_int, [c_void_p, POINTER(UpdateParams), POINTER(UpdateStats)]),
    "trpo_device_count": (c_int, [POINTER(c_int)]),
    "trpo_discount": (c_int, [c_void_p, c_void_p, c_int64, c_double, c_void_p, c_int]),
    "trpo_set_option": (c_int, [c_char_p, c_int]),
    "trpo_get_option": (c_int, [c_char_p, POINTER(c_int)]),
    "trpo_profile_enable": (c_int, [c_void_p, c_int]),
    "trpo_profile_query": (c_int, [c_void_p, c_char_p, c_int]),
    "trpo_profile_reset": (c_int, [c_void_p]),
    # sampling / rollouts (trpo_inksci.py:76-87, utils.py:18-45,95-105)
    "trpo_default_rollout_params": (None, [POINTER(RolloutParams)]),
    "trpo_rollout_cartpole": (c_int, [c_void_p, POINTER(RolloutParams), POINTER(c_int64), POINTER(c_int64)]),
    "trpo_rollout_fetch": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_int]),
    "trpo_set_baseline": (c_int, [c_void_p, c_void_p, c_int]),
    "trpo_get_feed_view": (c_int, [c_void_p, POINTER(FeedView)]),
    "trpo_vf_set_features_view": (c_int, [c_void_p, POINTER(FeedView), c_int]),
    "trpo_explained_variance": (c_int, [c_void_p, POINTER(c_double)]),
    "trpo_rollout_to_batch": (c_int, [c_void_p, c_int64]),
    "trpo_act": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int, c_void_p, c_void_p, c_int]),
    "trpo_cat_sample": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_int]),
    "trpo_cartpole_step": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int]),
    # value-function baseline (utils.py:48-92)
    "trpo_vf_create": (c_int, [POINTER(c_void_p), c_int, POINTER(c_int), c_int, c_int64, c_int]),
    "trpo_vf_destroy": (None, [c_void_p]),
    "trpo_vf_num_params": (c_int64, [c_void_p]),
    "trpo_vf_set_params": (c_int, [c_void_p, c_void_p, c_int]),
    "trpo_vf_get_params": (c_int, [c_void_p, c_void_p, c_int]),
    "trpo_vf_set_adam": (c_int, [c_void_p, c_float, c_float, c_float, c_float]),
    "trpo_vf_reset_optimizer": (c_int, [c_void_p]),
    "trpo_vf_get_optimizer": (c_int, [c_void_p, c_void_p, c_void_p, POINTER(c_float), POINTER(c_int64), c_int]),
    "trpo_vf_set_features": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_int, c_void_p, c_int, c_void_p,
                                     c_int]),
    "trpo_vf_set_feature_matrix": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_int]),
    "trpo_vf_get_feature_matrix": (c_int, [c_void_p, c_void_p, c_int]),
    "trpo_vf_set_targets": (c_int, [c_void_p, c_void_p, c_int, c_int]),
    "trpo_vf_fit": (c_int, [c_void_p, c_int]),
    "trpo_vf_gradient": (c_int, [c_void_p, c_void_p, POINTER(c_double), c_int]),
    "trpo_vf_predict": (c_int, [c_void_p, c_void_p, c_int, c_int]),
    "trpo_vf_comm_init": (c_int, [c_void_p, POINTER(c_uint8), c_int, c_int]),
    "trpo_vf_comm_set_host_allreduce": (c_int, [c_void_p, ALLREDUCE_CB, c_void_p, c_int, c_int]),
}


class EngineError(RuntimeError):
    pass


def _load():
    if not os.path.isfile(LIB_PATH):
        raise ImportError(
            f"trpo_amd: HIP engine library not found at {LIB_PATH}; build it with "
            f"`python -c 'import __graft_entry__ as g; g.build()'` (there is no CPU fallback)")
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as exc:  # pragma: no cover - load failure is fatal by design
        raise ImportError(f"trpo_amd: failed to load {LIB_PATH}: {exc}") from exc
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib.trpo_last_error()
        raise EngineError(f"{what} failed (rc={rc}): {msg.decode() if msg else ''}")
    return rc


def device_count() -> int:
    n = c_int(0)
    check(lib.trpo_device_count(ctypes.byref(n)), "trpo_device_count")
    return n.value


def set_option(name: str, value: int):
    """Process-wide kernel-variant switch (see include/trpo_engine.h)."""
    check(lib.trpo_set_option(name.encode(), int(value)), f"trpo_set_option({name})")


def get_option(name: str) -> int:
    out = c_int(0)
    check(lib.trpo_get_option(name.encode(), byref(out)), f"trpo_get_option({name})")
    return out.value
