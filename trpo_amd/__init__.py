"""trpo_amd — MI355X-native TRPO policy-update engine.

The hot path of inksci/TRPO's update (``trpo_inksci.py:101-158``) — policy
gradient, eps-exact Fisher-vector product, conjugate gradient, step scaling,
line search, discounted returns and advantage standardisation — runs as
hand-written HIP kernels for gfx950 behind the C-ABI in
``include/trpo_engine.h``.  Importing this package loads that library and
fails loudly if it is missing; there is no CPU fallback.
"""
from .engine import Engine, UpdateParams, cg_callback, discount_device  # noqa: F401
from . import utils  # noqa: F401
from .agent import TRPOAgent, Session, xavier_theta, paths_to_batch  # noqa: F401

__version__ = "0.1.0"
