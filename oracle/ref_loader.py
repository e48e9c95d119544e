"""Import the reference's numpy half (``/root/reference/utils.py``) — build container only.

TEST INFRASTRUCTURE.  Used by ``tests/golden/make_golden.py`` to record golden
vectors from the reference's own ``discount`` / ``conjugate_gradient`` /
``linesearch`` / ``explained_variance`` (``utils.py:14-16,170-201,208-211``),
and by CPU tests that re-check the committed fixtures when the reference is
mounted.  ``/root/reference`` does not exist on the GPU box; nothing there
calls this.

``utils.py`` imports ``tensorflow`` and ``prettytensor`` at module level
(``utils.py:2,5``) and calls ``tf.set_random_seed`` / reads ``tf.float32``
(``utils.py:10,12``); it also uses the Python-2 builtin ``xrange``
(``utils.py:27,100,190``).  Stub modules stand in for the two libraries (the
functions used here never touch them) and ``builtins.xrange = range``.
Bytecode writing is disabled so nothing is written into the read-only tree.
"""
from __future__ import annotations

import builtins
import importlib.util
import os
import sys
import types

REFERENCE_DIR = os.environ.get("TRPO_REFERENCE_DIR", "/root/reference")


def reference_available() -> bool:
    return os.path.isfile(os.path.join(REFERENCE_DIR, "utils.py"))


def load_reference_utils():
    if not reference_available():
        raise FileNotFoundError(f"{REFERENCE_DIR}/utils.py not present")
    sys.dont_write_bytecode = True
    saved = {k: sys.modules.get(k) for k in ("tensorflow", "prettytensor")}
    tf = types.ModuleType("tensorflow")
    tf.set_random_seed = lambda seed: None
    tf.float32 = "float32"
    pt = types.ModuleType("prettytensor")
    sys.modules["tensorflow"] = tf
    sys.modules["prettytensor"] = pt
    had_xrange = hasattr(builtins, "xrange")
    builtins.xrange = range
    try:
        spec = importlib.util.spec_from_file_location(
            "_trpo_reference_utils", os.path.join(REFERENCE_DIR, "utils.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    mod.__dict__.setdefault("xrange", range)
    if not had_xrange:
        # keep xrange visible to the module's functions (they resolve builtins at call time)
        pass
    return mod
