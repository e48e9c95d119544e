"""The C-ABI library loads and exports every symbol include/trpo_engine.h declares,
and the ctypes binding covers exactly that set.  No compute calls. CPU only."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "trpo_engine.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(trpo_[a-z0-9_]+)\s*\(", src))
    names.discard("trpo_fax_cb")
    return names


def test_header_declares_api():
    names = header_functions()
    for must in ("trpo_create", "trpo_fvp", "trpo_cg", "trpo_linesearch", "trpo_update", "trpo_discount",
                 "trpo_policy_grad", "trpo_set_flat", "trpo_get_flat", "trpo_comm_init"):
        assert must in names


def test_library_exports_every_header_symbol():
    from trpo_amd import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (trpo_[a-z0-9_]+)", out))
    missing = header_functions() - exported
    assert not missing, f"declared but not exported: {sorted(missing)}"


def test_ctypes_binding_matches_header():
    from trpo_amd import _lib
    assert set(_lib.SIGNATURES) == header_functions()
    for name in _lib.SIGNATURES:
        assert hasattr(_lib.lib, name)


def test_default_params_match_reference_config():
    """trpo_default_params is pure host code: the reference's defaults."""
    import ctypes
    from trpo_amd import _lib
    p = _lib.UpdateParams()
    _lib.lib.trpo_default_params(ctypes.byref(p))
    assert p.cg_iters == 10                                # utils.py:185
    assert p.residual_tol == pytest.approx(1e-10)          # utils.py:185
    assert p.cg_damping == pytest.approx(0.1)              # trpo_inksci.py:17
    assert p.max_kl == 0.01                                # trpo_inksci.py:17
    assert p.gamma == 0.95                                 # trpo_inksci.py:17


def test_errors_are_reported_not_crashes():
    import ctypes
    from trpo_amd import _lib
    h = ctypes.c_void_p()
    rc = _lib.lib.trpo_create(ctypes.byref(h), 4, (ctypes.c_int * 1)(64), 1, 200, 100, 0)   # A > 128
    assert rc != 0
    assert b"n_actions" in _lib.lib.trpo_last_error()


def test_option_roundtrip():
    """Kernel-variant switches are readable and writable without a GPU; unknown names fail."""
    from trpo_amd._lib import EngineError, get_option, set_option
    old = get_option("split_mfma")
    try:
        set_option("split_mfma", 5)
        assert get_option("split_mfma") == 5
    finally:
        set_option("split_mfma", old)
    with pytest.raises(EngineError, match="unknown option"):
        set_option("no_such_option", 1)


def test_every_documented_option_is_known():
    """Every switch the header documents answers get_option; the defaults are the measured best
    configuration: f16 split on, 256x256 two-stage split tile, chain auto, graphs on."""
    import re
    from trpo_amd._lib import get_option
    text = open(os.path.join(ROOT, "include", "trpo_engine.h")).read()
    block = text[text.index("kernel-variant switches"):text.index("int trpo_set_option")]
    names = set(re.findall(r'"([a-z_0-9]+)"', block))
    assert {"split_mfma", "split_f16", "chain", "graphs", "split_min_k", "low_seg", "planes"} <= names
    for n in names:
        get_option(n)
    assert get_option("split_f16") == 1
    assert get_option("split_mfma") == 5
    assert get_option("chain") == 1
    assert get_option("graphs") == 1
    assert get_option("hbwd2") == 2 and get_option("head_fwd") == 1 and get_option("ls_fused") == 1
    assert get_option("cg_fuse_reduce") == 1 and get_option("rfwd01") == 1 and get_option("cg_p_img") == 1
    assert get_option("fwd01") == 1
