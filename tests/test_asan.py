"""Host AddressSanitizer run of the C++ runtime: `make -C trpo_amd/csrc asan`
instruments engine.cpp / vf.cpp (host code; GPU ASan is not available on this pool) and links the
C-ABI driver tools/asan/abi_asan.cpp, which exercises every entry's argument validation, error
codes and the release of a partially initialised engine.  CPU only, leak detection on."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_abi_under_asan():
    csrc = os.path.join(ROOT, "trpo_amd", "csrc")
    b = subprocess.run(["make", "-C", csrc, "-j4", "asan"], capture_output=True, text=True, timeout=900)
    assert b.returncode == 0, b.stdout[-2000:] + b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1")
    r = subprocess.run([os.path.join(ROOT, "build", "asan", "abi_asan")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ABI ASAN OK" in r.stdout
    assert "AddressSanitizer" not in r.stderr
