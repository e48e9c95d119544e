"""Build ``trpo_amd/libtrpo_engine.so`` for gfx950 in-tree (hipcc; no torch extension)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")


def build(jobs: int = 8, verbose: bool = False) -> str:
    env = dict(os.environ)
    cmd = ["make", "-C", CSRC, f"-j{max(1, min(jobs, 16))}"]
    res = subprocess.run(cmd, env=env, capture_output=not verbose, text=True)
    if res.returncode != 0:
        sys.stderr.write((res.stdout or "") + (res.stderr or ""))
        raise RuntimeError("building libtrpo_engine.so failed")
    out = os.path.join(HERE, "libtrpo_engine.so")
    if not os.path.isfile(out):
        raise RuntimeError(f"{out} missing after build")
    return out


if __name__ == "__main__":
    print(build(verbose=True))
