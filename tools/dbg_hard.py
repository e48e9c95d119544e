"""Per-block errors of the FVP paths against the float64 oracle on tests/test_gpu_fused16_hard.py's batches
(debugging aid, GPU box): fused = 3 (fused16.hip), 2 (fused.hip bf16x6), 0 (chain + weight-gradient GEMMs).

    python tools/dbg_hard.py c2 mixed,mixed_illcond,mixed_illcond:8 3001
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import trpo_oracle as O  # noqa: E402
from test_gpu_fused16_hard import hard_batch  # noqa: E402


def main():
    from trpo_amd import Engine
    from trpo_amd._lib import get_option, set_option
    dims, n = sys.argv[1], int(sys.argv[3])
    for regime in sys.argv[2].split(","):
        spec, b = hard_batch(dims, regime, n, seed=1000 + n)
        th = b["theta"].astype(np.float64)
        v = np.random.RandomState(n + 9).standard_normal(spec.n_params).astype(np.float32)
        ref = O.fvp_undamped(th, b["X"], v.astype(np.float64), spec)
        blocks = O.unflatten(ref.copy(), spec)
        saved = get_option("fused")
        line = [f"{dims} {regime:9s}"]
        for mode in (3, 2, 0):
            set_option("fused", mode)
            e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=max(n, 16))
            e.set_flat(b["theta"])
            e.set_batch(b["X"], b["actions"], b["advant"].astype(np.float32), b["old_dist"])
            hv = e.fvp(v, 0.0)
            e.close()
            off, errs = 0, []
            for l, (Wl, bl) in enumerate(blocks):
                for nm, blk in (("W", Wl), ("b", bl)):
                    r = ref[off:off + blk.size]
                    errs.append(f"{nm}{l} {np.linalg.norm(hv[off:off + blk.size] - r) / max(np.linalg.norm(r), 1e-300):.1e}")
                    off += blk.size
            line.append(f"[{mode}] " + " ".join(errs))
        set_option("fused", saved)
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
