"""Per-block errors of the one-launch FVP forms (fused = 2: fused.hip, 3: fused16.hip) against the float64
oracle, for full and one-block tangents (debugging aid, GPU box).

    python tools/dbg_fused16.py [obs hidden1 hidden2 A n]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import trpo_oracle as O  # noqa: E402


def main():
    from trpo_amd import Engine
    from trpo_amd._lib import set_option
    args = [int(x) for x in sys.argv[1:]] or [128, 64, 64, 18, 3000]
    obs, h1, h2, A, n = args
    spec = O.PolicySpec(obs, [h1, h2], A)
    dd = O.synthetic_batch(spec, n, seed=5)
    shapes = spec.param_shapes()
    sizes = [int(np.prod(s)) for s in shapes]
    offs = np.concatenate([[0], np.cumsum(sizes)])
    names = ["W0", "b0", "W1", "b1", "W2", "b2"]
    rng = np.random.RandomState(6)
    full = rng.standard_normal(spec.n_params).astype(np.float32)
    tangents = {"full": full}
    for i, nm in enumerate(names):
        v = np.zeros_like(full)
        v[offs[i]:offs[i + 1]] = full[offs[i]:offs[i + 1]]
        tangents["only_" + nm] = v
    engines = {}
    for mode in (2, 3):
        set_option("fused", mode)
        e = Engine(obs, [h1, h2], A, max_rows=n)
        e.set_flat(dd["theta"])
        e.set_batch(dd["X"], dd["actions"], dd["advant"].astype(np.float32), dd["old_dist"])
        engines[mode] = e
    for tn, v in tangents.items():
        ref = O.fvp_undamped(dd["theta"].astype(np.float64), dd["X"], v.astype(np.float64), spec)
        outs = {}
        for mode, e in engines.items():
            set_option("fused", mode)
            outs[mode] = e.fvp(v, 0.0)
        line = [f"{tn:8s}"]
        for mode in (2, 3):
            errs = []
            for i, nm in enumerate(names):
                r = ref[offs[i]:offs[i + 1]]
                d = outs[mode][offs[i]:offs[i + 1]] - r
                errs.append(f"{nm} {np.linalg.norm(d) / max(np.linalg.norm(r), 1e-300):.1e}")
            tot = np.linalg.norm(outs[mode] - ref) / np.linalg.norm(ref)
            line.append(f"[{mode}] tot {tot:.1e} " + " ".join(errs))
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
