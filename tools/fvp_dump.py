"""Dump the engine's undamped FVP and one update's step for a seeded C4-dims batch (A/B of two engine builds:
run once per TRPO_ENGINE_LIB, then compare the .npz files bitwise).  usage: python tools/fvp_dump.py out.npz [n]"""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import trpo_oracle as O  # noqa: E402  (test infrastructure: the seeded synthetic batch)
from trpo_amd import Engine, UpdateParams  # noqa: E402

n = int(sys.argv[2]) if len(sys.argv) > 2 else 40000
spec = O.PolicySpec(128, [256, 256], 18)
d = O.synthetic_batch(spec, n, seed=7)
v = np.random.RandomState(8).standard_normal(spec.n_params).astype(np.float32)
e = Engine(128, [256, 256], 18, max_rows=n)
e.set_flat(d["theta"])
e.set_batch(d["X"], d["actions"], d["advant"].astype(np.float32), d["old_dist"])
hv = e.fvp(v, 0.0)
st = e.update(UpdateParams(cg_iters=10, residual_tol=0.0))
np.savez(sys.argv[1], hv=hv, theta=e.get_flat())
print("dumped", sys.argv[1], float(np.abs(hv).max()), st["k"], st["cg_iters"])
