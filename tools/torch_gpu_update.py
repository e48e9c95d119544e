"""The C4 update (8M states, 128 -> 256 -> 256 -> 18) as plain torch autograd on the same MI355X, float32,
batch resident in HBM: the reference's TF graph restated (oracle/chunked_f64.py, 1M-row chunks), CG and line
search as the reference's numpy loops. A point of comparison for the engine's hand-written kernels
(measurement aid; not the product, not the bench's cpu_baseline)."""
import sys
import time

import numpy as np
import torch

torch.cuda.init()
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from bign_data import PATH_LEN, SPEC, make_batch, make_rewards  # noqa: E402
from oracle import trpo_oracle as O  # noqa: E402
from oracle.chunked_f64 import ChunkedGraph, advantages_equal_paths  # noqa: E402

b = make_batch()
rewards, _ = make_rewards()
adv = advantages_equal_paths(rewards, PATH_LEN)
# pi_old = p(theta) (steady state), in float32 on the GPU
G0 = ChunkedGraph(SPEC, b["X"], b["actions"], adv, np.zeros((b["X"].shape[0], SPEC.n_actions), np.float32),
                  device="cuda", chunk=1 << 20, dtype=torch.float32, resident=True)
with torch.no_grad():
    vl = G0._vars(b["theta"], False)
    old = torch.cat([G0._dist(vl, X) for X, _, _, _ in G0._chunks()]).cpu().numpy()
del G0
torch.cuda.empty_cache()
G = ChunkedGraph(SPEC, b["X"], b["actions"], adv, old, device="cuda", chunk=1 << 20, dtype=torch.float32,
                 resident=True)
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.time()
    out = G.update(b["theta"], residual_tol=0.0)
    torch.cuda.synchronize()
    dt = time.time() - t0
    print(f"torch float32 autograd update on the GPU: {dt * 1e3:.0f} ms ({1.0 / dt:.3f} updates/s), k {out['k']}",
          flush=True)
t0 = time.time()
th = np.asarray(b["theta"], np.float32)
v = np.random.RandomState(3).standard_normal(SPEC.n_params).astype(np.float32)
torch.cuda.synchronize()
t0 = time.time()
for _ in range(3):
    G.fvp(th, v)
torch.cuda.synchronize()
print(f"one FVP: {(time.time() - t0) / 3 * 1e3:.0f} ms", flush=True)
