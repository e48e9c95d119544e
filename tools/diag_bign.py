"""Diagnostic (GPU): the 8M-state C4 update of tests/test_gpu_bigN.py under several kernel-option sets,
printing g / stepdir / theta rel L2 against an f32-MFMA run (split_mfma = split_wg = 0) and against the
exact bf16x6 split. Used to attribute a parity drift to one option."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from oracle import trpo_oracle as O  # noqa: E402

from bign_data import CONFIGS  # noqa: E402

CFG = sys.argv[1] if len(sys.argv) > 1 else "c4"
SPEC, N = CONFIGS[CFG]
SETS = sys.argv[2] if len(sys.argv) > 2 else "default"


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def main():
    import torch
    torch.cuda.init()   # torch's bundled HIP runtime must start before the engine's (engine.py rollout_fetch)
    from trpo_amd import Engine, UpdateParams
    from trpo_amd._lib import VEC_G, VEC_STEPDIR, VEC_THETA, get_option, set_option
    rng = np.random.default_rng(0)
    X = rng.standard_normal((N, SPEC.obs_dim), dtype=np.float32)
    actions = rng.integers(0, SPEC.n_actions, N, dtype=np.int64)
    theta = O.init_theta(SPEC, np.random.RandomState(1)).astype(np.float32)
    rng = np.random.default_rng(5)
    rewards = rng.random(N)
    starts = (np.arange(N) % 200 == 0).astype(np.uint8)
    e = Engine(SPEC.obs_dim, SPEC.hidden, SPEC.n_actions, max_rows=N)
    e.set_flat(theta)
    e.set_batch(X, actions, None, np.full((N, SPEC.n_actions), 1.0 / SPEC.n_actions, np.float32), n_global=N)
    old = e.action_dist()
    e.close()

    import time
    import torch
    from oracle.chunked_f64 import ChunkedGraph, advantages_equal_paths
    t0 = time.time()
    G = ChunkedGraph(SPEC, X, actions, advantages_equal_paths(rewards, 200), old, device="cuda", chunk=1 << 20)
    truth = G.update(theta, residual_tol=0.0)
    del G
    torch.cuda.empty_cache()
    print(f"f64 truth: {time.time() - t0:.1f} s, k {truth['k']}, shs {truth['shs']:.6e}", flush=True)
    bounds, off = [], 0
    for shape in SPEC.param_shapes():
        n = int(np.prod(shape))
        bounds.append((f"{'W' if len(shape) == 2 else 'b'}{len(bounds) // 2}", off, off + n))
        off += n
    G32 = ChunkedGraph(SPEC, X, actions, advantages_equal_paths(rewards, 200), old, device="cuda", chunk=1 << 20,
                       dtype=torch.float32)
    g32 = G32.update(theta, residual_tol=0.0)
    del G32
    torch.cuda.empty_cache()
    for k in ("g", "stepdir"):
        print(f"   {k} per block vs f64: " + " ".join(f"{nm} {rel(g32[k][a:b], truth[k][a:b]):.1e}"
                                                  for nm, a, b in bounds), flush=True)
    print("torch float32 graph | vs f64: " + " ".join(f"{k} {rel(g32[k], truth[k]):.2e}" for k in ("g", "stepdir", "theta")),
          flush=True)

    def run(opts):
        saved = {k: get_option(k) for k in opts}
        for k, v in opts.items():
            set_option(k, v)
        try:
            e = Engine(SPEC.obs_dim, SPEC.hidden, SPEC.n_actions, max_rows=N)
            e.set_flat(theta)
            e.set_batch(X, actions, None, old, n_global=N)
            e.set_rewards(rewards, starts)
            e.update(UpdateParams(cg_iters=10, residual_tol=0.0, compute_advantages=True))
            out = {"g": e.get_vector(VEC_G), "stepdir": e.get_vector(VEC_STEPDIR), "theta": e.get_vector(VEC_THETA)}
            e.close()
        finally:
            for k, v in saved.items():
                set_option(k, v)
        return out

    sets = {
        "f32": {"split_mfma": 0, "split_wg": 0, "hbwd2": 0, "head_fwd": 0},
        "default": {},
        "pg_splits=512": {"pg_splits": 512},
        "splits=2048": {"splits": 2048},
        "bf16x6": {"split_f16": 0},
        "low_seg=0": {"low_seg": 0},
    }
    if SETS == "c5":
        sets = {
            "default": {},
            "pg_splits=1024": {"pg_splits": 1024},
            "splits=256,pg=1024": {"splits": 256, "pg_splits": 1024},
            "splits=512,pg=2048": {"splits": 512, "pg_splits": 2048},
        }
    res = {}
    for name, opts in sets.items():
        res[name] = run(opts)
        r = res[name]
        line = [f"{name:14s}", "vs f64: " + " ".join(f"{k} {rel(r[k], truth[k]):.2e}" for k in ("g", "stepdir", "theta"))]
        for k in ("g", "stepdir"):
            print(f"   {k} per block vs f64: " + " ".join(f"{nm} {rel(r[k][a:b], truth[k][a:b]):.1e}"
                                                      for nm, a, b in bounds), flush=True)
        for ref in ("f32", "bf16x6"):
            if ref in res and ref != name:
                line += [f"vs {ref}: " + " ".join(f"{k} {rel(r[k], res[ref][k]):.2e}" for k in ("g", "stepdir", "theta"))]
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
