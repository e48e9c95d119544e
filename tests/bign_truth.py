"""Float64 truth of test_gpu_bigN.py's whole 8M-state update, and the same update in float32 (the reference's
own arithmetic), computed in a child process (oracle/chunked_f64.py on the GPU through torch).
TEST INFRASTRUCTURE ONLY.

A child process because torch's bundled HIP runtime must start before the engine's in a process
(trpo_amd/engine.py, rollout_fetch), and the test session has started the engine's long before.
usage: python tests/bign_truth.py <old.npy> <out.npz> [c4|c3|c2|c5]
The batch is regenerated from bign_data's seeds; old.npy is the engine's pi_old [N, A] f32 (the engine call's
exact input). Advantages are the reference discount + standardisation of the rewards on equal-length paths."""
import os
import sys

import numpy as np
import torch

torch.cuda.init()
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE]
from bign_data import CONFIGS, PATH_LEN, make_batch, make_rewards  # noqa: E402
from oracle.chunked_f64 import ChunkedGraph, advantages_equal_paths  # noqa: E402


def main(old_path, out, config="c4"):
    SPEC, n = CONFIGS[config]
    b = make_batch(n, SPEC)
    old = np.load(old_path, allow_pickle=False)
    rewards, _ = make_rewards(n)
    adv = advantages_equal_paths(rewards, PATH_LEN)
    res = {}
    for tag, dt in (("f64", torch.float64), ("f32", torch.float32)):
        G = ChunkedGraph(SPEC, b["X"], b["actions"], adv, old, device="cuda", chunk=1 << 20, dtype=dt)
        t = G.update(b["theta"], residual_tol=0.0)
        res.update({f"{tag}_{k}": np.asarray(v) for k, v in t.items()})
        del G
        torch.cuda.empty_cache()
    np.savez(out, **res)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *sys.argv[3:4])
