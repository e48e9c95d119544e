"""Two ranks on the visible GPU(s): engine RCCL all-reduce vs single-rank result (GPU box helper).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 tools/mrank_check.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    ndev = torch.cuda.device_count()
    dev = int(os.environ.get("LOCAL_RANK", "0")) % max(1, ndev)
    torch.cuda.set_device(dev)
    from trpo_amd import Engine, UpdateParams
    from trpo_amd.dist import init_engine_comm, shard_bounds
    from oracle import trpo_oracle as O
    spec = O.PolicySpec(128, [64, 64], 18)
    n = 40_000
    d = O.synthetic_batch(spec, n, seed=3, episode_len=200)
    lo, hi = shard_bounds(n, world, d["starts"])[rank]
    e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=hi - lo, device=dev)
    if "--host-allreduce" in sys.argv:
        # ranks share a GPU (RCCL refuses duplicate devices): all-reduce through gloo on the host
        def ar(arr):
            t = torch.from_numpy(arr)
            dist.all_reduce(t)
        e.comm_set_host_allreduce(ar, rank, world)
    else:
        init_engine_comm(e, rank, world)
    e.set_flat(d["theta"])
    e.set_batch(d["X"][lo:hi], d["actions"][lo:hi], None, d["old_dist"][lo:hi], n_global=n)
    e.set_rewards(d["rewards"][lo:hi], d["starts"][lo:hi])
    v = np.random.RandomState(1).standard_normal(spec.n_params).astype(np.float32)
    e.compute_advantages(0.95)
    hv = e.fvp(v, 0.0)
    st = e.update(UpdateParams(residual_tol=0.0, compute_advantages=True))
    th = e.get_flat()
    # every rank must hold the same parameters; compare with a single-engine run on rank 0
    allth = [None] * world
    dist.all_gather_object(allth, th)
    if rank == 0:
        for t in allth[1:]:
            assert np.array_equal(t, allth[0]), "ranks diverged"
        e1 = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n, device=dev)
        e1.set_flat(d["theta"])
        e1.set_batch(d["X"], d["actions"], None, d["old_dist"])
        e1.set_rewards(d["rewards"], d["starts"])
        e1.compute_advantages(0.95)
        hv1 = e1.fvp(v, 0.0)
        st1 = e1.update(UpdateParams(residual_tol=0.0, compute_advantages=True))
        th1 = e1.get_flat()
        r1 = np.linalg.norm(hv - hv1) / np.linalg.norm(hv1)
        r2 = np.linalg.norm(th - th1) / np.linalg.norm(th1)
        print(f"world={world} FVP rel {r1:.2e} theta rel {r2:.2e} k={st['k']}/{st1['k']} "
              f"iters={st['cg_iters']}/{st1['cg_iters']}", flush=True)
        assert r1 < 1e-5 and r2 < 1e-5 and st["k"] == st1["k"]
        print("MRANK OK", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
