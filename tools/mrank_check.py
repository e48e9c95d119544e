"""Several ranks on the visible GPU(s): the engine's multi-rank update vs a single-rank engine.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 \
        tools/mrank_check.py [--host-allreduce] [--dims c3|c4|c5] [--rows N] [--graphs]

--host-allreduce  ranks share a GPU (RCCL refuses duplicate devices): the engine's all-reduces run
                  through its stream-ordered host transport, summed by gloo on the host
--dims c4         obs 128, 256x256, 18 actions: the wide layers take the f16-split MFMA row GEMMs
--dims c5         obs 376, 1024x1024, 17 actions (BASELINE configs[4]'s layer shapes)
--graphs          also replay the update as a captured hipGraph (all-reduces inside it) and require
                  every replay to be bitwise identical to the eager update
Checks: ranks bitwise identical; Hv and theta within 1e-5 of one rank holding all rows; same k.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

DIMS = {"c3": (128, [64, 64], 18), "c4": (128, [256, 256], 18), "c5": (376, [1024, 1024], 17)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--host-allreduce", action="store_true")
    ap.add_argument("--dims", default="c3", choices=sorted(DIMS))
    ap.add_argument("--rows", type=int, default=40_000)
    ap.add_argument("--graphs", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    ndev = torch.cuda.device_count()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not args.host_allreduce and local >= ndev:
        raise SystemExit(f"LOCAL_RANK {local} but only {ndev} GPU(s): pass --host-allreduce to share them")
    dev = local % max(1, ndev)
    torch.cuda.set_device(dev)
    from trpo_amd import Engine, UpdateParams
    from trpo_amd._lib import get_option, set_option
    from trpo_amd.dist import init_engine_comm, shard_bounds
    from oracle import trpo_oracle as O
    obs, hidden, A = DIMS[args.dims]
    spec = O.PolicySpec(obs, hidden, A)
    n = args.rows
    d = O.synthetic_batch(spec, n, seed=3, episode_len=200)
    lo, hi = shard_bounds(n, world, d["starts"])[rank]
    e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=hi - lo, device=dev)
    if args.host_allreduce:
        def ar(arr):
            dist.all_reduce(torch.from_numpy(arr))
        e.comm_set_host_allreduce(ar, rank, world)
    else:
        init_engine_comm(e, rank, world)
    e.set_flat(d["theta"])
    e.set_batch(d["X"][lo:hi], d["actions"][lo:hi], None, d["old_dist"][lo:hi], n_global=n)
    e.set_rewards(d["rewards"][lo:hi], d["starts"][lo:hi])
    v = np.random.RandomState(1).standard_normal(spec.n_params).astype(np.float32)
    e.compute_advantages(0.95)
    hv = e.fvp(v, 0.0)
    prm = UpdateParams(residual_tol=0.0, compute_advantages=True)
    saved = get_option("graphs")
    set_option("graphs", 0)
    st = e.update(prm)
    th = e.get_flat()
    replays = []
    if args.graphs:
        # graphs on: the 1st update with this key runs eagerly, the 2nd captures and launches,
        # the 3rd and 4th replay
        set_option("graphs", 1)
        for _ in range(4):
            e.set_flat(d["theta"])
            stg = e.update(prm)
            replays.append((stg, e.get_flat()))
    set_option("graphs", saved)
    for i, (stg, thg) in enumerate(replays):
        assert np.array_equal(thg, th), f"rank {rank}: graph update {i} differs from eager"
        assert stg == st, f"rank {rank}: graph update {i} stats differ: {stg} vs {st}"
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
        st1 = e1.update(prm)
        th1 = e1.get_flat()
        r1 = np.linalg.norm(hv - hv1) / np.linalg.norm(hv1)
        r2 = np.linalg.norm(th - th1) / np.linalg.norm(th1)
        print(f"world={world} dims={args.dims} rows={n} FVP rel {r1:.2e} theta rel {r2:.2e} "
              f"k={st['k']}/{st1['k']} iters={st['cg_iters']}/{st1['cg_iters']} graph replays={len(replays)}",
              flush=True)
        assert r1 < 1e-5 and r2 < 1e-5 and st["k"] == st1["k"]
        print("MRANK OK", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
