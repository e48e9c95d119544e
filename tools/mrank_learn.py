"""Several ranks of the learn() loop (trpo_inksci.py:89-177) against one rank holding every row.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29556 \
        tools/mrank_learn.py [--host-allreduce] [--iters 3]

--host-allreduce  ranks share a GPU (RCCL refuses duplicate devices): the engine's and the VF's all-reduces
                  run through the stream-ordered host transport, summed by gloo
Each rank rolls out its share of the timestep budget with its own draws (TRPOAgent.set_ranks). Checks:
  * after every iteration all ranks hold bitwise-identical policy and VF parameters and the same stats;
  * the episode count and mean reward are those of the ranks' rollouts concatenated;
  * iteration 0's update (zero baseline, trpo_inksci.py:103) equals a one-rank engine's update of the
    concatenated rollouts from the same parameters: theta, surr / kl / ent within 1e-5, k exact.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--host-allreduce", action="store_true")
    ap.add_argument("--iters", type=int, default=3)
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
    from trpo_amd import Engine, TRPOAgent, UpdateParams

    agent = TRPOAgent(4, 2, hidden=(64,), max_rows=8192, device=dev)
    agent.set_ranks(rank, world, host_allreduce=args.host_allreduce)
    hist = agent.learn(max_iterations=args.iters, n_envs=4, seed=5, log=None, record=True)
    keep = ("steps", "paths", "train", "reward_mean", "episodes", "k", "kl", "surr", "entropy",
            "explained_variance", "reverted", "theta_before", "theta", "vf_params")
    mine = [{k: h[k] for k in keep if k in h} | {"rollout": {k: h["rollout"][k] for k in
                                                              ("obs", "actions", "action_dists", "rewards",
                                                               "starts")}} for h in hist]
    objs = [None] * world
    dist.all_gather_object(objs, mine)
    if rank == 0:
        n_it = len(objs[0])
        assert all(len(o) == n_it for o in objs), [len(o) for o in objs]
        total_eps = 0
        for i in range(n_it):
            ref = objs[0][i]
            for r in range(1, world):
                o = objs[r][i]
                for k in ("reward_mean", "episodes", "k", "kl", "surr", "entropy", "explained_variance",
                          "reverted", "train"):
                    assert o.get(k) == ref.get(k), (i, r, k, o.get(k), ref.get(k))
                for k in ("theta_before", "theta", "vf_params"):
                    if k in ref:
                        assert np.array_equal(o[k], ref[k]), (i, r, k)
            ro = [objs[r][i]["rollout"] for r in range(world)]
            rewards = np.concatenate([x["rewards"] for x in ro])
            starts = np.concatenate([x["starts"] for x in ro]).astype(bool)
            eps = np.add.reduceat(rewards, np.flatnonzero(starts))
            assert abs(ref["reward_mean"] - eps.mean()) <= 1e-12 * abs(eps.mean()), (i, ref["reward_mean"], eps.mean())
            if ref.get("train"):
                total_eps += len(eps)
                assert ref["episodes"] == total_eps, (i, ref["episodes"], total_eps)
        # iteration 0 against one engine holding the concatenated rollouts
        h0 = objs[0][0]
        ro = [objs[r][0]["rollout"] for r in range(world)]
        X = np.concatenate([x["obs"] for x in ro]).astype(np.float32)
        acts = np.concatenate([x["actions"] for x in ro])
        dists = np.concatenate([x["action_dists"] for x in ro])
        rewards = np.concatenate([x["rewards"] for x in ro])
        starts = np.concatenate([x["starts"] for x in ro])
        N = X.shape[0]
        e = Engine(4, [64], 2, max_rows=N, device=dev)
        e.set_flat(h0["theta_before"])
        e.set_batch(X, acts, None, dists)
        e.set_rewards(rewards, starts)
        st = e.update(UpdateParams(cg_iters=10, residual_tol=1e-10, cg_damping=0.1, max_kl=0.01,
                                   compute_advantages=True, gamma=0.95))
        th = e.get_flat()
        e.close()
        r_th = rel(h0["theta"], th)
        assert r_th <= 1e-5, ("theta", r_th)
        assert st["k"] == h0["k"], (st["k"], h0["k"])
        for k, hk in (("surr_after", "surr"), ("kl_after", "kl"), ("ent_after", "entropy")):
            assert abs(st[k] - h0[hk]) <= 1e-5 * abs(st[k]) + 1e-9, (k, st[k], h0[hk])
        print(f"{world} ranks x {n_it} learn() iterations: ranks bitwise identical; iteration 0 vs one rank: "
              f"theta rel L2 {r_th:.2e}, k {st['k']}, rows {N}")
        print("MRANK LEARN OK")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
