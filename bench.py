#!/usr/bin/env python
"""bench.py — TRPO policy-update throughput on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One *step* = one full TRPO update of BASELINE.json's metric ("10-iter CG +
linesearch") over the synthetic batch, exactly the unit of SURVEY.md §8(d):
discount + standardise + policy gradient + 10 CG iterations (residual_tol = 0,
so all 10 run) + the shs FVP + line search + final losses / revert check.
Inputs are resident in HBM before the timed region.  Each step restarts from
the same theta_0 (a device-to-device copy of P floats) so every step does the
same work (steady state: pi_old = p(theta_0)).

Default workload (N=1 and the scaling runs): C4 = 8,000,000 states, obs 128,
256x256 tanh MLP, 18 actions (BASELINE.json configs[3]); with N ranks the 8M
states are split row-wise (path-aligned), so ``scaling`` is "strong".

Rank 0 prints ONE JSON line.  ``roofline`` prices the dominant kernel (largest
share of HIP-event time over the timed region, on the engine's stream) against
the roof that bounds it: its algorithmic FLOPs at the ceiling of its MFMA path
-- the f32 MFMA peak (157.3 TF/s), or for the split GEMMs (fp32 operands scaled
and split into f16 hi+lo pieces, 3 MFMA products per fp32 product) the f16 dense
peak / 3 = 833.3 TF/s of fp32 work (bf16 hi+mid+lo, 6 products: / 6) -- versus
its algorithmic HBM bytes (every operand read once, every output written once)
at 8 TB/s; the larger time is the bound ("mfma" or "hbm"), and `achieved` /
`peak` are in that roof's unit.
``traffic`` is the HBM bytes per launch of that kernel measured by rocprofv3
FETCH_SIZE / WRITE_SIZE passes of this same command (tools/prof.sh ->
tools/pmc_traffic.py -> profiles/<round>/traffic.json), when a committed file
matches the workload.
``cpu_baseline`` (N=1, rank 0 only) times the TF-faithful float32 CPU mirror of
the reference (oracle/tf_graph_torch.py: every FVP recomputes forward + both
backward passes, as each session.run does) on a bounded row sample and
extrapolates linearly in N (every op of the update is O(N)).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "TRPO updates/sec (10-iter CG + linesearch) at N states; FVP GB/s vs HBM peak"
PEAK_F32_TFLOPS = 157.3        # MI355X_MICROARCH.md: FP32 vector = FP32 MFMA peak (dense)
PEAK_BF16_TFLOPS = 2500.0      # MI355X_MICROARCH.md: BF16 / F16 MFMA dense peak


def split_products() -> int:
    """MFMA products per fp32 product on the split path: f16 hi+lo (hh, hl, lh) or bf16 hi+mid+lo."""
    from trpo_amd._lib import get_option
    return 3 if get_option("split_f16") else 6


def peak_split_tflops() -> float:
    return PEAK_BF16_TFLOPS / split_products()
PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
EPISODE_LEN = 200              # CartPole-v0 cap

CONFIGS = {
    "c2": dict(n=50_000, obs=11, hidden=[64, 64], A=3, cpu_rows=50_000,
               name="C2: 50k states, obs 11, 64x64 tanh MLP, 3 actions"),
    "c3": dict(n=1_000_000, obs=128, hidden=[64, 64], A=18, cpu_rows=100_000,
               name="C3: 1M states, obs 128, 64x64 tanh MLP, 18 actions"),
    "c4": dict(n=8_000_000, obs=128, hidden=[256, 256], A=18, cpu_rows=150_000,
               name="C4: 8M states, obs 128, 256x256 tanh MLP, 18 actions"),
    "c5": dict(n=4_000_000, obs=376, hidden=[1024, 1024], A=17, cpu_rows=4_000,
               name="C5: 4M states, obs 376, 1024x1024 tanh MLP, 17 actions"),
}


def chain_flops_per_row(widths) -> float:
    """Fused FVP chain (R-forward + R-head + R-backward): 2 a1 b1 + 8 sum_{l>=2} a_l b_l per state."""
    f = 0.0
    for l in range(len(widths) - 1):
        ab = widths[l] * widths[l + 1]
        f += 2 * ab if l == 0 else 8 * ab
    return f


def tag_flops(tag: str, widths, n: int) -> float:
    """Algorithmic FLOPs of one launch of the kernel behind a profile tag."""
    if tag == "fvp_chain":
        return n * chain_flops_per_row(widths)
    role, _, l = tag.rpartition("_l")
    if not l.isdigit():
        return 0.0
    l = int(l)
    a, b = widths[l], widths[l + 1]
    ab = 2.0 * n * a * b
    if role in ("fwd", "ls_fwd", "bwd", "pg_bwd", "pg_wgrad"):
        return ab
    if role in ("fvp_rfwd", "fvp_wgrad"):
        return ab if l == 0 else 2 * ab
    if role == "fvp_rbwd":
        return 2 * ab
    if role == "fvp_head":          # R-forward (2ab) + R-backward (2ab) + wgrad (2ab) of the last layer
        return 3 * ab
    if role == "fvp_headbwd":       # R-backward (2ab) + wgrad (2ab) of the last layer
        return 2 * ab
    return 0.0


def tag_is_split(tag: str, widths) -> bool:
    """Whether the kernel behind a tag runs on the split-bf16 MFMA path (gemm.hip dispatch rules)."""
    from trpo_amd._lib import get_option
    if tag == "fvp_chain":
        return True
    role, _, l = tag.rpartition("_l")
    if not l.isdigit():
        return False
    l = int(l)
    pad = lambda v: (v + 3) // 4 * 4
    a, b = pad(widths[l]), pad(widths[l + 1])
    if role.endswith("wgrad"):
        return get_option("split_wg") != 0 and b > 128
    if role in ("fvp_head", "fvp_headbwd"):
        return False
    last = l == len(widths) - 2
    out = a if role in ("bwd", "pg_bwd", "fvp_rbwd") else b
    head = last and role in ("fwd", "ls_fwd", "fvp_rfwd")
    return get_option("split_mfma") != 0 and out > 128 and not head


def tag_peak(tag: str, widths) -> float:
    return peak_split_tflops() if tag_is_split(tag, widths) else PEAK_F32_TFLOPS


def tag_bytes(tag: str, widths, n: int) -> float:
    """Algorithmic HBM bytes of one launch: each activation operand read once and each output written
    once (f32, real widths; weights and slabs are O(P) and left out)."""
    role, _, l = tag.rpartition("_l")
    if not l.isdigit():
        return 0.0
    l = int(l)
    L = len(widths) - 1
    w = widths
    cols = 0
    if role == "fvp_rfwd":
        if l == 0:
            cols = w[0] + 2 * w[1]                          # X ; H1 (epilogue) ; RH1 out
        elif l < L - 1:
            cols = 2 * w[l] + 2 * w[l + 1]                  # RH_l, H_l ; H_{l+1} ; RH_{l+1} out
        else:
            cols = 2 * w[l] + 2 * w[l + 1]                  # RH, H ; P ; RD_L out
    elif role == "fvp_rbwd":
        cols = 2 * w[l + 1] + 4 * w[l]                      # RD_l, D_l ; H_l, E, RH_l ; RD_{l-1} out
    elif role == "fvp_wgrad":
        cols = w[0] + w[1] if l == 0 else 2 * w[l] + 2 * w[l + 1]
    elif role in ("fwd", "ls_fwd"):
        cols = w[l] + w[l + 1] + (2 * w[l + 1] if l == L - 1 else 0)
    elif role == "bwd":
        cols = w[l + 1] + 3 * w[l]                          # D_l ; H ; D, E out
    elif role == "pg_bwd":
        cols = w[l + 1] + 2 * w[l]
    elif role == "pg_wgrad":
        cols = w[l] + w[l + 1]
    return 4.0 * n * cols


def tag_roof(tag: str, widths, n: int):
    """(bound, seconds at the roof) of one launch."""
    t_mfma = tag_flops(tag, widths, n) / (tag_peak(tag, widths) * 1e12)
    t_hbm = tag_bytes(tag, widths, n) / (PEAK_HBM_GBS * 1e9)
    return ("hbm", t_hbm) if t_hbm > t_mfma else ("mfma", t_mfma)


def committed_traffic(config: str, rows: int, tag: str):
    """Per-launch HBM bytes of `tag` from the newest matching profiles/*/traffic.json."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("config") == config and d.get("rows") == rows and tag in d.get("tags", {}):
            best = (os.path.relpath(f, ROOT), d["tags"][tag])
    return best


def fvp_flops_per_row(widths) -> float:
    """4 a1 b1 + 12 sum_{l>=2} a_l b_l."""
    f = 0.0
    for l in range(len(widths) - 1):
        ab = widths[l] * widths[l + 1]
        f += 4 * ab if l == 0 else 12 * ab
    return f


def synthetic_theta(widths, rng) -> np.ndarray:
    """W ~ U(+-sqrt(6/(fan_in+fan_out))), b ~ N(0, 0.1^2), flat [W1,b1,...]."""
    parts = []
    for a, b in zip(widths[:-1], widths[1:]):
        lim = (6.0 / (a + b)) ** 0.5
        parts.append(rng.uniform(-lim, lim, size=a * b))
        parts.append(rng.normal(0.0, 0.1, size=b))
    return np.concatenate(parts).astype(np.float32)


def cpu_baseline(cfg, rows: int, threads: int):
    """TF-faithful float32 CPU update on `rows` states; returns a cpu_baseline dict."""
    import torch
    from oracle import trpo_oracle as O
    from oracle.tf_graph_torch import TFFaithfulCPU
    torch.set_num_threads(threads)
    spec = O.PolicySpec(cfg["obs"], cfg["hidden"], cfg["A"])
    # warm the torch CPU kernels on a small batch (allocator / thread pool start-up)
    small = O.synthetic_batch(spec, 512, seed=11)
    TFFaithfulCPU(spec, small["X"], small["actions"], small["advant"], small["old_dist"],
                  small["theta"]).update(cg_iters=2, residual_tol=0.0)
    d = O.synthetic_batch(spec, rows, seed=12, episode_len=EPISODE_LEN)
    mirror = TFFaithfulCPU(spec, d["X"], d["actions"], d["advant"], d["old_dist"], d["theta"])
    t0 = time.perf_counter()
    ret = O.discount_segmented(d["rewards"], d["starts"], 0.95)       # discount + standardise too
    O.standardize(ret)
    mirror.update(cg_iters=10, residual_tol=0.0)
    dt = time.perf_counter() - t0
    per_update_full = dt * cfg["n"] / rows
    return {"value": 1.0 / per_update_full, "unit": "updates/s", "cores": threads, "kind": "port",
            "sample": f"one full update (10 CG iters, residual_tol=0) on {rows:,} of the {cfg['n']:,} states "
                      f"({dt:.2f} s), TF-faithful torch-CPU fp32 mirror, extrapolated linearly in N"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--rows", type=int, default=0, help="override total states (testing only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=0)
    ap.add_argument("--profile-out", default="", help="write the per-tag HIP-event profile here (JSON)")
    args = ap.parse_args()

    cfg = dict(CONFIGS[args.config])
    if args.rows:
        cfg["n"] = args.rows
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    # ranks beyond the visible GPUs share them (a rehearsal on a 1-GPU box); on a full node this is local_rank
    local_rank %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    from trpo_amd import Engine, UpdateParams
    from trpo_amd.dist import init_engine_comm, shard_bounds

    N = cfg["n"]
    widths = [cfg["obs"], *cfg["hidden"], cfg["A"]]
    starts_all = None   # episodes every EPISODE_LEN rows -> shard cuts on path starts
    bounds = shard_bounds(N, world, (np.arange(N) % EPISODE_LEN == 0) if N <= 50_000_000 else starts_all)
    lo, hi = bounds[rank]
    n = hi - lo

    eng = Engine(cfg["obs"], cfg["hidden"], cfg["A"], max_rows=max(n, 16), device=local_rank)
    if world > torch.cuda.device_count():
        # ranks share a GPU (rehearsal only; RCCL refuses duplicate devices): all-reduce through gloo on the host
        def host_allreduce(arr):
            dist.all_reduce(torch.from_numpy(arr))
        eng.comm_set_host_allreduce(host_allreduce, rank, world)
    else:
        init_engine_comm(eng, rank, world)

    # ---- synthetic inputs, generated on the device ----
    theta0 = synthetic_theta(widths, np.random.RandomState(0))
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    X = torch.randn((n, cfg["obs"]), generator=g, device=dev, dtype=torch.float32)
    actions = torch.randint(0, cfg["A"], (n,), generator=g, device=dev, dtype=torch.int64)
    rewards = torch.rand((n,), generator=g, device=dev, dtype=torch.float64)
    starts = ((torch.arange(lo, hi, device=dev) % EPISODE_LEN) == 0).to(torch.uint8)
    uniform = torch.full((n, cfg["A"]), 1.0 / cfg["A"], device=dev, dtype=torch.float32)
    zeros = torch.zeros((n,), device=dev, dtype=torch.float32)
    eng.set_flat(theta0)
    eng.set_batch(X, actions, zeros, uniform, n_global=N)
    old = torch.empty((n, cfg["A"]), device=dev, dtype=torch.float32)
    eng.action_dist(out=old)                       # steady state: pi_old = p(theta_0)
    eng.set_batch(X, actions, zeros, old, n_global=N)
    eng.set_rewards(rewards, starts)
    del uniform, X
    theta0_dev = torch.from_numpy(theta0).to(dev)
    params = UpdateParams(cg_iters=10, residual_tol=0.0, cg_damping=0.1, max_kl=0.01,
                          compute_advantages=True, gamma=0.95)

    last = {}

    def step():
        eng.set_flat(theta0_dev)
        last.update(eng.update(params))

    for _ in range(args.warmup):
        step()

    def barrier():
        if world > 1:
            dist.barrier()

    eng.synchronize()
    torch.cuda.synchronize()
    barrier()
    eng.profile_reset()
    eng.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.synchronize()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    prof = eng.profile_query()
    eng.profile_enable(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if args.profile_out and rank == 0:
        with open(args.profile_out, "w") as f:
            json.dump({"profile": prof, "steps": args.steps, "n_local": n, "widths": widths}, f, indent=1)

    if rank == 0:
        # ---- roofline of the dominant kernel (HIP events on the engine stream) ----
        kernel_tags = {t: v for t, v in prof.items() if tag_flops(t, widths, n) > 0}
        dom = max(kernel_tags, key=lambda t: kernel_tags[t][1])
        cnt, tot_ms = kernel_tags[dom]
        avg_s = tot_ms / cnt / 1e3
        fl = tag_flops(dom, widths, n)
        by = tag_bytes(dom, widths, n)
        bound, _ = tag_roof(dom, widths, n)
        if bound == "hbm":
            achieved, peak, unit = by / avg_s / 1e9, PEAK_HBM_GBS, "GB/s"
            peak_basis = "HBM3E 8.0 TB/s"
        else:
            achieved, peak, unit = fl / avg_s / 1e12, tag_peak(dom, widths), "TFLOP/s"
            peak_basis = ("split MFMA: f16/bf16 dense peak / %d products" % split_products()
                          if tag_is_split(dom, widths) else "f32 MFMA peak")
        upd_flops = sum(tag_flops(t, widths, n) * c for t, (c, _) in kernel_tags.items()) / args.steps
        # seconds one update would take with every kernel at its own roof (max of MFMA and HBM time)
        upd_peak_s = sum(tag_roof(t, widths, n)[1] * c for t, (c, _) in kernel_tags.items()) / args.steps
        tr = committed_traffic(args.config, N, dom) if world == 1 else None
        upd_s = elapsed / args.steps
        fvp_ms = sum(ms for t, (c, ms) in prof.items() if t.startswith("fvp_") or t == "reduce")
        fvp_calls = prof.get("fvp_wgrad_l0", [0, 0])[0]
        fvp_s = fvp_ms / max(1, fvp_calls) / 1e3 if fvp_calls else float("nan")
        fvp_bytes = n * cfg["obs"] * 4 + 3 * eng.num_params * 4
        out = {
            "metric": METRIC,
            "value": args.steps / elapsed,
            "unit": "updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32",
            "arithmetic": ("fp32 in HBM and f32 accumulation; GEMMs wider than 128 columns on f16 MFMA with each "
                           "fp32 operand scaled by a power of two and split into hi+lo f16 pieces (3 products, "
                           "error 2^-22 relative)" if split_products() == 3 else
                           "fp32 in HBM and f32 accumulation; GEMMs wider than 128 columns on bf16 MFMA with "
                           "each fp32 operand split exactly into hi+mid+lo bf16 pieces (6 products)") +
                          "; narrower GEMMs on f32 MFMA; softmax heads and CG scalars in f64",
            "data": "synthetic (X~N(0,1), a~U{0..A-1}, rewards~U(0,1), paths of 200 steps, "
                    "random-init policy, pi_old = p(theta_0))",
            "config": {"workload": cfg["name"] + "; full update = discount+standardise+pg+10 CG+shs FVP+"
                                                 "line search+final losses",
                       "n_states": N, "obs_dim": cfg["obs"], "hidden": cfg["hidden"], "n_actions": cfg["A"],
                       "num_params": eng.num_params, "cg_iters": 10, "residual_tol": 0.0,
                       "parallelism": f"dp{world} (row shards, RCCL all-reduce of [P] FVP/grad + loss scalars)"
                       if world <= torch.cuda.device_count() else
                       f"dp{world} on {torch.cuda.device_count()} GPU(s): rehearsal, ranks share GPUs, "
                       "gloo host all-reduce (not a measurement)"},
            "roofline": {"bound": bound, "kernel": dom, "achieved": achieved, "peak": peak,
                         "unit": unit, "frac": achieved / peak,
                         "traffic": tr[1]["traffic_bytes"] if tr else None,
                         "peak_basis": peak_basis,
                         "algorithmic_bytes_per_launch": by, "flops_per_launch": fl,
                         "mfma_tflops": fl / avg_s / 1e12, "mfma_peak": tag_peak(dom, widths),
                         "hbm_gbs_algorithmic": by / avg_s / 1e9,
                         "hbm_gbs_at_traffic": tr[1]["traffic_bytes"] / avg_s / 1e9 if tr else None,
                         "traffic_source": tr[0] if tr else None,
                         "avg_launch_ms": avg_s * 1e3, "launches": cnt},
            "update_roofline": {"algorithmic_tflop_per_update": upd_flops * world / 1e12,
                                "achieved_tflops": upd_flops * world / upd_s / 1e12,
                                "roof_ms_per_update": upd_peak_s * 1e3,
                                "frac_of_roof": upd_peak_s / upd_s},
            "fvp": {"ms_per_fvp": fvp_s * 1e3, "gbps_algorithmic": fvp_bytes / fvp_s / 1e9,
                    "hbm_frac": fvp_bytes / fvp_s / 1e9 / PEAK_HBM_GBS,
                    "tflops": fvp_flops_per_row(widths) * n / fvp_s / 1e12},
            "last_update": {k: last[k] for k in ("cg_iters", "k", "reverted", "kl_after", "surr_after")},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = min(16, os.cpu_count() or 1)
            if os.environ.get("OMP_NUM_THREADS", "").isdigit():
                threads = min(threads, int(os.environ["OMP_NUM_THREADS"]))
            rows = args.cpu_rows or min(cfg["cpu_rows"], N)
            out["cpu_baseline"] = cpu_baseline(cfg, rows, threads)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
