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

Rank 0 prints ONE JSON line.  The timed region is K updates on the production path: the
update's sync-free prefix replayed from its captured hipGraph.  Per-kernel times come from a
separate eager pass with per-launch HIP events on the engine's stream (events disable the
replay; the kernels are the same launches).

``roofline`` prices the dominant kernel (largest share of that event time) the way SURVEY.md
§8(d) defines the work: ``achieved`` = its share of the FVP's algorithmic FLOPs (4ab per state
and layer for each of R-forward, R-backward and the weight R-gradient; 2ab for layer 1's
R-forward and weight gradient) / its average launch time, against the dense peak of the
arithmetic it actually issues -- the f16 MFMA peak / 3 for the scaled f16 hi+lo split
(833.3 TF/s of fp32 work), / 6 for the exact bf16 hi+mid+lo split (416.7), or the f32 MFMA
peak (157.3).  The bytes the kernel itself streams (its materialised operands) are reported
beside it (``own_traffic_*``), and ``traffic`` is the HBM bytes per launch measured by
rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this command (tools/prof.sh ->
tools/pmc_traffic.py -> profiles/<round>/traffic.json) when a committed file matches.
``fvp.traffic_vs_algorithmic`` = bytes the FVP's kernels move / §8(d)'s N*obs*4 + 3P*4.
``alt_arithmetic`` re-times the same workload with the exact bf16x6 split.
``cpu_baseline`` (N=1, rank 0 only) times the TF-faithful float32 CPU mirror of the reference
(oracle/tf_graph_torch.py: every FVP recomputes forward + both backward passes, as each
session.run does) on a bounded row sample with every core the process may use (``host``
reports nproc, the affinity mask and any cgroup quota) and extrapolates linearly in N.
"""
from __future__ import annotations

import argparse
import glob
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
    # BASELINE configs[0] is one CartPole-v0 update on the CPU reference; "c1" is that policy's shape (obs 4, one
    # 64-wide tanh layer, 2 actions, trpo_inksci.py:38-40) on a device-sized synthetic batch (an A/B line, not the
    # headline)
    "c1": dict(n=1_000_000, obs=4, hidden=[64], A=2, cpu_rows=100_000,
               name="C1 shape: 1M states, obs 4, one 64-wide tanh layer, 2 actions"),
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
    if tag == "fvp_fused":            # fused.hip: the whole FVP incl. weight R-gradients
        return n * fvp_flops_per_row(widths)
    if tag == "pg_fused":             # fused16.hip PG form: the surr backward below the head + every H_l^T DS_l
        w = widths
        L = len(w) - 1
        return 2.0 * n * (sum(w[l] * w[l + 1] for l in range(1, L)) + sum(w[l] * w[l + 1] for l in range(L)))
    if tag in ("fwd", "ls_fwd"):      # fused16.hip fwd_loss16: the whole policy forward (prepare / line search)
        return 2.0 * n * sum(widths[l] * widths[l + 1] for l in range(len(widths) - 1))
    if tag == "fvp_rfwd01":           # rfwd.hip: X V0 (2 a0 a1) + RH1 W1 + H1 V1 (4 a1 a2)
        return 2.0 * n * widths[0] * widths[1] + 4.0 * n * widths[1] * widths[2]
    if tag in ("fwd_l01", "ls_fwd_l01"):   # rfwd.hip fwd01_kernel: X W0 + H1 W1
        return 2.0 * n * (widths[0] * widths[1] + widths[1] * widths[2])
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
    if role == "fvp_rbwdwg":        # rbwd0.hip: layer l's R-backward (2ab) + layer l-1's weight R-gradient
        return 2 * ab + 2.0 * n * widths[l - 1] * widths[l]
    if role == "pg_bwdwg":          # rbwd0.hip: the surr backward into layer l-1 + its weight gradient
        return ab + 2.0 * n * widths[l - 1] * widths[l]
    if role == "fvp_tail":          # fused last layer: R-forward (2ab) + R-backward (2ab) + weight R-gradient (2ab)
        return 6 * ab
    return 0.0


def tag_is_split(tag: str, widths) -> bool:
    """Whether the kernel behind a tag runs on the split-bf16 MFMA path (gemm.hip dispatch rules)."""
    from trpo_amd._lib import get_option
    if tag in ("fvp_chain", "fvp_fused", "pg_fused", "fwd", "ls_fwd", "fvp_rfwd01", "fwd_l01", "ls_fwd_l01"):
        return True
    role, _, l = tag.rpartition("_l")
    if not l.isdigit():
        return False
    l = int(l)
    pad = lambda v: (v + 3) // 4 * 4
    a, b = pad(widths[l]), pad(widths[l + 1])
    if role.endswith("wgrad"):
        return get_option("split_wg") != 0 and b > 128
    if role in ("fvp_tail", "fvp_rbwdwg", "pg_bwdwg"):   # tail.hip / rbwd0.hip: always the f16 hi+lo split
        return True
    last = l == len(widths) - 2
    out = a if role in ("bwd", "pg_bwd", "fvp_rbwd") else b
    head = last and role in ("fwd", "ls_fwd", "fvp_rfwd")
    return get_option("split_mfma") != 0 and out > 128 and not head


def fused16_used(widths) -> bool:
    """Whether the one-launch FVP runs on the f16 split (engine.cpp use_fused16, fused16.hip fused16_eligible)."""
    from trpo_amd._lib import get_option
    w = widths
    return (get_option("fused") == 3 and get_option("split_f16") != 0 and len(w) in (3, 4) and 1 <= w[0] <= 128 and
            all(1 <= h <= 64 for h in w[1:-1]) and 1 <= w[-1] <= 32)


def tag_products(tag: str, widths) -> int:
    """MFMA products per fp32 product of a split kernel: chain.hip / fused.hip take the exact bf16 hi+mid+lo
    split (6), fused16.hip the scaled f16 hi+lo (3), the row GEMMs the engine's split option."""
    if tag == "fvp_chain" or (tag == "fvp_fused" and not fused16_used(widths)):
        return 6
    return 3 if tag in ("fvp_fused", "pg_fused", "fwd", "ls_fwd", "fvp_rfwd01", "fwd_l01", "ls_fwd_l01") \
        else split_products()


def tag_peak(tag: str, widths) -> float:
    if tag_is_split(tag, widths):
        return PEAK_BF16_TFLOPS / tag_products(tag, widths)
    return PEAK_F32_TFLOPS


def tag_bytes(tag: str, widths, n: int) -> float:
    """Algorithmic HBM bytes of one launch: each activation operand read once and each output written
    once (f32, real widths; weights and slabs are O(P) and left out)."""
    if tag == "fvp_fused":            # X, P, D_{L-1} ; H_l, E_{l-1} per hidden layer ; D_l of the hidden layers
        L = len(widths) - 1
        cols = widths[0] + 2 * widths[L] + 2 * sum(widths[1:L]) + sum(widths[2:L])
        return 4.0 * n * cols
    if tag == "pg_fused":             # X, DS_{L-1}, H_l
        return 4.0 * n * sum(widths)
    if tag == "fvp_rfwd01":           # X (its f16 planes) ; H1 ; RH1, RZ2 out
        return 4.0 * n * (widths[0] + 2 * widths[1] + widths[2])
    if tag == "fwd_l01":              # X (its f16 planes) ; H1, H2 out
        return 4.0 * n * (widths[0] + widths[1] + widths[2])
    if tag == "ls_fwd_l01":           # X ; H2 out (H1 stays on chip)
        return 4.0 * n * (widths[0] + widths[2])
    if tag == "ls_fwd":               # X ; pi_old (the row terms are O(n))
        return 4.0 * n * (widths[0] + widths[-1])
    if tag == "fwd":                  # X ; pi_old ; H_l, P, D_L, DS_L out
        return 4.0 * n * (widths[0] + 4 * widths[-1] + sum(widths[1:-1]))
    role, _, l = tag.rpartition("_l")
    if not l.isdigit():
        return 0.0
    l = int(l)
    L = len(widths) - 1
    w = widths
    cols = 0
    if role == "fvp_rfwd":
        rz = l == L - 2 and tail_used(widths)               # kRZ: the tail applies (1-H^2), H_{l+1} not read
        if l == 0:
            cols = w[0] + (1 if rz else 2) * w[1]           # X ; H1 (epilogue) ; RH1 out
        elif l < L - 1:
            cols = 2 * w[l] + (1 if rz else 2) * w[l + 1]   # RH_l, H_l ; H_{l+1} ; RH_{l+1} (or RZ) out
        else:
            cols = 2 * w[l] + 2 * w[l + 1]                  # RH, H ; P ; RD_L out
    elif role == "fvp_rbwd":
        cols = 2 * w[l + 1] + 4 * w[l]                      # RD_l, D_l ; H_l, E, RH_l ; RD_{l-1} out
    elif role == "fvp_rbwdwg":
        # RD_l, D_l's f16 hi plane (the one-product D_l V_l^T segment; f32 D_l when the binade test does not
        # fire -- it fires at C4) ; H_l, E, RH_l ; X (RD_{l-1} stays on chip)
        cols = 1.5 * w[l + 1] + 3 * w[l] + w[l - 1]
    elif role == "pg_bwdwg":
        cols = w[l + 1] + w[l] + w[l - 1]                   # DS_l ; H_l ; X
    elif role == "fvp_tail":
        cols = 3 * w[l] + 2 * w[l + 1]                      # RH_l, H_l ; P, D_L ; RD_{l-1} out
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


def tail_used(widths) -> bool:
    """Whether the engine runs the fused last-layer tail (engine.cpp use_tail, tail.hip tail_eligible)."""
    from trpo_amd._lib import get_option
    pad = lambda v: (v + 3) // 4 * 4
    L = len(widths) - 1
    if L < 2 or not (get_option("tail") and get_option("split_f16") and get_option("split_mfma")):
        return False
    a, b = pad(widths[L - 1]), pad(widths[L])
    return 128 < a <= 256 and a % 32 == 0 and 16 < b <= 32 and widths[L] <= 32


def tag_x_bytes(tag: str, widths, n: int) -> float:
    """SURVEY.md §8(d)'s algorithmic bytes of one launch: the states' X rows (N*obs*4) when the kernel
    reads X, else 0 (every other operand is an intermediate the algorithm need not materialise)."""
    if tag in ("fvp_chain", "fvp_fused", "pg_fused", "fwd", "ls_fwd", "fvp_rfwd01", "fwd_l01", "ls_fwd_l01"):
        return 4.0 * n * widths[0]
    role, _, l = tag.rpartition("_l")
    if not l.isdigit():
        return 0.0
    l = int(l)
    reads_x = (l == 0 and role in ("fvp_rfwd", "fvp_wgrad", "fwd", "ls_fwd", "pg_wgrad")) or \
        (l == 1 and role in ("fvp_rbwdwg", "pg_bwdwg"))
    return 4.0 * n * widths[0] if reads_x else 0.0


def tag_roof(tag: str, widths, n: int):
    """(bound, seconds at the roof) of one launch."""
    t_mfma = tag_flops(tag, widths, n) / (tag_peak(tag, widths) * 1e12)
    t_hbm = tag_bytes(tag, widths, n) / (PEAK_HBM_GBS * 1e9)
    return ("hbm", t_hbm) if t_hbm > t_mfma else ("mfma", t_mfma)


def committed_traffic(config: str, rows: int, tag: str):
    """Per-launch HBM bytes of `tag` from profiles/*/traffic.json: the file measured on this source build if one
    is committed, else the last matching one in name order."""
    best = same = None
    build = source_build_id()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("config") == config and d.get("rows") == rows and tag in d.get("tags", {}):
            best = (os.path.relpath(f, ROOT), d["tags"][tag], d.get("build"))
            if d.get("build") == build:
                same = best
    return same or best


def source_build_id() -> str:
    """sha256 (16 hex) over the kernel and runtime sources the library is built from (trpo_amd/csrc,
    include): the same id on the GPU box as here, with no git needed; profiles/*/traffic.json records
    the id of the build its PMC pass measured."""
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "trpo_amd", "csrc", "*")) + glob.glob(os.path.join(ROOT, "include", "*.h")))
    for f in files:
        if os.path.isfile(f) and not f.endswith((".o", ".so")):
            h.update(os.path.relpath(f, ROOT).encode())
            h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def fvp_flops_per_row(widths) -> float:
    """4 a1 b1 + 12 sum_{l>=2} a_l b_l."""
    f = 0.0
    for l in range(len(widths) - 1):
        ab = widths[l] * widths[l + 1]
        f += 4 * ab if l == 0 else 12 * ab
    return f


def update_flops_8d(widths, n: int) -> float:
    """SURVEY.md §8(d)'s full update (k = 1): N*(grad + 11*FVP + 1*fwd), with grad = 4a1b1 + 6 sum_{l>=2} a_l b_l
    and fwd = 2 sum_l a_l b_l."""
    ab = [widths[l] * widths[l + 1] for l in range(len(widths) - 1)]
    grad = 4 * ab[0] + 6 * sum(ab[1:])
    fwd = 2 * sum(ab)
    return float(n) * (grad + 11 * fvp_flops_per_row(widths) + fwd)


def synthetic_theta(widths, rng) -> np.ndarray:
    """W ~ U(+-sqrt(6/(fan_in+fan_out))), b ~ N(0, 0.1^2), flat [W1,b1,...]."""
    parts = []
    for a, b in zip(widths[:-1], widths[1:]):
        lim = (6.0 / (a + b)) ** 0.5
        parts.append(rng.uniform(-lim, lim, size=a * b))
        parts.append(rng.normal(0.0, 0.1, size=b))
    return np.concatenate(parts).astype(np.float32)


def host_cores():
    """(threads to use, report): every core this process may run on, capped by a cgroup CPU quota
    when one is set (the GPU box allots a CPU share per GPU; nproc shows the whole machine)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:   # pragma: no cover
        aff = nproc
    quota = None
    for f in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(f).read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
        except (OSError, ValueError):
            pass
    threads = min(aff, quota) if quota else aff
    return threads, {"nproc": nproc, "affinity_cpus": aff, "cgroup_quota_cpus": quota,
                     "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(cfg, rows: int, threads: int, core_report: dict):
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
            "host": core_report,
            "sample": f"one full update (10 CG iters, residual_tol=0) on {rows:,} of the {cfg['n']:,} states "
                      f"({dt:.2f} s on {threads} threads), TF-faithful torch-CPU fp32 mirror, extrapolated "
                      f"linearly in N"}


class Workload:
    """The synthetic C-config batch of one rank, resident in HBM."""

    def __init__(self, cfg, rank, world, local_rank, dev):
        import torch
        from trpo_amd.dist import shard_bounds
        self.cfg = cfg
        N = cfg["n"]
        self.widths = [cfg["obs"], *cfg["hidden"], cfg["A"]]
        # episodes every EPISODE_LEN rows -> shard cuts on path starts
        starts = (np.arange(N) % EPISODE_LEN == 0) if N <= 50_000_000 else None
        self.lo, self.hi = shard_bounds(N, world, starts)[rank]
        self.n = self.hi - self.lo
        self.rank, self.world, self.local_rank, self.dev = rank, world, local_rank, dev
        self.theta0 = synthetic_theta(self.widths, np.random.RandomState(0))
        self.theta0_dev = torch.from_numpy(self.theta0).to(dev)

    def engine(self, comm_setup):
        """A fresh engine holding this rank's batch (steady state: pi_old = p(theta_0))."""
        import torch
        from trpo_amd import Engine
        cfg, n, dev = self.cfg, self.n, self.dev
        eng = Engine(cfg["obs"], cfg["hidden"], cfg["A"], max_rows=max(n, 16), device=self.local_rank)
        comm_setup(eng)
        g = torch.Generator(device=dev)
        g.manual_seed(1000 + self.rank)
        X = torch.randn((n, cfg["obs"]), generator=g, device=dev, dtype=torch.float32)
        actions = torch.randint(0, cfg["A"], (n,), generator=g, device=dev, dtype=torch.int64)
        rewards = torch.rand((n,), generator=g, device=dev, dtype=torch.float64)
        starts = ((torch.arange(self.lo, self.hi, device=dev) % EPISODE_LEN) == 0).to(torch.uint8)
        uniform = torch.full((n, cfg["A"]), 1.0 / cfg["A"], device=dev, dtype=torch.float32)
        zeros = torch.zeros((n,), device=dev, dtype=torch.float32)
        eng.set_flat(self.theta0)
        eng.set_batch(X, actions, zeros, uniform, n_global=cfg["n"])
        old = torch.empty((n, cfg["A"]), device=dev, dtype=torch.float32)
        eng.action_dist(out=old)                       # steady state: pi_old = p(theta_0)
        eng.set_batch(X, actions, zeros, old, n_global=cfg["n"])
        eng.set_rewards(rewards, starts)
        del uniform, X, old
        torch.cuda.synchronize()
        return eng


PARAMS = dict(cg_iters=10, residual_tol=0.0, cg_damping=0.1, max_kl=0.01, compute_advantages=True, gamma=0.95)


def timed_updates(eng, wl, steps, warmup, barrier):
    """W warmup + K timed updates (graph replay on: the production path), each from theta_0.
    Returns (seconds, last stats)."""
    import torch
    from trpo_amd import UpdateParams
    params = UpdateParams(**PARAMS)
    last = {}

    def step():
        eng.set_flat(wl.theta0_dev)
        last.update(eng.update(params))

    for _ in range(warmup):
        step()
    eng.synchronize()
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    eng.synchronize()
    torch.cuda.synchronize()
    barrier()
    return time.perf_counter() - t0, dict(last)


def profile_pass(eng, wl, steps):
    """Per-kernel HIP events on the engine stream over `steps` eager updates (events disable the
    graph replay, so this pass is separate from the timed one; kernel bodies are identical)."""
    from trpo_amd import UpdateParams
    params = UpdateParams(**PARAMS)
    eng.profile_reset()
    eng.profile_enable(True)
    for _ in range(steps):
        eng.set_flat(wl.theta0_dev)
        eng.update(params)
    eng.synchronize()
    prof = eng.profile_query()
    eng.profile_enable(False)
    return prof


def fvp_tags_per_call(prof):
    """The FVP's launch tags and the number of FVPs: every FVP launches each of its kernels once (the
    per-layer kernels on the wide path, `fvp_fused` alone on the one-launch path)."""
    tags = {t: v for t, v in prof.items() if t.startswith("fvp_") or t == "split_v"}
    calls = max((c for t, (c, _) in tags.items() if t.startswith("fvp_")), default=0)
    return tags, calls


def comm_block(eng, world, rank, rehearsal, dist):
    """The line's proof of what carried the all-reduces: the engine's transport, the RCCL communicator's
    rank count, and every rank's HIP device and PCI bus id (gathered over torch.distributed).  Outside a
    rehearsal, two ranks on one device end the run: that would not be a measurement of N GPUs."""
    ci = eng.comm_info()
    mine = {"rank": rank, "device": ci["device"], "pci_bus_id": ci["pci_bus_id"], "comm_rank": ci["comm_rank"],
            "comm_device": ci["comm_device"]}
    ranks = [mine]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
    buses = [r["pci_bus_id"] for r in ranks]
    if len(set(buses)) != len(buses) and not rehearsal:
        raise SystemExit(f"ranks share a device outside --rehearsal: {buses}")
    if ci["transport"] == "rccl" and ci["comm_count"] != world:
        raise SystemExit(f"RCCL communicator has {ci['comm_count']} ranks, world is {world}")
    return {"transport": ci["transport"], "ranks": ci["comm_count"] if ci["transport"] == "rccl" else world,
            "world": world, "distinct_devices": len(set(buses)), "per_rank": ranks}


DIGEST_STATS = ("cg_iters", "k", "reverted", "shs", "lm", "rate", "rdotr", "gdotstepdir", "surr_after", "kl_after",
                "ent_after")


def rank_digest(vectors, stats) -> str:
    """sha256 (16 hex) over the bytes of an update's replicated outputs: theta, g, stepdir and fullstep as
    float32 arrays and the CG / step / line-search scalars (every rank must end an update
    with bitwise-identical theta and CG scalars, since the CG and line-search branches run redundantly)."""
    import hashlib
    import struct
    h = hashlib.sha256()
    for v in vectors:
        h.update(np.ascontiguousarray(v, dtype=np.float32).tobytes())
    for k in DIGEST_STATS:
        h.update(k.encode())
        h.update(struct.pack("<d", float(stats[k])))
    return h.hexdigest()[:16]


def engine_digest(eng, stats) -> str:
    from trpo_amd._lib import VEC_FULLSTEP, VEC_G, VEC_STEPDIR, VEC_THETA
    return rank_digest([eng.get_vector(w) for w in (VEC_THETA, VEC_G, VEC_STEPDIR, VEC_FULLSTEP)], stats)


def gather_rank_check(digest: str, fvp_ms: float, world: int, dist) -> dict:
    """All-gather every rank's update digest and FVP time (outside the timed region).  The result goes into
    the line's `comm` block; `ranks_bitwise_equal` is False when any rank's digest differs."""
    mine = {"digest": digest, "fvp_ms": fvp_ms}
    allr = [mine]
    if world > 1:
        allr = [None] * world
        dist.all_gather_object(allr, mine)
    digests = [r["digest"] for r in allr]
    return {"ranks_bitwise_equal": len(set(digests)) == 1, "rank_digests": digests,
            "fvp_ms_per_rank": [r["fvp_ms"] for r in allr]}


def enforce_rank_check(check: dict):
    """Exit non-zero (status 3) when the ranks' updates differ: a multi-GPU line whose ranks diverged is
    not a measurement of the algorithm."""
    if not check["ranks_bitwise_equal"]:
        sys.stderr.write(f"bench.py: ranks ended the update with different bits: {check['rank_digests']}\n")
        sys.stderr.flush()
        raise SystemExit(3)


def launch_ranks(argv, gpus: int, rehearsal: bool, visible_gpus: int) -> int:
    """`bench.py --gpus N` with no WORLD_SIZE in the environment: start N ranks on this node as one child
    process (`python -m torch.distributed.run`, rendezvous on 127.0.0.1), relay their output and return
    the launcher's exit status (non-zero when any rank fails).  Nothing here touches the GPU: the parent
    only counts devices, then waits.  More ranks than visible GPUs is refused unless --rehearsal."""
    import socket
    import subprocess
    if gpus > visible_gpus and not rehearsal:
        sys.stderr.write(f"bench.py: --gpus {gpus} but {visible_gpus} GPU(s) visible; "
                         f"pass --rehearsal to let ranks share GPUs\n")
        return 2
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", "--max-restarts=0",
           os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return subprocess.call(cmd, env=env)


def visible_gpu_count() -> int:
    """Devices this process could use, counted without initialising the GPU runtime."""
    import torch
    return torch.cuda.device_count()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--rows", type=int, default=0, help="override total states (testing only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=0)
    ap.add_argument("--profile-steps", type=int, default=1, help="eager updates of the HIP-event profile pass")
    ap.add_argument("--no-alt", action="store_true", help="skip the exact bf16x6-split comparison line")
    ap.add_argument("--rehearsal", action="store_true",
                    help="allow more ranks per node than GPUs (they share GPUs through a host all-reduce)")
    ap.add_argument("--profile-out", default="", help="write the per-tag HIP-event profile here (JSON)")
    ap.add_argument("--rccl-world1", action="store_true",
                    help="at one rank, still create a (one-rank) RCCL communicator: every all-reduce runs "
                         "through RCCL, and the comm block records it")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the driver's form `python bench.py --gpus N`: become the launcher of N ranks
        sys.exit(launch_ranks(sys.argv[1:], args.gpus, args.rehearsal, visible_gpu_count()))

    cfg = dict(CONFIGS[args.config])
    if args.rows:
        cfg["n"] = args.rows
        cfg["name"] = cfg["name"].split(":")[0] + f" dims at {args.rows:,} states (--rows override)"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    ndev = torch.cuda.device_count()
    # one rank per GPU; ranks of this node beyond its GPUs only in an explicit rehearsal
    rehearsal = args.rehearsal
    if local_world > ndev and not rehearsal:
        raise SystemExit(f"{local_world} ranks on this node but {ndev} GPU(s): pass --rehearsal to share GPUs")
    if local_rank >= ndev and not rehearsal:
        raise SystemExit(f"LOCAL_RANK {local_rank} has no GPU ({ndev} visible)")
    gpu = local_rank % max(1, ndev)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)

    from trpo_amd.dist import init_engine_comm

    def comm_setup(eng):
        if world <= 1:
            if args.rccl_world1:
                eng.comm_init(eng.comm_unique_id(), 0, 1)
            return
        if rehearsal:
            # ranks share a GPU (RCCL refuses duplicate devices): all-reduce through gloo on the host
            def host_allreduce(arr):
                dist.all_reduce(torch.from_numpy(arr))
            eng.comm_set_host_allreduce(host_allreduce, rank, world)
        else:
            init_engine_comm(eng, rank, world)

    def barrier():
        if world > 1:
            dist.barrier()

    wl = Workload(cfg, rank, world, gpu, dev)
    n, widths, N = wl.n, wl.widths, cfg["n"]
    eng = wl.engine(comm_setup)
    comm = comm_block(eng, world, rank, rehearsal, dist)
    elapsed, last = timed_updates(eng, wl, args.steps, args.warmup, barrier)
    digest = engine_digest(eng, last)   # after the timed region: the last timed update's outputs
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    prof = profile_pass(eng, wl, max(1, args.profile_steps))
    fvp_tags, fvp_calls = fvp_tags_per_call(prof)
    fvp_ms = sum(ms for _, (_, ms) in fvp_tags.items()) + prof.get("reduce", [0, 0])[1] * (
        fvp_calls / max(1, prof.get("reduce", [1, 1])[0]))
    fvp_s = fvp_ms / max(1, fvp_calls) / 1e3 if fvp_calls else float("nan")
    comm.update(gather_rank_check(digest, fvp_s * 1e3, world, dist))
    num_params = eng.num_params
    prod = split_products()
    eng.close()
    del eng
    torch.cuda.empty_cache()

    alt = None
    if not args.no_alt and world == 1:
        # the exact bf16 hi+mid+lo split (6 products) on the same workload, beside the default
        from trpo_amd._lib import get_option, set_option
        saved = get_option("split_f16")
        set_option("split_f16", 0)
        try:
            e2 = wl.engine(comm_setup)
            t2, _ = timed_updates(e2, wl, max(1, min(args.steps, 3)), 1, barrier)
            e2.close()
            del e2
            torch.cuda.empty_cache()
        finally:
            set_option("split_f16", saved)
        k2 = max(1, min(args.steps, 3))
        alt = {"arithmetic": "bf16x6: every fp32 operand split exactly into hi+mid+lo bf16 (6 products)",
               "value": k2 / t2, "unit": "updates/s", "ms_per_step": 1e3 * t2 / k2, "steps": k2}

    if args.profile_out and rank == 0:
        with open(args.profile_out, "w") as f:
            json.dump({"profile": prof, "profile_steps": args.profile_steps, "n_local": n, "widths": widths}, f,
                      indent=1)

    if rank == 0:
        # ---- roofline of the dominant kernel (HIP events on the engine stream, profile pass) ----
        psteps = max(1, args.profile_steps)
        kernel_tags = {t: v for t, v in prof.items() if tag_flops(t, widths, n) > 0}
        dom = max(kernel_tags, key=lambda t: kernel_tags[t][1])
        cnt, tot_ms = kernel_tags[dom]
        avg_s = tot_ms / cnt / 1e3
        fl = tag_flops(dom, widths, n)
        by = tag_bytes(dom, widths, n)
        alg_by = tag_x_bytes(dom, widths, n)
        peak = tag_peak(dom, widths)
        achieved = fl / avg_s / 1e12
        bound, _ = tag_roof(dom, widths, n)   # max(own bytes / HBM peak, FLOPs / MFMA peak)
        dom_prod = tag_products(dom, widths)
        peak_basis = (f"split MFMA: f16/bf16 dense peak 2.5 PF / {dom_prod} products" if tag_is_split(dom, widths)
                      else "f32 MFMA peak")
        upd_own_peak_s = sum(tag_roof(t, widths, n)[1] * c for t, (c, _) in kernel_tags.items()) / psteps
        tr = committed_traffic(args.config, N, dom) if world == 1 else None
        upd_s = elapsed / args.steps
        upd_flops_8d = update_flops_8d(widths, N)          # the whole job's (all ranks') §8(d) FLOPs
        upd_peak = peak   # the dominant (FVP) kernel's issued arithmetic: f16x3 833.3, bf16x6 416.7 or f32 157.3
        fvp_alg_bytes = n * cfg["obs"] * 4 + 3 * num_params * 4
        fvp_moved = sum(tag_bytes(t, widths, n) * c for t, (c, _) in fvp_tags.items()) / max(1, fvp_calls)
        # the split actually issued: the wide GEMMs' (f16x3 or bf16x6) unless the whole FVP is one fused
        # launch (fused.hip bf16x6, fused16.hip f16x3) and no other kernel is a split GEMM
        wide_split = any(tag_is_split(t, widths) for t in kernel_tags if t not in ("fvp_chain", "fvp_fused"))
        fvp_prod = tag_products("fvp_fused" if "fvp_fused" in kernel_tags else "fvp_chain", widths)
        arith = ("f16x3" if prod == 3 else "bf16x6") if wide_split else ("f16x3" if fvp_prod == 3 else "bf16x6")
        value = args.steps / elapsed
        metric = METRIC
        out = {
            "metric": metric,
            "value": value,
            "unit": "updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": f"fp32 ({arith} split)",
            "arithmetic": ("fp32 in HBM and f32 accumulation; GEMMs wider than 128 columns on f16 MFMA with each "
                           "fp32 operand scaled by a power of two and split into hi+lo f16 pieces (3 products, "
                           "error 2^-22 relative; a K-segment whose product scale is >= 14 binades below the "
                           "other's, the O(eps) KL_ff terms, on one product)" if prod == 3 else
                           "fp32 in HBM and f32 accumulation; GEMMs wider than 128 columns on bf16 MFMA with "
                           "each fp32 operand split exactly into hi+mid+lo bf16 pieces (6 products)") +
                          (("; the one-launch FVP (fused16.hip) on the scaled f16 hi+lo split (3 products)"
                            if fvp_prod == 3 else
                            "; the one-launch FVP (fused.hip) on the exact bf16 hi+mid+lo split (6 products)")
                           if "fvp_fused" in kernel_tags else "") +
                          "; narrower GEMMs on f32 MFMA; softmax heads and CG scalars in f64",
            "data": "synthetic (X~N(0,1), a~U{0..A-1}, rewards~U(0,1), paths of 200 steps, "
                    "random-init policy, pi_old = p(theta_0))",
            "timing": "timed region = K updates replayed from the captured update hipGraph (production path); "
                      "kernel times from a separate eager pass with per-launch HIP events",
            "config": {"workload": cfg["name"] + "; full update = discount+standardise+pg+10 CG+shs FVP+"
                                                 "line search+final losses",
                       "n_states": N, "obs_dim": cfg["obs"], "hidden": cfg["hidden"], "n_actions": cfg["A"],
                       "num_params": num_params, "cg_iters": 10, "residual_tol": 0.0,
                       "parallelism": f"dp{world} (row shards, RCCL all-reduce of [P] FVP/grad + loss scalars)"
                       if not rehearsal or world == 1 else
                       f"dp{world} on {ndev} GPU(s): rehearsal, ranks share GPUs, gloo host all-reduce"},
            "roofline": {"bound": "mfma", "kernel": dom,
                         "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
                         "traffic": tr[1]["traffic_bytes"] if tr else None,
                         "bound_basis": "SURVEY.md §8(d): the FVP is compute-bound at every config (arithmetic "
                                        "intensity >= 187 flop/B of algorithmic bytes)",
                         "achieved_basis": "SURVEY.md §8(d) algorithmic FLOPs of this kernel's share of the FVP "
                                           "(4ab R-forward / 4ab R-backward / 4ab weight-R-gradient per state and "
                                           "layer, 2ab for layer 1's R-forward and weight R-gradient) / its average "
                                           "launch time (HIP events on the engine stream)",
                         "peak_basis": peak_basis,
                         "flops_per_launch": fl, "avg_launch_ms": avg_s * 1e3, "launches": cnt,
                         "algorithmic_bytes_per_launch": alg_by,
                         "algorithmic_bytes_frac": alg_by / avg_s / 1e9 / PEAK_HBM_GBS,
                         "own_bytes_bound": bound,
                         "own_traffic_bytes_per_launch": by,
                         "own_traffic_hbm_gbs": by / avg_s / 1e9,
                         "own_traffic_hbm_frac": by / avg_s / 1e9 / PEAK_HBM_GBS,
                         "hbm_gbs_at_traffic": tr[1]["traffic_bytes"] / avg_s / 1e9 if tr else None,
                         "traffic_source": tr[0] if tr else None,
                         "traffic_build": tr[2] if tr else None,
                         "build": source_build_id(),
                         "traffic_same_build": bool(tr and tr[2] == source_build_id())},
            "update_roofline": {"algorithmic_tflop_per_update": upd_flops_8d / 1e12,
                                "achieved_tflops": upd_flops_8d / upd_s / 1e12,
                                "peak_tflops": upd_peak,
                                "roof_ms_per_update": upd_flops_8d / (upd_peak * 1e12) * 1e3,
                                "frac": upd_flops_8d / upd_s / 1e12 / upd_peak,
                                "frac_of_f32_peak": upd_flops_8d / upd_s / 1e12 / PEAK_F32_TFLOPS,
                                "basis": "SURVEY.md §8(d): N*(grad + 11*FVP + 1*fwd) FLOPs per update (grad = "
                                         "4a1b1 + 6 sum a_l b_l, FVP = 4a1b1 + 12 sum, fwd = 2 sum over layers) / "
                                         "ms_per_step / the dense peak of the arithmetic the dominant FVP kernel issues "
                                         "(frac_of_f32_peak: against §8(d)'s fp32 roof)",
                                "own_bytes_roof_ms_per_update": upd_own_peak_s * 1e3,
                                "own_bytes_frac_of_roof": upd_own_peak_s / upd_s},
            "fvp": {"ms_per_fvp": fvp_s * 1e3,
                    "gbps_algorithmic": fvp_alg_bytes / fvp_s / 1e9,
                    "hbm_frac_algorithmic": fvp_alg_bytes / fvp_s / 1e9 / PEAK_HBM_GBS,
                    "algorithmic_bytes": fvp_alg_bytes,
                    "moved_bytes": fvp_moved,
                    "traffic_vs_algorithmic": fvp_moved / fvp_alg_bytes,
                    "tflops": fvp_flops_per_row(widths) * n / fvp_s / 1e12},
            "alt_arithmetic": alt,
            "comm": comm,
            "last_update": {k: last[k] for k in ("cg_iters", "k", "reverted", "kl_after", "surr_after")},
            "cpu_baseline": None,
        }
        if rehearsal and world > 1:
            # ranks shared GPUs: not a measurement of N GPUs
            out["rehearsal"] = True
            out["n_gpus"] = min(ndev, local_world)
            out["rehearsal_updates_per_s"] = value
            out["value"] = None
            out["update_roofline"]["achieved_tflops"] = None
        if world == 1 and not args.no_cpu_baseline:
            threads, rep = host_cores()
            rows = args.cpu_rows or min(cfg["cpu_rows"], N)
            out["cpu_baseline"] = cpu_baseline(cfg, rows, threads, rep)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    enforce_rank_check(comm)


if __name__ == "__main__":
    main()
