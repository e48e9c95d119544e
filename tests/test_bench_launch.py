"""bench.py's multi-rank launch logic (CPU only: no rank ever reaches the GPU here).

`python bench.py --gpus N` without WORLD_SIZE must start N ranks itself (the driver's scaling run uses
that form), refuse more ranks than visible GPUs unless --rehearsal, and print no JSON line when it
refuses.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _env_without_world():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    return env


def test_more_ranks_than_gpus_fails_cleanly():
    # this container has no GPU: --gpus 8 must exit non-zero before any GPU work, with no JSON line
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], cwd=ROOT,
                       env=_env_without_world(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr
    for line in r.stdout.splitlines():
        with pytest.raises(ValueError):
            json.loads(line)


def test_launcher_command(monkeypatch):
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    monkeypatch.setattr(subprocess, "call", fake_call)
    rc = bench.launch_ranks(["--gpus", "4", "--steps", "2"], 4, False, visible_gpus=8)
    assert rc == 7                                  # the launcher's status is the parent's exit status
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "2"]
    assert cmd[-5].endswith("bench.py")
    assert any(c.startswith("--master-port=") and int(c.split("=")[1]) > 0 for c in cmd)


def test_launcher_refuses_without_rehearsal(monkeypatch):
    monkeypatch.setattr(subprocess, "call", lambda *a, **k: pytest.fail("must not launch"))
    assert bench.launch_ranks(["--gpus", "2"], 2, False, visible_gpus=1) != 0


def test_launcher_rehearsal_allows_shared_gpus(monkeypatch):
    monkeypatch.setattr(subprocess, "call", lambda cmd, env=None: 0)
    assert bench.launch_ranks(["--gpus", "2", "--rehearsal"], 2, True, visible_gpus=1) == 0


def test_world_size_mismatch_is_refused():
    env = _env_without_world()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_committed_traffic_prefers_the_current_build(tmp_path, monkeypatch):
    """The bench's roofline `traffic` comes from the committed PMC file measured on its own source build when
    there is one (a later-named file of another build must not shadow it), else from the last file in name order."""
    build = bench.source_build_id()
    for name, b, val in (("r9a", build, 1.0), ("r9z", "0000000000000000", 2.0)):
        d = tmp_path / "profiles" / name
        d.mkdir(parents=True)
        (d / "traffic.json").write_text(json.dumps({"config": "c4", "rows": 8, "build": b,
                                                    "tags": {"fvp_x": {"bytes": val}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "source_build_id", lambda: build)
    path, entry, b = bench.committed_traffic("c4", 8, "fvp_x")
    assert path.endswith(os.path.join("r9a", "traffic.json")) and b == build and entry["bytes"] == 1.0
    monkeypatch.setattr(bench, "source_build_id", lambda: "ffffffffffffffff")
    path, entry, b = bench.committed_traffic("c4", 8, "fvp_x")
    assert path.endswith(os.path.join("r9z", "traffic.json")) and entry["bytes"] == 2.0


def _rank_check_worker(rank, world, port, digests, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        chk = bench.gather_rank_check(digests[rank], 10.0 + rank, world, dist)
        try:
            bench.enforce_rank_check(chk)
            code = 0
        except SystemExit as e:
            code = e.code
        q.put((rank, chk, code))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("digests,equal", [(("aa", "aa"), True), (("aa", "ab"), False)])
def test_rank_check_two_gloo_ranks(digests, equal):
    """World-size-2 gloo: bench.py's post-timing self-check gathers every rank's update digest and FVP time;
    differing digests give ranks_bitwise_equal = False and exit status 3 on every rank."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_check_worker, args=(r, 2, port, digests, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=120) for _ in range(2)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, chk, code in outs:
        assert chk["ranks_bitwise_equal"] is equal
        assert chk["rank_digests"] == list(digests)
        assert chk["fvp_ms_per_rank"] == [10.0, 11.0]
        assert code == (0 if equal else 3)


def test_rank_digest_sees_every_bit():
    import numpy as np
    stats = {k: 1.0 for k in bench.DIGEST_STATS}
    v = [np.arange(10, dtype=np.float32), np.ones(10, np.float32)]
    d0 = bench.rank_digest(v, stats)
    assert d0 == bench.rank_digest([x.copy() for x in v], dict(stats))
    w = v[0].copy()
    w.view(np.uint32)[3] ^= 1                      # one ulp of one element
    assert bench.rank_digest([w, v[1]], stats) != d0
    assert bench.rank_digest(v, dict(stats, rdotr=np.nextafter(1.0, 2.0))) != d0


def test_fused_fvp_roofline_follows_the_issued_arithmetic():
    """The one-launch FVP is priced at the peak of the split it issues: f16 hi+lo (3 products) for fused16.hip's
    shapes with fused = 3, the exact bf16 split (6) for fused.hip; the fused policy gradient at 3, with its FLOPs
    (backward below the head + every weight gradient) and bytes (X, H_l, DS_{L-1})."""
    from trpo_amd._lib import get_option, set_option
    c3 = [128, 64, 64, 18]
    saved = get_option("fused"), get_option("split_f16")
    try:
        set_option("split_f16", 1)
        set_option("fused", 3)
        assert bench.fused16_used(c3) and bench.tag_products("fvp_fused", c3) == 3
        assert bench.tag_peak("fvp_fused", c3) == pytest.approx(bench.PEAK_BF16_TFLOPS / 3)
        assert bench.fused16_used([4, 64, 2])                  # one hidden layer (the reference policy): fused16
        assert bench.tag_products("fvp_fused", [4, 64, 2]) == 3
        assert bench.fused16_used([37, 50, 33, 7])             # hidden widths below 49: padded images
        assert not bench.fused16_used([4, 65, 2])              # wider than 64: not a fused shape
        assert not bench.fused16_used([4, 64, 64, 64, 2])      # three hidden layers
        set_option("fused", 2)
        assert bench.tag_products("fvp_fused", c3) == 6
        set_option("fused", 3)
        set_option("split_f16", 0)
        assert bench.tag_products("fvp_fused", c3) == 6       # fused16 needs the f16 split
    finally:
        set_option("fused", saved[0])
        set_option("split_f16", saved[1])
    n = 1000
    assert bench.tag_flops("pg_fused", c3, n) == 2.0 * n * ((64 * 64 + 64 * 18) + (128 * 64 + 64 * 64 + 64 * 18))
    assert bench.tag_bytes("pg_fused", c3, n) == 4.0 * n * sum(c3)
    assert bench.tag_is_split("pg_fused", c3) and bench.tag_products("pg_fused", c3) == 3
    # fwd_loss16 (one-launch policy forwards): the whole forward's FLOPs; X + pi_old for the line search, plus
    # H_1, H_2, P, D_2, DS_2 out for the prepare pass; per-layer tags keep their own pricing
    fwd_flops = 2.0 * n * (128 * 64 + 64 * 64 + 64 * 18)
    for tag in ("fwd", "ls_fwd"):
        assert bench.tag_flops(tag, c3, n) == fwd_flops
        assert bench.tag_is_split(tag, c3) and bench.tag_products(tag, c3) == 3
        assert bench.tag_x_bytes(tag, c3, n) == 4.0 * n * 128
    assert bench.tag_bytes("ls_fwd", c3, n) == 4.0 * n * (128 + 18)
    assert bench.tag_bytes("fwd", c3, n) == 4.0 * n * (128 + 4 * 18 + 64 + 64)
    assert bench.tag_flops("ls_fwd_l1", c3, n) == 2.0 * n * 64 * 64


def test_rfwd_tags_price_layers_0_and_1_together():
    """rfwd.hip's one-launch tags at C4 widths: fvp_rfwd01 (X V0 + RH1 W1 + H1 V1; X planes, H1 in, RH1 and RZ2 out)
    and the forwards' fwd_l01 / ls_fwd_l01 (X W0 + H1 W1; H1 out only in the prepare pass), all on the 3-product
    f16 split and reading X -- not the per-layer pricing their "_l01" suffix would otherwise select."""
    c4 = [128, 256, 256, 18]
    n = 1000
    assert bench.tag_flops("fvp_rfwd01", c4, n) == 2.0 * n * 128 * 256 + 4.0 * n * 256 * 256
    assert bench.tag_bytes("fvp_rfwd01", c4, n) == 4.0 * n * (128 + 2 * 256 + 256)
    for tag in ("fwd_l01", "ls_fwd_l01"):
        assert bench.tag_flops(tag, c4, n) == 2.0 * n * (128 * 256 + 256 * 256)
        assert bench.tag_is_split(tag, c4) and bench.tag_products(tag, c4) == 3
        assert bench.tag_x_bytes(tag, c4, n) == 4.0 * n * 128
    assert bench.tag_bytes("fwd_l01", c4, n) == 4.0 * n * (128 + 256 + 256)
    assert bench.tag_bytes("ls_fwd_l01", c4, n) == 4.0 * n * (128 + 256)
    assert bench.tag_products("fvp_rfwd01", c4) == 3 and bench.tag_x_bytes("fvp_rfwd01", c4, n) == 4.0 * n * 128
