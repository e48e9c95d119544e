"""GPU parity: the HIP engine (through the C-ABI) vs the golden fixtures and the
CPU oracle on the same seeded inputs.  Bar: vectors
norm-relative <= 1e-5 plus elementwise allclose(rtol=1e-5, atol=1e-5 max|b|);
scalars relative 1e-5; CG iteration count and line-search k exact; integer
index work exact."""
import numpy as np
import pytest

from conftest import assert_vec_close, golden, rel_l2, spec_of, update_fixtures
from oracle import trpo_oracle as O

pytestmark = pytest.mark.gpu
REL = 1e-5


def make_engine(d, n=None, **kw):
    from trpo_amd import Engine
    spec = spec_of(d)
    n = n or d["X"].shape[0]
    eng = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=max(n, 16), **kw)
    eng.set_flat(d["theta"])
    eng.set_batch(d["X"], d["actions"], np.asarray(d["advant"], np.float32), d["old_dist"])
    return eng, spec


@pytest.mark.parametrize("name", update_fixtures())
def test_fvp_and_grad_vs_golden(gpu_available, name):
    d = golden(name)
    eng, spec = make_engine(d)
    hv = eng.fvp(d["v"].astype(np.float32), damping=0.0)
    assert_vec_close(hv, d["hv"], REL, f"{name} Hv")
    damped = eng.fvp(d["v"].astype(np.float32), damping=0.1)
    assert_vec_close(damped, d["hv"] + 0.1 * d["v"].astype(np.float32), REL, f"{name} Hv+0.1v")
    g = eng.policy_grad()
    assert_vec_close(g, d["g"], REL, f"{name} g")
    ls = eng.losses()
    lb = d["losses_before"]
    # surr and ent are O(1); kl at theta_prev is ~0 in steady state -> absolute bar
    assert ls[0] == pytest.approx(lb[0], rel=REL, abs=1e-7)
    assert ls[2] == pytest.approx(lb[2], rel=REL)
    assert ls[1] == pytest.approx(lb[1], rel=REL, abs=1e-6)


def _cg_margin_ok(d, spec):
    """True when no CG residual lands within 2x of residual_tol (fp32 could flip the exit)."""
    tol = float(d["residual_tol"])
    if tol <= 0:
        return True
    th = d["theta"].astype(np.float64)
    b = -d["g"]
    p, r, rr = b.copy(), b.copy(), b.dot(b)
    for _ in range(int(d["cg_iters"])):
        z = O.fisher_vector_product(th, d["X"], p, spec)
        v = rr / p.dot(z)
        r = r - v * z
        new = r.dot(r)
        p = r + (new / rr) * p
        rr = new
        if 0.5 * tol < rr < 2 * tol:
            return False
    return True


@pytest.mark.parametrize("name", update_fixtures())
def test_update_vs_golden(gpu_available, name):
    from trpo_amd import UpdateParams
    from trpo_amd._lib import VEC_STEPDIR, VEC_FULLSTEP, VEC_THETA_LS, VEC_G
    d = golden(name)
    eng, spec = make_engine(d)
    st = eng.update(UpdateParams(cg_iters=10, residual_tol=float(d["residual_tol"]), max_kl=float(d["max_kl"])))
    if _cg_margin_ok(d, spec):
        assert st["cg_iters"] == int(d["cg_iters"])
        assert_vec_close(eng.get_vector(VEC_STEPDIR), d["stepdir"], REL, f"{name} stepdir")
        assert st["shs"] == pytest.approx(float(d["shs"]), rel=REL)
        assert st["lm"] == pytest.approx(float(d["lm"]), rel=REL)
    assert_vec_close(eng.get_vector(VEC_G), d["g"], REL, f"{name} g")
    assert st["k"] == int(d["k"])
    assert bool(st["reverted"]) == bool(d["reverted"])
    if _cg_margin_ok(d, spec):
        assert_vec_close(eng.get_vector(VEC_FULLSTEP), d["fullstep"], REL, f"{name} fullstep")
        assert_vec_close(eng.get_vector(VEC_THETA_LS), d["theta_ls"], REL, f"{name} theta_ls")
    assert_vec_close(eng.get_flat(), d["theta_new"], REL, f"{name} theta_new")
    la = d["losses_after"]
    assert st["surr_after"] == pytest.approx(la[0], rel=REL, abs=1e-7)
    assert st["kl_after"] == pytest.approx(la[1], rel=REL, abs=1e-7)
    assert st["ent_after"] == pytest.approx(la[2], rel=REL)


@pytest.mark.parametrize("name", ["update_c2.npz", "update_c3.npz", "update_deep_odd.npz"])
def test_update_forced_iters_vs_oracle(gpu_available, name):
    """residual_tol = 0 (benchmark mode, exactly 10 CG iterations) vs the oracle run live."""
    from trpo_amd import UpdateParams
    from trpo_amd._lib import VEC_STEPDIR
    d = golden(name)
    eng, spec = make_engine(d)
    st = eng.update(UpdateParams(cg_iters=10, residual_tol=0.0))
    r = O.trpo_update(d["theta"].astype(np.float64), O.Batch(d["X"], d["actions"], d["advant"], d["old_dist"]),
                      spec, np.float64, 10, 0.0)
    assert st["cg_iters"] == 10 == r.cg_iters
    assert st["k"] == r.k
    assert_vec_close(eng.get_vector(VEC_STEPDIR), r.stepdir, REL, "stepdir")
    assert st["shs"] == pytest.approx(r.shs, rel=REL)
    assert_vec_close(eng.get_flat(), r.theta_new, REL, "theta_new")


def test_stepwise_utils_surface_matches_fused(gpu_available):
    """trpo_inksci.py:144-158 written over trpo_amd.utils == the fused trpo_update."""
    from trpo_amd import TRPOAgent
    d = golden("update_c2.npz")
    spec = spec_of(d)
    batch = {"state": d["X"], "action": d["actions"], "action_dist": d["old_dist"],
             "advant": np.asarray(d["advant"], np.float32)}
    a1 = TRPOAgent(spec.obs_dim, spec.n_actions, spec.hidden, max_rows=4096, theta=d["theta"])
    a2 = TRPOAgent(spec.obs_dim, spec.n_actions, spec.hidden, max_rows=4096, theta=d["theta"])
    s1 = a1.update(batch)
    s2 = a2.update_stepwise(batch)
    assert_vec_close(a2.gf(), d["theta_new"], REL, "stepwise theta_new")
    assert_vec_close(a1.gf(), a2.gf(), REL, "fused vs stepwise")
    assert s2["kl_after"] == pytest.approx(s1["kl_after"], rel=REL)


def test_advantages_from_rewards(gpu_available):
    d = golden("update_c3.npz")
    eng, spec = make_engine(d)
    eng.set_rewards(d["rewards"], d["starts"])
    ret, adv = eng.compute_advantages(0.95)
    np.testing.assert_allclose(ret, d["returns"], rtol=1e-13)
    np.testing.assert_allclose(adv, d["advant"], rtol=1e-11, atol=1e-12)
    # the update that starts from rewards equals the one fed the advantages
    from trpo_amd import UpdateParams
    st = eng.update(UpdateParams(compute_advantages=True, gamma=0.95))
    assert st["k"] == int(d["k"])
    assert_vec_close(eng.get_flat(), d["theta_new"], REL, "theta_new from rewards")


def test_discount_vs_golden(gpu_available):
    from trpo_amd import utils
    d = golden("discount.npz")
    for k in sorted(x[:-2] for x in d.files if x.endswith("_x")):
        gamma = float(k.split("_")[0][1:])
        np.testing.assert_allclose(utils.discount(d[k + "_x"], gamma), d[k + "_y"], rtol=1e-13, err_msg=k)


@pytest.mark.parametrize("n,p_start", [(1, 0.0), (2, 1.0), (4097, 0.0), (100_003, 0.005),
                                       (1_000_000, 0.0), (2_000_000, 1.0 / 200)])
def test_discount_segmented_large(gpu_available, n, p_start):
    """Sizes past one scan tile / one block-map pass; checked against scipy's lfilter per path."""
    import scipy.signal
    from trpo_amd.engine import discount_device
    rng = np.random.RandomState(n)
    x = rng.uniform(0, 1, n)
    starts = (rng.uniform(size=n) < p_start).astype(np.uint8)
    starts[0] = 1
    y = discount_device(x, 0.99, starts)
    idx = list(np.flatnonzero(starts)) + [n]
    ref = np.empty(n)
    for a, b in zip(idx[:-1], idx[1:]):
        ref[a:b] = scipy.signal.lfilter([1], [1, -0.99], x[a:b][::-1])[::-1]
    np.testing.assert_allclose(y, ref, rtol=1e-12)


def test_generic_cg_vs_golden(gpu_available):
    from trpo_amd import utils
    d = golden("cg.npz")
    for case in d["cases"]:
        base = str(d[case + "_base"])
        A, b = d[base + "_A"], d[base + "_b"]
        x, it = utils.conjugate_gradient(lambda p: A @ p, b, int(d[case + "_maxit"]), float(d[case + "_tol"]),
                                         return_iters=True)
        assert x.dtype == b.dtype
        want = d[case + "_x"]
        if b.dtype == np.float64:
            assert it == int(d[case + "_iters"]), case
            assert rel_l2(x, want) < 1e-9, case
        else:
            assert abs(it - int(d[case + "_iters"])) <= 1, case
            assert rel_l2(A.astype(np.float64) @ x, A.astype(np.float64) @ want) < 1e-3 or rel_l2(x, want) < 1e-4, case


def test_engine_linesearch_vs_oracle(gpu_available):
    """linesearch(loss, x, fullstep, rate) on the device vs the oracle, large max_kl
    fixture (backtracks to k=2) and a rejected search."""
    from trpo_amd import utils
    from trpo_amd.utils import EngineLoss
    d = golden("update_c2_bigkl.npz")
    eng, spec = make_engine(d)
    loss = EngineLoss(eng)
    x = d["theta"].astype(np.float32)
    full = d["fullstep"].astype(np.float32)
    res = utils.linesearch(loss, x, full, float(d["rate"]))
    assert_vec_close(res, d["theta_ls"], REL, "theta_ls")
    # rejected: a step along +g increases surr -> returns x itself
    g = d["g"].astype(np.float32)
    res2 = utils.linesearch(loss, x, g * 10, 1.0)
    assert res2 is x


def test_sharded_partials_sum_to_full(gpu_available):
    """Two engines on two halves with n_global = N: their partial FVP / grad sum to the full one
    (what RCCL's all-reduce adds up across ranks)."""
    from trpo_amd import Engine
    d = golden("update_c3.npz")
    spec = spec_of(d)
    n = d["X"].shape[0]
    cut = n // 2
    parts_hv, parts_g = [], []
    v = d["v"].astype(np.float32)
    for lo, hi in ((0, cut), (cut, n)):
        e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
        e.set_flat(d["theta"])
        e.set_batch(d["X"][lo:hi], d["actions"][lo:hi], np.asarray(d["advant"][lo:hi], np.float32),
                    d["old_dist"][lo:hi], n_global=n)
        parts_hv.append(e.fvp(v, 0.0).astype(np.float64))
        parts_g.append(e.policy_grad().astype(np.float64))
    assert_vec_close(parts_hv[0] + parts_hv[1], d["hv"], REL, "sharded Hv")
    assert_vec_close(parts_g[0] + parts_g[1], d["g"], REL, "sharded g")


def test_deterministic(gpu_available):
    d = golden("update_c3.npz")
    eng, spec = make_engine(d)
    v = d["v"].astype(np.float32)
    a = eng.fvp(v, 0.1)
    b = eng.fvp(v, 0.1)
    np.testing.assert_array_equal(a, b)


def test_large_batch_properties(gpu_available):
    """At sizes the oracle cannot run quickly: symmetry u.Hv = v.Hu, linearity, and
    sharding invariance of the FVP; C3 dims, 300k states."""
    from trpo_amd import Engine
    spec = O.PolicySpec(128, [64, 64], 18)
    n = 300_000
    rng = np.random.RandomState(0)
    X = rng.standard_normal((n, spec.obs_dim)).astype(np.float32)
    th = O.init_theta(spec, rng)
    act = rng.randint(0, spec.n_actions, n)
    adv = rng.standard_normal(n).astype(np.float32)
    eng = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
    eng.set_flat(th)
    # old_dist = p(theta): the engine's own forward via a first batch with uniform old_dist
    old = np.full((n, spec.n_actions), 1.0 / spec.n_actions, np.float32)
    eng.set_batch(X, act, adv, old)
    u = rng.standard_normal(spec.n_params).astype(np.float32)
    v = rng.standard_normal(spec.n_params).astype(np.float32)
    Hu = eng.fvp(u, 0.0).astype(np.float64)
    Hv = eng.fvp(v, 0.0).astype(np.float64)
    assert abs(u @ Hv - v @ Hu) <= 1e-5 * abs(u @ Hv)
    Hw = eng.fvp((2.0 * u - 3.0 * v).astype(np.float32), 0.0).astype(np.float64)
    assert rel_l2(Hw, 2.0 * Hu - 3.0 * Hv) < 1e-5
    assert u @ Hu > 0 and v @ Hv > 0          # KL Hessian is PSD
    # a slice checked directly against the oracle
    m = 3000
    ref = O.fvp_undamped(th.astype(np.float64), X[:m], u.astype(np.float64), spec, n_global=n)
    e2 = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=m)
    e2.set_flat(th)
    e2.set_batch(X[:m], act[:m], adv[:m], old[:m], n_global=n)
    assert_vec_close(e2.fvp(u, 0.0), ref, REL, "slice Hv")


def test_bad_actions_fail_loudly(gpu_available):
    from trpo_amd import Engine
    from trpo_amd._lib import EngineError
    e = Engine(4, [8], 2, max_rows=8)
    with pytest.raises(EngineError, match="action"):
        e.set_batch(np.zeros((4, 4), np.float32), np.array([0, 1, 2, 0]), np.zeros(4, np.float32),
                    np.full((4, 2), .5, np.float32))


@pytest.mark.parametrize("opts", [
    {"chain": 2}, {"chain": 3},               # fused FVP chain forms (default 1 = auto)
    {"chain": 0},                               # per-layer row-GEMM FVP
    {"split_mfma": 0}, {"chain": 0, "split_mfma": 1}, {"chain": 0, "split_mfma": 5},
    {"split_mfma": 6}, {"chain": 0, "split_mfma": 6},         # 256 x 256 at BK 16 (round-3 default)
    {"split_wg": 0}, {"split_wg": 1},
    {"split_mfma": 5, "split_wg": 1},
    {"split_f16": 0}, {"split_f16": 0, "split_wg": 1},        # bf16 three-piece split (6 products)
    {"split_f16": 0, "chain": 2}, {"chain": 2, "split_wg": 1},
    {"split_min_k": 64}, {"split_min_k": 64, "chain": 0},  # few-k row GEMMs on the f32 tile
    {"fused": 0}, {"fused": 1},                               # chain + GEMM weight gradients ; 8-wave fused FVP
    {"fused": 2}, {"fused": 3, "split_f16": 0},               # bf16 4-wave fused FVP ; the f16 default without f16
    {"low_seg": 0}, {"low_seg": 0, "chain": 0},               # every split segment on three products
    {"planes": 0},                                            # register-staged split instead of the plane kernel
    {"tail": 0}, {"tail": 0, "chain": 0},                     # per-layer last-layer kernels instead of tail.hip
    {"rbwd0": 0}, {"rbwd0": 0, "chain": 0},                   # per-layer R-backward + layer-0 weight gradient
    {"hbwd2": 0}, {"hbwd2": 0, "chain": 0},                   # separate head backwards (prepare / policy gradient)
    {"hbwd2": 1},                                             # the dual head backward on VALU fmaf chains
    {"head_fwd": 0}, {"head_fwd": 2}, {"head_fwd": 0, "chain": 0},   # the f32 MFMA row GEMM's 32-lane softmax head
    {"splits": 64, "pg_splits": 256}, {"splits": 3000, "pg_splits": 100},   # other split-K geometries
    {"ls_fused": 0},                                          # the line search's per-layer forward on fused16 shapes
    {"ls_fused": 2},                                          # per-layer prepare forward, one-launch trial forwards
    {"cg_fuse_reduce": 0},                                    # the CG's separate slab reduction on fused16 shapes
    {"cg_fuse_reduce": 2},                                    # the whole CG iteration after the FVP in one launch
    {"cg_p_img": 0},                                          # the CG's p update and the V images as two launches
    {"rfwd01": 0},                                            # R-forward of layers 0 / 1 as two launches (C4 dims)
    {"fwd01": 0},                                             # the forward's layers 0 / 1 as two launches (C4 dims)
], ids=lambda o: ",".join(f"{k}={v}" for k, v in o.items()))
def test_kernel_variants_parity(gpu_available, opts):
    """Every selectable kernel variant reproduces the golden FVP / gradient / update at C3 and
    C1 dims, plus a 256-wide case that exercises the wide row-GEMM tiles and the widest chain."""
    from trpo_amd import Engine, UpdateParams
    from trpo_amd._lib import get_option, set_option
    defaults = {k: get_option(k) for k in ("split_mfma", "split_wg", "chain", "split_f16", "split_min_k", "fused",
                                           "low_seg", "planes", "tail", "rbwd0", "hbwd2", "head_fwd",
                                           "splits", "pg_splits", "ls_fused", "cg_fuse_reduce", "rfwd01",
                                           "cg_p_img", "fwd01")}
    try:
        for k, v in opts.items():
            set_option(k, v)
        for name in ("update_c3.npz", "update_c1.npz"):
            d = golden(name)
            eng, spec = make_engine(d)
            assert_vec_close(eng.fvp(d["v"].astype(np.float32), 0.0), d["hv"], REL, f"{name} Hv {opts}")
            assert_vec_close(eng.policy_grad(), d["g"], REL, f"{name} g {opts}")
            st = eng.update(UpdateParams(residual_tol=float(d["residual_tol"])))
            assert st["k"] == int(d["k"])
            assert_vec_close(eng.get_flat(), d["theta_new"], REL, f"{name} theta {opts}")
        # wide layers (row GEMM N = 256 path, 256x256 weight gradient)
        spec = O.PolicySpec(128, [256, 256], 18)
        dd = O.synthetic_batch(spec, 700, seed=21)
        e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=700)
        e.set_flat(dd["theta"])
        e.set_batch(dd["X"], dd["actions"], dd["advant"].astype(np.float32), dd["old_dist"])
        v = np.random.RandomState(22).standard_normal(spec.n_params).astype(np.float32)
        ref = O.fvp_undamped(dd["theta"].astype(np.float64), dd["X"], v.astype(np.float64), spec)
        assert_vec_close(e.fvp(v, 0.0), ref, REL, f"wide Hv {opts}")
        gref = O.policy_grad(dd["theta"].astype(np.float64), dd["X"], dd["actions"], dd["advant"], dd["old_dist"], spec)
        assert_vec_close(e.policy_grad(), gref, REL, f"wide g {opts}")
        # odd wide widths: K not a multiple of 16, a partial 256-column tile, 3 hidden layers
        spec = O.PolicySpec(37, [200, 264, 144], 5)
        dd = O.synthetic_batch(spec, 1337, seed=23)
        e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=1337)
        e.set_flat(dd["theta"])
        e.set_batch(dd["X"], dd["actions"], dd["advant"].astype(np.float32), dd["old_dist"])
        v = np.random.RandomState(24).standard_normal(spec.n_params).astype(np.float32)
        ref = O.fvp_undamped(dd["theta"].astype(np.float64), dd["X"], v.astype(np.float64), spec)
        assert_vec_close(e.fvp(v, 0.0), ref, REL, f"odd-wide Hv {opts}")
        gref = O.policy_grad(dd["theta"].astype(np.float64), dd["X"], dd["actions"], dd["advant"], dd["old_dist"], spec)
        assert_vec_close(e.policy_grad(), gref, REL, f"odd-wide g {opts}")
        st = e.update(UpdateParams(residual_tol=0.0))
        r = O.trpo_update(dd["theta"].astype(np.float64), O.Batch(dd["X"], dd["actions"], dd["advant"], dd["old_dist"]),
                          spec, np.float64, 10, 0.0)
        assert st["k"] == r.k
        assert_vec_close(e.get_flat(), r.theta_new, REL, f"odd-wide theta {opts}")
    finally:
        for k, v in defaults.items():
            set_option(k, v)


@pytest.mark.parametrize("obs,hidden,A,n", [
    (11, [64, 64], 3, 3001),           # C2 dims, a partial last 16-state group
    (128, [64, 64], 18, 100_000),      # C3 dims, many groups per wave
    (40, [64, 49], 32, 777),           # 4 obs tiles, a partial hidden tile, two action tiles
    (20, [56, 64], 17, 1),             # one state
    (64, [64, 64], 16, 40_000),        # two obs chunks, one action tile exactly full
    (4, [64], 2, 1000),                # C1 dims: one hidden layer (the reference policy, trpo_inksci.py:38-40)
    (128, [32], 32, 4099),             # one hidden layer of 32 (padded to 64), two action tiles
    (37, [50, 33], 7, 129),            # hidden widths below 49 (padded images)
    (16, [17, 48], 17, 37),            # narrow widths, one partial group
])
def test_fused16_loss_forward_vs_oracle(gpu_available, obs, hidden, A, n):
    """The policy forward in one launch (fused16.hip fwd_loss16, ls_fused = 1) against the float64 oracle and the
    per-layer forward (ls_fused = 0): surr / kl / ent of trpo_inksci.py:46-53 at a trial theta through loss()
    (:127-129, the line search), and at theta through the prepare pass (its softmax P and loss_before)."""
    from trpo_amd import Engine
    from trpo_amd._lib import get_option, set_option
    spec = O.PolicySpec(obs, hidden, A)
    dd = O.synthetic_batch(spec, n, seed=n + 5)
    rs = np.random.RandomState(n + 6)
    trial = (dd["theta"] + 0.02 * rs.standard_normal(spec.n_params)).astype(np.float32)
    ref = O.losses(trial.astype(np.float64), dd["X"], dd["actions"], dd["advant"], dd["old_dist"], spec)
    saved = get_option("ls_fused")
    out = {}
    try:
        for mode in (1, 0):
            set_option("ls_fused", mode)
            e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
            e.set_flat(dd["theta"])
            e.set_batch(dd["X"], dd["actions"], dd["advant"].astype(np.float32), dd["old_dist"])
            out[(mode, "p")] = e.action_dist().astype(np.float64)
            out[(mode, "lb")] = e.losses().astype(np.float64)
            out[mode] = e.eval_losses(trial).astype(np.float64)
            out[(mode, "again")] = e.eval_losses(trial).astype(np.float64)
            e.close()
    finally:
        set_option("ls_fused", saved)
    _, p_ref = O.forward(dd["theta"].astype(np.float64), dd["X"], spec)
    lb_ref = O.losses(dd["theta"].astype(np.float64), dd["X"], dd["actions"], dd["advant"], dd["old_dist"], spec)
    for mode in (1, 0):
        assert np.max(np.abs(out[(mode, "p")] - p_ref)) <= 1e-6, mode
        assert out[(mode, "lb")][0] == pytest.approx(lb_ref[0], rel=REL, abs=1e-7), (mode, out[(mode, "lb")], lb_ref)
        assert out[(mode, "lb")][1] == pytest.approx(lb_ref[1], rel=REL, abs=1e-7), (mode, out[(mode, "lb")], lb_ref)
        assert out[(mode, "lb")][2] == pytest.approx(lb_ref[2], rel=REL), (mode, out[(mode, "lb")], lb_ref)
    for mode in (1, 0):
        got = out[mode]
        assert got[0] == pytest.approx(ref[0], rel=REL, abs=1e-7), (mode, got, ref)
        assert got[1] == pytest.approx(ref[1], rel=REL, abs=1e-7), (mode, got, ref)
        assert got[2] == pytest.approx(ref[2], rel=REL), (mode, got, ref)
        assert np.array_equal(out[mode], out[(mode, "again")])   # deterministic


@pytest.mark.parametrize("obs,hidden,A,n", [
    (11, [64, 64], 3, 3001),           # C2 dims, partial last group
    (128, [64, 64], 18, 100_000),      # C3 dims, many groups per persistent workgroup
    (40, [64, 49], 32, 777),           # 4 obs tiles, a partial hidden tile, A = 32
    (20, [56, 64], 17, 1),             # one state
    (4, [64], 2, 1000),                # C1 dims: one hidden layer
    (128, [32], 32, 63),               # one hidden layer of 32, a single partial group
    (37, [50, 33], 7, 129),            # hidden widths below 49
])
def test_fused16_policy_grad_vs_oracle(gpu_available, obs, hidden, A, n):
    """The policy gradient in one launch (fused16.hip's PG form, fused = 3) against the float64 oracle and the
    row-GEMM backward + weight-gradient path (fused = 2), deterministic (trpo_inksci.py:54, utils.py:160)."""
    from trpo_amd import Engine
    from trpo_amd._lib import get_option, set_option
    spec = O.PolicySpec(obs, hidden, A)
    dd = O.synthetic_batch(spec, n, seed=n + 11)
    ref = O.policy_grad(dd["theta"].astype(np.float64), dd["X"], dd["actions"], dd["advant"], dd["old_dist"], spec)
    saved = get_option("fused")
    out = {}
    try:
        for mode in (3, 2):
            set_option("fused", mode)
            e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
            e.set_flat(dd["theta"])
            e.set_batch(dd["X"], dd["actions"], dd["advant"].astype(np.float32), dd["old_dist"])
            out[mode] = e.policy_grad()
            out[(mode, "again")] = e.policy_grad()
            e.close()
    finally:
        set_option("fused", saved)
    assert_vec_close(out[3], ref, REL, f"fused16 g {obs} {hidden} {A} n={n}")
    assert_vec_close(out[3], out[2], REL, f"fused16 vs row-GEMM g {obs} {hidden} {A} n={n}")
    assert np.array_equal(out[3], out[(3, "again")]), "fused16 policy gradient is not deterministic"


@pytest.mark.parametrize("obs,hidden,A,n", [
    (37, [200, 72, 144], 5, 1337),     # odd widths, 3 hidden layers, 16 register tiles, partial workgroup
    (128, [256, 256], 18, 3001),       # C4 dims, two head tiles
    (11, [64], 32, 500),               # one hidden layer (the reference policy's depth), A = 32
    (5, [16, 16], 17, 129),            # narrowest tiles
])
def test_chain_shapes_vs_oracle(gpu_available, obs, hidden, A, n):
    """The fused FVP chain (default) against the oracle and against the per-layer row-GEMM FVP."""
    from trpo_amd import Engine
    from trpo_amd._lib import get_option, set_option
    spec = O.PolicySpec(obs, hidden, A)
    dd = O.synthetic_batch(spec, n, seed=n)
    v = np.random.RandomState(n + 1).standard_normal(spec.n_params).astype(np.float32)
    ref = O.fvp_undamped(dd["theta"].astype(np.float64), dd["X"], v.astype(np.float64), spec)
    saved = get_option("chain"), get_option("fused")
    out = {}
    try:
        set_option("fused", 0)     # the chain itself, also where the one-launch FVP (fused.hip) applies
        for mode in (1, 0):
            set_option("chain", mode)
            e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
            e.set_flat(dd["theta"])
            e.set_batch(dd["X"], dd["actions"], dd["advant"].astype(np.float32), dd["old_dist"])
            out[mode] = e.fvp(v, 0.0)
            e.close()
    finally:
        set_option("chain", saved[0])
        set_option("fused", saved[1])
    assert_vec_close(out[1], ref, REL, f"chain Hv {obs} {hidden} {A}")
    assert_vec_close(out[1], out[0], REL, f"chain vs row-GEMM Hv {obs} {hidden} {A}")


@pytest.mark.parametrize("obs,hidden,A,n", [
    (4, [64], 2, 1000),                # C1 dims (the reference policy)
    (11, [64, 64], 3, 3001),           # C2 dims, partial last group
    (128, [64, 64], 18, 2048),         # C3 dims, whole groups
    (37, [50, 33], 7, 129),            # odd widths, one state past a group
    (128, [64], 32, 63),               # one hidden layer, A = 32, a single partial group
    (16, [16, 48], 17, 1),             # one state
    (128, [64, 64], 18, 100_000),      # many groups per persistent workgroup
    (128, [64, 64], 3, 4099),          # f16 form: 8 obs tiles, one head tile
    (40, [64, 49], 32, 777),           # f16 form: 4 obs tiles, a partial hidden tile, A = 32
    (20, [56, 64], 17, 300),           # f16 form: 2 obs tiles
    (4, [64], 2, 100_000),             # C1 dims, many groups per persistent workgroup
    (11, [17], 3, 3001),               # one hidden layer of 17 (padded to 64)
])
def test_fused_fvp_vs_oracle(gpu_available, obs, hidden, A, n):
    """The one-launch FVP (fused.hip, both workgroup forms; fused16.hip on the f16 split, mode 3: every shape here,
    one or two hidden layers of width <= 64) against the float64 oracle and against the chain + weight-gradient GEMM
    path it replaces (trpo_inksci.py:56-70)."""
    from trpo_amd import Engine
    from trpo_amd._lib import get_option, set_option
    spec = O.PolicySpec(obs, hidden, A)
    dd = O.synthetic_batch(spec, n, seed=n + 7)
    v = np.random.RandomState(n + 8).standard_normal(spec.n_params).astype(np.float32)
    ref = O.fvp_undamped(dd["theta"].astype(np.float64), dd["X"], v.astype(np.float64), spec)
    saved = get_option("fused")
    out = {}
    try:
        for mode in (1, 2, 3, 0):
            set_option("fused", mode)
            e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
            e.set_flat(dd["theta"])
            e.set_batch(dd["X"], dd["actions"], dd["advant"].astype(np.float32), dd["old_dist"])
            out[mode] = e.fvp(v, 0.0)
            out[(mode, "again")] = e.fvp(v, 0.0)
            e.close()
    finally:
        set_option("fused", saved)
    for mode in (1, 2, 3):
        assert_vec_close(out[mode], ref, REL, f"fused({mode}) Hv {obs} {hidden} {A} n={n}")
        assert_vec_close(out[mode], out[0], REL, f"fused({mode}) vs chain Hv {obs} {hidden} {A} n={n}")
        assert np.array_equal(out[mode], out[(mode, "again")]), "fused FVP is not deterministic"


def run_mrank(*extra, nproc=2, timeout=600):
    """tools/mrank_check.py under torch.distributed.run (gloo rendezvous on 127.0.0.1)."""
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "tools", "mrank_check.py"),
           *extra]
    res = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=timeout)
    assert res.returncode == 0, res.stdout[-3000:] + res.stderr[-3000:]
    assert "MRANK OK" in res.stdout
    print(res.stdout.strip().splitlines()[-2])


def test_two_ranks_share_gpu_host_allreduce(gpu_available):
    """Two processes, one GPU: the engine's whole multi-rank sequence (path-aligned shards,
    1/N_global partials, all-reduced FVP / gradient / losses / standardisation sums, replicated
    CG) with the all-reduce carried by gloo; ranks must end bitwise identical and equal a
    single-rank engine; the captured update graph (host all-reduce nodes inside) replays
    bitwise identically to the eager update."""
    run_mrank("--host-allreduce", "--graphs")


def test_two_ranks_c4_dims_f16_split(gpu_available):
    """The same at C4 layer shapes (obs 128, 256x256, 18 actions), where the 256-wide GEMMs run
    on the scaled f16 hi+lo split: the running-max operand scales are per rank, the all-reduced
    partials must still give bitwise-identical ranks within 1e-5 of one rank (trpo_inksci.py:56-70,147)."""
    run_mrank("--host-allreduce", "--graphs", "--dims", "c4", "--rows", "120000")


def test_two_ranks_c5_dims_f16_split(gpu_available):
    """The same at C5 layer shapes (obs 376, 1024x1024, 17 actions: BASELINE configs[4], which the
    reference quotes on 8 GPUs), 40k rows over two ranks (trpo_inksci.py:56-70,147)."""
    run_mrank("--host-allreduce", "--dims", "c5", "--rows", "40000")


def _graph_sequence(eng, d, n_small):
    """A fixed sequence of updates exercising graph capture, replay and re-keying: repeated
    updates from theta_0, consecutive updates, a cg_iters change, a batch-size change, an
    update from rewards.  Returns every stat dict and theta after each update."""
    from trpo_amd import UpdateParams
    out = []
    th0 = d["theta"]
    adv = np.asarray(d["advant"], np.float32)

    def rec(st):
        out.append((dict(st), eng.get_flat().copy()))

    for _ in range(3):                       # eager, capture, replay
        eng.set_flat(th0)
        rec(eng.update(UpdateParams(cg_iters=10, residual_tol=0.0)))
    for _ in range(2):                       # consecutive updates (theta moves; replay)
        rec(eng.update(UpdateParams(cg_iters=10, residual_tol=0.0)))
    for _ in range(3):                       # new key: cg_iters and the default tolerance
        eng.set_flat(th0)
        rec(eng.update(UpdateParams(cg_iters=5)))
    eng.set_batch(d["X"][:n_small], d["actions"][:n_small], adv[:n_small], d["old_dist"][:n_small])
    for _ in range(3):                       # new key: rows
        eng.set_flat(th0)
        rec(eng.update(UpdateParams(cg_iters=10, residual_tol=0.0, max_kl=100.0)))
    eng.set_batch(d["X"], d["actions"], adv, d["old_dist"])
    eng.set_rewards(d["rewards"], d["starts"])
    for _ in range(3):                       # new key: advantages inside the graph
        eng.set_flat(th0)
        rec(eng.update(UpdateParams(compute_advantages=True, gamma=0.95)))
    return out


@pytest.mark.parametrize("name,hidden", [("update_c3.npz", None), ("update_c2.npz", None),
                                         ("update_c3.npz", [256, 160])])
def test_graph_replay_matches_eager(gpu_available, name, hidden):
    """The hipGraph-replayed update prefix (option `graphs`, default on) gives bit-identical
    results to the eager launches across capture, replay and every re-keying event; the
    [256, 160] policy runs the split-MFMA row GEMMs instead of the fused chain."""
    from trpo_amd._lib import get_option, set_option
    d = dict(golden(name))
    if hidden is not None:
        spec = O.PolicySpec(d["X"].shape[1], hidden, spec_of(d).n_actions)
        d.update(O.synthetic_batch(spec, d["X"].shape[0], seed=5))
    saved = get_option("graphs")
    runs = {}
    try:
        for mode in (0, 1):
            set_option("graphs", mode)
            eng, _ = make_engine(d) if hidden is None else _make_spec_engine(d, hidden)
            runs[mode] = _graph_sequence(eng, d, d["X"].shape[0] // 2 + 3)
            eng.close()
    finally:
        set_option("graphs", saved)
    assert len(runs[0]) == len(runs[1])
    for i, ((s0, t0), (s1, t1)) in enumerate(zip(runs[0], runs[1])):
        np.testing.assert_array_equal(t0, t1, err_msg=f"theta after update {i}")
        for k in ("cg_iters", "k", "reverted", "shs", "lm", "rate", "surr_after", "kl_after", "ent_after"):
            assert s0[k] == s1[k], (i, k, s0[k], s1[k])
    # the re-keyed updates really ran with their own parameters
    assert runs[1][5][0]["cg_iters"] <= 5 and runs[1][0][0]["cg_iters"] == 10
    assert not np.array_equal(runs[1][2][1], d["theta"])


def _make_spec_engine(d, hidden):
    from trpo_amd import Engine
    spec = O.PolicySpec(d["X"].shape[1], hidden, spec_of(d).n_actions)
    n = d["X"].shape[0]
    eng = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
    eng.set_flat(d["theta"])
    eng.set_batch(d["X"], d["actions"], np.asarray(d["advant"], np.float32), d["old_dist"])
    return eng, spec


@pytest.mark.parametrize("obs,hidden,A,n", [(128, [256, 256], 18, 3000), (376, [1024, 1024], 17, 1200)],
                         ids=["c4_dims", "c5_dims"])
def test_update_bench_dims_vs_oracle(gpu_available, obs, hidden, A, n):
    """The benchmark configurations' layer shapes (BASELINE.json configs[3] and configs[4]: split-f16 row
    GEMMs and weight gradients, 1024-wide tiles) at a row count the float64 oracle runs in seconds:
    undamped FVP, policy gradient, CG step direction (residual_tol = 0) and the updated parameters."""
    from trpo_amd import Engine, UpdateParams
    from trpo_amd._lib import VEC_G, VEC_STEPDIR
    spec = O.PolicySpec(obs, hidden, A)
    d = O.synthetic_batch(spec, n, seed=11)
    eng = Engine(obs, hidden, A, max_rows=n)
    eng.set_flat(d["theta"])
    eng.set_batch(d["X"], d["actions"], d["advant"].astype(np.float32), d["old_dist"])
    v = np.random.RandomState(12).standard_normal(spec.n_params).astype(np.float32)
    hv = eng.fvp(v, 0.0)
    ref = O.fvp_undamped(d["theta"].astype(np.float64), d["X"], v.astype(np.float64), spec)
    assert_vec_close(hv, ref, REL, "Hv")
    st = eng.update(UpdateParams(cg_iters=10, residual_tol=0.0))
    r = O.trpo_update(d["theta"].astype(np.float64), O.Batch(d["X"], d["actions"], d["advant"], d["old_dist"]),
                      spec, np.float64, 10, 0.0)
    assert_vec_close(eng.get_vector(VEC_G), r.g, REL, "g")
    assert st["cg_iters"] == 10 == r.cg_iters
    assert st["k"] == r.k
    assert_vec_close(eng.get_vector(VEC_STEPDIR), r.stepdir, REL, "stepdir")
    assert st["shs"] == pytest.approx(r.shs, rel=REL)
    assert_vec_close(eng.get_flat(), r.theta_new, REL, "theta_new")
    eng.close()


@pytest.mark.parametrize("obs,hidden,A,n", [(128, [256, 256], 18, 3001), (376, [1024, 1024], 17, 1200),
                                            (64, [512, 256], 18, 255)], ids=["c4_dims", "c5_dims", "k64_lt_tile"])
def test_planes_bit_identical_to_register_split(gpu_available, obs, hidden, A, n):
    """Layer 0's row GEMMs (forward and R-forward) on the pre-split k-blocked X planes and the LDS-DMA
    plane kernel (option planes, plane.hip) give bit-identical FVP, gradient and update to the
    register-staged split of the same f16 arithmetic (ragged row tiles, K = 64 .. 384)."""
    from trpo_amd import Engine, UpdateParams
    from trpo_amd._lib import get_option, set_option
    spec = O.PolicySpec(obs, hidden, A)
    d = O.synthetic_batch(spec, n, seed=13)
    v = np.random.RandomState(14).standard_normal(spec.n_params).astype(np.float32)
    saved = get_option("planes")
    saved_r0, saved_rf, saved_f = get_option("rbwd0"), get_option("rfwd01"), get_option("fwd01")
    set_option("rbwd0", 0)   # the fused layer-1 R-backward needs X's planes: compare the row GEMMs alone
    set_option("rfwd01", 0)  # so do the one-launch R-forward and forward of layers 0 and 1 (rfwd.hip)
    set_option("fwd01", 0)
    out = {}
    try:
        for mode in (0, 1):
            set_option("planes", mode)
            eng = Engine(obs, hidden, A, max_rows=n + 300)
            eng.set_flat(d["theta"])
            eng.set_batch(d["X"], d["actions"], d["advant"].astype(np.float32), d["old_dist"])
            hv, g = eng.fvp(v, 0.0), eng.policy_grad()
            st = eng.update(UpdateParams(cg_iters=10, residual_tol=0.0))
            out[mode] = (hv, g, eng.get_flat(), st)
            eng.close()
    finally:
        set_option("planes", saved)
        set_option("rbwd0", saved_r0)
        set_option("rfwd01", saved_rf)
        set_option("fwd01", saved_f)
    for i, what in enumerate(("Hv", "g", "theta")):
        np.testing.assert_array_equal(out[0][i], out[1][i], err_msg=what)
    for k in ("cg_iters", "k", "shs", "lm", "surr_after", "kl_after"):
        assert out[0][3][k] == out[1][3][k], k


@pytest.mark.parametrize("obs,hidden,A,n", [
    (128, [256, 256], 18, 3001),      # C4 dims (the bench workload's layer shapes), ragged last tile
    (37, [200, 192], 17, 777),         # hidden 192: three of the four waves' column blocks, 17 actions
    (9, [64, 160, 256], 32, 1500),     # depth 3, A = 32 (one full action tile)
    (128, [256], 20, 64),              # the reference's depth (one hidden layer), fewer rows than a split
])
def test_fused_tail_vs_oracle_and_per_layer(gpu_available, obs, hidden, A, n):
    """tail.hip (head R-forward + R-softmax + R-backward + last-layer weight R-gradient in one
    launch, E recomputed from D_L) against the float64 oracle and against the per-layer kernels it
    replaces (option tail = 0), for the FVP and a whole update (trpo_inksci.py:56-70,144-158)."""
    from trpo_amd import Engine, UpdateParams
    from trpo_amd._lib import get_option, set_option
    spec = O.PolicySpec(obs, hidden, A)
    dd = O.synthetic_batch(spec, n, seed=n + A)
    v = np.random.RandomState(n).standard_normal(spec.n_params).astype(np.float32)
    ref = O.fvp_undamped(dd["theta"].astype(np.float64), dd["X"], v.astype(np.float64), spec)
    r = O.trpo_update(dd["theta"].astype(np.float64), O.Batch(dd["X"], dd["actions"], dd["advant"], dd["old_dist"]),
                      spec, np.float64, 10, 0.0)
    saved = get_option("tail")
    out = {}
    try:
        for mode in (1, 0):
            set_option("tail", mode)
            e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
            e.set_flat(dd["theta"])
            e.set_batch(dd["X"], dd["actions"], dd["advant"].astype(np.float32), dd["old_dist"])
            hv = e.fvp(v, 0.0)
            st = e.update(UpdateParams(cg_iters=10, residual_tol=0.0))
            out[mode] = (hv, st, e.get_flat())
            e.close()
    finally:
        set_option("tail", saved)
    for mode in (1, 0):
        hv, st, th = out[mode]
        assert_vec_close(hv, ref, REL, f"Hv tail={mode} {obs} {hidden} {A}")
        assert st["k"] == r.k
        assert_vec_close(th, r.theta_new, REL, f"theta tail={mode} {obs} {hidden} {A}")
    assert_vec_close(out[1][0], out[0][0], REL, "fused tail vs per-layer Hv")


@pytest.mark.parametrize("obs,hidden,A,n", [
    (16, [64, 64], 64, 2000),          # f32 MFMA path, two 32-column softmax tiles per row
    (32, [256, 256], 100, 1500),       # f16-split path (the fused tail takes <= 32 actions: per-layer)
    (11, [64], 33, 777),               # one action past a single tile
])
def test_many_actions_vs_oracle(gpu_available, obs, hidden, A, n):
    """More than 32 actions (trpo_inksci.py:40's softmax_classifier(action_dim) has no bound):
    losses, policy gradient, Hv and a whole update against the float64 oracle."""
    from trpo_amd import Engine, UpdateParams
    spec = O.PolicySpec(obs, hidden, A)
    dd = O.synthetic_batch(spec, n, seed=A)
    th = dd["theta"].astype(np.float64)
    e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
    e.set_flat(dd["theta"])
    e.set_batch(dd["X"], dd["actions"], dd["advant"].astype(np.float32), dd["old_dist"])
    ref_l = O.losses(th, dd["X"], dd["actions"], dd["advant"], dd["old_dist"], spec)
    assert np.allclose(e.losses(), ref_l, rtol=1e-5, atol=1e-7)
    assert_vec_close(e.action_dist(), O.action_dist(th, dd["X"], spec), REL, "action_dist")
    assert_vec_close(e.policy_grad(), O.policy_grad(th, dd["X"], dd["actions"], dd["advant"], dd["old_dist"], spec),
                     REL, f"g A={A}")
    v = np.random.RandomState(A).standard_normal(spec.n_params).astype(np.float32)
    assert_vec_close(e.fvp(v, 0.0), O.fvp_undamped(th, dd["X"], v.astype(np.float64), spec), REL, f"Hv A={A}")
    st = e.update(UpdateParams(cg_iters=10, residual_tol=0.0))
    r = O.trpo_update(th, O.Batch(dd["X"], dd["actions"], dd["advant"], dd["old_dist"]), spec, np.float64, 10, 0.0)
    assert st["k"] == r.k
    assert_vec_close(e.get_flat(), r.theta_new, REL, f"theta A={A}")
    if A > 64:
        # the update takes up to 128 actions; acting (one wave per state) stops at 64 and says so
        with pytest.raises(RuntimeError, match="n_actions must be <= 64"):
            e.act(dd["X"][:4], train=False)
    e.close()


@pytest.mark.parametrize("scale", [6.0, 25.0], ids=["peaked", "saturated"])
@pytest.mark.parametrize("low_seg", [14, 0], ids=["low_seg", "three_products"])
def test_saturated_softmax_fvp_vs_oracle(gpu_available, scale, low_seg):
    """C4 layer shapes with the head's weights scaled up until the softmax is near-deterministic: many
    p_j fall to or below eps, the O(eps) KL_ff terms (D_l, E_l) become comparable to the R-terms, and
    the one-product low segment (option low_seg) must fall back to three products by its own binade
    test.  Undamped FVP and one update against the float64 oracle (trpo_inksci.py:56-70)."""
    from trpo_amd import Engine, UpdateParams
    from trpo_amd._lib import VEC_STEPDIR, get_option, set_option
    spec = O.PolicySpec(128, [256, 256], 18)
    n = 3000
    d = O.synthetic_batch(spec, n, seed=21)
    params = O.unflatten(d["theta"].astype(np.float64).copy(), spec)
    W, b = params[-1]
    W *= scale
    b *= scale
    theta = O.flatten(params).astype(np.float32)
    old = O.action_dist(theta.astype(np.float64), d["X"], spec, np.float64).astype(np.float32)
    assert (old < 1e-6).mean() > (0.2 if scale > 10 else 0.01)   # the regime this test is about
    # actions drawn from the policy, as a rollout would (a uniform draw would hit p_old[a] = 0 in f32,
    # where the reference's un-eps'd ratio p/p_old is inf and every result NaN: test_gpu_degenerate.py)
    u = np.random.RandomState(23).uniform(size=(n, 1))
    d["actions"] = np.minimum((np.cumsum(old.astype(np.float64), axis=1) < u).sum(axis=1), spec.n_actions - 1)
    assert old[np.arange(n), d["actions"]].min() > 0
    saved = get_option("low_seg")
    set_option("low_seg", low_seg)
    try:
        eng = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
        eng.set_flat(theta)
        eng.set_batch(d["X"], d["actions"], d["advant"].astype(np.float32), old)
        v = np.random.RandomState(22).standard_normal(spec.n_params).astype(np.float32)
        hv = eng.fvp(v, 0.0)
        ref = O.fvp_undamped(theta.astype(np.float64), d["X"], v.astype(np.float64), spec)
        assert_vec_close(hv, ref, REL, "Hv")
        # element-level parity per parameter block (each W_l and b_l against its own scale, so a small
        # block -- the biases, the head -- is not judged against the largest block's magnitude): the
        # one-product segment's 2^-11 relative error on its own terms must not surface in any block
        off = 0
        for l, (Wl, bl) in enumerate(O.unflatten(ref.copy(), spec)):
            for name, blk in (("W", Wl), ("b", bl)):
                sz = blk.size
                assert_vec_close(hv[off:off + sz], ref[off:off + sz], REL, f"Hv block {name}{l}")
                off += sz
        st = eng.update(UpdateParams(cg_iters=10, residual_tol=0.0))
        r = O.trpo_update(theta.astype(np.float64), O.Batch(d["X"], d["actions"], d["advant"], old),
                          spec, np.float64, 10, 0.0)
        assert st["k"] == r.k
        assert_vec_close(eng.get_vector(VEC_STEPDIR), r.stepdir, REL, "stepdir")
        eng.close()
    finally:
        set_option("low_seg", saved)


def test_path_switch_after_prepare_rewrites_e(gpu_available):
    """Under the fused tail the prepare pass skips E_{L-2} (tail.hip recomputes it); switching the same
    engine to the per-layer R-backward afterwards must re-prepare rather than read an E that was never
    written (engine.cpp fvp(), prep_e_top)."""
    from trpo_amd import Engine
    from trpo_amd._lib import get_option, set_option
    spec = O.PolicySpec(128, [256, 256], 18)
    n = 2000
    d = O.synthetic_batch(spec, n, seed=31)
    v = np.random.RandomState(32).standard_normal(spec.n_params).astype(np.float32)
    ref = O.fvp_undamped(d["theta"].astype(np.float64), d["X"], v.astype(np.float64), spec)
    saved = get_option("tail")
    try:
        set_option("tail", 1)
        e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
        e.set_flat(d["theta"])
        e.set_batch(d["X"], d["actions"], d["advant"].astype(np.float32), d["old_dist"])
        assert_vec_close(e.fvp(v, 0.0), ref, REL, "Hv, fused tail")
        set_option("tail", 0)
        assert_vec_close(e.fvp(v, 0.0), ref, REL, "Hv, per-layer after the switch")
        set_option("tail", 1)
        assert_vec_close(e.fvp(v, 0.0), ref, REL, "Hv, back on the tail")
        e.close()
    finally:
        set_option("tail", saved)


def test_fused16_switch_after_prepare(gpu_available):
    """prepare() on the fused16 path writes D_1 / E_1 / E_0 and the policy gradient's slabs from one launch
    (bwd_pg), not the per-layer path's outputs. Switching option fused on the same engine afterwards must
    re-prepare (engine.cpp reprepare_if_path_changed), in both directions, for fvp() and policy_grad()."""
    from trpo_amd import Engine
    from trpo_amd._lib import get_option, set_option
    spec = O.PolicySpec(128, [64, 64], 18)
    n = 3001
    d = O.synthetic_batch(spec, n, seed=41)
    v = np.random.RandomState(42).standard_normal(spec.n_params).astype(np.float32)
    th = d["theta"].astype(np.float64)
    ref = O.fvp_undamped(th, d["X"], v.astype(np.float64), spec)
    gref = O.policy_grad(th, d["X"], d["actions"], d["advant"], d["old_dist"], spec)
    saved = get_option("fused")
    try:
        set_option("fused", 3)
        e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
        e.set_flat(d["theta"])
        e.set_batch(d["X"], d["actions"], d["advant"].astype(np.float32), d["old_dist"])
        assert_vec_close(e.policy_grad(), gref, REL, "g, fused16")
        for mode in (2, 0, 3, 0):
            set_option("fused", mode)
            assert_vec_close(e.policy_grad(), gref, REL, f"g after switching to fused={mode}")
            assert_vec_close(e.fvp(v, 0.0), ref, REL, f"Hv after switching to fused={mode}")
            assert_vec_close(e.policy_grad(), gref, REL, f"g after an FVP on fused={mode}")
        e.close()
    finally:
        set_option("fused", saved)


def test_flatgrad_of_gvp_is_the_fvp(gpu_available):
    """The reference's spelling of the FVP node, ``self.fvp = flatgrad(gvp, var_list)`` with ``gvp`` the
    tangent-dotted gradient of KL_firstfixed (trpo_inksci.py:56-70), and its damped closure
    ``fisher_vector_product(p) = session.run(fvp) + 0.1 p`` (:124-126): through the utils surface against
    the fixture's undamped Hv, and as the operator the device CG consumes."""
    from trpo_amd.utils import FisherVectorProduct, KLFirstFixedGVP, conjugate_gradient, flatgrad
    d = golden("update_c3.npz")
    eng, spec = make_engine(d)
    fvp = flatgrad(KLFirstFixedGVP(eng))
    assert isinstance(fvp, FisherVectorProduct) and fvp.damping == 0.0
    v = d["v"].astype(np.float32)
    assert_vec_close(fvp(v), d["hv"], REL, "flatgrad(gvp)(v)")
    fisher_vector_product = fvp.damped(0.1)
    assert_vec_close(fisher_vector_product(v), d["hv"] + 0.1 * v, REL, "flatgrad(gvp)(v) + 0.1 v")
    stepdir = conjugate_gradient(fisher_vector_product, -d["g"].astype(np.float32), int(d["cg_iters"]),
                                 float(d["residual_tol"]))
    assert_vec_close(stepdir, d["stepdir"], REL, "CG over the flatgrad(gvp) operator")
    eng.close()


@pytest.mark.parametrize("obs,hidden,A,n", [
    (128, [256, 256], 18, 3001),       # C4 dims, ragged last tile of the last split
    (37, [192, 200], 17, 2500),        # obs 37 (X planes 64 wide), hidden 192 (two idle waves), K = 200
    (128, [256], 18, 1500),            # one hidden layer: the policy gradient's backward only (FVP in the tail)
    (64, [256, 256, 256], 20, 900),    # depth 3
    (128, [256, 160], 18, 1100),       # K = 160: 10 k-tiles per segment (the policy gradient's is not a multiple of 4)
    (100, [256, 200], 7, 700),         # K = 200: a partial last k-tile, 13 per segment
    (128, [256], 40, 800),             # one hidden layer, 40 actions (no tail): K = 40 for both backward paths
], ids=["c4_dims", "odd", "one_hidden", "depth3", "k160", "k200", "one_hidden_a40"])
def test_rbwd0_fused_vs_per_layer_and_oracle(gpu_available, obs, hidden, A, n):
    """rbwd0.hip: layer 1's R-backward with layer 0's weight R-gradient in one launch (RD_0 never stored),
    and the same for the policy gradient's DS_0 (trpo_inksci.py:54,56-70), against the per-layer kernels
    (option rbwd0 = 0) and the float64 oracle: Hv, g and a whole update."""
    from trpo_amd import Engine, UpdateParams
    from trpo_amd._lib import get_option, set_option
    spec = O.PolicySpec(obs, hidden, A)
    dd = O.synthetic_batch(spec, n, seed=n + obs)
    th = dd["theta"].astype(np.float64)
    v = np.random.RandomState(n).standard_normal(spec.n_params).astype(np.float32)
    ref = O.fvp_undamped(th, dd["X"], v.astype(np.float64), spec)
    gref = O.policy_grad(th, dd["X"], dd["actions"], dd["advant"], dd["old_dist"], spec)
    r = O.trpo_update(th, O.Batch(dd["X"], dd["actions"], dd["advant"], dd["old_dist"]), spec, np.float64, 10, 0.0)
    saved = get_option("rbwd0")
    out = {}
    try:
        for mode in (1, 0):
            set_option("rbwd0", mode)
            e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
            e.set_flat(dd["theta"])
            e.set_batch(dd["X"], dd["actions"], dd["advant"].astype(np.float32), dd["old_dist"])
            hv, g = e.fvp(v, 0.0), e.policy_grad()
            st = e.update(UpdateParams(cg_iters=10, residual_tol=0.0))
            out[mode] = (hv, g, st, e.get_flat())
            e.close()
    finally:
        set_option("rbwd0", saved)
    for mode in (1, 0):
        hv, g, st, theta = out[mode]
        assert_vec_close(hv, ref, REL, f"Hv rbwd0={mode}")
        assert_vec_close(g, gref, REL, f"g rbwd0={mode}")
        assert st["k"] == r.k
        assert_vec_close(theta, r.theta_new, REL, f"theta rbwd0={mode}")
    assert_vec_close(out[1][0], out[0][0], REL, "fused vs per-layer Hv")
    assert_vec_close(out[1][1], out[0][1], REL, "fused vs per-layer g")


@pytest.mark.parametrize("obs,hidden,A,n", [
    (128, [256, 256], 18, 3001),       # C4 dims, ragged last tile (D_1's hi plane per 32-row tile)
    (128, [256, 256], 18, 40037),      # several splits
    (37, [192, 200], 17, 2500),        # K = 200 for the fused R-backward, 17 actions
    (64, [256, 256, 256], 32, 900),    # depth 3: D_2 / DS_2 (no hi plane), A = 32
    (128, [256, 256], 18, -3001),      # C4 dims with tail = 0: the per-layer FVP reads E_1, written here as well
], ids=["c4_dims", "many_splits", "odd", "depth3", "c4_dims_e1"])
def test_head_bwd2_vs_rowgemm_and_oracle(gpu_available, obs, hidden, A, n):
    """hbwd.hip: the prepare pass's D_{L-2} and the policy gradient's DS_{L-2} in one read of H (and D_1's f16 hi
    plane scaled per 32-row tile, or E_{L-2} where the fused FVP reads it) against the two row-GEMM backwards
    (option hbwd2 = 0) and the float64 oracle, on f32 MFMA (hbwd2 = 2, the default) and on VALU fmaf chains
    (hbwd2 = 1): g, Hv and a whole update (trpo_inksci.py:54,56-70,144-158)."""
    from trpo_amd import Engine, UpdateParams
    from trpo_amd._lib import get_option, set_option
    no_tail = n < 0                       # negative n: the same rows with the fused tail off
    n = abs(n)
    spec = O.PolicySpec(obs, hidden, A)
    dd = O.synthetic_batch(spec, n, seed=n + 5)
    th = dd["theta"].astype(np.float64)
    v = np.random.RandomState(n + 2).standard_normal(spec.n_params).astype(np.float32)
    ref = O.fvp_undamped(th, dd["X"], v.astype(np.float64), spec)
    gref = O.policy_grad(th, dd["X"], dd["actions"], dd["advant"], dd["old_dist"], spec)
    r = O.trpo_update(th, O.Batch(dd["X"], dd["actions"], dd["advant"], dd["old_dist"]), spec, np.float64, 10, 0.0)
    saved = get_option("hbwd2")
    saved_tail = get_option("tail")
    if no_tail:
        set_option("tail", 0)
    out = {}
    try:
        for mode in (2, 1, 0):
            set_option("hbwd2", mode)
            e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
            e.set_flat(dd["theta"])
            e.set_batch(dd["X"], dd["actions"], dd["advant"].astype(np.float32), dd["old_dist"])
            g = e.policy_grad()
            hv = e.fvp(v, 0.0)
            g2 = e.policy_grad()          # after an FVP wrote RD: the policy gradient recomputes DS_{L-2}
            st = e.update(UpdateParams(cg_iters=10, residual_tol=0.0))
            out[mode] = (g, hv, g2, st, e.get_flat())
            e.close()
    finally:
        set_option("hbwd2", saved)
        set_option("tail", saved_tail)
    for mode in (2, 1, 0):
        g, hv, g2, st, theta = out[mode]
        assert_vec_close(g, gref, REL, f"g hbwd2={mode}")
        assert_vec_close(g2, gref, REL, f"g after fvp hbwd2={mode}")
        assert_vec_close(hv, ref, REL, f"Hv hbwd2={mode}")
        assert st["k"] == r.k
        assert_vec_close(theta, r.theta_new, REL, f"theta hbwd2={mode}")
    assert_vec_close(out[1][0], out[0][0], REL, "dual vs row-GEMM backward g")
    assert_vec_close(out[2][0], out[0][0], REL, "f32 MFMA dual vs row-GEMM backward g")


@pytest.mark.parametrize("opt,modes", [
    ("cg_fuse_reduce", (1, 2)),   # 2: x / r / p and the next V image in the slab reduction's launch (last workgroup)
    ("cg_p_img", (0, 1)),         # 1 (default): the p update and the next V images in one launch (p ping-pongs)
], ids=lambda v: str(v))
@pytest.mark.parametrize("obs,hidden,A,n", [
    (11, [64, 64], 3, 50_000),         # C2: the CG step builds the next FVP's V images
    (128, [64, 64], 18, 20_000),       # C3 dims: P = 13,586, 213 reduction blocks
    (4, [64], 2, 1000),                # C1 dims: one hidden layer
    (37, [50, 33], 7, 129),            # padded widths, one FVP workgroup
])
def test_cg_step_one_launch_bitwise(gpu_available, obs, hidden, A, n, opt, modes):
    """The fused CG-step launches are bit-identical to the separate ones: cg_fuse_reduce = 2 (the iteration's x / r / p
    updates and the next V image in the slab reduction's launch, run by the workgroup that arrives last) against 1,
    and cg_p_img = 1 (the p update with the next V images) against 0: the CG solution at residual_tol 0 and with
    early exits (utils.py:199-200), and whole updates, eager and replayed from the captured graph."""
    from trpo_amd import Engine, UpdateParams
    from trpo_amd._lib import get_option, set_option
    spec = O.PolicySpec(obs, hidden, A)
    dd = O.synthetic_batch(spec, n, seed=31)
    b = np.random.RandomState(32).standard_normal(spec.n_params).astype(np.float32)
    dflt = get_option(opt)
    runs = {}
    try:
        for mode in modes:
            set_option(opt, mode)
            e = Engine(obs, hidden, A, max_rows=n)
            e.set_flat(dd["theta"])
            e.set_batch(dd["X"], dd["actions"], dd["advant"].astype(np.float32), dd["old_dist"])
            x0, it0 = e.cg(b, cg_iters=10, residual_tol=0.0)
            out = {"x0": x0, "it0": it0}
            bb = float(np.dot(b.astype(np.float64), b))
            for f in (0.5, 1e-2, 1e-4):   # early exits after the p update (utils.py:199-200)
                out[f"x{f}"], out[f"it{f}"] = e.cg(b, cg_iters=10, residual_tol=bb * f)
            for u in range(3):   # eager, capture, replay
                e.set_flat(dd["theta"])
                st = e.update(UpdateParams(residual_tol=1e-3 if u == 2 else 0.0))
                out[f"theta{u}"] = e.get_flat()
                out[f"stepdir{u}"] = e.get_vector(3)
                out[f"iters{u}"] = st["cg_iters"]
            runs[mode] = out
            e.close()
    finally:
        set_option(opt, dflt)
    m0, m1 = modes
    for k, v in runs[m0].items():
        if isinstance(v, np.ndarray):
            assert np.array_equal(v, runs[m1][k]), (k, float(np.abs(v - runs[m1][k]).max()))
        else:
            assert v == runs[m1][k], (k, v, runs[m1][k])
    ref = O.fvp_undamped(dd["theta"].astype(np.float64), dd["X"], b.astype(np.float64), spec)
    assert np.all(np.isfinite(ref)) and runs[m1]["it0"] == 10
    assert min(runs[m1][f"it{f}"] for f in (0.5, 1e-2, 1e-4)) < 10   # an early exit was exercised


def _block_slices(spec):
    """(W_l, b_l) flat slices in the reference's order [W1, b1, W2, b2, ...] (trpo_inksci.py:49)."""
    w = [spec.obs_dim] + list(spec.hidden) + [spec.n_actions]
    out, o = [], 0
    for l in range(len(w) - 1):
        out.append((slice(o, o + w[l] * w[l + 1]), slice(o + w[l] * w[l + 1], o + w[l] * w[l + 1] + w[l + 1])))
        o += w[l] * w[l + 1] + w[l + 1]
    return out


@pytest.mark.parametrize("n,case", [
    (1, "plain"), (129, "plain"), (1000, "plain"), (40_000, "plain"),   # one state, partial tiles, many tiles
    (3001, "v0_big"), (3001, "v0_small"),        # RH1 W1 dominant / H1 V1 dominant in the shared exponent
    (3001, "tanh_sat"),                           # saturated first layer: 1 - H1^2 near 0
    (3001, "mixed"),       # a few states per 32 with RH1 2^15 larger than their neighbours' (W_0's last rows zero,
                           # those states' X large there only: X W_0 exact, H1 unsaturated)
    (3001, "illcond"),     # whole X rows 2^12 larger: X W_0 ill-conditioned for any float32 evaluation
])
def test_rfwd01_vs_two_launches_and_oracle(gpu_available, n, case):
    """The one-launch R-forward of layers 0 / 1 (rfwd.hip) at C4 widths: Hv against the float64 oracle and against
    the two-launch path (rfwd01 = 0) at 1e-5, in the regimes its per-tile product exponent has to cover."""
    from trpo_amd import Engine
    from trpo_amd._lib import get_option, set_option
    spec = O.PolicySpec(128, [256, 256], 18)
    dd = O.synthetic_batch(spec, n, seed=41)
    th = dd["theta"].astype(np.float32).copy()
    X = dd["X"].astype(np.float32).copy()
    v = np.random.RandomState(42).standard_normal(spec.n_params).astype(np.float32)
    (w0, b0), (w1, b1), _ = _block_slices(spec)
    if case == "v0_big":
        v[w0] *= 100.0
        v[b0] *= 100.0
    elif case == "v0_small":
        v[w0] *= 1e-3
        v[b0] *= 1e-3
    elif case == "tanh_sat":
        th[w0] *= 20.0
    elif case == "mixed":
        th64 = th.astype(np.float64)
        W0 = th64[w0].reshape(spec.obs_dim, spec.hidden[0])
        W0[-3:, :] = 0.0
        th[w0] = W0.reshape(-1).astype(np.float32)
        rs = np.random.RandomState(43)
        for i in range(5, n, 29):
            X[i, -3:] = (2.0 ** 15 * rs.standard_normal(3)).astype(np.float32)
    elif case == "illcond":
        X[::97] *= 4096.0
    # (Hv does not read pi_old or the actions: KL_ff compares p with itself at the same theta, trpo_inksci.py:56-58)
    dflt = get_option("rfwd01")
    hv = {}
    try:
        for mode in (1, 0):
            set_option("rfwd01", mode)
            e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
            e.set_flat(th)
            e.set_batch(X, dd["actions"], dd["advant"].astype(np.float32), dd["old_dist"])
            hv[mode] = e.fvp(v, 0.0)
            e.close()
    finally:
        set_option("rfwd01", dflt)
    ref = O.fvp_undamped(th.astype(np.float64), X.astype(np.float64), v.astype(np.float64), spec)
    # 1e-5 wherever float32 arithmetic can meet it: max(1e-5, 4 x the float32 graph's own error) per block
    # (test_gpu_fused16_hard.py); only "illcond" needs the 4x
    ref32 = O.fvp_undamped(th, X, v, spec, dtype=np.float32)
    for sl in [s_ for blk in _block_slices(spec) for s_ in blk]:
        bar = max(REL, 4.0 * rel_l2(ref32[sl], ref[sl]))
        assert rel_l2(hv[1][sl], ref[sl]) <= bar, (case, rel_l2(hv[1][sl], ref[sl]), rel_l2(hv[0][sl], ref[sl]), bar)
    if case != "illcond":
        assert_vec_close(hv[1], hv[0], REL, f"rfwd01 {case} vs two launches")


@pytest.mark.parametrize("n,case", [
    (1, "plain"), (129, "plain"), (3001, "plain"), (40_000, "plain"),
    (3001, "tanh_sat"), (3001, "mixed"), (3001, "illcond"),   # as in test_rfwd01_vs_two_launches_and_oracle
])
def test_fwd01_vs_per_layer_and_oracle(gpu_available, n, case):
    """The prepare / line-search forward of layers 0 / 1 in one launch (rfwd.hip fwd01_kernel) at C4 widths: the
    policy gradient and Hv (both read the prepare pass's H1 / H2) against the float64 oracle, per block at
    max(1e-5, 4 x the float32 graph's error), and with one update (its line search reads the trial forward)
    against the per-layer forwards (fwd01 = 0): g, Hv, the step and the losses at 1e-5, k and the CG count exact."""
    from trpo_amd import Engine, UpdateParams
    from trpo_amd._lib import get_option, set_option
    spec = O.PolicySpec(128, [256, 256], 18)
    dd = O.synthetic_batch(spec, n, seed=51)
    th = dd["theta"].astype(np.float32).copy()
    X = dd["X"].astype(np.float32).copy()
    v = np.random.RandomState(52).standard_normal(spec.n_params).astype(np.float32)
    (w0, b0), _, _ = _block_slices(spec)
    if case == "tanh_sat":
        th[w0] *= 20.0
    elif case == "mixed":   # rfwd01's case: W_0's last rows zero, so X W_0 stays exact for the large states
        th64 = th.astype(np.float64)
        W0 = th64[w0].reshape(spec.obs_dim, spec.hidden[0])
        W0[-3:, :] = 0.0
        th[w0] = W0.reshape(-1).astype(np.float32)
        rs = np.random.RandomState(53)
        for i in range(5, n, 29):
            X[i, -3:] = (2.0 ** 15 * rs.standard_normal(3)).astype(np.float32)
    elif case == "illcond":
        X[::97] *= 4096.0
    adv = dd["advant"].astype(np.float32)
    dflt = get_option("fwd01")
    out = {}
    try:
        for mode in (1, 0):
            set_option("fwd01", mode)
            e = Engine(spec.obs_dim, spec.hidden, spec.n_actions, max_rows=n)
            e.set_flat(th)
            e.set_batch(X, dd["actions"], adv, dd["old_dist"])
            g, hv = e.policy_grad(), e.fvp(v, 0.0)
            st = e.update(UpdateParams(cg_iters=10, residual_tol=0.0))
            out[mode] = (g, hv, e.get_flat(), st)
            e.close()
    finally:
        set_option("fwd01", dflt)
    th64, X64 = th.astype(np.float64), X.astype(np.float64)
    gref = O.policy_grad(th64, X64, dd["actions"], dd["advant"], dd["old_dist"], spec)
    g32 = O.policy_grad(th, X, dd["actions"], dd["advant"], dd["old_dist"], spec, dtype=np.float32)
    href = O.fvp_undamped(th64, X64, v.astype(np.float64), spec)
    h32 = O.fvp_undamped(th, X, v, spec, dtype=np.float32)
    for sl in [s_ for blk in _block_slices(spec) for s_ in blk]:
        gb = max(REL, 4.0 * rel_l2(g32[sl], gref[sl]))
        hb = max(REL, 4.0 * rel_l2(h32[sl], href[sl]))
        assert rel_l2(out[1][0][sl], gref[sl]) <= gb, (case, "g", rel_l2(out[1][0][sl], gref[sl]), gb)
        assert rel_l2(out[1][1][sl], href[sl]) <= hb, (case, "Hv", rel_l2(out[1][1][sl], href[sl]), hb)
    if case != "illcond":
        assert_vec_close(out[1][0], out[0][0], REL, f"fwd01 {case} g vs per-layer")
        assert_vec_close(out[1][1], out[0][1], REL, f"fwd01 {case} Hv vs per-layer")
        assert_vec_close(out[1][2], out[0][2], REL, f"fwd01 {case} theta vs per-layer")
        for k in ("k", "cg_iters"):
            assert out[1][3][k] == out[0][3][k], (case, k)
        for k in ("surr_after", "kl_after"):   # (kl of the accepted step: max_kl 0.01 is its scale)
            a1, a0 = float(out[1][3][k]), float(out[0][3][k])
            assert abs(a1 - a0) <= REL * max(abs(a0), 1e-2), (case, k, a1, a0)
