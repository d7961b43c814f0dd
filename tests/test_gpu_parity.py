"""GPU parity: every HIP entry point, called through the C ABI (libvcmpc.so),
against the CPU oracle and the committed golden vectors.

Tolerances (written here, per the north star): u* to ||u* - u*_ref||_inf < 1e-5
(the BASELINE.json contract); model steps / rollout / Jacobians / condensed QP
data are fp64 restatements of the same formulas, checked to 1e-12 relative.
"""
import numpy as np
import pytest

from oracle import ltv_qp as Q
from oracle import models as M

pytestmark = pytest.mark.gpu

U_TOL = 1e-5
N, L = 20, 2.5


@pytest.fixture(scope="module")
def ctx(kin_cfg):
    from vcmpc import Context, _abi
    from vcmpc.config import load_config
    c = Context(model=_abi.VC_MODEL_KINEMATIC, N=N, max_batch=8192, kin_car=load_config("kinematic_car"),
                kin_mpc=kin_cfg)
    yield c
    c.close()


@pytest.fixture(scope="module")
def dyn_ctx():
    from vcmpc import Context, _abi
    from vcmpc.config import load_config
    c = Context(model=_abi.VC_MODEL_DYNAMIC, N=40, max_batch=4096, dyn_car=load_config("dynamic_car"))
    yield c
    c.close()


def test_dyn_plant_step_vs_reference_traces(dyn_ctx, dyn_kat):
    d = dyn_kat
    x = np.ascontiguousarray(d["x"]); u = np.ascontiguousarray(d["u"]); k = np.ascontiguousarray(d["kappa"])
    xn = dyn_ctx.plant_step(x, u, k, float(d["dt"]))
    rel = np.abs(xn - d["x_next"]) / np.maximum(np.abs(d["x_next"]), 1e-9)
    assert rel.max() < 1e-11


def test_dyn_spatial_step_vs_oracle(dyn_ctx, dyn_kat, dyn_params):
    d = dyn_kat
    ds = np.full(len(d["x"]), 0.7)
    xn = dyn_ctx.spatial_step(np.ascontiguousarray(d["x"]), np.ascontiguousarray(d["u"]),
                              np.ascontiguousarray(d["kappa"]), ds)
    ref = M.dyn_spatial_transition(d["x"], d["u"], d["kappa"], ds, dyn_params)
    np.testing.assert_allclose(xn, ref, rtol=1e-11, atol=1e-11)


def test_kin_plant_and_spatial_step(ctx):
    rng = np.random.default_rng(0)
    B = 1000
    x = np.column_stack([rng.uniform(2, 10, B), rng.uniform(-.3, .3, B), rng.uniform(0, 300, B),
                         rng.uniform(-2, 2, B), rng.uniform(-.3, .3, B), rng.uniform(0, 5, B)])
    u = np.column_stack([rng.uniform(-3, 3, B), rng.uniform(-.4, .4, B)])
    k = rng.uniform(0, .05, B); ds = rng.uniform(.3, .9, B)
    np.testing.assert_allclose(ctx.plant_step(x, u, k, 0.05), M.kin_transition(x, u, k, 0.05, L), rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(ctx.spatial_step(x, u, k, ds), M.kin_spatial_transition(x, u, k, ds, L),
                               rtol=1e-13, atol=1e-13)


def test_model_vector_field_f(ctx, dyn_ctx, dyn_kat, dyn_params):
    """vc_ode / VehicleModel.f(x, u, curvature): the continuous vector field the reference's
    integrators wrap (utils/integrators.py:18,29) -- temporal and spatial, kinematic and dynamic
    -- against the oracle's ODEs (same fp64 formulas: 1e-13 relative), and the Euler identity
    spatial_transition = x + ds f_spatial."""
    rng = np.random.default_rng(1)
    B = 500
    x = np.column_stack([rng.uniform(2, 10, B), rng.uniform(-.3, .3, B), rng.uniform(0, 300, B),
                         rng.uniform(-2, 2, B), rng.uniform(-.3, .3, B), rng.uniform(0, 5, B)])
    u = np.column_stack([rng.uniform(-3, 3, B), rng.uniform(-.4, .4, B)])
    k = rng.uniform(0, .05, B)
    np.testing.assert_allclose(ctx.ode(x, u, k), M.kin_temporal_ode(x, u, k, L), rtol=1e-13, atol=1e-13)
    fs = ctx.ode(x, u, k, space=True)
    np.testing.assert_allclose(fs, M.kin_spatial_ode(x, u, k, L), rtol=1e-13, atol=1e-13)
    ds = rng.uniform(.3, .9, B)
    np.testing.assert_allclose(ctx.spatial_step(x, u, k, ds), x + ds[:, None] * fs, rtol=1e-14, atol=1e-14)
    d = dyn_kat
    xd, ud, kd = (np.ascontiguousarray(d[key]) for key in ("x", "u", "kappa"))
    np.testing.assert_allclose(dyn_ctx.ode(xd, ud, kd), M.dyn_temporal_ode(xd, ud, kd, dyn_params),
                               rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(dyn_ctx.ode(xd, ud, kd, space=True), M.dyn_spatial_ode(xd, ud, kd, dyn_params),
                               rtol=1e-12, atol=1e-9)


def test_drop_in_f_alias():
    """KinematicCar.f(x, u, curvature) (the north star's VehicleModel.f) is the temporal ODE:
    transition(x, u, k, dt) = x + dt f(x, u, k) for the Euler kinematic car (kinematic_car.py:34-45)."""
    from vcmpc.config import load_config
    from vcmpc.models import KinematicCar

    class _T:
        def k(self, s):
            return 0.02

    car = KinematicCar(load_config("kinematic_car"), _T())
    x = np.array([6.0, 0.1, 10.0, 0.5, 0.05, 1.0]); u = np.array([1.0, -0.2])
    f = car.f(x, u, 0.02)
    np.testing.assert_allclose(f, M.kin_temporal_ode(x[None], u[None], np.array([0.02]), L)[0], rtol=1e-13)
    np.testing.assert_allclose(car.transition(x, u, 0.02, 0.05), x + 0.05 * f, rtol=1e-14)
    np.testing.assert_allclose(car.f_spatial(x, u, 0.02), M.kin_spatial_ode(x[None], u[None], np.array([0.02]), L)[0],
                               rtol=1e-13)


def test_rollout_and_linearize_vs_golden(ctx, kin_golden):
    g = kin_golden
    xbar = ctx.rollout(g["x0"], g["ubar"], g["kappa"], g["ds"])
    np.testing.assert_allclose(xbar, g["xbar"], rtol=1e-12, atol=1e-12)
    A, Bm = ctx.linearize(np.ascontiguousarray(g["xbar"][:16]), np.ascontiguousarray(g["ubar"][:16]),
                          np.ascontiguousarray(g["kappa"][:16]), np.ascontiguousarray(g["ds"][:16]))
    np.testing.assert_allclose(A, g["A"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(Bm, g["Bm"], rtol=1e-12, atol=1e-12)


def test_condense_vs_golden(ctx, kin_golden):
    g = kin_golden
    sl = slice(0, 16)
    H, gv = ctx.condense(*(np.ascontiguousarray(g[k][sl]) for k in ("x0", "ubar", "kappa", "ds")))
    np.testing.assert_allclose(H, g["H"], rtol=1e-10, atol=1e-10 * np.abs(g["H"]).max())
    np.testing.assert_allclose(gv, g["g"], rtol=1e-10, atol=1e-10 * np.abs(g["g"]).max())


def _solve(ctx, d):
    ub = d["ubar"].copy()
    u0, xbar, ustar, status, iters = ctx.solve(d["x0"], d["kappa"], d["ds"], ub)
    return u0, xbar, ustar, status, iters


def test_solve_vs_golden(ctx, kin_golden):
    g = kin_golden
    u0, xbar, ustar, status, iters = _solve(ctx, g)
    assert (status == 0).all(), (status, iters)
    err = np.abs(ustar - g["u_star"]).max()
    assert err < U_TOL, err
    np.testing.assert_allclose(u0, g["u0"], atol=U_TOL)
    np.testing.assert_allclose(xbar, g["x_star"], atol=1e-4)


@pytest.mark.parametrize("seed", [1, 2])
def test_solve_vs_oracle_fresh(ctx, kin_W, seed):
    from vcmpc.workload import kinematic_batch
    d = kinematic_batch(96, seed=seed)
    ref = Q.kin_ltv_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], L, kin_W)
    assert ref["polished"].all()
    u0, xbar, ustar, status, iters = _solve(ctx, d)
    assert (status == 0).mean() == 1.0, np.unique(status, return_counts=True)
    assert np.abs(ustar - ref["u_star"]).max() < U_TOL


def test_solve_full_batch_properties(ctx, kin_W):
    """At the C4 per-GPU shard size: every problem solved, u* inside the input
    boxes, x* consistent with the linearised rollout, deterministic reruns, and a
    sampled subset against the oracle."""
    from vcmpc.workload import kinematic_batch
    d = kinematic_batch(8192, seed=11)
    u0, xbar, ustar, status, iters = _solve(ctx, d)
    assert (status == 0).all()
    W = kin_W
    assert ustar[..., 0].min() >= W["a_min"] - 1e-9 and ustar[..., 0].max() <= W["a_max"] + 1e-9
    assert ustar[..., 1].min() >= W["w_min"] - 1e-9 and ustar[..., 1].max() <= W["w_max"] + 1e-9
    # delta rows bind stages 1..N-1 (kinematic_mpc.py:80-85 run over n < N; x_N is free)
    assert xbar[:, 1:N, 1].max() <= W["delta_max"] + 1e-8 and xbar[:, 1:N, 1].min() >= W["delta_min"] - 1e-8
    u0b, _, ustarb, _, _ = _solve(ctx, d)
    np.testing.assert_array_equal(ustar, ustarb)
    idx = np.arange(0, 8192, 257)
    ref = Q.kin_ltv_solve(d["x0"][idx], d["ubar"][idx], d["kappa"][idx], d["ds"][idx], L, W)
    assert np.abs(ustar[idx] - ref["u_star"]).max() < U_TOL


def test_c4_early_polish_regressions(ctx, kin_W):
    """C4 problems (kinematic_batch(65536, seed=31)) where the polish's first attempt at 100 x the
    interior point's tolerance once certified a point 9e-3 off the optimum (23921: an active state
    row with every variable fixed went unchecked), plus the C4 problems that sat furthest from the
    oracle in the r04 comparison (profiles/r04/kinab_c4diff.txt)."""
    from vcmpc.workload import kinematic_batch
    d = kinematic_batch(65536, seed=31)
    idx = np.array([23921, 7832, 39971, 13063])
    sub = {k: np.ascontiguousarray(v[idx]) for k, v in d.items()}
    ref = Q.kin_ltv_solve(sub["x0"], sub["ubar"], sub["kappa"], sub["ds"], L, kin_W)
    assert ref["polished"].all()
    u0, xbar, ustar, status, iters = _solve(ctx, sub)
    assert (status == 0).all()
    assert np.abs(ustar - ref["u_star"]).max() < U_TOL


def test_edge_batches(ctx, kin_golden):
    g = kin_golden
    e = {k: np.ascontiguousarray(g[k][:0]) for k in ("x0", "kappa", "ds", "ubar")}
    u0, xbar, ustar, status, iters = _solve(ctx, e)
    assert u0.shape == (0, 2)
    one = {k: np.ascontiguousarray(g[k][-3:-2]) for k in ("x0", "kappa", "ds", "ubar")}
    u0, xbar, ustar, status, iters = _solve(ctx, one)
    assert np.abs(ustar - g["u_star"][-3:-2]).max() < U_TOL


def test_nonfinite_problem_flagged(ctx, kin_golden):
    """v = 0 makes the spatial ODE singular (q = rho / (v cos epsi)); the problem is
    flagged VC_NONFINITE instead of raising (the reference's simulator swallows the
    IPOPT exception instead, racing.py:416-423) and the rest of the batch solves."""
    g = kin_golden
    d = {k: np.ascontiguousarray(g[k][:4]).copy() for k in ("x0", "kappa", "ds", "ubar")}
    d["x0"][1, 0] = 0.0
    u0, xbar, ustar, status, iters = _solve(ctx, d)
    assert status[1] == 2 and (status[[0, 2, 3]] == 0).all()
    assert np.abs(ustar[[0, 2, 3]] - g["u_star"][[0, 2, 3]]).max() < U_TOL


def test_api_errors(ctx, kin_golden):
    from vcmpc import _abi
    g = kin_golden
    with pytest.raises(ValueError):
        ctx.solve(g["x0"][:2].astype(np.float32), g["kappa"][:2], g["ds"][:2], g["ubar"][:2].copy())
    with pytest.raises(ValueError):
        big = {k: np.zeros((9000,) + g[k].shape[1:]) for k in ("x0", "kappa", "ds", "ubar")}
        ctx.solve(big["x0"], big["kappa"], big["ds"], big["ubar"])
    lib = ctx.lib
    rc = lib.vc_solve(ctx._h, -1, None, None, None, None, None, None, None, None, 0)
    assert rc == _abi.VC_E_ARG and b"batch" in lib.vc_last_error(ctx._h)


def test_device_pointer_path(ctx, kin_golden):
    import torch
    g = kin_golden
    dev = torch.device("cuda:0")
    t = {k: torch.from_numpy(np.ascontiguousarray(g[k])).to(dev) for k in ("x0", "kappa", "ds", "ubar")}
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        u0, xbar, ustar, status, iters = ctx.solve(t["x0"], t["kappa"], t["ds"], t["ubar"])
        torch.cuda.synchronize()
    finally:
        ctx.set_stream(None)
    assert (status.cpu().numpy() == 0).all()
    assert np.abs(ustar.cpu().numpy() - g["u_star"]).max() < U_TOL


def test_solve_from_matches_in_place_solve(ctx, kin_golden):
    """vc_solve_from (ABI 13): warm start read from ubar_in, left unchanged, u* into u_out --
    bit-identical to vc_solve's in-place answer, on device pointers (the kinematic kernel reads
    and writes through the two pointers) and host pointers, and on a dynamic context (which copies
    ubar_in to u_out and solves in place)."""
    import torch
    from vcmpc.workload import dynamic_batch, kinematic_batch
    dev = torch.device("cuda:0")
    d = kinematic_batch(512, N=N, seed=41)
    ref = ctx.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())
    # host pointers
    ub_in = d["ubar"].copy()
    u_out = np.empty_like(ub_in)
    got = ctx.solve_from(d["x0"], d["kappa"], d["ds"], ub_in, u_out)
    assert np.array_equal(ub_in, d["ubar"])
    for a, b in zip(ref, got):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    # device pointers
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items()}
    tu = torch.empty_like(t["ubar"])
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        u0, xbar, uo, st, it = ctx.solve_from(t["x0"], t["kappa"], t["ds"], t["ubar"], tu)
        torch.cuda.synchronize()
    finally:
        ctx.set_stream(None)
    assert np.array_equal(t["ubar"].cpu().numpy(), d["ubar"])
    assert np.array_equal(uo.cpu().numpy(), ref[2])
    assert np.array_equal(st.cpu().numpy(), ref[3]) and np.array_equal(xbar.cpu().numpy(), ref[1])
    # an SQP context (single-track, the C3 shape)
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    params = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=load_config("dynamic_mpc"), tyre="linear")
    dd = {k: v.astype(np.float64) for k, v in dynamic_batch(64, N=40, seed=3).items()}
    with Context(model=_abi.VC_MODEL_DYNAMIC, N=40, max_batch=64, dtype=_abi.VC_F64, params=params) as dc:
        dref = dc.solve(dd["x0"], dd["kappa"], dd["ds"], dd["ubar"].copy())
        dub = dd["ubar"].copy()
        dgot = dc.solve_from(dd["x0"], dd["kappa"], dd["ds"], dub, np.empty_like(dub))
    assert np.array_equal(dub, dd["ubar"])
    assert np.array_equal(dgot[2], dref[2]) and np.array_equal(dgot[3], dref[3])


def test_controller_drop_in_closed_loop(kin_cfg):
    """KinematicMPC(car, config).command(state) -> action, then car.drive: the
    reference's simulator step (kinracing.py:283-290) on a constant-curvature track."""
    from vcmpc.config import load_config
    from vcmpc.controllers import KinematicMPC
    from vcmpc.environment import CurvatureTrack
    from vcmpc.models import KinematicCar
    np.random.seed(31)
    car = KinematicCar(load_config("kinematic_car"), CurvatureTrack(constant=1 / 25))
    car.state = car.create_state(v=5.0, s=1.0)
    mpc = KinematicMPC(car, kin_cfg)
    solved = 0
    for _ in range(100):
        a = mpc.command(car.state)
        solved += int(mpc.status[0] == 0)
        assert -3 - 1e-9 <= a.a <= 3 + 1e-9 and -0.4 - 1e-9 <= a.w <= 0.4 + 1e-9
        car.drive(a)
    assert mpc.state_prediction.shape == (6, N + 1) and mpc.action_prediction.shape == (2, N)
    assert solved == 100, solved
    assert np.isfinite(car.state.values).all() and abs(car.state.ey) < 3.0 and car.state.v > 5.0


def test_solve_trust_region_vs_oracle(kin_cfg):
    """The trust-region tightening of the input boxes (vc_qp.trust_a/w, used by the
    closed-loop controller) against the oracle's identical contract."""
    from vcmpc import Context
    from vcmpc.config import load_config
    from vcmpc.workload import kinematic_batch
    cfg = dict(kin_cfg)
    cfg["qp"] = dict(kin_cfg["qp"], trust_a=0.8, trust_w=0.05)
    W = Q.kin_weights(cfg)
    d = kinematic_batch(64, seed=9)
    ref = Q.kin_ltv_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], L, W)
    assert ref["polished"].all()
    with Context(N=N, max_batch=64, kin_car=load_config("kinematic_car"), kin_mpc=cfg) as c:
        u0, xbar, ustar, status, iters = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())
    assert (status == 0).all()
    assert np.abs(ustar - ref["u_star"]).max() < U_TOL
    assert np.abs(ustar - d["ubar"])[..., 1].max() <= 0.05 + 1e-9
