"""GPU parity of the kinematic globalised SQP step (vc_qp.kin_sqp > 0: QP step through
kin_ltv.hip / kin_ric.hip, then the merit line search of csrc/kin_merit.hip) through the C ABI,
against the oracle (oracle/kin_sqp.py) on the obstacle golden problems
(tests/golden/obs_golden.npz), whose predictions pass close to or through ippodromo's obstacles.

Tolerance: the north star's 1e-5 on u* (m/s^2, rad/s); the line search is a discrete choice,
so the accepted step sizes must agree exactly.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import kin_sqp as KS
from oracle import ltv_qp as Q

pytestmark = pytest.mark.gpu

U_TOL = 1e-5


@pytest.fixture(scope="module")
def golden():
    return dict(np.load(os.path.join(GOLDEN, "obs_golden.npz")))


def _obs(g):
    return [tuple(float(v) for v in o) for o in g["obstacles"]]


def _cfg(kin_sqp, solver=0, N=20):
    from vcmpc.config import load_config
    cfg = load_config("kinematic_mpc")
    cfg["horizon"] = N
    cfg["qp"] = dict(cfg["qp"], kin_sqp=kin_sqp, solver=solver)
    return cfg


def _ctx(cfg, obstacles, B, N=20):
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=cfg, obstacles=obstacles)
    return Context(model=_abi.VC_MODEL_KINEMATIC, N=N, max_batch=B, dtype=_abi.VC_F64, params=p)


@pytest.mark.parametrize("solver", [0, 1], ids=["kin_ltv", "kin_ric"])
def test_kin_sqp_obstacles_vs_oracle(golden, solver):
    g = golden
    obs = _obs(g)
    S = 3
    cfg = _cfg(S, solver)
    W = Q.kin_weights(cfg)
    W["obstacles"] = obs
    x0, ub, kap, ds = (g[k].astype(np.float64) for k in ("kin_x0", "kin_ubar", "kin_kappa", "kin_ds"))
    ref = KS.kin_sqp_solve(x0, ub, kap, ds, 2.5, W, S)
    with _ctx(cfg, obs, len(x0)) as c:
        u0, xs, us, st, it = c.solve(x0, kap, ds, ub.copy())
        xr = c.rollout(x0, us, kap, ds)    # the device's own rollout of u* (vc_rollout)
    err = np.abs(us - ref["u_star"]).max(axis=(1, 2))
    alphas = np.array([h["alpha"] for h in ref["hist"]])
    print(f"solver {solver}: |u* - u*_oracle| max {err.max():.2e}; oracle step sizes per iteration "
          f"{[np.unique(a).tolist() for a in alphas]}; status {np.bincount(st)}")
    assert (st == 0).all(), st
    assert err.max() < U_TOL, np.argsort(err)[-5:]
    np.testing.assert_array_equal(u0, us[:, 0])
    # x* = rollout(u*): against the device rollout kernel to 1e-12 (same model code), and against
    # the host rollout to 1e-8 (numpy's cos / tan vs the device's differ by ulps, amplified over 20
    # stages of trajectories that swerve round obstacles: 8.9e-10 .. 1.2e-9 measured on epsi_N)
    assert np.abs(xs - xr).max() <= 1e-12 * (1.0 + np.abs(xr).max())
    x_own = Q.kin_predict(x0, us, kap, ds, 2.5)     # x* = rollout(u*) of the kernel's own u*
    dx = np.abs(xs - x_own)
    print("x* vs rollout(u*): max %.2e at %s" % (dx.max(), np.unravel_index(dx.argmax(), dx.shape)))
    assert dx.max() < 1e-8
    # the merit of the final iterate never exceeds the start's
    phi_start = KS.merit(x0, ub, kap, ds, 2.5, W)
    phi_end = KS.merit(x0, us, kap, ds, 2.5, W)
    assert (phi_end <= phi_start + 1e-9 * np.abs(phi_start)).all()


def test_kin_sqp_without_obstacles_is_descent(golden):
    """kin_sqp = 2 on the plain C2 sampler: every accepted iterate lowers the merit, and the
    first SQP iteration's full QP step is taken where the merit allows it (oracle agrees)."""
    from vcmpc.workload import kinematic_batch
    d = kinematic_batch(64, seed=5)
    cfg = _cfg(2)
    W = Q.kin_weights(cfg)
    ref = KS.kin_sqp_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], 2.5, W, 2)
    with _ctx(cfg, [], 64) as c:
        u0, xs, us, st, it = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())
    assert (st == 0).all()
    assert np.abs(us - ref["u_star"]).max() < U_TOL
    phi0 = KS.merit(d["x0"], d["ubar"], d["kappa"], d["ds"], 2.5, W)
    assert (KS.merit(d["x0"], us, d["kappa"], d["ds"], 2.5, W) <= phi0 + 1e-9 * np.abs(phi0)).all()


def test_kin_sqp_zero_is_the_ltv_contract(golden):
    """kin_sqp = 0 keeps the one-step LTV-QP contract bit for bit (the C2 hot path)."""
    from vcmpc.workload import kinematic_batch
    d = kinematic_batch(32, seed=6)
    with _ctx(_cfg(0), [], 32) as c:
        r0 = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())
    W = Q.kin_weights(_cfg(0))
    ref = Q.kin_ltv_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], 2.5, W)
    assert np.abs(r0[2] - ref["u_star"]).max() < U_TOL


def test_kin_sqp_multiple_shooting_vs_oracle(golden):
    """vc_qp.ms = 1 with kin_sqp = 3 on the obstacle golden problems, the state iterate a plan
    that clears the obstacles (the rollout of the mean of ubar and a converged SQP solution;
    nonzero defects): 15 of 44 problems start in the multiple-shooting merit, the rest in the
    rollout's (oracle/kin_sqp.py line_search_ms).  u* matches the oracle to 1e-5, x* (the state
    iterate, or the rollout where that was reset) to 1e-6, and the merit never increases."""
    g = golden
    obs = _obs(g)
    S = 3
    cfg = _cfg(S, 1)
    cfg["qp"]["ms"] = 1
    W = Q.kin_weights(cfg)
    W["obstacles"] = obs
    x0, ub, kap, ds = (g[k].astype(np.float64) for k in ("kin_x0", "kin_ubar", "kin_kappa", "kin_ds"))
    good = KS.kin_sqp_solve(x0, ub, kap, ds, 2.5, W, 6)["u_star"]
    xw = Q.kin_predict(x0, 0.5 * (ub + good), kap, ds, 2.5)
    ps0 = KS.merit(x0, ub, kap, ds, 2.5, W)
    pm0 = KS.merit(x0, ub, kap, ds, 2.5, W, x=xw)
    assert (pm0 < ps0).sum() >= 10
    ref = KS.kin_sqp_solve(x0, ub, kap, ds, 2.5, W, S, x_ws=xw)
    with _ctx(cfg, obs, len(x0)) as c:
        u0, xs, us, st, it = c.solve(x0, kap, ds, ub.copy(), xbar=xw.copy())
    err = np.abs(us - ref["u_star"]).max(axis=(1, 2))
    ex = np.abs(xs - ref["x_star"]).max()
    alphas = np.array([h["alpha"] for h in ref["hist"]])
    print(f"ms: |u* - u*_oracle| max {err.max():.2e}, |x* - x*_oracle| {ex:.2e}; oracle step sizes "
          f"{[np.unique(a).tolist() for a in alphas]}; resets {[int(h['reset'].sum()) for h in ref['hist']]}; "
          f"status {np.bincount(st)}")
    assert (st == 0).all(), st
    assert err.max() < U_TOL, np.argsort(err)[-5:]
    # x*: the state iterate, or its rollout where the last step reset it -- a discrete choice
    # between two merits; where the oracle's two merits were within 1e-6 (relative) of each
    # other, u* differences of ~1e-8 can flip it, so there x* may equal either candidate
    tie = np.abs(ref["hist"][-1]["reset_gap"]) < 1e-6
    exb = np.abs(xs - ref["x_star"]).max(axis=(1, 2))
    x_roll = Q.kin_predict(x0, us, kap, ds, 2.5)
    exb = np.where(tie, np.minimum(exb, np.abs(xs - x_roll).max(axis=(1, 2))), exb)
    print(f"reset near-ties: {np.nonzero(tie)[0].tolist()}; |x* - x*_oracle| max outside them "
          f"{exb.max():.2e}")
    assert exb.max() < 1e-6
    np.testing.assert_array_equal(u0, us[:, 0])
    phi_end = np.minimum(KS.merit(x0, us, kap, ds, 2.5, W), KS.merit(x0, us, kap, ds, 2.5, W, x=xs))
    assert (phi_end <= np.minimum(ps0, pm0) * (1 + 1e-9)).all()


@pytest.mark.parametrize("ms", [0, 1], ids=["single_shooting", "multiple_shooting"])
def test_kin_sqp_later_qp_failure_keeps_iterate(golden, ms):
    """A later QP of the globalised step that fails with non-finite output (injected through
    vc_debug_qp_fault after SQP iteration 1 on one problem) refuses its step: the accepted
    iterate is the one before it (no 0 * NaN), finite, equal to a run that stops one iteration
    earlier, and the step's status stays the first QP's.  The oracle restates the same rule
    (oracle/kin_sqp.py kin_sqp_solve: alpha = 0 keeps the iterate)."""
    g = golden
    obs = _obs(g)
    cfg = _cfg(3, 1)
    cfg["qp"]["ms"] = ms
    x0, ub, kap, ds = (g[k].astype(np.float64) for k in ("kin_x0", "kin_ubar", "kin_kappa", "kin_ds"))
    xw = Q.kin_predict(x0, ub, kap, ds, 2.5)
    bad = 7
    cfg2 = _cfg(2, 1)
    cfg2["qp"]["ms"] = ms
    with _ctx(cfg2, obs, len(x0)) as c:
        u0r, xsr, usr, str_, _ = c.solve(x0, kap, ds, ub.copy(), xbar=xw.copy())
    with _ctx(cfg, obs, len(x0)) as c:
        c._check(c.lib.vc_debug_qp_fault(c._h, 2, bad))
        u0, xs, us, st, it = c.solve(x0, kap, ds, ub.copy(), xbar=xw.copy())
    assert np.isfinite(us[bad]).all() and np.isfinite(xs[bad]).all() and np.isfinite(u0[bad]).all()
    assert st[bad] == str_[bad] == 0
    np.testing.assert_array_equal(us[bad], usr[bad])   # the third step was refused
    # x*: the state iterate before the refused step, or (multiple shooting, where its merit is
    # no lower) the rollout of the accepted inputs
    roll = Q.kin_predict(x0[bad:bad + 1], usr[bad:bad + 1], kap[bad:bad + 1], ds[bad:bad + 1], 2.5)[0]
    assert np.array_equal(xs[bad], xsr[bad]) or np.abs(xs[bad] - roll).max() < 1e-9
    np.testing.assert_array_equal(u0[bad], u0r[bad])
    assert (st == 0).all(), st


@pytest.mark.parametrize("N", [20, 50])
def test_kin_sqp_elastic_on_failure_vs_oracle(N):
    """vc_qp.elastic = -rho (the obstacle controller's setting): the SQP iteration solves the
    hard-row QP and re-solves the ones it leaves non-solved with elastic rows.  Problems: the C2
    sampler with the delta box tightened to +-0.05 rad and the closed loop's trust region, so
    most first QPs are infeasible with hard rows.  Before, those steps were non-solved; now every
    step is solved.  One SQP iteration, so the kernel's retry decision is its hard pass's status:
    it must agree with oracle/kin_sqp.py's (a diverged or unpolished hard interior point) and
    u* must match the oracle's elastic-on-failure step to 1e-5."""
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.workload import kinematic_batch
    S = 1
    cfg = _cfg(S, solver=1, N=N)
    cfg["qp"] = dict(cfg["qp"], trust_a=1.0, trust_w=0.1, elastic=-1e3, max_iter=80)
    cfg["state_constraints"] = dict(cfg["state_constraints"], delta_max=0.05, delta_min=-0.05)
    W = Q.kin_weights(cfg)
    d = kinematic_batch(32, N=N, seed=91)
    ref = KS.kin_sqp_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], 2.5, W, S, elastic=-1e3)
    p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=cfg)
    with Context(model=_abi.VC_MODEL_KINEMATIC, N=N, max_batch=32, dtype=_abi.VC_F64, params=p) as c:
        u0, xs, us, st, it = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())
    cfg_h = dict(cfg, qp=dict(cfg["qp"], elastic=0.0))
    with Context(model=_abi.VC_MODEL_KINEMATIC, N=N, max_batch=32, dtype=_abi.VC_F64,
                 params=make_params(kin_car=load_config("kinematic_car"), kin_mpc=cfg_h)) as c:
        st_hard = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())[3]
    retried = ref["hist"][0]["elastic_retry"]
    err = np.abs(us - ref["u_star"]).max(axis=(1, 2))
    print(f"N={N}: hard rows non-solved {int((st_hard != 0).sum())} of {len(st)} (oracle {int(retried.sum())}); "
          f"elastic on failure non-solved {int((st != 0).sum())}; |u* - u*_oracle| max {err.max():.2e}")
    assert (st_hard != 0).sum() >= len(st) // 2
    np.testing.assert_array_equal(st_hard != 0, retried)
    assert (st == 0).all(), st
    assert err.max() < U_TOL, err
