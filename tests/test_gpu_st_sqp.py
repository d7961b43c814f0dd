"""GPU parity of the fp64 single-track SQP kernel (csrc/st_sqp.hip: stagewise Riccati
interior point) through the C ABI, against the fp64 oracle (oracle/dyn_sqp.py, exact
dense QPs) and its golden vectors -- BASELINE config 3's contract at N = 40 and the
reference's own horizons N = 50 / 60 (config/controllers/singletrack.yaml:2, recorded runs
experiments/data/*/singletrack_config.yaml).

Tolerance: the north star's ||u* - u*_ref||_inf < 1e-5, here in the reference's own
units (Fx [N], w [rad/s]) -- no scaling needed in fp64.
"""
import copy

import numpy as np
import pytest

from oracle import dyn_sqp as D
from oracle import models as M

pytestmark = pytest.mark.gpu

U_TOL = 1e-5   # max |u* - u*_oracle|, Fx in N and w in rad/s
X_TOL = 1e-6   # x* = rollout(u*), absolute


def _ctx(N, mpc_cfg=None, tyre="linear", max_batch=4096, obstacles=None):
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    cfg = mpc_cfg if mpc_cfg is not None else load_config("dynamic_mpc")
    params = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=cfg, tyre=tyre, obstacles=obstacles)
    return Context(model=_abi.VC_MODEL_DYNAMIC, N=N, max_batch=max_batch, dtype=_abi.VC_F64, params=params)


@pytest.fixture(scope="module")
def golden():
    import os
    from conftest import GOLDEN
    return {k: v.astype(np.float64) for k, v in np.load(os.path.join(GOLDEN, "dyn_sqp_golden.npz")).items()}


def _W(cfg_name="dynamic_mpc"):
    from vcmpc.config import load_config
    return D.dyn_weights(load_config(cfg_name))


def test_st_sqp_vs_golden_n40(golden):
    g = golden
    with _ctx(40) as ctx:
        ub = g["ubar"].copy()
        u0, xs, us, st, it, dg = ctx.solve(g["x0"], g["kappa"], g["ds"], ub, diag=True)
    assert (st == 0).all(), (st, dg)
    err = np.abs(us - g["u_star"]).max()
    print(f"N=40 golden: max |u* - u*_oracle| = {err:.3e} (Fx in N), IPM iterations {it.min()}..{it.max()}")
    assert err < U_TOL
    np.testing.assert_array_equal(u0, us[:, 0])
    assert np.abs(xs - g["x_star"]).max() < X_TOL


@pytest.mark.parametrize("N,tyre,cfg_name", [(40, "fiala", "dynamic_mpc"), (50, "fiala", "singletrack_mpc"),
                                             (60, "fiala", "singletrack_mpc"), (60, "linear", "singletrack_mpc")])
def test_st_sqp_reference_horizons_vs_oracle(N, tyre, cfg_name, dyn_params):
    """Fresh C3-sampler problems at the reference's horizons vs the oracle run here."""
    from vcmpc.config import load_config
    from vcmpc.workload import dynamic_batch
    cfg = load_config(cfg_name)
    W = D.dyn_weights(cfg)
    d = {k: v.astype(np.float64) for k, v in dynamic_batch(6, N=N, seed=100 + N, tyre=tyre).items()}
    ref = D.dyn_sqp_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], dyn_params, W, tyre)
    with _ctx(N, cfg, tyre) as ctx:
        ub = d["ubar"].copy()
        u0, xs, us, st, it = ctx.solve(d["x0"], d["kappa"], d["ds"], ub)
    assert (st == 0).all(), st
    err = np.abs(us - ref["u_star"]).max()
    print(f"N={N} {tyre}: max |u* - u*_oracle| = {err:.3e}, IPM iterations {it.min()}..{it.max()}")
    assert err < U_TOL
    assert np.abs(xs - ref["x_star"]).max() < X_TOL


def test_st_sqp_obstacles_vs_oracle(dyn_params):
    """Obstacle barrier terms (cascaded_mpc.py:173-176) on problems whose
    horizon crosses ippodromo's obstacle field."""
    import os
    from conftest import GOLDEN
    from vcmpc.config import load_config
    g = np.load(os.path.join(GOLDEN, "obs_golden.npz"))
    if "dyn_x0" not in g:
        pytest.skip("no dynamic obstacle problems in obs_golden.npz")
    d = {k: g["dyn_" + k].astype(np.float64) for k in ("x0", "kappa", "ds", "ubar")}
    obs = [tuple(r) for r in g["obstacles"]]
    cfg = load_config("dynamic_mpc")
    W = D.dyn_weights(cfg)
    W["obstacles"] = obs
    ref = D.dyn_sqp_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], dyn_params, W, "linear")
    with _ctx(40, cfg, "linear", obstacles=obs) as ctx:
        ub = d["ubar"].copy()
        u0, xs, us, st, it = ctx.solve(d["x0"], d["kappa"], d["ds"], ub)
    err = np.abs(us - ref["u_star"]).max()
    print(f"obstacles: max |u* - u*_oracle| = {err:.3e}, status {np.bincount(st)}")
    assert (st == 0).all()
    assert err < U_TOL


def test_st_sqp_batch_properties():
    """C3-sized batch (B = 4096, N = 40) in fp64: every problem solved, inputs inside
    their boxes, bit-identical reruns, host = device pointers."""
    import torch
    from vcmpc.config import load_config
    from vcmpc.workload import dynamic_batch
    B = 4096
    d = {k: v.astype(np.float64) for k, v in dynamic_batch(B, N=40, seed=77).items()}
    cfg = load_config("dynamic_mpc")
    with _ctx(40, cfg, "linear", max_batch=B) as ctx:
        ub = d["ubar"].copy()
        u0, xs, us, st, it = ctx.solve(d["x0"], d["kappa"], d["ds"], ub)
        t = {k: torch.from_numpy(v).cuda() for k, v in d.items()}
        r = ctx.solve(t["x0"], t["kappa"], t["ds"], t["ubar"])
        torch.cuda.synchronize()
        us2 = r[2].cpu().numpy()
    print(f"B=4096: solved {(st == 0).mean():.4f}, IPM iterations mean {it.mean():.1f} max {it.max()}")
    assert (st == 0).all(), np.bincount(st)
    np.testing.assert_array_equal(us, us2)
    ic = cfg["input_constraints"]
    assert us[..., 1].max() <= ic["w_max"] + 1e-9 and us[..., 1].min() >= ic["w_min"] - 1e-9


def test_st_sqp_n60_batch_nonsolved_are_infeasible(dyn_params):
    """The bench's N = 60 leg (singletrack_mpc.yaml, B = 4096, seed 31): every problem solved
    unless one of its SQP iterations meets a linearised QP with no feasible point -- decided
    by a phase-1 LP (oracle/feasibility.py, HiGHS) with a checked Farkas certificate, on the
    oracle's own SQP iterates up to the first such QP.  (Round 2's seven non-solved problems
    all came from full SQP steps whose rollout left the spatial model's domain; with the
    domain cut-back of the contract, oracle/dyn_sqp.py domain_step, the oracle solves every QP
    of all seven and the kernel is expected to as well.)"""
    from oracle import feasibility as F
    from vcmpc.config import load_config
    from vcmpc.workload import dynamic_batch
    B, N = 4096, 60
    cfg = load_config("singletrack_mpc")
    d = {k: v.astype(np.float64) for k, v in dynamic_batch(B, N=N, seed=31).items()}
    with _ctx(N, cfg, "linear", max_batch=B) as ctx:
        u0, xs, us, st, it, dg = ctx.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
    bad = np.nonzero(st != 0)[0]
    print(f"N=60 B={B}: solved {(st == 0).mean():.5f}, IPM iterations mean {it.mean():.1f} max {it.max()}, "
          f"non-solved {[(int(i), dg[i].tolist()) for i in bad[:10]]}")
    assert len(bad) <= 12
    if len(bad):
        W = D.dyn_weights(cfg)
        sub = {k: v[bad] for k, v in d.items()}
        ref = D.dyn_sqp_solve(sub["x0"], sub["ubar"], sub["kappa"], sub["ds"], dyn_params, W, "linear",
                              keep_qps=True)
        first, farkas = F.first_infeasible_iteration(ref["hist"])
        print("first SQP iteration with an infeasible QP (-1: none):", first.tolist(), "Farkas ok:", farkas.tolist())
        assert (first >= 0).all() and farkas.all()
    ok = st == 0
    assert np.isfinite(us[ok]).all()


def test_st_sqp_newton_rollout_is_the_rollout():
    """Round 4: after the second QP step the linear-tyre kernel re-rolls the plan by chord-Newton
    sweeps from the pre-step trajectory (st_sqp.hip ST_NEWTON_ROLLOUT).  Its x* must be the serial
    rollout of u* (vc_rollout, one lane walking the stages) up to the accepted defects (1e-14
    relative per stage) carried through the dynamics, on a C3-sized batch at 3 and at 10 SQP
    iterations (more Newton rollouts).  Measured at a 1e-13 acceptance: 1.4e-13 and 3.0e-10 (the
    low-speed lateral mode amplifies a stage defect); the bar, 1e-9, is 4 orders below X_TOL."""
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.workload import dynamic_batch
    B = 4096
    d = {k: v.astype(np.float64) for k, v in dynamic_batch(B, N=40, seed=78).items()}
    for sqp in (3, 10):
        cfg = load_config("dynamic_mpc")
        cfg["qp"] = dict(cfg["qp"], sqp_iters=sqp)
        with _ctx(40, cfg, "linear", max_batch=B) as ctx:
            u0, xs, us, st, it = ctx.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())
            xr = ctx.rollout(d["x0"], us, d["kappa"], d["ds"])[:, :40]
        rel = np.abs(xs - xr).max(axis=(1, 2)) / (1.0 + np.abs(xr).max(axis=(1, 2)))
        print(f"sqp {sqp}: solved {(st == 0).mean():.4f}, |x* - rollout(u*)| / scale max {rel.max():.2e}")
        assert (st == 0).all()
        assert rel.max() < 1e-9


def test_st_sqp_newton_rollout_low_speed_n60():
    """The chord-Newton rollout where the RK4 step's lateral mode is unstable (|eig A_k| 3-5 below
    ~6 m/s): N = 60 (singletrack.yaml), linear tyre, starts like the reference's recorded
    runs (Ux ~ U(4, 6) m/s, Uy = r = 0, small delta / ey / epsi) with a neutral warm start (constant
    Fx, w = 0) and ds = mpc_dt Ux0.  A defect the chord iteration accepts at 1e-14 grows through 59
    expansive stages, so below ST_NEWTON_UX_MIN (8 m/s along the pre-step plan) the kernel rolls out
    serially.  The plan is then defined only up to the rollout's own rounding amplification (vc_rollout
    itself moves by up to 8.6e-8 relative when u* changes by one ulp, r05i), and the kernel's serial
    rollout (algebraic tan-alpha form) and vc_rollout's differ at rounding level: x* must equal
    vc_rollout(u*) to X_TOL relative.  (Before the switch, on a harsher low-speed set: 0.28.)"""
    from vcmpc.config import load_config
    B, N = 1024, 60
    rng = np.random.default_rng(79)
    x0 = np.zeros((B, 8))
    x0[:, 0] = rng.uniform(4.0, 6.0, B)
    x0[:, 3] = rng.uniform(-0.02, 0.02, B)
    x0[:, 4] = rng.uniform(0.0, 300.0, B)
    x0[:, 5] = rng.uniform(-1.0, 1.0, B)
    x0[:, 6] = rng.uniform(-0.05, 0.05, B)
    kappa = np.repeat(rng.uniform(0.0, 0.047, (B, 4)), N // 4, axis=1)
    ds = np.repeat(0.03 * x0[:, :1], N, axis=1)
    ubar = np.zeros((B, N, 2))
    ubar[:, :, 0] = rng.uniform(300.0, 1500.0, (B, 1))
    for sqp in (3, 10):
        cfg = load_config("singletrack_mpc")
        cfg["qp"] = dict(cfg["qp"], sqp_iters=sqp)
        with _ctx(N, cfg, "linear", max_batch=B) as ctx:
            u0, xs, us, st, it = ctx.solve(x0, kappa, ds, ubar.copy())
            xr = ctx.rollout(x0, us, kappa, ds)[:, :N]
            xp = ctx.rollout(x0, np.ascontiguousarray(us * (1 + 2.0 ** -52)), kappa, ds)[:, :N]
        ok = st == 0
        scale = 1.0 + np.abs(xr).max(axis=(1, 2))
        rel = np.abs(xs - xr).max(axis=(1, 2)) / scale
        spread = np.abs(xp - xr).max(axis=(1, 2)) / scale
        print(f"N=60 low speed, sqp {sqp}: solved {ok.mean():.4f}, |x* - rollout(u*)| / scale max {rel[ok].max():.2e}; "
              f"rollout spread under a 1-ulp input change: median {np.median(spread[ok]):.1e} max {spread[ok].max():.1e}")
        assert ok.sum() >= 100
        assert rel[ok].max() < X_TOL   # measured 1.6e-7 (r05i), the 1-ulp spread reaching 8.6e-8


def test_st_sqp_low_speed_obstacles_converge():
    """Round 4: the reference's RK4 step is unstable in the lateral mode at low speed (|eig A_k| 3-5
    at Ux = 4 m/s, Fx = 0), so the open-loop dual-residual sweep amplified rounding ~1e30 over 60
    stages once an obstacle's barrier gradient excited that mode and the interior point never met
    its tolerance (every step of the recorded shoe obstacle run failed).  With the residual through
    the closed-loop A + BK the first step from the recorded start (Ux = 4, s = 1, neutral warm
    start, N = 60, shoe's 9 obstacles) solves, with and without obstacles, on both tracks."""
    from vcmpc.config import load_config, obstacle_list
    from vcmpc.controllers.cascaded_mpc import dyn_horizon_params
    from vcmpc.environment import Track
    x0 = np.array([[4.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0]])
    for name in ("shoe", "ippodromo"):
        tr = Track.load(name)
        for obs in (True, False):
            cfg = load_config("singletrack_mpc")
            cfg["horizon"], cfg["obstacles"] = 60, obs
            ds, kap = dyn_horizon_params(x0[:, 4], np.full((1, 60), 4.0), float(cfg["mpc_dt"]), tr.k)
            with _ctx(60, cfg, "fiala", max_batch=1, obstacles=obstacle_list(tr, cfg)) as ctx:
                u0, xs, us, st, it, dg = ctx.solve(x0, kap, ds, np.zeros((1, 60, 2)), diag=True)
            print(f"{name} obstacles={obs}: status {int(st[0])}, iterations {int(it[0])}, diag {np.round(dg[0], 9)}")
            assert st[0] == 0


@pytest.mark.parametrize("N,tyre", [(60, "linear"), (50, "fiala")])
def test_st_sqp_j_placement_bit_identical(N, tyre):
    """Round 5: for N >= 45 the launcher keeps the stage Jacobians in LDS while the batch fits the
    machine at that kernel's occupancy (three workgroups per CU: <= 768 problems on 256 CUs) and
    moves them to a global workspace beyond (four per CU; csrc/st_sqp.hip st_jg_pick).  The
    placement changes where J lives, not one floating-point operation: every problem of a 4,096
    batch (global J) must equal the same problem solved in LDS-J chunks of 512 bit for bit (ADVICE
    r05: the whole batch, so an addressing error in the per-problem workspace at any problem
    index -- the bounds-checked loads would return zeros, not fault -- shows as a mismatch)."""
    from vcmpc.config import load_config
    from vcmpc.workload import dynamic_batch
    B, CH = 4096, 512   # CH <= 768: LDS J at three workgroups per CU on 256 CUs
    d = {k: v.astype(np.float64) for k, v in dynamic_batch(B, N=N, seed=55, tyre=tyre).items()}
    cfg = load_config("singletrack_mpc")
    with _ctx(N, cfg, tyre, max_batch=B) as ctx:
        big = ctx.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
        parts = [ctx.solve(d["x0"][i:i + CH], d["kappa"][i:i + CH], d["ds"][i:i + CH], d["ubar"][i:i + CH].copy(),
                           diag=True) for i in range(0, B, CH)]
    small = [np.concatenate([p[j] for p in parts]) for j in range(len(big))]
    print(f"N={N} {tyre}: solved {(big[3] == 0).mean():.4f} of {B}")
    for a, b in zip(big, small):
        np.testing.assert_array_equal(a, b)
