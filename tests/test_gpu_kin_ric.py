"""GPU parity of the stagewise-Riccati kinematic kernel (csrc/kin_ric.hip) through the C ABI,
against the fp64 oracle of the LTV-QP contract (oracle/ltv_qp.py, exact dense QP + active-set
polish) and its golden vectors -- at BASELINE's N = 20 (qp.solver = 1 forces this kernel
where the condensed kin_ltv.hip is built) and at the reference's own kinematic horizon
N = 50 (config/controllers/kinematic.yaml:2), plus N = 10 .. 60.

Tolerance: the north star's ||u* - u*_oracle||_inf < 1e-5 (a in m/s^2, w in rad/s); x* (the
linearised prediction x* = xbar + G du*) to 1e-6.
"""
import numpy as np
import pytest

from oracle import ltv_qp as Q

pytestmark = pytest.mark.gpu

U_TOL = 1e-5
X_TOL = 1e-6
L = 2.5


def _ctx(N, B=256, obstacles=None, solver=1, qp=None):
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    cfg = load_config("kinematic_mpc")
    cfg["qp"] = dict(cfg.get("qp") or {}, solver=solver, **(qp or {}))
    p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=cfg, obstacles=obstacles)
    return Context(model=_abi.VC_MODEL_KINEMATIC, N=N, max_batch=B, dtype=_abi.VC_F64, params=p)


def test_kin_ric_vs_golden_n20(kin_golden):
    g = kin_golden
    with _ctx(20) as c:
        u0, xs, us, st, it, dg = c.solve(g["x0"], g["kappa"], g["ds"], g["ubar"].copy(), diag=True)
    err = np.abs(us - g["u_star"]).max()
    print(f"N=20 golden: |u* - u*_oracle| = {err:.3e}, IPM iterations {it.min()}..{it.max()}, "
          f"polished {(dg[:, 2].astype(int) & 4 > 0).mean():.3f}")
    assert (st == 0).all(), (st, dg)
    assert err < U_TOL
    np.testing.assert_array_equal(u0, us[:, 0])
    assert np.abs(xs - g["x_star"]).max() < X_TOL


@pytest.mark.parametrize("N", [10, 30, 40, 50, 60])
def test_kin_ric_horizons_vs_oracle(N, kin_W):
    """Fresh C2-sampler problems at each built horizon; N = 50 is kinematic.yaml's."""
    from vcmpc.workload import kinematic_batch
    d = kinematic_batch(24, N=N, seed=300 + N)
    ref = Q.kin_ltv_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], L, kin_W)
    with _ctx(N) as c:
        u0, xs, us, st, it = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())
    err = np.abs(us - ref["u_star"]).max()
    xerr = np.abs(xs - ref["x_star"]).max()
    print(f"N={N}: |u* - u*_oracle| = {err:.3e}, |x* - x*_oracle| = {xerr:.3e}, iterations {it.min()}..{it.max()}")
    assert (st == 0).all(), st
    assert err < U_TOL
    assert xerr < X_TOL


def test_kin_ric_matches_condensed_kernel():
    """N = 20: the stagewise and the condensed kernel (kin_ltv.hip) solve the same QP."""
    from vcmpc.workload import kinematic_batch
    d = kinematic_batch(1024, N=20, seed=41)
    with _ctx(20, B=1024, solver=1) as c:
        r1 = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())
    with _ctx(20, B=1024, solver=0) as c:
        r0 = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())
    assert (r1[3] == 0).all() and (r0[3] == 0).all()
    err = np.abs(r1[2] - r0[2]).max()
    print(f"N=20, 1024 problems: |u*_riccati - u*_condensed| = {err:.3e}")
    assert err < U_TOL


def test_kin_ric_obstacles_vs_golden():
    import os
    from conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, "obs_golden.npz"))
    obs = [tuple(float(v) for v in o) for o in g["obstacles"]]
    with _ctx(20, obstacles=obs) as c:
        u0, xs, us, st, it = c.solve(g["kin_x0"], g["kin_kappa"], g["kin_ds"], g["kin_ubar"].copy())
    err = np.abs(us - g["kin_u_star"]).max()
    print(f"obstacles: |u* - u*_oracle| = {err:.3e}, status {np.bincount(st)}")
    assert (st == 0).all()
    assert err < U_TOL


def test_kin_ric_trust_region_vs_oracle(kin_W):
    """The closed-loop controller's real-time-iteration trust region (qp.trust_a/trust_w)."""
    from vcmpc.workload import kinematic_batch
    d = kinematic_batch(16, N=50, seed=9)
    W = dict(kin_W, trust_a=1.0, trust_w=0.1)
    ref = Q.kin_ltv_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], L, W)
    with _ctx(50, qp={"trust_a": 1.0, "trust_w": 0.1}) as c:
        u0, xs, us, st, it = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())
    assert (st == 0).all()
    assert np.abs(us - ref["u_star"]).max() < U_TOL
    assert np.abs(us - d["ubar"])[..., 0].max() <= 1.0 + 1e-9


def test_kin_ric_batch_properties_n50(kin_W):
    """kinematic.yaml's horizon at a C4-shard-sized batch: all solved, inputs inside their
    boxes, bit-identical reruns, host = device pointers, sampled oracle checks."""
    import torch
    from vcmpc.workload import kinematic_batch
    B = 8192
    d = kinematic_batch(B, N=50, seed=77)
    with _ctx(50, B=B) as c:
        u0, xs, us, st, it, dg = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
        t = {k: torch.from_numpy(v).cuda() for k, v in d.items()}
        r = c.solve(t["x0"], t["kappa"], t["ds"], t["ubar"])
        torch.cuda.synchronize()
        us2 = r[2].cpu().numpy()
    print(f"N=50 B={B}: solved {(st == 0).mean():.5f}, iterations mean {it.mean():.1f} max {it.max()}")
    bad = np.nonzero(st != 0)[0]
    assert len(bad) == 0, [(int(b), dg[b].tolist()) for b in bad[:4]]
    np.testing.assert_array_equal(us, us2)
    assert us[..., 0].max() <= 3 + 1e-9 and us[..., 0].min() >= -3 - 1e-9
    assert np.abs(us[..., 1]).max() <= 0.4 + 1e-9
    assert xs[:, 1:-1, 1].max() <= 0.3 + 1e-8 and xs[:, 1:-1, 1].min() >= -0.3 - 1e-8
    idx = np.arange(0, B, B // 8)
    ref = Q.kin_ltv_solve(d["x0"][idx], d["ubar"][idx], d["kappa"][idx], d["ds"][idx], L, kin_W)
    assert np.abs(us[idx] - ref["u_star"]).max() < U_TOL


def test_kin_ric_closed_loop_n20():
    """The batched simulator with the stagewise kernel forced at N = 20 (qp.solver = 1): 64
    vehicles x 200 steps on ippodromo, like the condensed kernel (test_gpu_closed_loop)."""
    from vcmpc.config import load_config
    from vcmpc.environment import Track
    from vcmpc.models import KinematicCar
    from vcmpc.simulation import BatchedRacingSimulator
    track = Track.load("ippodromo")
    car = KinematicCar(load_config("kinematic_car"), track)
    B, K = 64, 200
    rng = np.random.default_rng(3)
    x0 = np.zeros((B, 6))
    x0[:, 0] = rng.uniform(4, 9, B)
    x0[:, 2] = rng.uniform(0, track.length, B)
    x0[:, 3] = rng.uniform(-1.5, 1.5, B)
    res = {}
    for solver in (0, 1):
        cfg = load_config("kinematic_mpc")
        cfg["qp"] = dict(cfg.get("qp") or {}, solver=solver)
        sim = BatchedRacingSimulator(car, cfg, track, batch=B)
        out = sim.reset(x0).run(K)
        X = out["state_traj"]
        res[solver] = (np.abs(X[:, :, 3]).max(), int(out["nfail"].sum()), np.median(X[-1, :, 2] - X[0, :, 2]))
        print(f"solver={solver}: max |ey| {res[solver][0]:.2f}, non-solved steps {res[solver][1]}, "
              f"median progress {res[solver][2]:.1f} m")
        assert np.isfinite(X).all()
        assert res[solver][1] <= 0.01 * B * K
        assert res[solver][0] < track.width / 2
    assert abs(res[1][2] - res[0][2]) < 1.0


def test_kinematic_closed_loop_reference_horizon():
    """BatchedRacingSimulator with the kinematic controller at the reference's horizon N = 50
    (config/controllers/kinematic.yaml:2) on ippodromo, 64 vehicles x 400 steps: every vehicle
    on the track, <= 1 % non-solved steps (measured 0.06 %).  The controller takes the shifted
    warm start from N = 30 on (controllers/kinematic_mpc.py KIN_SHIFT_FROM_N, vc_qp.shift):
    with the reference's unshifted one, the single-shooting rollout of the lagging warm start
    crosses the spatial model's eps = +-pi/2 singularity and 52 of 64 vehicles leave the track
    (scripts/kin_shift_test.py, scripts/kin_obs_fail_modes.py)."""
    from vcmpc.config import load_config
    from vcmpc.environment import Track
    from vcmpc.models import KinematicCar
    from vcmpc.simulation import BatchedRacingSimulator
    tr = Track.load("ippodromo")
    B, K = 64, 400
    rng = np.random.default_rng(3)
    x0 = np.zeros((B, 6))
    x0[:, 0] = rng.uniform(5, 8, B)
    x0[:, 2] = rng.uniform(0, 15, B)
    x0[:, 3] = rng.uniform(-0.5, 0.5, B)
    cfg = load_config("kinematic_mpc")
    cfg["horizon"] = 50
    sim = BatchedRacingSimulator(KinematicCar(load_config("kinematic_car"), tr), cfg, tr, batch=B)
    out = sim.reset(x0).run(K)
    X = out["state_traj"]
    print(f"N=50: max |ey| {np.abs(X[:, :, 3]).max():.2f}, non-solved {int(out['nfail'].sum())} of {B * K}, "
          f"progress median {np.median(X[-1, :, 2] - X[0, :, 2]):.1f} m")
    assert np.isfinite(X).all()
    assert (np.abs(X[:, :, 3]) < tr.width / 2).all()
    assert out["nfail"].sum() <= 0.01 * B * K
    assert np.median(X[-1, :, 2] - X[0, :, 2]) > 250.0


def _ms_ctx(N, B, ms, obstacles=None, kin_sqp=0):
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    cfg = load_config("kinematic_mpc")
    cfg["horizon"] = N
    cfg["qp"] = dict(cfg["qp"], solver=1, ms=ms, kin_sqp=kin_sqp)
    p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=cfg, obstacles=obstacles)
    return cfg, Context(model=_abi.VC_MODEL_KINEMATIC, N=N, max_batch=B, dtype=_abi.VC_F64, params=p)


@pytest.mark.parametrize("N", [20, 50])
def test_kin_ric_multiple_shooting_vs_oracle(N):
    """vc_qp.ms = 1: the QP linearised at given warm-start states (the rollout perturbed, so the
    defects are nonzero) matches the oracle's multiple-shooting QP (oracle/ltv_qp.py
    kin_qp(..., x_ws=)) to 1e-5; with consistent states (the rollout itself) it equals the
    single-shooting step."""
    from vcmpc.workload import kinematic_batch
    d = kinematic_batch(16, N=N, seed=11 + N)
    cfg, c1 = _ms_ctx(N, 16, 1)
    W = Q.kin_weights(cfg)
    xr = Q.kin_predict(d["x0"], d["ubar"], d["kappa"], d["ds"], 2.5)
    rng = np.random.default_rng(N)
    xw = xr.copy()
    xw[:, 1:, [0, 1, 3, 4]] += rng.normal(scale=[0.05, 0.003, 0.02, 0.005], size=(16, N, 4))
    with c1:
        r = c1.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), xbar=xw.copy())
        rc = c1.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), xbar=xr.copy())
    ref = Q.kin_ltv_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], 2.5, W, x_ws=xw)
    ref_ss = Q.kin_ltv_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], 2.5, W)
    err = np.abs(r[2] - ref["u_star"]).max()
    err_c = np.abs(rc[2] - ref_ss["u_star"]).max()
    print(f"N={N}: multiple shooting |u* - u*_oracle| {err:.2e} (x* {np.abs(r[1] - ref['x_star']).max():.2e}); "
          f"consistent states vs the single-shooting oracle {err_c:.2e}")
    assert (r[3] == 0).all() and (rc[3] == 0).all()
    assert err < 1e-5 and err_c < 1e-5
    assert np.abs(r[1] - ref["x_star"]).max() < 1e-6


@pytest.mark.parametrize("N", [20, 50])
def test_kin_ric_elastic_rows_vs_oracle(N):
    """vc_qp.elastic = rho: the v / delta rows get slacks t >= 0 at cost rho t + 1e-8 t^2
    (oracle/ltv_qp.py elastic_qp, the QP of the kinematic obstacle SQP).  Problems: the C2
    sampler with the delta box tightened to +-0.05 rad and the closed loop's trust region
    (1.0 / 0.1), so most QPs have no feasible point with hard rows (phase-1 LP certificates,
    oracle/feasibility.py) and every elastic QP has a solution.  Bar: solved, u* within the
    north star's 1e-5 of the oracle's elastic optimum."""
    from oracle.feasibility import phase1
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.workload import kinematic_batch
    cfg = load_config("kinematic_mpc")
    cfg["qp"] = dict(cfg.get("qp") or {}, solver=1, trust_a=1.0, trust_w=0.1, elastic=1e3)
    cfg["state_constraints"] = dict(cfg["state_constraints"], delta_max=0.05, delta_min=-0.05)
    W = Q.kin_weights(cfg)
    d = kinematic_batch(48, N=N, seed=77)
    Qd = Q.kin_qp(d["x0"], d["ubar"], d["kappa"], d["ds"], L, W)
    infeasible = sum(not phase1(Qd["C"][b], Qd["d"][b])["feasible"] for b in range(len(d["x0"])))
    ref = Q.kin_ltv_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], L, W, elastic=1e3)
    assert ref["polished"].all() and ref["kkt"]["pfeas"].max() < 1e-9
    p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=cfg)
    with Context(model=_abi.VC_MODEL_KINEMATIC, N=N, max_batch=48, dtype=_abi.VC_F64, params=p) as c:
        u0, xs, us, st, it, dg = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
    err = np.abs(us - ref["u_star"]).max(axis=(1, 2))
    print(f"N={N}: {infeasible} of {len(err)} hard-row QPs infeasible; elastic |u* - u*_oracle| max "
          f"{err.max():.2e}, t max {ref['t'].max():.3f}, iterations {it.min()}..{it.max()}, "
          f"polished {(dg[:, 2].astype(int) & 4 > 0).mean():.2f}")
    assert infeasible >= len(err) // 2
    assert (st == 0).all(), (st, dg[st != 0])
    assert err.max() < U_TOL, err
