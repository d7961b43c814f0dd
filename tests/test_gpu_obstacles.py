"""GPU parity of the obstacle barrier terms (``obstacles: True``; kinematic_mpc.py:130-133,
cascaded_mpc.py:173-176) through the C ABI, against the oracle's
golden vectors (tests/golden/obs_golden.npz, make_obs_golden.py).

Tolerances: kinematic fp64 u* < 1e-5 (north star), H / g to 1e-10 relative; dynamic fp64
(st_sqp.hip, the parity path) scaled u* < 1e-5; dynamic fp32 (dyn_sqp.hip) scaled u* < 5e-4:
most golden predictions pass through an obstacle, where the floored margin gives curvatures
~1e5 and QP condition numbers up to 1.4e6 (vs <= 5e4 without obstacles, where the bar is
1e-4), so fp32 rounding is amplified ~30x more (the measured fp32 floor: DESIGN.md 2b).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

U_TOL_KIN = 1e-5
U_TOL_DYN = 1e-5          # fp64 st_sqp
U_TOL_DYN_F32 = 5e-4      # fp32 dyn_sqp (measured floor)
SCALE = np.array([1000.0, 1.0])


@pytest.fixture(scope="module")
def golden():
    return dict(np.load(os.path.join(GOLDEN, "obs_golden.npz")))


def _obs(g):
    return [tuple(float(v) for v in o) for o in g["obstacles"]]


def _kin_ctx(obstacles, B=64):
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=load_config("kinematic_mpc"), obstacles=obstacles)
    return Context(model=_abi.VC_MODEL_KINEMATIC, N=20, max_batch=B, dtype=_abi.VC_F64, params=p)


def _dyn_ctx(obstacles, B=64, tyre="linear", fp64=False):
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    p = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=load_config("dynamic_mpc"), tyre=tyre,
                    obstacles=obstacles)
    return Context(model=_abi.VC_MODEL_DYNAMIC, N=40, max_batch=B, dtype=_abi.VC_F64 if fp64 else _abi.VC_F32,
                   params=p)


def _kin_solve(c, g):
    return c.solve(g["kin_x0"], g["kin_kappa"], g["kin_ds"], g["kin_ubar"].copy())


def test_kin_condense_with_obstacles(golden):
    g = golden
    with _kin_ctx(_obs(g)) as c:
        H, gv = c.condense(g["kin_x0"][:8], g["kin_ubar"][:8], g["kin_kappa"][:8], g["kin_ds"][:8])
    np.testing.assert_allclose(H, g["kin_H"], rtol=1e-10, atol=1e-10 * np.abs(g["kin_H"]).max())
    np.testing.assert_allclose(gv, g["kin_g"], rtol=1e-10, atol=1e-10 * np.abs(g["kin_g"]).max())


def test_kin_solve_with_obstacles_vs_golden(golden):
    g = golden
    with _kin_ctx(_obs(g)) as c:
        u0, xs, us, st, it = _kin_solve(c, g)
    assert (st == 0).all(), st
    assert np.abs(us - g["kin_u_star"]).max() < U_TOL_KIN
    np.testing.assert_allclose(u0, us[:, 0])


@pytest.mark.parametrize("fp64", [True, False], ids=["fp64", "fp32"])
def test_dyn_solve_with_obstacles_vs_golden(golden, fp64):
    g = golden
    z = np.float64 if fp64 else np.float32
    with _dyn_ctx(_obs(g), fp64=fp64) as c:
        u0, xs, us, st, it = c.solve(g["dyn_x0"].astype(z), g["dyn_kappa"].astype(z), g["dyn_ds"].astype(z),
                                     g["dyn_ubar"].astype(z))
    assert (st == 0).all(), st
    err = np.abs((us.astype(np.float64) - g["dyn_u_star"]) / SCALE).max(axis=(1, 2))
    print("scaled |u* - u*_oracle| per problem:", np.array2string(err, precision=1))
    assert err.max() < (U_TOL_DYN if fp64 else U_TOL_DYN_F32), err.max()


def test_set_obstacles_switches_terms(golden):
    from vcmpc import _abi
    g = golden
    with _kin_ctx([]) as plain:
        ref_off = _kin_solve(plain, g)[2]
    with _kin_ctx(_obs(g)) as c:
        on = _kin_solve(c, g)[2]
        c.set_obstacles([])
        off = _kin_solve(c, g)[2]
        c.set_obstacles(_obs(g))
        on2 = _kin_solve(c, g)[2]
        with pytest.raises(_abi.VcError):
            c.set_obstacles([(0.0, 0.0, 1.0)] * (_abi.VC_MAX_OBSTACLES + 1))
        with pytest.raises(_abi.VcError):
            c.set_obstacles([(np.nan, 0.0, 1.0)])
    np.testing.assert_array_equal(off, ref_off)
    np.testing.assert_array_equal(on2, on)
    assert np.abs(on - off).max() > 1e-3


def _min_clearance(X, obstacles, i_s, i_ey):
    """min over steps and obstacles of dist((s, ey), obstacle) - radius, per vehicle."""
    s, ey = X[..., i_s], X[..., i_ey]
    return np.min([np.hypot(s - so, ey - eo) - r for so, eo, r in obstacles], axis=0).min(axis=0)


def test_kinematic_closed_loop_with_obstacles():
    """BatchedRacingSimulator with the kinematic controller and ``obstacles: True`` on
    ippodromo (the reference's kinematic default, config/controllers/kinematic.yaml:4),
    vehicles starting on the centre line ahead of the obstacle field.  Without the barrier
    terms every vehicle drives through an obstacle; with them the controller takes the
    globalised step (10 SQP steps with the merit line search per control step, in multiple
    shooting: controllers/kinematic_mpc.py KIN_OBS_SQP / KIN_OBS_MS, csrc/kin_merit.hip): no
    vehicle touches an obstacle, every vehicle stays on the track, <= 2 % non-solved steps
    (measured 0.03 %; single shooting 0.04 %; round 1's one convexified QP per step: 39 of 64 hit,
    21 % non-solved)."""
    from vcmpc.config import load_config
    from vcmpc.environment import Track
    from vcmpc.models import KinematicCar
    from vcmpc.simulation import BatchedRacingSimulator
    tr = Track.load("ippodromo")
    obs = [(o.s, o.ey, o.radius) for o in tr.obstacles]
    B, K = 64, 400
    rng = np.random.default_rng(3)
    x0 = np.zeros((B, 6))
    x0[:, 0] = rng.uniform(5, 8, B)
    x0[:, 2] = rng.uniform(0, 15, B)
    x0[:, 3] = rng.uniform(-0.5, 0.5, B)
    res = {}
    for flag in (True, False):
        cfg = load_config("kinematic_mpc")
        cfg["obstacles"] = flag
        car = KinematicCar(load_config("kinematic_car"), tr)
        sim = BatchedRacingSimulator(car, cfg, tr, batch=B)
        out = sim.reset(x0.copy()).run(K)
        X = out["state_traj"]
        assert np.isfinite(X).all()
        res[flag] = (_min_clearance(X, obs, 2, 3), X, out["nfail"])
    clear_on, X_on, nfail_on = res[True]
    clear_off, _, _ = res[False]
    print("clearance with obstacles: median %.3f, %d/%d clear; without: median %.3f, %d/%d clear; "
          "non-solved steps %d of %d; max |ey| %.2f"
          % (np.median(clear_on), int((clear_on > 0).sum()), B, np.median(clear_off), int((clear_off > 0).sum()), B,
             int(nfail_on.sum()), B * K, np.abs(X_on[:, :, 3]).max()))
    assert (clear_off < 0).sum() >= B // 2          # the obstacle field is in the way
    assert (clear_on > 0).all()                      # no vehicle touches an obstacle
    assert (np.abs(X_on[:, :, 3]) < tr.width / 2).all()
    assert np.median(X_on[-1, :, 2]) > 200.0         # through the field (obstacles up to s = 185)
    assert nfail_on.sum() <= 0.02 * B * K, nfail_on.sum()


def _kin_obstacle_loop(N, seed, B=64, K=400):
    from vcmpc.config import load_config
    from vcmpc.environment import Track
    from vcmpc.models import KinematicCar
    from vcmpc.simulation import BatchedRacingSimulator
    tr = Track.load("ippodromo")
    obs = [(o.s, o.ey, o.radius) for o in tr.obstacles]
    rng = np.random.default_rng(seed)
    x0 = np.zeros((B, 6))
    x0[:, 0] = rng.uniform(5, 8, B)
    x0[:, 2] = rng.uniform(0, 15, B)
    x0[:, 3] = rng.uniform(-0.5, 0.5, B)
    cfg = load_config("kinematic_mpc")
    cfg["obstacles"] = True
    cfg["horizon"] = N
    car = KinematicCar(load_config("kinematic_car"), tr)
    sim = BatchedRacingSimulator(car, cfg, tr, batch=B)
    out = sim.reset(x0.copy()).run(K)
    X = out["state_traj"]
    clear = _min_clearance(X, obs, 2, 3)
    on = (np.abs(X[:, :, 3]) < tr.width / 2).all(axis=0)
    print(f"N={N} seed={seed}: {int((clear > 0).sum())}/{B} clear, {int(on.sum())}/{B} on track, non-solved "
          f"{int(out['nfail'].sum())} of {B * K}, max |ey| {np.abs(X[:, :, 3]).max():.2f}, median s_end "
          f"{np.median(X[-1, :, 2]):.1f}")
    return X, clear, on, out["nfail"], tr


def test_kinematic_closed_loop_with_obstacles_n30():
    """The same obstacle loop at N = 30: every vehicle clear and on track, <= 0.2 % non-solved."""
    X, clear, on, nfail, tr = _kin_obstacle_loop(30, 3)
    assert (clear > 0).all()
    assert on.all()
    assert nfail.sum() <= 0.002 * nfail.size * 400


@pytest.mark.parametrize("seed", [3, 5, 7, 11])
def test_kinematic_closed_loop_with_obstacles_reference_horizon(seed):
    """The reference's default kinematic controller (config/controllers/kinematic.yaml: N = 50,
    obstacles True; kinematic_mpc.py:110-133) on the obstacle loop, four seeds.  Round 3 lost
    vehicles here (seed 5: |ey| 35.5 m and 32.5 m, seed 11: 58 m, after runs of non-solved steps;
    0.9-1.7 % non-solved).  Round 4 found three causes on the captured failing steps
    (scripts/kin_lost_capture.py + kin_lost_replay.py, kin_loop_cpu.py): the merit line
    search stopped short (8 step sizes, no steps below the merit's rounding level: the SQP stalled
    on a stale plan), an accepted multiple-shooting iterate could leave the model's domain (plans
    spinning to |epsi| >> pi/2, whose defect rollout made the next QP infeasible), and the QPs
    through an obstacle needed more than the 40 interior-point iterations of the C2 cap.  Bars
    (VERDICT r03 item 1): nobody lost (|ey| < width / 2 + 2.5 m for every vehicle at every step),
    every vehicle clear of every obstacle, <= 0.5 % non-solved steps."""
    X, clear, on, nfail, tr = _kin_obstacle_loop(50, seed)
    assert np.isfinite(X).all()
    assert np.abs(X[:, :, 3]).max() < tr.width / 2 + 2.5
    assert (clear > 0).all()
    assert nfail.sum() <= 0.005 * nfail.size * 400
    assert np.median(X[-1, :, 2]) > 200.0         # through the field (obstacles up to s = 185)


def test_dynamic_closed_loop_avoids_obstacles():
    """The single-track NMPC with ``obstacles: True`` through vc_simulate (3 SQP
    iterations per control step, 40-stage preview): on track, and no vehicle touches
    an obstacle, while without the barrier terms every one does."""
    from vcmpc.config import load_config
    from vcmpc.environment import Track
    from vcmpc.models import DynamicCar
    from vcmpc.simulation import BatchedRacingSimulator
    tr = Track.load("ippodromo")
    obs = [(o.s, o.ey, o.radius) for o in tr.obstacles]
    B, K = 64, 300
    rng = np.random.default_rng(4)
    x0 = np.zeros((B, 8))
    x0[:, 0] = rng.uniform(8, 11, B)
    x0[:, 4] = rng.uniform(0, 15, B)
    x0[:, 5] = rng.uniform(-0.5, 0.5, B)
    hits = {}
    for flag in (True, False):
        cfg = load_config("dynamic_mpc")
        cfg["mpc_dt"] = 0.045
        cfg["obstacles"] = flag
        car = DynamicCar(load_config("dynamic_car"), tr, tyre="fiala")
        sim = BatchedRacingSimulator(car, cfg, tr, batch=B)
        out = sim.reset(x0.copy()).run(K)
        X = out["state_traj"]
        assert np.isfinite(X).all()
        if flag:
            assert (np.abs(X[:, :, 5]) < tr.width / 2).mean() > 0.99
            assert out["nfail"].sum() <= 0.02 * B * K
        hits[flag] = int((_min_clearance(X, obs, 4, 5) < 0).sum())
    print("dynamic obstacle hits with / without barrier terms:", hits)
    assert hits[False] >= B // 2
    assert hits[True] == 0
