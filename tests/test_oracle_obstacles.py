"""CPU checks of the obstacle barrier contract (oracle/obstacles.py) and its host
plumbing; the GPU side is tests/test_gpu_obstacles.py.

The reference's term (kinematic_mpc.py:130-133, cascaded_mpc.py:173-176) is
w ds / (dist - (r + 0.1)); the QP takes its convexified second-order model in ey.
"""
import os

import numpy as np
import pytest

from oracle import dyn_sqp as D
from oracle import ltv_qp as Q
from oracle import models as M
from oracle import obstacles as OB

from conftest import GOLDEN

OBS = [(30.0, 0.0, 1.0), (60.0, 0.0, 2.0), (100.0, 3.0, 2.0), (100.0, -3.0, 2.0)]


@pytest.fixture(scope="module")
def golden():
    return dict(np.load(os.path.join(GOLDEN, "obs_golden.npz")))


def test_slope_and_curvature_vs_finite_differences():
    rng = np.random.default_rng(0)
    s = rng.uniform(20, 110, 4000)
    ey = rng.uniform(-4, 4, 4000)
    wds = rng.uniform(1, 5, 4000)
    d = np.min([np.hypot(s - so, ey - eo) - (r + 0.1) for so, eo, r in OBS], axis=0)
    keep = d > 0.3  # away from the margin floor and the singular boundary
    s, ey, wds = s[keep], ey[keep], wds[keep]
    p, q = OB.ey_model(s, ey, wds, OBS)
    h = 1e-5
    f = lambda e: OB.barrier(s, e, wds, OBS)  # noqa: E731
    fd1 = (f(ey + h) - f(ey - h)) / (2 * h)
    fd2 = (f(ey + 1e-3) - 2 * f(ey) + f(ey - 1e-3)) / 1e-6
    np.testing.assert_allclose(p, fd1, rtol=1e-6, atol=1e-8)
    conv = fd2 > 1e-3
    np.testing.assert_allclose(q[conv], fd2[conv], rtol=1e-4, atol=1e-6)
    assert (q >= 0).all()
    assert (q[fd2 < -1e-3] == 0).all()   # the non-convex region is clamped to zero curvature


def test_behind_an_obstacle_is_a_saddle():
    # straight behind an obstacle the barrier has a local max in ey: slope 0, curvature clamped
    p, q = OB.ey_model(np.array([25.0]), np.array([0.0]), 3.0, [(30.0, 0.0, 1.0)])
    assert abs(p[0]) < 1e-15 and q[0] == 0.0


def test_margin_floor():
    # inside the margin the derivatives use margin_min (finite, large, convex push-out)
    p, q = OB.ey_model(np.array([30.0]), np.array([0.5]), 1.0, [(30.0, 0.0, 1.0)], margin_min=0.05)
    assert np.isfinite(p).all() and np.isfinite(q).all()
    assert p[0] < 0 and q[0] > 0            # pushes towards larger ey (away from the centre)


def test_kin_qp_with_obstacles_adds_ey_terms(kin_W):
    from vcmpc.workload import kinematic_batch
    d = kinematic_batch(6, seed=3)
    d["x0"][:, 2] = 25.0
    d["x0"][:, 3] = np.linspace(-1.5, 1.5, 6)
    W0 = dict(kin_W)
    W1 = dict(kin_W, obstacles=[(30.0, 0.0, 1.0)], w_obs=5.0)
    a = Q.kin_qp(d["x0"], d["ubar"], d["kappa"], d["ds"], 2.5, W0)
    b = Q.kin_qp(d["x0"], d["ubar"], d["kappa"], d["ds"], 2.5, W1)
    dH, dg = b["H"] - a["H"], b["g"] - a["g"]
    # the difference is sum_k q_k G_ey,k G_ey,k' and sum_k p_k G_ey,k
    G = a["G"][:, :, 3]
    p, q = OB.ey_model(a["xbar"][:, 1:20, 2], a["xbar"][:, 1:20, 3], 5.0 * d["ds"][:, 1:20], W1["obstacles"])
    np.testing.assert_allclose(dH, np.einsum("bk,bki,bkj->bij", q, G[:, 1:20], G[:, 1:20]), atol=1e-12)
    np.testing.assert_allclose(dg, np.einsum("bk,bki->bi", p, G[:, 1:20]), atol=1e-12)
    assert (np.linalg.eigvalsh(b["H"]) > 0).all()


def test_golden_kinematic_reproduces_and_obstacles_matter(golden, kin_W):
    g = golden
    sl = slice(0, 12)
    W1 = dict(kin_W, obstacles=[tuple(o) for o in g["obstacles"]])
    r = Q.kin_ltv_solve(g["kin_x0"][sl], g["kin_ubar"][sl], g["kin_kappa"][sl], g["kin_ds"][sl], 2.5, W1)
    np.testing.assert_allclose(r["u_star"], g["kin_u_star"][sl], atol=1e-9)
    r0 = Q.kin_ltv_solve(g["kin_x0"][sl], g["kin_ubar"][sl], g["kin_kappa"][sl], g["kin_ds"][sl], 2.5, kin_W)
    assert np.abs(r0["u_star"] - r["u_star"]).max(axis=(1, 2)).min() > 1e-4


def test_golden_dynamic_reproduces(golden, dyn_params):
    from vcmpc.config import load_config
    g = golden
    sl = slice(0, 3)
    W = D.dyn_weights(load_config("dynamic_mpc"))
    W["obstacles"] = [tuple(o) for o in g["obstacles"]]
    f = {k: g["dyn_" + k][sl].astype(np.float64) for k in ("x0", "ubar", "kappa", "ds")}
    R = D.dyn_sqp_solve(f["x0"], f["ubar"], f["kappa"], f["ds"], dyn_params, W, tyre="linear")
    np.testing.assert_allclose(R["u_star"], g["dyn_u_star"][sl], atol=1e-6)


def test_host_packing_and_track_obstacles():
    from vcmpc import _abi
    from vcmpc.config import load_config, obstacle_list, obstacles_struct
    from vcmpc.environment import Track
    tr = Track.load("ippodromo")
    assert [(o.s, o.ey, o.radius) for o in tr.obstacles][:2] == [(30.0, 0.0, 1.0), (60.0, 0.0, 2.0)]
    cx, cy, _ = tr.rel2glob(30.0, 0.0, 0.0)
    assert abs(tr.obstacles[0].cx - cx) < 1e-12 and abs(tr.obstacles[0].cy - cy) < 1e-12
    cfg = dict(load_config("kinematic_mpc"))
    assert obstacle_list(tr, cfg) == []
    cfg["obstacles"] = True
    rows = obstacle_list(tr, cfg)
    assert len(rows) == 7
    o = obstacles_struct(rows)
    assert o.n == 7 and o.radius[0] == 1.0 and o.ey[2] == 3.0 and o.margin_min == _abi.OBS_MARGIN_MIN
    with pytest.raises(ValueError):
        obstacles_struct([(0, 0, 1)] * (_abi.VC_MAX_OBSTACLES + 1))


def test_inside_mode_is_the_reference_barrier_inside():
    """vc_obstacles.inside (ABI 11): inside an obstacle beyond the floor band the QP model is the
    reference's own barrier w ds / (dist - r - 0.1) (negative there, cascaded_mpc.py:173-176): its
    slope is the central difference of phi; the curvature is phi'' clamped at 0.  In the band
    |margin| <= margin_min and outside the obstacle the two modes agree; default mode unchanged."""
    obs = [(30.0, 0.0, 1.0)]
    wds = 0.7
    s = np.full(5, 30.4)
    ey = np.array([0.0, 0.3, -0.5, 1.1, 2.5])          # margins -1.1, -0.8, -0.47, ~0.07, 1.43
    m0 = np.hypot(s - 30.0, ey) - 1.1
    p1, q1 = OB.ey_model(s, ey, wds, obs, inside=True)
    p0, q0 = OB.ey_model(s, ey, wds, obs)
    h = 1e-6
    fd = (OB.barrier(s, ey + h, wds, obs) - OB.barrier(s, ey - h, wds, obs)) / (2 * h)
    fdd = (OB.barrier(s, ey + h, wds, obs) - 2 * OB.barrier(s, ey, wds, obs) + OB.barrier(s, ey - h, wds, obs)) / h ** 2
    deep = m0 < -OB.MARGIN_MIN
    assert deep.sum() == 3
    np.testing.assert_allclose(p1[deep], fd[deep], rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(q1[deep], np.maximum(fdd[deep], 0.0), rtol=1e-3, atol=1e-6)
    np.testing.assert_array_equal(p1[~deep], p0[~deep])
    np.testing.assert_array_equal(q1[~deep], q0[~deep])
    assert not np.allclose(p1[deep], p0[deep])
