"""CPU: the oracle against the reference's golden data and its own certificates."""
import numpy as np
import pytest

from oracle import ltv_qp as Q
from oracle import models as M
from oracle import qp as QP


def test_dyn_plant_matches_reference_traces(dyn_kat, dyn_params):
    """DynamicCar temporal RK4 (dynamic_car.py:144-167) reproduces the reference's
    recorded closed-loop traces (experiments/data/*)."""
    d = dyn_kat
    pred = M.dyn_transition(d["x"], d["u"], d["kappa"], float(d["dt"]), dyn_params)
    rel = np.abs(pred - d["x_next"]) / np.maximum(np.abs(d["x_next"]), 1e-9)
    assert rel.max() < 1e-12
    # Ux, Uy, r, delta do not depend on the back-solved curvature: genuine check
    assert rel[:, :4].max() < 1e-13


def test_dyn_negative_control(dyn_kat, dyn_params):
    p = dict(dyn_params, Caf=dyn_params["Caf"] * 1.01)
    pred = M.dyn_transition(dyn_kat["x"], dyn_kat["u"], dyn_kat["kappa"], 0.05, p)
    assert np.abs(pred - dyn_kat["x_next"]).max() > 1e-6


def _fd_jac(x, u, k, h, L, eps=1e-6):
    A = np.zeros((6, 6)); B = np.zeros((6, 2))
    for j in range(6):
        e = np.zeros(6); e[j] = eps
        A[:, j] = (M.kin_spatial_transition(x + e, u, k, h, L) - M.kin_spatial_transition(x - e, u, k, h, L)) / (2 * eps)
    for j in range(2):
        e = np.zeros(2); e[j] = eps
        B[:, j] = (M.kin_spatial_transition(x, u + e, k, h, L) - M.kin_spatial_transition(x, u - e, k, h, L)) / (2 * eps)
    return A, B


@pytest.mark.parametrize("seed", range(5))
def test_kin_jacobians_vs_finite_differences(seed):
    rng = np.random.default_rng(seed)
    x = np.array([rng.uniform(2, 10), rng.uniform(-.3, .3), 5.0, rng.uniform(-2, 2), rng.uniform(-.4, .4), 1.0])
    u = np.array([rng.uniform(-3, 3), rng.uniform(-.4, .4)])
    k, h = rng.uniform(0, .05), rng.uniform(.3, .9)
    A, B = M.kin_spatial_jacobians(x, u, k, h, 2.5)
    Af, Bf = _fd_jac(x, u, k, h, 2.5)
    np.testing.assert_allclose(A, Af, atol=1e-8)
    np.testing.assert_allclose(B, Bf, atol=1e-8)


def test_kin_temporal_matches_formula():
    x = np.array([5.0, 0.1, 3.0, 0.5, 0.05, 0.0]); u = np.array([1.0, 0.2])
    k, dt, L = 0.02, 0.05, 2.5
    sd = 5 * np.cos(0.05) / (1 - 0.5 * k)
    ref = x + dt * np.array([1.0, 0.2, sd, 5 * np.sin(0.05), 5 * np.tan(0.1) / L - sd * k, 1.0])
    np.testing.assert_allclose(M.kin_transition(x, u, k, dt, L), ref, rtol=1e-15)


def test_golden_solutions_certified(kin_golden, kin_W):
    """Re-derive the QP of every golden problem and check its KKT certificate."""
    g = kin_golden
    D = Q.kin_qp(g["x0"], g["ubar"], g["kappa"], g["ds"], float(g["L"]), kin_W)
    np.testing.assert_allclose(D["xbar"], g["xbar"], rtol=1e-14, atol=1e-14)
    np.testing.assert_allclose(D["H"][:16], g["H"], rtol=1e-12, atol=1e-12)
    dz = (g["u_star"] - g["ubar"]).reshape(len(g["x0"]), -1)
    k = QP.kkt_residuals(D["H"], D["g"], D["C"], D["d"], dz, g["lam"])
    assert max(v.max() for v in k.values()) < 1e-9
    x_star = D["xbar"] + np.einsum("bkin,bn->bki", D["G"], dz)
    np.testing.assert_allclose(x_star, g["x_star"], atol=1e-12)


def test_qp_solver_random_certificate():
    rng = np.random.default_rng(7)
    B, n, m = 8, 12, 30
    Mx = rng.normal(size=(B, n, n)); H = Mx @ np.swapaxes(Mx, 1, 2) + 0.1 * np.eye(n)
    g = rng.normal(size=(B, n)); C = rng.normal(size=(B, m, n)); d = rng.uniform(0.1, 1, (B, m))
    s = QP.solve_qp_batch(H, g, C, d)
    assert s["polished"].all()
    assert max(v.max() for v in s["kkt"].values()) < 1e-9


def test_horizon_params_quirks():
    """kinematic_mpc.py:177-187: ds uses v_pred[:N] + 0.5; kappa at the off-by-one s."""
    from vcmpc.controllers.kinematic_mpc import horizon_params
    N = 5
    sp = np.zeros((6, N + 1)); sp[0] = np.arange(N + 1) + 1.0
    ds_o, k_o = Q.kin_horizon_params(np.array([1, 0, 7.0, 0, 0, 0]), sp, 0.03, N, lambda s: s * 10)
    ds_h, k_h = horizon_params(np.array([7.0]), sp[0][None], 0.03, lambda s: s * 10)
    np.testing.assert_allclose(ds_h[0], ds_o); np.testing.assert_allclose(k_h[0], k_o)
    np.testing.assert_allclose(ds_o, 0.03 * sp[0, :N] + 0.5)
    s_expect = 7.0 + np.concatenate([[0], np.cumsum(ds_o[1:])])  # ds_traj[0] = 0, then ds_traj[1..]
    np.testing.assert_allclose(k_o, 10 * s_expect)
