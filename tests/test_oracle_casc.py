"""CPU checks of the cascaded SQP oracle (oracle/casc_sqp.py): the point-mass model
and switching map restated from models/dynamic_point_mass.py and cascaded_mpc.py:256-277,
their complex-step Jacobians, the condensed sensitivities, the golden vectors and the
horizon-parameter quirks of cascaded_mpc.py:316-338.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import casc_sqp as CS
from oracle import models as M


@pytest.fixture(scope="module")
def W():
    from vcmpc.config import load_config
    return CS.casc_weights(load_config("cascaded_mpc"))


@pytest.fixture(scope="module")
def golden():
    return dict(np.load(os.path.join(GOLDEN, "casc_sqp_golden.npz")))


def test_pm_ode_matches_reference_equations(dyn_params):
    p = dyn_params
    x = np.array([[15.0, 10.0, 0.5, 0.05, 1.0]])
    u = np.array([[800.0, 3000.0]])
    k = np.array([0.02])
    f = M.pm_temporal_ode(x, u, k, p)[0]
    V, s, ey, ep, t = x[0]
    sdot = V * np.cos(ep) / (1 - 0.02 * ey)
    assert np.isclose(f[0], (800 - p["Frr"] - p["Cd"] * V ** 2) / p["m"])   # dynamic_point_mass.py:79-82
    assert np.isclose(f[1], sdot)                                           # :83
    assert np.isclose(f[3], 3000 / (p["m"] * V) - 0.02 * sdot)              # :85
    fs = M.pm_spatial_ode(x, u, k, p)[0]
    assert fs[1] == 1.0 and np.isclose(fs[4], 1 / sdot) and np.isclose(fs[2], V * np.sin(ep) / sdot)


def test_jacobians_vs_central_differences(dyn_params, W):
    from vcmpc.workload import cascaded_batch
    d = cascaded_batch(3, seed=2)
    xs, xp = CS.casc_predict(d["x0"], d["ubar"], d["kappa"], d["ds"], dyn_params, W)
    As, Bs, Sw, Ap, Bp = CS.casc_linearize(xs, xp, d["ubar"], d["kappa"], d["ds"], dyn_params, W)
    N = W["N"]
    h = 1e-6
    # point-mass Euler step, stage m = 5
    m, j = 5, N + 5
    f = lambda x, u: M.pm_spatial_transition(x, u, d["kappa"][:, j], d["ds"][:, j], dyn_params)  # noqa: E731
    for i in range(5):
        e = np.zeros(5); e[i] = h * max(1.0, abs(xp[0, m, i]))
        fd = (f(xp[:, m] + e, d["ubar"][:, j]) - f(xp[:, m] - e, d["ubar"][:, j])) / (2 * e[i])
        np.testing.assert_allclose(Ap[:, m, :, i], fd, rtol=1e-6, atol=1e-8)
    for i in range(2):
        e = np.zeros(2); e[i] = 1e-3
        fd = (f(xp[:, m], d["ubar"][:, j] + e) - f(xp[:, m], d["ubar"][:, j] - e)) / 2e-3
        np.testing.assert_allclose(Bp[:, m, :, i], fd, rtol=1e-6, atol=1e-10)
    # switch map
    for i in range(8):
        e = np.zeros(8); e[i] = 1e-6
        fd = (M.st_to_pm(xs[:, N - 1] + e) - M.st_to_pm(xs[:, N - 1] - e)) / 2e-6
        np.testing.assert_allclose(Sw[:, :, i], fd, rtol=1e-6, atol=1e-9)


def test_condensed_sensitivities_predict_the_rollout(dyn_params, W):
    from vcmpc.workload import cascaded_batch
    d = cascaded_batch(2, seed=4)
    Q = CS.casc_qp(d["x0"], d["ubar"], d["kappa"], d["ds"], dyn_params, W)
    n = Q["g"].shape[1]
    rng = np.random.default_rng(0)
    dz = rng.uniform(-1, 1, (2, n)) * 1e-4
    scale = np.ones((n // 2, 2)); scale[:, 0] = W["fx_scale"]; scale[W["N"]:, 1] = W["fx_scale"]
    u2 = d["ubar"] + dz.reshape(2, -1, 2) * scale
    xs2, xp2 = CS.casc_predict(d["x0"], u2, d["kappa"], d["ds"], dyn_params, W)
    lin_s = Q["xs"] + np.einsum("bkin,bn->bki", Q["Gs"], dz)
    lin_p = Q["xp"] + np.einsum("bkin,bn->bki", Q["Gp"], dz)
    assert np.abs(xs2 - lin_s).max() < 1e-5 and np.abs(xp2 - lin_p).max() < 1e-5
    assert np.abs(xp2 - Q["xp"]).max() > 1e-4                     # the step is visible
    assert (np.linalg.eigvalsh(Q["H"]) > 0).all()


def test_golden_first_sqp_iteration_reproduces(golden, dyn_params, W):
    g = golden
    sl = slice(0, 2)
    Q = CS.casc_qp(g["x0"][sl], g["ubar"][sl], g["kappa"][sl], g["ds"][sl], dyn_params, W, "fiala")
    np.testing.assert_allclose(Q["H"], g["H0"][sl], rtol=1e-10, atol=1e-10)
    from oracle.qp import solve_qp_batch
    sol = solve_qp_batch(Q["H"], Q["g"], Q["C"], Q["d"])
    assert sol["polished"].all()
    np.testing.assert_allclose(sol["z"], g["dz0"][sl, 0], atol=1e-8)


def test_golden_shapes_and_trust_region(golden, W):
    g = golden
    H_ = W["N"] + W["M"]
    assert g["u_star"].shape[1:] == (H_, 2) and g["x_star"].shape[1:] == (H_, 8)
    S = W["fx_scale"]
    du = np.abs(g["u_star"] - g["ubar"])
    assert du[:, :, 0].max() <= 3 * W["trust_Fx"] + 1e-6                 # 3 SQP steps of the trust region
    assert du[:, W["N"]:, 1].max() <= 3 * W["trust_Fx"] + 1e-6
    assert (np.abs(g["u_star"][:, :W["N"], 1]) <= 0.4 + 1e-9).all()      # w box
    assert np.isfinite(g["x_star"]).all() and S == 1000.0


def test_horizon_params_quirks():
    N, Mh, ds_pm = 4, 3, 3.0
    x = np.zeros(8); x[4] = 10.0
    pred = np.zeros((8, N + Mh)); pred[0, :] = [10, 11, 12, 13, 1, 1, 1]
    ds, kap = CS.casc_horizon_params(x, pred, 0.1, N, Mh, ds_pm, lambda s: np.asarray(s) * 0.001)
    np.testing.assert_allclose(ds, [1.0, 1.1, 1.2, 1.3, 3, 3, 3])
    s_traj = np.cumsum([1.0, 1.1, 1.2, 1.3]) - 1.0 + 10.0              # cascaded_mpc.py:328
    s_pm = np.cumsum([3.0, 3, 3]) - 1.3 + s_traj[-1]                   # :335
    np.testing.assert_allclose(kap, np.concatenate([s_traj, s_pm]) * 0.001)
