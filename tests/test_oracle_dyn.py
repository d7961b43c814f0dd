"""CPU: the dynamic single-track SQP oracle (oracle/dyn_sqp.py) against finite
differences, its own KKT certificates and the committed golden vectors."""
import numpy as np
import pytest

from oracle import dyn_sqp as D
from oracle import models as M
from oracle import qp as QP


@pytest.fixture(scope="module")
def dyn_W():
    from vcmpc.config import load_config
    return D.dyn_weights(load_config("dynamic_mpc"))


@pytest.fixture(scope="module")
def dyn_golden():
    import os
    from conftest import GOLDEN
    return dict(np.load(os.path.join(GOLDEN, "dyn_sqp_golden.npz")))


def _sample(rng):
    x = np.array([rng.uniform(8, 20), rng.uniform(-.3, .3), rng.uniform(-.2, .5), rng.uniform(-.1, .2),
                  rng.uniform(0, 100), rng.uniform(-2, 2), rng.uniform(-.3, .3), 1.0])
    u = np.array([rng.uniform(-2000, 2000), rng.uniform(-.3, .3)])
    return x, u, rng.uniform(0, .04), rng.uniform(.3, .6)


@pytest.mark.parametrize("tyre", ["linear", "fiala"])
@pytest.mark.parametrize("seed", range(3))
def test_complex_step_jacobians_vs_finite_differences(dyn_params, tyre, seed):
    """Complex-step A, B of the RK4 spatial step (dynamic_car.py:169-191) agree with
    central differences of the same step."""
    x, u, k, h = _sample(np.random.default_rng(seed))
    A, Bm = D.dyn_linearize(x[None, None], np.stack([u, u])[None], np.full((1, 2), k), np.full((1, 2), h),
                            dyn_params, tyre)
    f = lambda xx, uu: M.dyn_spatial_transition(xx, uu, k, h, dyn_params, tyre)
    for j in range(8):
        e = np.zeros(8); e[j] = 1e-6 * max(1.0, abs(x[j]))
        fd = (f(x + e, u) - f(x - e, u)) / (2 * e[j])
        np.testing.assert_allclose(A[0, 0, :, j], fd, rtol=1e-5, atol=1e-6)
    for j in range(2):
        e = np.zeros(2); e[j] = 1e-6 * max(1.0, abs(u[j]))
        fd = (f(x, u + e) - f(x, u - e)) / (2 * e[j])
        np.testing.assert_allclose(Bm[0, 0, :, j], fd, rtol=1e-5, atol=1e-9)


def test_stage_term_gradients_vs_finite_differences(dyn_params):
    rng = np.random.default_rng(4)
    for _ in range(5):
        x, u, _, _ = _sample(rng)
        T = D.stage_terms(x[None, None], u[None, None], dyn_params)
        X5 = np.concatenate([x[:4], u[:1]])
        for name, (v, gr) in T.items():
            for j in range(5):
                e = np.zeros(5); e[j] = 1e-6 * max(1.0, abs(X5[j]))
                fp = D.stage_functions(X5 + e, dyn_params)[name]
                fm = D.stage_functions(X5 - e, dyn_params)[name]
                np.testing.assert_allclose(gr[0, 0, j], (fp - fm) / (2 * e[j]), rtol=1e-5, atol=1e-7)


def test_linear_tyre_is_first_fiala_term(dyn_params):
    a = np.linspace(-0.05, 0.05, 11)
    assert np.allclose(M.linear_lateral_force(a, dyn_params["Caf"]), -dyn_params["Caf"] * np.tan(a))


def test_golden_qps_certified(dyn_golden, dyn_params, dyn_W):
    """Re-derive the first QP of every golden problem from its float32 inputs and
    check the stored first step against the KKT conditions; the stored first-QP
    data of four problems match bit-for-bit up to fp64 rounding."""
    g = dyn_golden
    f = {k: g[k].astype(np.float64) for k in ("x0", "ubar", "kappa", "ds")}
    Q0 = D.dyn_qp(f["x0"], f["ubar"], f["kappa"], f["ds"], dyn_params, dyn_W, "linear")
    np.testing.assert_allclose(Q0["xbar"][:4], g["xbar0"], rtol=1e-13, atol=1e-12)
    np.testing.assert_allclose(Q0["H"][:4], g["H0"], rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(Q0["g"][:4], g["g0"], rtol=1e-10, atol=1e-10)
    sol = QP.solve_qp_batch(Q0["H"], Q0["g"], Q0["C"], Q0["d"])
    np.testing.assert_allclose(sol["z"], g["dz"][:, 0], atol=1e-8)
    assert sol["polished"].all()
    assert g["kkt"].max() < 1e-9


def test_sqp_output_is_rollout_of_u_star(dyn_golden, dyn_params):
    g = dyn_golden
    x = D.dyn_predict(g["x0"].astype(np.float64), g["u_star"], g["kappa"].astype(np.float64),
                      g["ds"].astype(np.float64), dyn_params, "linear")
    np.testing.assert_allclose(x, g["x_star"], rtol=1e-12, atol=1e-12)


def test_dyn_horizon_params_quirks():
    """cascaded_mpc.py:323-330: ds = mpc_dt * Ux_pred[:N] (no +0.5), curvature at
    s0 + cumsum(ds) - ds[0]."""
    N = 5
    sp = np.zeros((8, N)); sp[0] = np.arange(N) + 10.0
    ds, k = D.dyn_horizon_params(np.array([0, 0, 0, 0, 7.0, 0, 0, 0]), sp, 0.03, N, lambda s: 2 * s)
    np.testing.assert_allclose(ds, 0.03 * sp[0])
    np.testing.assert_allclose(k, 2 * (7.0 + np.cumsum(ds) - ds[0]))


def test_c3_workload_is_well_posed():
    from vcmpc.workload import dynamic_batch
    d = dynamic_batch(64, seed=3)
    assert all(v.dtype == np.float32 and v.flags.c_contiguous for v in d.values())
    assert d["x0"].shape == (64, 8) and d["ubar"].shape == (64, 40, 2)
    assert (d["x0"][:, 0] >= 8).all() and (np.abs(d["ubar"][..., 1]) <= 0.1).all()
