"""CPU: the reference NLP fixture (tests/golden/kin_nlp_golden.npz, oracle/kin_nlp.py) and the
oracle's kinematic SQP iterated to convergence.

1. The fixture's solutions are KKT points of the NLP of controllers/mpc/kinematic_mpc.py:15-158
   (certificate recomputed here: relative stationarity and feasibility < 1e-10) and satisfy its
   bounds; the NLP solver's own derivatives match finite differences.
2. The oracle's SQP contract (oracle/kin_sqp.py: Gauss-Newton QP + proximal term + merit line
   search, the algorithm csrc/kin_merit.hip runs) iterated 40 times from the golden warm starts
   reaches the same U* to the north star's 1e-5 (single shooting, a subset for time).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import kin_nlp as KN
from oracle import kin_sqp as KS
from oracle import ltv_qp as Q


@pytest.fixture(scope="module")
def data():
    from vcmpc.config import load_config
    g = dict(np.load(os.path.join(GOLDEN, "kin_ltv_golden.npz")))
    g.update(np.load(os.path.join(GOLDEN, "kin_nlp_golden.npz")))
    W = Q.kin_weights(load_config("kinematic_mpc"))
    W["obstacles"] = []
    return g, W


def _prob(g, W, b):
    return KN.KinNLP(g["x0"][b], g["kappa"][b], g["ds"][b], float(g["L"]), W)


def test_nlp_derivatives_match_finite_differences(data):
    g, W = data
    P = _prob(g, W, 3)
    rng = np.random.default_rng(0)
    z = P.pack(KN.warm_start(g["x0"][3], g["ubar"][3], g["kappa"][3], g["ds"][3], float(g["L"])), g["ubar"][3])
    z = z + 1e-3 * rng.standard_normal(z.shape)
    h = 1e-6
    for j in rng.choice(P.nz, 12, replace=False):
        e = np.zeros(P.nz)
        e[j] = h
        assert abs((P.f(z + e) - P.f(z - e)) / (2 * h) - P.grad(z)[j]) < 1e-6
        np.testing.assert_allclose((P.c(z + e) - P.c(z - e)) / (2 * h), P.jac_c(z)[:, j], atol=1e-6)


def test_fixture_is_a_kkt_point_of_the_reference_nlp(data):
    g, W = data
    conv = g["converged"]
    assert conv.sum() >= 0.9 * len(conv)
    for b in np.nonzero(conv)[0][::4]:
        P = _prob(g, W, b)
        z = P.pack(g["x_nlp"][b], g["u_nlp"][b])
        k = P.kkt(z)
        assert k["stat"] < 1e-10 and k["pfeas"] < 1e-10, (b, k)
        lb, ub = P.bounds()
        assert (z >= lb - 1e-12).all() and (z <= ub + 1e-12).all()


def test_oracle_sqp_fixed_point_is_the_nlp_optimum(data):
    g, W = data
    idx = np.nonzero(g["converged"])[0][:16]
    sl = lambda k: g[k][idx]
    r = KS.kin_sqp_solve(sl("x0"), sl("ubar"), sl("kappa"), sl("ds"), float(g["L"]), W, 40)
    err = np.abs(r["u_star"] - g["u_nlp"][idx]).max(axis=(1, 2))
    print("oracle SQP (40 iterations) vs NLP optimum: max |du| %.2e" % err.max())
    assert err.max() < 1e-5


def test_obstacle_fixture_is_a_kkt_point_of_the_reference_nlp():
    """tests/golden/kin_nlp_obs_golden.npz (make_kin_nlp_obs_golden.py): the reference NLP with its
    obstacle barrier (kinematic_mpc.py:130-133) at N = 20 and kinematic.yaml's N = 50.  Every
    converged entry is a KKT point of that NLP (certificate recomputed here, < 1e-10), its stored
    barrier margin is the one along X*, and the margin-above-floor entries the GPU test compares
    exist at both horizons."""
    from vcmpc.config import load_config
    g = dict(np.load(os.path.join(GOLDEN, "kin_nlp_obs_golden.npz")))
    W = Q.kin_weights(load_config("kinematic_mpc"))
    W["obstacles"] = [tuple(float(v) for v in o) for o in g["obstacles"]]
    for N in (20, 50):
        conv, margin = g[f"n{N}_converged"], g[f"n{N}_margin"]
        assert (conv & (margin > 0.05)).sum() >= 5, N
        for b in np.nonzero(conv)[0][::3]:
            P = KN.KinNLP(g[f"n{N}_x0"][b], g[f"n{N}_kappa"][b], g[f"n{N}_ds"][b], 2.5, W)
            X, U = g[f"n{N}_x_nlp"][b], g[f"n{N}_u_nlp"][b]
            k = P.kkt(P.pack(X, U))
            assert k["stat"] < 1e-10 and k["pfeas"] < 1e-10, (N, b, k)
            m = min(float(np.min(np.hypot(X[1:N, 2] - so, X[1:N, 3] - eo) - (r + 0.1))) for so, eo, r in W["obstacles"])
            assert abs(m - margin[b]) < 1e-12
