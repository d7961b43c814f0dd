"""CPU tests of the phase-1 LP certificates (oracle/feasibility.py) and of the SQP contract's
domain cut-back (oracle/dyn_sqp.py domain_step) on the problems that round 2's kernel left
non-solved (bench N = 60 leg, seed 31): each of them had taken a full SQP step whose rollout
left the spatial model's domain (s' < 0 or Ux < 0 along the horizon)."""
import numpy as np
import pytest

from oracle import dyn_sqp as D
from oracle import feasibility as F

R02_N60_NONSOLVED = [418, 828, 1847, 2334, 2499, 2697, 3255]


def test_phase1_farkas_on_infeasible_box():
    C = np.array([[1.0, 0.0], [-1.0, 0.0], [0.0, 1.0]])
    d = np.array([-1.0, -1.0, 5.0])          # x <= -1 and x >= 1
    o = F.phase1(C, d)
    assert not o["feasible"] and o["farkas_ok"] and o["t"] > 0.5
    y = o["y"]
    assert (y >= 0).all() and np.abs(C.T @ y).max() < 1e-12 and d @ y < 0


def test_phase1_feasible_and_margin():
    rng = np.random.default_rng(0)
    C = rng.normal(size=(30, 6))
    z0 = rng.normal(size=6)
    d = C @ z0 + 0.3
    o = F.phase1(C, d)
    assert o["feasible"] and o["viol"] <= 1e-9
    m = F.phase1(C, d, t_min=-1.0)
    assert m["t"] < 0          # strictly feasible: an interior margin


@pytest.fixture(scope="module")
def n60_problems():
    import os
    from conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, "st_n60_cases.npz"))   # make_st_n60_cases.py
    assert g["idx"].tolist() == R02_N60_NONSOLVED
    return {k: g[k] for k in ("x0", "kappa", "ds", "ubar")}


def test_domain_step_solves_round2_nonsolved(n60_problems, dyn_params):
    """With the domain cut-back every QP of the seven problems' SQP is feasible (LP) and solved
    by the oracle to a KKT certificate; some steps are cut back (alpha < 1)."""
    from vcmpc.config import load_config
    d = n60_problems
    W = D.dyn_weights(load_config("singletrack_mpc"))
    ref = D.dyn_sqp_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], dyn_params, W, "linear", keep_qps=True)
    first, _ = F.first_infeasible_iteration(ref["hist"])
    assert (first == -1).all()
    for h in ref["hist"]:
        assert (h["kkt"]["pfeas"] < 1e-9).all() and (h["kkt"]["stat"] < 1e-6).all()
    # the full step left the domain somewhere (alpha < 1) -- the round-2 failure mode -- and a
    # cut-back step always exists here
    alphas = np.array([h["alpha"] for h in ref["hist"]])
    assert (alphas < 1).any(axis=0).sum() >= 5 and (alphas > 0).all()
    assert D.in_domain(D.dyn_predict(d["x0"], ref["u_star"], d["kappa"], d["ds"], dyn_params, "linear"),
                       d["kappa"]).all()
