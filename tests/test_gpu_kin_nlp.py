"""GPU: the kinematic SQP iterated to convergence reaches the reference NLP's optimum
(VERDICT r03 "next" item 3; SURVEY 8(c): IPOPT cannot run here, so the reference's optimum is
the same NLP -- controllers/mpc/kinematic_mpc.py:15-158 -- solved independently by
oracle/kin_nlp.py into tests/golden/kin_nlp_golden.npz, make_kin_nlp_golden.py).

The build's contract takes SQP steps on a Gauss-Newton QP with a proximal term and the
`if_else` branches frozen at each iterate (oracle/kin_sqp.py, csrc/kin_merit.hip); at a fixed
point the proximal term and the Gauss-Newton model drop out of the first-order conditions, so
the fixed point is a KKT point of the reference NLP.  Here the device SQP (vc_qp.kin_sqp = 40,
no trust region, single and multiple shooting) runs on the C2 golden problems from their warm
starts and u* must equal the NLP's U* to the north star's 1e-5 wherever the NLP solve
converged (KKT certificate < 1e-10) and the device reports solved; the others are listed.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import kin_nlp as KN
from oracle import ltv_qp as Q

pytestmark = pytest.mark.gpu

U_TOL = 1e-5
SQP_ITERS = 40


@pytest.fixture(scope="module")
def data():
    g = dict(np.load(os.path.join(GOLDEN, "kin_ltv_golden.npz")))
    g.update(np.load(os.path.join(GOLDEN, "kin_nlp_golden.npz")))
    return g


@pytest.mark.parametrize("ms", [0, 1], ids=["single_shooting", "multiple_shooting"])
def test_kin_sqp_converges_to_reference_nlp_optimum(data, ms):
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    g = data
    cfg = load_config("kinematic_mpc")
    cfg["qp"] = dict(cfg["qp"], kin_sqp=SQP_ITERS, ms=ms, trust_a=0.0, trust_w=0.0)
    p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=cfg, obstacles=[])
    B = len(g["x0"])
    L = float(g["L"])
    x_ws = Q.kin_predict(g["x0"], g["ubar"], g["kappa"], g["ds"], L) if ms else None
    with Context(model=_abi.VC_MODEL_KINEMATIC, N=20, max_batch=B, dtype=_abi.VC_F64, params=p) as c:
        u0, xs, us, st, it = c.solve(g["x0"], g["kappa"], g["ds"], g["ubar"].copy(),
                                     xbar=None if x_ws is None else np.ascontiguousarray(x_ws))
    W = Q.kin_weights(cfg)
    W["obstacles"] = []
    err = np.abs(us - g["u_nlp"]).max(axis=(1, 2))
    stat_sqp = np.array([KN.KinNLP(g["x0"][b], g["kappa"][b], g["ds"][b], L, W).kkt(
        KN.KinNLP(g["x0"][b], g["kappa"][b], g["ds"][b], L, W).pack(
            KN.warm_start(g["x0"][b], us[b], g["kappa"][b], g["ds"][b], L), us[b]))["stat"] for b in range(B)])
    both = g["converged"] & (st == 0)
    print(f"ms={ms}: NLP converged {int(g['converged'].sum())}/{B}, device solved {int((st == 0).sum())}/{B}; "
          f"where both: |u*_SQP - U*_NLP| max {err[both].max():.2e}, median {np.median(err[both]):.2e}; "
          f"device SQP KKT stat (on the NLP) median {np.median(stat_sqp):.1e} max {stat_sqp.max():.1e}")
    for b in np.nonzero(~both)[0]:
        print(f"  not compared: problem {b}: NLP converged {bool(g['converged'][b])} (stat {g['stat'][b]:.1e}), "
              f"device status {int(st[b])}, |du| {err[b]:.2e}")
    for b in np.nonzero(both & (err >= U_TOL))[0]:
        print(f"  MISMATCH: problem {b}: |du| {err[b]:.2e}, NLP f {g['f'][b]:.9f}, SQP KKT stat {stat_sqp[b]:.1e}")
    assert both.sum() >= 0.9 * B
    assert err[both].max() < U_TOL


# Round 5: the reference's default kinematic controller -- obstacles: True
# (config/controllers/kinematic.yaml:2,4; barrier kinematic_mpc.py:130-133) -- at N = 20 and its own
# N = 50, against the reference NLP with the barrier solved independently (tests/golden/
# kin_nlp_obs_golden.npz, make_kin_nlp_obs_golden.py).  The reference's barrier w ds / (dist - r - 0.1)
# is negative inside an obstacle and unbounded below at its boundary from inside, so many of its
# "optima" sit inside an obstacle (trust-constr then runs to f ~ -1e16: no KKT point); the build's
# barrier equals it wherever the margin dist - r - 0.1 is above its 0.05 m floor.
# Compared: problems whose NLP solve converged (KKT < 1e-10) with the optimum's margin above the
# floor everywhere, and the device SQP solved.  Where the device's answer is a KKT point of the same
# NLP with the same objective (the same local optimum, |f_SQP - f_NLP| <= 1e-9 (1 + |f|)) it must equal
# U_NLP to the north star's 1e-5; every other compared problem is listed with both NLP objective
# values (a different local optimum is shown, not asserted).
# The reference NLP is nearly flat along the acceleration inputs (only the 1e-4 slew term prices them,
# kinematic.yaml), and the barrier's curvature changes fast along the plan: the SQP converges slowly there
# (r05d at 40 iterations: equal objectives to 9 digits with |du| up to 7e-3, KKT stat 1e-8..3e-6), so the
# comparison runs 200 SQP iterations with the proximal weight at 1e-6 (the SQP's fixed point does not
# depend on it; at the contract's 1e-4 each step only closes ~30 % of the gap along directions of
# curvature ~4e-5, r05e: |du| up to 8e-2 at equal objectives after 200 iterations).
SQP_ITERS_OBS = 200
PROX_OBS = 1e-6


@pytest.fixture(scope="module")
def obs_data():
    path = os.path.join(GOLDEN, "kin_nlp_obs_golden.npz")
    if not os.path.exists(path):
        pytest.skip("kin_nlp_obs_golden.npz not generated")
    return dict(np.load(path))


@pytest.mark.parametrize("N", [20, 50])
@pytest.mark.parametrize("ms", [0, 1], ids=["single_shooting", "multiple_shooting"])
def test_kin_sqp_obstacles_vs_reference_nlp(obs_data, N, ms):
    from oracle import ltv_qp as Q
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    g = {k[len(f"n{N}_"):]: v for k, v in obs_data.items() if k.startswith(f"n{N}_")}
    obs = [tuple(float(v) for v in o) for o in obs_data["obstacles"]]
    L = 2.5
    cfg = load_config("kinematic_mpc")
    cfg["qp"] = dict(cfg["qp"], kin_sqp=SQP_ITERS_OBS, ms=ms, trust_a=0.0, trust_w=0.0, max_iter=80,
                     solver=1, prox=PROX_OBS)
    p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=cfg, obstacles=obs)
    B = len(g["x0"])
    x_ws = Q.kin_predict(g["x0"], g["ubar"], g["kappa"], g["ds"], L) if ms else None
    with Context(model=_abi.VC_MODEL_KINEMATIC, N=N, max_batch=B, dtype=_abi.VC_F64, params=p) as c:
        u0, xs, us, st, it = c.solve(g["x0"], g["kappa"], g["ds"], g["ubar"].copy(),
                                     xbar=None if x_ws is None else np.ascontiguousarray(x_ws))
    W = Q.kin_weights(cfg)
    W["obstacles"] = obs
    f_sqp, stat_sqp = np.full(B, np.nan), np.full(B, np.nan)
    for b in range(B):
        P = KN.KinNLP(g["x0"][b], g["kappa"][b], g["ds"][b], L, W)
        z = P.pack(KN.warm_start(g["x0"][b], us[b], g["kappa"][b], g["ds"][b], L), us[b])
        if np.isfinite(z).all():
            f_sqp[b], stat_sqp[b] = P.f(z), P.kkt(z)["stat"]
    err = np.abs(us - g["u_nlp"]).max(axis=(1, 2))
    comparable = g["converged"] & (g["margin"] > 0.05) & (st == 0)
    same = comparable & (stat_sqp < 1e-10) & (np.abs(f_sqp - g["f"]) <= 1e-9 * (1 + np.abs(g["f"])))
    print(f"N={N} ms={ms}: {B} problems, NLP converged {int(g['converged'].sum())} (optimum inside an obstacle's "
          f"margin floor: {int((g['converged'] & (g['margin'] <= 0.05)).sum())}), device solved {int((st == 0).sum())}; "
          f"compared {int(comparable.sum())}, same KKT point {int(same.sum())}, "
          f"|u_SQP - U_NLP| max there {err[same].max() if same.any() else float('nan'):.2e}")
    for b in np.nonzero(comparable & ~same)[0]:
        print(f"  different point: problem {b}: f_NLP {g['f'][b]:.9f}, f_SQP {f_sqp[b]:.9f} (SQP KKT stat on the NLP "
              f"{stat_sqp[b]:.1e}), |du| {err[b]:.2e}")
    assert same.sum() >= 1
    assert err[same].max() < U_TOL
