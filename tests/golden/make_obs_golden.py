"""Generate tests/golden/obs_golden.npz: golden vectors of the obstacle barrier terms
(``obstacles: True``; kinematic_mpc.py:130-133, cascaded_mpc.py:173-176) inside the
kinematic LTV-QP and the dynamic SQP contracts, produced by the CPU oracle
(oracle/obstacles.py, oracle/ltv_qp.py, oracle/dyn_sqp.py).

Parity status: unpinned by the reference (no recorded run of the reference holds a
QP, and IPOPT cannot run here); every QP solution carries a KKT
certificate.  Obstacles: the `obstacle_data` of the reference's ippodromo track
(config/environment/ippodromo.yaml).  Inputs: the C2 / C3 samplers
(vcmpc/workload.py) moved so that every horizon sweeps past an obstacle, plus
edge cases (lined up behind an obstacle: the barrier's non-convex point; a
prediction inside the margin floor; beside an obstacle on the other lap side).

Run from the repo root:  python tests/golden/make_obs_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))

from oracle import dyn_sqp as D  # noqa: E402
from oracle import ltv_qp as Q  # noqa: E402
from oracle import models as M  # noqa: E402
from vcmpc.config import load_config  # noqa: E402
from vcmpc.workload import dynamic_batch, kinematic_batch  # noqa: E402

L = 2.5
OBS = [tuple(float(v) for v in o) for o in load_config(
    os.path.join(ROOT, "vehicle-control_amd", "config", "tracks", "ippodromo.yaml"))["obstacles"]]


def place(x0, rng, i_s, i_ey, before):
    """Move each problem's start to `before` metres ahead of a random obstacle."""
    B = len(x0)
    j = rng.integers(0, len(OBS), B)
    so = np.array([OBS[i][0] for i in j])
    eo = np.array([OBS[i][1] for i in j])
    x0[:, i_s] = so - rng.uniform(*before, B)
    x0[:, i_ey] = np.clip(eo + rng.uniform(-2.0, 2.0, B), -3.5, 3.5)
    return x0


def kin_cases():
    rng = np.random.default_rng(11)
    d = kinematic_batch(40, seed=7)
    d["x0"] = place(d["x0"].copy(), rng, 2, 3, (1.0, 14.0))
    # rebuild ds from the new x0 is unnecessary: ds depends on v only (kinematic_mpc.py:178-182)
    e = kinematic_batch(4, seed=8)
    x0 = e["x0"].copy()
    x0[0, 2], x0[0, 3] = 30.0 - 6.0, 0.0     # straight behind obstacle 0 (ey = 0): phi'' < 0 there
    x0[1, 2], x0[1, 3] = 30.0 - 2.5, 0.3     # margin floor active along the prediction
    x0[2, 2], x0[2, 3] = 100.0 - 5.0, 0.0    # between the two obstacles at s = 100 (ey = +-3)
    x0[3, 2], x0[3, 3] = 170.0 - 8.0, -1.5   # towards obstacle 5 (ey = -2.5)
    e["x0"] = x0
    return {k: np.concatenate([d[k], e[k]]) for k in d}


def dyn_cases():
    rng = np.random.default_rng(12)
    d = dynamic_batch(16, seed=9)
    x0 = d["x0"].astype(np.float64)
    x0 = place(x0, rng, 4, 5, (2.0, 10.0))
    d["x0"] = x0.astype(np.float32)
    return d


def main():
    kcfg = load_config("kinematic_mpc")
    WK = Q.kin_weights(kcfg)
    WK["obstacles"] = OBS
    k = kin_cases()
    sk = Q.kin_ltv_solve(k["x0"], k["ubar"], k["kappa"], k["ds"], L, WK)
    kk = sk["kkt"]
    print("kin B", len(k["x0"]), "iters", sk["iters"].max(), {n: float(v.max()) for n, v in kk.items()},
          "polished", sk["polished"].all())
    assert sk["polished"].all() and max(v.max() for v in kk.values()) < 1e-9

    dcfg = load_config("dynamic_mpc")
    WD = D.dyn_weights(dcfg)
    WD["obstacles"] = OBS
    p = M.dyn_params_from_config(load_config("dynamic_car"))
    d = dyn_cases()
    f64 = {n: v.astype(np.float64) for n, v in d.items()}
    R = D.dyn_sqp_solve(f64["x0"], f64["ubar"], f64["kappa"], f64["ds"], p, WD, tyre="linear")
    dk = max(float(h["kkt"][n].max()) for h in R["hist"] for n in ("stat", "pfeas", "dfeas", "comp"))
    print("dyn B", len(d["x0"]), "kkt max", dk)
    assert dk < 1e-8

    out = {"obstacles": np.array(OBS)}
    out.update({"kin_" + n: v for n, v in k.items()})
    out.update(kin_H=sk["H"][:8], kin_g=sk["g"][:8], kin_u_star=sk["u_star"], kin_x_star=sk["x_star"])
    out.update({"dyn_" + n: v for n, v in d.items()})
    out.update(dyn_u_star=R["u_star"], dyn_x_star=R["x_star"])
    np.savez_compressed(os.path.join(HERE, "obs_golden.npz"), **out)


if __name__ == "__main__":
    main()
