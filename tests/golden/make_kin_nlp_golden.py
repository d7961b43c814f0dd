"""Generate tests/golden/kin_nlp_golden.npz: the reference NLP's own optimum on the C2 golden
problems (VERDICT r03 "next" item 3).

For every problem of tests/golden/kin_ltv_golden.npz (x0, kappa, ds, warm start ubar) this
solves the multiple-shooting NLP of controllers/mpc/kinematic_mpc.py:15-158 directly with
oracle/kin_nlp.py (scipy trust-constr + Newton on the KKT system; no proximal term, no trust
region, every `if_else` exact) from the rollout of the warm start, and from the neutral guess
u = 0 where that does not converge.  Stored: U*, X*, the KKT certificate (relative
stationarity, primal feasibility), the objective and a `converged` flag (stat < 1e-10, pfeas
< 1e-10).  tests/test_gpu_kin_nlp.py compares the build's kinematic SQP iterated to
convergence (vc_qp.kin_sqp) with U*; tests/test_oracle_kin_nlp.py re-checks the certificates.

Parity status: the reference's IPOPT cannot run here; this is the same NLP solved by
an independent method, so agreement ties the build's SQP fixed point to the reference's
optimum, not to IPOPT's iterates.

Run from the repo root:  python tests/golden/make_kin_nlp_golden.py
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))

from oracle import kin_nlp as KN  # noqa: E402
from oracle import ltv_qp as Q  # noqa: E402
from vcmpc.config import load_config  # noqa: E402

TOL = 1e-10


def main():
    g = np.load(os.path.join(HERE, "kin_ltv_golden.npz"))
    W = Q.kin_weights(load_config("kinematic_mpc"))
    W["obstacles"] = []
    L = float(g["L"])
    B, N = g["ubar"].shape[:2]
    U = np.zeros((B, N, 2))
    X = np.zeros((B, N + 1, 6))
    stat, pfeas, fval = np.zeros(B), np.zeros(B), np.zeros(B)
    start = np.zeros(B, np.int32)      # 0: rollout of the warm start, 1: neutral guess
    t0 = time.time()
    for b in range(B):
        for k, ub in enumerate((g["ubar"][b], np.zeros((N, 2)))):
            Ub, Xb, info = KN.solve_nlp(g["x0"][b], ub, g["kappa"][b], g["ds"][b], L, W)
            if info["stat"] < TOL and info["pfeas"] < TOL:
                break
        U[b], X[b] = Ub, Xb
        stat[b], pfeas[b], fval[b], start[b] = info["stat"], info["pfeas"], info["f"], k
        print(f"{b:3d} start {k} status {info['status']} nit {info['nit']:4d} refined {info['refined']} "
              f"stat {info['stat']:.1e} pfeas {info['pfeas']:.1e} f {info['f']:.6f}", flush=True)
    conv = (stat < TOL) & (pfeas < TOL)
    print(f"{int(conv.sum())} of {B} converged ({time.time() - t0:.0f} s)")
    np.savez_compressed(os.path.join(HERE, "kin_nlp_golden.npz"), u_nlp=U, x_nlp=X, stat=stat, pfeas=pfeas,
                        f=fval, start=start, converged=conv, tol=TOL)


if __name__ == "__main__":
    main()
