"""Generate tests/golden/kin_nlp_obs_golden.npz: the reference kinematic NLP's own optimum WITH
the obstacle barrier on -- the reference's default kinematic controller
(config/controllers/kinematic.yaml: N = 50, obstacles: True; barrier kinematic_mpc.py:130-133).

Problems:
  N = 20: the 44 obstacle golden problems (tests/golden/obs_golden.npz: C2-sampler starts moved
          in front of ippodromo's obstacles, plus the hand-built edge cases);
  N = 50: 32 C2-sampler problems at kinematic.yaml's horizon, moved 1..14 m in front of a random
          ippodromo obstacle the same way (make_obs_golden.py `place`).
Obstacles: ippodromo's obstacle_data (config/environment/ippodromo.yaml).  The NLP is
oracle/kin_nlp.py's (scipy trust-constr + Newton on the KKT system, the reference's barrier
w_obs ds / (dist - r - 0.1) exactly, no margin floor, no proximal term), solved from the rollout
of the warm start and, where that does not converge, from the neutral guess u = 0.  Stored per
problem: U*, X*, the KKT certificate, the objective, `converged` (stat, pfeas < 1e-10) and the
smallest barrier margin min (dist - r - 0.1) along X* -- where it is above the build's margin
floor (0.05 m) the build's barrier equals the reference's near the optimum.

Run from the repo root (8 processes):  python tests/golden/make_kin_nlp_obs_golden.py
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

TOL = 1e-10
L = 2.5


def problems():
    from make_obs_golden import OBS, place
    from vcmpc.workload import kinematic_batch
    g = np.load(os.path.join(HERE, "obs_golden.npz"))
    p20 = {k: np.asarray(g["kin_" + k], np.float64) for k in ("x0", "kappa", "ds", "ubar")}
    rng = np.random.default_rng(50)
    d = kinematic_batch(32, N=50, seed=50)
    d["x0"] = place(d["x0"].copy(), rng, 2, 3, (1.0, 14.0))
    return OBS, {20: p20, 50: d}


def _solve(job):
    from threadpoolctl import threadpool_limits

    from oracle import kin_nlp as KN
    x0, kap, ds, ub, W = job
    N = len(kap)
    with threadpool_limits(limits=1):
        for k, u in enumerate((ub, np.zeros((N, 2)))):
            try:
                U, X, info = KN.solve_nlp(x0, u, kap, ds, L, W)
            except Exception as e:  # a start the barrier cannot be evaluated from
                info = dict(stat=np.inf, pfeas=np.inf, f=np.inf, status=-9, nit=0, refined=False, err=repr(e))
                U, X = np.full((N, 2), np.nan), np.full((N + 1, 6), np.nan)
            if info["stat"] < TOL and info["pfeas"] < TOL:
                break
    margin = np.inf
    if np.isfinite(X).all():
        for so, eo, r in W["obstacles"]:
            margin = min(margin, float(np.min(np.hypot(X[1:N, 2] - so, X[1:N, 3] - eo) - (r + 0.1))))
    return U, X, info, k, margin


def main():
    import multiprocessing as mp

    from oracle import ltv_qp as Q
    from vcmpc.config import load_config
    OBS, sets = problems()
    W = Q.kin_weights(load_config("kinematic_mpc"))
    W["obstacles"] = OBS
    out = {"obstacles": np.array(OBS), "tol": TOL}
    t0 = time.time()
    with mp.get_context("spawn").Pool(8) as pool:
        for N, d in sets.items():
            jobs = [(d["x0"][b], d["kappa"][b], d["ds"][b], d["ubar"][b], W) for b in range(len(d["x0"]))]
            res = pool.map(_solve, jobs, chunksize=1)
            B = len(jobs)
            U = np.stack([r[0] for r in res]); X = np.stack([r[1] for r in res])
            stat = np.array([r[2]["stat"] for r in res]); pfeas = np.array([r[2]["pfeas"] for r in res])
            fval = np.array([r[2]["f"] for r in res]); start = np.array([r[3] for r in res], np.int32)
            margin = np.array([r[4] for r in res])
            conv = (stat < TOL) & (pfeas < TOL)
            for b in range(B):
                print(f"N={N} {b:3d} start {start[b]} stat {stat[b]:.1e} pfeas {pfeas[b]:.1e} f {fval[b]:.6f} "
                      f"margin {margin[b]:.3f}", flush=True)
            print(f"N={N}: {int(conv.sum())} of {B} converged ({time.time() - t0:.0f} s)", flush=True)
            for k in ("x0", "kappa", "ds", "ubar"):
                out[f"n{N}_{k}"] = d[k]
            out.update({f"n{N}_u_nlp": U, f"n{N}_x_nlp": X, f"n{N}_stat": stat, f"n{N}_pfeas": pfeas,
                        f"n{N}_f": fval, f"n{N}_start": start, f"n{N}_converged": conv, f"n{N}_margin": margin})
    np.savez_compressed(os.path.join(HERE, "kin_nlp_obs_golden.npz"), **out)


if __name__ == "__main__":
    sys.path.insert(0, HERE)
    main()
