"""Parity of the dynamic SQP kernel vs the oracle as a function of SQP iterations
and interior-point tolerance (GPU box).  usage: python scripts/dyn_sweep.py"""
import copy
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]

from oracle import dyn_sqp as D  # noqa: E402
from oracle import models as M  # noqa: E402
from vcmpc import Context, _abi  # noqa: E402
from vcmpc.config import load_config, make_params  # noqa: E402

g = dict(np.load(os.path.join(ROOT, "tests", "golden", "dyn_sqp_golden.npz")))
B = len(g["x0"])
S = np.array([1000.0, 1.0])
p = M.dyn_params_from_config(load_config("dynamic_car"))
f64 = {k: g[k].astype(np.float64) for k in ("x0", "ubar", "kappa", "ds")}
for prox in [float(a) for a in (sys.argv[1:] or ["0.1"])]:
    for iters in (1, 3):
        for tol in (1e-5, 1e-6):
            cfg = copy.deepcopy(load_config("dynamic_mpc"))
            cfg["qp"]["sqp_iters"] = iters
            cfg["qp"]["tol"] = tol
            cfg["qp"]["prox"] = prox
            cfg["qp"]["max_iter"] = 80
            W = D.dyn_weights(cfg)
            ref = D.dyn_sqp_solve(f64["x0"], f64["ubar"], f64["kappa"], f64["ds"], p, W, "linear")["u_star"]
            ctx = Context(model=_abi.VC_MODEL_DYNAMIC, N=40, max_batch=B, dtype=_abi.VC_F32,
                          params=make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=cfg, tyre="linear"))
            ub = g["ubar"].copy()
            u0, xs, us, st, it, dg = ctx.solve(g["x0"], g["kappa"], g["ds"], ub, diag=True)
            err = np.abs((us - ref) / S).max(axis=(1, 2))
            print(f"prox {prox:g} sqp {iters} tol {tol:g}: solved {int((st == 0).sum())}/{B} iters {int(it.max())} "
                  f"max err {err.max():.2e} median {np.median(err):.2e} worst {np.argsort(err)[-3:].tolist()}", flush=True)
