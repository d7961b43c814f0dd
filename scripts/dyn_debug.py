"""Stage-by-stage check of the dynamic SQP kernel's first QP against the oracle
(GPU box).  usage: python scripts/dyn_debug.py"""
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
B = 4
cfgm = load_config("dynamic_mpc")
W = D.dyn_weights(cfgm)
p = M.dyn_params_from_config(load_config("dynamic_car"))
params = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=cfgm, tyre="linear")
ctx = Context(model=_abi.VC_MODEL_DYNAMIC, N=40, max_batch=64, dtype=_abi.VC_F32, params=params)
sl = slice(0, B)
r = ctx.solve_debug(g["x0"][sl].copy(), g["kappa"][sl].copy(), g["ds"][sl].copy(), g["ubar"][sl].copy())
f64 = {k: g[k][sl].astype(np.float64) for k in ("x0", "ubar", "kappa", "ds")}
Q = D.dyn_qp(f64["x0"], f64["ubar"], f64["kappa"], f64["ds"], p, W, "linear")
n = 80
for b in range(B):
    H, gg, C, d = Q["H"][b], Q["g"][b], Q["C"][b], Q["d"][b]
    s0 = np.maximum(d, 1.0)
    w = 1.0 / s0
    Mo = H + C.T @ (w[:, None] * C)
    rp = s0 - d
    rhs = -gg - C.T @ (w * rp)
    dz = np.linalg.solve(Mo, rhs)
    Mk = r["M"][b]
    low = np.tril(np.ones((n, n), bool))
    rel = lambda a, o: float(np.abs(a - o).max() / (np.abs(o).max() + 1e-30))
    print(f"problem {b}: g rel {rel(r['g'][b], gg):.2e}  M(lower) rel {rel(Mk[low], Mo[low]):.2e}  "
          f"rhs rel {rel(r['rhs'][b], rhs):.2e}  dz rel {rel(r['dz'][b], dz):.2e}")
    Y = np.triu(r["Y"][b])
    Minv = Y @ Y.T
    print(f"   Y check: |Y Y' M - I| = {np.abs(Minv @ Mo - np.eye(n)).max():.2e}   cond(M) = {np.linalg.cond(Mo):.2e}")
    if rel(Mk[low], Mo[low]) > 1e-4:
        e = np.abs(Mk - Mo) * low
        i, j = np.unravel_index(np.argmax(e), e.shape)
        print(f"   worst M entry ({i},{j}): kernel {Mk[i, j]:.6g} oracle {Mo[i, j]:.6g}")
    if rel(r['g'][b], gg) > 1e-4:
        j = np.argmax(np.abs(r['g'][b] - gg)); print(f"   worst g entry {j}: kernel {r['g'][b][j]:.6g} oracle {gg[j]:.6g}")
print("status", r["status"], "iters", r["iters"])
