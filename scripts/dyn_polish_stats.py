"""Polish statistics of the dynamic SQP kernel on a fresh C3 batch vs the oracle
(GPU box).  usage: python scripts/dyn_polish_stats.py [B] [sqp_iters] [polish]"""
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
from vcmpc.workload import dynamic_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 48
cfg = copy.deepcopy(load_config("dynamic_mpc"))
if len(sys.argv) > 2:
    cfg["qp"]["sqp_iters"] = int(sys.argv[2])
if len(sys.argv) > 3:
    cfg["qp"]["polish"] = int(sys.argv[3])
if len(sys.argv) > 4:
    cfg["qp"]["tol"] = float(sys.argv[4])
W = D.dyn_weights(cfg)
p = M.dyn_params_from_config(load_config("dynamic_car"))
d = dynamic_batch(B, seed=8)
ctx = Context(model=_abi.VC_MODEL_DYNAMIC, N=40, max_batch=B, dtype=_abi.VC_F32,
              params=make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=cfg, tyre="linear"))
ub = d["ubar"].copy()
u0, xs, us, st, it, dg = ctx.solve(d["x0"], d["kappa"], d["ds"], ub, diag=True)
f = {k: v.astype(np.float64) for k, v in d.items()}
ref = D.dyn_sqp_solve(f["x0"], f["ubar"], f["kappa"], f["ds"], p, W, "linear")
err = np.abs((us - ref["u_star"]) / np.array([1000.0, 1.0])).max(axis=(1, 2))
npol = dg[:, 2].astype(int) >> 4
print(f"cfg sqp {cfg['qp']['sqp_iters']} polish {cfg['qp']['polish']} tol {cfg['qp']['tol']}")
print("status", np.bincount(st, minlength=3).tolist(), "polished QPs per problem", np.bincount(npol).tolist())
print(f"err max {err.max():.2e} median {np.median(err):.2e}; err where all polished max "
      f"{err[npol == cfg['qp']['sqp_iters']].max() if (npol == cfg['qp']['sqp_iters']).any() else -1:.2e}")
bad = np.argsort(err)[-5:]
for b in bad:
    print(f"  problem {b}: err {err[b]:.2e} polished {npol[b]} iters {it[b]} res {dg[b, 0]:.1e} mu {dg[b, 1]:.1e} "
          f"oracle polished {[bool(h['polished'][b]) for h in ref['hist']]}")
