"""Kernel-vs-oracle first-QP internals for one C3 problem (GPU box).
usage: python scripts/dyn_debug2.py B seed index [polish]"""
import copy
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]

from oracle import dyn_sqp as D  # noqa: E402
from oracle import models as M  # noqa: E402
from oracle import qp as QP  # noqa: E402
from vcmpc import Context, _abi  # noqa: E402
from vcmpc.config import load_config, make_params  # noqa: E402
from vcmpc.workload import dynamic_batch  # noqa: E402

Bw, seed, b = (int(a) for a in sys.argv[1:4])
cfg = copy.deepcopy(load_config("dynamic_mpc"))
cfg["qp"]["sqp_iters"] = 1
if len(sys.argv) > 4:
    cfg["qp"]["polish"] = int(sys.argv[4])
W = D.dyn_weights(cfg)
p = M.dyn_params_from_config(load_config("dynamic_car"))
d = dynamic_batch(Bw, seed=seed)
one = {k: np.ascontiguousarray(v[b:b + 1]) for k, v in d.items()}
ctx = Context(model=_abi.VC_MODEL_DYNAMIC, N=40, max_batch=4, dtype=_abi.VC_F32,
              params=make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=cfg, tyre="linear"))
r = ctx.solve_debug(one["x0"], one["kappa"], one["ds"], one["ubar"].copy())
f = {k: v.astype(np.float64) for k, v in one.items()}
Q = D.dyn_qp(f["x0"], f["ubar"], f["kappa"], f["ds"], p, W, "linear")
H, g, C, dd = Q["H"][0], Q["g"][0], Q["C"][0], Q["d"][0]
s0 = np.maximum(dd, 1.0)
Mo = H + C.T @ (C / s0[:, None])
n = 80
low = np.tril(np.ones((n, n), bool))
rel = lambda a, o: np.abs(a - o).max() / np.abs(o).max()
print(f"g rel {rel(r['g'][0], g):.2e}  M rel {rel(r['M'][0][low], Mo[low]):.2e}")
sol = QP.solve_qp_batch(Q["H"], Q["g"], Q["C"], Q["d"])
dz_k = ((r["ubar"][0] - one["ubar"][0]) / np.array([1000.0, 1.0])).reshape(-1)
print(f"final dz err {np.abs(dz_k - sol['z'][0]).max():.2e}   status {r['status']} iters {r['iters']}")
# what QP does the kernel's answer solve?  KKT of the kernel dz on the oracle QP
lam = sol["lam"][0]
act = lam > 1e-9
print("oracle active", int(act.sum()), " kernel dz: max violation", float((C @ dz_k - dd).max()),
      " stationarity w/ oracle multipliers", float(np.abs(H @ dz_k + g + C.T @ lam).max()))
e = np.abs(dz_k - sol["z"][0]); j = int(np.argmax(e))
print("worst column", j, "kernel", dz_k[j], "oracle", sol["z"][0][j])
