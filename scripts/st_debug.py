"""GPU diagnostic for the fp64 single-track SQP kernel: status / diagnostics per problem and
the first SQP iteration's step against the oracle's exact QP, for one tyre and horizon.

    python scripts/st_debug.py [fiala|linear] [N]
"""
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

tyre = sys.argv[1] if len(sys.argv) > 1 else "fiala"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 40
cfg = load_config("dynamic_mpc" if N == 40 else "singletrack_mpc")
W = D.dyn_weights(cfg)
p = M.dyn_params_from_config(load_config("dynamic_car"))
d = {k: v.astype(np.float64) for k, v in dynamic_batch(6, N=N, seed=100 + N, tyre=tyre).items()}
for sq in (1, 3):
    c2 = dict(cfg)
    c2["qp"] = dict(cfg["qp"], sqp_iters=sq)
    W2 = dict(W, sqp_iters=sq)
    ref = D.dyn_sqp_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], p, W2, tyre)
    prm = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=c2, tyre=tyre)
    with Context(model=_abi.VC_MODEL_DYNAMIC, N=N, max_batch=8, dtype=_abi.VC_F64, params=prm) as ctx:
        u0, xs, us, st, it, dg = ctx.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
    err = np.abs(us - ref["u_star"]).max(axis=(1, 2))
    print(f"{tyre} N={N} sqp_iters={sq}: status {st.tolist()} iters {it.tolist()}")
    print(f"   diag res {dg[:, 0]} mu {dg[:, 1]} flags {dg[:, 2]} itmax {dg[:, 3]}")
    print(f"   max |u* - u*_oracle| per problem {err}")
    print(f"   xs finite {np.isfinite(xs).all()}, us range Fx {us[..., 0].min():.1f}..{us[..., 0].max():.1f}")
