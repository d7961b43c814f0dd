"""Diagnose a non-solved problem of the N = 60 single-track leg that the oracle certifies
feasible (bench seed 31, B = 4096; index from tests/test_gpu_st_sqp.py): kernel status /
residual / mu / flags at the contract's max_iter and at larger caps, against the oracle.

    python scripts/st_n60_case.py [--idx 2334]
"""
import argparse
import copy
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--idx", type=int, nargs="+", default=[2334, 828])
    args = ap.parse_args()
    from oracle import dyn_sqp as D
    from oracle import models as Mo
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.workload import dynamic_batch
    N = 60
    d = {k: v.astype(np.float64) for k, v in dynamic_batch(4096, N=N, seed=31).items()}
    sub = {k: np.ascontiguousarray(v[args.idx]) for k, v in d.items()}
    base = load_config("singletrack_mpc")
    p = Mo.dyn_params_from_config(load_config("dynamic_car"))
    ref = D.dyn_sqp_solve(sub["x0"], sub["ubar"], sub["kappa"], sub["ds"], p, D.dyn_weights(base), "linear")
    for h_i, h in enumerate(ref["hist"]):
        print(f"oracle SQP iteration {h_i}: QP iters {h['iters'].tolist()} pfeas {h['kkt']['pfeas']} "
              f"stat {h['kkt']['stat']}")
    for mi in (60, 120, 400):
        cfg = copy.deepcopy(base)
        cfg["qp"] = dict(cfg["qp"], max_iter=mi)
        prm = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=cfg, tyre="linear")
        with Context(model=_abi.VC_MODEL_DYNAMIC, N=N, max_batch=8, dtype=_abi.VC_F64, params=prm) as c:
            u0, xs, us, st, it, dg = c.solve(sub["x0"], sub["kappa"], sub["ds"], sub["ubar"].copy(), diag=True)
        err = np.abs((us - ref["u_star"]) / np.array([1000.0, 1.0])).max(axis=(1, 2))
        print(f"max_iter {mi}: status {st.tolist()} iters {it.tolist()} diag (res, mu, flags, it_max) "
              f"{np.round(dg[:, :4], 14).tolist()} scaled err vs oracle {err.tolist()}")


if __name__ == "__main__":
    main()
