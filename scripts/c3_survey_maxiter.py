"""C3 survey-range problems the kernel does not solve or stops early on (r06k: 610 max_iter; 1371 /
1802 stopped at a later QP): their status, diag and SQP iterates at the config's qp.max_iter and at
higher limits, against the oracle's own SQP.   python scripts/c3_survey_maxiter.py [probs ...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]


def main():
    from oracle import dyn_sqp as D
    from oracle import models as M
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.workload import dynamic_batch
    probs = [int(a) for a in sys.argv[1:]] or [610, 1371, 1802]
    d = {k: v.astype(np.float64) for k, v in dynamic_batch(4096, N=40, seed=31, ranges="survey").items()}
    sub = {k: np.ascontiguousarray(v[probs]) for k, v in d.items()}
    cfg = load_config("dynamic_mpc")
    p = M.dyn_params_from_config(load_config("dynamic_car"))
    ref = D.dyn_sqp_solve(sub["x0"], sub["ubar"], sub["kappa"], sub["ds"], p, D.dyn_weights(cfg), "linear")
    for mi in (60, 120, 240):
        ck = dict(cfg, qp=dict(cfg["qp"], max_iter=mi))
        params = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=ck, tyre="linear")
        with Context(model=_abi.VC_MODEL_DYNAMIC, N=40, max_batch=len(probs), dtype=_abi.VC_F64, params=params) as c:
            u0, xs, u, st, it, dg = c.solve(sub["x0"], sub["kappa"], sub["ds"], sub["ubar"].copy(), diag=True)
        err = np.abs(u - ref["u_star"]).max(axis=(1, 2))
        print(json.dumps({"max_iter": mi, "problems": probs, "status": st.tolist(), "ipm_iters": it.tolist(),
                          "diag": dg.tolist(), "u_err_vs_oracle_sqp": err.tolist()}), flush=True)


if __name__ == "__main__":
    main()
