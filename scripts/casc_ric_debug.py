"""Debug the stagewise cascaded kernel on a few problems: per tail length M, 1 SQP iteration with
max_iter = 1, 2, 4, 80: status / diag, and x* = rollout(u*) against the oracle's prediction of
the same u* (checks the device rollout), u* against the oracle's one-iteration SQP.

    python scripts/casc_ric_debug.py [--M 15 25]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]

from oracle import casc_sqp as CS  # noqa: E402
from oracle import models as MD  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[15, 25, 35, 40])
    args = ap.parse_args()
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.workload import cascaded_batch
    p = MD.dyn_params_from_config(load_config("dynamic_car"))
    np.set_printoptions(precision=4, linewidth=180)
    for M in args.M:
        d = cascaded_batch(2, M=M, seed=400 + M)
        cfg = load_config("cascaded_mpc")
        cfg["horizon_pm"] = M
        W = CS.casc_weights(cfg)
        W1 = dict(W, sqp_iters=1)
        ref1 = CS.casc_sqp_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], p, W1, tyre="fiala")
        for mi in (1, 2, 4, 80):
            c2 = dict(cfg)
            c2["qp"] = dict(cfg["qp"], sqp_iters=1, max_iter=mi)
            prm = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=c2, tyre="fiala")
            with Context(model=_abi.VC_MODEL_CASCADED, N=20, max_batch=2, dtype=_abi.VC_F64, params=prm) as c:
                u0, xs, us, st, it, dg = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
            xs_o, xp_o = CS.casc_predict(d["x0"], us, d["kappa"], d["ds"], p, W, "fiala")
            xref = CS.pack_states(xs_o, xp_o)
            ex = np.abs(xs - xref).max(axis=(1, 2))
            eu = np.abs(us - ref1["u_star"]).max(axis=(1, 2))
            print(f"M={M} max_iter={mi}: status {st} iters {it} diag {dg.round(6).tolist()} "
                  f"|x* - predict(u*)| {ex} |u* - u*_oracle(1 SQP)| {eu}", flush=True)
            if mi == 1:
                bad = np.nonzero(~np.isfinite(xs[0]).all(axis=1) | (np.abs(xs[0] - xref[0]) > 1e-6).any(axis=1))[0]
                print(f"   rows of x* off the oracle prediction (problem 0): {bad[:10]}; x*[N-1..N+1]:\n"
                      f"{xs[0, 19:22]}\n   oracle:\n{xref[0, 19:22]}")


if __name__ == "__main__":
    main()
