"""Trace the stagewise kinematic kernel on single problems: re-run with max_iter = 1, 2, ...
(polish off) and print the kernel's residual / mu next to the numpy prototype's
(scripts/kin_riccati_proto.py) at the same iteration.

    python scripts/kin_ric_trace.py [--N 50] [--batch 8192] [--seed 77] [--index 6373]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd"), os.path.join(ROOT, "scripts")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=50)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--seed", type=int, default=77)
    ap.add_argument("--index", type=int, nargs="+", default=[6373])
    args = ap.parse_args()
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.workload import kinematic_batch
    d = kinematic_batch(args.batch, N=args.N, seed=args.seed)
    d = {k: np.ascontiguousarray(v[args.index]) for k, v in d.items()}
    np.set_printoptions(precision=3, linewidth=160)
    for max_iter, polish in [(i, 0) for i in range(1, 16)] + [(40, 10)]:
        cfg = load_config("kinematic_mpc")
        cfg["qp"] = dict(cfg.get("qp") or {}, solver=1, max_iter=max_iter, polish=polish)
        p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=cfg)
        with Context(model=_abi.VC_MODEL_KINEMATIC, N=args.N, max_batch=len(args.index), dtype=_abi.VC_F64,
                     params=p) as c:
            u0, xs, us, st, it, dg = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
        print(f"max_iter {max_iter:2d} polish {polish}: status {st} iters {it} diag {dg.ravel()}", flush=True)


if __name__ == "__main__":
    main()
