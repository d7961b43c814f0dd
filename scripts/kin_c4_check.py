"""Solve the bench's C4 kinematic problem set (65536 problems, bench.py:c4_shard) once with the
library VCMPC_LIB points at and report status / iteration statistics, the non-solved
problems' indices and the oracle's verdict on them (certified optimum or infeasible).

    VCMPC_LIB=... python scripts/kin_c4_check.py [--total 65536] [--save out.npz]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total", type=int, default=65536)
    ap.add_argument("--seed", type=int, default=31)
    args = ap.parse_args()
    from bench import c4_shard
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    _, _, d = c4_shard(args.total, 0, 1, args.seed)
    p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=load_config("kinematic_mpc"))
    with Context(N=20, max_batch=args.total, params=p, dtype=_abi.VC_F64) as c:
        u0, xs, us, st, it, dg = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
    print(f"lib {_abi.LIB_PATH}: solved {np.mean(st == 0):.6f}, iterations mean {it.mean():.3f} max {it.max()}, "
          f"histogram tail {np.bincount(it)[12:].tolist()}")
    bad = np.nonzero(st != 0)[0]
    print("non-solved:", [(int(b), int(st[b]), int(it[b]), dg[b].tolist()) for b in bad[:10]])
    if len(bad):
        from oracle.ltv_qp import kin_ltv_solve, kin_weights
        W = kin_weights(load_config("kinematic_mpc"))
        sub = {k: v[bad] for k, v in d.items()}
        ref = kin_ltv_solve(sub["x0"], sub["ubar"], sub["kappa"], sub["ds"], 2.5, W)
        print("oracle on them: pfeas", ref["kkt"]["pfeas"].tolist(), "polished", ref["polished"].tolist())
        print("kernel u* vs oracle (scaled max):", np.abs(us[bad] - ref["u_star"]).max(axis=(1, 2)).tolist())


if __name__ == "__main__":
    main()
