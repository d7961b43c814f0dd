"""Run the C2 sampler at a large batch through vc_solve_diag and dump the problems
that do not come back VC_SOLVED (or that disagree with... nothing: no oracle on the
box side here) into gpurun_out/diag_<tag>.npz for offline analysis with the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))

from vcmpc import Context  # noqa: E402
from vcmpc.config import load_config  # noqa: E402
from vcmpc.workload import kinematic_batch  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "x"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
seeds = [11, 31, 5]
out = {}
with Context(N=20, max_batch=B, kin_car=load_config("kinematic_car"), kin_mpc=load_config("kinematic_mpc")) as ctx:
    for sd in seeds:
        d = kinematic_batch(B, seed=sd)
        u0, xbar, ustar, st, it, dg = ctx.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
        bad = np.nonzero(st != 0)[0]
        flags = dg[:, 2].astype(int)
        print(f"seed {sd}: status counts {np.unique(st, return_counts=True)}, iters mean {it.mean():.2f} max {it.max()}, "
              f"polished {np.mean(flags & 4 > 0):.4f}, chol_fail {np.mean(flags & 1 > 0):.4f}, "
              f"pchol_fail {np.mean(flags & 8 > 0):.4f}, rounds mean {dg[:, 3].mean():.2f}")
        for i in bad[:10]:
            print("   bad", i, "st", st[i], "it", it[i], "diag", dg[i])
        for k, v in d.items():
            out[f"s{sd}_{k}"] = v[bad]
        out[f"s{sd}_idx"] = bad
        out[f"s{sd}_diag"] = dg[bad]
        out[f"s{sd}_ustar"] = ustar[bad]
        # unpolished-but-solved problems too (PDIP-only accuracy matters for parity)
        unp = np.nonzero((st == 0) & ((flags & 4) == 0))[0]
        out[f"s{sd}_unpol_idx"] = unp
        for k, v in d.items():
            out[f"s{sd}_unpol_{k}"] = v[unp[:64]]
        out[f"s{sd}_unpol_ustar"] = ustar[unp[:64]]
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", f"diag_{tag}.npz"), **out)
