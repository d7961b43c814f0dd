"""Solve one C2-sampler batch on the GPU and save inputs + outputs (+ diagnostics)
to gpurun_out/solve_<tag>.npz for offline comparison with the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))
from vcmpc import Context  # noqa: E402
from vcmpc.config import load_config  # noqa: E402
from vcmpc.workload import kinematic_batch  # noqa: E402

tag, B, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
d = kinematic_batch(B, seed=seed)
with Context(N=20, max_batch=B, kin_car=load_config("kinematic_car"), kin_mpc=load_config("kinematic_mpc")) as ctx:
    u0, xbar, ustar, st, it, dg = ctx.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
    xroll = ctx.rollout(d["x0"], d["ubar"], d["kappa"], d["ds"])
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", f"solve_{tag}.npz"), **d, u0=u0, xstar=xbar, ustar=ustar, status=st,
         iters=it, diag=dg, xroll=xroll)
print("saved", B, "status", np.unique(st, return_counts=True))
