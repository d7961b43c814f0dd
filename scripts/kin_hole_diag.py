"""Round-6 diagnosis: the two C4 problems (c4_shard seed 31: 6021, 9204) that a kin_ltv build with the
interior point's step fraction at 0.998 (KIN_STEP_F) reports solved but off the certified optimum.
Prints status, iterations and the diag flags (1 IPM factorisation failed, 2 IPM converged, 4 polish
certified, 8 polish factorisation failed; rounds) for the library in VCMPC_LIB.
usage: VCMPC_LIB=... python scripts/kin_hole_diag.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]
from vcmpc import Context, _abi  # noqa: E402
from vcmpc.config import load_config  # noqa: E402
from vcmpc.workload import c4_shard  # noqa: E402

d = c4_shard(65536, 0, 1, 31)[2]
idx = [6021, 9204]
sub = {k: np.ascontiguousarray(v[idx]) for k, v in d.items()}
with Context(model=_abi.VC_MODEL_KINEMATIC, N=20, max_batch=8, kin_car=load_config("kinematic_car"),
             kin_mpc=load_config("kinematic_mpc")) as c:
    u0, xb, us, st, it, dg = c.solve(sub["x0"], sub["kappa"], sub["ds"], sub["ubar"].copy(), diag=True)
for j, b in enumerate(idx):
    print(f"{os.path.basename(os.environ.get('VCMPC_LIB', 'libvcmpc.so'))} problem {b}: status {int(st[j])} iters {int(it[j])} "
          f"res {dg[j, 0]:.2e} mu {dg[j, 1]:.2e} flags {int(dg[j, 2])} rounds {int(dg[j, 3])} u*[0:4] {np.round(us[j].ravel()[:4], 6)}")
