"""GPU diagnostic: per-section s_memtime cycles of the cascaded SQP kernel
(csrc/casc_sqp.hip built with -DVC_TIMING, `make -C vehicle-control_amd/csrc timing`,
loaded through VCMPC_LIB=.../libvcmpc_timing.so).  Prints cycles per problem per
section and per interior-point iteration."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["VCMPC_LIB"] = os.path.join(ROOT, "vehicle-control_amd", "vcmpc", "libvcmpc_timing.so")
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))
import numpy as np  # noqa: E402

from vcmpc import Context, _abi  # noqa: E402
from vcmpc.config import load_config, make_params  # noqa: E402
from vcmpc.workload import cascaded_batch  # noqa: E402

NAMES = ["predict", "linearize", "condense", "setup", "local+rows", "dual resid", "W assembly", "build",
         "cholesky", "tri solves", "directions", "update", "total"]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
d = cascaded_batch(B, seed=3)
p = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=load_config("cascaded_mpc"), tyre="fiala")
c = Context(model=_abi.VC_MODEL_CASCADED, N=20, max_batch=B, dtype=_abi.VC_F64, params=p)
diag = np.zeros((B, 4 + len(NAMES)))
u0, xs, us, st, it, dg = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=diag)
ipm = it.mean()
print(f"B={B} solved {(st == 0).mean():.3f} IPM iterations/problem mean {ipm:.1f} max {it.max()}")
cyc = dg[:, 4:]
for i, nm in enumerate(NAMES):
    print(f"  {nm:12s} {cyc[:, i].mean():12.0f} cycles/problem  {100 * cyc[:, i].mean() / cyc[:, -1].mean():5.1f} %"
          f"  per IPM iteration {cyc[:, i].mean() / ipm:10.0f}")
