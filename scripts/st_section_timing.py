"""GPU diagnostic: per-section s_memtime cycles of the fp64 single-track SQP kernel
(csrc/st_sqp.hip) from the timing build (make -C vehicle-control_amd/csrc timing ->
libvcmpc_timing.so, diag[b][4 + slot]).  Prints cycles per problem (lane-0 clock of the
problem's wavefront) and per interior-point iteration, at B problems of the C3 sampler.

    VCMPC_LIB=vehicle-control_amd/vcmpc/libvcmpc_timing.so python scripts/st_section_timing.py [B] [N] [tyre]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))
os.environ.setdefault("VCMPC_LIB", os.path.join(ROOT, "vehicle-control_amd", "vcmpc", "libvcmpc_timing.so"))
from vcmpc import Context, _abi  # noqa: E402
from vcmpc.config import load_config, make_params  # noqa: E402
from vcmpc.workload import dynamic_batch  # noqa: E402

SLOTS = ["predict", "linearize", "setup", "residuals", "dual residual", "riccati factor", "lq solves (2)",
         "rhs + steps", "total"]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
N = int(sys.argv[2]) if len(sys.argv) > 2 else 40
TYRE = sys.argv[3] if len(sys.argv) > 3 else "linear"
cfg = load_config("dynamic_mpc" if N == 40 else "singletrack_mpc")
d = {k: v.astype(np.float64) for k, v in dynamic_batch(B, N=N, seed=3, tyre=TYRE).items()}
p = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=cfg, tyre=TYRE)
with Context(model=_abi.VC_MODEL_DYNAMIC, N=N, max_batch=B, dtype=_abi.VC_F64, params=p) as ctx:
    diag = np.zeros((B, 4 + len(SLOTS)))
    u0, xs, us, st, it, dg = ctx.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=diag)
cyc = dg[:, 4:]
tot = cyc[:, -1].mean()
iters = it.mean()
print(f"B={B} N={N} {TYRE}: solved {(st == 0).mean():.4f}, IPM iterations per problem {iters:.1f} (max {it.max()})")
print(f"{'section':<18}{'cycles/problem':>16}{'share':>9}{'per IPM iter':>14}")
for i, name in enumerate(SLOTS):
    c = cyc[:, i].mean()
    per = f"{c / iters:14.0f}" if 3 <= i <= 7 else " " * 14
    print(f"{name:<18}{c:16.0f}{100 * c / tot:8.1f}%{per}")
