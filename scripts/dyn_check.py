"""GPU check of the dynamic SQP kernel against the oracle's golden vectors, plus a
timed C3 batch.  usage: python scripts/dyn_check.py [B]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]

from vcmpc import Context, _abi  # noqa: E402
from vcmpc.config import load_config, make_params  # noqa: E402
from vcmpc.workload import dynamic_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
g = dict(np.load(os.path.join(ROOT, "tests", "golden", "dyn_sqp_golden.npz")))
params = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=load_config("dynamic_mpc"), tyre="linear")
ctx = Context(model=_abi.VC_MODEL_DYNAMIC, N=40, max_batch=max(B, 64), dtype=_abi.VC_F32, params=params)
ub = g["ubar"].copy()
u0, xs, us, st, it, dg = ctx.solve(g["x0"], g["kappa"], g["ds"], ub, diag=True)
S = np.array([1000.0, 1.0])
err = np.abs((us - g["u_star"]) / S)
print("status", st.tolist())
print("iters", it.tolist())
print("diag", np.round(dg, 7).tolist()[:6])
print("|du*|/scale max per problem", np.round(err.max(axis=(1, 2)), 6).tolist())
print("x* rel err max", float(np.abs(xs - g["x_star"]).max()))
d = dynamic_batch(B, seed=11)
ub = d["ubar"].copy()
ctx.solve(d["x0"], d["kappa"], d["ds"], ub)  # warm-up
import torch
t = {k: torch.from_numpy(v).cuda() for k, v in d.items()}
u = t["ubar"].clone()
out = [torch.empty((B, 40, 8), dtype=torch.float32, device="cuda"), torch.empty((B, 2), dtype=torch.float32, device="cuda"),
       torch.empty(B, dtype=torch.int32, device="cuda"), torch.empty(B, dtype=torch.int32, device="cuda")]
ctx.set_stream(torch.cuda.current_stream().cuda_stream)
for rep in range(3):
    u.copy_(t["ubar"])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.solve(t["x0"], t["kappa"], t["ds"], u, xbar=out[0], u0=out[1], status=out[2], iters=out[3])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"B={B}: {dt*1e3:.2f} ms  {B/dt:.0f} solves/s  solved {(out[2]==0).float().mean().item():.3f} "
          f"iters mean {out[3].float().mean().item():.1f}")
