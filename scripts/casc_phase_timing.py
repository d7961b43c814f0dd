"""GPU diagnostic: where the cascaded SQP kernel's time goes (csrc/casc_sqp.hip).
Times vc_condense (predict + linearize + condense + setup + one normal-matrix build)
and vc_solve with 1 SQP iteration and qp.max_iter in {1, 2, 4, 8}: the slope is the
cost of one interior-point iteration (build + Cholesky + 2 x 2 triangular sweeps +
the row / stage passes)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))
from vcmpc import Context, _abi  # noqa: E402
from vcmpc.config import load_config, make_params  # noqa: E402
from vcmpc.workload import cascaded_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dev = torch.device("cuda", 0)
stream = torch.cuda.Stream(dev)   # a real stream: the null stream's handle 0 means "the context's own"
torch.cuda.set_stream(stream)
d = cascaded_batch(B, seed=3)
t = {k: torch.from_numpy(v).to(dev) for k, v in d.items()}
H = d["ubar"].shape[1]


def ctx_for(max_iter, sqp):
    cfg = load_config("cascaded_mpc")
    cfg["qp"] = dict(cfg["qp"], max_iter=max_iter, sqp_iters=sqp)
    p = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=cfg, tyre="fiala")
    c = Context(model=_abi.VC_MODEL_CASCADED, N=20, max_batch=B, dtype=_abi.VC_F64, params=p)
    c.set_stream(stream.cuda_stream)
    return c


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


c = ctx_for(80, 3)
print(f"B={B}  condense (predict+lin+condense+setup+1 build): "
      f"{timed(lambda: c.condense(t['x0'], t['ubar'], t['kappa'], t['ds'])):.3f} ms", flush=True)
for mi in (1, 2, 4, 8):
    c = ctx_for(mi, 1)
    ub = t["ubar"].clone()
    ms = timed(lambda: (ub.copy_(t["ubar"]), c.solve(t["x0"], t["kappa"], t["ds"], ub)))
    print(f"  sqp 1, max_iter {mi}: {ms:.3f} ms", flush=True)
c = ctx_for(80, 3)
ub = t["ubar"].clone()
r = None
ms = timed(lambda: (ub.copy_(t["ubar"]), c.solve(t["x0"], t["kappa"], t["ds"], ub)))
u0, xs, us, st, it = c.solve(t["x0"], t["kappa"], t["ds"], t["ubar"].clone())
print(f"  full (3 SQP, max_iter 80): {ms:.3f} ms, iters mean {it.float().mean().item():.1f} max {it.max().item()}, "
      f"solved {(st == 0).float().mean().item():.3f}", flush=True)
