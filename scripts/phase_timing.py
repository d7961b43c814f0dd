"""Per-phase timing of the fused kernel on the GPU: condense only (vc_condense),
then the solve with the interior point capped at k iterations, with and without
the polish.  Differences give the cost of one interior-point iteration and of
the polish.  Prints one line per variant (ms per launch, B problems)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))
from vcmpc import Context, make_params  # noqa: E402
from vcmpc.config import load_config  # noqa: E402
from vcmpc.workload import kinematic_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dev = torch.device("cuda:0")
d = kinematic_batch(B, seed=31)
t = {k: torch.from_numpy(v).to(dev) for k, v in d.items()}
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
kc, kcfg = load_config("kinematic_car"), load_config("kinematic_mpc")


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def ctx_with(max_iter, polish):
    p = make_params(kin_car=kc, kin_mpc=kcfg)
    p.qp.max_iter = max_iter
    p.qp.polish = polish
    c = Context(N=20, max_batch=B, params=p)
    c.set_stream(stream.cuda_stream)
    return c


c = ctx_with(40, 10)
print(f"B={B} condense-only: {timed(lambda: c.condense(t['x0'], t['ubar'], t['kappa'], t['ds'])):.4f} ms")
for mi, pol in ((0, 0), (1, 0), (2, 0), (4, 0), (8, 0), (40, 0), (40, 10)):
    c = ctx_with(mi, pol)
    ub = t["ubar"].clone()
    ms = timed(lambda: c.solve(t["x0"], t["kappa"], t["ds"], ub.copy_(t["ubar"])))
    _, _, _, st, it = c.solve(t["x0"], t["kappa"], t["ds"], ub.copy_(t["ubar"]))
    print(f"B={B} max_iter={mi:2d} polish={pol:2d}: {ms:.4f} ms  iters mean {it.float().mean().item():.2f} "
          f"solved {(st == 0).float().mean().item():.3f}")
