"""kin_ltv_kernel<20> launch time against the batch size (one wave per problem, one wave per
SIMD, 1,024 SIMDs): B <= 1024 leaves SIMDs idle, so the launch time there is the slowest
problem's time plus the launch's fixed cost; beyond 1024 problems queue per SIMD and the time
per problem approaches the mean.  Also times B = 1024 made of one problem repeated (no
iteration tail: every wave does the same work) for the median-iteration problem and the
slowest one.  usage: python scripts/kin_b_sweep.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))
from vcmpc import Context, _abi  # noqa: E402
from vcmpc.config import load_config, make_params  # noqa: E402
from vcmpc.workload import kinematic_batch  # noqa: E402

dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
params = make_params(kin_car=load_config("kinematic_car"), kin_mpc=load_config("kinematic_mpc"))
BMAX = 16384
ctx = Context(model=_abi.VC_MODEL_KINEMATIC, N=20, max_batch=BMAX, device=0, params=params)
ctx.set_stream(stream.cuda_stream)


def time_batch(d, reps=20):
    B = len(d["x0"])
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items()}
    ub0 = t["ubar"].clone()
    xbar = torch.empty((B, 21, 6), dtype=torch.float64, device=dev)
    u0 = torch.empty((B, 2), dtype=torch.float64, device=dev)
    st = torch.empty((B,), dtype=torch.int32, device=dev)
    it = torch.empty((B,), dtype=torch.int32, device=dev)
    ms = []
    with torch.cuda.stream(stream):
        for r in range(reps + 2):
            t["ubar"].copy_(ub0)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            ctx.solve(t["x0"], t["kappa"], t["ds"], t["ubar"], xbar, u0, st, it)
            b.record(stream)
            b.synchronize()
            if r >= 2:
                ms.append(a.elapsed_time(b))
    return float(np.median(ms)), it.cpu().numpy(), st.cpu().numpy()


full = kinematic_batch(BMAX, seed=31)
for B in (64, 256, 512, 1024, 2048, 4096, 8192, 16384):
    d = {k: v[:B] for k, v in full.items()}
    ms, it, st = time_batch(d)
    print(f"B={B:6d}: kernel {ms:.4f} ms  {B / ms * 1e3 / 1e6:.3f} M solves/s  per-problem {ms / B * 1e3:.3f} us  "
          f"iters mean {it.mean():.2f} max {it.max()} solved {(st == 0).mean():.4f}", flush=True)

c2 = {k: v[:1024] for k, v in full.items()}
_, it, _ = time_batch(c2, reps=1)
for name, b in (("median", int(np.argsort(it)[len(it) // 2])), ("slowest", int(np.argmax(it)))):
    d = {k: np.repeat(v[b:b + 1], 1024, axis=0) for k, v in c2.items()}
    ms, it2, _ = time_batch(d)
    print(f"B=1024 x problem {b} ({name}, {it[b]} iterations): kernel {ms:.4f} ms", flush=True)
ctx.close()
