"""Per-section cycle counts of the dynamic SQP kernel (timing build: make -C
vehicle-control_amd/csrc timing; runs libvcmpc_timing.so).  Prints the mean s_memtime
cycles per problem of each section.  usage: python scripts/dyn_section_timing.py [B]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))
os.environ.setdefault("VCMPC_LIB", os.path.join(ROOT, "vehicle-control_amd", "vcmpc", "libvcmpc_timing.so"))
from vcmpc import Context, _abi, make_params  # noqa: E402
from vcmpc.config import load_config  # noqa: E402
from vcmpc.workload import dynamic_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
names = ["predict", "linearize", "condense", "qp_setup", "residual", "build", "chol", "predictor", "corrector",
         "polish", "output", "total", "b:wblocks", "b:mfma+zero", "b:diag"]
dev = torch.device("cuda:0")
d = dynamic_batch(B, seed=31)
t = {k: torch.from_numpy(v).to(dev) for k, v in d.items()}
p = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=load_config("dynamic_mpc"), tyre="linear")
with Context(model=_abi.VC_MODEL_DYNAMIC, N=40, max_batch=B, dtype=_abi.VC_F32, params=p) as c:
    xbar = torch.empty((B, 40, 8), dtype=torch.float32, device=dev)
    u0 = torch.empty((B, 2), dtype=torch.float32, device=dev)
    st = torch.empty((B,), dtype=torch.int32, device=dev)
    it = torch.empty((B,), dtype=torch.int32, device=dev)
    dg = torch.zeros((B, 19), dtype=torch.float32, device=dev)
    c.set_stream(torch.cuda.current_stream().cuda_stream)
    for rep in range(2):
        u = t["ubar"].clone()
        ptr = lambda a: C.c_void_p(a.data_ptr())
        _abi.check(c.lib, c._h, c.lib.vc_solve_diag(c._h, B, ptr(t["x0"]), ptr(t["kappa"]), ptr(t["ds"]), ptr(xbar),
                                                    ptr(u), ptr(u0), ptr(st), ptr(it), ptr(dg), _abi.VC_DEVICE_PTRS))
        torch.cuda.synchronize()
    D = dg.cpu().numpy()
    itn = it.cpu().numpy()
    cyc = D[:, 4:4 + len(names)]
    print(f"B={B} solved {(st.cpu().numpy() == 0).mean():.3f} PDIP iterations/problem mean {itn.mean():.1f} "
          f"max {itn.max()}")
    tot = cyc[:, -1].mean()
    for i, nme in enumerate(names):
        print(f"  {nme:10s} {cyc[:, i].mean():12.0f} cycles/problem  {100 * cyc[:, i].mean() / tot:5.1f} %  "
              f"per PDIP iteration {cyc[:, i].mean() / max(itn.mean(), 1):9.0f}")
