"""A/B of kin_ric's Tapia active-set guess (KR_TAPIA): N = 50 batch of 1024 with
diagnostics -- kernel time, interior-point iterations, polish rounds used, polished fraction.
Each library in its own child process (VCMPC_LIB is read at import).
usage: python scripts/kr_tapia_ab.py lib0.so lib1.so"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    os.environ["VCMPC_LIB"] = lib
    sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))
    import torch
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.workload import kinematic_batch
    B, N = 1024, 50
    d = kinematic_batch(B, N=N, seed=31 + N)
    cfg = load_config("kinematic_mpc")
    cfg["qp"] = dict(cfg["qp"], solver=1)
    p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=cfg)
    dev = torch.device("cuda:0")
    t = {k: torch.from_numpy(v).to(dev) for k, v in d.items()}
    with Context(model=_abi.VC_MODEL_KINEMATIC, N=N, max_batch=B, params=p) as c:
        ms = []
        for r in range(13):
            ub = t["ubar"].clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = c.solve(t["x0"], t["kappa"], t["ds"], ub, diag=True)
            e1.record()
            torch.cuda.synchronize()
            if r >= 3:
                ms.append(e0.elapsed_time(e1))
        st, it, dg = (x.cpu().numpy() for x in (out[3], out[4], out[5]))
    fl = dg[:, 2].astype(int)
    print(json.dumps({"lib": os.path.basename(lib), "kernel_ms": float(np.mean(ms)), "solved": float((st == 0).mean()),
                      "iters_mean": float(it.mean()), "iters_max": int(it.max()),
                      "polish_rounds_mean": float(dg[:, 3].mean()), "polish_rounds_max": int(dg[:, 3].max()),
                      "polished": float(((fl & 4) > 0).mean()), "ipm_converged": float(((fl & 2) > 0).mean()),
                      "factor_fail": float(((fl & 1) > 0).mean()), "polish_factor_fail": float(((fl & 8) > 0).mean())}),
          flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        for lib in sys.argv[1:]:
            subprocess.run([sys.executable, __file__, "--child", lib], check=True, timeout=300)
