"""A/B of the single-track SQP kernel's active-set polish (st_sqp.hip ST_POLISH / ST_AL_*): on the bench's
N = 60 batch (4,096, seed 31, singletrack_mpc.yaml) and C3 (N = 40, dynamic_mpc.yaml), count the solved
problems whose QPs were not all certified by the polish (diag[2] bit 4), the kernel time at the configs'
SQP iterations, and the KKT certificate (oracle/certify.py) of the first QP of every unpolished problem.
Each library in its own child process (VCMPC_LIB is read at import).
usage: python scripts/st_polish_ab.py lib0.so lib1.so ..."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    os.environ["VCMPC_LIB"] = lib
    sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]
    import torch
    from oracle import certify as CF
    from oracle import dyn_sqp as D
    from oracle import models as M
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.workload import dynamic_batch
    res = {"lib": os.path.basename(lib)}
    pcar = M.dyn_params_from_config(load_config("dynamic_car"))
    for name, N, cfg_name in (("n60", 60, "singletrack_mpc"), ("c3", 40, "dynamic_mpc")):
        d = {k: v.astype(np.float64) for k, v in dynamic_batch(4096, N=N, seed=31).items()}
        cfg = load_config(cfg_name)
        out = {}
        for k in (1, int(cfg["qp"]["sqp_iters"])):
            ck = dict(cfg, qp=dict(cfg["qp"], sqp_iters=k))
            p = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=ck, tyre="linear")
            with Context(model=_abi.VC_MODEL_DYNAMIC, N=N, max_batch=4096, dtype=_abi.VC_F64, params=p) as c:
                t = {kk: torch.from_numpy(v).cuda() for kk, v in d.items()}
                ms = []
                for r in range(4):
                    ub = t["ubar"].clone()
                    torch.cuda.synchronize()
                    t0 = torch.cuda.Event(enable_timing=True); t1 = torch.cuda.Event(enable_timing=True)
                    c.set_stream(torch.cuda.current_stream().cuda_stream)
                    t0.record()
                    o = c.solve(t["x0"], t["kappa"], t["ds"], ub, diag=True)
                    t1.record()
                    torch.cuda.synchronize()
                    if r:
                        ms.append(t0.elapsed_time(t1))
            st, dg, us = o[3].cpu().numpy(), o[5].cpu().numpy(), o[2].cpu().numpy()
            unpol = np.nonzero((st == 0) & ((dg[:, 2].astype(int) & 4) == 0))[0]
            out[f"sqp{k}"] = {"kernel_ms": float(np.mean(ms)), "solved": float((st == 0).mean()),
                              "unpolished": int(len(unpol)), "unpolished_idx": unpol[:8].tolist()}
            if k == 1 and len(unpol):
                W = D.dyn_weights(cfg)
                sub = {kk: v[unpol] for kk, v in d.items()}
                Q = D.dyn_qp(sub["x0"], sub["ubar"], sub["kappa"], sub["ds"], pcar, W, "linear")
                sc = CF.sqp_scale("dyn", N, N)
                z = ((us[unpol] - sub["ubar"]) / sc).reshape(len(unpol), -1)
                cert = CF.certify(Q["H"], Q["g"], Q["C"], Q["d"], z)
                out["sqp1"]["unpolished_stat_over_scale"] = (cert["stat"] / cert["scale"])[:8].tolist()
        res[name] = out
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        for lib in sys.argv[1:]:
            subprocess.run([sys.executable, __file__, "--child", lib], check=True, timeout=400)
