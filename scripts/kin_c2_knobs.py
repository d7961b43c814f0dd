"""C2 kernel (kin_ltv_kernel<20>, B = 1024) under different interior-point knobs: kernel time
(HIP events on the context stream), iterations, and |u* - u*_oracle| against the exact oracle QP
(oracle/ltv_qp.py) on the same problems -- what each knob costs in accuracy.

    python scripts/kin_c2_knobs.py [--batch 1024] [--reps 20] "tol=1e-10 polish=10" "tol=1e-8 polish=10" ...
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--seed", type=int, default=31)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import torch
    from oracle import ltv_qp as Q
    from vcmpc import Context, make_params
    from vcmpc.config import load_config
    from vcmpc.workload import kinematic_batch
    dev = torch.device("cuda:0")
    B, N = a.batch, 20
    d = kinematic_batch(B, seed=a.seed)
    cfg0 = load_config("kinematic_mpc")
    ref = Q.kin_ltv_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], 2.5, Q.kin_weights(cfg0))["u_star"]
    t = {k: torch.from_numpy(v).to(dev) for k, v in d.items()}
    stream = torch.cuda.Stream(dev)
    for var in a.variants:
        kv = {k: float(v) if ("." in v or "e" in v) else int(v) for k, v in (x.split("=") for x in var.split())}
        cfg = load_config("kinematic_mpc")
        cfg["qp"] = dict(cfg["qp"], **kv)
        p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=cfg)
        with Context(N=N, max_batch=B, params=p) as c:
            c.set_stream(stream.cuda_stream)
            xbar = torch.empty((B, N + 1, 6), dtype=torch.float64, device=dev)
            u0 = torch.empty((B, 2), dtype=torch.float64, device=dev)
            st = torch.empty((B,), dtype=torch.int32, device=dev)
            it = torch.empty((B,), dtype=torch.int32, device=dev)
            ub = t["ubar"].clone()
            ms = []
            for r in range(a.reps + 3):
                with torch.cuda.stream(stream):
                    ub.copy_(t["ubar"])
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                c.solve(t["x0"], t["kappa"], t["ds"], ub, xbar, u0, st, it)
                e1.record(stream)
                torch.cuda.synchronize(dev)
                if r >= 3:
                    ms.append(e0.elapsed_time(e1))
            u = ub.cpu().numpy()
            s_, i_ = st.cpu().numpy(), it.cpu().numpy()
        err = np.abs(u - ref).max(axis=(1, 2))
        print(json.dumps({"variant": var, "kernel_ms": float(np.mean(ms)), "kernel_ms_min": float(np.min(ms)),
                          "solves_per_s": B / (np.mean(ms) * 1e-3), "solved": float((s_ == 0).mean()),
                          "iters_mean": float(i_.mean()), "iters_max": int(i_.max()),
                          "err_max": float(err.max()), "err_p99": float(np.percentile(err, 99)),
                          "n_err_gt_1e-5": int((err > 1e-5).sum())}), flush=True)


if __name__ == "__main__":
    main()
