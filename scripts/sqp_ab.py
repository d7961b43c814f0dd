"""A/B of SQP-kernel builds (scripts/build_kin_variants.sh with SRC=st_sqp / casc_ric): the bench legs'
kernel time (HIP events on the context stream) and u* of each library against the first one, each library
in its own child process (VCMPC_LIB is read at import).  Legs: `st60` = singletrack_n60_f64 (B = 4096,
N = 60, singletrack_mpc.yaml, linear tyre), `casc` = cascaded (B = 4096, 20 + 40, Fiala), `c3` (N = 40).
usage: python scripts/sqp_ab.py [--leg st60] [--reps R] lib1.so lib2.so ..."""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib, leg, reps, out):
    os.environ["VCMPC_LIB"] = lib
    sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))
    import torch
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.workload import cascaded_batch, dynamic_batch
    dev = torch.device("cuda:0")
    B = 4096
    if leg == "casc":
        d = cascaded_batch(B, seed=31)
        cfg, model, tyre, N = load_config("cascaded_mpc"), _abi.VC_MODEL_CASCADED, "fiala", 20
    else:
        N = 60 if leg == "st60" else 40
        d = {k: v.astype(np.float64) for k, v in dynamic_batch(B, N=N, seed=31).items()}
        cfg, model, tyre = load_config("singletrack_mpc" if leg == "st60" else "dynamic_mpc"), _abi.VC_MODEL_DYNAMIC, "linear"
    t = {k: torch.from_numpy(v).to(dev) for k, v in d.items()}
    p = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=cfg, tyre=tyre)
    stream = torch.cuda.Stream(dev)
    with Context(model=model, N=N, max_batch=B, dtype=_abi.VC_F64, params=p) as c:
        c.set_stream(stream.cuda_stream)
        NS = t["ubar"].shape[1]
        xbar = torch.empty((B, NS, 8), dtype=torch.float64, device=dev)
        u0 = torch.empty((B, 2), dtype=torch.float64, device=dev)
        st = torch.empty((B,), dtype=torch.int32, device=dev)
        it = torch.empty((B,), dtype=torch.int32, device=dev)
        ub = t["ubar"].clone()
        ms = []
        for r in range(reps + 1):
            with torch.cuda.stream(stream):
                ub.copy_(t["ubar"])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            c.solve(t["x0"], t["kappa"], t["ds"], ub, xbar, u0, st, it)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            if r >= 1:
                ms.append(e0.elapsed_time(e1))
        np.savez(out, u=ub.cpu().numpy(), st=st.cpu().numpy(), it=it.cpu().numpy(), ms=np.array(ms))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--leg", default="st60", choices=["st60", "casc", "c3"])
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--child", nargs=2)
    ap.add_argument("libs", nargs="*")
    a = ap.parse_args()
    if a.child:
        child(a.child[0], a.leg, a.reps, a.child[1])
        return
    ref = None
    for i, lib in enumerate(a.libs):
        out = f"/tmp/sqp_ab_{i}.npz"
        subprocess.run([sys.executable, __file__, "--leg", a.leg, "--reps", str(a.reps), "--child", lib, out],
                       check=True, timeout=600)
        z = np.load(out)
        if ref is None:
            ref = z
        r = {"leg": a.leg, "kernel_ms_mean": float(z["ms"].mean()), "kernel_ms_min": float(z["ms"].min()),
             "solves_per_s": 4096 / (z["ms"].mean() * 1e-3), "solved": float((z["st"] == 0).mean()),
             "bit_identical_to_first": bool(np.array_equal(z["u"], ref["u"])),
             "u_maxdiff_vs_first": float(np.abs(z["u"] - ref["u"]).max())}
        print(os.path.basename(lib), json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
