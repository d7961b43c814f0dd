"""A/B of kinematic-kernel builds (scripts/build_kin_variants.sh): C2 kernel time (HIP events
on the context stream) and u* of each library against the first one, each library in its own
child process (VCMPC_LIB is read at import).
usage: python scripts/kin_ab.py [--batch B] [--reps R] lib1.so lib2.so ..."""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib, batch, reps, out):
    os.environ["VCMPC_LIB"] = lib
    sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))
    import torch
    from vcmpc import Context, make_params
    from vcmpc.config import load_config
    from vcmpc.workload import kinematic_batch
    dev = torch.device("cuda:0")
    d = kinematic_batch(batch, seed=31)
    t = {k: torch.from_numpy(v).to(dev) for k, v in d.items()}
    p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=load_config("kinematic_mpc"))
    N = 20
    stream = torch.cuda.Stream(dev)
    with Context(N=N, max_batch=batch, params=p) as c:
        c.set_stream(stream.cuda_stream)
        xbar = torch.empty((batch, N + 1, 6), dtype=torch.float64, device=dev)
        u0 = torch.empty((batch, 2), dtype=torch.float64, device=dev)
        st = torch.empty((batch,), dtype=torch.int32, device=dev)
        it = torch.empty((batch,), dtype=torch.int32, device=dev)
        ub = t["ubar"].clone()
        ms = []
        for r in range(reps + 3):
            with torch.cuda.stream(stream):
                ub.copy_(t["ubar"])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            c.solve(t["x0"], t["kappa"], t["ds"], ub, xbar, u0, st, it)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            if r >= 3:
                ms.append(e0.elapsed_time(e1))
        np.savez(out, u=ub.cpu().numpy(), st=st.cpu().numpy(), it=it.cpu().numpy(), ms=np.array(ms))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--child", nargs=2)
    ap.add_argument("--keep", help="directory to keep each library's u / status / iters (.npz) in")
    ap.add_argument("libs", nargs="*")
    a = ap.parse_args()
    if a.child:
        child(a.child[0], a.batch, a.reps, a.child[1])
        return
    res, ref = {}, None
    for i, lib in enumerate(a.libs):
        out = f"/tmp/kin_ab_{i}.npz"
        subprocess.run([sys.executable, __file__, "--batch", str(a.batch), "--reps", str(a.reps),
                        "--child", lib, out], check=True, timeout=300)
        z = np.load(out)
        if a.keep:
            os.makedirs(a.keep, exist_ok=True)
            np.savez(os.path.join(a.keep, f"{i}_{os.path.basename(lib)}.npz"), u=z["u"], st=z["st"], it=z["it"])
        if ref is None:
            ref = z
        r = {"kernel_ms_mean": float(z["ms"].mean()), "kernel_ms_min": float(z["ms"].min()),
             "solves_per_s": a.batch / (z["ms"].mean() * 1e-3),
             "solved": float((z["st"] == 0).mean()), "iters_mean": float(z["it"].mean()),
             "iters_max": int(z["it"].max()),
             "u_maxdiff_vs_first": float(np.abs(z["u"] - ref["u"]).max()),
             "bit_identical_to_first": bool(np.array_equal(z["u"], ref["u"]))}
        res[os.path.basename(lib)] = r
        print(os.path.basename(lib), json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
