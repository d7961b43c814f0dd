"""Capture the QPs behind the kinematic obstacle loop's non-solved steps (GPU diagnostic).

Runs the N = 50 obstacle closed loop (tests/test_gpu_obstacles.py, seedable) one control step at
a time.  Before each step it records every vehicle's solver inputs -- the plant state, the warm
start (xbar, ubar) and the horizon parameters vc_horizon derives from them -- and after the step,
for each vehicle whose nfail went up, re-solves exactly those inputs through the simulator's own
context (vc_solve with diagnostics) to confirm the failure reproduces, then stores the case.

    python scripts/kin_fail_capture.py [--seed 7] [--qp elastic=1000.0 ...] [--max 60] --out F.npz
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=50)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--max", type=int, default=60)
    ap.add_argument("--qp", nargs="*", default=[])
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    from vcmpc.config import load_config
    from vcmpc.environment import Track
    from vcmpc.models import KinematicCar
    from vcmpc.simulation import BatchedRacingSimulator
    qp = {k: float(v) if "." in v or "e" in v else int(v) for k, v in (kv.split("=") for kv in a.qp)}
    tr = Track.load("ippodromo")
    B = 64
    rng = np.random.default_rng(a.seed)
    x0 = np.zeros((B, 6))
    x0[:, 0] = rng.uniform(5, 8, B)
    x0[:, 2] = rng.uniform(0, 15, B)
    x0[:, 3] = rng.uniform(-0.5, 0.5, B)
    cfg = load_config("kinematic_mpc")
    cfg["obstacles"] = True
    cfg["horizon"] = a.N
    cfg["qp"] = dict(cfg.get("qp") or {}, **qp)
    car = KinematicCar(load_config("kinematic_car"), tr)
    sim = BatchedRacingSimulator(car, cfg, tr, batch=B, use_torch=False)
    sim.reset(x0.copy())
    cases = {k: [] for k in ("step", "vehicle", "x0", "kappa", "ds", "ubar", "xbar", "status", "iters", "diag",
                             "status_resolve")}
    prev = np.zeros(B, np.int64)
    nfail_total = 0
    for k in range(a.steps):
        xs = sim.states.copy()
        xb = np.array(sim.xbar, copy=True)
        ub = np.array(sim.ubar, copy=True)
        kap, ds = sim.ctx.horizon(xs, xb, sim.mpc_dt)
        kap, ds = np.array(kap, copy=True), np.array(ds, copy=True)
        out = sim.run(1, log=False)
        nf = out["nfail"].astype(np.int64)
        failed = np.nonzero(nf > prev)[0]
        prev = nf
        nfail_total += len(failed)
        if len(failed) and len(cases["step"]) < a.max:
            idx = failed[: a.max - len(cases["step"])]
            r = sim.ctx.solve(xs[idx].copy(), kap[idx].copy(), ds[idx].copy(), ub[idx].copy(), xb[idx].copy(),
                              diag=True)
            st, it, dg = r[3], r[4], r[5]
            for j, b in enumerate(idx):
                for key, v in (("step", k), ("vehicle", b), ("x0", xs[b]), ("kappa", kap[b]), ("ds", ds[b]),
                               ("ubar", ub[b]), ("xbar", xb[b]), ("status", st[j]), ("iters", it[j]),
                               ("diag", dg[j]), ("status_resolve", st[j])):
                    cases[key].append(v)
    print(f"seed {a.seed} qp {qp}: {nfail_total} non-solved steps; captured {len(cases['step'])}, "
          f"re-solve non-solved {int(np.sum(np.array(cases['status']) != 0))}")
    for j in range(len(cases["step"])):
        print(f"  step {cases['step'][j]:4d} vehicle {cases['vehicle'][j]:2d} status {cases['status'][j]} "
              f"iters {cases['iters'][j]:4d} diag {np.array2string(cases['diag'][j], precision=3)}")
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    np.savez_compressed(a.out, **{k: np.array(v) for k, v in cases.items()}, qp=str(qp), seed=a.seed, N=a.N)


if __name__ == "__main__":
    main()
