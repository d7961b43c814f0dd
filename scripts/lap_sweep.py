"""Closed-loop single-track laps on ippodromo at the reference's recorded configs (N 50/60 x
max_speed 18/20, mpc_dt 0.03, x0 = (Ux 4, s 1)) for a sweep of the build's SQP-contract
knobs (the `qp` block of config/singletrack_mpc.yaml: sqp_iters, prox, trust region), next
to the recorded IPOPT laps (tests/golden/closed_loop_bands.json).

    python scripts/lap_sweep.py [--steps 520]
"""
import argparse
import copy
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]

VARIANTS = [
    dict(),
    dict(sqp_iters=5),
    dict(prox=0.01),
    dict(prox=0.01, sqp_iters=5),
    dict(prox=0.001, sqp_iters=5),
    dict(prox=0.01, sqp_iters=5, trust_Fx=4000.0),
    dict(prox=0.01, sqp_iters=10),
]


def lap(cfg, x0, steps, track, car):
    from vcmpc.simulation import BatchedRacingSimulator
    sim = BatchedRacingSimulator(car, cfg, track, batch=1)
    t0 = time.perf_counter()
    out = sim.reset(np.array([x0])).run(steps)
    dt = time.perf_counter() - t0
    X, U = out["state_traj"][:, 0], out["action_traj"][:, 0]
    done = np.nonzero(X[:, 4] > track.length - 0.1)[0]
    n = int(done[0]) if len(done) else steps
    return dict(steps=n if len(done) else None, s_end=float(X[n - 1, 4]), Ux_median=float(np.median(X[:n, 0])),
                Fx=(float(U[:n, 0].min()), float(U[:n, 0].max())), w_absmax=float(np.abs(U[:n, 1]).max()),
                ey_absmax=float(np.abs(X[:n, 5]).max()), nfail=int(out["nfail"].sum()), wall_s=dt)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=520)
    ap.add_argument("--cascaded", action="store_true", help="the recorded cascaded laps (point-mass tail M)")
    args = ap.parse_args()
    from vcmpc.config import load_config
    from vcmpc.environment import Track
    from vcmpc.models import DynamicCar
    track = Track.load("ippodromo")
    car = DynamicCar(load_config("dynamic_car"), track, tyre="fiala")
    ctl = "cascaded" if args.cascaded else "singletrack"
    with open(os.path.join(ROOT, "tests", "golden", "closed_loop_bands.json")) as f:
        runs = [r for r in json.load(f)["runs"] if r["controller"] == ctl and r["complete"]]
    rec = {}
    for r in runs:
        rec.setdefault((r["horizon"], r["horizon_pm"], r["max_speed"]), r)
    for (N, M, vmax), r in sorted(rec.items()):
        print(f"== N={N} M={M} vmax={vmax}: recorded steps={r['steps']} Ux_median={r['Ux_median']:.2f} "
              f"Fx=[{r['Fx_min']:.0f},{r['Fx_max']:.0f}] |ey|max={r['ey_absmax']:.2f}", flush=True)
        for v in VARIANTS:
            cfg = load_config("cascaded_mpc" if args.cascaded else "singletrack_mpc")
            cfg["horizon"] = N
            cfg["horizon_pm"] = M
            cfg["state_constraints"]["max_speed"] = vmax
            cfg["qp"] = dict(cfg["qp"], **v)
            res = lap(cfg, r["x0"], args.steps, track, car)
            print(f"   {json.dumps(v):50s} {json.dumps(res)}", flush=True)


if __name__ == "__main__":
    main()
