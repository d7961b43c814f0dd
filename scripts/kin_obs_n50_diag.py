"""Where do the N = 50 obstacle closed loop's off-track excursions come from?

Runs tests/test_gpu_obstacles.py's long-horizon loop (ippodromo, 64 vehicles, 400 steps,
obstacles on) one control step at a time and records, per vehicle and step, whether the step
was non-solved (nfail increment), the plant's |ey| and the plan's max |ey| over the horizon.
For every vehicle that leaves the track (|ey| >= width / 2) it prints the first off-track step,
the non-solved steps before it and the plan's max |ey| in the steps leading there: a plan that
already crosses the boundary while every QP solved is the NLP's own trade-off (the boundary is
a cost term, kinematic_mpc.py:110-122), not a failed-QP restart.

    python scripts/kin_obs_n50_diag.py [--N 50] [--sqp 10 20] [--out gpurun_out/kin_obs_diag.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))


def run(N, sqp, B=64, K=400, qp=None, seed=3):
    from vcmpc.config import load_config
    from vcmpc.environment import Track
    from vcmpc.models import KinematicCar
    from vcmpc.simulation import BatchedRacingSimulator
    tr = Track.load("ippodromo")
    rng = np.random.default_rng(seed)
    x0 = np.zeros((B, 6))
    x0[:, 0] = rng.uniform(5, 8, B)
    x0[:, 2] = rng.uniform(0, 15, B)
    x0[:, 3] = rng.uniform(-0.5, 0.5, B)
    cfg = load_config("kinematic_mpc")
    cfg["obstacles"] = True
    cfg["horizon"] = N
    cfg["qp"] = dict(cfg.get("qp") or {}, kin_sqp=sqp, **(qp or {}))
    car = KinematicCar(load_config("kinematic_car"), tr)
    sim = BatchedRacingSimulator(car, cfg, tr, batch=B)
    sim.reset(x0.copy())
    ey = np.zeros((K + 1, B))
    ey[0] = x0[:, 3]
    sa = np.zeros((K + 1, B))
    sa[0] = x0[:, 2]
    plan_ey = np.zeros((K, B))
    fail = np.zeros((K, B), bool)
    prev = np.zeros(B, np.int64)
    for k in range(K):
        out = sim.run(1)
        nf = out["nfail"].astype(np.int64)
        fail[k] = nf > prev
        prev = nf
        ey[k + 1] = out["state_traj"][-1, :, 3]
        sa[k + 1] = out["state_traj"][-1, :, 2]
        plan_ey[k] = np.abs(sim.state_prediction[:, 3, :]).max(axis=1)
    half = tr.width / 2
    off = np.abs(ey) >= half
    obs = [(o.s, o.ey, o.radius) for o in tr.obstacles]
    clear = np.min([np.hypot(sa - so, ey - eo) - r for so, eo, r in obs], axis=0).min(axis=0)
    res = {"N": N, "sqp": sqp, "qp": qp or {}, "seed": seed, "off_track": int(off.any(axis=0).sum()),
           "hit": int((clear <= 0).sum()), "nonsolved": int(fail.sum()),
           "max_abs_ey": float(np.abs(ey).max()), "vehicles": []}
    for b in np.nonzero(off.any(axis=0))[0]:
        k_off = int(np.argmax(off[:, b]))           # state index (after k_off - 1 steps)
        lo = max(0, k_off - 40)
        res["vehicles"].append({
            "vehicle": int(b), "first_off_step": k_off,
            "nonsolved_before": int(fail[:k_off, b].sum()),
            "nonsolved_last40": int(fail[lo:k_off, b].sum()),
            "plan_max_ey_last40": float(plan_ey[lo:k_off, b].max()) if k_off > 0 else None,
            "max_ey": float(np.abs(ey[:, b]).max())})
    print(json.dumps({k: v for k, v in res.items() if k != "vehicles"}))
    for v in res["vehicles"]:
        print("  ", v)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=50)
    ap.add_argument("--sqp", type=int, nargs="+", default=[10, 20])
    ap.add_argument("--out", default=None)
    ap.add_argument("--seeds", type=int, nargs="+", default=[3])
    ap.add_argument("--qp", nargs="*", default=[], help="qp overrides key=value (e.g. elastic=0 max_iter=80)")
    a = ap.parse_args()
    qp = {k: float(v) if "." in v or "e" in v else int(v) for k, v in (kv.split("=") for kv in a.qp)}
    allres = [run(a.N, s, qp=qp, seed=sd) for s in a.sqp for sd in a.seeds]
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(allres, f, indent=1)


if __name__ == "__main__":
    main()
