"""Generate tests/golden/closed_loop_bands.json: per-run summary statistics of the
reference's recorded closed-loop laps ("closed-loop sanity bands").

For every recorded run on ippodromo without obstacles (experiments/data/*/<ctl>_state_traj.npy,
<ctl>_action_traj.npy, <ctl>_config.yaml; float64 arrays read with numpy's default
allow_pickle=False, configs with yaml.safe_load) this records the controller config the run
used (horizon, horizon_pm, ds_pm, mpc_dt, max_speed, Fx/Fy weights) and what the lap looked
like: steps until the simulator's stop rule s > L - 0.1 (simulation/racing.py:219), the lap
time t at the last row (racing.py:99), Ux median / p99 / max, Fx min / max, |w| max and
|ey| max.  Runs where a second car stopped the simulation early (race*_: both controllers
share one simulator and it stops when the first car finishes, racing.py:218-228) are marked
`complete = false`.

Round 4 adds "runs_r4": every recorded run with the obstacle barrier on and every shoe-track
run (the giant-obstacle runs excluded: their obstacle set was never recorded), each with its
full controller config, its track, the steps until the stop rule on that track, s at the last
row, Ux median, |ey| max and the smallest clearance dist - r to the track's obstacles.

Run from the repo root (needs /root/reference):  python tests/golden/make_st_bands.py
"""
from __future__ import annotations

import glob
import json
import os

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = "/root/reference/experiments/data"
IPPODROMO_LENGTH = 315.5  # approximate; the stop rule is evaluated against the recorded s


R4 = [("singletrack_obstacles_shoe", "singletrack"), ("cascaded_obstacles1_ippodromo", "cascaded"),
      ("cascaded_obstacles2_ippodromo", "cascaded"), ("cascaded_obstacles_shoe", "cascaded"),
      ("race_obstacles_shoe", "singletrack"), ("race_obstacles_shoe", "cascaded"),
      ("singletrack_shoe", "singletrack"), ("race1_shoe", "singletrack"), ("race1_shoe", "cascaded"),
      ("race2_shoe", "singletrack"), ("race2_shoe", "cascaded")]


def r4_runs():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "vehicle-control_amd"))
    from vcmpc.environment import Track
    out = []
    for run, ctl in R4:
        d = os.path.join(DATA, run)
        X = np.load(os.path.join(d, f"{ctl}_state_traj.npy"), allow_pickle=False)
        with open(os.path.join(d, f"{ctl}_config.yaml")) as f:
            cfg = yaml.safe_load(f)
        tname = run.rsplit("_", 1)[1]
        tr = Track.load(tname)
        done = np.nonzero(X[:, 4] > tr.length - 0.1)[0]
        clear = None
        if cfg.get("obstacles"):
            clear = float(min(np.hypot(X[:, 4] - o.s, X[:, 5] - o.ey).min() - o.radius for o in tr.obstacles))
        out.append(dict(key=f"{run}:{ctl}", run=run, controller=ctl, track=tname, length=float(tr.length),
                        obstacles=bool(cfg.get("obstacles")), config=cfg, steps=int(len(X)),
                        complete=bool(len(done)), lap_steps=int(done[0]) if len(done) else None,
                        s_end=float(X[-1, 4]), Ux_median=float(np.median(X[:, 0])),
                        ey_absmax=float(np.abs(X[:, 5]).max()), clearance_min=clear, x0=[float(v) for v in X[0]]))
    return out


def main():
    runs = []
    for sf in sorted(glob.glob(os.path.join(DATA, "*_ippodromo", "*_state_traj.npy"))):
        run = os.path.basename(os.path.dirname(sf))
        ctl = os.path.basename(sf)[: -len("_state_traj.npy")]
        X = np.load(sf, allow_pickle=False)
        U = np.load(sf.replace("_state_traj", "_action_traj"), allow_pickle=False)
        with open(sf.replace("_state_traj.npy", "_config.yaml")) as f:
            cfg = yaml.safe_load(f)
        if cfg.get("obstacles"):
            continue
        s_end = float(X[-1, 4])
        runs.append(dict(
            run=run, controller=ctl, horizon=int(cfg["horizon"]), horizon_pm=int(cfg.get("horizon_pm") or 0),
            ds_pm=float(cfg.get("ds_pm") or 0), mpc_dt=float(cfg["mpc_dt"]),
            max_speed=float(cfg["state_constraints"]["max_speed"]),
            w_Fx=float(cfg["cost_weights"]["Fx"]), w_Fy=float(cfg["cost_weights"]["Fy"]),
            steps=int(len(X)), s_end=s_end, complete=bool(s_end > IPPODROMO_LENGTH - 1.0),
            lap_time=float(X[-1, 7]),
            Ux_median=float(np.median(X[:, 0])), Ux_p99=float(np.percentile(X[:, 0], 99)), Ux_max=float(X[:, 0].max()),
            Fx_min=float(U[:, 0].min()), Fx_max=float(U[:, 0].max()), w_absmax=float(np.abs(U[:, 1]).max()),
            ey_absmax=float(np.abs(X[:, 5]).max()), x0=[float(v) for v in X[0]]))
    runs_r4 = r4_runs()
    with open(os.path.join(HERE, "closed_loop_bands.json"), "w") as f:
        json.dump({"source": "reference experiments/data/*_ippodromo (no obstacles)", "runs": runs,
                   "source_r4": "reference experiments/data: obstacle runs and shoe-track runs", "runs_r4": runs_r4},
                  f, indent=1)
    for r in runs_r4:
        print(f"{r['key']:42s} track={r['track']} obstacles={r['obstacles']} steps={r['steps']} "
              f"complete={r['complete']} Ux_med={r['Ux_median']:.2f} |ey|max={r['ey_absmax']:.2f} "
              f"clearance={r['clearance_min']}")
    for r in runs:
        print(f"{r['run']:36s} {r['controller']:11s} N={r['horizon']} M={r['horizon_pm']} vmax={r['max_speed']} "
              f"steps={r['steps']} complete={r['complete']} lap={r['lap_time']:.2f}s Ux_med={r['Ux_median']:.2f} "
              f"Fx=[{r['Fx_min']:.0f},{r['Fx_max']:.0f}] |ey|max={r['ey_absmax']:.2f}")


if __name__ == "__main__":
    main()
