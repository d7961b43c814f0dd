"""Closed-loop band statistics of one recorded run (tests/golden/closed_loop_bands.json "runs_r4")
at several SQP settings: the test's (5 SQP iterations, prox of the config), 10 iterations, and the
converged setting (40 iterations, prox 0.01).  Prints lap steps, median / mean Ux, |ey| max, clearance
and the speed quartiles beside the recorded run's.
usage: python scripts/band_settings.py [key ...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vehicle-control_amd"), os.path.join(ROOT, "scripts")]
from replay_recorded import config_for  # noqa: E402
from vcmpc.config import load_config  # noqa: E402
from vcmpc.environment import Track  # noqa: E402
from vcmpc.models import DynamicCar  # noqa: E402
from vcmpc.simulation import BatchedRacingSimulator  # noqa: E402

with open(os.path.join(ROOT, "tests", "golden", "closed_loop_bands.json")) as f:
    RUNS = {r["key"]: r for r in json.load(f)["runs_r4"]}
keys = sys.argv[1:] or ["cascaded_obstacles1_ippodromo:cascaded"]
for key in keys:
    rec = RUNS[key]
    track = Track.load(rec["track"])
    print(f"{key}: recorded lap_steps {rec.get('lap_steps')} Ux median {rec['Ux_median']:.2f} "
          f"|ey|max {rec['ey_absmax']:.2f} clearance {rec['clearance_min']}", flush=True)
    for sqp, prox in ((5, None), (10, None), (40, 0.01)):
        cfg = config_for(key, rec["config"])
        q = dict(cfg["qp"], sqp_iters=sqp)
        if prox is not None:
            q["prox"] = prox
        cfg["qp"] = q
        car = DynamicCar(load_config("dynamic_car"), track, tyre="fiala")
        sim = BatchedRacingSimulator(car, cfg, track, batch=1)
        K = int(rec["steps"] * 1.08)
        out = sim.reset(np.array([rec["x0"]])).run(K)
        X = out["state_traj"][:, 0]
        done = np.nonzero(X[:, 4] > track.length - 0.1)[0]
        n = int(done[0]) if len(done) else K
        Xl = X[:n]
        clear = None
        if rec["obstacles"]:
            clear = float(min(np.hypot(Xl[:, 4] - o.s, Xl[:, 5] - o.ey).min() - o.radius for o in track.obstacles))
        qs = np.percentile(Xl[:, 0], [25, 50, 75])
        print(f"  sqp {sqp:2d} prox {q['prox']}: lap steps {n} Ux median {qs[1]:.2f} mean {Xl[:, 0].mean():.2f} "
              f"quartiles {qs[0]:.2f}/{qs[2]:.2f} |ey|max {np.abs(Xl[:, 5]).max():.2f} clearance {clear} "
              f"nfail {int(out['nfail'].sum())}", flush=True)
