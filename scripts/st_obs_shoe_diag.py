"""Why does the single-track closed loop fail every step on the shoe track with obstacles
(test_gpu_bands singletrack_obstacles_shoe, r04d: nfail = all steps, the car coasting straight into
the obstacle at s = 30)?  Runs the first steps of the device closed loop (vc_simulate) and of the
host controller (BatchedSingleTrackMPC.command + DynamicCar.drive) from the recorded x0 for
several (track, N, obstacles) combinations and prints each step's status / iterations.
usage: python scripts/st_obs_shoe_diag.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vehicle-control_amd"), os.path.join(ROOT, "scripts")]
from replay_recorded import config_for  # noqa: E402
from vcmpc.config import load_config  # noqa: E402
from vcmpc.controllers.cascaded_mpc import BatchedSingleTrackMPC  # noqa: E402
from vcmpc.environment import Track  # noqa: E402
from vcmpc.models import DynamicCar  # noqa: E402
from vcmpc.simulation import BatchedRacingSimulator  # noqa: E402

with open(os.path.join(ROOT, "tests", "golden", "closed_loop_bands.json")) as f:
    RUNS = {r["key"]: r for r in json.load(f)["runs_r4"]}
rec = RUNS["singletrack_obstacles_shoe:singletrack"]
x0 = np.array([rec["x0"]])
for track_name, N, obs in (("shoe", 60, True), ("shoe", 60, False), ("shoe", 40, True), ("ippodromo", 60, True),
                           ("ippodromo", 40, True)):
    track = Track.load(track_name)
    cfg = config_for("singletrack_obstacles_shoe:singletrack", rec["config"])
    cfg["horizon"] = N
    cfg["obstacles"] = obs
    car = DynamicCar(load_config("dynamic_car"), track, tyre="fiala")
    sim = BatchedRacingSimulator(car, cfg, track, batch=1)
    sim.reset(x0.copy())
    nf = []
    for step in range(8):
        out = sim.run(1)
        nf.append(int(out["nfail"][0]))
    X = sim.states[0]
    print(f"{track_name} N={N} obstacles={obs}: device loop cumulative nfail after steps 1..8 {nf}; "
          f"x after 8 steps Ux {X[0]:.2f} s {X[4]:.2f} ey {X[5]:.3f}", flush=True)
    # host controller, same start
    car2 = DynamicCar(load_config("dynamic_car"), track, tyre="fiala")
    ctl = BatchedSingleTrackMPC(car2, cfg, batch=1)
    u = ctl.command(x0.copy())
    print(f"   host controller at x0: status {int(ctl.status[0])} iters {int(ctl.iters[0])} u0 {np.round(u[0], 4).tolist()}",
          flush=True)
