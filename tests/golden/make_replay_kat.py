"""Generate tests/golden/replay_kat.npz: the reference's recorded closed-loop runs at the
controller shapes this build solves, for the open-loop *replay* test (tests/test_gpu_replay.py):
the recorded state at every control step, the action IPOPT applied there and its predicted
plan (get_state_prediction(), global x, y, psi per stage; simulation/racing.py:239-240,446).

Runs: cascaded7_ippodromo (N = 20 + M = 40, cascaded.yaml's shape and weights),
singletrack_ippodromo (N = 60), and (round 4) every recorded run with the obstacle barrier on
(singletrack_obstacles_shoe, cascaded_obstacles{1,2}_ippodromo, cascaded_obstacles_shoe,
race_obstacles_shoe's two cars) plus the shoe-track runs without obstacles (singletrack_shoe,
race{1,2}_shoe's two cars), (round 5) race1_ippodromo's single-track N = 50 and the cascaded
tails M = 15 / 25 / 35 of race1/2/3_ippodromo -- every recorded horizon shape -- and (round 6) the
24 remaining ippodromo controller runs (singletrack{2,3,4}, singletrack_slip_angle{,2,3},
cascaded{1..6}, cascaded_slip_angle{,2}, race{4..7} both cars, race{2,3} single-track).  Not included: cascaded_giantObstacle{1,2,3}_ippodromo -- their
obstacle set is recorded nowhere (the runs' configs hold only the controller; the reference's
ippodromo.yaml has the ordinary obstacles, and the recorded paths swerve to |ey| 5-6 m round a
different large obstacle in each run: at s ~ 30 in run 1, s ~ 170-185 on opposite sides in runs
2 and 3), so their QPs cannot be rebuilt.  Each run key is
"<dir>:<controller>".  float64 arrays read as plain numpy (allow_pickle=False); configs from each
run's <ctl>_config.yaml (yaml.safe_load).

Run from the repo root (needs /root/reference):  python tests/golden/make_replay_kat.py
"""
from __future__ import annotations

import json
import os

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = "/root/reference/experiments/data"
RUNS = [("cascaded7_ippodromo", "cascaded"), ("singletrack_ippodromo", "singletrack"),
        ("singletrack_obstacles_shoe", "singletrack"), ("cascaded_obstacles1_ippodromo", "cascaded"),
        ("cascaded_obstacles2_ippodromo", "cascaded"), ("cascaded_obstacles_shoe", "cascaded"),
        ("race_obstacles_shoe", "singletrack"),
        ("race_obstacles_shoe", "cascaded"), ("singletrack_shoe", "singletrack"), ("race1_shoe", "singletrack"),
        ("race1_shoe", "cascaded"), ("race2_shoe", "singletrack"), ("race2_shoe", "cascaded"),
        # round 5: every remaining recorded horizon shape -- single-track N = 50 (race1_ippodromo,
        # BASELINE.md's first row) and the cascaded tails M = 15 / 25 / 35 (race1/2/3_ippodromo)
        ("race1_ippodromo", "singletrack"), ("race1_ippodromo", "cascaded"), ("race2_ippodromo", "cascaded"),
        ("race3_ippodromo", "cascaded"),
        # round 6: every other replayable recorded controller run (their shapes are covered above,
        # but each carries its own max_speed cap 18 / 20 / 26 / 30, slip-angle weights and recorded
        # trajectory): 24 run x controller keys
        ("singletrack2_ippodromo", "singletrack"), ("singletrack3_ippodromo", "singletrack"),
        ("singletrack4_ippodromo", "singletrack"), ("singletrack_slip_angle_ippodromo", "singletrack"),
        ("singletrack_slip_angle2_ippodromo", "singletrack"), ("singletrack_slip_angle3_ippodromo", "singletrack"),
        ("cascaded1_ippodromo", "cascaded"), ("cascaded2_ippodromo", "cascaded"), ("cascaded3_ippodromo", "cascaded"),
        ("cascaded4_ippodromo", "cascaded"), ("cascaded5_ippodromo", "cascaded"), ("cascaded6_ippodromo", "cascaded"),
        ("cascaded_slip_angle_ippodromo", "cascaded"), ("cascaded_slip_angle2_ippodromo", "cascaded"),
        ("race2_ippodromo", "singletrack"), ("race3_ippodromo", "singletrack"),
        ("race4_ippodromo", "singletrack"), ("race4_ippodromo", "cascaded"),
        ("race5_ippodromo", "singletrack"), ("race5_ippodromo", "cascaded"),
        ("race6_ippodromo", "singletrack"), ("race6_ippodromo", "cascaded"),
        ("race7_ippodromo", "singletrack"), ("race7_ippodromo", "cascaded")]


def key(run, ctl):
    """fixture key of one recorded controller: the two legacy runs keep their directory name"""
    return run if (run, ctl) in RUNS[:2] else f"{run}:{ctl}"


def main():
    out, cfgs = {}, {}
    for run, ctl in RUNS:
        d = os.path.join(DATA, run)
        x = np.load(os.path.join(d, f"{ctl}_state_traj.npy"), allow_pickle=False)
        u = np.load(os.path.join(d, f"{ctl}_action_traj.npy"), allow_pickle=False)
        p = np.load(os.path.join(d, f"{ctl}_preds.npy"), allow_pickle=False)
        k = key(run, ctl)
        with open(os.path.join(d, f"{ctl}_config.yaml")) as f:
            cfgs[k] = yaml.safe_load(f)
        out[f"{k}/state_traj"] = x
        out[f"{k}/action_traj"] = u
        out[f"{k}/preds"] = p[:, :, :2].astype(np.float32)   # global x, y per stage (plots-grade)
    out["configs"] = np.array(json.dumps(cfgs))
    np.savez_compressed(os.path.join(HERE, "replay_kat.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
