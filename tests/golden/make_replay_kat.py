"""Generate tests/golden/replay_kat.npz: the reference's recorded closed-loop runs at the
controller shapes this build solves, for the open-loop *replay* test (tests/test_gpu_replay.py):
the recorded state at every control step, the action IPOPT applied there and its predicted
plan (get_state_prediction(), global x, y, psi per stage; simulation/racing.py:239-240,446).

Runs: cascaded7_ippodromo (N = 20 + M = 40, cascaded.yaml's shape and weights),
singletrack_ippodromo (N = 60), and (round 4) every recorded run with the obstacle barrier on
(singletrack_obstacles_shoe, cascaded_obstacles{1,2}_ippodromo, cascaded_obstacles_shoe,
race_obstacles_shoe's two cars) plus the shoe-track runs without obstacles (singletrack_shoe,
race{1,2}_shoe's two cars), and (round 5) race1_ippodromo's single-track N = 50 and the cascaded
tails M = 15 / 25 / 35 of race1/2/3_ippodromo -- every recorded horizon shape.  Not included: cascaded_giantObstacle{1,2,3}_ippodromo -- their
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
        ("race3_ippodromo", "cascaded")]


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
