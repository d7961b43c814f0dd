"""Generate tests/golden/replay_kat.npz: the reference's recorded closed-loop runs at the
controller shapes this build solves, for the open-loop *replay* test (tests/test_gpu_replay.py):
the recorded state at every control step, the action IPOPT applied there and its predicted
plan (get_state_prediction(), global x, y, psi per stage; simulation/racing.py:239-240,446).

Runs: cascaded7_ippodromo (N = 20 + M = 40, cascaded.yaml's shape and weights) and
singletrack_ippodromo (N = 60).  float64 arrays read as plain numpy (allow_pickle=False);
configs from each run's <ctl>_config.yaml (yaml.safe_load).

Run from the repo root (needs /root/reference):  python tests/golden/make_replay_kat.py
"""
from __future__ import annotations

import json
import os

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = "/root/reference/experiments/data"
RUNS = [("cascaded7_ippodromo", "cascaded"), ("singletrack_ippodromo", "singletrack")]


def main():
    out, cfgs = {}, {}
    for run, ctl in RUNS:
        d = os.path.join(DATA, run)
        x = np.load(os.path.join(d, f"{ctl}_state_traj.npy"), allow_pickle=False)
        u = np.load(os.path.join(d, f"{ctl}_action_traj.npy"), allow_pickle=False)
        p = np.load(os.path.join(d, f"{ctl}_preds.npy"), allow_pickle=False)
        with open(os.path.join(d, f"{ctl}_config.yaml")) as f:
            cfgs[run] = yaml.safe_load(f)
        out[f"{run}/state_traj"] = x
        out[f"{run}/action_traj"] = u
        out[f"{run}/preds"] = p[:, :, :2].astype(np.float32)   # global x, y per stage (plots-grade)
    out["configs"] = np.array(json.dumps(cfgs))
    np.savez_compressed(os.path.join(HERE, "replay_kat.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
