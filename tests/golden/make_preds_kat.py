"""Generate tests/golden/preds_kat.npz: known-answer rows for the track geometry and the
controllers' global-frame predictions, from the reference's recorded closed-loop runs.

The reference's simulator stores, after every control step n, the controller's
get_state_prediction() (simulation/racing.py:239-240, saved as <ctl>_preds.npy with shape
(T-1, H, 3) at :446).  Column 0 is rel2glob of the predicted state at stage 0
(cascaded_mpc.py:340-352, racing_car.py rel2glob -> environment/track.py:102-107), and the
NLP pins stage 0 to the measured state (x_0 = x0, cascaded_mpc.py:26-28), so

    preds[n, 0] == rel2glob(s, ey, epsi of state_traj[n])

exactly: a pin on the track's x(s), y(s), orientation and rel2glob, independent of IPOPT.
Rows: every 3rd step of all 44 recorded runs (experiments/data/*/*_{preds,state_traj}.npy,
float64, read as plain numpy arrays); configs from each run's <ctl>_config.yaml.

Run from the repo root (needs /root/reference):  python tests/golden/make_preds_kat.py
"""
from __future__ import annotations

import glob
import os

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = "/root/reference/experiments/data"
STRIDE = 3


def main():
    runs, rows = [], []
    for i, pf in enumerate(sorted(glob.glob(os.path.join(DATA, "*", "*_preds.npy")))):
        run = os.path.basename(os.path.dirname(pf))
        ctl = os.path.basename(pf)[: -len("_preds.npy")]
        preds = np.load(pf, allow_pickle=False)
        states = np.load(pf.replace("_preds", "_state_traj"), allow_pickle=False)
        with open(pf.replace("_preds.npy", "_config.yaml")) as f:
            cfg = yaml.safe_load(f)
        track = 1 if "shoe" in run else 0
        runs.append((run, ctl, track, int(cfg["horizon"]), int(cfg.get("horizon_pm", 0) or 0),
                     float(cfg.get("ds_pm", 0) or 0), float(cfg["mpc_dt"])))
        for n in range(0, len(preds), STRIDE):
            rows.append(np.concatenate([[i, track, n], states[n], preds[n, 0]]))
    rows = np.array(rows)
    np.savez_compressed(
        os.path.join(HERE, "preds_kat.npz"),
        run_id=rows[:, 0].astype(np.int32), track=rows[:, 1].astype(np.int32), step=rows[:, 2].astype(np.int32),
        state=rows[:, 3:11], pred0=rows[:, 11:14],
        run_name=np.array([f"{r[0]}/{r[1]}" for r in runs]), run_track=np.array([r[2] for r in runs], np.int32),
        run_N=np.array([r[3] for r in runs], np.int32), run_M=np.array([r[4] for r in runs], np.int32),
        run_ds_pm=np.array([r[5] for r in runs]), run_mpc_dt=np.array([r[6] for r in runs]))
    print(f"{len(runs)} runs, {len(rows)} rows")


if __name__ == "__main__":
    main()
