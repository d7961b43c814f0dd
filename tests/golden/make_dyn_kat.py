"""Generate tests/golden/dyn_plant_kat.npz from the reference's recorded traces.

Runs only where the reference checkout is mounted (``/root/reference``); the
GPU box uses the committed .npz.  Nothing from the reference's source is read:
only its data files ``experiments/data/<run>/<ctrl>_{state,action}_traj.npy``
(loaded with numpy's default allow_pickle=False).

Known-answer test: the reference simulator appends the car state
after ``car.drive(action)`` (simulation/racing.py:230-241, racing_car.py:34-46), so
``state[n+1] = DynamicCar.transition(state[n], action[n+1], k(s_n), dt=0.05)`` with
the temporal RK4 of dynamic_car.py:144-167 / integrators.py:26-37.  The curvature
k(s_n) of the CasADi track spline is not stored; it is back-solved per step from
the epsi component (secant on the oracle's RK4), so the epsi column is matched by
construction and the Ux, Uy, r, delta (kappa-independent) and s, ey, t columns are
the genuine checks.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import models as M  # noqa: E402

REF = "/root/reference/experiments/data"
RUNS = [  # (run directory, controller file prefix, max rows kept)
    ("race1_ippodromo", "singletrack", 431),
    ("race1_ippodromo", "cascaded", 200),
    ("singletrack_ippodromo", "singletrack", 200),
    ("race2_shoe", "cascaded", 300),
]
DT = 0.05


def backsolve_kappa(x, u, xn, p):
    k = np.zeros(len(x))
    h = 1e-7
    for _ in range(40):
        f0 = M.dyn_transition(x, u, k, DT, p)[:, 6] - xn[:, 6]
        f1 = M.dyn_transition(x, u, k + h, DT, p)[:, 6] - xn[:, 6]
        den = np.where(f1 - f0 == 0, 1.0, f1 - f0)
        step = f0 * h / den
        k = k - step
        if np.max(np.abs(step)) < 1e-17:
            break
    return k


def main():
    cfg = yaml.safe_load(open(os.path.join(ROOT, "vehicle-control_amd", "config", "dynamic_car.yaml")))
    p = M.dyn_params_from_config(cfg)
    xs, us, ks, xns, tags = [], [], [], [], []
    for run, ctrl, keep in RUNS:
        X = np.load(f"{REF}/{run}/{ctrl}_state_traj.npy")
        U = np.load(f"{REF}/{run}/{ctrl}_action_traj.npy")
        x, u, xn = X[:-1][:keep], U[1:][:keep], X[1:][:keep]
        k = backsolve_kappa(x, u, xn, p)
        xs.append(x); us.append(u); ks.append(k); xns.append(xn)
        tags += [f"{run}/{ctrl}"] * len(x)
    out = dict(x=np.concatenate(xs), u=np.concatenate(us), kappa=np.concatenate(ks),
               x_next=np.concatenate(xns), dt=np.float64(DT), run=np.array(tags))
    pred = M.dyn_transition(out["x"], out["u"], out["kappa"], DT, p)
    rel = np.abs(pred - out["x_next"]) / np.maximum(np.abs(out["x_next"]), 1e-12)
    print("rows", len(out["x"]), "max rel err per state", rel.max(axis=0))
    np.savez_compressed(os.path.join(HERE, "dyn_plant_kat.npz"), **out)


if __name__ == "__main__":
    main()
