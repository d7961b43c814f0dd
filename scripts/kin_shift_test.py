"""Kinematic closed loop at the reference's horizon N = 50 (config/controllers/kinematic.yaml)
through the host controller (BatchedKinematicMPC), with the reference's unshifted warm start
(kinematic_mpc.py:170-187 keeps the previous prediction as is) or a one-step-shifted one.
The unshifted warm start, re-rolled out from the new state (single shooting), crosses the
spatial model's eps = +-pi/2 singularity over a 40 m horizon (scripts/kin_obs_fail_modes.py).

    python scripts/kin_shift_test.py [--N 50] [--steps 400] [--shift]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=50)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--shift", action="store_true")
    ap.add_argument("--obstacles", action="store_true")
    args = ap.parse_args()
    from oracle import models as M
    from vcmpc.config import load_config
    from vcmpc.controllers.kinematic_mpc import BatchedKinematicMPC
    from vcmpc.environment import Track
    from vcmpc.models import KinematicCar
    tr = Track.load("ippodromo")
    car = KinematicCar(load_config("kinematic_car"), tr)
    cfg = load_config("kinematic_mpc")
    cfg["horizon"] = args.N
    cfg["obstacles"] = args.obstacles
    B = 64
    rng = np.random.default_rng(3)
    x = np.zeros((B, 6))
    x[:, 0] = rng.uniform(5, 8, B)
    x[:, 2] = rng.uniform(0, 15, B)
    x[:, 3] = rng.uniform(-0.5, 0.5, B)
    ctl = BatchedKinematicMPC(car, cfg, batch=B)
    ctl.action_prediction[:] = 0.0          # the neutral first guess (simulation.py)
    dt = float(car.dt)
    X, nfail = [x.copy()], 0
    for k in range(args.steps):
        u = ctl.command(x)
        bad = ctl.status != 0
        nfail += int(bad.sum())
        u[bad] = 0.0
        if bad.any():
            ctl.action_prediction[bad] = 0.0
            ctl.state_prediction[bad] = x[bad][:, :, None]
        if args.shift:
            ctl.action_prediction[:, :, :-1] = ctl.action_prediction[:, :, 1:].copy()
            ctl.state_prediction[:, :, :-1] = ctl.state_prediction[:, :, 1:].copy()
        x = M.kin_transition(x, u, np.asarray(tr.k(x[:, 2]), np.float64), dt, 2.5)
        X.append(x.copy())
    X = np.array(X)
    off = (np.abs(X[..., 3]) > tr.width / 2).any(0)
    print(f"N={args.N} shift={args.shift} obstacles={args.obstacles}: non-solved {nfail} of {B * args.steps} "
          f"({nfail / (B * args.steps):.3%}), vehicles off track {off.sum()} of {B}, max |ey| {np.abs(X[..., 3]).max():.2f}, "
          f"final s median {np.median(X[-1, :, 2]):.1f}")


if __name__ == "__main__":
    main()
