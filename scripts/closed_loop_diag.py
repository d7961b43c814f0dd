"""Closed-loop diagnostics on ippodromo: device loop (vc_simulate) vs the Python
controller loop (BatchedSingleTrackMPC + DynamicCar.drive), several SQP settings.
Writes gpurun_out/cl_diag.npz."""
import copy
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]

from vcmpc.config import load_config  # noqa: E402
from vcmpc.controllers.cascaded_mpc import BatchedSingleTrackMPC  # noqa: E402
from vcmpc.environment import Track  # noqa: E402
from vcmpc.models import DynamicCar  # noqa: E402
from vcmpc.simulation import BatchedRacingSimulator  # noqa: E402


def states(B, L, seed):
    rng = np.random.default_rng(seed)
    x = np.zeros((B, 8))
    x[:, 0] = rng.uniform(8, 14, B)
    x[:, 1] = rng.uniform(-0.1, 0.1, B)
    x[:, 2] = rng.uniform(-0.05, 0.2, B)
    x[:, 3] = rng.uniform(-0.03, 0.1, B)
    x[:, 4] = rng.uniform(0, L, B)
    x[:, 5] = rng.uniform(-1.5, 1.5, B)
    x[:, 6] = rng.uniform(-0.1, 0.1, B)
    return x


def main():
    B, K = int(sys.argv[1]) if len(sys.argv) > 1 else 64, int(sys.argv[2]) if len(sys.argv) > 2 else 200
    tr = Track.load("ippodromo")
    car = DynamicCar(load_config("dynamic_car"), tr, tyre="fiala")
    x0 = states(B, tr.length, 21)
    out = {}
    for tag, iters, mdt in (("sqp3", 3, 0.03), ("sqp3_dt045", 3, 0.045), ("sqp5_dt045", 5, 0.045)):
        cfg = copy.deepcopy(load_config("dynamic_mpc"))
        cfg["qp"]["sqp_iters"] = iters
        cfg["mpc_dt"] = mdt
        sim = BatchedRacingSimulator(car, cfg, tr, batch=B)
        t = time.time()
        r = sim.reset(x0).run(K)
        dt = time.time() - t
        X = r["state_traj"]
        print(f"{tag}: {dt:.2f}s  nfail {r['nfail'].sum()}  on-track {(np.abs(X[:, :, 5]) < 4.5).all(0).mean():.3f} "
              f"max|ey| {np.abs(X[:, :, 5]).max():.2f}  Ux [{X[:, :, 0].min():.1f},{X[:, :, 0].max():.1f}]", flush=True)
        out[f"{tag}_X"], out[f"{tag}_U"], out[f"{tag}_nfail"] = X, r["action_traj"], r["nfail"]
    # Python controller loop (host horizon via track.k, immediate neutral retry)
    cfg = copy.deepcopy(load_config("dynamic_mpc"))
    cfg["mpc_dt"] = 0.045
    mpc = BatchedSingleTrackMPC(car, cfg, batch=B)
    x = x0.copy()
    Xs, Us, fails = [x.copy()], [], 0
    for k in range(K):
        u = mpc.command(x)
        fails += int((mpc.status != 0).sum())
        x = car.transition(x, u, tr.k(x[:, 4]), 0.05)
        Xs.append(x.copy()); Us.append(u.copy())
    X = np.array(Xs)
    print(f"python loop: fails {fails} on-track {(np.abs(X[:, :, 5]) < 4.5).all(0).mean():.3f} "
          f"max|ey| {np.abs(X[:, :, 5]).max():.2f}", flush=True)
    out["py_X"], out["py_U"] = X, np.array(Us)
    out["x0"] = x0
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "cl_diag.npz"), **out)


if __name__ == "__main__":
    main()
