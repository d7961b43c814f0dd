"""C5 preview check: 256 vehicles x 300 steps on ippodromo with the dynamic NMPC at N = 40 and
the reference's mpc_dt = 0.03 (singletrack.yaml) under two SQP contracts -- dynamic_mpc.yaml's
(prox 0.1, 3 iterations) and singletrack_mpc.yaml's closed-loop knobs (prox 0.01, 5 iterations)
-- against mpc_dt = 0.045 (the 1.8 s preview of N = 60 x 0.03 at N = 40).

    python scripts/c5_preview.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]


def main():
    from vcmpc.config import load_config
    from vcmpc.environment import Track
    from vcmpc.models import DynamicCar
    from vcmpc.simulation import BatchedRacingSimulator
    from vcmpc.workload import closed_loop_states
    track = Track.load("ippodromo")
    car = DynamicCar(load_config("dynamic_car"), track, tyre="fiala")
    B, K = 256, 300
    x0 = closed_loop_states(B, track.length, seed=31)
    for mpc_dt, qp in ((0.045, {}), (0.03, {}), (0.03, {"prox": 0.01, "sqp_iters": 5}),
                       (0.045, {"prox": 0.01, "sqp_iters": 5})):
        cfg = load_config("dynamic_mpc")
        cfg["mpc_dt"] = mpc_dt
        cfg["qp"] = dict(cfg["qp"], **qp)
        sim = BatchedRacingSimulator(car, cfg, track, batch=B)
        out = sim.reset(x0).run(K)
        X = out["state_traj"]
        ey = np.abs(X[:, :, 5]).max(axis=0)
        print(f"mpc_dt {mpc_dt} qp {qp}: on track {(ey < track.width / 2).mean():.4f}, max |ey| {ey.max():.2f}, "
              f"non-solved {out['nfail'].sum()}, median progress {np.median(X[-1, :, 4] - X[0, :, 4]):.1f} m, "
              f"median Ux {np.median(X[:, :, 0]):.2f}", flush=True)


if __name__ == "__main__":
    main()
