"""Kinematic closed loop with obstacle terms: non-solved steps vs the interior point's
iteration cap and tolerance (tests/test_gpu_obstacles.py workload)."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))
from vcmpc.config import load_config
from vcmpc.environment import Track
from vcmpc.models import KinematicCar
from vcmpc.simulation import BatchedRacingSimulator

tr = Track.load("ippodromo")
obs = [(o.s, o.ey, o.radius) for o in tr.obstacles]
B, K = 64, 400
rng = np.random.default_rng(3)
x0 = np.zeros((B, 6)); x0[:, 0] = rng.uniform(5, 8, B); x0[:, 2] = rng.uniform(0, 15, B); x0[:, 3] = rng.uniform(-0.5, 0.5, B)
for qp in ({"max_iter": 40}, {"max_iter": 100}, {"max_iter": 40, "tol": 1e-8}, {"max_iter": 100, "tol": 1e-8}):
    cfg = load_config("kinematic_mpc"); cfg["obstacles"] = True
    q = dict(cfg["qp"]); q.update(qp); q.update({"trust_a": 1.0, "trust_w": 0.1}); cfg["qp"] = q
    sim = BatchedRacingSimulator(KinematicCar(load_config("kinematic_car"), tr), cfg, tr, batch=B)
    out = sim.reset(x0.copy()).run(K)
    X = out["state_traj"]
    s, ey = X[..., 2], X[..., 3]
    clr = np.min([np.hypot(s - so, ey - eo) - r for so, eo, r in obs], axis=0).min(axis=0)
    print(qp, "nfail %.3f" % (out["nfail"].sum() / (B * K)), "clear %d/%d" % ((clr > 0).sum(), B),
          "median clearance %.3f" % np.median(clr), "median s %.1f" % np.median(X[-1, :, 2]), flush=True)
