"""Step-by-step trace of one recorded-run closed loop (tests/golden/closed_loop_bands.json "runs_r4"):
where the non-solved steps happen (s, Ux, ey, epsi, the nearest obstacle) and what the plan looked like.
usage: python scripts/band_trace.py <key> [sqp_iters]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vehicle-control_amd"), os.path.join(ROOT, "scripts")]
from replay_recorded import config_for  # noqa: E402
from vcmpc.config import load_config  # noqa: E402
from vcmpc.environment import Track  # noqa: E402
from vcmpc.models import DynamicCar  # noqa: E402
from vcmpc.simulation import BatchedRacingSimulator  # noqa: E402

with open(os.path.join(ROOT, "tests", "golden", "closed_loop_bands.json")) as f:
    RUNS = {r["key"]: r for r in json.load(f)["runs_r4"]}
key = sys.argv[1] if len(sys.argv) > 1 else "singletrack_obstacles_shoe:singletrack"
rec = RUNS[key]
track = Track.load(rec["track"])
cfg = config_for(key, rec["config"])
if len(sys.argv) > 2:
    cfg["qp"] = dict(cfg["qp"], sqp_iters=int(sys.argv[2]))
car = DynamicCar(load_config("dynamic_car"), track, tyre="fiala")
sim = BatchedRacingSimulator(car, cfg, track, batch=1)
sim.reset(np.array([rec["x0"]]))
K = int(rec["steps"] * 1.08)
prev = 0
shown = 0
for step in range(K):
    out = sim.run(1)
    nf = int(out["nfail"][0])
    x = sim.states[0]
    if nf > prev and shown < 40:
        obs = min(((o.s, o.ey, np.hypot(x[4] - o.s, x[5] - o.ey) - o.radius) for o in track.obstacles), key=lambda t: t[2])
        xp = sim.state_prediction[0]
        print(f"step {step}: non-solved #{nf}  s {x[4]:.1f} Ux {x[0]:.2f} Uy {x[1]:.3f} r {x[2]:.3f} delta {x[3]:.3f} "
              f"ey {x[5]:.2f} epsi {x[6]:.3f} | nearest obstacle s {obs[0]:.0f} ey {obs[1]:.1f} clearance {obs[2]:.2f}",
              flush=True)
        shown += 1
    prev = nf
    if x[4] > track.length - 0.1:
        print(f"lap at step {step}")
        break
print(f"{key}: steps {step + 1}, nfail {prev}, s {sim.states[0][4]:.1f}")

# the first non-solved step after the start: re-solve its QP sequence directly with diagnostics
if len(sys.argv) > 3:
    from vcmpc import Context, _abi
    from vcmpc.config import make_params, obstacle_list
    from vcmpc.controllers.cascaded_mpc import dyn_horizon_params
    S = int(sys.argv[3])
    sim = BatchedRacingSimulator(car, cfg, track, batch=1)
    sim.reset(np.array([rec["x0"]]))
    sim.run(S)
    x = sim.states.copy()
    xb = sim._to_host(sim.xbar).copy()
    ub = sim._to_host(sim.ubar).copy()
    ds, kap = dyn_horizon_params(x[:, 4], xb[:, :, 0], float(cfg["mpc_dt"]), track.k)
    for label, qp in (("config", {}), ("max_iter 200", {"max_iter": 200}), ("sqp 10", {"sqp_iters": 10}),
                      ("prox 0.1", {"prox": 0.1}), ("neutral warm start", None)):
        c2 = dict(cfg)
        c2["qp"] = dict(cfg["qp"], **(qp or {}))
        p = make_params(dyn_car=car.config, dyn_mpc=c2, tyre="fiala", obstacles=obstacle_list(track, c2))
        with Context(model=_abi.VC_MODEL_DYNAMIC, N=sim.N, max_batch=1, dtype=_abi.VC_F64, params=p) as ctx:
            u_ws = np.zeros_like(ub) if qp is None else ub.copy()
            r = ctx.solve(x, kap, ds, u_ws, diag=True)
        print(f"  step {S} re-solve [{label}]: status {int(r[3][0])} iters {int(r[4][0])} diag {np.round(r[5][0], 6).tolist()} "
              f"u0 {np.round(r[0][0], 3).tolist()}", flush=True)
