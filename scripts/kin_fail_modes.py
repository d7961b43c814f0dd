"""Why do kinematic closed-loop steps end non-solved?  Runs the 64-vehicle x 200-step ippodromo
loop of tests/test_gpu_kin_ric.py one step at a time, re-solves every non-solved step's QP
(same x0, warm start, horizon parameters from the host table) with diagnostics through both
kernels, and classifies it with the oracle: infeasible linearised QP (the oracle's certificate
has a primal residual) or a solver failure on a feasible QP.

    python scripts/kin_fail_modes.py [--solver 1] [--steps 200]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]

from oracle import ltv_qp as Q  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--solver", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--N", type=int, default=20)
    args = ap.parse_args()
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.controllers.kinematic_mpc import RTI_TRUST
    from vcmpc.environment import Track
    from vcmpc.models import KinematicCar
    from vcmpc.simulation import BatchedRacingSimulator
    track = Track.load("ippodromo")
    car = KinematicCar(load_config("kinematic_car"), track)
    B, N = 64, args.N
    rng = np.random.default_rng(3)
    x0 = np.zeros((B, 6))
    x0[:, 0] = rng.uniform(4, 9, B)
    x0[:, 2] = rng.uniform(0, track.length, B)
    x0[:, 3] = rng.uniform(-1.5, 1.5, B)
    cfg = load_config("kinematic_mpc")
    cfg["horizon"] = N
    cfg["qp"] = dict(cfg.get("qp") or {}, solver=args.solver)
    sim = BatchedRacingSimulator(car, cfg, track, batch=B)
    sim.reset(x0)
    W = Q.kin_weights(cfg)
    W.update(RTI_TRUST)
    qcfg = dict(cfg)
    qcfg["qp"] = dict(RTI_TRUST, **cfg["qp"])
    ctxs = {s: Context(model=_abi.VC_MODEL_KINEMATIC, N=N, max_batch=B, dtype=_abi.VC_F64,
                       params=make_params(kin_car=load_config("kinematic_car"),
                                          kin_mpc=dict(qcfg, qp=dict(qcfg["qp"], solver=s)))) for s in (0, 1)}
    cats = {"infeasible": 0, "feasible": 0}
    rows = []
    for k in range(args.steps):
        xk, xb, ub = sim.states.copy(), sim.state_prediction.copy(), sim.action_prediction.copy()
        before = sim._to_host(sim.nfail).copy()
        sim.run(1, log=False)
        nf = sim._to_host(sim.nfail) - before
        for b in np.nonzero(nf)[0]:
            ds, kap = Q.kin_horizon_params(xk[b], xb[b], cfg["mpc_dt"], N, track.k)
            u = np.swapaxes(ub[b:b + 1], 1, 2).copy()
            ref = Q.kin_ltv_solve(xk[b:b + 1], u, kap[None], ds[None], 2.5, W)
            pf = float(ref["kkt"]["pfeas"][0])
            cat = "infeasible" if pf > 1e-6 else "feasible"
            cats[cat] += 1
            res = {}
            for s, c in ctxs.items():
                r = c.solve(xk[b:b + 1], kap[None], ds[None], u.copy(), diag=True)
                res[s] = (int(r[3][0]), int(r[4][0]), r[5][0].round(12).tolist(),
                          float(np.abs(r[2][0] - ref["u_star"][0]).max()))
            rows.append((k, int(b), cat, pf, res))
            if len(rows) <= 30:
                print(f"step {k} vehicle {b}: {cat} (oracle pfeas {pf:.2e}, polished {ref['polished'][0]}); "
                      f"kin_ltv {res[0]}; kin_ric {res[1]}; x {np.round(xk[b], 3)}", flush=True)
    print(f"non-solved steps: {sum(cats.values())} -- {cats}")


if __name__ == "__main__":
    main()
