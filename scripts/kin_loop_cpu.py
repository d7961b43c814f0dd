"""CPU mirror of the kinematic obstacle closed loop (vc_simulate with the kinematic controller's qp
block: csrc/track.hip horizon / drive kernels + the globalised SQP step of oracle/kin_sqp.py), for
trying failure policies off the GPU on a few vehicles.  Same loop as tests/test_gpu_obstacles.py:
ippodromo, obstacles on, seeded x0; per step: _init_horizon from the (shifted) warm start, the SQP
step (multiple shooting at the warm-start states), then the plant (Euler, dt = 0.05, k(s)); a
non-solved step applies u = 0 and restarts the warm start from the neutral guess.

    python scripts/kin_loop_cpu.py --seed 11 --vehicles 42 --steps 60 [--N 50] [--workers 8]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]


def run_vehicle(args):
    seed, b, N, steps, qp_over, verbose, dump = args
    from oracle import kin_sqp as KS
    from oracle import ltv_qp as Q
    from oracle import models as M
    from vcmpc.config import load_config
    from vcmpc.controllers.kinematic_mpc import horizon_params, kin_qp_block
    from vcmpc.environment import Track
    tr = Track.load("ippodromo")
    obs = [(o.s, o.ey, o.radius) for o in tr.obstacles]
    cfg = load_config("kinematic_mpc")
    cfg["obstacles"] = True
    cfg["horizon"] = N
    qp = kin_qp_block(cfg)
    qp.update(qp_over)
    W = Q.kin_weights(cfg)
    W.update(trust_a=qp["trust_a"], trust_w=qp["trust_w"], prox=qp.get("prox", W["prox"]))
    W["obstacles"] = obs
    rng = np.random.default_rng(seed)
    B0 = 64
    x0 = np.zeros((B0, 6))
    x0[:, 0] = rng.uniform(5, 8, B0)
    x0[:, 2] = rng.uniform(0, 15, B0)
    x0[:, 3] = rng.uniform(-0.5, 0.5, B0)
    x = x0[b].copy()
    xbar = np.zeros((N + 1, 6))
    xbar[:, 0] = 0.1
    ubar = np.zeros((N, 2))
    S = int(qp["kin_sqp"])
    log = []
    for k in range(steps):
        ds, kap = horizon_params(np.array([x[2]]), xbar[None, :, 0], float(cfg["mpc_dt"]), tr.k)
        if dump is not None and k in dump:
            np.savez(f"/tmp/kin_step_s{seed}_v{b}_k{k}.npz", x0=x, ubar=ubar, xbar=xbar, kappa=kap[0], ds=ds[0],
                     W=repr({kk: v for kk, v in W.items() if kk != "obstacles"}), S=S)
        r = KS.kin_sqp_solve(x[None], ubar[None], kap, ds, 2.5, W, S, x_ws=xbar[None] if qp.get("ms") else None,
                             elastic=float(qp.get("elastic", 0.0)), max_iter=200)
        h0 = r["hist"][0]
        ok0 = bool(h0["qp_ok"][0])
        restarted = bool(h0.get("restart", np.zeros(1, bool))[0])
        ok = ok0 or (restarted and len(r["hist"]) > 1 and bool(r["hist"][1]["qp_ok"][0]))
        u = r["u_star"][0]
        xs = r["x_star"][0]
        if ok:
            u0 = u[0].copy()
            ubar, xbar = u.copy(), xs.copy()
            if qp.get("shift"):
                ubar[:-1] = ubar[1:].copy()
                xbar[:-1] = xbar[1:].copy()
        else:
            u0 = np.zeros(2)
        kap0 = float(tr.k(np.array([x[2]]))[0])
        x = M.kin_transition(x, u0, kap0, 0.05, 2.5)
        if not ok:
            ubar = np.zeros((N, 2))
            xbar = np.repeat(x[None], N + 1, axis=0)
        alphas = [float(h["alpha"][0]) for h in r["hist"]]
        log.append(dict(k=k, ok=ok, ok0=ok0, restart=restarted, x=x.copy(), u0=u0, alphas=alphas))
        if verbose:
            print(f"v{b} step {k:3d} {'ok ' if ok else 'NS '} first-QP {'ok' if ok0 else 'FAIL'}"
                  f"{' restart' if restarted else ''} | v {x[0]:.2f} d {x[1]:+.3f} s {x[2]:.1f} ey {x[3]:+.2f} "
                  f"ep {x[4]:+.3f} | u0 {u0[0]:+.2f} {u0[1]:+.3f} | alpha {alphas}", flush=True)
    return b, log


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--vehicles", type=int, nargs="+", default=[42])
    ap.add_argument("--N", type=int, default=50)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--qp", nargs="*", default=[])
    ap.add_argument("--dump", type=int, nargs="*", default=None, help="save the solver inputs of these steps")
    a = ap.parse_args()
    qp = {k: float(v) if "." in v or "e" in v else int(v) for k, v in (kv.split("=") for kv in a.qp)}
    t0 = time.time()
    jobs = [(a.seed, b, a.N, a.steps, qp, a.workers == 1, a.dump) for b in a.vehicles]
    if a.workers > 1:
        from multiprocessing import Pool
        with Pool(a.workers) as p:
            res = p.map(run_vehicle, jobs)
    else:
        res = [run_vehicle(j) for j in jobs]
    for b, log in res:
        ey = np.array([r["x"][3] for r in log])
        ns = sum(not r["ok"] for r in log)
        print(f"vehicle {b}: non-solved {ns}/{len(log)}, max |ey| {np.abs(ey).max():.2f}, s_end {log[-1]['x'][2]:.1f}")
    print(f"{time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
