"""CPU prototype of the kinematic closed loop with obstacles through the oracle (the loop of
tests/test_gpu_obstacles.py::test_kinematic_closed_loop_with_obstacles on a few vehicles):
one LTV-QP step per control step (the round-1 contract) vs the globalised SQP with the merit
line search of oracle/kin_sqp.py.  Reports collisions, off-track excursions and failed steps.

    python scripts/kin_obs_cpu_loop.py [--B 8] [--steps 400] [--sqp 1 3] [--no-ls]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--sqp", type=int, default=3)
    ap.add_argument("--no-ls", action="store_true", help="take the full QP step (alpha = 1)")
    ap.add_argument("--trust", default="rti", help="rti (1.0 / 0.1) or off")
    ap.add_argument("--N", type=int, default=0)
    ap.add_argument("--vehicle", type=int, default=-1, help="run only this vehicle of the 64 and trace it")
    ap.add_argument("--elastic", action="store_true", help="elastic state rows (oracle/kin_sqp.py elastic_qp_step)")
    ap.add_argument("--no-obstacles", action="store_true")
    args = ap.parse_args()
    from oracle import kin_sqp as KS
    from oracle import ltv_qp as Q
    from oracle import models as M
    from vcmpc.config import load_config
    from vcmpc.controllers.kinematic_mpc import RTI_TRUST
    from vcmpc.environment import Track
    tr = Track.load("ippodromo")
    obs = [(o.s, o.ey, o.radius) for o in tr.obstacles]
    kc = load_config("kinematic_car")
    L = 2.5
    dt = float(kc.get("dt", 0.05)) if hasattr(kc, "get") else 0.05
    cfg = load_config("kinematic_mpc")
    if args.N:
        cfg["horizon"] = args.N
    N, mpc_dt = cfg["horizon"], cfg["mpc_dt"]
    W = Q.kin_weights(cfg)
    if args.trust == "rti":
        W.update(RTI_TRUST)
    W["obstacles"] = [] if args.no_obstacles else obs
    rng = np.random.default_rng(3)
    B0 = 64
    x0 = np.zeros((B0, 6))
    x0[:, 0] = rng.uniform(5, 8, B0)
    x0[:, 2] = rng.uniform(0, 15, B0)
    x0[:, 3] = rng.uniform(-0.5, 0.5, B0)
    B = args.B
    x = x0[:B].copy()
    if args.vehicle >= 0:
        B = 1
        x = x0[args.vehicle:args.vehicle + 1].copy()
    ub = np.zeros((B, N, 2))
    xb = np.repeat(x[:, None, :], N + 1, axis=1)
    X = [x.copy()]
    nfail = np.zeros(B, int)
    alphas = []
    t0 = time.time()
    for k in range(args.steps):
        ds = np.zeros((B, N))
        kap = np.zeros((B, N))
        for b in range(B):
            ds[b], kap[b] = Q.kin_horizon_params(x[b], xb[b].T, mpc_dt, N, tr.k)
        u = ub.copy()
        fail = np.zeros(B, bool)
        for it in range(args.sqp):
            if args.elastic:
                ustar, kkt, _ = KS.elastic_qp_step(x, u, kap, ds, L, W)
            else:
                sol = Q.kin_ltv_solve(x, u, kap, ds, L, W)
                ustar, kkt = sol["u_star"], sol["kkt"]
            bad = (kkt["pfeas"] > 1e-6) | ~np.isfinite(ustar).all(axis=(1, 2))
            fail |= bad
            dz = np.where(bad[:, None, None], 0.0, ustar - u)
            if args.no_ls:
                alpha = np.ones(B)
            else:
                alpha = KS.line_search(x, u, dz, kap, ds, L, W)[0]
            alphas.append(alpha)
            u = u + alpha[:, None, None] * dz
        xs = Q.kin_predict(x, u, kap, ds, L)
        u0 = np.where(fail[:, None], 0.0, u[:, 0])
        ub = np.where(fail[:, None, None], 0.0, u)
        xb = np.where(fail[:, None, None], np.repeat(x[:, None, :], N + 1, axis=1), xs)
        nfail += fail
        if args.vehicle >= 0:
            print(f"step {k:3d}: v {x[0, 0]:6.2f} delta {x[0, 1]:+.3f} s {x[0, 2]:7.2f} ey {x[0, 3]:+7.2f} "
                  f"epsi {x[0, 4]:+.3f} | u0 ({u0[0, 0]:+.2f}, {u0[0, 1]:+.3f}) fail {int(fail[0])} "
                  f"alphas {[float(a[0]) for a in alphas[-args.sqp:]]} pred ey [{xs[0, :, 3].min():+.2f}, "
                  f"{xs[0, :, 3].max():+.2f}] pred s [{xs[0, 0, 2]:.1f}, {xs[0, -1, 2]:.1f}]", flush=True)
        kk = np.asarray(tr.k(x[:, 2]), np.float64)
        x = M.kin_transition(x, u0, kk, dt, L)
        X.append(x.copy())
    X = np.array(X)
    clear = np.min([np.hypot(X[..., 2] - so, X[..., 3] - eo) - r for so, eo, r in obs], axis=0)
    al = np.array(alphas)
    print(f"N={N} elastic={args.elastic} obstacles={not args.no_obstacles} trust={args.trust} sqp={args.sqp} ls={not args.no_ls} B={B} steps={args.steps} ({time.time() - t0:.0f} s): "
          f"vehicles hitting an obstacle {(clear < 0).any(0).sum()}, min clearance {clear.min(0).round(2).tolist()}, "
          f"max |ey| {np.abs(X[..., 3]).max(0).round(2).tolist()}, failed steps {nfail.tolist()}, "
          f"final s {X[-1, :, 2].round(1).tolist()}, alpha<1 fraction {np.mean(al < 1):.3f}, alpha=0 {np.mean(al == 0):.3f}")


if __name__ == "__main__":
    main()
