"""Diagnostics of the stagewise kinematic kernel (csrc/kin_ric.hip): per-problem errors vs
the oracle with the solver diagnostics (diag: residual, mu, flags 1 fail / 2 IPM converged /
4 polished / 8 polish factorisation failed, polish rounds), and the kinematic closed loop at
N = 20 (both kernels) and N = 50.

    python scripts/kin_ric_diag.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]

from oracle import ltv_qp as Q  # noqa: E402


def ctx(N, B, solver=1, qp=None):
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    cfg = load_config("kinematic_mpc")
    cfg["qp"] = dict(cfg.get("qp") or {}, solver=solver, **(qp or {}))
    p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=cfg)
    return Context(model=_abi.VC_MODEL_KINEMATIC, N=N, max_batch=B, dtype=_abi.VC_F64, params=p)


def main():
    from vcmpc.config import load_config
    from vcmpc.workload import kinematic_batch
    W = Q.kin_weights(load_config("kinematic_mpc"))
    np.set_printoptions(precision=3, linewidth=160)
    for N, B, seed in ((60, 24, 360), (50, 24, 350)):
        d = kinematic_batch(B, N=N, seed=seed)
        ref = Q.kin_ltv_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], 2.5, W)
        with ctx(N, B) as c:
            u0, xs, us, st, it, dg = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
        e = np.abs(us - ref["u_star"]).max(axis=(1, 2))
        print(f"== N={N}: worst problems")
        for b in np.argsort(-e)[:5]:
            print(f"   b={b} err {e[b]:.2e} status {st[b]} iters {it[b]} diag {dg[b]}", flush=True)
    d = kinematic_batch(8192, N=50, seed=77)
    with ctx(50, 8192) as c:
        u0, xs, us, st, it, dg = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
    bad = np.nonzero(st != 0)[0]
    print(f"== N=50 B=8192: non-solved {bad.tolist()}")
    for b in bad[:5]:
        print(f"   b={b} status {st[b]} iters {it[b]} diag {dg[b]}")
        ref = Q.kin_ltv_solve(d["x0"][b:b + 1], d["ubar"][b:b + 1], d["kappa"][b:b + 1], d["ds"][b:b + 1], 2.5, W)
        print(f"   err vs oracle {np.abs(us[b] - ref['u_star'][0]).max():.2e}, oracle polished {ref['polished']}")
    fl = dg[:, 2].astype(int)
    print(f"   flags: polished {(fl & 4 > 0).mean():.4f} ipm-conv {(fl & 2 > 0).mean():.4f} "
          f"fail {(fl & 1 > 0).mean():.4f} polish-fact-fail {(fl & 8 > 0).mean():.4f}; rounds max {dg[:, 3].max()}")
    # closed loop
    from vcmpc.environment import Track
    from vcmpc.models import KinematicCar
    from vcmpc.simulation import BatchedRacingSimulator
    track = Track.load("ippodromo")
    car = KinematicCar(load_config("kinematic_car"), track)
    Bv, K = 64, 200
    rng = np.random.default_rng(3)
    x0 = np.zeros((Bv, 6))
    x0[:, 0] = rng.uniform(4, 9, Bv)
    x0[:, 2] = rng.uniform(0, track.length, Bv)
    x0[:, 3] = rng.uniform(-1.5, 1.5, Bv)
    for N, solver, qp, neutral in ((20, 0, {}, False), (50, 1, {}, False), (50, 1, {}, True),
                                   (50, 1, {"trust_a": 3.0, "trust_w": 0.4}, True),
                                   (50, 1, {"trust_a": 0.0, "trust_w": 0.0}, True),
                                   (50, 1, {"trust_a": 0.5, "trust_w": 0.05}, True),
                                   (30, 1, {"trust_a": 0.0, "trust_w": 0.0}, True)):
        cfg = load_config("kinematic_mpc")
        cfg["horizon"] = N
        cfg["qp"] = dict(cfg.get("qp") or {}, solver=solver, **qp)
        sim = BatchedRacingSimulator(car, cfg, track, batch=Bv)
        if neutral:  # first guess: ubar = 0, xbar = the start state (the restart's neutral warm start)
            sim.ubar.zero_()
            sim.xbar.copy_(sim.torch.from_numpy(np.repeat(x0[:, None, :], N + 1, axis=1)).cuda())
        out = sim.reset(x0).run(K)
        X = out["state_traj"]
        print(f"== closed loop N={N} solver={solver} qp={qp} neutral={neutral}: max |ey| {np.abs(X[:, :, 3]).max():.2f}, "
              f"non-solved {out['nfail'].sum()}, off-track vehicles {(np.abs(X[:, :, 3]).max(0) >= track.width / 2).sum()}, "
              f"median progress {np.median(X[-1, :, 2] - X[0, :, 2]):.1f} m, max |delta| {np.abs(X[:, :, 1]).max():.3f}",
              flush=True)
        if False:
            # one-step re-runs of the first failing vehicle: diag of its solves
            bad = np.nonzero(out["nfail"])[0]
            if len(bad):
                b = int(bad[0])
                sub = BatchedRacingSimulator(car, cfg, track, batch=1)
                sub.reset(x0[b:b + 1])
                for k in range(40):
                    xcur = sub.states.copy()
                    xb = sub.state_prediction.copy()
                    ub = sub.action_prediction.copy()
                    r = sub.run(1)
                    if r["nfail"].sum():
                        from vcmpc.environment import Track as _T  # noqa: F401
                        ds, kap = Q.kin_horizon_params(xcur[0], xb[0], cfg["mpc_dt"], N, track.k)
                        with ctx(N, 1, qp={"trust_a": 1.0, "trust_w": 0.1}) as c:
                            res = c.solve(xcur[:, :6].copy(), kap[None], ds[None], np.swapaxes(ub, 1, 2).copy(),
                                          diag=True)
                        print(f"   vehicle {b} step {k}: x {xcur[0]} status {res[3]} iters {res[4]} diag {res[5]}")
                        break


if __name__ == "__main__":
    main()
