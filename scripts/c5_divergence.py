"""Find the C5 vehicles that leave the track and record their history.

Runs the bench's C5 job once (8192 vehicles x 500 steps on ippodromo, the same seeds as
bench.py run_c5), picks every vehicle whose |ey| exceeds width/2, then re-runs only those
vehicles one step per vc_simulate call (K steps in one call = K one-step calls bit for
bit, and vehicles are independent) to log per step: plant state, applied u0, the warm
start (xbar, ubar) the solve started from, and whether the step was non-solved.
Writes gpurun_out/c5_div.npz and prints a summary.

    python scripts/c5_divergence.py [--vehicles 8192] [--steps 500]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vehicles", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--seed", type=int, default=31)
    ap.add_argument("--fp32", action="store_true", help="fp32 solve (dyn_sqp.hip) instead of fp64 (st_sqp.hip)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "c5_div.npz"))
    args = ap.parse_args()
    import torch

    from vcmpc import _abi
    from vcmpc.config import load_config
    from vcmpc.environment import Track
    from vcmpc.models import DynamicCar
    from vcmpc.simulation import BatchedRacingSimulator
    from vcmpc.workload import C5_MPC_DT, closed_loop_states

    track = Track.load("ippodromo")
    x_all = closed_loop_states(args.vehicles, track.length, seed=args.seed)
    cfg = load_config("dynamic_mpc")
    cfg["mpc_dt"] = C5_MPC_DT
    car = DynamicCar(load_config("dynamic_car"), track, tyre="fiala")
    B, K = args.vehicles, args.steps
    dt = _abi.VC_F32 if args.fp32 else _abi.VC_F64
    sim = BatchedRacingSimulator(car, cfg, track, batch=B, device=0, dtype=dt)
    sim.reset(x_all)
    sim._init_warm_start(args.seed)
    xb0, ub0 = sim.xbar.clone(), sim.ubar.clone()
    sim.nfail.zero_()
    log_x, _, nfail = sim.ctx.simulate(sim.x, sim.xbar, sim.ubar, K, sim.mpc_dt, sim.dt, log=True, nfail=sim.nfail)
    torch.cuda.synchronize()
    ey = log_x[:, :, 5].abs()
    half = track.width / 2
    bad = torch.nonzero(ey.max(0).values >= half).flatten().cpu().numpy()
    print(f"full run: {B} vehicles x {K} steps, {len(bad)} leave the track (|ey| >= {half}); "
          f"max |ey| {float(ey.max()):.2f}; non-solved steps {int(nfail.sum())}", flush=True)
    full_x = log_x[:, bad].cpu().numpy()
    nfail_full = nfail[bad].cpu().numpy()
    del log_x
    if len(bad) == 0:
        np.savez(args.out, bad=bad)
        return
    nb = len(bad)
    sub = BatchedRacingSimulator(car, cfg, track, batch=nb, device=0, dtype=dt)
    sub.reset(x_all[bad])
    sub.xbar.copy_(xb0[bad])
    sub.ubar.copy_(ub0[bad])
    sub.nfail.zero_()
    X = np.zeros((K + 1, nb, 8))
    U = np.zeros((K, nb, 2), np.float32)
    XB = np.zeros((K, nb) + tuple(sub.xbar.shape[1:]), np.float32)
    UB = np.zeros((K, nb) + tuple(sub.ubar.shape[1:]), np.float32)
    NF = np.zeros((K, nb), np.int32)
    X[0] = sub.x.cpu().numpy()
    for k in range(K):
        XB[k] = sub.xbar.cpu().numpy()
        UB[k] = sub.ubar.cpu().numpy()
        before = sub.nfail.clone()
        lx, lu, nf = sub.ctx.simulate(sub.x, sub.xbar, sub.ubar, 1, sub.mpc_dt, sub.dt, log=True, nfail=sub.nfail)
        torch.cuda.synchronize()
        X[k + 1] = lx[1].cpu().numpy()
        U[k] = lu[0].cpu().numpy()
        NF[k] = (nf - before).cpu().numpy()
    same = np.array_equal(X, full_x)
    print(f"subset rerun reproduces the full run bit for bit: {same} (max diff {np.abs(X - full_x).max():.3e})")
    for j, b in enumerate(bad):
        e = np.abs(X[:, j, 5])
        first = int(np.argmax(e >= half))
        fails = np.nonzero(NF[:, j])[0]
        print(f"vehicle {b}: x0 {np.array2string(x_all[b], precision=3)}; |ey| >= {half} first at step {first} "
              f"(s = {X[first, j, 4]:.1f}, Ux = {X[first, j, 0]:.2f}); non-solved steps {len(fails)} "
              f"(first {fails[:10].tolist()}), nfail full run {nfail_full[j]}")
        lo = max(0, first - 12)
        for k in range(lo, min(first + 3, K)):
            print(f"   step {k:3d}: Ux {X[k, j, 0]:6.2f} Uy {X[k, j, 1]:6.2f} r {X[k, j, 2]:6.3f} "
                  f"delta {X[k, j, 3]:6.3f} s {X[k, j, 4]:7.2f} ey {X[k, j, 5]:6.2f} epsi {X[k, j, 6]:6.3f} "
                  f"| u0 Fx {U[k, j, 0]:8.1f} w {U[k, j, 1]:6.3f} | fail {NF[k, j]}")
    np.savez_compressed(args.out, bad=bad, x0=x_all[bad], X=X, U=U, XB=XB, UB=UB, NF=NF,
                        xbar0=xb0[bad].cpu().numpy(), ubar0=ub0[bad].cpu().numpy())
    print(f"wrote {args.out}")


if __name__ == "__main__":
    main()
