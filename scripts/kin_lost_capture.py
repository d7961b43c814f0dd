"""Capture the full closed-loop history of the vehicles the kinematic obstacle loop loses
(GPU diagnostic for VERDICT r03 "next" item 1).

Runs tests/test_gpu_obstacles.py's long-horizon loop (ippodromo, 64 vehicles, 400 steps,
obstacles on, N = 50 by default) one control step at a time for each seed, records every
vehicle's solver inputs before each step (plant state x0, warm start xbar / ubar, the
horizon parameters kappa / ds that vc_horizon derives from them) and whether the step was
non-solved, then keeps the histories of the vehicles with a non-solved step or |ey| beyond
the track (width / 2).  The CPU replay (scripts/kin_lost_replay.py) re-solves those steps
with the oracle.

    python scripts/kin_lost_capture.py --seeds 5 11 [--N 50] --out gpurun_out/kin_lost
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))


def x0_batch(seed, B=64):
    rng = np.random.default_rng(seed)
    x0 = np.zeros((B, 6))
    x0[:, 0] = rng.uniform(5, 8, B)
    x0[:, 2] = rng.uniform(0, 15, B)
    x0[:, 3] = rng.uniform(-0.5, 0.5, B)
    return x0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=50)
    ap.add_argument("--seeds", type=int, nargs="+", default=[5, 11])
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--qp", nargs="*", default=[])
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    from vcmpc.config import load_config
    from vcmpc.environment import Track
    from vcmpc.models import KinematicCar
    from vcmpc.simulation import BatchedRacingSimulator
    qp = {k: float(v) if "." in v or "e" in v else int(v) for k, v in (kv.split("=") for kv in a.qp)}
    tr = Track.load("ippodromo")
    B, K = 64, a.steps
    os.makedirs(a.out, exist_ok=True)
    for seed in a.seeds:
        t0 = time.time()
        cfg = load_config("kinematic_mpc")
        cfg["obstacles"] = True
        cfg["horizon"] = a.N
        if qp:
            cfg["qp"] = dict(cfg.get("qp") or {}, **qp)
        car = KinematicCar(load_config("kinematic_car"), tr)
        sim = BatchedRacingSimulator(car, cfg, tr, batch=B, use_torch=False)
        sim.reset(x0_batch(seed, B))
        N = a.N
        X = np.zeros((K + 1, B, 6))
        XB = np.zeros((K, B, N + 1, 6))
        UB = np.zeros((K, B, N, 2))
        KAP = np.zeros((K, B, N))
        DS = np.zeros((K, B, N))
        UOUT = np.zeros((K, B, N, 2))   # the warm start after the step (shifted when vc_qp.shift)
        FAIL = np.zeros((K, B), bool)
        prev = np.zeros(B, np.int64)
        X[0] = sim.states
        for k in range(K):
            XB[k] = np.array(sim.xbar, copy=True)
            UB[k] = np.array(sim.ubar, copy=True)
            kap, ds = sim.ctx.horizon(X[k].copy(), XB[k].copy(), sim.mpc_dt)
            KAP[k], DS[k] = kap, ds
            out = sim.run(1, log=False)
            nf = out["nfail"].astype(np.int64)
            FAIL[k] = nf > prev
            prev = nf
            X[k + 1] = sim.states
            UOUT[k] = np.array(sim.ubar, copy=True)
            if k % 50 == 49:
                print(f"  seed {seed} step {k + 1}: non-solved so far {int(FAIL.sum())} ({time.time() - t0:.1f} s)",
                      flush=True)
        ey = np.abs(X[:, :, 3])
        keep = np.nonzero(FAIL.any(axis=0) | (ey.max(axis=0) > tr.width / 2 + 0.5))[0]
        print(f"seed {seed}: non-solved {int(FAIL.sum())} of {B * K}, max |ey| {ey.max():.2f}, "
              f"kept vehicles {keep.tolist()} ({time.time() - t0:.1f} s)", flush=True)
        for b in keep:
            fs = np.nonzero(FAIL[:, b])[0]
            off = np.nonzero(ey[:, b] > tr.width / 2)[0]
            print(f"   vehicle {b}: {len(fs)} non-solved (first {fs[:8].tolist()}), first off-track step "
                  f"{off[0] if len(off) else -1}, max |ey| {ey[:, b].max():.2f}", flush=True)
        np.savez_compressed(os.path.join(a.out, f"seed{seed}_N{N}.npz"), vehicles=keep, X=X[:, keep],
                            XB=XB[:, keep], UB=UB[:, keep], KAP=KAP[:, keep], DS=DS[:, keep],
                            UOUT=UOUT[:, keep], FAIL=FAIL[:, keep], fail_all=FAIL, ey_all=X[:, :, 3],
                            s_all=X[:, :, 2], seed=seed, N=N, qp=str(qp))


if __name__ == "__main__":
    main()
