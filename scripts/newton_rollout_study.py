"""Chord-Newton rollout study (csrc/st_sqp.hip ST_NEWTON_ROLLOUT): for the SQP steps the oracle takes
on C3 problems, how many stage-parallel defect evaluations re-roll x = rollout(u + du) from the
pre-step trajectory with the pre-step Jacobians A_k, to defects <= 1e-14 relative (99 = not within
12).  usage: python scripts/newton_rollout_study.py"""
import sys, numpy as np
sys.path[:0] = ['.', 'vehicle-control_amd']
from oracle import dyn_sqp as D
from oracle import models as M
from vcmpc.config import load_config
from vcmpc.workload import dynamic_batch
p = M.dyn_params_from_config(load_config("dynamic_car"))
for tyre, cfgn in (("linear", "dynamic_mpc"), ("fiala", "dynamic_mpc")):
    B = 16
    d = dynamic_batch(B, N=40, seed=31, tyre=tyre)
    x0, ub, kap, ds = (np.asarray(d[k], np.float64) for k in ("x0", "ubar", "kappa", "ds"))
    W = D.dyn_weights(load_config(cfgn))
    W["sqp_iters"] = 5
    out = D.dyn_sqp_solve(x0, ub, kap, ds, p, W, tyre=tyre, keep_qps=True)
    N = ub.shape[1]
    counts = []
    for i, rec in enumerate(out["hist"]):
        u_old = rec["ubar"]
        u_new = out["hist"][i + 1]["ubar"] if i + 1 < len(out["hist"]) else out["u_star"]
        xb0, A = rec["xbar"], rec["A"]
        xtrue = D.dyn_predict(x0, u_new, kap, ds, p, tyre)
        x = xb0.copy(); n_it = np.full(B, 99)
        for it in range(12):
            Fx = D.spatial_step(x[:, :N-1], u_new[:, :N-1], kap[:, :N-1], ds[:, :N-1], p, tyre)
            c = Fx - x[:, 1:]
            cm = np.abs(c).max(axis=(1, 2)) / (1 + np.abs(x).max(axis=(1, 2)))
            n_it = np.where((n_it == 99) & (cm <= 1e-14), it, n_it)
            dl = np.zeros((B, 8))
            for k in range(N - 1):
                dl = c[:, k] + np.einsum("bij,bj->bi", A[:, k], dl)
                x[:, k + 1] += dl
        du = np.abs(u_new - u_old).max(axis=1)
        counts.append(n_it)
        print(f"{tyre} SQP step {i+1}: |dFx| max {du[:,0].max():.0f} |dw| max {du[:,1].max():.3f}; "
              f"defect evaluations to 1e-14: {n_it.tolist()}", flush=True)
