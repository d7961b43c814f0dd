"""Open-loop replay of the reference's recorded closed-loop runs through the drop-in
controllers (tests/golden/replay_kat.npz, make_replay_kat.py): at every recorded control step
the controller gets the recorded state (and its own previous solution as the unshifted warm
start, as the reference's controller does), and its first input is compared with the input
IPOPT computed there (action_traj[n + 1]: racing.py:77-84 logs a zero action first and then
the command made from state_traj[n] at :230-237), its plan with IPOPT's recorded plan (global x, y per stage).

If the build's SQP converges to the same local optimum of the NLP as IPOPT, the two agree
to solver tolerance; the script sweeps the SQP iteration count.

    python scripts/replay_recorded.py [--sqp 3 5 10 20] [--runs cascaded7_ippodromo]
"""
import argparse
import copy
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]


def track_of(run):
    """The recorded run's track: the experiment directory's suffix (<name>_<track>[:<ctl>])."""
    return run.split(":")[0].rsplit("_", 1)[1]


def config_for(run, rec):
    """The build's config (its `qp` block) with the recorded run's horizons, weights, bounds and
    obstacle switch (the barrier then uses the run's track's obstacle_data, cascaded_mpc.py:173-176)."""
    from vcmpc.config import load_config
    cfg = copy.deepcopy(load_config("cascaded_mpc" if rec.get("horizon_pm", 0) else "singletrack_mpc"))
    for k in ("horizon", "mpc_dt", "horizon_pm", "ds_pm", "obstacles"):
        if k in rec:
            cfg[k] = rec[k]
    for k in ("cost_weights", "input_constraints", "state_constraints", "state_pm_constraints"):
        if k in rec:
            cfg[k] = dict(cfg.get(k) or {}, **rec[k])
    return cfg


def replay(run, g, rec, sqp, skip=5, qp=None, dump=None, segments=1, cfg_extra=None):
    """segments > 1: the run's T steps are cut into that many contiguous windows, replayed side
    by side as one batch (each window starts from the controller's own initial guess, so its
    first `skip` steps are the warm-up and are not compared) -- the same per-step comparison
    in T / segments sequential solves."""
    from vcmpc.config import load_config
    from vcmpc.controllers.cascaded_mpc import BatchedCascadedMPC, BatchedSingleTrackMPC
    from vcmpc.environment import Track
    from vcmpc.models import DynamicCar
    track = Track.load(track_of(run))
    car = DynamicCar(load_config("dynamic_car"), track, tyre="fiala")
    cfg = config_for(run, rec)
    cfg.update(cfg_extra or {})   # e.g. obstacle_inside (vc_obstacles.inside: the reference's barrier inside)
    cfg["qp"] = dict(cfg["qp"], sqp_iters=sqp, **(qp or {}))
    X, U, P = g[f"{run}/state_traj"], g[f"{run}/action_traj"], g[f"{run}/preds"]
    T = min(len(X), len(U))
    K = max(1, min(int(segments), T // (4 * skip + 1)))
    bounds = np.linspace(0, T, K + 1).astype(int)
    ctl = (BatchedCascadedMPC if cfg.get("horizon_pm", 0) else BatchedSingleTrackMPC)(car, cfg, batch=K)
    N = int(cfg["horizon"])
    du, dplan, rel_u, nfail, dbg = [], [], [], 0, None
    us = np.full((T, 2), np.nan)
    rec_nan = own_nan = nonfinite = 0
    st_counts = {}
    for j in range(int(np.max(np.diff(bounds)))):
        idx = np.minimum(bounds[:-1] + j, bounds[1:] - 1)          # a finished window repeats its last row
        live = bounds[:-1] + j < bounds[1:]
        u = ctl.command(X[idx])
        for k in np.nonzero(live)[0]:
            n = int(idx[k])
            us[n] = u[k]
            nfail += int(ctl.status[k] != 0)
            st_counts[int(ctl.status[k])] = st_counts.get(int(ctl.status[k]), 0) + 1
            # the controller's output and its next warm start are finite at every step
            nonfinite += int(not (np.isfinite(u[k]).all() and np.isfinite(ctl.state_prediction[k]).all()
                                  and np.isfinite(ctl.action_prediction[k]).all()))
            if j < skip:
                continue
            if n + 1 < len(U):   # racing.py:230-241: action_traj[n + 1] is the command at state_traj[n]
                du.append(u[k] - U[n + 1])
                rel_u.append(U[n + 1])
            if n < len(P):
                sp = ctl.state_prediction[k]
                xy = np.array([track.rel2glob(sp[4, i], sp[5, i], sp[6, i])[:2] for i in range(min(N, 20))])
                # the recorded plans hold NaN past the reference track's spline range (its k / x / y
                # do not wrap; e.g. cascaded7 step 406, stages >= 17): compare on the recorded stages
                # that exist, and count our own non-finite plans separately
                rec_ok = np.isfinite(P[n, :len(xy)]).all(axis=1)
                rec_nan += int(not rec_ok.all())
                own_nan += int(not np.isfinite(xy).all())
                dplan.append(np.hypot(*(xy[rec_ok] - P[n, :len(xy)][rec_ok]).T).max())
                if dbg is None and n >= 50:
                    dbg = dict(step=n, ours=xy[:3].tolist(), recorded=P[n, :3].tolist())
    du, dplan = np.abs(np.array(du)), np.array(dplan)
    if dump:   # per-step arrays for a closer look (our u0, the recorded command, the state)
        np.savez(dump, u=us, U=U, X=X, du=du, dplan=dplan, skip=skip, bounds=bounds)
    rel = du / np.maximum(np.abs(np.array(rel_u)), [100.0, 0.01])
    return dict(run=run, sqp=sqp, qp=cfg["qp"], steps=len(du), segments=K, nonsolved=nfail,
                nonfinite_steps=nonfinite, status_counts={str(k): v for k, v in sorted(st_counts.items())},
                obstacles=bool(cfg.get("obstacles")), track=track_of(run),
                dFx_median=float(np.median(du[:, 0])), dFx_p90=float(np.percentile(du[:, 0], 90)),
                dFx_max=float(du[:, 0].max()), dw_median=float(np.median(du[:, 1])),
                dw_p90=float(np.percentile(du[:, 1], 90)), dw_max=float(du[:, 1].max()),
                plan_dev_median_m=float(np.nanmedian(dplan)), plan_dev_p90_m=float(np.nanpercentile(dplan, 90)),
                plan_nan_steps=int(np.isnan(dplan).sum()) + own_nan, recorded_plan_nan_steps=rec_nan,
                Fx_scale=float(np.abs(U[:, 0]).max()), w_scale=float(np.abs(U[:, 1]).max()),
                frac_within_1pct=float(np.mean((rel < 0.01).all(axis=1))), example_plan=dbg)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sqp", type=int, nargs="+", default=[3, 5, 10, 20])
    ap.add_argument("--runs", nargs="+", default=["cascaded7_ippodromo", "singletrack_ippodromo"],
                    help="fixture keys (tests/golden/make_replay_kat.py), or 'all'")
    ap.add_argument("--out", default=None)
    ap.add_argument("--prox", type=float, nargs="+", default=[None], help="override qp.prox (sweep)")
    ap.add_argument("--dump", default=None, help="npz prefix for per-step arrays")
    ap.add_argument("--segments", type=int, default=1, help="replay windows side by side (see replay())")
    ap.add_argument("--inside", action="store_true", help="the reference's barrier inside obstacles (vc_obstacles.inside)")
    ap.add_argument("--table", action="store_true", help="print a markdown table of the results at the end")
    args = ap.parse_args()
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "replay_kat.npz"), allow_pickle=False))
    recs = json.loads(str(g["configs"]))
    res = []
    for run in (sorted(recs) if args.runs == ["all"] else args.runs):
        for prox in args.prox:
            for sqp in args.sqp:
                r = replay(run, g, recs[run], sqp, qp=None if prox is None else {"prox": prox},
                           dump=None if args.dump is None else f"{args.dump}_{run}_p{prox}_s{sqp}.npz",
                           segments=args.segments, cfg_extra={"obstacle_inside": True} if args.inside else None)
                res.append(r)
                print(json.dumps({k: v for k, v in r.items() if k != "example_plan"}), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    if args.table:
        print("| run | steps | non-solved | median \\|ΔFx\\| [N] | median \\|Δw\\| [rad/s] | within 1 % | plan dev median [m] |")
        print("|---|---|---|---|---|---|---|")
        for r in res:
            print(f"| {r['run']} | {r['steps']} | {r['nonsolved']} | {r['dFx_median']:.3g} | {r['dw_median']:.2g} | "
                  f"{100 * r['frac_within_1pct']:.1f} % | {r['plan_dev_median_m']:.2g} |")


if __name__ == "__main__":
    main()
