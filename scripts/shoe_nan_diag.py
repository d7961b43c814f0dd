"""Find the first non-finite output in the race_obstacles_shoe single-track replay.

Runs scripts/replay_recorded.py's replay loop with the controller's Context.solve wrapped: every
solve call (the first solve and the neutral re-solve of BatchedSingleTrackMPC.command) is
re-issued through vc_solve_diag, and the first problem whose u0 / u* / x* holds a non-finite value
(or a finite x* with |Ux| > 200 m/s or Ux <= 0: the next step's ds = mpc_dt * Ux) is reported with its window, step, recorded state, status and diag row, for both calls.

    python scripts/shoe_nan_diag.py [--inside] [--run race_obstacles_shoe:singletrack] [--out f.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd"), os.path.join(ROOT, "scripts")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--run", default="race_obstacles_shoe:singletrack")
    ap.add_argument("--inside", action="store_true")
    ap.add_argument("--sqp", type=int, default=40)
    ap.add_argument("--segments", type=int, default=24)
    ap.add_argument("--out", default=None)
    ap.add_argument("--max-events", type=int, default=8)
    args = ap.parse_args()

    import replay_recorded as R
    from vcmpc import solver

    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "replay_kat.npz"), allow_pickle=False))
    recs = json.loads(str(g["configs"]))
    events, absurd, calls = [], [], {"n": 0}
    orig = solver.Context.solve

    def solve(self, x0, kappa, ds, ubar, *a, **kw):
        ub_in = np.array(ubar, copy=True)
        u0, xbar, ustar, status, iters, diag = orig(self, x0, kappa, ds, ubar, diag=True)
        calls["n"] += 1
        for b in range(len(status)):
            ux = np.asarray(xbar[b])[:, 0]
            if np.isfinite(ux).all() and (np.abs(ux).max() > 200 or ux.min() <= 0) and len(absurd) < args.max_events:
                absurd.append(dict(call=calls["n"], row=b, status=int(status[b]), iters=int(iters[b]),
                                   diag=diag[b].tolist(), x0=np.asarray(x0[b]).tolist(), ux=ux.tolist(),
                                   ustar=np.asarray(ustar[b]).tolist(), ubar_in=ub_in[b].tolist(),
                                   ds=np.asarray(ds[b]).tolist(), kappa=np.asarray(kappa[b]).tolist()))
            fin = dict(u0=bool(np.isfinite(u0[b]).all()), ustar=bool(np.isfinite(ustar[b]).all()),
                       xstar=bool(np.isfinite(xbar[b]).all()))
            if not all(fin.values()) and len(events) < args.max_events:
                events.append(dict(call=calls["n"], row=b, status=int(status[b]), iters=int(iters[b]),
                                   diag=diag[b].tolist(), finite=fin, x0=np.asarray(x0[b]).tolist(),
                                   ubar_in_finite=bool(np.isfinite(ub_in[b]).all()),
                                   kappa_finite=bool(np.isfinite(kappa[b]).all()),
                                   ds_finite=bool(np.isfinite(ds[b]).all()),
                                   ds_min=float(np.min(ds[b])),
                                   first_bad_stage=int(np.argmax(~np.isfinite(xbar[b]).all(axis=1)))))
        return u0, xbar, ustar, status, iters

    solver.Context.solve = solve
    err = None
    try:
        r = R.replay(args.run, g, recs[args.run], args.sqp, qp={"prox": 0.01}, segments=args.segments,
                     cfg_extra={"obstacle_inside": True} if args.inside else None)
        r.pop("example_plan", None)
    except Exception as e:  # noqa: BLE001 -- the point is to see what raised
        r, err = None, f"{type(e).__name__}: {e}"
    out = dict(run=args.run, inside=args.inside, calls=calls["n"], error=err, result=r, nonfinite_events=events,
               absurd_events=absurd)
    print(json.dumps(out, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
