"""When could the kinematic interior point hand over to the active-set polish?  (CPU study
for kin_ltv's iteration tail, VERDICT r01 item 6: 8.8 mean vs 15 max IPM iterations at C2.)

For C2 problems (vcmpc.workload.kinematic_batch, N = 20) it runs the oracle's Mehrotra
iteration (oracle/qp.py, the kernel's start point and step rule) and, after every iteration,
tries the polish (oracle/qp.py:polish, at most `--changes` active-set changes) from that
iterate.  It reports, per problem, the iterations to the kernel's stopping rule (tol 1e-10
scaled) and the first iteration whose polish certifies the exact optimum (== the converged
polish to 1e-12), with mu and the residual at that point.

    python scripts/early_polish_study.py [--B 256] [--changes 10]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]


def ipm_trace(H, g, C, d, tol=1e-10, max_iter=40):
    """Single-problem Mehrotra iteration (oracle/qp.py:pdip_batch), iterates recorded."""
    n, m = len(g), len(d)
    z, s, lam = np.zeros(n), np.maximum(d, 1.0), np.ones(m)
    scale = 1.0 + max(np.abs(g).max(), np.abs(d).max())
    out = []
    for it in range(max_iter + 1):
        rd = H @ z + g + C.T @ lam
        rp = C @ z + s - d
        mu = (s * lam).mean()
        res = max(np.abs(rd).max(), np.abs(rp).max())
        out.append((z.copy(), lam.copy(), s.copy(), mu / scale, res / scale))
        if res <= tol * scale and mu <= tol * scale:
            break
        w = lam / s
        try:
            L = np.linalg.cholesky(H + C.T @ (w[:, None] * C))
        except np.linalg.LinAlgError:   # barrier weights ~1/mu: the kernel stops here too
            break

        def solve(rc):
            rhs = -rd - C.T @ (w * rp - rc / s)
            dz = np.linalg.solve(L.T, np.linalg.solve(L, rhs))
            return dz, -rp - C @ dz, w * (C @ dz + rp) - rc / s

        def step(v, dv):
            r = np.where(dv < 0, -v / np.where(dv < 0, dv, -1), np.inf)
            return min(1.0, r.min())
        dz, dsa, dla = solve(s * lam)
        a = min(step(s, dsa), step(lam, dla))
        sig = (((s + a * dsa) * (lam + a * dla)).mean() / mu) ** 3
        dz, ds_, dl = solve(s * lam + dsa * dla - sig * mu)
        al = 0.99 * min(step(s, ds_), step(lam, dl))
        z, s, lam = z + al * dz, s + al * ds_, lam + al * dl
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--changes", type=int, default=10)
    args = ap.parse_args()
    from oracle.ltv_qp import kin_qp, kin_weights
    from oracle.qp import polish
    from vcmpc.config import load_config
    from vcmpc.workload import kinematic_batch
    cfg = load_config("kinematic_mpc")
    W = kin_weights(cfg)
    d = kinematic_batch(args.B, seed=31)
    Q = kin_qp(d["x0"], d["ubar"], d["kappa"], d["ds"], 2.5, W)
    conv, first, changes_at, mu_at, traces = [], [], [], [], []
    for b in range(args.B):
        H, g, C, dd = Q["H"][b], Q["g"][b], Q["C"][b], Q["d"][b]
        tr = ipm_trace(H, g, C, dd)
        zf, _, okf = polish(H, g, C, dd, *tr[-1][:3])
        conv.append(len(tr) - 1)
        hit = None
        for it, (z, lam, s, mu, res) in enumerate(tr):
            act0 = lam > s
            zp, _, ok = polish(H, g, C, dd, z, lam, s, max_changes=args.changes)
            if ok and okf and np.abs(zp - zf).max() <= 1e-12 * (1 + np.abs(zf).max()):
                hit = it
                changes_at.append(int(np.sum(act0 != (np.abs(C @ zp - dd) <= 1e-12 * (1 + np.abs(dd).max())))))
                mu_at.append(mu)
                break
        first.append(hit if hit is not None else -1)
        # rounds (equality solves) each iterate's polish needs to certify, capped at --changes
        need = []
        for (z, lam, s, mu, res) in tr:
            r_ok = None
            for r in range(1, args.changes + 1):
                zp, _, ok = polish(H, g, C, dd, z, lam, s, max_changes=r)
                if ok:
                    r_ok = r if np.abs(zp - zf).max() <= 1e-12 * (1 + np.abs(zf).max()) else None
                    break
            need.append((mu, res, r_ok))
        traces.append(need)
    conv, first = np.array(conv), np.array(first)
    # policies: from the first iterate with mu/scale <= T, try a polish of at most R rounds after
    # every iteration; cost = IPM iterations + rounds spent (a round ~ one iteration's factorisation)
    print("policy (T, R): cost mean / max in iteration units (baseline: converge, then polish)")
    base = [len(t) - 1 + (t[-1][2] or args.changes) for t in traces]
    print(f"  baseline           : {np.mean(base):.2f} / {np.max(base)}")
    for T in (1e-3, 1e-4, 1e-5, 1e-6):
        for R in (1, 2, 3):
            cost = []
            for t in traces:
                c = 0
                for it, (mu, res, r_ok) in enumerate(t):
                    if it > 0:
                        c += 1
                    if it == len(t) - 1:
                        c += r_ok or args.changes
                        break
                    if mu <= T:
                        if r_ok is not None and r_ok <= R:
                            c += r_ok
                            break
                        c += R
                cost.append(c)
            print(f"  T={T:.0e} R={R}     : {np.mean(cost):.2f} / {np.max(cost)}")
    print(f"B={args.B}: IPM iterations to tol 1e-10: mean {conv.mean():.2f} max {conv.max()}; "
          f"first certifying polish at iteration mean {first[first >= 0].mean():.2f} max {first.max()} "
          f"(never: {(first < 0).sum()})")
    print("  histogram conv :", np.bincount(conv).tolist())
    print("  histogram first:", np.bincount(first[first >= 0]).tolist())
    print(f"  active-set changes at the first certifying polish: mean {np.mean(changes_at):.2f} "
          f"max {np.max(changes_at)}; mu/scale there: median {np.median(mu_at):.1e} max {np.max(mu_at):.1e}")


if __name__ == "__main__":
    main()
