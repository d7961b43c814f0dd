"""How many interior-point iterations does the C2 LTV-QP need before the active-set polish can
finish it?  (CPU study for kin_ltv's iteration tail; not test infrastructure.)

kin_ltv runs its Mehrotra interior point to res, mu <= tol * scale (tol = 1e-10) and only then
polishes.  This restates that loop on the C2 workload (vcmpc/workload.py, seeded as bench.py)
with numpy -- the same start point, Mehrotra sigma, 0.99 fraction to the boundary and stopping
test as kin_ltv.hip:760-882 (= oracle/qp.py pdip_batch with the kernel's mu / scale) -- and at
every iteration tries the polish (oracle/qp.py polish: the active set lam > s, repaired one
constraint at a time) to find the first iteration from which it certifies.  Policies "polish
as soon as mu <= T" are then priced in iteration units (a polish round = one factorisation and
solves, about one iteration).

    python scripts/ipm_tail_study.py [--B 512] [--seed 31]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))


def kernel_pdip(H, g, C, d, tol=1e-10, max_iter=40):
    """kin_ltv's loop on one problem; returns per-iteration snapshots (z, lam, s, mu, res)."""
    n, m = len(g), len(d)
    z = np.zeros(n)
    s = np.maximum(d, 1.0)
    lam = np.ones(m)
    scale = 1.0 + max(np.abs(g).max(), np.abs(d).max())
    snaps = []
    for it in range(max_iter + 1):
        rd = H @ z + g + C.T @ lam
        rp = C @ z + s - d
        mu = float((s * lam).mean())
        res = float(max(np.abs(rd).max(), np.abs(rp).max()))
        snaps.append((z.copy(), lam.copy(), s.copy(), mu / scale, res / scale))
        if (res <= tol * scale and mu <= tol * scale) or it == max_iter:
            break
        w = lam / s
        try:
            Lc = np.linalg.cholesky(H + C.T @ (w[:, None] * C))
        except np.linalg.LinAlgError:
            break

        def solve(rc):
            rhs = -rd - C.T @ (w * rp - rc / s)
            dz = np.linalg.solve(Lc.T, np.linalg.solve(Lc, rhs))
            dl = w * (C @ dz + rp) - rc / s
            ds_ = -rp - C @ dz
            return dz, ds_, dl

        def amax(ds_, dl):
            r = np.concatenate([np.where(ds_ < 0, -s / np.where(ds_ < 0, ds_, -1), np.inf),
                                np.where(dl < 0, -lam / np.where(dl < 0, dl, -1), np.inf)])
            return min(1.0, r.min())

        dz_a, ds_a, dl_a = solve(s * lam)
        aa = amax(ds_a, dl_a)
        mua = float(((s + aa * ds_a) * (lam + aa * dl_a)).mean())
        sm = (mua / mu) ** 3 * mu
        dz, ds_, dl = solve(s * lam + ds_a * dl_a - sm)
        al = 0.99 * amax(ds_, dl)
        z, s, lam = z + al * dz, s + al * ds_, lam + al * dl
    return snaps, scale


def polish_rounds(H, g, C, d, lam, s, max_changes=10):
    """Rounds the polish needs from the active set lam > s (1 = first candidate certifies), or
    None if it does not certify within max_changes + 1 rounds."""
    from oracle.qp import _eqp
    act = lam > s
    dscale = 1.0 + np.abs(d).max()
    for r in range(max_changes + 1):
        zp, lp = _eqp(H, g, C, d, act)
        if zp is None:
            return None
        viol = C @ zp - d
        viol[act] = -np.inf
        neg = np.where(act, lp, np.inf)
        if neg.min() < -1e-9 * (1.0 + np.abs(lp).max()):
            act[np.argmin(neg)] = False
        elif viol.max() > 1e-9 * dscale:
            act[np.argmax(viol)] = True
        else:
            return r + 1
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--seed", type=int, default=31)
    a = ap.parse_args()
    from oracle import ltv_qp as Q
    from vcmpc.config import load_config
    from vcmpc.workload import kinematic_batch
    W = Q.kin_weights(load_config("kinematic_mpc"))
    data = kinematic_batch(a.B, seed=a.seed)
    Qd = Q.kin_qp(data["x0"], data["ubar"], data["kappa"], data["ds"], 2.5, W)
    H, g, C, d = Qd["H"], Qd["g"], Qd["C"], Qd["d"]
    iters, firsts = [], []
    mus = []   # per problem: list of scaled mu per iteration
    prs = []   # per problem: polish rounds from each iteration's active set
    for b in range(a.B):
        snaps, _ = kernel_pdip(H[b], g[b], C[b], d[b])
        iters.append(len(snaps) - 1)
        mus.append([sn[3] for sn in snaps])
        prs.append([polish_rounds(H[b], g[b], C[b], d[b], sn[1], sn[2]) for sn in snaps])
    iters = np.array(iters)
    print(f"B={a.B}: IPM iterations to tol 1e-10: mean {iters.mean():.2f} max {iters.max()} "
          f"hist {np.bincount(iters).tolist()}")
    base = iters + np.array([p[-1] if p[-1] is not None else 10 for p in prs])
    print(f"  current (converge, then polish): cost mean {base.mean():.2f} max {base.max()}")
    for T in (1e-2, 1e-3, 1e-4, 1e-5, 1e-6, 1e-7):
        cost = []
        for b in range(a.B):
            c, thr = None, T
            spent = 0
            for i, (mu, pr) in enumerate(zip(mus[b], prs[b])):
                if mu <= thr and i < len(mus[b]) - 1:
                    # attempt: pr rounds if it certifies, else the full budget of failed rounds (>= 1)
                    if pr is not None and pr <= 3:
                        c = i + spent + pr
                        break
                    spent += 3
                    thr *= 1e-3
            if c is None:
                pr = prs[b][-1]
                c = len(mus[b]) - 1 + spent + (pr if pr is not None else 10)
            cost.append(c)
        cost = np.array(cost)
        print(f"  polish at mu <= {T:.0e} (<= 3 rounds, retry at 1e-3 T): cost mean {cost.mean():.2f} "
              f"max {cost.max()}  p99 {np.percentile(cost, 99):.0f}")


if __name__ == "__main__":
    main()
