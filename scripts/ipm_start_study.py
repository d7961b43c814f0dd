"""Interior-point start points, step-length rules and Gondzio centrality correctors vs
iteration count on C2 problems (CPU study for kin_ltv's
iteration tail; the optimum, hence parity, does not depend on the start).  Runs the
kernel's Mehrotra rule (scripts/early_polish_study.py:ipm_trace, generalised to a given
start) under several (z0, s0, lam0) / step rules and reports mean / max iterations to the stopping
rule (tol 1e-10 scaled).

    python scripts/ipm_start_study.py [--B 256]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]


def ipm_iters(H, g, C, d, z, s, lam, tol=1e-10, max_iter=60, sigma_pow=3, eta=None, gondzio=0, gamma=0.0):
    scale = 1.0 + max(np.abs(g).max(), np.abs(d).max())
    for it in range(max_iter + 1):
        rd = H @ z + g + C.T @ lam
        rp = C @ z + s - d
        mu = (s * lam).mean()
        if max(np.abs(rd).max(), np.abs(rp).max()) <= tol * scale and mu <= tol * scale:
            return it
        w = lam / s
        try:
            L = np.linalg.cholesky(H + C.T @ (w[:, None] * C))
        except np.linalg.LinAlgError:
            return it

        def solve(rc):
            rhs = -rd - C.T @ (w * rp - rc / s)
            dz = np.linalg.solve(L.T, np.linalg.solve(L, rhs))
            return dz, -rp - C @ dz, w * (C @ dz + rp) - rc / s

        def step(v, dv):
            r = np.where(dv < 0, -v / np.where(dv < 0, dv, -1), np.inf)
            return min(1.0, r.min())
        dz, dsa, dla = solve(s * lam)
        a = min(step(s, dsa), step(lam, dla))
        sig = (((s + a * dsa) * (lam + a * dla)).mean() / mu) ** sigma_pow
        dz, ds_, dl = solve(s * lam + dsa * dla - sig * mu)
        amax = min(step(s, ds_), step(lam, dl))
        for _ in range(gondzio):   # Gondzio centrality correctors (one extra solve each)
            at = min(1.0, 1.5 * amax + 0.1)
            v = (s + at * ds_) * (lam + at * dl)
            t = np.clip(v, 0.1 * sig * mu, 10.0 * sig * mu)
            # complementarity-only correction: (s dl + lam ds) = -(t - v) ... rc carries it
            rc = -(t - v)
            rhs = -C.T @ (-rc / s)
            cz = np.linalg.solve(L.T, np.linalg.solve(L, rhs))
            cs_ = -C @ cz
            cl = w * (C @ cz) - rc / s
            nz, ns, nl = dz + cz, ds_ + cs_, dl + cl
            an = min(step(s, ns), step(lam, nl))
            if an >= amax + 0.1 * (at - amax) * 0 + 0.01:
                dz, ds_, dl, amax = nz, ns, nl, an
            else:
                break
        e = 0.99 if eta is None else eta(mu / scale)
        if gamma > 0 and e > 0.99:   # centrality safeguard: keep min s_i lam_i >= gamma * mean
            sn, ln = s + e * amax * ds_, lam + e * amax * dl
            if (sn * ln).min() < gamma * (sn * ln).mean():
                e = 0.99
        al = e * amax
        z, s, lam = z + al * dz, s + al * ds_, lam + al * dl
    return max_iter


def start_current(H, g, C, d):
    return np.zeros(len(g)), np.maximum(d, 1.0), np.ones(len(d))


def start_const(t_s, t_l):
    def f(H, g, C, d):
        return np.zeros(len(g)), np.maximum(d, t_s), np.full(len(d), t_l)
    return f


def start_mehrotra(H, g, C, d):
    """Gertz-Wright style: one affine-scaling solve from (0, 1, 1), then shift s, lam
    into the interior by their most negative entry plus a margin."""
    n, m = len(g), len(d)
    z, s, lam = np.zeros(n), np.ones(m), np.ones(m)
    rd = g + C.T @ lam
    rp = s - d
    L = np.linalg.cholesky(H + C.T @ C)
    rhs = -rd - C.T @ (rp - s * lam / s)
    dz = np.linalg.solve(L.T, np.linalg.solve(L, rhs))
    z1 = dz
    s1 = d - C @ z1
    lam1 = lam + (C @ dz + rp) - lam
    ds_ = max(-1.5 * s1.min(), 0.0)
    dl_ = max(-1.5 * lam1.min(), 0.0)
    s1, lam1 = s1 + ds_, lam1 + dl_
    p = s1 @ lam1
    s1 += 0.5 * p / max(lam1.sum(), 1e-12)
    lam1 += 0.5 * p / max(s1.sum(), 1e-12)
    return z1, np.maximum(s1, 1e-2), np.maximum(lam1, 1e-2)


def start_unconstrained(H, g, C, d):
    """z0 = the unconstrained minimiser clipped into the box rows' reach; s0 = max(d - C z0, 1)."""
    z = -np.linalg.solve(H, g)
    r = d - C @ z
    return z, np.maximum(r, 1.0), np.ones(len(d))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--only", default="", help="comma-separated substrings of the rule names")
    args = ap.parse_args()
    from oracle.ltv_qp import kin_qp, kin_weights
    from vcmpc.config import load_config
    from vcmpc.workload import kinematic_batch
    W = kin_weights(load_config("kinematic_mpc"))
    d = kinematic_batch(args.B, seed=31)
    Q = kin_qp(d["x0"], d["ubar"], d["kappa"], d["ds"], 2.5, W)
    eta_mu = lambda m: 1 - min(0.01, max(m, 1e-6))
    rules = {"current (0, max(d,1), 1)": (start_current, {}),
             "s=max(d,0.3), lam=0.3": (start_const(0.3, 0.3), {}),
             "Mehrotra-shift": (start_mehrotra, {}), "unconstrained z0": (start_unconstrained, {}),
             "sigma^2": (start_current, dict(sigma_pow=2)),
             "eta 0.995": (start_current, dict(eta=lambda m: 0.995)),
             "eta 1-min(.01, mu)": (start_current, dict(eta=eta_mu)),
             "gondzio 1": (start_current, dict(gondzio=1)),
             "gondzio 2": (start_current, dict(gondzio=2)),
             "gondzio 1 + eta(mu)": (start_current, dict(gondzio=1, eta=eta_mu)),
             "gondzio 2 + eta(mu)": (start_current, dict(gondzio=2, eta=eta_mu)),
             "eta(mu) guarded 1e-2": (start_current, dict(eta=eta_mu, gamma=1e-2)),
             "eta(mu) guarded 1e-1": (start_current, dict(eta=eta_mu, gamma=1e-1)),
             "eta(mu) guarded 1e-3": (start_current, dict(eta=eta_mu, gamma=1e-3))}
    if args.only:
        rules = {k: v for k, v in rules.items() if any(o in k for o in args.only.split(","))}
    for name, (rule, kw) in rules.items():
        its = []
        for b in range(args.B):
            H, g, C, dd = Q["H"][b], Q["g"][b], Q["C"][b], Q["d"][b]
            its.append(ipm_iters(H, g, C, dd, *rule(H, g, C, dd), **kw))
        its = np.array(its)
        print(f"{name:28s}: mean {its.mean():.2f}  p99 {np.percentile(its, 99):.0f}  max {its.max()}  "
              f"hist {np.bincount(its).tolist()}", flush=True)


if __name__ == "__main__":
    main()
