"""Exact dense convex-QP solver for the oracle (TEST INFRASTRUCTURE ONLY).

    min 1/2 z'H z + g'z   s.t.  C z <= d          (H symmetric positive definite)

Algorithm: batched Mehrotra predictor-corrector primal-dual interior point in
float64, run to a 1e-12 scaled tolerance, followed by an *active-set polish*
(solve the equality-constrained KKT system on the identified active set, accept
it when it is primal and dual feasible), and a KKT certificate

    stat = ||H z + g + C'lam||_inf,  pfeas = max(C z - d)_+,
    dfeas = max(-lam)_+,             comp = max|lam_i (d_i - C_i z)|.

This is *not* the kernel's algorithm restated; it is an independent solver whose
solutions are certified optimal, so that the GPU path's PDIP is checked against
the QP's unique optimum (H is positive definite thanks to the proximal term).
The reference has no QP (its IPOPT + HSL MA27 backend, kinematic_mpc.py:39-52,
solves the NLP directly); see oracle/ltv_qp.py for the contract.
"""
from __future__ import annotations

import numpy as np


class Gram:
    """Gauss-Newton Hessian H += sum_t c_t row_t row_t' over a batch, collected term by term
    and formed as one batched matrix product R' diag(c) R at flush() -- the same sum as
    rank-1 updates one at a time, in one BLAS call (the rank-1 loop was 80 % of building a
    single-track N = 60 QP)."""

    def __init__(self, B, n):
        self.B, self.n = B, n
        self.c, self.rows = [], []

    def add(self, c, row):
        self.c.append(np.broadcast_to(np.asarray(c, np.float64), (self.B,)))
        self.rows.append(np.broadcast_to(np.asarray(row, np.float64), (self.B, self.n)))

    def flush(self, H):
        if self.rows:
            R = np.stack(self.rows, axis=1)
            Cw = np.stack(self.c, axis=1)
            H += np.matmul(np.swapaxes(R * Cw[..., None], 1, 2), R)
        self.c, self.rows = [], []


def _max_step(v, dv):
    """Largest a in (0, 1] with v + a dv >= 0 (rowwise over the batch)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.where(dv < 0, -v / dv, np.inf)
    return np.minimum(1.0, r.min(axis=-1))


def _chol_batch(Mx, done):
    """Batched Cholesky; a problem whose matrix has lost definiteness (barrier
    weights ~1e14 near the end) is frozen at its current iterate."""
    try:
        return np.linalg.cholesky(Mx)
    except np.linalg.LinAlgError:
        Lc = np.empty_like(Mx)
        for b in range(len(Mx)):
            try:
                Lc[b] = np.linalg.cholesky(Mx[b])
            except np.linalg.LinAlgError:
                done[b] = True
                Lc[b] = np.eye(Mx.shape[1])
        return Lc


def pdip_batch(H, g, C, d, tol=1e-12, max_iter=200):
    H = np.asarray(H, np.float64); g = np.asarray(g, np.float64)
    C = np.asarray(C, np.float64); d = np.asarray(d, np.float64)
    B, n = g.shape
    m = d.shape[1]
    z = np.zeros((B, n))
    s = np.maximum(d, 1.0)
    lam = np.ones((B, m))
    iters = np.zeros(B, np.int64)
    done = np.zeros(B, bool)
    diverged = np.zeros(B, bool)
    scale = 1.0 + np.maximum(np.abs(g).max(axis=1), np.abs(d).max(axis=1))
    for it in range(max_iter):
        # an infeasible QP drives the iterate off to infinity (multipliers and barrier weights
        # lam / s beyond any finite KKT point's): such a problem is frozen and reported as
        # diverged instead of overflowing; feasibility itself is decided by oracle/feasibility.py
        blow = ~done & ((lam.max(1) > 1e60 * scale) | (np.abs(z).max(1) > 1e60 * scale)
                        | ((lam / s).max(1) > 1e250))
        diverged |= blow
        done |= blow
        rd = np.einsum("bij,bj->bi", H, z) + g + np.einsum("bmi,bm->bi", C, lam)
        rp = np.einsum("bmi,bi->bm", C, z) + s - d
        mu = (s * lam).mean(axis=1)
        conv = (np.abs(rd).max(1) <= tol * scale) & (np.abs(rp).max(1) <= tol * scale) & (mu <= tol * scale)
        done |= conv
        if done.all():
            break
        iters += ~done
        w = np.where(done[:, None], 1.0, lam / s)
        Mx = H + np.einsum("bmi,bm,bmj->bij", C, w, C)
        Lc = _chol_batch(Mx, done)

        def solve(rc):
            # (H + C'WC) dz = -rd - C'(W rp - rc/s)
            rhs = -rd - np.einsum("bmi,bm->bi", C, w * rp - rc / s)
            y = np.linalg.solve(Lc, rhs[..., None])
            dz = np.linalg.solve(np.swapaxes(Lc, 1, 2), y)[..., 0]
            dlam = w * (np.einsum("bmi,bi->bm", C, dz) + rp) - rc / s
            ds_ = -rp - np.einsum("bmi,bi->bm", C, dz)
            return dz, ds_, dlam

        # predictor
        rc = s * lam
        with np.errstate(over="ignore", invalid="ignore"):
            dz_a, ds_a, dl_a = solve(rc)
        bad = ~done & ~(np.isfinite(dz_a).all(1) & np.isfinite(ds_a).all(1) & np.isfinite(dl_a).all(1))
        diverged |= bad
        done |= bad
        dz_a, ds_a, dl_a = (np.where(done[:, None], 0.0, v) for v in (dz_a, ds_a, dl_a))
        a_aff = np.minimum(_max_step(s, ds_a), _max_step(lam, dl_a))
        mu_aff = ((s + a_aff[:, None] * ds_a) * (lam + a_aff[:, None] * dl_a)).mean(1)
        sigma = (mu_aff / np.maximum(mu, 1e-300)) ** 3
        # corrector
        rc = s * lam + ds_a * dl_a - (sigma * mu)[:, None]
        with np.errstate(over="ignore", invalid="ignore"):
            dz, ds_, dl = solve(rc)
        bad = ~done & ~(np.isfinite(dz).all(1) & np.isfinite(ds_).all(1) & np.isfinite(dl).all(1))
        diverged |= bad
        done |= bad
        dz, ds_, dl = (np.where(done[:, None], 0.0, v) for v in (dz, ds_, dl))
        alpha = 0.99 * np.minimum(_max_step(s, ds_), _max_step(lam, dl))
        alpha = np.minimum(alpha, 1.0)
        alpha = np.where(done, 0.0, alpha)[:, None]
        z = z + alpha * dz
        s = s + alpha * ds_
        lam = lam + alpha * dl
        s = np.maximum(s, 1e-300)
        lam = np.maximum(lam, 1e-300)
    return z, lam, s, iters, done & ~diverged, diverged


def kkt_residuals(H, g, C, d, z, lam):
    stat = np.abs(np.einsum("bij,bj->bi", H, z) + g + np.einsum("bmi,bm->bi", C, lam)).max(1)
    slack = d - np.einsum("bmi,bi->bm", C, z)
    pfeas = np.maximum(-slack, 0).max(1)
    dfeas = np.maximum(-lam, 0).max(1)
    comp = np.abs(lam * slack).max(1)
    return dict(stat=stat, pfeas=pfeas, dfeas=dfeas, comp=comp)


def polish(H, g, C, d, z, lam, s, max_changes=40):
    """Active-set polish of one problem; returns (z, lam, ok).

    Starts from the active set the interior-point iterate suggests
    (lam_i > s_i) and repairs it one constraint at a time (add the most violated
    inactive constraint, else drop the most negative multiplier) until the
    equality-constrained KKT solution is primal and dual feasible.  Degenerate
    constraints (s_i, lam_i -> 0 together), which the interior point only
    approaches linearly, are settled exactly this way."""
    act = lam > s
    dscale = 1.0 + np.abs(d).max()
    for _ in range(max_changes):
        zp, lp = _eqp(H, g, C, d, act)
        if zp is None:
            return z, lam, False
        viol = C @ zp - d
        viol[act] = -np.inf
        neg = np.where(act, lp, np.inf)
        if neg.min() < -1e-12 * (1.0 + np.abs(lp).max()):
            act[np.argmin(neg)] = False
        elif viol.max() > 1e-12 * dscale:
            act[np.argmax(viol)] = True
        else:
            return zp, np.maximum(lp, 0.0), True
    return z, lam, False


def _eqp(H, g, C, d, act):
    """Solve min 1/2 z'Hz + g'z s.t. C_act z = d_act via the full KKT matrix."""
    n = len(g)
    Ca = C[act]
    k = Ca.shape[0]
    K = np.zeros((n + k, n + k))
    K[:n, :n] = H
    K[:n, n:] = Ca.T
    K[n:, :n] = Ca
    rhs = np.concatenate([-g, d[act]])
    try:
        sol = np.linalg.solve(K, rhs)
        bad = np.abs(K @ sol - rhs).max() > 1e-10 * (1.0 + np.abs(rhs).max())
    except np.linalg.LinAlgError:
        bad = True
    if bad:
        # linearly dependent active rows (e.g. the dynamic contract's stage-0 force
        # bounds, which all act on Fx_0 alone): minimum-norm multipliers; the primal
        # part is still unique because H is positive definite
        sol = np.linalg.lstsq(K, rhs, rcond=1e-13)[0]
        if np.abs(K @ sol - rhs).max() > 1e-9 * (1.0 + np.abs(rhs).max()):
            return None, None
    lp = np.zeros(len(d))
    lp[act] = sol[n:]
    return sol[:n], lp


def solve_qp_batch(H, g, C, d, tol=1e-13, max_iter=200, do_polish=True):
    z, lam, s, iters, done, diverged = pdip_batch(H, g, C, d, tol=tol, max_iter=max_iter)
    polished = np.zeros(len(g), bool)
    if do_polish:
        for b in range(len(g)):
            z[b], lam[b], polished[b] = polish(H[b], g[b], C[b], d[b], z[b], lam[b], s[b])
    kkt = kkt_residuals(H, g, C, d, z, lam)
    return dict(z=z, lam=lam, iters=iters, converged=done, diverged=diverged, polished=polished, kkt=kkt)
