"""The reference's kinematic MPC NLP, solved directly (TEST INFRASTRUCTURE ONLY).

The reference solves, at every control step, the multiple-shooting NLP that
controllers/mpc/kinematic_mpc.py:15-158 transcribes with CasADi Opti and hands to IPOPT:

    variables  X[6, N+1], U[2, N]                                     (:57-60)
    min  sum_{n<N} [ w_b ds_n (ey_n - ey_min)^2 [ey_n < ey_min]                 (:110-114)
                   + w_b ds_n (ey_n - ey_max)^2 [ey_n > ey_max]                 (:116-120)
                   + w_dev ds_n ey_n^2 + w_w w_n^2                              (:122-124)
                   + w_a (a_{n+1} - a_n)^2 [n < N-1]                            (:126-128)
                   + w_obs ds_n sum_j 1 / (dist_nj - (r_j + 0.1)) [obstacles] ] (:130-133)
         + w_v (v_N - v_max)^2 [v_N >= v_max] + w_time t_N + w_ey ey_N^2 + w_epsi epsi_N^2   (:136-158)
    s.t. X[:, 0] = x0                                                   (:23-25)
         v_n >= v_min, delta_min <= delta_n <= delta_max,
         a_min <= a_n <= a_max, w_min <= w_n <= w_max,  n = 0..N-1       (:71-93)
         X[:, n+1] = spatial_transition(X[:, n], U[:, n], kappa_n, ds_n) (:95-99, Euler, kinematic_car.py:47-64)

IPOPT (and CasADi) cannot run here, so this module solves the same NLP with an
independent method: scipy's ``trust-constr`` (a trust-region interior point, byrd-omojokun
SQP inside) on the full-space multiple-shooting problem, with exact first derivatives
(analytic objective gradient; the dynamics Jacobians of oracle/models.py, which are
finite-difference-checked) and the Hessian of the Lagrangian from central differences of
those exact Jacobians, then Newton's method on the KKT system with trust-constr's active set
held (``refine``; converges in a few steps from trust-constr's 1e-8..1e-11 to ~1e-15).  A
converged point is then certified as a KKT point of the NLP with
its own multipliers (``kkt``), independently of how it was found.  Nothing here shares code
with the build's SQP contract (oracle/ltv_qp.py, oracle/kin_sqp.py) except the model.

Since x_0 = x0 is fixed, the stage-0 terms and the n = 0 state bounds are constants / true
at a feasible x0 and are left out; the variables are z = [X[:, 1..N] (6N), U (2N)].
"""
from __future__ import annotations

import numpy as np
from scipy import optimize, sparse

from . import models as M

IV, ID, IS, IEY, IEP, IT = range(6)
IA, IW = 0, 1


class KinNLP:
    """One problem of the reference NLP: x0[6], kappa[N], ds[N], weights W (oracle/ltv_qp.py
    kin_weights keys; W["obstacles"] = [(s, ey, r), ...] when on)."""

    def __init__(self, x0, kappa, ds, L, W):
        self.x0 = np.asarray(x0, np.float64)
        self.kappa = np.asarray(kappa, np.float64)
        self.ds = np.asarray(ds, np.float64)
        self.N = len(self.kappa)
        self.L = float(L)
        self.W = W
        self.obs = list(W.get("obstacles") or [])
        self.nz = 8 * self.N

    # -- variables ---------------------------------------------------------------------------
    def split(self, z):
        N = self.N
        X = np.vstack([self.x0[None], z[:6 * N].reshape(N, 6)])   # [N+1, 6]
        U = z[6 * N:].reshape(N, 2)
        return X, U

    def pack(self, X, U):
        return np.concatenate([np.asarray(X)[1:].ravel(), np.asarray(U).ravel()])

    def ix(self, n, i):
        """index of X[n, i] in z (n >= 1)"""
        return 6 * (n - 1) + i

    def iu(self, n, i):
        return 6 * self.N + 2 * n + i

    # -- objective ---------------------------------------------------------------------------
    def f(self, z):
        X, U = self.split(z)
        W, ds, N = self.W, self.ds, self.N
        ey = X[1:N, IEY]
        dsn = ds[1:N]
        c = np.sum(np.where(ey < W["ey_min"], W["w_b"] * dsn * (ey - W["ey_min"]) ** 2, 0.0))
        c += np.sum(np.where(ey > W["ey_max"], W["w_b"] * dsn * (ey - W["ey_max"]) ** 2, 0.0))
        c += np.sum(W["w_dev"] * dsn * ey ** 2)
        c += np.sum(W["w_w"] * U[:, IW] ** 2)
        c += np.sum(W["w_a"] * np.diff(U[:, IA]) ** 2)
        for so, eo, r in self.obs:
            d = np.hypot(X[1:N, IS] - so, ey - eo)
            c += np.sum(W["w_obs"] * dsn / (d - (r + 0.1)))
        vN = X[N, IV]
        if vN >= W["v_max"]:
            c += W["w_v"] * (vN - W["v_max"]) ** 2
        c += W["w_time"] * X[N, IT] + W["w_ey"] * X[N, IEY] ** 2 + W["w_epsi"] * X[N, IEP] ** 2
        return float(c)

    def grad(self, z):
        X, U = self.split(z)
        W, ds, N = self.W, self.ds, self.N
        gX = np.zeros((N + 1, 6))
        gU = np.zeros((N, 2))
        ey = X[1:N, IEY]
        dsn = ds[1:N]
        g = 2 * W["w_dev"] * dsn * ey
        g += np.where(ey < W["ey_min"], 2 * W["w_b"] * dsn * (ey - W["ey_min"]), 0.0)
        g += np.where(ey > W["ey_max"], 2 * W["w_b"] * dsn * (ey - W["ey_max"]), 0.0)
        gs = np.zeros(N - 1)
        for so, eo, r in self.obs:
            a, e = X[1:N, IS] - so, ey - eo
            d = np.hypot(a, e)
            m = d - (r + 0.1)
            coef = -W["w_obs"] * dsn / (m * m * d)
            gs += coef * a
            g += coef * e
        gX[1:N, IEY] = g
        gX[1:N, IS] = gs
        gU[:, IW] = 2 * W["w_w"] * U[:, IW]
        da = np.diff(U[:, IA])
        gU[:-1, IA] -= 2 * W["w_a"] * da
        gU[1:, IA] += 2 * W["w_a"] * da
        vN = X[N, IV]
        if vN >= W["v_max"]:
            gX[N, IV] = 2 * W["w_v"] * (vN - W["v_max"])
        gX[N, IT] = W["w_time"]
        gX[N, IEY] = 2 * W["w_ey"] * X[N, IEY]
        gX[N, IEP] = 2 * W["w_epsi"] * X[N, IEP]
        return self.pack(gX, gU)

    def hess_f(self, z, h=1e-6):
        """Hessian of the objective: analytic for the quadratic terms (each `if_else` on the
        branch z is in), central differences of the exact gradient for the obstacle terms."""
        X, U = self.split(z)
        W, ds, N = self.W, self.ds, self.N
        H = np.zeros((self.nz, self.nz))
        for n in range(1, N):
            ey = X[n, IEY]
            j = self.ix(n, IEY)
            H[j, j] = 2 * W["w_dev"] * ds[n] + (2 * W["w_b"] * ds[n] if (ey < W["ey_min"] or ey > W["ey_max"]) else 0.0)
        for n in range(N):
            j = self.iu(n, IW)
            H[j, j] = 2 * W["w_w"]
        for n in range(N - 1):
            i, j = self.iu(n, IA), self.iu(n + 1, IA)
            H[i, i] += 2 * W["w_a"]
            H[j, j] += 2 * W["w_a"]
            H[i, j] -= 2 * W["w_a"]
            H[j, i] -= 2 * W["w_a"]
        if X[N, IV] >= W["v_max"]:
            H[self.ix(N, IV), self.ix(N, IV)] = 2 * W["w_v"]
        H[self.ix(N, IEY), self.ix(N, IEY)] = 2 * W["w_ey"]
        H[self.ix(N, IEP), self.ix(N, IEP)] = 2 * W["w_epsi"]
        if self.obs:
            W0 = dict(W)
            obs_only = KinNLP.__new__(KinNLP)
            obs_only.__dict__.update(self.__dict__)
            obs_only.W = {k: (0.0 if k.startswith("w_") and k != "w_obs" else v) for k, v in W0.items()}
            for n in range(1, N):
                for i in (IS, IEY):
                    j = self.ix(n, i)
                    e = np.zeros(self.nz)
                    e[j] = h
                    col = (obs_only.grad(z + e) - obs_only.grad(z - e)) / (2 * h)
                    for i2 in (IS, IEY):
                        H[self.ix(n, i2), j] += col[self.ix(n, i2)]
        return 0.5 * (H + H.T)

    # -- dynamics ------------------------------------------------------------------------------
    def c(self, z):
        """defects X[n+1] - F(X[n], U[n]), n = 0..N-1  ->  [6N]"""
        X, U = self.split(z)
        F = M.kin_spatial_transition(X[:-1], U, self.kappa, self.ds, self.L)
        return (X[1:] - F).ravel()

    def jac_c(self, z):
        X, U = self.split(z)
        A, Bm = M.kin_spatial_jacobians(X[:-1], U, self.kappa, self.ds, self.L)
        N = self.N
        J = np.zeros((6 * N, self.nz))
        for n in range(N):
            r = slice(6 * n, 6 * n + 6)
            J[r, self.ix(n + 1, 0):self.ix(n + 1, 0) + 6] = np.eye(6)
            if n >= 1:
                J[r, self.ix(n, 0):self.ix(n, 0) + 6] = -A[n]
            J[r, self.iu(n, 0):self.iu(n, 0) + 2] = -Bm[n]
        return J

    def hess_c(self, z, lam, h=1e-6):
        """sum_i lam_i Hess c_i: central differences of jac_c' lam (stage-local, so only the
        8 variables of stage n move row block n)."""
        N = self.N
        H = np.zeros((self.nz, self.nz))
        X, U = self.split(z)
        lam = np.asarray(lam).reshape(N, 6)
        for n in range(N):
            cols = ([self.ix(n, i) for i in range(6)] if n >= 1 else []) + [self.iu(n, 0), self.iu(n, 1)]
            for j in cols:
                def jt(sign):
                    Xp, Up = X.copy(), U.copy()
                    if j >= 6 * N:
                        Up[n, j - self.iu(n, 0)] += sign * h
                    else:
                        Xp[n, j - self.ix(n, 0)] += sign * h
                    A, Bm = M.kin_spatial_jacobians(Xp[n:n + 1], Up[n:n + 1], self.kappa[n:n + 1],
                                                    self.ds[n:n + 1], self.L)
                    # d/dz of -F(X_n, U_n)' lam_n over stage n's variables
                    gx = -A[0].T @ lam[n]
                    gu = -Bm[0].T @ lam[n]
                    return gx, gu
                gxp, gup = jt(+1)
                gxm, gum = jt(-1)
                gx, gu = (gxp - gxm) / (2 * h), (gup - gum) / (2 * h)
                if n >= 1:
                    H[self.ix(n, 0):self.ix(n, 0) + 6, j] += gx
                H[self.iu(n, 0):self.iu(n, 0) + 2, j] += gu
        return 0.5 * (H + H.T)

    # -- bounds ---------------------------------------------------------------------------------
    def bounds(self):
        W, N = self.W, self.N
        lb = np.full(self.nz, -np.inf)
        ub = np.full(self.nz, np.inf)
        for n in range(1, N):
            lb[self.ix(n, IV)] = W["v_min"]
            lb[self.ix(n, ID)] = W["delta_min"]
            ub[self.ix(n, ID)] = W["delta_max"]
        for n in range(N):
            lb[self.iu(n, IA)], ub[self.iu(n, IA)] = W["a_min"], W["a_max"]
            lb[self.iu(n, IW)], ub[self.iu(n, IW)] = W["w_min"], W["w_max"]
        return lb, ub

    # -- KKT certificate ------------------------------------------------------------------------
    def kkt(self, z):
        """Residuals of the NLP's first-order conditions at z, with the multipliers that best fit
        them: nu (dynamics) and the bound multipliers from a bounded least-squares fit of
        grad f + J' nu = mu_lb - mu_ub (mu >= 0 only on active bounds).  Returns dict of
        stationarity (inf-norm, relative to |grad f|), primal feasibility (defects, bound
        violation) and the active-set size."""
        lb, ub = self.bounds()
        g = self.grad(z)
        J = self.jac_c(z)
        scale = max(1.0, np.abs(g).max())
        act_lo = np.isfinite(lb) & (z - lb <= 1e-7 * np.maximum(1.0, np.abs(lb)))
        act_hi = np.isfinite(ub) & (ub - z <= 1e-7 * np.maximum(1.0, np.abs(ub)))
        nl, nh = int(act_lo.sum()), int(act_hi.sum())
        E_lo = np.eye(self.nz)[:, act_lo]
        E_hi = np.eye(self.nz)[:, act_hi]
        # g + J' nu - E_lo mu_lo + E_hi mu_hi = 0, mu >= 0
        Amat = np.hstack([J.T, -E_lo, E_hi])
        lo = np.concatenate([np.full(J.shape[0], -np.inf), np.zeros(nl + nh)])
        res = optimize.lsq_linear(Amat, -g, bounds=(lo, np.full(Amat.shape[1], np.inf)), tol=1e-14,
                                  lsmr_tol="auto", method="bvls")
        stat = np.abs(Amat @ res.x + g).max() / scale
        pfeas = max(np.abs(self.c(z)).max(), np.maximum(lb - z, 0).max(), np.maximum(z - ub, 0).max())
        return dict(stat=float(stat), pfeas=float(pfeas), n_active=nl + nh)

    # -- Newton refinement on the KKT system -----------------------------------------------------
    def refine(self, z, iters=30, tol=1e-15):
        """Newton's method on the first-order conditions with the active bounds of z held fixed:
        grad f + J' nu = 0 on the free variables, c(z) = 0 (exact Hessian of the Lagrangian).
        Returns the refined z (or z itself when the refined point leaves the bounds)."""
        lb, ub = self.bounds()
        act = (np.isfinite(lb) & (z - lb <= 1e-7 * np.maximum(1.0, np.abs(lb)))) | \
              (np.isfinite(ub) & (ub - z <= 1e-7 * np.maximum(1.0, np.abs(ub))))
        z = z.copy()
        z[act] = np.where(np.abs(z[act] - lb[act]) < np.abs(z[act] - ub[act]), lb[act], ub[act])
        fr = ~act
        J = self.jac_c(z)
        nu = np.linalg.lstsq(J[:, fr].T, -self.grad(z)[fr], rcond=None)[0]
        nfr, m = int(fr.sum()), J.shape[0]
        for _ in range(iters):
            g = self.grad(z)
            J = self.jac_c(z)
            r = np.concatenate([(g + J.T @ nu)[fr], self.c(z)])
            if np.abs(r).max() <= tol * max(1.0, np.abs(g).max()):
                break
            Hl = self.hess_f(z) + self.hess_c(z, nu)
            K = np.zeros((nfr + m, nfr + m))
            K[:nfr, :nfr] = Hl[np.ix_(fr, fr)]
            K[:nfr, nfr:] = J[:, fr].T
            K[nfr:, :nfr] = J[:, fr]
            step = np.linalg.solve(K, -r)
            z[fr] += step[:nfr]
            nu += step[nfr:]
        if (z < lb - 1e-12).any() or (z > ub + 1e-12).any():
            return None
        return z

    # -- solve ----------------------------------------------------------------------------------
    def solve(self, z0, gtol=1e-11, xtol=1e-14, maxiter=3000):
        lb, ub = self.bounds()
        zc = np.clip(z0, np.where(np.isfinite(lb), lb, -np.inf), np.where(np.isfinite(ub), ub, np.inf))
        con = optimize.NonlinearConstraint(self.c, 0.0, 0.0, jac=lambda z: sparse.csr_matrix(self.jac_c(z)),
                                           hess=lambda z, v: self.hess_c(z, v))
        r = optimize.minimize(self.f, zc, jac=self.grad, hess=self.hess_f, method="trust-constr",
                              constraints=[con], bounds=optimize.Bounds(lb, ub, keep_feasible=False),
                              options=dict(gtol=gtol, xtol=xtol, barrier_tol=1e-12, maxiter=maxiter,
                                           initial_barrier_parameter=1e-3, verbose=0))
        return r


def warm_start(x0, ubar, kappa, ds, L):
    """The reference's initial point for the NLP from a warm start ubar: the rollout of ubar
    (what IPOPT's multiple shooting would receive as state_prediction after a solve)."""
    X = np.zeros((len(ubar) + 1, 6))
    X[0] = x0
    for n in range(len(ubar)):
        X[n + 1] = M.kin_spatial_transition(X[n], ubar[n], kappa[n], ds[n], L)
    return X


def solve_nlp(x0, ubar, kappa, ds, L, W, **kw):
    """-> (U[N, 2], X[N+1, 6], info) for one problem, from the rollout of ubar."""
    P = KinNLP(x0, kappa, ds, L, W)
    X0 = warm_start(x0, ubar, kappa, ds, L)
    r = P.solve(P.pack(X0, ubar), **kw)
    z = r.x
    zr = P.refine(z) if r.status in (1, 2) else None
    refined = zr is not None and P.kkt(zr)["stat"] <= P.kkt(z)["stat"]
    if refined:
        z = zr
    X, U = P.split(z)
    cert = P.kkt(z)
    info = dict(status=int(r.status), nit=int(r.nit), f=P.f(z), refined=bool(refined), **cert)
    return U, X, info
