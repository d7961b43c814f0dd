"""Oracle restatement of the kinematic SQP step with a merit line search (TEST INFRASTRUCTURE
ONLY).

The kinematic LTV-QP contract (oracle/ltv_qp.py) takes one convexified QP step per control
step.  With the obstacle barrier of kinematic_mpc.py:130-133 that is not enough: the QP's
second-order barrier model at a prediction that passes close to (or through) an obstacle
extrapolates the barrier's steep slope, and successive control steps keep steering away long
after the trajectory is clear, off the track.  The reference avoids this
because IPOPT solves the NLP with the exact barrier.  The build's globalised step:

    repeat sqp_iters times:
        dz    = the LTV-QP step at ubar (oracle/ltv_qp.py, trust region included)
        alpha = the first of 1, 1/2, ..., 2^-(LS_STEPS-1) with
                phi(ubar + alpha dz) <= phi(ubar) + ARMIJO * alpha * D,
                D = (phi(ubar + EPS_FD dz) - phi(ubar)) / EPS_FD  (one-sided derivative),
                and no step at all (alpha = 0) if none qualifies or D >= 0 -- unless |D| is at
                its own rounding level and the full step does not raise phi (noise_step: the
                flat directions near a KKT point)
        ubar += alpha dz

phi is the exact NLP cost of the QP contract (the same terms, each `if_else` evaluated on
the trial rollout instead of frozen at the prediction, no proximal term) plus an exact L1
penalty on the state rows:

    sum_{n=1}^{N-1} [ w_b ds_n (ey_n - ey_min)^2 [ey_n < ey_min] + w_b ds_n (ey_n - ey_max)^2 [ey_n > ey_max]
                      + w_dev ds_n ey_n^2 + w_obs ds_n sum_j b(dist_nj - (r_j + 0.1)) ]
  + sum_{n=0}^{N-1} w_w w_n^2 + sum_{n=0}^{N-2} w_a (a_{n+1} - a_n)^2
  + w_v (v_N - v_max)^2 [v_N >= v_max] + w_time t_N + w_ey ey_N^2 + w_epsi epsi_N^2
  + RHO sum_{n=1}^{N-1} [ (v_min - v_n)_+ + (delta_n - delta_max)_+ + (delta_min - delta_n)_+ ]

with b(m) = 1/m for m >= m0 = margin_min (the reference's barrier) and its second-order
Taylor extension 1/m0 - (m - m0)/m0^2 + (m - m0)^2/m0^3 below (finite, convex and decreasing
through the obstacle, so a trajectory that passes through one is pushed out rather than
rewarded by the reference's negative values inside).  The device code is
csrc/kin_merit.hip; the operation order below is the same.  Parity unpinned by the
reference (IPOPT cannot run here; no recorded kinematic run exists).

Multiple shooting (vc_qp.ms; ltv_qp.kin_qp(x_ws=)): the iterate is the pair (x, u); the QP step
is taken at the state iterate x (x_0 = x0), the line search moves both, (x, u) + alpha (dx, du),
and the merit evaluates every term at the state iterate instead of a rollout, plus an exact L1
penalty RHO_DEF sum_n |F(x_n, u_n) - x_{n+1}|_1 on the defects (merit(..., x=)) -- unless the
rollout of u has no larger merit, in which case the step is the plain single-shooting one
(line_search_ms).  After each step the state iterate is reset to the rollout of u where the
rollout's merit is no larger (a defect-free point).  So where the rollout is well behaved the
iteration is the single-shooting SQP (the L1 defect penalty's second-order growth would
otherwise reject every step of a long horizon: the Maratos effect), and where it runs through
the eps = +-pi/2 singularity (merit huge or not finite) the multiple-shooting iterate carries on.
"""
from __future__ import annotations

import numpy as np

from . import ltv_qp as Q
from . import models as M

LS_STEPS = 24       # alpha = 1 .. 2^-23 (one lane each in kin_merit.hip)
ARMIJO = 1e-4
EPS_FD = 1e-7
RHO = 1e3           # L1 penalty on the state rows (above every multiplier seen in the contract's QPs)
RHO_DEF = 1e3       # L1 penalty on the multiple-shooting defects
NOISE_D = 8.0 * 2.220446049250313e-16 / 1e-7   # rounding level of the one-sided difference D (x max(1, |phi|))
NOISE_PHI = 1e-13   # a noise-level step may not raise phi by more than this (x max(1, |phi|))
V_DOM = 0.5        # merit domain: v > V_DOM, |epsi| < EPSI_DOM, rho > 0 on stages 0..N-1
EPSI_DOM = 1.2
TIE = 1e-9          # the rollout is preferred unless the state iterate's merit is lower by more
IV, ID, IS, IEY, IEP, IT = Q.IV, Q.ID, Q.IS, Q.IEY, Q.IEP, Q.IT
IA, IW = Q.IA, Q.IW


def barrier_ext(m, m0):
    """b(m): 1/m above m0, the quadratic Taylor extension of 1/m at m0 below."""
    m = np.asarray(m, np.float64)
    dm = m - m0
    ext = 1.0 / m0 - dm / (m0 * m0) + dm * dm / (m0 * m0 * m0)
    return np.where(m >= m0, 1.0 / np.maximum(m, m0), ext)


def defects(x0, x, u, kappa, ds, L):
    """F(x_n, u_n) - x_{n+1} [B, N, 6] of a state iterate x[B, N+1, 6] (x_0 taken as x0)."""
    x = np.array(x, np.float64, copy=True)
    x[:, 0] = x0
    u = np.asarray(u, np.float64)
    kappa, ds = np.asarray(kappa, np.float64), np.asarray(ds, np.float64)
    xn = np.stack([M.kin_spatial_transition(x[:, n], u[:, n], kappa[:, n], ds[:, n], L)
                   for n in range(u.shape[1])], axis=1)
    return xn - x[:, 1:]


def merit(x0, u, kappa, ds, L, W, x=None):
    """phi(u) per problem: x0[B,6], u[B,N,2], kappa/ds[B,N] -> [B].  With a state iterate
    x[B,N+1,6] (multiple shooting) the terms are evaluated on it, plus RHO_DEF |defects|_1."""
    u = np.asarray(u, np.float64)
    pdef = 0.0
    if x is None:
        x = Q.kin_predict(np.asarray(x0, np.float64), u, kappa, ds, L)  # [B, N+1, 6]
    else:
        pdef = RHO_DEF * np.abs(defects(x0, x, u, kappa, ds, L)).sum(axis=(1, 2))
        x = np.array(x, np.float64, copy=True)
        x[:, 0] = x0
    B, N = u.shape[:2]
    ds = np.asarray(ds, np.float64)
    ey = x[:, 1:N, IEY]
    dsn = ds[:, 1:N]
    phi = np.zeros(B)
    lo = ey < W["ey_min"]
    hi = ey > W["ey_max"]
    phi += np.sum(np.where(lo, W["w_b"] * dsn * (ey - W["ey_min"]) ** 2, 0.0), axis=1)
    phi += np.sum(np.where(hi, W["w_b"] * dsn * (ey - W["ey_max"]) ** 2, 0.0), axis=1)
    phi += np.sum(W["w_dev"] * dsn * ey * ey, axis=1)
    if W.get("obstacles"):
        m0 = W.get("obs_margin_min", 0.05)
        sa = x[:, 1:N, IS]
        for so, eo, r in W["obstacles"]:
            d = np.sqrt((sa - so) ** 2 + (ey - eo) ** 2)
            phi += np.sum(W["w_obs"] * dsn * barrier_ext(d - (r + 0.1), m0), axis=1)
    phi += np.sum(W["w_w"] * u[:, :, IW] ** 2, axis=1)
    phi += np.sum(W["w_a"] * (u[:, 1:, IA] - u[:, :-1, IA]) ** 2, axis=1)
    vN = x[:, N, IV]
    phi += np.where(vN >= W["v_max"], W["w_v"] * (vN - W["v_max"]) ** 2, 0.0)
    phi += W["w_time"] * x[:, N, IT] + W["w_ey"] * x[:, N, IEY] ** 2 + W["w_epsi"] * x[:, N, IEP] ** 2
    v, dl = x[:, 1:N, IV], x[:, 1:N, ID]
    viol = (np.maximum(W["v_min"] - v, 0.0) + np.maximum(dl - W["delta_max"], 0.0)
            + np.maximum(W["delta_min"] - dl, 0.0))
    phi += RHO * np.sum(viol, axis=1)
    # the spatial model's domain (kinematic_car.py:47-60 divides by v cos(epsi) and rho = 1 - ey kappa):
    # a trajectory whose stages 0..N-1 leave it (v <= V_DOM, |epsi| >= EPSI_DOM, rho <= 0) is no
    # candidate -- e.g. a plan spinning to |epsi| >> pi/2, which the defect rollout of the next
    # control step turns into delta ~ 1e10 and an infeasible QP
    xs = x[:, :N]
    rho_ = 1.0 - xs[:, :, IEY] * np.asarray(kappa, np.float64)
    inside = ((xs[:, :, IV] > V_DOM) & (np.abs(xs[:, :, IEP]) < EPSI_DOM) & (rho_ > 0.0)).all(axis=1)
    return np.where(inside, phi + pdef, np.inf)


def line_search(x0, ubar, dz, kappa, ds, L, W):
    """(alpha[B], phi0[B], phi_alpha[B], D[B]) of the rule in the module docstring."""
    ubar = np.asarray(ubar, np.float64)
    phi0 = merit(x0, ubar, kappa, ds, L, W)
    with np.errstate(invalid="ignore"):
        D = (merit(x0, ubar + EPS_FD * dz, kappa, ds, L, W) - phi0) / EPS_FD
    B = len(phi0)
    alpha = np.zeros(B)
    phia = phi0.copy()
    restore = ~np.isfinite(phi0)   # outside the domain: the largest step back inside it
    done = (D >= 0.0) & ~restore
    a = 1.0
    p1 = None
    for _ in range(LS_STEPS):
        pa = merit(x0, ubar + a * dz, kappa, ds, L, W)
        with np.errstate(invalid="ignore"):
            ok = ~done & np.isfinite(pa) & (restore | (pa <= phi0 + ARMIJO * a * D))
        p1 = pa if p1 is None else p1
        alpha[ok] = a
        phia[ok] = pa[ok]
        done |= ok
        a *= 0.5
    nz = noise_step(alpha, phi0, p1, D)
    alpha[nz] = 1.0
    phia[nz] = p1[nz]
    return alpha, phi0, phia, D


def noise_step(alpha, phi0, p1, D):
    """Where no step size passed the Armijo test and |D| is at the rounding level of its own
    one-sided difference, the full step is taken if it does not raise phi beyond rounding:
    near a solution the decrease a QP step promises (~|dz|^2 times the curvature of flat
    directions such as the last acceleration, whose only cost is the 1e-4 slew) is below what
    the merit can resolve, and the SQP would otherwise stop short of the KKT point."""
    sc = np.maximum(1.0, np.abs(phi0))
    # finite merits only (csrc/kin_merit.hip alike): from outside the domain (phi0 = inf) the tests
    # below hold for any p1, and the full step would leave the domain again
    with np.errstate(invalid="ignore"):
        return ((alpha == 0.0) & np.isfinite(phi0) & np.isfinite(p1) & (np.abs(D) <= NOISE_D * sc)
                & (p1 <= phi0 + NOISE_PHI * sc))


def line_search_ms(x0, ubar, dz, x, dx, kappa, ds, L, W):
    """The multiple-shooting line search: per problem, the merit is the single-shooting one
    (the rollout of u) where that is no larger than the multiple-shooting one at the current
    iterate ("roll" mode: the plain SQP of line_search), else merit(..., x=) along (dx, dz).
    Returns (alpha, phi0, phi_alpha, D, reset): reset where the accepted point's rollout has no
    larger merit than its state iterate (the next state iterate is then that rollout)."""
    ubar = np.asarray(ubar, np.float64)
    ps = lambda a: merit(x0, ubar + a * dz, kappa, ds, L, W)
    pm = lambda a: merit(x0, ubar + a * dz, kappa, ds, L, W, x=x + a * dx)
    ps0, pm0 = ps(0.0), pm(0.0)
    roll = np.isfinite(ps0) & (ps0 <= pm0 + TIE * np.abs(pm0))
    sel = lambda vs, vm: np.where(roll, vs, vm)
    phi0 = sel(ps0, pm0)
    with np.errstate(invalid="ignore"):
        D = (sel(ps(EPS_FD), pm(EPS_FD)) - phi0) / EPS_FD
    B = len(phi0)
    alpha = np.zeros(B)
    phia = phi0.copy()
    pr, pa_m = ps0.copy(), pm0.copy()
    restore = ~np.isfinite(phi0)   # both merits outside the domain: the largest step back inside
    done = (D >= 0.0) & ~restore
    a = 1.0
    first = None
    for _ in range(LS_STEPS):
        vs, vm = ps(a), pm(a)
        pa = sel(vs, vm)
        first = (pa, vs, vm) if first is None else first
        with np.errstate(invalid="ignore"):
            ok = ~done & np.isfinite(pa) & (restore | (pa <= phi0 + ARMIJO * a * D))
        alpha[ok] = a
        phia[ok] = pa[ok]
        pr[ok], pa_m[ok] = vs[ok], vm[ok]
        done |= ok
        a *= 0.5
    nz = noise_step(alpha, phi0, first[0], D)
    alpha[nz] = 1.0
    phia[nz] = first[0][nz]
    pr[nz], pa_m[nz] = first[1][nz], first[2][nz]
    reset = np.isfinite(pr) & (pr <= pa_m + TIE * np.abs(pa_m))
    line_search_ms.reset_gap = (pr - pa_m) / np.abs(pa_m)   # for tests: how close the reset decision was
    return alpha, phi0, phia, D, reset


def elastic_qp_step(x0, ubar, kappa, ds, L, W, rho=RHO, **qp_kw):
    """The single-shooting LTV-QP step with elastic state rows (ltv_qp.elastic_qp: v >= v_min
    and the delta bounds get slacks t >= 0 at cost rho t + eps_t t^2, the QP model of the
    merit's L1 penalty).  Returns (u_star, kkt, t)."""
    sol = Q.kin_ltv_solve(x0, ubar, kappa, ds, L, W, elastic=rho, **qp_kw)
    return sol["u_star"], sol["kkt"], sol["t"]


def kin_sqp_solve(x0, ubar, kappa, ds, L, W, sqp_iters, x_ws=None, elastic=0.0, **qp_kw):
    """The globalised step: u_star[B,N,2], x_star[B,N+1,6] (x at u_star; under multiple
    shooting, x_ws given, the state iterate), per-iteration (alpha, phi0, phi, D, QP certificates).
    elastic = rho > 0 (vc_qp.elastic): every QP's state rows are elastic (ltv_qp.elastic_qp),
    so every step has a QP solution; with rho = RHO the QP's L1 model is the merit's own.
    elastic = -rho < 0: elastic on failure -- the hard-row QP, and where that has no certified
    solution (infeasible: the interior point diverges, the polish fails) the elastic one."""
    u = np.array(ubar, np.float64, copy=True)
    x = None
    if x_ws is not None:
        x = np.array(x_ws, np.float64, copy=True)
        x[:, 0] = x0
        x[:, 1:, IS] = x0[:, None, IS] + np.cumsum(ds, axis=1)     # s' = 1 (kin_ric.hip)
    hist = []
    for it in range(sqp_iters):
        sol = Q.kin_ltv_solve(x0, u, kappa, ds, L, W, x_ws=x, elastic=max(elastic, 0.0), **qp_kw)
        if elastic < 0.0:
            bad = ~sol["polished"] | sol["diverged"]
            if bad.any():
                xs = None if x is None else x[bad]
                se = Q.kin_ltv_solve(x0[bad], u[bad], np.asarray(kappa)[bad], np.asarray(ds)[bad], L, W,
                                     x_ws=xs, elastic=-elastic, **qp_kw)
                for key in ("u_star", "x_star", "polished"):
                    sol[key][bad] = se[key]
                for key in sol["kkt"]:
                    sol["kkt"][key][bad] = se["kkt"][key]
            sol["elastic_retry"] = bad
        dz = sol["u_star"] - u
        if x is None:
            alpha, phi0, phia, D = line_search(x0, u, dz, kappa, ds, L, W)
        else:
            dx = sol["x_star"] - x
            alpha, phi0, phia, D, reset = line_search_ms(x0, u, dz, x, dx, kappa, ds, L, W)
        # a QP without a certified solution refuses its step (kin_merit.hip qp_ok)
        ok = sol["polished"] | (sol["converged"] & ~sol["diverged"])
        alpha = np.where(ok, alpha, 0.0)
        hist.append(dict(alpha=alpha, phi0=phi0, phi=phia, D=D, kkt=sol["kkt"], polished=sol["polished"],
                         elastic_retry=sol.get("elastic_retry", np.zeros(len(alpha), bool)), qp_ok=ok))
        # a refused step (alpha = 0) keeps the iterate as it is: u + 0 * dz would carry a failed
        # QP's non-finite output into it (kin_merit.hip step_to)
        acc = (alpha > 0.0)[:, None, None]
        u = np.where(acc, u + alpha[:, None, None] * dz, u)
        if x is not None:
            x = np.where(acc, x + alpha[:, None, None] * dx, x)
            x[reset] = Q.kin_predict(np.asarray(x0, np.float64)[reset], u[reset], np.asarray(kappa)[reset],
                                     np.asarray(ds)[reset], L)
            hist[-1]["reset"] = reset
            hist[-1]["reset_gap"] = line_search_ms.reset_gap
        # a first QP without a solution restarts the iterate from the neutral guess (u = 0, the
        # state iterate x0 at every stage); the next QP's status is then the step's (kin_merit.hip)
        if it == 0 and sqp_iters > 1 and not ok.all():
            u[~ok] = 0.0
            if x is not None:
                x[~ok] = np.asarray(x0, np.float64)[~ok, None, :]
            hist[-1]["restart"] = ~ok
    x_star = Q.kin_predict(np.asarray(x0, np.float64), u, kappa, ds, L) if x is None else x
    return dict(u_star=u, x_star=x_star, u0=u[:, 0].copy(), hist=hist)
