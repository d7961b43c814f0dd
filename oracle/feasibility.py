"""Phase-1 LP feasibility certificates for the oracle's linearised QPs (TEST INFRASTRUCTURE ONLY).

A kernel that reports a problem non-solved must be facing a QP with no feasible point; the
oracle's interior point cannot prove that (on an infeasible QP it diverges and its residuals
describe a diverged iterate).  This module decides the constraint set C z <= d of one QP by
linear programming (scipy.optimize.linprog, HiGHS) and returns a checkable certificate either
way:

  phase 1:   min t   s.t.  C_i z / r_i - t <= d_i / r_i,  t >= 0      (r_i = max(1, |C_i|_inf))

  feasible   -> t* = 0 and a point z with max(C z - d)_+ <= tol (checked here, in numpy);
  infeasible -> t* > 0 and a Farkas vector y >= 0 with C'y = 0, d'y < 0 (the rows' scaled
                duals of the phase-1 LP; checked here: |C'y|_inf <= tol |y| |C|, d'y < 0),
                i.e. no z can satisfy every row: y'C z = 0 > y'd would be needed.

The QPs are the SQP contracts' (oracle/dyn_sqp.py dyn_qp, oracle/casc_sqp.py casc_qp): the
reference has no QP (its NLP goes to IPOPT, cascaded_mpc.py:308), so these certify a property
of the build's contract at a given warm start, not of the reference.
"""
from __future__ import annotations

import numpy as np


def phase1(C, d, tol=1e-9, t_min=0.0):
    """Certificate for one constraint set C[m, n] z <= d[m].  Returns dict(feasible, t, z,
    viol, y, farkas_ok, farkas_gap).  With t_min < 0 the LP's t may go negative: -t* is then the
    largest uniform scaled slack of any point (the feasible set's interior margin).  `viol` = max(C z - d)_+ of the returned point (feasible),
    `farkas_ok` whether y certifies infeasibility (infeasible), `farkas_gap` = -d'y / |y|_1."""
    from scipy.optimize import linprog
    C = np.asarray(C, np.float64)
    d = np.asarray(d, np.float64)
    m, n = C.shape
    r = np.maximum(1.0, np.abs(C).max(axis=1))
    Cs, ds_ = C / r[:, None], d / r
    A = np.hstack([Cs, -np.ones((m, 1))])
    c = np.zeros(n + 1)
    c[-1] = 1.0
    bounds = [(None, None)] * n + [(t_min, None)]
    # tight HiGHS tolerances first; the simplex occasionally stops without a status at 1e-10
    # ("Not Set"), then looser ones -- the returned point / Farkas vector is checked below either way
    for tol_lp in (1e-10, 1e-9, None):
        opts = {} if tol_lp is None else dict(primal_feasibility_tolerance=tol_lp, dual_feasibility_tolerance=tol_lp)
        res = linprog(c, A_ub=A, b_ub=ds_, bounds=bounds, method="highs", options=opts)
        if res.status == 0:
            break
    if res.status != 0:
        raise RuntimeError(f"phase-1 LP: {res.message}")
    z, t = res.x[:n], float(res.x[-1])
    viol = float(np.maximum(C @ z - d, 0.0).max()) if m else 0.0
    scale = 1.0 + np.abs(d).max()
    out = dict(t=t, z=z, viol=viol, y=None, farkas_ok=False, farkas_gap=0.0)
    if t_min < 0.0:   # interior margin: t* < 0 is the largest uniform slack of a strictly feasible point
        out["feasible"] = t <= tol
        return out
    if t <= tol:
        out["feasible"] = viol <= 1e3 * tol * scale
        return out
    # the phase-1 duals: y_s >= 0 (HiGHS marginals of <= rows are <= 0), sum y_s = 1 at t* > 0,
    # Cs'y_s = 0, -ds'y_s = t*; unscaled y = y_s / r certifies C'y = 0, d'y = -t* < 0
    ys = np.maximum(-res.ineqlin.marginals, 0.0)
    y = ys / r
    cty = np.abs(C.T @ y).max()
    gap = -float(d @ y) / max(y.sum(), 1e-300)
    out["y"] = y
    out["farkas_gap"] = gap
    out["farkas_ok"] = bool(float(d @ y) < 0.0 and cty <= 1e-9 * max(np.abs(C).max(), 1.0) * y.sum())
    out["feasible"] = False
    return out


def certify_batch(C, d, tol=1e-9):
    """phase1 over a batch C[B, m, n], d[B, m]: (feasible[B], farkas_ok[B], t[B])."""
    outs = [phase1(C[b], d[b], tol) for b in range(len(d))]
    return (np.array([o["feasible"] for o in outs]), np.array([o["farkas_ok"] for o in outs]),
            np.array([o["t"] for o in outs]))


def first_infeasible_iteration(hist, tol=1e-9):
    """For SQP histories recorded with keep_qps=True: per problem, the first SQP iteration whose
    QP is certified infeasible (-1 if every QP is feasible), and whether its Farkas vector checks.
    Iterations after the first infeasible one are not examined (their iterate is the oracle's
    step on an infeasible QP, meaningless)."""
    B = hist[0]["C"].shape[0]
    first = np.full(B, -1)
    farkas = np.zeros(B, bool)
    for b in range(B):
        for i, h in enumerate(hist):
            o = phase1(h["C"][b], h["d"][b], tol)
            if not o["feasible"]:
                first[b] = i
                farkas[b] = o["farkas_ok"]
                break
    return first, farkas
