"""Oracle restatement of the cascaded (single-track + point-mass) SQP contract
(TEST INFRASTRUCTURE ONLY).

The reference's headline controller (README "cascaded MPC") is ``CascadedMPC`` with
``horizon_pm > 0`` (controllers/mpc/cascaded_mpc.py:17-39, config
config/controllers/cascaded.yaml: N = 20 single-track stages + M = 40 point-mass
stages every ds_pm = 3 m).  One multiple-shooting NLP over H = N + M stages:

* single-track stages n = 0..N-1: DynamicCar spatial RK4 for n < N-1
  (:116-122), stage constraints and costs of the single-track mode (:91-179);
* switching (:241-277): the point mass starts at V = |(Ux, Uy)|, s, ey,
  epsi + atan(Uy / Ux), t of the last single-track state, and the cost
  (switch_F / ds_{N-1}) [(Fx_N - Fx_{N-1})^2 + (Fy_N - Fy_f - Fy_r)^2];
* point-mass stages m = N..H-1: DynamicPointMass spatial Euler for m < H-1
  (:181-202, models/dynamic_point_mass.py:26-103), V >= V_min, Fx <= Peng / V,
  boundary / deviation / Fx and Fy slew costs (:204-239);
* terminal cost on the last point-mass state (:279-304).

The build replaces the IPOPT solve by ``sqp_iters`` sequential-QP iterations,
defined here once and implemented identically by ``csrc/casc_sqp.hip`` (fp64):

  for it in 1..sqp_iters:
    1. predict    single-track RK4 rollout, switch map, point-mass Euler rollout
    2. linearize  exact Jacobians of the three maps (complex step here)
    3. condense   dx = G dz in the scaled variable dz = [dFx_0/S, dw_0, ...,
                  dFx_N/S, dFy_N/S, ...]  (S = fx_scale; Fy is a force too)
    4. QP         Gauss-Newton cost of the NLP (every ``if_else`` frozen at the
                  prediction; the switching cost's lateral residual linearised
                  through Fy_f + Fy_r) + prox ||dz||^2, subject to the linearised
                  rows below, solved exactly (oracle/qp.py)
    5. update     ubar <- ubar + alpha du*, alpha = the first of 1, 1/2, ... whose prediction
                  stays in the models' domain (casc_in_domain; oracle/dyn_sqp.py domain_step)
  output u* = ubar, x* = predict(u*), u0 = u*_0.

Constraint rows (one-sided, linearised at the prediction; force rows divided by S):
  single-track n >= 1: Ux >= Ux_min, delta_min <= delta <= delta_max     :101-107
  single-track n:      Fx <= Peng / Ux, longitudinal tyre bounds f / r    :110,124-128
                       w_min <= w <= w_max (tightened by trust_w)         :111-113
  point mass m:        V >= V_min, Fx <= Peng / V                         :190-195
  every stage:         |dFx| <= trust_Fx; point mass also |dFy| <= trust_Fx (build's
                       trust region, SQP globalisation; 0 = off)
Deviation from the reference: the point-mass states' unused rows 5..7 of the
(8, H) state variable (free in the NLP) are reported as 0.
"""
from __future__ import annotations

import numpy as np

from . import dyn_sqp as D
from . import models as M
from . import obstacles as OB
from .qp import Gram

IUX, IUY, IR, ID, IS, IEY, IEP, IT = range(8)
PV, PS, PEY, PEP, PT = range(5)
CSTEP = D.CSTEP


def casc_weights(cfg: dict) -> dict:
    """Numbers the QP consumes, from a cascaded controller config (reference schema
    config/controllers/cascaded.yaml) plus the build's `qp` block."""
    W = D.dyn_weights(cfg)
    cw, pc = cfg["cost_weights"], cfg["state_pm_constraints"]
    W.update(N=int(cfg["horizon"]), M=int(cfg["horizon_pm"]), ds_pm=float(cfg["ds_pm"]),
             w_dev_pm=float(cw["deviation_pm"]), w_Fy=float(cw["Fy"]), w_switch=float(cw["switch_F"]),
             V_min=float(pc["V_min"]), ey_min_pm=float(pc["ey_min"]), ey_max_pm=float(pc["ey_max"]))
    return W


# ----------------------------------------------------------------------------
# step 1: predict
# ----------------------------------------------------------------------------
def casc_predict(x0, ubar, kappa, ds, p, W, tyre="fiala"):
    """xs[B,N,8] single-track states, xp[B,M,5] point-mass states."""
    N, Mh = W["N"], W["M"]
    B = ubar.shape[0]
    dt = np.result_type(x0, ubar)
    xs = np.empty((B, N, 8), dtype=dt)
    xs[:, 0] = x0
    for k in range(N - 1):
        xs[:, k + 1] = M.dyn_spatial_transition(xs[:, k], ubar[:, k], kappa[:, k], ds[:, k], p, tyre)
    xp = np.empty((B, Mh, 5), dtype=dt)
    xp[:, 0] = M.st_to_pm(xs[:, N - 1])
    for m in range(Mh - 1):
        j = N + m
        xp[:, m + 1] = M.pm_spatial_transition(xp[:, m], ubar[:, j], kappa[:, j], ds[:, j], p)
    return xs, xp


def casc_in_domain(xs, xp, kappa):
    """[B] both predictions inside their spatial models' domain: the single-track stages as
    oracle/dyn_sqp.py in_domain, the point-mass stages finite with V > 0 and
    s' = V cos(epsi) / (1 - kappa ey) > 0 (dynamic_point_mass.py:90-100 divides by s')."""
    N = xs.shape[1]
    kp = np.asarray(kappa)[:, N:N + xp.shape[1]]
    V, ey, ep = xp[..., PV], xp[..., PEY], xp[..., PEP]
    with np.errstate(invalid="ignore", over="ignore"):
        sdot = V * np.cos(ep) / (1.0 - kp * ey)
        ok = np.isfinite(xp).all(axis=(1, 2)) & (V > 0).all(axis=1) & (sdot > 0).all(axis=1)
    return D.in_domain(xs, kappa) & ok


def pack_states(xs, xp):
    """(8, H)-style state prediction [B, H, 8]: point-mass rows in slots 0..4."""
    B, N = xs.shape[:2]
    out = np.zeros((B, N + xp.shape[1], 8))
    out[:, :N] = xs
    out[:, N:, :5] = xp
    return out


# ----------------------------------------------------------------------------
# step 2: linearize (complex step)
# ----------------------------------------------------------------------------
def _cs_jac(f, x, u, nx_out):
    """Complex-step Jacobians of f(x, u) w.r.t. x and u."""
    xc, uc = x.astype(complex), u.astype(complex)
    A = np.empty(x.shape[:-1] + (nx_out, x.shape[-1]))
    Bm = np.empty(x.shape[:-1] + (nx_out, u.shape[-1]))
    for j in range(x.shape[-1]):
        xp_ = xc.copy(); xp_[..., j] += 1j * CSTEP
        A[..., j] = f(xp_, uc).imag / CSTEP
    for j in range(u.shape[-1]):
        up_ = uc.copy(); up_[..., j] += 1j * CSTEP
        Bm[..., j] = f(xc, up_).imag / CSTEP
    return A, Bm


def casc_linearize(xs, xp, ubar, kappa, ds, p, W, tyre="fiala"):
    N, Mh = W["N"], W["M"]
    As, Bs = _cs_jac(lambda x, u: M.dyn_spatial_transition(x, u, kappa[:, :N - 1], ds[:, :N - 1], p, tyre),
                     xs[:, :N - 1], ubar[:, :N - 1], 8)
    Sw, _ = _cs_jac(lambda x, u: M.st_to_pm(x), xs[:, N - 1], ubar[:, N - 1], 5)
    sl = slice(N, N + Mh - 1)
    Ap, Bp = _cs_jac(lambda x, u: M.pm_spatial_transition(x, u, kappa[:, sl], ds[:, sl], p),
                     xp[:, :Mh - 1], ubar[:, sl], 5)
    return As, Bs, Sw, Ap, Bp


def casc_condense(As, Bs, Sw, Ap, Bp, W):
    """G_st[B,N,8,n], G_pm[B,M,5,n] in the scaled variable (ST (S, 1), PM (S, S))."""
    N, Mh, S = W["N"], W["M"], W["fx_scale"]
    B = As.shape[0]
    n = 2 * (N + Mh)
    Gs = np.zeros((B, N, 8, n))
    Bss = Bs * np.array([S, 1.0])
    for k in range(N - 1):
        Gs[:, k + 1] = np.einsum("bij,bjn->bin", As[:, k], Gs[:, k])
        Gs[:, k + 1, :, 2 * k:2 * k + 2] += Bss[:, k]
    Gp = np.zeros((B, Mh, 5, n))
    Gp[:, 0] = np.einsum("bij,bjn->bin", Sw, Gs[:, N - 1])
    Bps = Bp * S
    for m in range(Mh - 1):
        j = N + m
        Gp[:, m + 1] = np.einsum("bij,bjn->bin", Ap[:, m], Gp[:, m])
        Gp[:, m + 1, :, 2 * j:2 * j + 2] += Bps[:, m]
    return Gs, Gp


def switch_lateral(xs_last, u_last, p, tyre="fiala"):
    """Value and gradient (Ux, Uy, r, delta, Fx) of Fy_f + Fy_r at the last
    single-track stage (the switching cost's lateral residual, cascaded_mpc.py:250-255)."""
    X5 = np.concatenate([xs_last[..., :4], u_last[..., :1]], axis=-1)

    def f(X):
        x8 = np.concatenate([X[..., :4], np.zeros(X.shape[:-1] + (4,), X.dtype)], axis=-1)
        fyf, fyr = M.dyn_lateral_forces(x8, X[..., 4:5], p, tyre)
        return fyf + fyr
    v = np.real(f(X5))
    g = np.empty(X5.shape)
    Xc = X5.astype(complex)
    for j in range(5):
        Xp = Xc.copy(); Xp[..., j] += 1j * CSTEP
        g[..., j] = f(Xp).imag / CSTEP
    return v, g


# ----------------------------------------------------------------------------
# steps 1-4: QP data
# ----------------------------------------------------------------------------
def casc_qp(x0, ubar, kappa, ds, p, W, tyre="fiala"):
    x0, ubar, kappa, ds = (np.asarray(a, np.float64) for a in (x0, ubar, kappa, ds))
    N, Mh, S = W["N"], W["M"], W["fx_scale"]
    H_ = N + Mh
    B = ubar.shape[0]
    n = 2 * H_
    xs, xp = casc_predict(x0, ubar, kappa, ds, p, W, tyre)
    As, Bs, Sw, Ap, Bp = casc_linearize(xs, xp, ubar, kappa, ds, p, W, tyre)
    Gs, Gp = casc_condense(As, Bs, Sw, Ap, Bp, W)
    T = D.stage_terms(xs, ubar[:, :N], p)

    Hm = np.zeros((B, n, n))
    g = np.zeros((B, n))
    eye = np.eye(n)
    gram = Gram(B, n)

    def add_square(c, r0, row):
        c = np.broadcast_to(np.asarray(c, np.float64), (B,))
        row = np.broadcast_to(row, (B, n))
        gram.add(2.0 * c, row)
        g[:] += 2.0 * (c * r0)[:, None] * row

    def ey_terms(ey, row, s, dsk, lo, hi, wdev):
        add_square(wdev * dsk, ey, row)
        add_square(np.where(ey < lo, W["w_b"] * dsk, 0.0), ey - lo, row)
        add_square(np.where(ey > hi, W["w_b"] * dsk, 0.0), ey - hi, row)
        if W.get("obstacles"):
            p_o, q_o = OB.ey_model(s, ey, W["w_obs"] * dsk, W["obstacles"], W.get("obs_margin_min", OB.MARGIN_MIN),
                                   inside=bool(W.get("obs_inside", False)))
            gram.add(q_o, row)
            g[:] += p_o[:, None] * row

    def lin_row(grad, k):
        return np.einsum("bi,bin->bn", grad[:, k, :4], Gs[:, k, :4]) + grad[:, k, 4:5] * S * eye[2 * k]

    # single-track stages (cascaded_mpc.py:131-179)
    for k in range(N):
        ey_terms(xs[:, k, IEY], Gs[:, k, IEY], xs[:, k, IS], ds[:, k], W["ey_min"], W["ey_max"], W["w_dev"])
        add_square(W["w_w"], ubar[:, k, 1], eye[2 * k + 1])
        for ax in ("f", "r"):
            v, gr = T["slip_" + ax]
            add_square(np.where(v[:, k] >= 0.0, W["w_slip"], 0.0), v[:, k], lin_row(gr, k))
        if k < N - 1:
            e = np.zeros(n); e[2 * k + 2] = S; e[2 * k] = -S
            add_square(W["w_Fx"] / ds[:, k], ubar[:, k + 1, 0] - ubar[:, k, 0], e)
    # switching cost (cascaded_mpc.py:241-255)
    kN = N - 1
    csw = W["w_switch"] / ds[:, kN]
    e = np.zeros(n); e[2 * N] = S; e[2 * kN] = -S
    add_square(csw, ubar[:, N, 0] - ubar[:, kN, 0], e)
    fy, gfy = switch_lateral(xs[:, kN], ubar[:, kN], p, tyre)
    row = S * eye[2 * N + 1] - (np.einsum("bi,bin->bn", gfy[:, :4], Gs[:, kN, :4]) + gfy[:, 4:5] * S * eye[2 * kN])
    add_square(csw, ubar[:, N, 1] - fy, row)
    # point-mass stages (cascaded_mpc.py:204-239)
    for m in range(Mh):
        j = N + m
        ey_terms(xp[:, m, PEY], Gp[:, m, PEY], xp[:, m, PS], ds[:, j], W["ey_min_pm"], W["ey_max_pm"], W["w_dev_pm"])
        if m < Mh - 1:
            for c, w in ((0, W["w_Fx"]), (1, W["w_Fy"])):
                e = np.zeros(n); e[2 * j + 2 + c] = S; e[2 * j + c] = -S
                add_square(w / ds[:, j], ubar[:, j + 1, c] - ubar[:, j, c], e)
    # terminal cost on the last point-mass state (cascaded_mpc.py:279-304, M > 0)
    xl, Gl = xp[:, Mh - 1], Gp[:, Mh - 1]
    add_square(np.where(xl[:, PV] >= W["max_speed"], W["w_speed"], 0.0), xl[:, PV] - W["max_speed"], Gl[:, PV])
    g[:] += W["w_time"] * Gl[:, PT]
    add_square(W["w_ey"], xl[:, PEY], Gl[:, PEY])
    add_square(W["w_epsi"], xl[:, PEP], Gl[:, PEP])
    gram.flush(Hm)
    Hm[:] += 2.0 * W["prox"] * eye

    rows, rhs = [], []

    def add(row, r):
        rows.append(np.broadcast_to(row, (B, n))); rhs.append(np.broadcast_to(r, (B,)))

    tw, tf = W["trust_w"], W["trust_Fx"]
    for k in range(N):
        if k >= 1:
            add(-Gs[:, k, IUX], xs[:, k, IUX] - W["Ux_min"])
            add(Gs[:, k, ID], W["delta_max"] - xs[:, k, ID])
            add(-Gs[:, k, ID], xs[:, k, ID] - W["delta_min"])
        for name in ("peng", "tyre_f_up", "tyre_f_lo", "tyre_r_up", "tyre_r_lo"):
            v, gr = T[name]
            add(lin_row(gr, k) / S, -v[:, k] / S)
        up, dn = W["w_max"] - ubar[:, k, 1], ubar[:, k, 1] - W["w_min"]
        if tw > 0:
            up, dn = np.minimum(up, tw), np.minimum(dn, tw)
        add(eye[2 * k + 1], up)
        add(-eye[2 * k + 1], dn)
        if tf > 0:
            add(eye[2 * k], tf / S)
            add(-eye[2 * k], tf / S)
    for m in range(Mh):
        j = N + m
        V = xp[:, m, PV]
        add(-Gp[:, m, PV], V - W["V_min"])
        # Fx - Peng / V <= 0, divided by S
        add((p["Peng"] / V ** 2)[:, None] * Gp[:, m, PV] / S + eye[2 * j], -(ubar[:, j, 0] - p["Peng"] / V) / S)
        if tf > 0:
            for c in (0, 1):
                add(eye[2 * j + c], tf / S)
                add(-eye[2 * j + c], tf / S)
    C = np.stack(rows, axis=1)
    d = np.stack(rhs, axis=1)
    return dict(xs=xs, xp=xp, Gs=Gs, Gp=Gp, H=Hm, g=g, C=C, d=d)


def casc_sqp_solve(x0, ubar, kappa, ds, p, W, tyre="fiala", keep_qps=False, **qp_kw):
    """The full contract.  Returns u_star[B,H,2], x_star[B,H,8] (pack_states),
    u0[B,2] and per-iteration QP certificates."""
    from .qp import solve_qp_batch

    u = np.array(ubar, np.float64, copy=True)
    B, H_ = u.shape[:2]
    N, S = W["N"], W["fx_scale"]
    scale = np.ones((H_, 2))
    scale[:, 0] = S
    scale[N:, 1] = S
    hist = []
    # a QP after the first without a solution ends the SQP at the current iterate (casc_ric.hip
    # CR_KEEP_ITERATE; oracle/dyn_sqp.py)
    stopped = np.zeros(B, bool)
    for it_sqp in range(W["sqp_iters"]):
        Q = casc_qp(x0, u, kappa, ds, p, W, tyre)
        sol = solve_qp_batch(Q["H"], Q["g"], Q["C"], Q["d"], **qp_kw)
        if it_sqp > 0:
            stopped |= ~np.asarray(sol["converged"], bool)
        z = np.where(stopped[:, None], 0.0, sol["z"])
        rec = dict(ubar=u.copy(), dz=z, kkt=sol["kkt"], polished=sol["polished"], iters=sol["iters"])
        if keep_qps:
            rec.update({k: Q[k] for k in ("H", "g", "C", "d", "Gs", "Gp")})
        du = z.reshape(B, H_, 2) * scale
        alpha = D.domain_step(np.asarray(x0, np.float64), u, du, np.asarray(kappa, np.float64),
                              np.asarray(ds, np.float64), p, tyre,
                              lambda x0_, u_, k_, ds_, p_, t_: casc_predict(x0_, u_, k_, ds_, p_, W, t_),
                              in_domain=casc_in_domain)
        rec["alpha"] = alpha
        rec["stopped"] = stopped.copy()
        hist.append(rec)
        u = np.where(((alpha > 0) & ~stopped)[:, None, None], u + alpha[:, None, None] * du, u)
    xs, xp = casc_predict(np.asarray(x0, np.float64), u, np.asarray(kappa, np.float64),
                          np.asarray(ds, np.float64), p, W, tyre)
    # status VC_OUT_OF_DOMAIN where x* leaves the models' domain (csrc/casc_ric.hip, ABI 12)
    return dict(u_star=u, x_star=pack_states(xs, xp), u0=u[:, 0].copy(), hist=hist,
                in_domain=casc_in_domain(xs, xp, np.asarray(kappa, np.float64)))


def casc_horizon_params(state, state_prediction, mpc_dt, N, Mh, ds_pm, k_of_s):
    """``CascadedMPC._init_horizon`` (cascaded_mpc.py:316-338): ds = mpc_dt * Ux_pred[:N],
    curvature at s0 + cumsum(ds) - ds[0]; point mass ds = ds_pm, curvature at
    cumsum(ds_pm) - ds[-1] + s_traj[-1].  state[8], state_prediction[8, H]."""
    ds = np.full(N, mpc_dt) * state_prediction[IUX, :N]
    s_traj = np.cumsum(ds) - ds[0] + state[IS]
    ds_p = np.full(Mh, ds_pm)
    s_pm = np.cumsum(ds_p) - ds[-1] + s_traj[-1]
    kap = np.concatenate([np.asarray(k_of_s(s_traj), np.float64), np.asarray(k_of_s(s_pm), np.float64)])
    return np.concatenate([ds, ds_p]), kap
