"""Oracle restatement of the dynamic-bicycle SQP contract (TEST INFRASTRUCTURE ONLY).

The reference's dynamic controller is ``CascadedMPC`` in single-track mode
(``horizon_pm: 0``, controllers/mpc/cascaded_mpc.py:17-39, config
config/controllers/singletrack.yaml): a multiple-shooting NLP over the
DynamicCar spatial RK4 model solved by IPOPT at every control step
(cascaded_mpc.py:306-314).  The build replaces that solve by a fixed number of
*sequential-QP* iterations (BASELINE config 3), defined
here once and implemented identically by ``csrc/dyn_sqp.hip``:

  for it in 1..sqp_iters:
    1. predict    xbar_0 = x0, xbar_{k+1} = RK4_ds(xbar_k, ubar_k, kappa_k, ds_k),
                  k = 0..N-2 (the state has N columns and dynamics are imposed for
                  n < N-1 only, cascaded_mpc.py:70,116-122)
    2. linearize  A_k, B_k = exact Jacobians of the RK4 spatial step
                  (dynamic_car.py:169-191, integrators.py:26-37) -- here by complex-step
                  differentiation of oracle/models.py, in the kernel by dual numbers
    3. condense   dx_k = G_k dz in the scaled decision variable
                  dz = [dFx_0/S, dw_0, dFx_1/S, dw_1, ...]  (S = fx_scale, 1000 N)
    4. QP         min 1/2 dz'H dz + g'dz  s.t. C dz <= d  (below), solved exactly
    5. update     ubar <- ubar + alpha du*.  From an iterate whose prediction is inside the
                  spatial model's domain (in_domain: finite, Ux > 0 and s' > 0 at every stage),
                  alpha = the first of 1, 1/2, ..., 2^-(DOM_HALVINGS-1) whose prediction stays
                  inside, 0 if none -- IPOPT cuts its step back the same way when the NLP
                  functions cannot be evaluated at a trial point; alpha = 1 from an iterate
                  outside the domain, and wherever the full step stays inside
  A QP after the first without a solution (infeasible linearisation) refuses its step and ends
  the SQP at the current iterate.
  output u* = ubar, x* = predict(u*), u0 = u*_0; an x* outside the domain is not a solution
  (status VC_OUT_OF_DOMAIN: the SQP started outside and never got back in).

QP cost = the reference NLP cost in Gauss-Newton form about (xbar, ubar), with every
``if_else`` branch frozen at the prediction, plus prox * ||dz||^2:
  w_b ds_k (ey_k - ey_min)^2 if eybar_k < ey_min, mirror for ey_max   cascaded_mpc.py:139-149
  w_dev ds_k ey_k^2                                                  :151
  w_w w_k^2                                                          :153
  w_slip (|tan a_f| - tan amod_f(Fx))^2 if active at the prediction  :155-159 (front)
  w_slip (|tan a_r| - tan amod_r(Fx))^2 likewise                     :161-165 (rear)
  (w_Fx / ds_k) (Fx_{k+1} - Fx_k)^2, k < N-1                         :167-171
  obstacle barrier, convexified in ey_k (W["obstacles"] set)          :173-176, obstacles.py
  terminal (state column N-1, cascaded_mpc.py:283 with M = 0):
  w_speed (Ux - max_speed)^2 if Uxbar >= max_speed, w_time t, w_ey ey^2, w_epsi epsi^2  :290-303
Constraints (one-sided rows, each linearised at the prediction; state rows for
k = 1..N-1 -- column 0 is the fixed initial state, cascaded_mpc.py:26-28):
  Ux_k >= Ux_min; delta_min <= delta_k <= delta_max                  :101-107
  Fx_k <= Peng / Ux_k                                                :110
  w_min <= w_k <= w_max (tightened by the trust region trust_w)      :111-113
  -bound_f <= Fx_f(Fx_k) <= bound_f, bound_f = mu_f Fz_f cos(alpha_f), rear alike  :124-128
  |dFx_k| <= trust_Fx (trust region, SQP globalisation; 0 = off)
Force rows are divided by S so every row is O(1) in the scaled variables.
"""
from __future__ import annotations

import numpy as np

from . import models as M
from . import obstacles as OB
from .qp import Gram

IUX, IUY, IR, ID, IS, IEY, IEP, IT = range(8)
IFX, IW = 0, 1
CSTEP = 1e-30  # complex-step size


DOM_HALVINGS = 8    # step cut-backs tried when the full SQP step leaves the model's domain


def in_domain(xbar, kappa):
    """[B] prediction inside the spatial model's domain: finite, Ux > 0 and
    s' = (Ux cos epsi - Uy sin epsi) / (1 - kappa ey) > 0 at every stage (the spatial
    transformation dynamic_car.py:169-191 divides by s'; the slip angles by Ux)."""
    ux, uy, ey, ep = xbar[..., IUX], xbar[..., IUY], xbar[..., IEY], xbar[..., IEP]
    k = np.asarray(kappa)[:, :xbar.shape[1]]
    with np.errstate(invalid="ignore", over="ignore"):
        sdot = (ux * np.cos(ep) - uy * np.sin(ep)) / (1.0 - k * ey)
        ok = np.isfinite(xbar).all(axis=(1, 2)) & (ux > 0).all(axis=1) & (sdot > 0).all(axis=1)
    return ok


def domain_step(x0, u, du, kappa, ds, p, tyre, predict, in_domain=None):
    """alpha[B] of step 5: the first of 1, 1/2, ... with predict(u + alpha du) in the domain,
    0 where none is (or where du is not finite).  predict returns what in_domain takes
    (with kappa) -- the single-track prediction by default."""
    in_domain = in_domain or globals()["in_domain"]
    B = u.shape[0]
    alpha = np.zeros(B)
    todo = np.isfinite(du).all(axis=tuple(range(1, du.ndim)))
    # an iterate whose own prediction is outside the domain takes the full step (the test
    # cannot tell a better point from a worse one there)
    pred0 = predict(x0, u, kappa, ds, p, tyre)
    out0 = ~in_domain(*(pred0 if isinstance(pred0, tuple) else (pred0,)), kappa)
    alpha[todo & out0] = 1.0
    todo &= ~out0
    a = 1.0
    for _ in range(DOM_HALVINGS):
        if not todo.any():
            break
        idx = np.nonzero(todo)[0]
        pred = predict(x0[idx], u[idx] + a * du[idx], kappa[idx], ds[idx], p, tyre)
        ok = in_domain(*(pred if isinstance(pred, tuple) else (pred,)), kappa[idx])
        alpha[idx[ok]] = a
        todo[idx[ok]] = False
        a *= 0.5
    return alpha


def dyn_weights(cfg: dict) -> dict:
    """Numbers the QP consumes, from a singletrack controller config
    (reference schema: config/controllers/singletrack.yaml) plus the `qp` block."""
    cw, ic, sc = cfg["cost_weights"], cfg["input_constraints"], cfg["state_constraints"]
    qp = cfg.get("qp", {})
    return dict(
        w_time=float(cw["time"]), w_speed=float(cw["speed"]), w_ey=float(cw["ey"]),
        w_epsi=float(cw["epsi"]), w_w=float(cw["w"]), w_Fx=float(cw["Fx"]),
        w_dev=float(cw["deviation_st"]), w_b=float(cw["boundary"]), w_slip=float(cw["slip"]),
        w_min=float(ic["w_min"]), w_max=float(ic["w_max"]),
        Ux_min=float(sc["Ux_min"]), max_speed=float(sc["max_speed"]),
        delta_min=float(sc["delta_min"]), delta_max=float(sc["delta_max"]),
        ey_min=float(sc["ey_min"]), ey_max=float(sc["ey_max"]),
        prox=float(qp.get("prox", 0.1)), fx_scale=float(qp.get("fx_scale", 1000.0)),
        trust_Fx=float(qp.get("trust_Fx", 0.0)), trust_w=float(qp.get("trust_w", 0.0)),
        sqp_iters=int(qp.get("sqp_iters", 3)), w_obs=float(cw.get("obstacles", 0.0)), obstacles=[],
        obs_margin_min=OB.MARGIN_MIN,
    )


# ----------------------------------------------------------------------------
# model pieces
# ----------------------------------------------------------------------------
def spatial_step(x, u, kappa, ds, p, tyre):
    return M.dyn_spatial_transition(x, u, kappa, ds, p, tyre)


def dyn_predict(x0, ubar, kappa, ds, p, tyre="linear"):
    """Step 1: xbar[B,N,8] (N columns, dynamics for k < N-1)."""
    B, N = ubar.shape[:2]
    xbar = np.empty((B, N, 8), dtype=np.result_type(x0, ubar))
    xbar[:, 0] = x0
    for k in range(N - 1):
        xbar[:, k + 1] = spatial_step(xbar[:, k], ubar[:, k], kappa[:, k], ds[:, k], p, tyre)
    return xbar


def dyn_linearize(xbar, ubar, kappa, ds, p, tyre="linear"):
    """Step 2: A[B,N-1,8,8], Bm[B,N-1,8,2] (unscaled), complex-step derivatives of
    the RK4 spatial step at (xbar_k, ubar_k), k = 0..N-2."""
    N = ubar.shape[1]
    x = xbar[:, :N - 1].astype(complex)
    u = ubar[:, :N - 1].astype(complex)
    kap, h = kappa[:, :N - 1], ds[:, :N - 1]
    A = np.empty(x.shape[:2] + (8, 8))
    Bm = np.empty(x.shape[:2] + (8, 2))
    for j in range(8):
        xp = x.copy(); xp[..., j] += 1j * CSTEP
        A[..., j] = spatial_step(xp, u, kap, h, p, tyre).imag / CSTEP
    for j in range(2):
        up = u.copy(); up[..., j] += 1j * CSTEP
        Bm[..., j] = spatial_step(x, up, kap, h, p, tyre).imag / CSTEP
    return A, Bm


def stage_functions(X5, p):
    """Per-stage nonlinear terms of the NLP at X5[..., 5] = (Ux, Uy, r, delta, Fx):
    slip residuals (cascaded_mpc.py:155-165), the power limit (:110) and the
    longitudinal tyre-force bounds (:124-128).  Complex-step safe."""
    x4 = X5[..., :4]
    F = M.dyn_forces(x4, X5[..., 4:5], p)
    Fx = X5[..., 4]
    out = {}
    for ax, Ca, Fymax, alpha, mu, Fz, Fxa in (
            ("f", p["Caf"], F["Fymax_f"], F["alpha_f"], p["muf"], F["Fz_f"], F["Fx_f"]),
            ("r", p["Car"], F["Fymax_r"], F["alpha_r"], p["mur"], F["Fz_r"], F["Fx_r"])):
        amod = np.arctan((3 * Fymax * p["eps"]) / Ca)  # alphamod_f/r, dynamic_car.py:119,132
        out["slip_" + ax] = M.rabs(np.tan(alpha)) - np.tan(amod)
        bound = mu * Fz * np.cos(alpha)
        out["tyre_" + ax + "_up"] = Fxa - bound
        out["tyre_" + ax + "_lo"] = -Fxa - bound
    out["peng"] = Fx - p["Peng"] / X5[..., 0]
    return out


def stage_terms(xbar, ubar, p):
    """Values and gradients (w.r.t. Ux, Uy, r, delta, Fx) of stage_functions along
    the prediction.  Returns {name: (value[B,N], grad[B,N,5])}."""
    X5 = np.concatenate([xbar[..., :4], ubar[..., :1]], axis=-1)
    val = stage_functions(X5, p)
    grads = {k: np.empty(v.shape + (5,)) for k, v in val.items()}
    Xc = X5.astype(complex)
    for j in range(5):
        Xp = Xc.copy(); Xp[..., j] += 1j * CSTEP
        v = stage_functions(Xp, p)
        for k in grads:
            grads[k][..., j] = v[k].imag / CSTEP
    return {k: (np.real(val[k]), grads[k]) for k in val}


def dyn_condense(A, Bm, S):
    """Step 3: G[B,N,8,2N] with dx_k = G[:,k] @ dz, dz scaled (dFx / S, dw)."""
    B, N1 = A.shape[:2]
    N = N1 + 1
    G = np.zeros((B, N, 8, 2 * N))
    Bs = Bm * np.array([S, 1.0])
    for k in range(N - 1):
        G[:, k + 1] = np.einsum("bij,bjn->bin", A[:, k], G[:, k])
        G[:, k + 1, :, 2 * k:2 * k + 2] += Bs[:, k]
    return G


def dyn_qp(x0, ubar, kappa, ds, p, W, tyre="linear"):
    """Steps 1-4: QP data about ubar.  Returns dict xbar, A, Bm, G, H, g, C, d."""
    x0 = np.asarray(x0, np.float64); ubar = np.asarray(ubar, np.float64)
    kappa = np.asarray(kappa, np.float64); ds = np.asarray(ds, np.float64)
    B, N = ubar.shape[:2]
    n = 2 * N
    S = W["fx_scale"]
    xbar = dyn_predict(x0, ubar, kappa, ds, p, tyre)
    A, Bm = dyn_linearize(xbar, ubar, kappa, ds, p, tyre)
    G = dyn_condense(A, Bm, S)
    T = stage_terms(xbar, ubar, p)

    H = np.zeros((B, n, n))
    g = np.zeros((B, n))
    eye = np.eye(n)
    gram = Gram(B, n)

    def add_square(c, r0, row):
        c = np.broadcast_to(np.asarray(c, np.float64), (B,))
        gram.add(2.0 * c, row)
        g[:] += 2.0 * (c * r0)[:, None] * row

    def lin_row(grad, k):
        # gradient over (Ux,Uy,r,delta,Fx) of a stage-k function, as a row in dz
        return np.einsum("bi,bin->bn", grad[:, k, :4], G[:, k, :4]) + grad[:, k, 4:5] * S * eye[2 * k]

    for k in range(N):
        ey = xbar[:, k, IEY]
        row = G[:, k, IEY]
        add_square(W["w_dev"] * ds[:, k], ey, row)
        add_square(np.where(ey < W["ey_min"], W["w_b"] * ds[:, k], 0.0), ey - W["ey_min"], row)
        add_square(np.where(ey > W["ey_max"], W["w_b"] * ds[:, k], 0.0), ey - W["ey_max"], row)
        if W.get("obstacles"):  # cascaded_mpc.py:173-176, convexified in ey (obstacles.py)
            p_o, q_o = OB.ey_model(xbar[:, k, IS], ey, W["w_obs"] * ds[:, k], W["obstacles"],
                                   W.get("obs_margin_min", OB.MARGIN_MIN),
                                   inside=bool(W.get("obs_inside", False)))
            gram.add(q_o, row)
            g[:] += p_o[:, None] * row
        add_square(W["w_w"], ubar[:, k, IW], np.broadcast_to(eye[2 * k + 1], (B, n)))
        for ax in ("f", "r"):
            v, gr = T["slip_" + ax]
            add_square(np.where(v[:, k] >= 0.0, W["w_slip"], 0.0), v[:, k], lin_row(gr, k))
        if k < N - 1:
            e = np.zeros((B, n)); e[:, 2 * k + 2] = S; e[:, 2 * k] = -S
            add_square(W["w_Fx"] / ds[:, k], ubar[:, k + 1, IFX] - ubar[:, k, IFX], e)
    kN = N - 1
    UxN = xbar[:, kN, IUX]
    add_square(np.where(UxN >= W["max_speed"], W["w_speed"], 0.0), UxN - W["max_speed"], G[:, kN, IUX])
    g += W["w_time"] * G[:, kN, IT]
    add_square(W["w_ey"], xbar[:, kN, IEY], G[:, kN, IEY])
    add_square(W["w_epsi"], xbar[:, kN, IEP], G[:, kN, IEP])
    gram.flush(H)
    H += 2.0 * W["prox"] * eye

    rows, rhs = [], []

    def add(row, r):
        rows.append(np.broadcast_to(row, (B, n))); rhs.append(np.broadcast_to(r, (B,)))

    tw, tf = W["trust_w"], W["trust_Fx"]
    for k in range(N):
        if k >= 1:
            add(-G[:, k, IUX], xbar[:, k, IUX] - W["Ux_min"])
            add(G[:, k, ID], W["delta_max"] - xbar[:, k, ID])
            add(-G[:, k, ID], xbar[:, k, ID] - W["delta_min"])
        for name in ("peng", "tyre_f_up", "tyre_f_lo", "tyre_r_up", "tyre_r_lo"):
            v, gr = T[name]
            add(lin_row(gr, k) / S, -v[:, k] / S)
        up, dn = W["w_max"] - ubar[:, k, IW], ubar[:, k, IW] - W["w_min"]
        if tw > 0:
            up, dn = np.minimum(up, tw), np.minimum(dn, tw)
        add(eye[2 * k + 1], up)
        add(-eye[2 * k + 1], dn)
        if tf > 0:
            add(eye[2 * k], tf / S)
            add(-eye[2 * k], tf / S)
    C = np.stack(rows, axis=1)
    d = np.stack(rhs, axis=1)
    return dict(xbar=xbar, A=A, Bm=Bm, G=G, H=H, g=g, C=C, d=d, terms=T)


def dyn_sqp_solve(x0, ubar, kappa, ds, p, W, tyre="linear", keep_qps=False, **qp_kw):
    """The full contract.  Returns dict u_star[B,N,2], x_star[B,N,8], u0[B,2],
    per-iteration QP certificates (kkt), and optionally every QP's data."""
    from .qp import solve_qp_batch

    u = np.array(ubar, np.float64, copy=True)
    B, N = u.shape[:2]
    S = W["fx_scale"]
    hist = []
    # a QP after the first without a solution (converged False: the interior point diverged on an
    # infeasible linearisation) refuses its step and ends the SQP at the current iterate
    # (csrc/st_sqp.hip ST_KEEP_ITERATE, the kinematic SQP's rule)
    stopped = np.zeros(B, bool)
    for it_sqp in range(W["sqp_iters"]):
        Q = dyn_qp(x0, u, kappa, ds, p, W, tyre)
        sol = solve_qp_batch(Q["H"], Q["g"], Q["C"], Q["d"], **qp_kw)
        if it_sqp > 0:
            stopped |= ~np.asarray(sol["converged"], bool)
        dz = np.where(stopped[:, None], 0.0, sol["z"])
        rec = dict(ubar=u.copy(), dz=dz, lam=sol["lam"], kkt=sol["kkt"], polished=sol["polished"],
                   iters=sol["iters"])
        if keep_qps:
            rec.update({k: Q[k] for k in ("xbar", "A", "Bm", "G", "H", "g", "C", "d")})
        du = dz.reshape(B, N, 2) * np.array([S, 1.0])
        alpha = domain_step(np.asarray(x0, np.float64), u, du, np.asarray(kappa, np.float64),
                            np.asarray(ds, np.float64), p, tyre, dyn_predict)
        rec["alpha"] = alpha
        rec["stopped"] = stopped.copy()
        hist.append(rec)
        u = np.where(((alpha > 0) & ~stopped)[:, None, None], u + alpha[:, None, None] * du, u)
    x_star = dyn_predict(np.asarray(x0, np.float64), u, np.asarray(kappa, np.float64),
                         np.asarray(ds, np.float64), p, tyre)
    # status VC_OUT_OF_DOMAIN where x* leaves the model's domain (csrc/st_sqp.hip, ABI 12)
    return dict(u_star=u, x_star=x_star, u0=u[:, 0].copy(), hist=hist,
                in_domain=in_domain(x_star, np.asarray(kappa, np.float64)))


def dyn_horizon_params(state, state_prediction, mpc_dt, N, k_of_s):
    """``CascadedMPC._init_horizon`` for horizon_pm = 0 (cascaded_mpc.py:316-330):
    ds = mpc_dt * Ux_pred[:N] (no +0.5, unlike the kinematic controller) and the
    curvature at s0 + cumsum(ds) - ds[0].  state[8], state_prediction[8, N]."""
    ds = np.full(N, mpc_dt) * state_prediction[IUX, :N]
    s_traj = np.cumsum(ds) - ds[0] + state[IS]
    return ds, np.asarray(k_of_s(s_traj), np.float64)


def closed_loop_cost(X, U, dt, p, W, obstacles=()):
    """The reference NLP's single-track stage cost (cascaded_mpc.py:139-176, every if_else exact,
    no proximal term) summed along an EXECUTED closed loop instead of a plan: state X[T, 8] and the
    input U[T, 2] applied from it, with ds_n = s_{n+1} - s_n the arc length driven in step n, plus
    the time term w_time t (cascaded_mpc.py:290-291) at the end.  A scalar by which two closed
    loops of the same lap (the build's and the reference's recorded one) compare under the
    reference's own objective; returns the total and its terms."""
    X, U = np.asarray(X, np.float64), np.asarray(U, np.float64)
    T = min(len(X), len(U)) - 1
    x, u = X[:T], U[:T]
    ds = np.maximum(X[1:T + 1, IS] - X[:T, IS], 1e-9)
    ey = x[:, IEY]
    terms = {
        "deviation": W["w_dev"] * ds * ey ** 2,
        "boundary": W["w_b"] * ds * (np.where(ey < W["ey_min"], (ey - W["ey_min"]) ** 2, 0.0)
                                     + np.where(ey > W["ey_max"], (ey - W["ey_max"]) ** 2, 0.0)),
        "w": W["w_w"] * u[:, IW] ** 2,
    }
    sf = stage_functions(np.concatenate([x[:, :4], u[:, :1]], axis=1), p)
    terms["slip"] = W["w_slip"] * (np.maximum(np.real(sf["slip_f"]), 0.0) ** 2 + np.maximum(np.real(sf["slip_r"]), 0.0) ** 2)
    dFx = np.diff(u[:, IFX], append=u[-1, IFX])
    terms["Fx_slew"] = W["w_Fx"] / ds * dFx ** 2
    bar = np.zeros(T)
    for so, eo, r in obstacles:
        bar += W["w_obs"] * ds / (np.hypot(x[:, IS] - so, ey - eo) - (r + 0.1))
    terms["obstacles"] = bar
    out = {k: float(v.sum()) for k, v in terms.items()}
    out["time"] = float(W["w_time"] * T * dt)
    out["total"] = float(sum(out.values()))
    return out
