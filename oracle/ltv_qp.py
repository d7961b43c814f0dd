"""Oracle restatement of the LTV-QP contract for the kinematic MPC (TEST INFRASTRUCTURE ONLY).

The reference has no QP: every control step solves the nonlinear program of
controllers/mpc/kinematic_mpc.py:15-30 with IPOPT.  The build replaces that solve
by one *linear-time-varying QP step* (SURVEY 8a row A8), defined here once and
implemented identically by the HIP kernel:

1. predict    x_0 = x0,  x_{k+1} = x_k + ds_k f'(x_k, u_k, kappa_k)
              (spatial Euler, models/kinematic_car.py:47-64, integrators.py:15-23)
2. linearize  A_k = dx_{k+1}/dx_k,  B_k = dx_{k+1}/du_k  at (xbar_k, ubar_k)
3. condense   dx_k = G_k dz  (dx_0 = 0),  dz = [da_0, dw_0, da_1, dw_1, ...]
4. QP         min 1/2 dz'H dz + g'dz  s.t. input boxes and state rows below,
              where the cost is the reference NLP cost (kinematic_mpc.py:101-158)
              written exactly in the linearised states, with every ``if_else``
              branch frozen at the predicted trajectory, plus
              a proximal term  prox * ||dz||^2  (the NLP Hessian is
              singular along the acceleration directions).
5. output     u* = ubar + dz*,  x* = xbar + G dz*,  u0 = u*_0.

Cost terms (stage n = 0..N-1, terminal state x_N):
  w_b ds_n (ey_n - ey_min)^2  if  eybar_n < ey_min          kinematic_mpc.py:110-114
  w_b ds_n (ey_n - ey_max)^2  if  eybar_n > ey_max          kinematic_mpc.py:116-120
  w_dev ds_n ey_n^2                                          kinematic_mpc.py:122
  w_w w_n^2                                                  kinematic_mpc.py:124
  w_a (a_{n+1} - a_n)^2   for n < N-1                        kinematic_mpc.py:126-128
  obstacle barrier, convexified in ey_n (W["obstacles"] set)  kinematic_mpc.py:130-133, obstacles.py
  w_v (v_N - v_max)^2     if  vbar_N >= v_max                kinematic_mpc.py:144-148
  w_time t_N + w_ey ey_N^2 + w_epsi epsi_N^2                 kinematic_mpc.py:149-157
Constraints:
  a_min <= a_n <= a_max, w_min <= w_n <= w_max, n = 0..N-1  kinematic_mpc.py:88-93
  v_n >= v_min, delta_min <= delta_n <= delta_max, n = 1..N-1  kinematic_mpc.py:80-85
  (n = 0 is the fixed initial state, kinematic_mpc.py:23-25: a constant, dropped.)
  optional trust region |du_n| <= (trust_a, trust_w) tightening the input boxes
  (SQP globalisation used by the closed-loop controller; 0 = off, the default).
"""
from __future__ import annotations

import numpy as np

from . import models as M
from . import obstacles as OB
from .qp import Gram

IV, ID, IS, IEY, IEP, IT = range(6)
IA, IW = 0, 1
ELASTIC_EPS_T = 1e-8   # elastic slacks' quadratic cost (elastic_qp; kin_ric.hip uses the same)


def kin_weights(cfg: dict) -> dict:
    """Pull the numbers the QP consumes out of a kinematic controller config
    (reference schema: config/controllers/kinematic.yaml)."""
    cw, ic, sc = cfg["cost_weights"], cfg["input_constraints"], cfg["state_constraints"]
    qp = cfg.get("qp", {})
    return dict(
        w_time=float(cw["time"]), w_ey=float(cw["ey"]), w_epsi=float(cw["epsi"]),
        w_v=float(cw["v"]), w_w=float(cw["w"]), w_a=float(cw["a"]),
        w_dev=float(cw["deviation"]), w_b=float(cw["boundary"]),
        a_min=float(ic["a_min"]), a_max=float(ic["a_max"]),
        w_min=float(ic["w_min"]), w_max=float(ic["w_max"]),
        v_min=float(sc["v_min"]), v_max=float(sc["v_max"]),
        delta_min=float(sc["delta_min"]), delta_max=float(sc["delta_max"]),
        ey_min=float(sc["ey_min"]), ey_max=float(sc["ey_max"]),
        prox=float(qp.get("prox", 1e-4)), w_obs=float(cw.get("obstacles", 0.0)), obstacles=[],
        obs_margin_min=OB.MARGIN_MIN,
        trust_a=float(qp.get("trust_a", 0.0)), trust_w=float(qp.get("trust_w", 0.0)),
    )


def kin_predict(x0, ubar, kappa, ds, L):
    """Step 1: roll the warm-start inputs forward.  x0[B,6], ubar[B,N,2] -> xbar[B,N+1,6]."""
    B, N = ubar.shape[:2]
    xbar = np.empty((B, N + 1, 6))
    xbar[:, 0] = x0
    for k in range(N):
        xbar[:, k + 1] = M.kin_spatial_transition(xbar[:, k], ubar[:, k], kappa[:, k], ds[:, k], L)
    return xbar


def kin_linearize(xbar, ubar, kappa, ds, L):
    """Step 2: A[B,N,6,6], Bm[B,N,6,2] along the predicted trajectory."""
    N = ubar.shape[1]
    return M.kin_spatial_jacobians(xbar[:, :N], ubar, kappa, ds, L)


def kin_condense(A, Bm):
    """Step 3: G[B,N+1,6,2N] with dx_k = G[:,k] @ dz  (block lower triangular)."""
    B, N = A.shape[:2]
    G = np.zeros((B, N + 1, 6, 2 * N))
    for k in range(N):
        G[:, k + 1] = np.einsum("bij,bjn->bin", A[:, k], G[:, k])
        G[:, k + 1, :, 2 * k:2 * k + 2] += Bm[:, k]
    return G


def kin_qp(x0, ubar, kappa, ds, L, W, x_ws=None):
    """Steps 1-4.  Returns dict with xbar, G, H[B,n,n], g[B,n], and the inequality
    system C[B,m,n] dz <= d[B,m] (one-sided rows, m = 4N + 3(N-1)).

    x_ws[B,N+1,6] given: *multiple shooting* (vc_qp.ms, csrc/kin_ric.hip).  The QP is linearised
    at the warm-start states (x0 in column 0, s = s0 + cumsum ds since s' = 1) instead of the
    rollout of ubar; the defects c_k = F(x_k, u_k) - x_{k+1} enter through their linear rollout
    e (e_0 = 0, e_{k+1} = A_k e_k + c_k): dx_k = G_k dz + e_k.  Every `if_else` branch and the
    obstacle model stay frozen at the warm-start states; the residuals they multiply are taken
    at x_ws + e (the kernel's q + Q e, d - C e)."""
    x0 = np.asarray(x0, np.float64)
    ubar = np.asarray(ubar, np.float64)
    kappa = np.asarray(kappa, np.float64)
    ds = np.asarray(ds, np.float64)
    B, N = ubar.shape[:2]
    n = 2 * N
    if x_ws is None:
        xbar = kin_predict(x0, ubar, kappa, ds, L)
        eo = np.zeros_like(xbar)
    else:
        xbar = np.array(x_ws, np.float64, copy=True)
        xbar[:, 0] = x0
        xbar[:, 1:, IS] = x0[:, None, IS] + np.cumsum(ds, axis=1)
    A, Bm = kin_linearize(xbar, ubar, kappa, ds, L)
    G = kin_condense(A, Bm)
    if x_ws is not None:
        eo = np.zeros_like(xbar)
        for k in range(N):
            c = M.kin_spatial_transition(xbar[:, k], ubar[:, k], kappa[:, k], ds[:, k], L) - xbar[:, k + 1]
            eo[:, k + 1] = np.einsum("bij,bj->bi", A[:, k], eo[:, k]) + c
    xv = xbar + eo   # the values the residuals are taken at

    H = np.zeros((B, n, n))
    g = np.zeros((B, n))
    gram = Gram(B, n)

    def add_square(c, r0, row):
        # c * (r0 + row.dz)^2  -> H += 2c row row', g += 2c r0 row
        c = np.broadcast_to(np.asarray(c, np.float64), (B,))
        gram.add(2.0 * c, row)
        g[:] += 2.0 * (c * r0)[:, None] * row

    # stage costs on ey_n (n = 0 is constant: G[:,0] = 0)
    for k in range(1, N):
        ey = xbar[:, k, IEY]
        eyv = xv[:, k, IEY]
        row = G[:, k, IEY]
        add_square(W["w_dev"] * ds[:, k], eyv, row)
        lo = ey < W["ey_min"]
        hi = ey > W["ey_max"]
        add_square(np.where(lo, W["w_b"] * ds[:, k], 0.0), eyv - W["ey_min"], row)
        add_square(np.where(hi, W["w_b"] * ds[:, k], 0.0), eyv - W["ey_max"], row)
        if W.get("obstacles"):  # kinematic_mpc.py:130-133, convexified in ey (obstacles.py)
            p_o, q_o = OB.ey_model(xbar[:, k, IS], ey, W["w_obs"] * ds[:, k], W["obstacles"],
                                   W.get("obs_margin_min", OB.MARGIN_MIN),
                                   inside=bool(W.get("obs_inside", False)))
            gram.add(q_o, row)
            g[:] += (p_o + q_o * (eyv - ey))[:, None] * row
    # input costs: w_w w^2 and slew w_a (a_{n+1}-a_n)^2
    for k in range(N):
        e = np.zeros((B, n)); e[:, 2 * k + IW] = 1.0
        add_square(W["w_w"], ubar[:, k, IW], e)
    for k in range(N - 1):
        e = np.zeros((B, n)); e[:, 2 * (k + 1) + IA] = 1.0; e[:, 2 * k + IA] = -1.0
        add_square(W["w_a"], ubar[:, k + 1, IA] - ubar[:, k, IA], e)
    # terminal costs
    vN = xbar[:, N, IV]
    add_square(np.where(vN >= W["v_max"], W["w_v"], 0.0), xv[:, N, IV] - W["v_max"], G[:, N, IV])
    g += W["w_time"] * G[:, N, IT]
    add_square(W["w_ey"], xv[:, N, IEY], G[:, N, IEY])
    add_square(W["w_epsi"], xv[:, N, IEP], G[:, N, IEP])
    # proximal term prox*||dz||^2
    gram.flush(H)
    H += 2.0 * W["prox"] * np.eye(n)

    # inequalities C dz <= d
    rows, rhs = [], []
    I = np.eye(n)
    tr = {IA: W.get("trust_a", 0.0), IW: W.get("trust_w", 0.0)}
    for k in range(N):
        for j, (lo, hi) in ((IA, (W["a_min"], W["a_max"])), (IW, (W["w_min"], W["w_max"]))):
            e = np.broadcast_to(I[2 * k + j], (B, n))
            up, dn = hi - ubar[:, k, j], ubar[:, k, j] - lo
            if tr[j] > 0:  # trust region |du| <= tr (SQP globalisation; 0 = off)
                up, dn = np.minimum(up, tr[j]), np.minimum(dn, tr[j])
            rows.append(e); rhs.append(up)
            rows.append(-e); rhs.append(dn)
    for k in range(1, N):
        rows.append(-G[:, k, IV]); rhs.append(xv[:, k, IV] - W["v_min"])
        rows.append(G[:, k, ID]); rhs.append(W["delta_max"] - xv[:, k, ID])
        rows.append(-G[:, k, ID]); rhs.append(xv[:, k, ID] - W["delta_min"])
    C = np.stack(rows, axis=1)
    d = np.stack(rhs, axis=1)
    return dict(xbar=xbar, e=eo, A=A, Bm=Bm, G=G, H=H, g=g, C=C, d=d)


def elastic_qp(H, g, C, d, ne, rho, eps_t=ELASTIC_EPS_T):
    """The QP with its last `ne` rows made *elastic*: row i gets its own slack t_i >= 0,
    C_i z - t_i <= d_i, at cost rho t_i + eps_t t_i^2 (the QP model of an exact L1 penalty,
    Fletcher's Sl1QP; eps_t keeps the Hessian definite).  Always feasible; its z equals the plain
    QP's whenever that is feasible with the elastic rows' multipliers below rho.  Returns
    (H2, g2, C2, d2) over (z, t) -- csrc/kin_ric.hip's elastic rows (vc_qp.elastic = rho)."""
    B, n = g.shape
    m = C.shape[1]
    nb = m - ne
    H2 = np.zeros((B, n + ne, n + ne))
    H2[:, :n, :n] = H
    H2[:, n:, n:] = 2.0 * eps_t * np.eye(ne)
    g2 = np.concatenate([g, np.full((B, ne), rho)], axis=1)
    C2 = np.zeros((B, m + ne, n + ne))
    C2[:, :m, :n] = C
    C2[:, nb:m, n:] = -np.eye(ne)
    C2[:, m:, n:] = -np.eye(ne)
    d2 = np.concatenate([d, np.zeros((B, ne))], axis=1)
    return H2, g2, C2, d2


def kin_ltv_solve(x0, ubar, kappa, ds, L, W, x_ws=None, elastic=0.0, **qp_kw):
    """Steps 1-5 with the exact oracle QP solver.  Returns dict with u_star[B,N,2],
    x_star[B,N+1,6], u0[B,2], dz, lam, kkt (certificate), plus the QP data.  elastic = rho > 0:
    the v / delta state rows are elastic (elastic_qp; the slacks in `t`)."""
    from .qp import solve_qp_batch

    Q = kin_qp(x0, ubar, kappa, ds, L, W, x_ws=x_ws)
    B, N = np.asarray(ubar).shape[:2]
    if elastic > 0.0:
        n = 2 * N
        sol = solve_qp_batch(*elastic_qp(Q["H"], Q["g"], Q["C"], Q["d"], 3 * (N - 1), elastic), **qp_kw)
        sol["t"] = sol["z"][:, n:]
        sol["z"] = sol["z"][:, :n]
    else:
        sol = solve_qp_batch(Q["H"], Q["g"], Q["C"], Q["d"], **qp_kw)
    dz = sol["z"]
    u_star = np.asarray(ubar, np.float64) + dz.reshape(B, N, 2)
    x_star = Q["xbar"] + Q["e"] + np.einsum("bkin,bn->bki", Q["G"], dz)
    Q.update(sol)
    Q.update(dz=dz, u_star=u_star, x_star=x_star, u0=u_star[:, 0].copy())
    return Q


def kin_horizon_params(state, state_prediction, mpc_dt, N, k_of_s):
    """Host-side parameter construction of ``KinematicMPC._init_horizon``
    (kinematic_mpc.py:170-187), including its quirks: ds uses the *unshifted*
    warm-start speeds plus 0.5 m, and the curvature preview is evaluated at
    s0 + cumsum(ds_traj with ds_traj[0] = 0)[:N] (an off-by-one vs ds).
    state[6], state_prediction[6, N+1] -> (ds[N], kappa[N])."""
    ds_traj = np.full(N + 1, mpc_dt) * state_prediction[IV, :] + 0.5
    ds = ds_traj[:-1].copy()
    ds_traj[0] = 0.0
    s_traj = (np.cumsum(ds_traj) + state[IS])[:-1]
    return ds, np.asarray(k_of_s(s_traj), np.float64)
