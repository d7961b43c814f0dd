"""Oracle restatement of the reference vehicle models (TEST INFRASTRUCTURE ONLY).

Arrays are batch-first float64: ``x[..., nx]``, ``u[..., nu]``, scalars ``kappa[...]``
and step ``h[...]`` broadcast against the batch.  State/action orderings follow the
reference FancyVector keys:

* kinematic state  ``[v, delta, s, ey, epsi, t]``  (models/kinematic_car.py:116-117)
* kinematic action ``[a, w]``                       (models/kinematic_car.py:81-82)
* dynamic state    ``[Ux, Uy, r, delta, s, ey, epsi, t]`` (models/dynamic_car.py:246-247)
* dynamic action   ``[Fx, w]``                      (models/dynamic_car.py:208-209)
"""
from __future__ import annotations

import numpy as np

KIN_NX, KIN_NU = 6, 2
DYN_NX, DYN_NU = 8, 2
GRAVITY = 9.88  # models/dynamic_car.py:61


# ----------------------------------------------------------------------------
# complex-step-safe |x| and sign(x): identical to np.abs / np.sign on real input;
# on complex input (x + i h, h ~ 1e-30) they carry the derivative, so the
# oracle's Jacobians come from complex-step differentiation of these same
# model functions (dyn_sqp.py), independent of the kernel's dual numbers.
# ----------------------------------------------------------------------------
def rabs(x):
    return np.where(np.real(x) >= 0, x, -x)


def rsign(x):
    return np.sign(np.real(x))


# ----------------------------------------------------------------------------
# integrators  (utils/integrators.py)
# ----------------------------------------------------------------------------
def euler_step(f, x, u, kappa, h):
    """x+ = x + h*f(x,u,k)  -- utils/integrators.py:15-23 (Euler)."""
    h = np.asarray(h, dtype=np.float64)[..., None]
    return x + h * f(x, u, kappa)


def rk4_step(f, x, u, kappa, h):
    """Classic RK4 -- utils/integrators.py:26-37.

    ``x + h*(1/6)*(k1 + 2 k2 + 2 k3 + k4)`` with the stage states
    ``x + 0.5 h k1``, ``x + 0.5 h k2``, ``x + h k3`` (integrators.py:30-34)."""
    h = np.asarray(h)[..., None]
    k1 = f(x, u, kappa)
    k2 = f(x + 0.5 * h * k1, u, kappa)
    k3 = f(x + 0.5 * h * k2, u, kappa)
    k4 = f(x + h * k3, u, kappa)
    return x + h * (1.0 / 6.0) * (k1 + 2.0 * k2 + 2.0 * k3 + k4)


# ----------------------------------------------------------------------------
# kinematic bicycle  (models/kinematic_car.py:22-64)
# ----------------------------------------------------------------------------
def kin_temporal_ode(x, u, kappa, L):
    """Temporal ODE -- models/kinematic_car.py:34-41."""
    v, delta, s, ey, epsi, t = np.moveaxis(x, -1, 0)
    a, w = np.moveaxis(u, -1, 0)
    kappa = np.asarray(kappa, dtype=np.float64)
    s_dot = (v * np.cos(epsi)) / (1.0 - ey * kappa)
    ey_dot = v * np.sin(epsi)
    epsi_dot = v * (np.tan(delta) / L) - s_dot * kappa
    one = np.ones_like(v)
    return np.stack([a * one, w * one, s_dot, ey_dot, epsi_dot, one], axis=-1)


def kin_spatial_ode(x, u, kappa, L):
    """Spatial ODE (derivatives w.r.t. arc length s) -- models/kinematic_car.py:47-60.

    rho = 1 - ey*kappa, q = rho / (v cos(epsi)):
    f' = [q a, q w, 1, rho tan(epsi), (tan(delta)/L) rho/cos(epsi) - kappa, q]."""
    v, delta, s, ey, epsi, t = np.moveaxis(x, -1, 0)
    a, w = np.moveaxis(u, -1, 0)
    kappa = np.asarray(kappa, dtype=np.float64)
    rho = 1.0 - ey * kappa
    c = np.cos(epsi)
    q = rho / (v * c)
    v_p = q * a
    d_p = q * w
    s_p = np.ones_like(v)
    ey_p = rho * np.tan(epsi)
    epsi_p = (np.tan(delta) / L) * (rho / c) - kappa
    t_p = q
    return np.stack([v_p, d_p, s_p, ey_p, epsi_p, t_p], axis=-1)


def kin_transition(x, u, kappa, dt, L):
    """``KinematicCar.transition`` = Euler(temporal ODE, dt) -- kinematic_car.py:42-45,66-68."""
    return euler_step(lambda x_, u_, k_: kin_temporal_ode(x_, u_, k_, L), x, u, kappa, dt)


def kin_spatial_transition(x, u, kappa, ds, L):
    """``KinematicCar.spatial_transition`` = Euler(spatial ODE, ds) -- kinematic_car.py:61-64,70-72."""
    return euler_step(lambda x_, u_, k_: kin_spatial_ode(x_, u_, k_, L), x, u, kappa, ds)


def kin_spatial_jacobians(x, u, kappa, ds, L):
    """Analytic A = d x+/d x, B = d x+/d u of the Euler spatial step.

    Not in the reference (CasADi AD derives these inside IPOPT with
    ``expand: True``, controllers/mpc/kinematic_mpc.py:51); derived by hand from
    models/kinematic_car.py:48-60 and cross-checked against finite differences in
    tests/test_oracle_models.py.  Returns A[..., 6, 6], B[..., 6, 2]."""
    v, delta, s, ey, epsi, t = np.moveaxis(x, -1, 0)
    a, w = np.moveaxis(u, -1, 0)
    kappa = np.asarray(kappa, dtype=np.float64) * np.ones_like(v)
    ds = np.asarray(ds, dtype=np.float64) * np.ones_like(v)
    rho = 1.0 - ey * kappa
    c = np.cos(epsi)
    te = np.tan(epsi)
    td = np.tan(delta)
    q = rho / (v * c)
    # gradient of q over (v, ey, epsi)
    q_v = -q / v
    q_ey = -kappa / (v * c)
    q_ep = q * te
    shape = v.shape
    J = np.zeros(shape + (6, 6))
    # row v' = q a ; row delta' = q w ; row t' = q
    for row, mult in ((0, a), (1, w), (5, np.ones_like(v))):
        J[..., row, 0] = q_v * mult
        J[..., row, 3] = q_ey * mult
        J[..., row, 4] = q_ep * mult
    # row ey' = rho tan(epsi)
    J[..., 3, 3] = -kappa * te
    J[..., 3, 4] = rho / (c * c)
    # row epsi' = tan(delta)/L * rho / c - kappa
    J[..., 4, 1] = (1.0 + td * td) * rho / (L * c)
    J[..., 4, 3] = -kappa * td / (L * c)
    J[..., 4, 4] = td * rho * te / (L * c)
    A = np.eye(6) + ds[..., None, None] * J
    Bm = np.zeros(shape + (6, 2))
    Bm[..., 0, 0] = ds * q
    Bm[..., 1, 1] = ds * q
    return A, Bm


# ----------------------------------------------------------------------------
# dynamic bicycle  (models/dynamic_car.py:49-191)
# ----------------------------------------------------------------------------
def dyn_params_from_config(cfg: dict) -> dict:
    """Flatten a ``config/models/dynamic_car.yaml``-schema dict (dynamic_car.py:62-151)."""
    car, env = cfg["car"], cfg["env"]
    return dict(
        l=float(car["l"]), m=float(car["m"]), Izz=float(car["Izz"]),
        a=float(car["a"]), b=float(car["b"]), h=float(car["h"]), eps=float(car["eps"]),
        Peng=float(car["Peng"]),
        Xdf=float(car["Xd"]["f"]), Xdr=float(car["Xd"]["r"]),
        Xbf=float(car["Xb"]["f"]), Xbr=float(car["Xb"]["r"]),
        Caf=float(car["C_alpha"]["f"]), Car=float(car["C_alpha"]["r"]),
        Cd=float(env["Cd"]), muf=float(env["mu"]["f"]), mur=float(env["mu"]["r"]),
        theta=float(env["theta"]), phi=float(env["phi"]), Av2=float(env["Av2"]),
        Frr=float(env["Frr"]),
    )


def dyn_forces(x, u, p):
    """Tyre/load model -- dynamic_car.py:66-142.  Returns dict of intermediates."""
    Ux, Uy, r, delta = (x[..., i] for i in range(4))
    Fx = u[..., 0]
    # input model: drive/brake split (dynamic_car.py:78-86)
    Xf = (p["Xdf"] - p["Xbf"]) / 2 * np.tanh(2 * (Fx / 1000 + 0.5)) + (p["Xdf"] + p["Xbf"]) / 2
    Fx_f = Fx * Xf
    Xr = (p["Xbr"] - p["Xdr"]) / 2 * np.tanh(-2 * (Fx / 1000 + 0.5)) + (p["Xdr"] + p["Xbr"]) / 2
    Fx_r = Fx * Xr
    # normal load with longitudinal transfer (dynamic_car.py:98-102); note l = car.l
    gz = GRAVITY * np.cos(p["theta"]) * np.cos(p["phi"]) + p["Av2"] * Ux ** 2
    Fz_f = (p["b"] / p["l"]) * p["m"] * gz - p["h"] * Fx / p["l"]
    Fz_r = (p["a"] / p["l"]) * p["m"] * gz + p["h"] * Fx / p["l"]
    # friction-ellipse lateral capacity (dynamic_car.py:107-108)
    Fymax_f = ((p["muf"] * Fz_f) ** 2 - (0.99 * Fx_f) ** 2) ** 0.5
    Fymax_r = ((p["mur"] * Fz_r) ** 2 - (0.99 * Fx_r) ** 2) ** 0.5
    # slip angles (dynamic_car.py:111-115)
    alpha_f = np.arctan((Uy + p["a"] * r) / Ux) - delta
    alpha_r = np.arctan((Uy - p["b"] * r) / Ux)
    return dict(Xf=Xf, Xr=Xr, Fx_f=Fx_f, Fx_r=Fx_r, Fz_f=Fz_f, Fz_r=Fz_r,
                Fymax_f=Fymax_f, Fymax_r=Fymax_r, alpha_f=alpha_f, alpha_r=alpha_r)


def fiala_lateral_force(alpha, Calpha, Fymax, eps):
    """Modified Fiala/brush tyre -- dynamic_car.py:119-142.

    Cubic below alphamod = atan(3 Fymax eps / C_alpha), linear+sign above."""
    ta = np.tan(alpha)
    alphamod = np.arctan((3 * Fymax * eps) / Calpha)
    inner = (-Calpha * ta + Calpha ** 2 * rabs(ta) * ta / (3 * Fymax)
             - (Calpha ** 3 * ta ** 3) / (27 * Fymax ** 2))
    outer = (-Calpha * (1 - 2 * eps + eps ** 2) * ta
             - Fymax * (3 * eps ** 2 - 2 * eps ** 3) * rsign(alpha))
    return np.where(np.real(rabs(alpha)) <= np.real(alphamod), inner, outer)


def linear_lateral_force(alpha, Calpha):
    """Build-defined 'linear tyre' (BASELINE config 3): Fy = -C_alpha tan(alpha).

    The first term of the Fiala inner branch (dynamic_car.py:123); the reference
    itself has no linear-tyre model."""
    return -Calpha * np.tan(alpha)


def dyn_temporal_ode(x, u, kappa, p, tyre="fiala"):
    """Temporal ODE -- dynamic_car.py:144-163 (Fb = 0, flat track)."""
    Ux, Uy, r, delta, s, ey, epsi, t = np.moveaxis(x, -1, 0)
    w = u[..., 1]
    kappa = np.asarray(kappa)
    F = dyn_forces(x, u, p)
    if tyre == "fiala":
        Fy_f = fiala_lateral_force(F["alpha_f"], p["Caf"], F["Fymax_f"], p["eps"])
        Fy_r = fiala_lateral_force(F["alpha_r"], p["Car"], F["Fymax_r"], p["eps"])
    elif tyre == "linear":
        Fy_f = linear_lateral_force(F["alpha_f"], p["Caf"])
        Fy_r = linear_lateral_force(F["alpha_r"], p["Car"])
    else:
        raise ValueError(tyre)
    Fx_f, Fx_r = F["Fx_f"], F["Fx_r"]
    Fd = p["Frr"] + p["Cd"] * Ux ** 2
    m, Izz, a, b = p["m"], p["Izz"], p["a"], p["b"]
    cd, sd = np.cos(delta), np.sin(delta)
    Ux_dot = (Fx_f * cd - Fy_f * sd + Fx_r - Fd) / m + r * Uy
    Uy_dot = (Fy_f * cd + Fx_f * sd + Fy_r + 0.0) / m - r * Ux
    r_dot = (a * (Fy_f * cd + Fx_f * sd) - b * Fy_r) / Izz
    delta_dot = w * np.ones_like(Ux)
    s_dot = (Ux * np.cos(epsi) - Uy * np.sin(epsi)) / (1 - kappa * ey)
    ey_dot = Ux * np.sin(epsi) + Uy * np.cos(epsi)
    epsi_dot = r - kappa * s_dot
    t_dot = np.ones_like(Ux)
    return np.stack([Ux_dot, Uy_dot, r_dot, delta_dot, s_dot, ey_dot, epsi_dot, t_dot], axis=-1)


def dyn_spatial_ode(x, u, kappa, p, tyre="fiala"):
    """Spatial ODE = temporal / s_dot, s' = 1 -- dynamic_car.py:169-187."""
    fd = dyn_temporal_ode(x, u, kappa, p, tyre)
    s_dot = fd[..., 4]
    fp = fd / s_dot[..., None]
    fp[..., 4] = 1.0
    fp[..., 7] = 1.0 / s_dot
    return fp


def dyn_transition(x, u, kappa, dt, p, tyre="fiala"):
    """``DynamicCar.transition`` = RK4(temporal ODE, dt) -- dynamic_car.py:166-167."""
    return rk4_step(lambda x_, u_, k_: dyn_temporal_ode(x_, u_, k_, p, tyre), x, u, kappa, dt)


def dyn_spatial_transition(x, u, kappa, ds, p, tyre="fiala"):
    """``DynamicCar.spatial_transition`` = RK4(spatial ODE, ds) -- dynamic_car.py:188-191."""
    return rk4_step(lambda x_, u_, k_: dyn_spatial_ode(x_, u_, k_, p, tyre), x, u, kappa, ds)


# ----------------------------------------------------------------------------
# dynamic point mass  (models/dynamic_point_mass.py:26-103), the cascaded tail
# state [V, s, ey, epsi, t] (:147-161), action [Fx, Fy] (:115-126); same car config
# as the dynamic bicycle (simulation/racing.py:44-46 builds it from carconfig)
# ----------------------------------------------------------------------------
PM_NX, PM_NU = 5, 2


def pm_temporal_ode(x, u, kappa, p):
    """dynamic_point_mass.py:76-88 (Fb = 0)."""
    V, s, ey, epsi, t = np.moveaxis(x, -1, 0)
    Fx, Fy = u[..., 0], u[..., 1]
    kappa = np.asarray(kappa)
    Fd = p["Frr"] + p["Cd"] * V ** 2
    V_dot = (Fx - Fd) / p["m"]
    s_dot = (V * np.cos(epsi)) / (1 - kappa * ey)
    ey_dot = V * np.sin(epsi)
    epsi_dot = Fy / (p["m"] * V) - kappa * s_dot
    return np.stack([V_dot, s_dot, ey_dot, epsi_dot, np.ones_like(V)], axis=-1)


def pm_spatial_ode(x, u, kappa, p):
    """dynamic_point_mass.py:90-100: temporal / s_dot, s' = 1."""
    fd = pm_temporal_ode(x, u, kappa, p)
    s_dot = fd[..., 1]
    fp = fd / s_dot[..., None]
    fp[..., 1] = 1.0
    fp[..., 4] = 1.0 / s_dot
    return fp


def pm_spatial_transition(x, u, kappa, ds, p):
    """``DynamicPointMass.spatial_transition`` = Euler(spatial ODE, ds) (:98-100)."""
    return euler_step(lambda x_, u_, k_: pm_spatial_ode(x_, u_, k_, p), x, u, kappa, ds)


def st_to_pm(x):
    """Switching constraints of the cascaded MPC (cascaded_mpc.py:256-277): the point
    mass starts at V = |(Ux, Uy)|, s, ey, epsi + atan(Uy / Ux), t of the last
    single-track state."""
    Ux, Uy, s, ey, epsi, t = x[..., 0], x[..., 1], x[..., 4], x[..., 5], x[..., 6], x[..., 7]
    return np.stack([(Ux ** 2 + Uy ** 2) ** 0.5, s, ey, np.arctan(Uy / Ux) + epsi, t], axis=-1)


def dyn_lateral_forces(x, u, p, tyre="fiala"):
    """``DynamicCar.Fy_f`` / ``Fy_r`` (dynamic_car.py:120-142): (Fy_f, Fy_r)."""
    F = dyn_forces(x, u, p)
    if tyre == "fiala":
        return (fiala_lateral_force(F["alpha_f"], p["Caf"], F["Fymax_f"], p["eps"]),
                fiala_lateral_force(F["alpha_r"], p["Car"], F["Fymax_r"], p["eps"]))
    return linear_lateral_force(F["alpha_f"], p["Caf"]), linear_lateral_force(F["alpha_r"], p["Car"])
