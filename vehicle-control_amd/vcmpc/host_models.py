"""Host-side numpy dynamic-bicycle rollout used only to screen synthetic workloads
(workload.dynamic_batch): a sample whose warm-start prediction leaves the model's
domain is re-drawn before anything reaches the GPU.  It is not on the solve path
(every solve runs in libvcmpc.so) and is not the test oracle (oracle/)."""
from __future__ import annotations

import numpy as np

G = 9.88  # models/dynamic_car.py:61


def dyn_params(cfg) -> dict:
    car, env = cfg["car"], cfg["env"]
    return dict(l=float(car["l"]), m=float(car["m"]), Izz=float(car["Izz"]), a=float(car["a"]), b=float(car["b"]),
                h=float(car["h"]), Xdf=float(car["Xd"]["f"]), Xdr=float(car["Xd"]["r"]),
                Xbf=float(car["Xb"]["f"]), Xbr=float(car["Xb"]["r"]), Caf=float(car["C_alpha"]["f"]),
                Car=float(car["C_alpha"]["r"]), Cd=float(env["Cd"]), Frr=float(env["Frr"]),
                muf=float(env["mu"]["f"]), mur=float(env["mu"]["r"]), eps=float(car["eps"]))


def _ode(x, u, k, p, tyre):
    Ux, Uy, r, d, s, ey, ep, t = x.T
    Fx, w = u.T
    Xf = (p["Xdf"] - p["Xbf"]) / 2 * np.tanh(2 * (Fx / 1000 + 0.5)) + (p["Xdf"] + p["Xbf"]) / 2
    Xr = (p["Xbr"] - p["Xdr"]) / 2 * np.tanh(-2 * (Fx / 1000 + 0.5)) + (p["Xdr"] + p["Xbr"]) / 2
    Fxf, Fxr = Fx * Xf, Fx * Xr
    Fzf = p["b"] / p["l"] * p["m"] * G - p["h"] * Fx / p["l"]
    Fzr = p["a"] / p["l"] * p["m"] * G + p["h"] * Fx / p["l"]
    af = np.arctan((Uy + p["a"] * r) / Ux) - d
    ar = np.arctan((Uy - p["b"] * r) / Ux)
    if tyre == "linear":
        Fyf, Fyr = -p["Caf"] * np.tan(af), -p["Car"] * np.tan(ar)
    else:  # screening only: saturate at the friction limit
        Fyf = -np.clip(p["Caf"] * np.tan(af), -p["muf"] * Fzf, p["muf"] * Fzf)
        Fyr = -np.clip(p["Car"] * np.tan(ar), -p["mur"] * Fzr, p["mur"] * Fzr)
    cd, sd = np.cos(d), np.sin(d)
    sdot = (Ux * np.cos(ep) - Uy * np.sin(ep)) / (1 - k * ey)
    f = np.stack([(Fxf * cd - Fyf * sd + Fxr - p["Frr"] - p["Cd"] * Ux ** 2) / p["m"] + r * Uy,
                  (Fyf * cd + Fxf * sd + Fyr) / p["m"] - r * Ux,
                  (p["a"] * (Fyf * cd + Fxf * sd) - p["b"] * Fyr) / p["Izz"],
                  w, sdot, Ux * np.sin(ep) + Uy * np.cos(ep), r - k * sdot, np.ones_like(Ux)], 1)
    f = f / sdot[:, None]
    f[:, 4] = 1.0
    return f


def dyn_rollout_np(x0, ubar, kappa, ds, p, tyre="linear"):
    """Spatial RK4 rollout, x[B, N, 8] (N columns, dynamics for k < N - 1)."""
    B, N = ubar.shape[:2]
    X = np.empty((B, N, 8))
    X[:, 0] = x0
    with np.errstate(all="ignore"):
        for k in range(N - 1):
            x, u, kk, h = X[:, k], ubar[:, k], kappa[:, k], ds[:, k:k + 1]
            k1 = _ode(x, u, kk, p, tyre)
            k2 = _ode(x + 0.5 * h * k1, u, kk, p, tyre)
            k3 = _ode(x + 0.5 * h * k2, u, kk, p, tyre)
            k4 = _ode(x + h * k3, u, kk, p, tyre)
            X[:, k + 1] = x + h / 6 * (k1 + 2 * k2 + 2 * k3 + k4)
    return X


def pm_rollout_np(xs_last, u_pm, kappa, ds, p):
    """Point-mass spatial Euler rollout from the switch state of the last single-track
    state (cascaded_mpc.py:256-277), P[B, M, 5] = (V, s, ey, epsi, t)."""
    B, M = u_pm.shape[:2]
    P = np.empty((B, M, 5))
    Ux, Uy = xs_last[:, 0], xs_last[:, 1]
    with np.errstate(all="ignore"):
        P[:, 0] = np.stack([np.hypot(Ux, Uy), xs_last[:, 4], xs_last[:, 5], np.arctan(Uy / Ux) + xs_last[:, 6],
                            xs_last[:, 7]], 1)
        for m in range(M - 1):
            V, s, ey, ep, t = P[:, m].T
            Fx, Fy = u_pm[:, m].T
            k = kappa[:, m]
            sdot = V * np.cos(ep) / (1 - k * ey)
            f = np.stack([(Fx - p["Frr"] - p["Cd"] * V ** 2) / p["m"], sdot, V * np.sin(ep),
                          Fy / (p["m"] * V) - k * sdot, np.ones_like(V)], 1) / sdot[:, None]
            f[:, 1] = 1.0
            P[:, m + 1] = P[:, m] + ds[:, m:m + 1] * f
    return P
