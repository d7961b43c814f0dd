"""Synthetic batched workloads of BASELINE.json's configs.

C2/C4 (kinematic LTV-MPC, N = 20, fp64), seeded ``numpy.random.default_rng``:
  x0:    v ~ U(3, 10), delta ~ U(-0.15, 0.15), s ~ U(0, 315.5), ey ~ U(-2, 2),
         epsi ~ U(-0.2, 0.2), t = 0
  kappa: piecewise constant over 4 segments, each ~ U(0, 0.047) (ippodromo's
         range of back-solved curvature)
  ubar:  U(-1, 1) * (3, 0.4) (the input boxes of kinematic.yaml)
  ds:    per stage, ds_n = mpc_dt * vbar_n + 0.5 (kinematic_mpc.py:178-182) with
         vbar the speed prediction of the warm start: the rollout of ubar from x0 on the
         provisional grid mpc_dt * v0 + 0.5
Problems whose warm-start rollout (on the final grid) would leave the model's domain (v below
1 m/s, |epsi| above 1.2 rad, where v cos(epsi) -> 0 makes the spatial ODE singular) are
re-drawn, so every generated problem is well posed.
"""
from __future__ import annotations

import numpy as np

V_LO = 1.0
EPSI_HI = 1.2


def _kin_rollout(x0, ubar, kappa, ds, L, speeds=False):
    """Host-side Euler rollout used only to screen samples (kinematic_car.py:47-64); with
    ``speeds`` also the predicted speeds v[B, N+1]."""
    B, N = kappa.shape
    x = x0.copy()
    v_traj = [x[:, 0].copy()]
    vmin = x[:, 0].copy()
    emax = np.abs(x[:, 4])
    for k in range(N):
        v, d, s, ey, ep, t = x.T
        rho = 1.0 - ey * kappa[:, k]
        c = np.cos(ep)
        q = rho / (v * c)
        f = np.stack([q * ubar[:, k, 0], q * ubar[:, k, 1], np.ones(B), rho * np.tan(ep),
                      np.tan(d) / L * rho / c - kappa[:, k], q], 1)
        x = x + ds[:, k:k + 1] * f
        v_traj.append(x[:, 0].copy())
        vmin = np.minimum(vmin, x[:, 0])
        emax = np.maximum(emax, np.abs(x[:, 4]))
    ok = np.isfinite(x).all(1) & (vmin > V_LO) & (emax < EPSI_HI)
    return (ok, np.stack(v_traj, 1)) if speeds else ok


def kinematic_batch(B: int, N: int = 20, seed: int = 31, mpc_dt: float = 0.03, L: float = 2.5,
                    a_max: float = 3.0, w_max: float = 0.4):
    """Returns dict x0[B,6], kappa[B,N], ds[B,N], ubar[B,N,2] (float64, C-contiguous)."""
    rng = np.random.default_rng(seed)
    out = {k: [] for k in ("x0", "kappa", "ds", "ubar")}
    have = 0
    while have < B:
        m = max(2 * (B - have), 16)
        x0 = np.zeros((m, 6))
        x0[:, 0] = rng.uniform(3, 10, m)
        x0[:, 1] = rng.uniform(-0.15, 0.15, m)
        x0[:, 2] = rng.uniform(0, 315.5, m)
        x0[:, 3] = rng.uniform(-2, 2, m)
        x0[:, 4] = rng.uniform(-0.2, 0.2, m)
        seg = rng.uniform(0, 0.047, (m, 4))
        kappa = np.repeat(seg, -(-N // 4), axis=1)[:, :N]
        ubar = rng.uniform(-1, 1, (m, N, 2)) * np.array([a_max, w_max])
        ds_c = np.repeat(mpc_dt * x0[:, :1] + 0.5, N, axis=1)
        with np.errstate(all="ignore"):
            ok_pred, v_pred = _kin_rollout(x0, ubar, kappa, ds_c, L, speeds=True)
            ds = mpc_dt * v_pred[:, :N] + 0.5             # kinematic_mpc.py:178-182
            # both the speed prediction and the rollout on the final grid inside the domain
            ok = ok_pred & _kin_rollout(x0, ubar, kappa, ds, L) & np.isfinite(ds).all(1)
        for k, v in (("x0", x0), ("kappa", kappa), ("ds", ds), ("ubar", ubar)):
            out[k].append(v[ok])
        have += int(ok.sum())
    return {k: np.ascontiguousarray(np.concatenate(v)[:B]) for k, v in out.items()}


def shard(B_total: int, rank: int, world: int):
    """Contiguous shard [lo, hi) of rank `rank` (B/world per GPU)."""
    per = B_total // world
    rem = B_total % world
    lo = rank * per + min(rank, rem)
    return lo, lo + per + (1 if rank < rem else 0)


C4_CHUNK = 8192   # the C4 problem set is generated in 8192-problem chunks (seed + chunk index),
                  # so every world size solves the same problems


def c4_shard(total: int, rank: int, world: int, seed: int = 31, N: int = 20):
    """Contiguous shard [lo, hi) of the C4 problem set of `total` kinematic problems
    and its data; chunk c of C4_CHUNK problems is kinematic_batch(seed = seed + 1000003 (c + 1))."""
    lo, hi = shard(total, rank, world)
    parts = []
    for c in range(lo // C4_CHUNK, -(-hi // C4_CHUNK)):
        a, b = c * C4_CHUNK, min((c + 1) * C4_CHUNK, total)
        d = kinematic_batch(b - a, N=N, seed=seed + 1000003 * (c + 1))
        parts.append({k: v[max(lo, a) - a:min(hi, b) - a] for k, v in d.items()})
    return lo, hi, {k: np.ascontiguousarray(np.concatenate([p[k] for p in parts])) for k in parts[0]}


# ----------------------------------------------------------------------------
# C3 / C5: dynamic single-track SQP-MPC, N = 40, fp32
# ----------------------------------------------------------------------------
def _dyn_screen(x0, ubar, kappa, ds, p, tyre, domain_only=False):
    """Warm-start rollout inside the model's domain (host-side screen only).  domain_only: just
    the spatial model's own domain -- finite, Ux > 0 and s' = (Ux cos epsi - Uy sin epsi) /
    (1 - kappa ey) > 0 at every stage (dynamic_car.py:169-191 divides by s')."""
    from .host_models import dyn_rollout_np  # local numpy RK4 used only for screening
    X = dyn_rollout_np(x0, ubar, kappa, ds, p, tyre)
    ok = np.isfinite(X).all(axis=(1, 2))
    with np.errstate(invalid="ignore", over="ignore"):
        if domain_only:
            k = kappa[:, :X.shape[1]]
            sdot = (X[..., 0] * np.cos(X[..., 6]) - X[..., 1] * np.sin(X[..., 6])) / (1.0 - k * X[..., 5])
            return ok & (X[..., 0] > 0).all(1) & (sdot > 0).all(1)
        ok &= (X[..., 0] > 5.0).all(1) & (np.abs(X[..., 1]) < 3.0).all(1) & (np.abs(X[..., 2]) < 1.5).all(1)
        ok &= (np.abs(X[..., 3]) < 0.45).all(1) & (np.abs(X[..., 6]) < 0.8).all(1)
    return ok


def dynamic_batch(B: int, N: int = 40, seed: int = 31, mpc_dt: float = 0.03, tyre: str = "linear",
                  car_cfg=None, ranges: str = "traces", stats: dict | None = None):
    """BASELINE config 3 workload, float32, seeded:
      x0:    Ux ~ U(8, 22), Uy ~ U(-0.3, 0.3), r ~ U(-0.2, 0.6), delta ~ U(-0.07, 0.24),
             s ~ U(0, 300), ey ~ U(-2.5, 2.5), epsi ~ U(-0.3, 0.3), t = 0
             (the reference traces' ranges; Ux starts at 8 m/s because below that the
             spatial RK4 step ds = mpc_dt Ux of the stiff lateral dynamics, Calpha ~ 2-4e5,
             leaves RK4's stability region -- the reference's singletrack runs at 10-22 m/s)
      kappa: piecewise constant over 4 segments, each ~ U(0, 0.047)
      ds:    mpc_dt * Ux0 for every stage (cascaded_mpc.py:323-327, constant-speed prediction)
      ubar:  Fx = F0 + U(-300, 300) with F0 ~ U(-2000, 2000) per problem; w ~ U(-0.1, 0.1)
    Problems whose warm-start rollout leaves the model's domain are re-drawn.

    ranges="survey": SURVEY 8(d)'s C3 sampler as written -- Ux ~ U(5, 22), ey ~ U(-3, 3) and the
    Fx warm start ~ U(-6000, 6000) N per stage (the other ranges as above); only warm starts
    whose rollout leaves the spatial model's own domain (Ux <= 0, s' <= 0, non-finite) are
    re-drawn, so low-speed problems and hard-braking warm starts stay in the set.  ``stats``
    (a dict) receives the number drawn and the number re-drawn."""
    from .config import load_config
    from .host_models import dyn_params
    p = dyn_params(car_cfg if car_cfg is not None else load_config("dynamic_car"))
    rng = np.random.default_rng(seed)
    out = {k: [] for k in ("x0", "kappa", "ds", "ubar")}
    have = 0
    while have < B:
        m = max(2 * (B - have), 16)
        x0 = np.zeros((m, 8))
        survey = ranges == "survey"
        x0[:, 0] = rng.uniform(5 if survey else 8, 22, m)
        x0[:, 1] = rng.uniform(-0.3, 0.3, m)
        x0[:, 2] = rng.uniform(-0.2, 0.6, m)
        x0[:, 3] = rng.uniform(-0.07, 0.24, m)
        x0[:, 4] = rng.uniform(0, 300, m)
        x0[:, 5] = rng.uniform(-3, 3, m) if survey else rng.uniform(-2.5, 2.5, m)
        x0[:, 6] = rng.uniform(-0.3, 0.3, m)
        seg = rng.uniform(0, 0.047, (m, 4))
        kappa = np.repeat(seg, -(-N // 4), axis=1)[:, :N]
        ds = np.repeat(mpc_dt * x0[:, :1], N, axis=1)
        if survey:
            fx = rng.uniform(-6000, 6000, (m, N))
        else:
            fx = rng.uniform(-2000, 2000, (m, 1)) + rng.uniform(-300, 300, (m, N))
        ubar = np.stack([fx, rng.uniform(-0.1, 0.1, (m, N))], -1)
        ok = _dyn_screen(x0, ubar, kappa, ds, p, tyre, domain_only=survey)
        if stats is not None:
            stats["drawn"] = stats.get("drawn", 0) + m
            stats["redrawn"] = stats.get("redrawn", 0) + int((~ok).sum())
        for k, v in (("x0", x0), ("kappa", kappa), ("ds", ds), ("ubar", ubar)):
            out[k].append(v[ok])
        have += int(ok.sum())
    return {k: np.ascontiguousarray(np.concatenate(v)[:B].astype(np.float32)) for k, v in out.items()}


def cascaded_batch(B: int, N: int = 20, M: int = 40, ds_pm: float = 3.0, seed: int = 31, mpc_dt: float = 0.03,
                   tyre: str = "fiala", car_cfg=None):
    """Cascaded NMPC workload (single-track N + point-mass M stages), float64, seeded:
    the single-track part is dynamic_batch's (x0, kappa, ds, ubar over N stages); the
    point-mass stages get ds = ds_pm, piecewise-constant curvature ~ U(0, 0.047) over
    4 segments, Fx = the drag at Ux0 + U(-300, 300) N and Fy = m Ux0^2 kappa (the
    steady-state cornering force) + U(-300, 300) N.  Problems whose warm-start
    rollout leaves the model's domain (V < 5, |ey| > 4, |epsi| > 0.6) are re-drawn."""
    from .config import load_config
    from .host_models import dyn_params, dyn_rollout_np, pm_rollout_np
    p = dyn_params(car_cfg if car_cfg is not None else load_config("dynamic_car"))
    rng = np.random.default_rng(seed + 1)
    out = {k: [] for k in ("x0", "kappa", "ds", "ubar")}
    have, draw = 0, 0
    while have < B:
        m_ = max(2 * (B - have), 16)
        d = dynamic_batch(m_, N=N, seed=seed + 1000 * draw, mpc_dt=mpc_dt, tyre=tyre, car_cfg=car_cfg)
        draw += 1
        d = {k: v.astype(np.float64) for k, v in d.items()}
        seg = rng.uniform(0, 0.047, (m_, 4))
        kp = np.repeat(seg, -(-M // 4), axis=1)[:, :M]
        ux = d["x0"][:, :1]
        Fx = p["Frr"] + p["Cd"] * ux ** 2 + rng.uniform(-300, 300, (m_, M))
        Fy = p["m"] * ux ** 2 * kp + rng.uniform(-300, 300, (m_, M))
        u_pm = np.stack([Fx, Fy], -1)
        ds_p = np.full((m_, M), ds_pm)
        X = dyn_rollout_np(d["x0"], d["ubar"], d["kappa"], d["ds"], p, tyre)
        P = pm_rollout_np(X[:, -1], u_pm, kp, ds_p, p)
        with np.errstate(invalid="ignore"):
            ok = np.isfinite(P).all(axis=(1, 2)) & (P[..., 0] > 5).all(1) & (np.abs(P[..., 2]) < 4).all(1)
            ok &= (np.abs(P[..., 3]) < 0.6).all(1)
        parts = dict(x0=d["x0"], kappa=np.concatenate([d["kappa"], kp], 1), ds=np.concatenate([d["ds"], ds_p], 1),
                     ubar=np.concatenate([d["ubar"], u_pm], 1))
        for k, v in parts.items():
            out[k].append(v[ok])
        have += int(ok.sum())
    return {k: np.ascontiguousarray(np.concatenate(v)[:B]) for k, v in out.items()}


# ---- C5: closed-loop Monte-Carlo on a track --------------------------------------------
C5_MPC_DT = 0.045   # N = 40 stages x 0.045 s = the reference's 1.8 s preview (singletrack.yaml: 60 x 0.03 s)


def closed_loop_states(B: int, length: float, seed: int = 31) -> np.ndarray:
    """Initial plant states [B, 8] (dynamic_car.py:209 order) for BASELINE config 5:
    vehicles spread uniformly along the lap, at speeds, yaw rates, steering angles and
    track errors inside the ranges of the reference's recorded runs."""
    rng = np.random.default_rng(seed)
    x = np.zeros((B, 8))
    x[:, 0] = rng.uniform(8, 14, B)          # Ux
    x[:, 1] = rng.uniform(-0.1, 0.1, B)      # Uy
    x[:, 2] = rng.uniform(-0.05, 0.2, B)     # r
    x[:, 3] = rng.uniform(-0.03, 0.1, B)     # delta
    x[:, 4] = rng.uniform(0, length, B)      # s
    x[:, 5] = rng.uniform(-1.5, 1.5, B)      # ey
    x[:, 6] = rng.uniform(-0.1, 0.1, B)      # epsi
    return x
