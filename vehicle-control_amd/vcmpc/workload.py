"""Synthetic batched workloads of BASELINE.json's configs.

C2/C4 (kinematic LTV-MPC, N = 20, fp64), seeded ``numpy.random.default_rng``:
  x0:    v ~ U(3, 10), delta ~ U(-0.15, 0.15), s ~ U(0, 315.5), ey ~ U(-2, 2),
         epsi ~ U(-0.2, 0.2), t = 0
  kappa: piecewise constant over 4 segments, each ~ U(0, 0.047) (ippodromo's
         range of back-solved curvature)
  ds:    mpc_dt * v0 + 0.5 for every stage (kinematic_mpc.py:178-182 with a
         constant speed prediction)
  ubar:  U(-1, 1) * (3, 0.4) (the input boxes of kinematic.yaml)
Problems whose warm-start rollout would leave the model's domain (v below 1 m/s,
|epsi| above 1.2 rad, where v cos(epsi) -> 0 makes the spatial ODE singular) are
re-drawn, so every generated problem is well posed.
"""
from __future__ import annotations

import numpy as np

V_LO = 1.0
EPSI_HI = 1.2


def _kin_rollout(x0, ubar, kappa, ds, L):
    """Host-side Euler rollout used only to screen samples (kinematic_car.py:47-64)."""
    B, N = kappa.shape
    x = x0.copy()
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
        vmin = np.minimum(vmin, x[:, 0])
        emax = np.maximum(emax, np.abs(x[:, 4]))
    ok = np.isfinite(x).all(1) & (vmin > V_LO) & (emax < EPSI_HI)
    return ok


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
        ds = np.repeat(mpc_dt * x0[:, :1] + 0.5, N, axis=1)
        ubar = rng.uniform(-1, 1, (m, N, 2)) * np.array([a_max, w_max])
        ok = _kin_rollout(x0, ubar, kappa, ds, L)
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
