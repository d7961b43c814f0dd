"""Dynamic-bicycle (single-track) MPC on the GPU -- drop-in for
controllers/mpc/cascaded_mpc.py in single-track mode (``horizon_pm: 0``).

``CascadedMPC(car, point_mass, config).command(state) -> DynamicCarAction`` keeps the
reference's surface (cascaded_mpc.py:16-352): the same config schema
(config/controllers/singletrack.yaml), the same ``state_prediction`` (ns, N) /
``action_prediction`` (na, N) warm-start attributes with the reference's initial values
(cascaded_mpc.py:72-76: ones, Ux + 3, actions 1 + U[0, 1) from the numpy RNG seeded 31
at import, :13), the same horizon-parameter construction ``_init_horizon``
(cascaded_mpc.py:316-330: ds = mpc_dt * Ux_pred, curvature at s0 + cumsum(ds) - ds[0])
and ``get_state_prediction`` (:340-352).

What changes is the solve (cascaded_mpc.py:308, IPOPT + HSL MA27 on the NLP): a fixed
number of sequential-QP iterations in one fused fp32 gfx950 kernel (csrc/dyn_sqp.hip;
contract: oracle/dyn_sqp.py).  ``BatchedSingleTrackMPC`` is the same controller for B
vehicles at once.  The cascaded point-mass tail (``horizon_pm > 0``,
cascaded_mpc.py:181-277) is SURVEY 8(f) row 3 and raises; obstacle barrier terms
(`obstacles: True`, cascaded_mpc.py:173-176) enter each QP as in DESIGN.md 2c.
"""
from __future__ import annotations

import numpy as np

from .. import _abi
from ..config import make_params, obstacle_list
from ..solver import Context
from .controller import Controller

IUX, IS = 0, 4
IFX, IW = 0, 1


def dyn_horizon_params(s0, ux_pred, mpc_dt, k_of_s):
    """``_init_horizon`` for horizon_pm = 0 (cascaded_mpc.py:323-330), batched.

    s0[B], ux_pred[B, N] (the *unshifted* previous Ux prediction) ->
    ds[B, N] = mpc_dt * ux_pred and kappa[B, N] = k(s0 + cumsum(ds) - ds[:, :1])."""
    ds = mpc_dt * np.asarray(ux_pred, np.float64)
    s_traj = np.cumsum(ds, axis=1) - ds[:, :1] + np.asarray(s0, np.float64)[:, None]
    kappa = np.asarray(k_of_s(s_traj), np.float64).reshape(s_traj.shape)
    return ds, kappa


class BatchedSingleTrackMPC(Controller):
    """B independent single-track NMPCs solved in one launch (fp32, N = horizon)."""

    def __init__(self, car, config, batch: int, device: int = 0, seed: int | None = 31):
        super().__init__()
        if int(config.get("horizon_pm", 0)) > 0:
            raise NotImplementedError("the cascaded point-mass tail (cascaded_mpc.py:181-277) is SURVEY 8(f) row 3")
        self.config = config
        self.car = car
        self.N = int(config["horizon"])
        self.dt = float(config["mpc_dt"])
        self.ns, self.na = len(car.state), len(car.input)
        self.B = int(batch)
        self.ctx = Context(model=_abi.VC_MODEL_DYNAMIC, N=self.N, max_batch=self.B, dtype=_abi.VC_F32, device=device,
                           params=make_params(dyn_car=car.config, dyn_mpc=config, tyre=getattr(car, "tyre", "fiala"),
                                              obstacles=obstacle_list(car, config)))
        # warm starts: cascaded_mpc.py:72-76
        rng = np.random.RandomState(seed) if seed is not None else np.random
        self.state_prediction = np.ones((self.B, self.ns, self.N))
        self.state_prediction[:, IUX, :] += 3
        self.action_prediction = np.ones((self.B, self.na, self.N)) + rng.random_sample((self.B, self.na, self.N))
        self.status = np.zeros(self.B, np.int32)
        self.iters = np.zeros(self.B, np.int32)

    def command(self, states):
        """states[B, ns] -> actions[B, na] (u*_0 of every problem).

        The warm start is the previous solution, unshifted (cascaded_mpc.py:320-321),
        with w projected onto its box (the reference's first guess 1 + U[0, 1) exceeds
        w_max = 0.4; IPOPT recovers by globalisation, the SQP's trust region would only
        take it back 0.2 per iteration).  A problem that does not come back VC_SOLVED is
        re-solved once from the neutral warm start (Fx = 0, w = 0) -- the reference's
        simulator instead swallows the solver exception (racing.py:416-423)."""
        x0 = np.asarray(states, np.float64).reshape(self.B, self.ns)
        ds, kappa = dyn_horizon_params(x0[:, IS], self.state_prediction[:, IUX, :], self.dt, self.car.track.k)
        ubar = np.ascontiguousarray(np.swapaxes(self.action_prediction, 1, 2), dtype=np.float32)
        ic = self.config["input_constraints"]
        np.clip(ubar[..., IW], ic["w_min"], ic["w_max"], out=ubar[..., IW])
        f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32)
        x0f, kf, dsf = f32(x0), f32(kappa), f32(ds)
        u0, xbar, ustar, status, iters = self.ctx.solve(x0f, kf, dsf, ubar)
        bad = status != 0
        if bad.any():
            idx = np.nonzero(bad)[0]
            r = self.ctx.solve(f32(x0f[idx]), f32(kf[idx]), f32(dsf[idx]), np.zeros((len(idx), self.N, self.na), np.float32))
            u0[idx], xbar[idx], ustar[idx], status[idx], iters[idx] = r
        self.action_prediction = np.swapaxes(ustar, 1, 2).astype(np.float64)
        self.state_prediction = np.swapaxes(xbar, 1, 2).astype(np.float64)
        self.status, self.iters = status, iters
        return u0.astype(np.float64)


class CascadedMPC(BatchedSingleTrackMPC):
    """Single-vehicle drop-in for ``CascadedMPC(car, point_mass, config)`` (cascaded_mpc.py:16-39)
    with ``horizon_pm: 0``."""

    def __init__(self, car, point_mass, config, device: int = 0):
        self.point_mass = point_mass
        super().__init__(car, config, batch=1, device=device, seed=None)
        self.state_prediction = self.state_prediction[0]
        # cascaded_mpc.py:74-76 draws from the global numpy RNG seeded at import
        self.action_prediction = np.ones((self.na, self.N)) + np.random.random((self.na, self.N))

    def command(self, state):
        sp, ap = self.state_prediction, self.action_prediction
        self.state_prediction, self.action_prediction = sp[None], ap[None]
        try:
            u0 = super().command(state.values.reshape(1, -1))
        except Exception:
            self.state_prediction, self.action_prediction = sp, ap
            raise
        self.state_prediction = self.state_prediction[0]
        self.action_prediction = self.action_prediction[0]
        return self.car.create_action(*u0[0])

    def get_state_prediction(self):
        """Global (x, y, psi) of the N predicted states -- cascaded_mpc.py:340-352 (M = 0)."""
        return np.array([self.car.rel2glob(self.state_prediction[:, i]) for i in range(self.N)]).squeeze()
