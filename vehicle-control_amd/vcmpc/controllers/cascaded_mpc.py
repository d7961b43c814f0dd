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
number of sequential-QP iterations in one fused gfx950 kernel -- fp64 with a stagewise
Riccati interior point by default (csrc/st_sqp.hip, N = 20..60), or the condensed fp32
kernel of BASELINE config 3 (csrc/dyn_sqp.hip, N = 40, ``dtype="f32"``); contract:
oracle/dyn_sqp.py.  ``BatchedSingleTrackMPC`` is the same controller for B
vehicles at once.  With ``horizon_pm > 0`` (the cascaded point-mass tail,
cascaded_mpc.py:181-277) ``CascadedMPC`` / ``BatchedCascadedMPC`` run the fp64 cascaded
SQP (csrc/casc_ric.hip, stagewise Riccati; the condensed csrc/casc_sqp.hip with qp.solver = 2; contract oracle/casc_sqp.py); obstacle barrier terms
(`obstacles: True`, cascaded_mpc.py:173-176) enter each QP as in DESIGN.md 2c.
"""
from __future__ import annotations

import numpy as np

from .. import _abi
from ..config import make_params, obstacle_list
from ..solver import Context
from .controller import Controller, neutral_restart

IUX, IS = 0, 4
IFX, IW = 0, 1


# With the obstacle barrier on, one control step takes at least DYN_OBS_SQP SQP iterations (the
# kinematic controller's KIN_OBS_SQP, kinematic_mpc.py here): the barrier's curvature changes
# quickly along the plan, and at the configs' 3-5 iterations the recorded obstacle runs of the
# reference were not driven like IPOPT drives them (r04, tests/test_gpu_bands.py: cascaded
# obstacles2 no lap in 502 steps at 5, lap in 458 vs the recorded 464 at 10; single-track N = 60
# on the shoe track 7 non-solved steps at 5, 3 at 10; scripts/band_settings.py).
DYN_OBS_SQP = 10


def dyn_qp_block(config) -> dict:
    """The dynamic controllers' `qp` block: the config's own, with at least DYN_OBS_SQP SQP
    iterations per step when obstacles are on -- unless the block sets `obs_sqp_iters`, which
    then is the count with obstacles.  A raised count is reported once per process (a silent
    3 -> 10 roughly triples the cost of a step)."""
    qp = dict(config.get("qp") or {})
    if config.get("obstacles"):
        if qp.get("obs_sqp_iters") is not None:
            qp["sqp_iters"] = int(qp["obs_sqp_iters"])
        elif int(qp.get("sqp_iters", 0)) < DYN_OBS_SQP:
            global _OBS_WARNED
            if not _OBS_WARNED:
                import warnings
                warnings.warn(f"obstacles on: qp.sqp_iters {qp.get('sqp_iters')} raised to {DYN_OBS_SQP} per step "
                              f"(DYN_OBS_SQP); set qp.obs_sqp_iters to choose the count", stacklevel=2)
                _OBS_WARNED = True
            qp["sqp_iters"] = DYN_OBS_SQP
    qp.pop("obs_sqp_iters", None)
    return qp


_OBS_WARNED = False


def dyn_horizon_params(s0, ux_pred, mpc_dt, k_of_s):
    """``_init_horizon`` for horizon_pm = 0 (cascaded_mpc.py:323-330), batched.

    s0[B], ux_pred[B, N] (the *unshifted* previous Ux prediction) ->
    ds[B, N] = mpc_dt * ux_pred and kappa[B, N] = k(s0 + cumsum(ds) - ds[:, :1])."""
    ds = mpc_dt * np.asarray(ux_pred, np.float64)
    s_traj = np.cumsum(ds, axis=1) - ds[:, :1] + np.asarray(s0, np.float64)[:, None]
    kappa = np.asarray(k_of_s(s_traj), np.float64).reshape(s_traj.shape)
    return ds, kappa


class BatchedSingleTrackMPC(Controller):
    """B independent single-track NMPCs solved in one launch (N = horizon).

    ``dtype="f64"`` (default, the reference's precision) runs the stagewise-Riccati SQP
    (csrc/st_sqp.hip, N = 20..60, the reference's own horizons included); ``"f32"`` the
    condensed fp32 kernel of BASELINE config 3 (csrc/dyn_sqp.hip, N = 40)."""

    def __init__(self, car, config, batch: int, device: int = 0, seed: int | None = 31, dtype: str = "f64"):
        super().__init__()
        if int(config.get("horizon_pm", 0)) > 0:
            raise ValueError("horizon_pm > 0: use BatchedCascadedMPC (the point-mass tail, cascaded_mpc.py:181-277)")
        if dtype not in ("f64", "f32"):
            raise ValueError(f"dtype must be 'f64' or 'f32', got {dtype!r}")
        self.config = config
        self.car = car
        self.N = int(config["horizon"])
        self.dt = float(config["mpc_dt"])
        self.ns, self.na = len(car.state), len(car.input)
        self.B = int(batch)
        self.np_dtype = np.float64 if dtype == "f64" else np.float32
        vdt = _abi.VC_F64 if dtype == "f64" else _abi.VC_F32
        self.ctx = Context(model=_abi.VC_MODEL_DYNAMIC, N=self.N, max_batch=self.B, dtype=vdt, device=device,
                           params=make_params(dyn_car=car.config, dyn_mpc=dict(config, qp=dyn_qp_block(config)),
                                              tyre=getattr(car, "tyre", "fiala"),
                                              obstacles=obstacle_list(car, config),
                                              obstacle_inside=bool(config.get("obstacle_inside", False))))
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
        re-solved once from the neutral warm start (Fx = 0, w = 0) -- the build's own
        policy: in the reference a failed IPOPT solve raises, the simulator's step()
        returns None (racing.py:416-423) and unpacking it (racing.py:232) ends the run."""
        x0 = np.asarray(states, np.float64).reshape(self.B, self.ns)
        ds, kappa = dyn_horizon_params(x0[:, IS], self.state_prediction[:, IUX, :], self.dt, self.car.track.k)
        cast = lambda a: np.ascontiguousarray(a, dtype=self.np_dtype)
        ubar = cast(np.swapaxes(self.action_prediction, 1, 2))
        ic = self.config["input_constraints"]
        np.clip(ubar[..., IW], ic["w_min"], ic["w_max"], out=ubar[..., IW])
        x0f, kf, dsf = cast(x0), cast(kappa), cast(ds)
        u0, xbar, ustar, status, iters = self.ctx.solve(x0f, kf, dsf, ubar)
        bad = status != 0
        if bad.any():
            # the retry is neutral in its horizon too: ds, kappa from the state prediction x0 at
            # every stage (vc_simulate's restart), not from the previous plan the failed solve used
            idx = np.nonzero(bad)[0]
            ds_n, kap_n = dyn_horizon_params(x0[idx, IS], np.repeat(x0[idx, IUX, None], self.N, axis=1), self.dt,
                                             self.car.track.k)
            r = self.ctx.solve(cast(x0f[idx]), cast(kap_n), cast(ds_n),
                               np.zeros((len(idx), self.N, self.na), self.np_dtype))
            u0[idx], xbar[idx], ustar[idx], status[idx], iters[idx] = r
        self.action_prediction = np.swapaxes(ustar, 1, 2).astype(np.float64)
        self.state_prediction = np.swapaxes(xbar, 1, 2).astype(np.float64)
        u0 = u0.astype(np.float64)
        neutral_restart(status, x0, u0, self.state_prediction, self.action_prediction, None)
        self.status, self.iters = status, iters
        return u0


def casc_horizon_params(s0, ux_pred, mpc_dt, N, M, ds_pm, k_of_s):
    """``_init_horizon`` with a point-mass tail (cascaded_mpc.py:316-338), batched.

    s0[B], ux_pred[B, >= N] (the *unshifted* previous Ux prediction) -> ds[B, H], kappa[B, H]:
    single-track ds = mpc_dt * Ux_pred[:N], curvature at s0 + cumsum(ds) - ds[0]; point mass
    ds = ds_pm, curvature at cumsum(ds_pm) - ds[N-1] + s_traj[N-1] (:331-338)."""
    ds = mpc_dt * np.asarray(ux_pred, np.float64)[:, :N]
    s_traj = np.cumsum(ds, axis=1) - ds[:, :1] + np.asarray(s0, np.float64)[:, None]
    ds_p = np.full((ds.shape[0], M), float(ds_pm))
    s_pm = np.cumsum(ds_p, axis=1) - ds[:, -1:] + s_traj[:, -1:]
    s_all = np.concatenate([s_traj, s_pm], axis=1)
    kappa = np.asarray(k_of_s(s_all), np.float64).reshape(s_all.shape)
    return np.ascontiguousarray(np.concatenate([ds, ds_p], axis=1)), np.ascontiguousarray(kappa)


class BatchedCascadedMPC(Controller):
    """B independent cascaded NMPCs (single track N + point mass M = horizon_pm stages)
    solved in one launch (csrc/casc_ric.hip, fp64; contract oracle/casc_sqp.py)."""

    def __init__(self, car, config, batch: int, device: int = 0, seed: int | None = 31):
        Controller.__init__(self)
        self.config = config
        self.car = car
        self.N = int(config["horizon"])
        self.M = int(config["horizon_pm"])
        self.H = self.N + self.M
        self.dt = float(config["mpc_dt"])
        self.ds_pm = float(config["ds_pm"])
        self.ns, self.na = len(car.state), len(car.input)
        self.B = int(batch)
        self.ctx = Context(model=_abi.VC_MODEL_CASCADED, N=self.N, max_batch=self.B, dtype=_abi.VC_F64,
                           device=device,
                           params=make_params(dyn_car=car.config, dyn_mpc=dict(config, qp=dyn_qp_block(config)),
                                              tyre=getattr(car, "tyre", "fiala"),
                                              obstacles=obstacle_list(car, config),
                                              obstacle_inside=bool(config.get("obstacle_inside", False))))
        # warm starts: cascaded_mpc.py:72-76 (ones over H columns, Ux + 3 on the single-track part)
        rng = np.random.RandomState(seed) if seed is not None else np.random
        self.state_prediction = np.ones((self.B, self.ns, self.H))
        self.state_prediction[:, IUX, :self.N] += 3
        self.action_prediction = np.ones((self.B, self.na, self.H)) + rng.random_sample((self.B, self.na, self.H))
        self.status = np.zeros(self.B, np.int32)
        self.iters = np.zeros(self.B, np.int32)
        self._fresh = np.ones(self.B, bool)  # no solution yet: the tail gets the neutral guess

    def _neutral(self, x0, kappa):
        """Neutral warm start [B, H, 2]: single track Fx = w = 0; point mass Fx = the drag at
        the current speed and Fy = m V^2 kappa (steady cornering along the centre line).
        The condensed SQP rolls the point mass out from its inputs, so the reference's first
        guess 1 + U[0, 1) N (cascaded_mpc.py:74-76; harmless for IPOPT's multiple shooting)
        would turn the 120 m tail off the track in every corner."""
        car = self.car.config
        m, Frr, Cd = float(car["car"]["m"]), float(car["env"]["Frr"]), float(car["env"]["Cd"])
        V = np.maximum(np.hypot(x0[:, 0], x0[:, 1]), 3.0)[:, None]
        u = np.zeros((x0.shape[0], self.H, self.na))
        u[:, self.N:, 0] = Frr + Cd * V ** 2
        u[:, self.N:, 1] = m * V ** 2 * kappa[:, self.N:]
        return u

    def command(self, states):
        """states[B, 8] -> actions[B, 2] (Fx, w of the first stage).

        Warm start: the previous (8, H) / (2, H) predictions, unshifted
        (cascaded_mpc.py:320-321), w projected onto its box, the point-mass tail of a
        vehicle without a previous solution from :meth:`_neutral`; a problem that does not
        come back VC_SOLVED is re-solved once from the neutral warm start."""
        x0 = np.ascontiguousarray(np.asarray(states, np.float64).reshape(self.B, self.ns))
        ds, kappa = casc_horizon_params(x0[:, IS], self.state_prediction[:, IUX, :], self.dt, self.N, self.M,
                                        self.ds_pm, self.car.track.k)
        ubar = np.ascontiguousarray(np.swapaxes(self.action_prediction, 1, 2), dtype=np.float64)
        if self._fresh.any():
            ubar[self._fresh, self.N:] = self._neutral(x0, kappa)[self._fresh, self.N:]
        ic = self.config["input_constraints"]
        np.clip(ubar[:, :self.N, IW], ic["w_min"], ic["w_max"], out=ubar[:, :self.N, IW])
        u0, xbar, ustar, status, iters = self.ctx.solve(x0, kappa, ds, ubar)
        bad = status != 0
        if bad.any():
            idx = np.nonzero(bad)[0]
            ux_n = np.repeat(x0[idx, IUX, None], self.H, axis=1)   # neutral horizon (see BatchedSingleTrackMPC)
            ds_n, kap_n = casc_horizon_params(x0[idx, IS], ux_n, self.dt, self.N, self.M, self.ds_pm,
                                              self.car.track.k)
            r = self.ctx.solve(np.ascontiguousarray(x0[idx]), kap_n, ds_n,
                               np.ascontiguousarray(self._neutral(x0[idx], kap_n)))
            u0[idx], xbar[idx], ustar[idx], status[idx], iters[idx] = r
            kappa[idx] = kap_n
        self._fresh = status != 0
        self.action_prediction = np.swapaxes(ustar, 1, 2).copy()
        self.state_prediction = np.swapaxes(xbar, 1, 2).copy()
        neutral_restart(status, x0, u0, self.state_prediction, self.action_prediction,
                         lambda rows: np.swapaxes(self._neutral(x0[rows], kappa[rows]), 1, 2), self.N)
        self.status, self.iters = status, iters
        return u0


class CascadedMPC(BatchedSingleTrackMPC):
    """Single-vehicle drop-in for ``CascadedMPC(car, point_mass, config)`` (cascaded_mpc.py:16-39).
    ``horizon_pm: 0`` runs the single-track SQP (fp64 csrc/st_sqp.hip by default, fp32
    csrc/dyn_sqp.hip with ``dtype="f32"``); ``horizon_pm > 0``
    returns a :class:`CascadedTailMPC` (point-mass tail, csrc/casc_ric.hip, fp64)."""

    def __new__(cls, car, point_mass, config, device: int = 0, dtype: str = "f64"):
        if cls is CascadedMPC and int(config.get("horizon_pm", 0) or 0) > 0:
            return object.__new__(CascadedTailMPC)
        return object.__new__(cls)

    def __init__(self, car, point_mass, config, device: int = 0, dtype: str = "f64"):
        self.point_mass = point_mass
        super().__init__(car, config, batch=1, device=device, seed=None, dtype=dtype)
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


class CascadedTailMPC(BatchedCascadedMPC, CascadedMPC):
    """``CascadedMPC(car, point_mass, config)`` with ``horizon_pm > 0`` (the reference's
    cascaded controller, config/controllers/cascaded.yaml) for one vehicle."""

    def __init__(self, car, point_mass, config, device: int = 0, dtype: str = "f64"):
        self.point_mass = point_mass
        BatchedCascadedMPC.__init__(self, car, config, batch=1, device=device, seed=None)
        self.state_prediction = self.state_prediction[0]
        self.action_prediction = np.ones((self.na, self.H)) + np.random.random((self.na, self.H))

    def command(self, state):
        sp, ap = self.state_prediction, self.action_prediction
        self.state_prediction, self.action_prediction = sp[None], ap[None]
        try:
            u0 = BatchedCascadedMPC.command(self, state.values.reshape(1, -1))
        except Exception:
            self.state_prediction, self.action_prediction = sp, ap
            raise
        self.state_prediction = self.state_prediction[0]
        self.action_prediction = self.action_prediction[0]
        return self.car.create_action(*u0[0])

    def get_state_prediction(self):
        """cascaded_mpc.py:340-352: the car's N predicted states and the point mass's M,
        as global (x, y, psi) (point-mass columns hold V, s, ey, epsi, t in rows 0..4)."""
        sp = self.state_prediction
        car = [self.car.rel2glob(sp[:, i]) for i in range(self.N)]
        tr = self.car.track
        pm = [tr.rel2glob(sp[1, j], sp[2, j], sp[3, j]) for j in range(self.N, self.H)]
        return np.array(car + pm, dtype=np.float64).squeeze()
