"""Kinematic-bicycle MPC on the GPU -- drop-in for controllers/mpc/kinematic_mpc.py.

``KinematicMPC(car, config).command(state) -> KinematicCarAction`` keeps the
reference's surface (kinematic_mpc.py:14-193): the same config schema, the same
``state_prediction`` (ns, N+1) / ``action_prediction`` (na, N) warm-start
attributes with the same initial values (kinematic_mpc.py:64-68, seed 31 at
:11), the same horizon-parameter construction ``_init_horizon``
(kinematic_mpc.py:170-187, quirks included) and ``get_state_prediction``.

What changes is the solve (kinematic_mpc.py:162, IPOPT + HSL MA27 on the NLP):
one LTV-QP step (predict -> linearize -> condense -> interior point) in one
fused gfx950 kernel (csrc/kin_ltv.hip).  ``BatchedKinematicMPC`` is the same
controller for B vehicles at once -- the data-parallel hot path.
"""
from __future__ import annotations

import numpy as np

from .. import _abi
from ..config import make_params, obstacle_list
from ..solver import Context
from .controller import Controller, neutral_restart

IV, IS = 0, 2
# Real-time-iteration globalisation of the closed-loop controller: a trust region
# on the per-step input change (vc_qp.trust_a / trust_w).  The reference solves
# each NLP to convergence with IPOPT's line search; one LTV-QP step per control
# step linearised around a far-off warm start can otherwise overshoot into a
# region where the linearisation is meaningless (cos(epsi) -> 0).
RTI_TRUST = {"trust_a": 1.0, "trust_w": 0.1}
# With the obstacle barrier (``obstacles: True``, kinematic_mpc.py:130-133) one convexified
# QP per control step is not enough: the controller takes KIN_OBS_SQP SQP steps, each with a
# merit line search on the exact NLP cost (vc_qp.kin_sqp, csrc/kin_merit.hip, oracle/kin_sqp.py;
# 0 of 64 vehicles touch an obstacle on ippodromo with 10 steps).
KIN_OBS_SQP = 10


# Shifted warm start from this horizon on (vc_qp.shift): the reference keeps the previous
# prediction unshifted (kinematic_mpc.py:170-187), harmless for IPOPT's multiple shooting; the
# build's single-shooting step re-rolls the warm-start inputs from the new state, and over a
# 40 m horizon the one-step lag makes that rollout cross the spatial model's eps = +-pi/2
# singularity (N = 50: 52 of 64 vehicles off track unshifted, 0 shifted; scripts/kin_shift_test.py).
KIN_SHIFT_FROM_N = 30


# With obstacles the SQP runs in multiple shooting (vc_qp.ms): the previous plan's states are the
# state iterate, so a swerving plan is never re-rolled from the new state through eps = +-pi/2
# (ippodromo, 64 vehicles x 400 steps, 10 SQP steps: N = 50 single shooting 2 hit / 16 off
# track / 5.3 % non-solved, multiple shooting 0 / 10 (soft boundary, <= 1.7 m) / 0.11 %;
# N = 30 2 / 1 / 0.7 % vs 0 / 0 / 0.02 %; N = 20 0 / 0 / 0.04 % vs 0 / 0 / 0.03 %).
KIN_OBS_MS = 1

# A first QP without a solution (infeasible with the hard v / delta rows, or linearised where the
# spatial model is near-singular) restarts the step's iterate from the neutral guess and the
# remaining SQP iterations solve from there (kin_merit.hip, oracle/kin_sqp.py), instead of ending
# the control step non-solved.  Elastic rows (vc_qp.elastic: a slack per row at the merit's own
# L1 price, always or only on failure) make every QP solvable but were measured worse in closed
# loop at N >= 30 (64 vehicles x 400 steps x 4 seeds, hard + restart / elastic on failure +
# restart: N = 20 0 / 0 off track, 0 / 0 non-solved; N = 30 0 / 6 off, 14 / 319 non-solved,
# max |ey| 3.6 / 43 m; N = 50 36 / 40 off, 813 / 763 non-solved, 0 / 5 obstacle hits; DESIGN.md
# 2c), so the controller keeps hard rows; elastic stays available through the qp block.
KIN_OBS_ELASTIC = 0.0
# The obstacle QPs need more interior-point iterations than the C2 cap of 40: a plan that runs
# through an obstacle (e.g. the neutral restart's constant-ey plan) meets the barrier's floored
# margin, curvatures ~1e6 and condition numbers ~4e10 (44 iterations for the oracle on
# gpurun_out/kin_lost seed 3 vehicle 1, where the 40-iteration kernel reported max-iter), and elastic
# rows about twice the plain count (the multipliers start on rho = la + le): with obstacles on the
# cap is raised to 80 (the easy QPs stop at their own tolerance long before).
KIN_OBS_MAX_ITER = 80


def kin_qp_block(config) -> dict:
    """The kinematic controller's `qp` block: RTI_TRUST, the globalised multiple-shooting step
    when obstacles are on, the shifted warm start at long horizons, then the config's own `qp`
    entries."""
    qp = dict(RTI_TRUST)
    if config.get("obstacles"):
        qp["kin_sqp"] = KIN_OBS_SQP
        qp["ms"] = KIN_OBS_MS
        if KIN_OBS_ELASTIC:
            qp["elastic"] = KIN_OBS_ELASTIC
    if int(config["horizon"]) >= KIN_SHIFT_FROM_N:
        qp["shift"] = 1
    qp.update(config.get("qp") or {})
    if config.get("obstacles") or qp.get("elastic", 0.0) != 0.0:
        qp["max_iter"] = max(int(qp.get("max_iter", 0)), KIN_OBS_MAX_ITER)
    return qp


def horizon_params(s0, v_pred, mpc_dt, k_of_s):
    """``_init_horizon`` parameter construction (kinematic_mpc.py:177-187), batched.

    s0[B], v_pred[B, N+1] (the *unshifted* previous speed prediction) ->
    ds[B, N] = mpc_dt * v_pred[:, :N] + 0.5 and kappa[B, N] = k(s) at
    s = s0 + cumsum(ds_traj with ds_traj[0] = 0)[:N] (the reference's off-by-one)."""
    ds_traj = mpc_dt * np.asarray(v_pred, np.float64) + 0.5
    ds = ds_traj[:, :-1].copy()
    ds_traj[:, 0] = 0.0
    s_traj = (np.cumsum(ds_traj, axis=1) + np.asarray(s0, np.float64)[:, None])[:, :-1]
    kappa = np.ascontiguousarray(np.asarray(k_of_s(s_traj), np.float64).reshape(s_traj.shape))
    return ds, kappa


class BatchedKinematicMPC(Controller):
    """B independent kinematic MPCs solved in one launch."""

    def __init__(self, car, config, batch: int, device: int = 0, seed: int | None = 31):
        super().__init__()
        self.config = config
        self.car = car
        self.N = int(config["horizon"])
        self.dt = float(config["mpc_dt"])
        self.ns, self.na = len(car.state), len(car.input)
        self.B = int(batch)
        cfg = dict(config)
        cfg["qp"] = kin_qp_block(config)
        self.shift = bool(cfg["qp"].get("shift", 0))
        self.ms = bool(cfg["qp"].get("ms", 0))
        self.ctx = Context(model=_abi.VC_MODEL_KINEMATIC, N=self.N, max_batch=self.B, dtype=_abi.VC_F64,
                           device=device, params=make_params(kin_car=car.config, kin_mpc=cfg,
                                                             obstacles=obstacle_list(car, config)))
        # warm starts: kinematic_mpc.py:64-68 (zeros, v = 0.1; actions 1 + U[0,1) seeded)
        rng = np.random.RandomState(seed) if seed is not None else np.random
        self.state_prediction = np.zeros((self.B, self.ns, self.N + 1))
        self.state_prediction[:, IV, :] += 0.1
        self.action_prediction = np.ones((self.B, self.na, self.N)) + rng.random_sample((self.B, self.na, self.N))
        self.status = np.zeros(self.B, np.int32)
        self.iters = np.zeros(self.B, np.int32)

    def command(self, states):
        """states[B, ns] -> actions[B, na] (u*_0 of every problem).

        The warm start is the previous solution, unshifted, as in the reference
        (kinematic_mpc.py:175-176) -- shifted one stage at horizons >= KIN_SHIFT_FROM_N
        (vc_qp.shift) -- projected onto the input box first: the LTV-QP
        linearises around the warm-start rollout, and the reference's initial guess
        1 + U[0, 1) (kinematic_mpc.py:65-67) is far outside w_max = 0.4 (IPOPT
        recovers from that by globalisation; one QP step cannot).  A problem that
        does not come back VC_SOLVED (e.g. linearised state rows infeasible) keeps
        the neutral retry's output as prediction (unshifted) and applies its first
        action.  Both are the build's own policy (vc_simulate differs: it applies
        u = 0 and restarts from the neutral warm start); in the reference a failed
        IPOPT solve raises, the simulator's step() prints it and returns None
        (racing.py:416-423), and unpacking that (racing.py:232) ends the run."""
        x0 = np.ascontiguousarray(np.asarray(states, np.float64).reshape(self.B, self.ns))
        ds, kappa = horizon_params(x0[:, IS], self.state_prediction[:, IV, :], self.dt, self.car.track.k)
        ubar = np.ascontiguousarray(np.swapaxes(self.action_prediction, 1, 2))
        ic = self.config["input_constraints"]
        np.clip(ubar[..., 0], ic["a_min"], ic["a_max"], out=ubar[..., 0])
        np.clip(ubar[..., 1], ic["w_min"], ic["w_max"], out=ubar[..., 1])
        # multiple shooting (vc_qp.ms): the previous plan's states are the state iterate
        xs = np.ascontiguousarray(np.swapaxes(self.state_prediction, 1, 2)) if self.ms else None
        u0, xbar, ustar, status, iters = self.ctx.solve(x0, kappa, ds, ubar, xbar=xs)
        bad = status != 0
        if bad.any():
            # retry from the neutral warm start u = 0 (steering held, speed held):
            # its linearised state rows are feasible at dz = 0 whenever x0 is
            idx = np.nonzero(bad)[0]
            xr = np.ascontiguousarray(np.repeat(x0[idx, None, :], self.N + 1, axis=1)) if self.ms else None
            r = self.ctx.solve(x0[idx], kappa[idx], ds[idx], np.zeros((len(idx), self.N, self.na)), xbar=xr)
            u0[idx], xbar[idx], ustar[idx], status[idx], iters[idx] = r
        self.action_prediction = np.swapaxes(ustar, 1, 2).copy()
        self.state_prediction = np.swapaxes(xbar, 1, 2).copy()
        # a retry without a finite plan restarts from the neutral warm start (u = 0, the state at
        # every stage), as vc_simulate does: a non-finite plan must not become the next ds
        nonfin = (status == _abi.VC_NONFINITE) | ~np.isfinite(ustar).all(axis=(1, 2)) | ~np.isfinite(xbar).all(axis=(1, 2))
        neutral_restart(nonfin, x0, u0, self.state_prediction, self.action_prediction, None)
        if self.shift:  # vc_qp.shift, as vc_simulate does: a solved vehicle's next warm start one stage on
            ok = status == 0
            self.action_prediction[ok, :, :-1] = self.action_prediction[ok, :, 1:].copy()
            self.state_prediction[ok, :, :-1] = self.state_prediction[ok, :, 1:].copy()
        self.status, self.iters = status, iters
        return u0


class KinematicMPC(BatchedKinematicMPC):
    """Single-vehicle drop-in for ``KinematicMPC(car, config)`` (kinematic_mpc.py:14)."""

    def __init__(self, car, config, device: int = 0):
        super().__init__(car, config, batch=1, device=device, seed=None)
        # kinematic_mpc.py:65-67 draws from the global numpy RNG seeded at import
        self.state_prediction = self.state_prediction[0]
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
        """Global (x, y, psi) of the first N predicted states -- kinematic_mpc.py:189-193."""
        preds = [self.car.rel2glob(self.state_prediction[:, i]) for i in range(self.N)]
        return np.array(preds).squeeze()
