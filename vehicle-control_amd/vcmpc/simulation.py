"""Batched closed-loop racing simulator on the device (BASELINE config 5).

The reference's ``RacingSimulator`` (simulation/racing.py:217-242, :416-423) steps
each car in a Python loop: ``controller.command(car.state)`` (IPOPT), then
``car.drive(action)`` (a CasADi plant call with ``track.k(s)``), then logs the
state and action.  ``BatchedRacingSimulator`` runs the same loop for B vehicles
with every step on the GPU (``vc_simulate``): horizon parameters from the
unshifted warm start and the curvature table, the fused MPC solve, the fp64
plant step -- no host round trip between steps.

Per-vehicle failure handling is the build's own policy.  In the reference a failed IPOPT
solve raises, the simulator's step() prints it and returns None (racing.py:416-423), and the
caller's unpacking ``action, state = self.step(...)`` (racing.py:232) raises TypeError, which
ends the run.  Here a solve whose status is not VC_SOLVED applies the neutral
input u = 0, is counted in ``nfail``, and the next step starts from the neutral
warm start (ubar = 0).  Almost every such step is the first one, whose linearised QP
around the reference's random first guess 1 + U[0, 1) is infeasible under the
real-time-iteration trust region (scripts/kin_fail_modes.py: 67 of 69).  The single-vehicle controllers instead re-solve at once from
the neutral warm start (controllers/*.py); both are documented deviations.
"""
from __future__ import annotations

import numpy as np

from . import _abi
from .config import make_params, obstacle_list
from .solver import Context

IV_KIN, IS_KIN = 0, 2
IUX, IS_DYN = 0, 4
ST_SQP_HORIZONS = (20, 30, 40, 50, 60)   # fp64 single-track kernel instances (csrc/st_sqp.hip)


def _is_dynamic(car) -> bool:
    return getattr(car, "MODEL", _abi.VC_MODEL_KINEMATIC) == _abi.VC_MODEL_DYNAMIC


class BatchedRacingSimulator:
    """B vehicles of one model on one track, one controller config, one GPU.

    ``car`` is a ``KinematicCar`` or ``DynamicCar`` (its config and tyre are used),
    ``controller_config`` the matching controller yaml (``kinematic_mpc`` /
    ``dynamic_mpc`` / ``singletrack_mpc`` / ``cascaded_mpc``: a ``horizon_pm > 0`` config runs
    the cascaded NMPC with its point-mass tail), ``track`` a ``vcmpc.environment.Track``.  ``dtype`` picks the
    dynamic solve precision (default fp64 where the fp64 kernel is built for N).  Buffers live on
    ``cuda:<device>`` as torch tensors when torch is importable (the fast path),
    else in host numpy arrays staged by every call."""

    def __init__(self, car, controller_config, track, batch: int, device: int = 0, seed: int | None = 31,
                 use_torch: bool = True, dtype: int | None = None):
        cfg = controller_config
        self.car, self.config, self.track = car, cfg, track
        self.dynamic = _is_dynamic(car)
        self.B, self.N = int(batch), int(cfg["horizon"])
        # the cascaded controller's point-mass tail (cascaded_mpc.py:181-338): arrays over H stages
        self.M = int(cfg.get("horizon_pm", 0) or 0) if self.dynamic else 0
        self.H = self.N + self.M
        self.mpc_dt = float(cfg["mpc_dt"])
        self.dt = float(car.dt)
        if self.dynamic:
            from .controllers.cascaded_mpc import dyn_qp_block  # obstacles: DYN_OBS_SQP iterations
            params = make_params(dyn_car=car.config, dyn_mpc=dict(cfg, qp=dyn_qp_block(cfg)),
                                 tyre=getattr(car, "tyre", "fiala"), obstacles=obstacle_list(track, cfg),
                                 obstacle_inside=bool(cfg.get("obstacle_inside", False)))
            if self.M > 0:  # cascaded SQP, fp64 (csrc/casc_ric.hip)
                model, dtype = _abi.VC_MODEL_CASCADED, _abi.VC_F64
            else:
                # fp64 (csrc/st_sqp.hip, the reference's own precision) where it is built, else
                # the fp32 condensed kernel (csrc/dyn_sqp.hip, N = 40)
                model = _abi.VC_MODEL_DYNAMIC
                if dtype is None:
                    dtype = _abi.VC_F64 if self.N in ST_SQP_HORIZONS else _abi.VC_F32
        else:
            # the kinematic controller's real-time-iteration trust region and, with obstacles,
            # its globalised SQP step (controllers/kinematic_mpc.py kin_qp_block) unless the
            # config's qp block sets its own
            from .controllers.kinematic_mpc import kin_qp_block
            kcfg = dict(cfg)
            kcfg["qp"] = kin_qp_block(cfg)
            params = make_params(kin_car=car.config, kin_mpc=kcfg, obstacles=obstacle_list(track, cfg))
            model, dtype = _abi.VC_MODEL_KINEMATIC, _abi.VC_F64
        self.ctx = Context(model=model, N=self.N, max_batch=self.B, dtype=dtype, device=device, params=params)
        self.ctx.set_track(track)
        self.nx, self.ns = self.ctx.nx, self.ctx.ns_solve
        self.np_dtype = np.float32 if dtype == _abi.VC_F32 else np.float64
        self.torch = None
        if use_torch:
            try:
                import torch
                if torch.cuda.is_available():
                    self.torch = torch
            except ImportError:
                pass
        if self.torch is not None:  # one stream for torch's copies and the vc_* kernels
            self.ctx.set_stream(self.torch.cuda.current_stream(device).cuda_stream)
        self._init_warm_start(seed)
        self.x = None
        self.nfail = self._to_dev(np.zeros(self.B, np.int32))

    # -- buffers ----------------------------------------------------------------------
    def _to_dev(self, a):
        a = np.ascontiguousarray(a)
        if self.torch is None:
            return a.copy()
        return self.torch.from_numpy(a).to(f"cuda:{self.ctx.device}")

    @staticmethod
    def _to_host(a):
        return a.detach().cpu().numpy() if hasattr(a, "detach") else np.array(a)

    def _init_warm_start(self, seed):
        """The controllers' initial predictions: kinematic_mpc.py:64-68 (zeros, v = 0.1)
        and cascaded_mpc.py:72-76 (ones, Ux + 3); actions: the dynamic controller's
        1 + U[0, 1) projected onto the input box (controllers/*.py), the kinematic
        controller's neutral guess (see below)."""
        rng = np.random.RandomState(seed) if seed is not None else np.random
        B, N, H, ns, nx = self.B, self.N, self.H, self.ns, self.nx
        ic = self.config["input_constraints"]
        if self.dynamic:
            xbar = np.ones((B, ns, nx))
            xbar[:, :N, IUX] += 3
        else:
            xbar = np.zeros((B, ns, nx))
            xbar[..., IV_KIN] += 0.1
        ubar = np.ones((B, H, 2)) + np.swapaxes(rng.random_sample((B, 2, H)), 1, 2)
        if self.dynamic:
            np.clip(ubar[:, :N, 1], ic["w_min"], ic["w_max"], out=ubar[:, :N, 1])
            self._fresh_tail = self.M > 0  # the point-mass tail gets the neutral guess at reset()
        else:
            # the neutral guess (a = w = 0, the restart value of a failed step): the reference's
            # 1 + U[0, 1) (kinematic_mpc.py:64-68) puts w at its bound on every stage, so the
            # predicted steering leaves the delta box and the trust-region QP of the first step
            # is infeasible for every vehicle (IPOPT has no trust region and recovers)
            ubar[:] = 0.0
        self.xbar = self._to_dev(xbar.astype(self.np_dtype))
        self.ubar = self._to_dev(ubar.astype(self.np_dtype))

    def reset(self, states):
        """Set the B plant states (fp64 [B, nx], reference FancyVector order).  A cascaded
        controller's point-mass tail starts from the neutral guess of
        controllers/cascaded_mpc.py (BatchedCascadedMPC._neutral: drag-level Fx, Fy = m V^2
        kappa), as the host controller does -- the reference's random first guess would roll
        the tail off the track in every corner."""
        states = np.asarray(states, np.float64).reshape(self.B, self.nx)
        self.x = self._to_dev(states)
        if getattr(self, "_fresh_tail", False):
            from .controllers.cascaded_mpc import casc_horizon_params
            xb = self._to_host(self.xbar)
            ds, kappa = casc_horizon_params(states[:, IS_DYN], xb[:, :, IUX], self.mpc_dt, self.N, self.M,
                                            float(self.config["ds_pm"]), self.track.k)
            car = self.car.config
            m, Frr, Cd = float(car["car"]["m"]), float(car["env"]["Frr"]), float(car["env"]["Cd"])
            V = np.maximum(np.hypot(states[:, 0], states[:, 1]), 3.0)[:, None]
            ub = self._to_host(self.ubar).copy()
            ub[:, self.N:, 0] = Frr + Cd * V ** 2
            ub[:, self.N:, 1] = m * V ** 2 * kappa[:, self.N:]
            self.ubar = self._to_dev(ub.astype(self.np_dtype))
            self._fresh_tail = False
        return self

    # -- loop ---------------------------------------------------------------------------
    def run(self, steps: int, log: bool = True):
        """``steps`` closed-loop steps of every vehicle.  Returns a dict with
        ``state_traj`` [steps+1, B, nx] (fp64) and ``action_traj`` [steps, B, nu]
        (host numpy, when ``log``) and ``nfail`` [B] (cumulative)."""
        if self.x is None:
            raise RuntimeError("reset(states) first")
        log_x, log_u, nf = self.ctx.simulate(self.x, self.xbar, self.ubar, steps, self.mpc_dt, self.dt, log=log,
                                             nfail=self.nfail)
        self.ctx.synchronize()
        out = {"nfail": self._to_host(nf)}
        if log:
            out["state_traj"] = self._to_host(log_x)
            out["action_traj"] = self._to_host(log_u)
        return out

    @property
    def states(self):
        return self._to_host(self.x)

    @property
    def state_prediction(self):
        """(B, nx, NS) like the controllers' ``state_prediction``."""
        return np.swapaxes(self._to_host(self.xbar), 1, 2)

    @property
    def action_prediction(self):
        return np.swapaxes(self._to_host(self.ubar), 1, 2)
