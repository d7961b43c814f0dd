"""Track-relative car base -- mirrors models/racing_car.py:15-52.

``transition(x, u, kappa, dt)`` and ``spatial_transition(x, u, kappa, ds)`` keep
the reference's CasADi-Function call signature but evaluate on the GPU through
``vc_plant_step`` / ``vc_spatial_step``; they accept one problem (``x[nx]``) or a
batch (``x[B, nx]``, ``kappa[B]``) and return numpy arrays of the same shape.
``f(x, u, curvature)`` is the north star's ``VehicleModel.f(x, u)``: the continuous temporal
vector field the reference's integrators wrap (``f = ca.Function("f", [state, action,
curvature], [f])``, utils/integrators.py:18,29; kinematic_car.py:34-40, dynamic_car.py:153-167),
evaluated by ``vc_ode``; ``f_spatial`` is the spatial one (kinematic_car.py:47-60,
dynamic_car.py:169-191), so ``spatial_transition(x, u, k, ds) == x + ds * f_spatial(x, u, k)``
for the (Euler) kinematic car.
"""
from __future__ import annotations

from abc import abstractmethod

import numpy as np

from .. import _abi
from ..solver import Context
from .robot import Robot

_MODEL_CTX_BATCH = 1 << 20


class RacingCar(Robot):
    MODEL = _abi.VC_MODEL_KINEMATIC

    def __init__(self, config, track):
        self.length = config["car"]["l"]
        self.track = track
        super().__init__(config)

    def _init_model(self):
        self._ctx = None

    def _context(self) -> Context:
        if self._ctx is None:
            self._ctx = Context(model=self.MODEL, N=1, max_batch=_MODEL_CTX_BATCH, dtype=_abi.VC_F64,
                                params=self._params())
        return self._ctx

    @abstractmethod
    def _params(self) -> _abi.vc_params:
        pass

    @staticmethod
    def _batchify(x, u, kappa, h, nx):
        x = np.asarray(x, np.float64)
        single = x.ndim == 1
        xb = np.ascontiguousarray(x.reshape(-1, nx))
        B = xb.shape[0]
        ub = np.ascontiguousarray(np.asarray(u, np.float64).reshape(B, 2))
        kb = np.ascontiguousarray(np.broadcast_to(np.asarray(kappa, np.float64).reshape(-1), (B,)))
        hb = np.ascontiguousarray(np.broadcast_to(np.asarray(h, np.float64).reshape(-1), (B,)))
        return single, xb, ub, kb, hb

    def _transition(self, x, u, curvature, dt):
        nx = len(self.state)
        single, xb, ub, kb, hb = self._batchify(x, u, curvature, dt, nx)
        if not np.all(hb == hb[0]):
            raise ValueError("transition: one dt per call")
        out = self._context().plant_step(xb, ub, kb, float(hb[0]))
        return out[0] if single else out

    def _spatial_transition(self, x, u, curvature, ds):
        nx = len(self.state)
        single, xb, ub, kb, hb = self._batchify(x, u, curvature, ds, nx)
        out = self._context().spatial_step(xb, ub, kb, hb)
        return out[0] if single else out

    @property
    def transition(self):
        return self._transition

    @property
    def spatial_transition(self):
        return self._spatial_transition

    def _ode(self, x, u, curvature, space=False):
        nx = len(self.state)
        single, xb, ub, kb, _ = self._batchify(x, u, curvature, 0.0, nx)
        out = self._context().ode(xb, ub, kb, space=space)
        return out[0] if single else out

    def f(self, x, u, curvature=0.0):
        """dx/dt = f(x, u, curvature) (utils/integrators.py:18; one problem or a batch)."""
        return self._ode(x, u, curvature)

    def f_spatial(self, x, u, curvature=0.0):
        """dx/ds = f'(x, u, curvature), the MPC's spatial vector field (kinematic_car.py:47-60)."""
        return self._ode(x, u, curvature, space=True)

    def drive(self, input):
        """Plant step at the track curvature -- racing_car.py:34-46."""
        curvature = self.track.k(self.state.s)
        next_state = self.transition(self.state.values, input.values, curvature, self.dt)
        self.state = self.__class__.create_state(*next_state)
        self.input = input
        return self.state

    def rel2glob(self, state):
        s = state[self.state.index("s")]
        ey = state[self.state.index("ey")]
        epsi = state[self.state.index("epsi")]
        return self.track.rel2glob(s, ey, epsi)
