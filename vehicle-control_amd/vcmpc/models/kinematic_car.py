"""Kinematic bicycle -- mirrors models/kinematic_car.py:10-152.

Temporal ODE (Euler, kinematic_car.py:34-45) and spatial ODE (Euler,
kinematic_car.py:47-64) are evaluated by the gfx950 kernels in
csrc/vc_models.hpp; this class only keeps the reference's surface."""
from __future__ import annotations

from .. import _abi
from ..config import make_params
from ..utils.fancy_vector import FancyVector
from .racing_car import RacingCar


class KinematicCarAction(FancyVector):
    """[a, w] -- kinematic_car.py:75-104."""
    _keys = ["a", "w"]

    def __init__(self, a=0.0, w=0.0):
        super().__init__(a, w)


class KinematicCarState(FancyVector):
    """[v, delta, s, ey, epsi, t] -- kinematic_car.py:107-152."""
    _keys = ["v", "delta", "s", "ey", "epsi", "t"]

    def __init__(self, v=0.0, delta=0.0, s=0.0, ey=0.0, epsi=0.0, t=0.0):
        super().__init__(v, delta, s, ey, epsi, t)


class KinematicCar(RacingCar):
    MODEL = _abi.VC_MODEL_KINEMATIC

    @classmethod
    def create_state(cls, *args, **kwargs):
        return KinematicCarState(*args, **kwargs)

    @classmethod
    def create_action(cls, *args, **kwargs):
        return KinematicCarAction(*args, **kwargs)

    def _params(self):
        return make_params(kin_car=self.config)
