"""Dynamic bicycle -- mirrors models/dynamic_car.py:10-290.

Drive/brake split, load transfer, modified Fiala tyre (or the build-defined
linear tyre), temporal RK4 and spatial RK4 run in csrc/vc_models.hpp."""
from __future__ import annotations

from .. import _abi
from ..config import make_params
from ..utils.fancy_vector import FancyVector
from .racing_car import RacingCar


class DynamicCarAction(FancyVector):
    """[Fx, w] -- dynamic_car.py:202-237."""
    _keys = ["Fx", "w"]

    def __init__(self, Fx=0.0, w=0.0):
        super().__init__(Fx, w)


class DynamicCarState(FancyVector):
    """[Ux, Uy, r, delta, s, ey, epsi, t] -- dynamic_car.py:240-290."""
    _keys = ["Ux", "Uy", "r", "delta", "s", "ey", "epsi", "t"]

    def __init__(self, Ux=0.0, Uy=0.0, r=0.0, delta=0.0, s=0.0, ey=0.0, epsi=0.0, t=0.0):
        super().__init__(Ux, Uy, r, delta, s, ey, epsi, t)


class DynamicCar(RacingCar):
    MODEL = _abi.VC_MODEL_DYNAMIC

    def __init__(self, config, track, tyre: str = "fiala"):
        self.tyre = tyre
        super().__init__(config, track)

    @classmethod
    def create_state(cls, *args, **kwargs):
        return DynamicCarState(*args, **kwargs)

    @classmethod
    def create_action(cls, *args, **kwargs):
        return DynamicCarAction(*args, **kwargs)

    def _params(self):
        return make_params(dyn_car=self.config, tyre=self.tyre)
