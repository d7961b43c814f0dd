"""Dynamic point mass -- mirrors models/dynamic_point_mass.py:10-188 (the cascaded
controller's tail model: state [V, s, ey, epsi, t], action [Fx, Fy]).

On the GPU path the point-mass dynamics live inside the cascaded solve
(csrc/vc_models.hpp ``pm_spatial_ode``, used by csrc/casc_sqp.hip); this class keeps
the reference's containers and ``rel2glob`` so ``CascadedMPC(car, point_mass, config)``
is constructed exactly as simulation/racing.py:44-46 does.  Stand-alone point-mass
transitions are not exposed (the reference only evaluates them inside the NLP)."""
from __future__ import annotations

from ..utils.fancy_vector import FancyVector


class DynamicPointMassAction(FancyVector):
    """[Fx, Fy] -- dynamic_point_mass.py:114-143."""
    _keys = ["Fx", "Fy"]

    def __init__(self, Fx=0.0, Fy=0.0):
        super().__init__(Fx, Fy)


class DynamicPointMassState(FancyVector):
    """[V, s, ey, epsi, t] -- dynamic_point_mass.py:146-188."""
    _keys = ["V", "s", "ey", "epsi", "t"]

    def __init__(self, V=0.0, s=0.0, ey=0.0, epsi=0.0, t=0.0):
        super().__init__(V, s, ey, epsi, t)
        self.delta = 0  # fictitious steering angle (dynamic_point_mass.py:160)


class DynamicPointMass:
    def __init__(self, config, track):
        self.config = config
        self.track = track
        self.dt = config["dt"]
        self.state = DynamicPointMassState()
        self.input = DynamicPointMassAction()

    @classmethod
    def create_state(cls, *args, **kwargs):
        return DynamicPointMassState(*args, **kwargs)

    @classmethod
    def create_action(cls, *args, **kwargs):
        return DynamicPointMassAction(*args, **kwargs)

    def rel2glob(self, state):
        """racing_car.py:48-52 on the point-mass state order (s, ey, epsi = rows 1..3)."""
        return self.track.rel2glob(state[1], state[2], state[3])
