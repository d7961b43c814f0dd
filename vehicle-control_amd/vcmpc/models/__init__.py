from .robot import Robot  # noqa: F401
from .racing_car import RacingCar  # noqa: F401
from .kinematic_car import KinematicCar, KinematicCarAction, KinematicCarState  # noqa: F401
from .dynamic_car import DynamicCar, DynamicCarAction, DynamicCarState  # noqa: F401
from .dynamic_point_mass import DynamicPointMass, DynamicPointMassAction, DynamicPointMassState  # noqa: F401
