from .controller import Controller  # noqa: F401
from .kinematic_mpc import KinematicMPC, BatchedKinematicMPC  # noqa: F401
from .cascaded_mpc import BatchedCascadedMPC, BatchedSingleTrackMPC, CascadedMPC, CascadedTailMPC  # noqa: F401
