from .curvature import CurvatureTrack  # noqa: F401
from .track import Track  # noqa: F401
