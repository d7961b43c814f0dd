from .curvature import CurvatureTrack  # noqa: F401
