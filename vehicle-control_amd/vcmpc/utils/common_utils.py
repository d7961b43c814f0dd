"""Host utilities mirrored from the reference (utils/common_utils.py)."""
import numpy as np

from ..config import load_config  # noqa: F401  (common_utils.py:16-19)


def wrap(angle):
    """Wrap an angle into [-pi, pi] -- utils/common_utils.py:22-31 (single wrap)."""
    if angle < -np.pi:
        return 2 * np.pi + angle
    if angle > np.pi:
        return angle - 2 * np.pi
    return angle
