"""Curvature provider k(s) for the controller and the plant.

The reference's ``Track`` (environment/track.py:83-361) builds a CasADi bspline
k(s) from sampled spline curvature every 0.05 m (track.py:156-167) and wraps s
modulo the track length (track.py:111).  The full Track restatement is SURVEY
8(f) row 1 (next); the hot path only needs k(s) as an input array, so this
class offers a sampled table with periodic linear interpolation (or a constant
curvature), which is all ``KinematicMPC._init_horizon`` and ``RacingCar.drive``
consume.
"""
from __future__ import annotations

import numpy as np


class CurvatureTrack:
    def __init__(self, s_samples=None, k_samples=None, length=None, constant=None):
        if constant is not None:
            self.length = float(length or 1e9)
            self._const = float(constant)
            self._s = self._k = None
        else:
            self._s = np.asarray(s_samples, np.float64)
            self._k = np.asarray(k_samples, np.float64)
            self.length = float(length if length is not None else self._s[-1])
            self._const = None
        self.obstacles = []

    def k(self, s):
        s = np.asarray(s, np.float64)
        if self._const is not None:
            return np.full(s.shape, self._const)
        return np.interp(np.mod(s, self.length), self._s, self._k)
