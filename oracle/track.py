"""Track geometry and curvature k(s) -- CPU restatement (TEST INFRASTRUCTURE ONLY).

Restates ``Track`` of environment/track.py:83-361 with the same third-party calls
where they exist here (scipy ``InterpolatedUnivariateSpline``, numpy
``trapezoid``).  CasADi 3.6.7 (pixi.lock:35) is not importable: its
``interpolant(..., "bspline", grid, values)`` with the default ``not_a_knot``
algorithm and degree 3 is the unique cubic spline through the data with
not-a-knot end conditions, i.e. scipy ``CubicSpline(bc_type="not-a-knot")``.

Pipeline (reference lines):

1. centre line: each polygon edge sampled ``int(len/resolution)`` times without
   the end point, moving average of 2*smoothing+1 points away from the ends, the
   closing point appended then dropped again by ``_construct_waypoints``'s
   ``range(len - 1)``  (track.py:254-296, :298-330);
2. x(t), y(t): interpolating cubic through the waypoints on the index grid
   t = 0..n-1, re-sampled at the integers and re-interpolated by the bspline
   (track.py:206-231);
3. length = trapezoid of |r'(t)| over the integer grid (track.py:233-241); the
   arc-length map is t = s / length * n (track.py:244-245 -- n, not n-1);
4. curvature |x'y'' - x''y'| / |r'|^3 sampled at s = arange(0, length-0.1, 0.05)
   (track.py:109-119, :156-161; invariant under the s -> t rescale);
5. k(s) = bspline through those samples (track.py:162-167).  ``k`` does not wrap s
   (only ``get_curvature`` does, track.py:111); beyond the last sample it
   extrapolates the last cubic piece.

Pinned: k(s_n) against the curvature back-solved from the reference's recorded
closed-loop traces (tests/golden/dyn_plant_kat.npz, ippodromo and shoe runs):
max |dk| 8e-10 over 1131 steps (tests/test_oracle_track.py).
"""
from __future__ import annotations

import numpy as np
import yaml
from scipy.interpolate import CubicSpline, InterpolatedUnivariateSpline

K_DS = 0.05          # curvature sample spacing, track.py:157
K_TAIL = 0.1         # samples stop at length - 0.1, track.py:159


def centre_line(corners, resolution, smoothing):
    """track.py:254-296 (+ the closing-point drop of :312)."""
    wx, wy = [], []
    for (x0, y0), (x1, y1) in zip(corners[:-1], corners[1:]):
        n = int(np.sqrt((x1 - x0) ** 2 + (y1 - y0) ** 2) / resolution)
        wx.extend(np.linspace(x0, x1, n, endpoint=False).tolist())
        wy.extend(np.linspace(y0, y1, n, endpoint=False).tolist())
    n = len(wx)
    xs, ys = [], []
    for i in range(n):
        if smoothing <= i <= n - smoothing - 1:
            xs.append(np.mean(wx[i - smoothing:i + smoothing + 1]))
            ys.append(np.mean(wy[i - smoothing:i + smoothing + 1]))
        else:
            xs.append(wx[i])
            ys.append(wy[i])
    return np.array(xs), np.array(ys)


class Track:
    def __init__(self, cfg):
        self.name = cfg["name"]
        self.width = float(cfg["width"])
        X, Y = centre_line(cfg["corners"], float(cfg["resolution"]), int(cfg["smoothing"]))
        self.n_waypoints = n = len(X)
        t = np.arange(n)
        xv = InterpolatedUnivariateSpline(t, X, k=3, ext=3)(t)
        yv = InterpolatedUnivariateSpline(t, Y, k=3, ext=3)(t)
        self._x = CubicSpline(t, xv, bc_type="not-a-knot")
        self._y = CubicSpline(t, yv, bc_type="not-a-knot")
        speed = np.sqrt(self._x(t, 1) ** 2 + self._y(t, 1) ** 2)
        self.length = float(np.trapezoid(speed, t))
        self.s_samples = np.arange(0, self.length - K_TAIL, K_DS)
        self.k_samples = self.curvature(self.s_samples)
        self._k = CubicSpline(self.s_samples, self.k_samples, bc_type="not-a-knot")

    def _t(self, s):
        return np.asarray(s, np.float64) / self.length * self.n_waypoints

    def x(self, s):
        return self._x(self._t(s))

    def y(self, s):
        return self._y(self._t(s))

    def curvature(self, s):
        """``get_curvature`` (track.py:109-119), with its fmod."""
        t = self._t(np.fmod(s, self.length))
        dx, dy, ddx, ddy = self._x(t, 1), self._y(t, 1), self._x(t, 2), self._y(t, 2)
        return np.abs(dx * ddy - ddx * dy) / (dx ** 2 + dy ** 2) ** 1.5

    def k(self, s):
        """``Track.k`` (track.py:162-166): no wrap, cubic extrapolation past the samples."""
        return self._k(np.asarray(s, np.float64))

    def k_periodic(self, s):
        """k(fmod(s, length)) -- the build's lap-periodic curvature (device table)."""
        return self._k(np.fmod(np.asarray(s, np.float64), self.length))

    def orientation(self, s):
        """track.py:121-129."""
        t = self._t(np.fmod(s, self.length))
        return np.arctan2(self._y(t, 1), self._x(t, 1))

    def rel2glob(self, s, ey, epsi):
        """track.py:102-107."""
        th = self.orientation(s)
        x = self.x(s) - np.sin(th) * ey
        y = self.y(s) + np.cos(th) * ey
        psi = np.arctan2(np.sin(th + epsi), np.cos(th + epsi))
        return x, y, psi


def load_track(path):
    with open(path) as f:
        return Track(yaml.safe_load(f))
