"""Race track: centre line, arc-length geometry and the curvature table k(s).

Mirrors ``Track`` of environment/track.py:83-361 for what the MPC path consumes:
``length``, ``width``, ``k(s)`` (track.py:162-166), ``get_curvature`` (:109-119),
``get_orientation`` (:121-129), ``rel2glob`` (:102-107), ``x``/``y`` (:244-245).

Construction follows the reference pipeline (track.py:206-296):

1. centre line: polygon edges sampled every ``resolution`` m (end point
   excluded), a (2*smoothing+1)-point moving average away from both ends, the
   closing point dropped (``_construct_waypoints`` iterates ``len - 1``);
2. x(t), y(t): the not-a-knot interpolating cubic on the index grid t = 0..n-1
   (the reference's scipy spline re-sampled into a CasADi degree-3 bspline, which
   is the same interpolant);
3. length: trapezoid rule of |r'(t)| on the integer grid; arc length maps to the
   index as t = s / length * n (n, not n - 1, as in the reference);
4. curvature |x'y'' - x''y'| / |r'|^3 sampled every 0.05 m on [0, length - 0.1),
   then the not-a-knot cubic through the samples is the table k(s).

The spline code here is this package's own (uniform-grid second-derivative form
with a tridiagonal sweep); the test oracle (oracle/track.py) builds the same
curve with scipy and is pinned against curvature back-solved from the
reference's recorded runs.  The table is uploaded to the device with
``Context.set_track`` and evaluated there by every closed-loop kernel; ``k`` below
is the host evaluation of the same table (used by the host-side ``_init_horizon``
of the single-vehicle controllers).

Deviation: ``k`` wraps s modulo the lap length (like ``get_curvature``,
track.py:111); the reference's ``k`` does not, because its simulator stops at
the end of the first lap (simulation/racing.py:219).
"""
from __future__ import annotations

import os

import numpy as np
import yaml

K_DS = 0.05    # curvature sample spacing [m] (track.py:157)
K_TAIL = 0.1   # samples stop at length - 0.1 (track.py:159)

_TRACK_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                          "config", "tracks")


def natural_pieces(y, h):
    """Cubic pieces (c0, c1, c2, c3) of the not-a-knot interpolating spline through
    y on a uniform grid of spacing h: piece i is c0 + c1 t + c2 t^2 + c3 t^3 on
    [x_i, x_i + h).  Returns coef[n-1][4]."""
    y = np.asarray(y, np.float64)
    n = len(y)
    if n < 4:
        raise ValueError("not-a-knot cubic needs at least 4 points")
    r = (6.0 / (h * h)) * (y[2:] - 2.0 * y[1:-1] + y[:-2])      # rows i = 1..n-2
    M = np.zeros(n)
    # not-a-knot (M0 = 2 M1 - M2, M_{n-1} = 2 M_{n-2} - M_{n-3}) turns rows 1 and
    # n-2 of M_{i-1} + 4 M_i + M_{i+1} = r_i into 6 M_1 = r_1, 6 M_{n-2} = r_{n-2}
    M[1] = r[0] / 6.0
    M[n - 2] = r[-1] / 6.0
    m = n - 4                                                    # unknowns M_2..M_{n-3}
    if m > 0:
        d = r[1:-1].copy()
        d[0] -= M[1]
        d[-1] -= M[n - 2]
        cp = np.empty(m)
        dp = np.empty(m)
        cp[0], dp[0] = 0.25, d[0] / 4.0
        for i in range(1, m):                                    # Thomas sweep, diag 4, off-diag 1
            den = 4.0 - cp[i - 1]
            cp[i] = 1.0 / den
            dp[i] = (d[i] - dp[i - 1]) / den
        sol = np.empty(m)
        sol[-1] = dp[-1]
        for i in range(m - 2, -1, -1):
            sol[i] = dp[i] - cp[i] * sol[i + 1]
        M[2:n - 2] = sol
    M[0] = 2.0 * M[1] - M[2]
    M[n - 1] = 2.0 * M[n - 2] - M[n - 3]
    coef = np.empty((n - 1, 4))
    coef[:, 0] = y[:-1]
    coef[:, 1] = (y[1:] - y[:-1]) / h - h * (2.0 * M[:-1] + M[1:]) / 6.0
    coef[:, 2] = M[:-1] / 2.0
    coef[:, 3] = (M[1:] - M[:-1]) / (6.0 * h)
    return coef


def eval_pieces(coef, h, x, deriv=0):
    """Evaluate piecewise cubic (uniform grid from 0, spacing h) or its 1st/2nd
    derivative; the end pieces extrapolate."""
    x = np.asarray(x, np.float64)
    i = np.clip(np.floor(x / h), 0, len(coef) - 1).astype(np.int64)
    t = x - i * h
    c = coef[i]
    if deriv == 0:
        return ((c[..., 3] * t + c[..., 2]) * t + c[..., 1]) * t + c[..., 0]
    if deriv == 1:
        return (3.0 * c[..., 3] * t + 2.0 * c[..., 2]) * t + c[..., 1]
    return 6.0 * c[..., 3] * t + 2.0 * c[..., 2]


def centre_line(corners, resolution, smoothing):
    xs, ys = [], []
    for (x0, y0), (x1, y1) in zip(corners[:-1], corners[1:]):
        n = int(np.hypot(x1 - x0, y1 - y0) / resolution)
        xs.append(np.linspace(x0, x1, n, endpoint=False))
        ys.append(np.linspace(y0, y1, n, endpoint=False))
    x, y = np.concatenate(xs), np.concatenate(ys)
    w = 2 * smoothing + 1
    if len(x) >= w:
        sl = slice(smoothing, len(x) - smoothing)
        x, y = x.copy(), y.copy()
        x[sl] = np.lib.stride_tricks.sliding_window_view(x.copy(), w).mean(axis=1)
        y[sl] = np.lib.stride_tricks.sliding_window_view(y.copy(), w).mean(axis=1)
    return x, y


class Obstacle:
    """Circular obstacle (environment/track.py:55-70): centre (cx, cy) in world
    coordinates, (s, ey) in track coordinates, radius in m."""

    def __init__(self, cx, cy, s, ey, radius):
        self.cx, self.cy, self.s, self.ey, self.radius = cx, cy, s, ey, radius

    def __repr__(self) -> str:
        return f"Obstacle(cx={self.cx}, cy={self.cy}, radius={self.radius})"


class Track:
    def __init__(self, config):
        self.name = config["name"]
        self.width = float(config["width"])
        self.resolution = float(config["resolution"])
        self.smoothing = int(config["smoothing"])
        self.obstacle_data = [tuple(o) for o in config.get("obstacles", [])]
        wx, wy = centre_line(config["corners"], self.resolution, self.smoothing)
        self.n_waypoints = n = len(wx)
        self._cx = natural_pieces(wx, 1.0)
        self._cy = natural_pieces(wy, 1.0)
        t = np.arange(n, dtype=np.float64)
        speed = np.hypot(eval_pieces(self._cx, 1.0, t, 1), eval_pieces(self._cy, 1.0, t, 1))
        self.length = float(np.sum(0.5 * (speed[1:] + speed[:-1])))
        self.s_samples = np.arange(0, self.length - K_TAIL, K_DS)
        self.k_samples = self.get_curvature(self.s_samples)
        self._ck = natural_pieces(self.k_samples, K_DS)
        self.obstacles = self._construct_obstacles(self.obstacle_data)

    def _construct_obstacles(self, obstacle_data):
        """track.py:131-138 (the occupancy grid of :140-153 is plotting-only, out of scope)."""
        out = []
        for s, ey, radius in obstacle_data:
            x, y, _ = self.rel2glob(s, ey, 0.0)
            out.append(Obstacle(float(x), float(y), float(s), float(ey), float(radius)))
        return out

    @classmethod
    def load(cls, name_or_path: str) -> "Track":
        """``Track.load("ippodromo")`` or a path to a track yaml."""
        path = name_or_path if os.path.exists(name_or_path) else os.path.join(_TRACK_DIR, f"{name_or_path}.yaml")
        with open(path) as f:
            return cls(yaml.safe_load(f))

    # -- geometry ---------------------------------------------------------------------
    def _t(self, s):
        return np.fmod(np.asarray(s, np.float64), self.length) / self.length * self.n_waypoints

    def x(self, s):
        return eval_pieces(self._cx, 1.0, self._t(s))

    def y(self, s):
        return eval_pieces(self._cy, 1.0, self._t(s))

    def get_curvature(self, s):
        """Unsigned curvature of the centre line (track.py:109-119)."""
        t = self._t(s)
        dx, dy = eval_pieces(self._cx, 1.0, t, 1), eval_pieces(self._cy, 1.0, t, 1)
        ddx, ddy = eval_pieces(self._cx, 1.0, t, 2), eval_pieces(self._cy, 1.0, t, 2)
        return np.abs(dx * ddy - ddx * dy) / (dx * dx + dy * dy) ** 1.5

    def get_orientation(self, s):
        t = self._t(s)
        return np.arctan2(eval_pieces(self._cy, 1.0, t, 1), eval_pieces(self._cx, 1.0, t, 1))

    def rel2glob(self, s, ey, epsi):
        th = self.get_orientation(s)
        x = self.x(s) - np.sin(th) * ey
        y = self.y(s) + np.cos(th) * ey
        psi = np.mod(th + epsi + np.pi, 2 * np.pi) - np.pi
        return x, y, psi

    # -- curvature table ----------------------------------------------------------------
    def kappa_table(self):
        """(coef[n][4], h, length) -- the layout ``vc_track_set`` takes."""
        return self._ck, K_DS, self.length

    def k(self, s):
        """k(s) from the table, s wrapped modulo the lap (host evaluation; the device
        evaluates the same table in vc_track_k / vc_horizon / vc_drive)."""
        return eval_pieces(self._ck, K_DS, np.fmod(np.asarray(s, np.float64), self.length))
