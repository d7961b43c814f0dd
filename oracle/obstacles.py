"""Oracle restatement of the obstacle barrier terms (TEST INFRASTRUCTURE ONLY).

The reference adds, for every stage n and every obstacle of the track
(``car.track.obstacles``, environment/track.py:131-138, data ``obstacle_data:
[s, ey, r]`` of config/environment/*.yaml), the barrier

    w_obs * ds_n / (dist - (r + 0.1)),   dist = sqrt((s_n - s_j)^2 + (ey_n - ey_j)^2)

to the NLP cost when the controller config says ``obstacles: True``
(kinematic_mpc.py:130-133, cascaded_mpc.py:173-176).  In both spatial models
s' = 1 (kinematic_car.py:56, dynamic_car.py:174), so s_n = s_0 + sum ds is not a
function of the decision variables and the barrier is a one-dimensional function
phi_n(ey_n) per stage.

The build's QP contract takes its *convexified* second-order model
at the prediction:

    phi_n(ey_bar + d) ~ phi_n(ey_bar) + p_n d + 1/2 q_n d^2,
    p_n = phi_n'(ey_bar),  q_n = max(phi_n''(ey_bar), 0)

(the barrier is not convex in ey: directly behind an obstacle it has a local
maximum, where the exact Hessian is negative), with the margin dist - (r + 0.1)
floored at ``margin_min`` in the derivatives (the reference's barrier is singular
at the obstacle boundary and negative inside it).  The device code is
``vc::obstacle_ey_model`` in csrc/vc_kernels.hpp; the operation order below is the
same.  Parity unpinned by the reference (no recorded run has ``obstacles: True``
with a QP to compare); checked against finite differences of phi itself
(tests/test_oracle_obstacles.py).
"""
from __future__ import annotations

import numpy as np

MARGIN_MIN = 0.05  # VC_OBS_MARGIN_MIN


def barrier(s, ey, wds, obstacles):
    """phi(ey) itself (the reference's cost term summed over obstacles)."""
    s, ey = np.asarray(s, np.float64), np.asarray(ey, np.float64)
    out = np.zeros(np.broadcast(s, ey).shape)
    for so, eo, r in obstacles:
        d = np.sqrt((s - so) ** 2 + (ey - eo) ** 2)
        out = out + wds / (d - (r + 0.1))
    return out


def ey_model(s, ey, wds, obstacles, margin_min=MARGIN_MIN, inside=False):
    """(p, q): slope and clamped curvature of phi at ey (arrays broadcast).  inside: beyond the
    band |margin| <= margin_min inside an obstacle the reference's own (negative) barrier
    instead of the floor (vc_obstacles.inside, csrc/vc_kernels.hpp)."""
    s, ey, wds = (np.asarray(v, np.float64) for v in (s, ey, wds))
    shape = np.broadcast(s, ey, wds).shape
    ps, qs = np.zeros(shape), np.zeros(shape)
    for so, eo, r in obstacles:
        a = s - so
        e = ey - eo
        d = np.sqrt(a * a + e * e)
        dc = np.maximum(d, 1e-6)
        m0 = d - (r + 0.1)
        m = np.where(inside & (m0 < -margin_min), m0, np.maximum(m0, margin_min))
        d1 = e / dc
        dd = (a * a) / (dc * dc * dc)
        im = 1.0 / m
        c1 = wds * im * im
        ps = ps - c1 * d1
        qs = qs + c1 * (2.0 * d1 * d1 * im - dd)
    return ps, np.maximum(qs, 0.0)
