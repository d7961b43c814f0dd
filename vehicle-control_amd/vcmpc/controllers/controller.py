"""Controller base -- mirrors controllers/controller.py:6-19 (``command`` contract).
``step`` is the north star's ``Controller.step(state) -> u`` alias."""
import numpy as np
from abc import ABC, abstractmethod


class Controller(ABC):
    def __init__(self, kp=None, kd=None):
        self.kp = kp
        self.kd = kd

    @abstractmethod
    def command(self, *args, **kwargs):
        pass

    def step(self, state):
        return self.command(state)


def neutral_restart(status, x0, u0, state_prediction, action_prediction, neutral_u, n_st=None):
    """A problem still not VC_SOLVED after the neutral retry restarts from the neutral warm start,
    as vc_simulate does (csrc/track.hip drive_kernel): it applies u = 0, and its next step's
    warm start is the current state at every stage with inputs ``neutral_u(rows)`` [b, 2, H] (zero
    when None) -- the failed retry's plan (possibly non-finite, or outside the spatial model's
    domain: VC_OUT_OF_DOMAIN) never becomes the next horizon's ds = mpc_dt * Ux.  In place."""
    bad = np.nonzero(np.asarray(status) != 0)[0]
    if len(bad) == 0:
        return
    u0[bad] = 0.0
    sp = np.repeat(x0[bad, :, None], state_prediction.shape[2], axis=2)
    if n_st is not None:   # cascaded: the point-mass columns hold (V, s, ey, epsi, t, 0, 0, 0)
        V = np.hypot(x0[bad, 0], x0[bad, 1])
        sp[:, :, n_st:] = 0.0
        for i, v in enumerate((V, x0[bad, 4], x0[bad, 5], x0[bad, 6], x0[bad, 7])):
            sp[:, i, n_st:] = v[:, None]
    state_prediction[bad] = sp
    action_prediction[bad] = 0.0 if neutral_u is None else neutral_u(bad)
