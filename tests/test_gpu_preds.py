"""GPU: the drop-in controllers' get_state_prediction() against the reference's recorded
predictions (tests/golden/preds_kat.npz, make_preds_kat.py).

The reference logs controller.get_state_prediction() after every step
(simulation/racing.py:239-240); column 0 is rel2glob of the state the controller was
given (x_0 = x0 in the NLP, cascaded_mpc.py:26-28,340-352).  Here the drop-in controller,
at the reference's recorded configuration (single-track N = 50 of race1_ippodromo through
the fp64 Riccati kernel; cascaded N = 20 + M = 40 of cascaded7_ippodromo), is commanded at
the recorded states: its prediction column 0 (state -> kernel xbar[0] -> rel2glob) must
reproduce the recorded one."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

XY_TOL = 5e-10
PSI_TOL = 2e-10


@pytest.fixture(scope="module")
def kat():
    return dict(np.load(os.path.join(GOLDEN, "preds_kat.npz"), allow_pickle=False))


def _rows(kat, run):
    i = int(np.nonzero(kat["run_name"] == run)[0][0])
    m = kat["run_id"] == i
    return i, kat["state"][m], kat["pred0"][m]


@pytest.mark.parametrize("run,cfg_name", [("race1_ippodromo/singletrack", "singletrack_mpc"),
                                          ("cascaded7_ippodromo/cascaded", "cascaded_mpc")])
def test_controller_prediction_column0_vs_recorded(kat, run, cfg_name):
    from vcmpc.config import load_config
    from vcmpc.controllers import CascadedMPC
    from vcmpc.environment import Track
    from vcmpc.models import DynamicCar, DynamicPointMass
    i, states, pred0 = _rows(kat, run)
    cfg = load_config(cfg_name)
    cfg["horizon"] = int(kat["run_N"][i])
    if int(kat["run_M"][i]) > 0:
        assert int(kat["run_M"][i]) == int(cfg["horizon_pm"]) and float(kat["run_ds_pm"][i]) == float(cfg["ds_pm"])
    cfg["mpc_dt"] = float(kat["run_mpc_dt"][i])
    tr = Track.load("ippodromo")
    np.random.seed(31)
    car = DynamicCar(load_config("dynamic_car"), tr, tyre="fiala")
    pm = DynamicPointMass(load_config("dynamic_car"), tr)
    mpc = CascadedMPC(car, pm, cfg)
    sel = np.linspace(0, len(states) - 1, 24).astype(int)
    exy = epsi = 0.0
    for j in sel:
        car.state = car.create_state(*states[j])
        mpc.command(car.state)
        p = np.asarray(mpc.get_state_prediction())
        assert p.shape == (cfg["horizon"] + int(cfg.get("horizon_pm", 0) or 0), 3)
        exy = max(exy, float(np.abs(p[0, :2] - pred0[j, :2]).max()))
        epsi = max(epsi, float(np.abs(np.angle(np.exp(1j * (p[0, 2] - pred0[j, 2]))))))
    print(f"{run}: max |xy - recorded| {exy:.2e} m, |psi - recorded| {epsi:.2e} rad over {len(sel)} steps")
    assert exy < XY_TOL and epsi < PSI_TOL
