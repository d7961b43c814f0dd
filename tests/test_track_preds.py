"""CPU: the track geometry and rel2glob pinned by the reference's recorded predictions.

Every recorded run stores get_state_prediction() per step (simulation/racing.py:239-240);
its column 0 is rel2glob of the measured state (x_0 = x0 in the NLP, cascaded_mpc.py:26-28,
:340-352; environment/track.py:102-107).  tests/golden/preds_kat.npz holds every 3rd step
of all 44 runs (make_preds_kat.py).  Both the oracle's scipy restatement (oracle/track.py)
and the package's own spline (vcmpc/environment/track.py) must reproduce them."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

XY_TOL = 5e-10    # [m]   measured max 1.1e-10 (shoe), residual of CasADi's B-spline fit
PSI_TOL = 2e-10   # [rad] measured max 4.8e-11


@pytest.fixture(scope="module")
def kat():
    return dict(np.load(os.path.join(GOLDEN, "preds_kat.npz"), allow_pickle=False))


def _wrap(a):
    return np.angle(np.exp(1j * a))


def _check(rel2glob_by_track, kat):
    worst = 0.0, 0.0
    for tid, name in ((0, "ippodromo"), (1, "shoe")):
        m = kat["track"] == tid
        st = kat["state"][m]
        x, y, psi = rel2glob_by_track[name](st[:, 4], st[:, 5], st[:, 6])
        exy = np.abs(np.stack([x, y], 1) - kat["pred0"][m, :2]).max()
        epsi = np.abs(_wrap(psi - kat["pred0"][m, 2])).max()
        worst = max(worst[0], exy), max(worst[1], epsi)
    return worst


def test_oracle_rel2glob_vs_recorded_predictions(kat):
    from oracle.track import load_track
    tr = {n: load_track(os.path.join(ROOT, "vehicle-control_amd", "config", "tracks", f"{n}.yaml"))
          for n in ("ippodromo", "shoe")}
    exy, epsi = _check({n: t.rel2glob for n, t in tr.items()}, kat)
    assert exy < XY_TOL and epsi < PSI_TOL, (exy, epsi)


def test_package_rel2glob_vs_recorded_predictions(kat):
    from vcmpc.environment import Track
    tr = {n: Track.load(n) for n in ("ippodromo", "shoe")}
    exy, epsi = _check({n: t.rel2glob for n, t in tr.items()}, kat)
    assert exy < XY_TOL and epsi < PSI_TOL, (exy, epsi)


def test_recorded_predictions_negative_control(kat):
    """A smoothing change (300 -> 280 window) moves the centre line: the pin must see it."""
    import yaml

    from oracle.track import Track
    with open(os.path.join(ROOT, "vehicle-control_amd", "config", "tracks", "ippodromo.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["smoothing"] = int(cfg["smoothing"]) - 20
    bad = Track(cfg)
    m = kat["track"] == 0
    st = kat["state"][m]
    x, y, _ = bad.rel2glob(st[:, 4], st[:, 5], st[:, 6])
    assert np.abs(np.stack([x, y], 1) - kat["pred0"][m, :2]).max() > 1e-3


def test_fixture_covers_every_recorded_run(kat):
    assert len(kat["run_name"]) == 44
    assert set(np.unique(kat["run_id"])) == set(range(44))
    # the reference's own horizons appear: single-track N = 50 / 60, cascaded M = 15 / 25 / 35 / 40
    assert {50, 60} <= set(kat["run_N"][kat["run_M"] == 0].tolist())
    assert {15, 25, 35, 40} <= set(kat["run_M"][kat["run_M"] > 0].tolist())
