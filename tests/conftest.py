import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "vehicle-control_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvcmpc.so on cuda:0)")


@pytest.fixture(scope="session")
def kin_cfg():
    from vcmpc.config import load_config
    return load_config("kinematic_mpc")


@pytest.fixture(scope="session")
def kin_W(kin_cfg):
    from oracle import ltv_qp as Q
    return Q.kin_weights(kin_cfg)


@pytest.fixture(scope="session")
def dyn_params():
    from oracle import models as M
    from vcmpc.config import load_config
    return M.dyn_params_from_config(load_config("dynamic_car"))


@pytest.fixture(scope="session")
def kin_golden():
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, "kin_ltv_golden.npz")))


@pytest.fixture(scope="session")
def dyn_kat():
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, "dyn_plant_kat.npz")))
