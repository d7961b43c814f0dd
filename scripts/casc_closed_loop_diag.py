"""GPU diagnostic: the single-vehicle cascaded controller's closed loop on ippodromo,
printing status / iterations / state every few steps (tests/test_gpu_casc.py runs the
same loop with assertions)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))
from vcmpc.config import load_config  # noqa: E402
from vcmpc.controllers import CascadedMPC  # noqa: E402
from vcmpc.environment import Track  # noqa: E402
from vcmpc.models import DynamicCar, DynamicPointMass  # noqa: E402

np.random.seed(31)
tr = Track.load("ippodromo")
car = DynamicCar(load_config("dynamic_car"), tr, tyre="fiala")
car.state = car.create_state(Ux=8.0, s=1.0)
mpc = CascadedMPC(car, DynamicPointMass(load_config("dynamic_car"), tr), load_config("cascaded_mpc"))
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
for k in range(steps):
    a = mpc.command(car.state)
    car.drive(a)
    if k % 10 == 0 or mpc.status[0] != 0:
        x = car.state.values
        print(f"{k:4d} st {mpc.status[0]} it {mpc.iters[0]:3d} Fx {a.Fx:8.1f} w {a.w:6.3f} | Ux {x[0]:5.2f} Uy {x[1]:6.3f} "
              f"r {x[2]:6.3f} d {x[3]:6.3f} s {x[4]:7.2f} ey {x[5]:6.2f} ep {x[6]:6.3f} | Vpm_end {mpc.state_prediction[0, -1]:6.2f}",
              flush=True)
