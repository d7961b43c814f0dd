"""CPU: host-side logic of the package (containers, config, workload, sharding)."""
import numpy as np

from vcmpc.config import AttrDict, load_config, make_params
from vcmpc.models.kinematic_car import KinematicCarAction, KinematicCarState
from vcmpc.models.dynamic_car import DynamicCarState
from vcmpc.workload import kinematic_batch, shard


def test_fancy_vector_surface():
    s = KinematicCarState(v=3.0, s=1.0)
    assert s.index("ey") == 3 and s.v == 3.0 and s["s"] == 1.0 and len(s) == 6
    s.ey = 0.5
    assert s.values[3] == 0.5
    a = KinematicCarAction(1.0, 0.1)
    assert a.values.dtype == np.float64 and a.w == 0.1
    d = DynamicCarState(*range(8))
    assert d.keys == ["Ux", "Uy", "r", "delta", "s", "ey", "epsi", "t"] and d.t == 7
    assert (s + s).v == 6.0


def test_config_and_params(kin_cfg):
    assert isinstance(kin_cfg, AttrDict) and kin_cfg.horizon == 20 and kin_cfg.cost_weights.time == 1
    p = make_params(kin_car=load_config("kinematic_car"), dyn_car=load_config("dynamic_car"), kin_mpc=kin_cfg)
    assert p.kin_car.l == 2.5 and p.dyn_car.m == 1700 and p.dyn_car.Caf == 234000
    assert p.kin_mpc.w_b == 5 and p.kin_mpc.delta_max == 0.3 and p.qp.prox == 1e-4


def test_workload_deterministic_and_well_posed():
    a = kinematic_batch(256, seed=3)
    b = kinematic_batch(256, seed=3)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])
        assert a[k].flags.c_contiguous and a[k].dtype == np.float64
    assert a["x0"].shape == (256, 6) and a["ubar"].shape == (256, 20, 2)
    from oracle import ltv_qp as Q
    xb = Q.kin_predict(a["x0"], a["ubar"], a["kappa"], a["ds"], 2.5)
    assert np.isfinite(xb).all() and xb[:, :, 0].min() > 1.0


def test_shard_covers_batch():
    for B, W in ((65536, 8), (1000, 3), (5, 8)):
        spans = [shard(B, r, W) for r in range(W)]
        assert spans[0][0] == 0 and spans[-1][1] == B
        assert all(spans[i][1] == spans[i + 1][0] for i in range(W - 1))
