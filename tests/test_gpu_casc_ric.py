"""GPU parity of the stagewise-Riccati cascaded SQP kernel (csrc/casc_ric.hip, fp64) through
the C ABI, against the fp64 oracle of the cascaded contract (oracle/casc_sqp.py, exact dense
QPs) -- at cascaded.yaml's N = 20 + M = 40 (golden vectors) and the recorded runs' tails
M = 15 / 25 / 35 (experiments/data/*/cascaded_config.yaml), with and without obstacles.

Tolerance: the north star's 1e-5 on u* in the scaled decision variable (Fx / 1000 N, w,
Fy / 1000 N), i.e. 1e-2 N on the forces.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import casc_sqp as CS

pytestmark = pytest.mark.gpu

U_TOL = 1e-5
N = 20


def _scale(M):
    s = np.ones((N + M, 2))
    s[:, 0] = 1000.0
    s[N:, 1] = 1000.0
    return s


def _cfg(M):
    from vcmpc.config import load_config
    cfg = load_config("cascaded_mpc")
    cfg["horizon_pm"] = M
    return cfg


def _ctx(M, B=64, obstacles=None, solver=0):
    from vcmpc import Context, _abi
    from vcmpc.config import make_params, load_config
    cfg = _cfg(M)
    cfg["qp"] = dict(cfg["qp"], solver=solver)
    p = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=cfg, tyre="fiala", obstacles=obstacles)
    return Context(model=_abi.VC_MODEL_CASCADED, N=N, max_batch=B, dtype=_abi.VC_F64, params=p)


def test_casc_ric_vs_golden_m40():
    g = dict(np.load(os.path.join(GOLDEN, "casc_sqp_golden.npz")))
    with _ctx(40) as c:
        u0, xs, us, st, it, dg = c.solve(g["x0"].copy(), g["kappa"].copy(), g["ds"].copy(), g["ubar"].copy(),
                                         diag=True)
    err = np.abs((us - g["u_star"]) / _scale(40)).max(axis=(1, 2))
    print("M=40 golden: scaled |u* - u*_oracle| max %.2e, status %s, IPM iterations %s, diag %s"
          % (err.max(), st, it, dg[:, :2].max(0)))
    assert (st == 0).all(), (st, dg)
    assert err.max() < U_TOL
    np.testing.assert_array_equal(u0, us[:, 0])
    assert np.abs(xs - g["x_star"]).max() < 1e-6


@pytest.mark.parametrize("M", [15, 25, 35])
def test_casc_ric_recorded_tails_vs_oracle(M, dyn_params):
    from vcmpc.workload import cascaded_batch
    W = CS.casc_weights(_cfg(M))
    d = cascaded_batch(3, M=M, seed=400 + M)
    ref = CS.casc_sqp_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], dyn_params, W, tyre="fiala")
    with _ctx(M) as c:
        u0, xs, us, st, it = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())
    err = np.abs((us - ref["u_star"]) / _scale(M)).max()
    print(f"M={M}: scaled |u* - u*_oracle| = {err:.2e}, status {st}, iterations {it}")
    assert (st == 0).all(), st
    assert err < U_TOL
    assert np.abs(xs - ref["x_star"]).max() < 1e-6


def test_casc_ric_obstacles_vs_oracle(dyn_params):
    from vcmpc.workload import cascaded_batch
    obs = [tuple(float(v) for v in o) for o in np.load(os.path.join(GOLDEN, "obs_golden.npz"))["obstacles"]]
    W = CS.casc_weights(_cfg(40))
    W["obstacles"] = obs
    d = cascaded_batch(3, seed=77)
    d["x0"][:, 4] = [20.0, 50.0, 90.0]
    ref = CS.casc_sqp_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], dyn_params, W, tyre="fiala")
    with _ctx(40, obstacles=obs) as c:
        u0, xs, us, st, it = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())
    err = np.abs((us - ref["u_star"]) / _scale(40)).max()
    print(f"obstacles: scaled |u* - u*_oracle| = {err:.2e}, status {st}")
    assert (st == 0).all()
    assert err < U_TOL


def test_casc_ric_matches_condensed_kernel():
    """M = 40: the stagewise kernel and the condensed casc_sqp.hip (qp.solver = 2) agree."""
    from vcmpc.workload import cascaded_batch
    d = cascaded_batch(128, seed=5)
    with _ctx(40, B=128, solver=0) as c:
        r0 = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())
    with _ctx(40, B=128, solver=2) as c:
        r2 = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())
    ok = (r0[3] == 0) & (r2[3] == 0)
    err = np.abs((r0[2] - r2[2]) / _scale(40))[ok].max()
    print(f"stagewise vs condensed on {ok.sum()} problems solved by both: scaled |du*| {err:.2e}; "
          f"solved {np.mean(r0[3] == 0):.3f} vs {np.mean(r2[3] == 0):.3f}")
    assert err < U_TOL
    assert (r0[3] == 0).mean() >= (r2[3] == 0).mean()


@pytest.mark.parametrize("M", [15, 40])
def test_casc_ric_batch_properties(M, dyn_params):
    """B = 4096 (the bench's cascaded batch): every problem solved unless one of its SQP
    iterations meets a linearised QP with no feasible point (phase-1 LP with a checked Farkas
    certificate -- a property of the contract at that warm start, not of the kernel); w inside
    its box, finite outputs, bit-identical host / device pointer runs."""
    import torch
    from vcmpc.workload import cascaded_batch
    B = 4096
    d = cascaded_batch(B, M=M, seed=9)
    with _ctx(M, B=B) as c:
        u0, xs, us, st, it, dg = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
        dev = {k: torch.from_numpy(v.copy()).cuda() for k, v in d.items()}
        r = c.solve(dev["x0"], dev["kappa"], dev["ds"], dev["ubar"])
        torch.cuda.synchronize()
    bad = np.nonzero(st != 0)[0]
    print(f"M={M} B={B}: solved {(st == 0).mean():.5f}, IPM iterations mean {it.mean():.1f} max {it.max()}; "
          f"non-solved {[(int(b), dg[b].tolist()) for b in bad[:4]]}")
    assert len(bad) <= 8
    if len(bad):
        # a non-solved problem must meet a QP with no feasible point: phase-1 LP + checked Farkas
        # certificate (oracle/feasibility.py) on the oracle's SQP iterates up to the first such QP
        from oracle import feasibility as F
        W = CS.casc_weights(_cfg(M))
        sub = {k: v[bad] for k, v in d.items()}
        ref = CS.casc_sqp_solve(sub["x0"], sub["ubar"], sub["kappa"], sub["ds"], dyn_params, W, tyre="fiala",
                                keep_qps=True)
        first, farkas = F.first_infeasible_iteration(ref["hist"])
        print("first SQP iteration with an infeasible QP (-1: none):", first.tolist(), "Farkas ok:", farkas.tolist())
        assert (first >= 0).all() and farkas.all()
    ok = st == 0
    assert np.isfinite(us[ok]).all() and np.isfinite(xs[ok]).all()
    assert (np.abs(us[:, :N, 1]) <= 0.4 + 1e-12).all()
    np.testing.assert_array_equal(r[2].cpu().numpy(), us)


@pytest.mark.parametrize("M", [35, 40])
def test_casc_ric_j_placement_bit_identical(M):
    """Round 5: M = 35 / 40 keep the stage Jacobians in LDS while the batch fits the machine at
    three workgroups per CU and in a global workspace beyond (four per CU; csrc/casc_ric.hip
    cr_launch): every problem of a 4,096 batch (global J) equals the same problem solved in LDS-J
    chunks of 512 bit for bit (the whole batch: ADVICE r05)."""
    from vcmpc.workload import cascaded_batch
    B, CH = 4096, 512
    d = cascaded_batch(B, M=M, seed=56)
    with _ctx(M, B=B) as c:
        big = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
        parts = [c.solve(d["x0"][i:i + CH], d["kappa"][i:i + CH], d["ds"][i:i + CH], d["ubar"][i:i + CH].copy(),
                         diag=True) for i in range(0, B, CH)]
    small = [np.concatenate([p[j] for p in parts]) for j in range(len(big))]
    print(f"M={M}: solved {(big[3] == 0).mean():.4f} of {B}")
    for a, b in zip(big, small):
        np.testing.assert_array_equal(a, b)
