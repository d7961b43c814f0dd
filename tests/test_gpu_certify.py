"""Every problem of every bench-size batch against the KKT conditions of the oracle-built QP.

The other parity tests compare the kernels with the oracle on golden sets and strided samples.
Every "solved" status at bench scale otherwise rests on the kernel's own certificate.  The round-4
early polish certified C4 problem 23921 9e-3 off the optimum, and only a kernel A/B caught it.
So here every returned answer of each bench batch is checked independently of the kernel:

* KKT certificate (oracle/certify.py): the QP (H, g, C, d) is rebuilt by the oracle restatement
  at the kernel's own linearisation point.  Multipliers are recovered by NNLS on the rows the
  answer makes active.  Stationarity, primal and dual feasibility and complementarity must all
  hold to CERT_TOL * scale for every problem the kernel reports solved.  scale = 1 + max(|g|, |d|)
  is the interior point's own scale.
* The oracle's exact optimum of the same QP (active-set polish, certified; interior point where
  the seeded polish does not certify): max ||u* - u*_oracle||_inf over the whole set is printed
  and held to the north star's 1e-5.  The unseeded oracle (interior point + polish from z = 0)
  runs on a strided sample and must agree with the seeded one.
* SQP batches (single-track, cascaded): every QP of the SQP is certified.  The kernel is run
  with sqp_iters = 1 .. K, so its iterates u_0 .. u_K are known, and QP k is rebuilt at u_{k-1}.
  The oracle's own SQP (exact QPs at its own iterates, the contract's domain and stopping rules)
  gives u*_oracle.

Sets: the C2 batch (1,024), the bench's C4 problem set (65,536, vcmpc.workload.c4_shard), the
C4-style kinematic_batch(65536, seed = 31) where 23921 lives, kinematic N = 50 (8,192), C3
(4,096, N = 40, 3 SQP iterations), C3 on SURVEY 8(d)'s full sampler ranges (4,096; round 6),
single-track N = 60 (4,096) and cascaded 20 + 40 (4,096).
These are the bench legs' own seeds (bench.py, rank 0).  A failure here is a kernel bug to fix.
"""
import numpy as np
import pytest

from oracle import certify as CF

pytestmark = pytest.mark.gpu

CERT_TOL = 1e-9     # KKT residuals, x scale
DIST_TOL = 1e-9     # SQP QPs: or |dz - dz_exact|_inf (scaled units) to the oracle's certified optimum
U_TOL = 1e-5        # north star: ||u* - u*_oracle||_inf (kinematic: m/s^2, rad/s; SQP: N, rad/s)
L = 2.5


def _kin_ctx(N, B, solver=0):
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    cfg = load_config("kinematic_mpc")
    cfg["qp"] = dict(cfg.get("qp") or {}, solver=solver)
    p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=cfg)
    return Context(model=_abi.VC_MODEL_KINEMATIC, N=N, max_batch=B, dtype=_abi.VC_F64, params=p)


def _kin_set(name):
    from vcmpc.workload import c4_shard, kinematic_batch
    if name == "c2":
        return 20, kinematic_batch(1024, N=20, seed=31)          # bench.py main(), rank 0
    if name == "c4_bench":
        return 20, c4_shard(65536, 0, 1, 31)[2]                   # bench.py run_c4, all ranks' shards
    if name == "c4_seed31":
        return 20, kinematic_batch(65536, N=20, seed=31)          # where 23921 lives
    if name == "n50":
        return 50, kinematic_batch(8192, N=50, seed=77)           # test_kin_ric_batch_properties_n50
    raise ValueError(name)


def _summary(name, solved, cert, ok, err):
    s = cert["scale"]
    print(f"{name}: {int(solved.sum())}/{len(solved)} solved, certified {int((ok & solved).sum())}; "
          f"max stat {np.max(cert['stat'][solved] / s[solved]):.2e}, pfeas {np.max(cert['pfeas'][solved] / s[solved]):.2e}, "
          f"comp {np.max(cert['comp'][solved] / s[solved]):.2e} (x scale); "
          f"max |u* - u*_oracle|_inf over the set {err:.3e}")


@pytest.mark.parametrize("name", ["c2", "c4_bench", "c4_seed31", "n50"])
def test_kinematic_batch_every_problem_certified(name, kin_W):
    N, d = _kin_set(name)
    B = len(d["x0"])
    with _kin_ctx(N, B) as c:
        u0, xs, us, st, it = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy())
    z = (us - d["ubar"]).reshape(B, 2 * N)
    r = CF.certify_batch("kin", z, dict(W=kin_W, L=L), {k: d[k] for k in ("x0", "ubar", "kappa", "ds")},
                         chunk=2048 if N == 20 else 512, independent_every=64 if N == 20 else 32)
    solved = st == 0
    ok = CF.kkt_ok(r, CERT_TOL)
    err_all = np.abs(z - r["z_exact"]).max(axis=1)
    _summary(f"kinematic {name} (N={N})", solved, r, ok, float(err_all[solved].max()))
    assert solved.all(), np.nonzero(~solved)[0][:10]
    bad = np.nonzero(solved & ~ok)[0]
    assert len(bad) == 0, [(int(b), float(r["stat"][b] / r["scale"][b]), float(err_all[b])) for b in bad[:10]]
    assert r["exact_ok"].all()
    assert err_all.max() < U_TOL
    # the unseeded oracle agrees with the seeded one (the optimum is unique)
    idx = r["indep_idx"]
    assert r["indep_ok"].all()
    assert np.abs(r["z_indep"] - r["z_exact"][idx]).max() < 1e-9


def _dyn_ctx(kind, N, B, cfg, tyre):
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    params = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=cfg, tyre=tyre)
    model = _abi.VC_MODEL_CASCADED if kind == "casc" else _abi.VC_MODEL_DYNAMIC
    return Context(model=model, N=N, max_batch=B, dtype=_abi.VC_F64, params=params)


def _sqp_set(name):
    from vcmpc.config import load_config
    from vcmpc.workload import cascaded_batch, dynamic_batch
    if name == "c3":          # bench.py run_c3, rank 0
        d = {k: v.astype(np.float64) for k, v in dynamic_batch(4096, N=40, seed=31).items()}
        return "dyn", 40, d, load_config("dynamic_mpc"), "linear"
    if name == "c3_survey":   # bench.py c3_survey: SURVEY 8(d)'s sampler ranges as written
        d = {k: v.astype(np.float64) for k, v in dynamic_batch(4096, N=40, seed=31, ranges="survey").items()}
        return "dyn", 40, d, load_config("dynamic_mpc"), "linear"
    if name == "st_n60":      # bench.py singletrack_n60_f64
        d = {k: v.astype(np.float64) for k, v in dynamic_batch(4096, N=60, seed=31).items()}
        return "dyn", 60, d, load_config("singletrack_mpc"), "linear"
    if name == "cascaded":    # bench.py run_casc
        return "casc", 20, cascaded_batch(4096, seed=31), load_config("cascaded_mpc"), "fiala"
    raise ValueError(name)


@pytest.mark.parametrize("name", ["c3", "st_n60", "cascaded", "c3_survey"])
def test_sqp_batch_every_qp_certified(name, dyn_params):
    from oracle import casc_sqp as CS
    from oracle import dyn_sqp as D
    kind, N, d, cfg, tyre = _sqp_set(name)
    B = len(d["x0"])
    K = int(cfg["qp"]["sqp_iters"])
    us, stop, st_k = [d["ubar"].copy()], [], []
    for k in range(1, K + 1):
        ck = dict(cfg, qp=dict(cfg["qp"], sqp_iters=k))
        with _dyn_ctx(kind, N, B, ck, tyre) as c:
            u0, xs, u, st, it, dg = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
        us.append(u)
        stop.append((dg[:, 2].astype(int) & 16) > 0)
        st_k.append(st)
    us, stop = np.stack(us), np.stack(stop)
    W = CS.casc_weights(cfg) if kind == "casc" else D.dyn_weights(cfg)
    r = CF.certify_sqp_batch(kind, us, stop, dict(W=W, p=dyn_params, tyre=tyre),
                             {k: d[k] for k in ("x0", "kappa", "ds")}, chunk=128)
    solved = st_k[-1] == 0
    lim = CERT_TOL * r["scale"]
    kkt = (r["stat"] <= lim) & (r["pfeas"] <= lim) & (r["dfeas"] <= lim) & (r["comp"] <= lim)
    # or within DIST_TOL (scaled units) of the oracle's certified exact optimum of the same QP: the
    # condensed Hessians of the long single-track horizons reach |H| ~ 1e7 with curvature ~ 3e-2 (cond
    # ~ 5e8, the RK4 lateral mode), where an answer 6e-11 from the optimum already reads 2e-9 x scale in
    # condensed stationarity (N = 60 problem 2531, r05e)
    near = (r["pfeas"] <= lim) & (r["dz_err"] <= DIST_TOL)
    ok = kkt | near
    if name == "c3_survey":
        # SURVEY 8(d)'s full ranges: Fx warm starts drawn independently per stage over +-6000 N make the
        # first QPs' Fx-slew terms huge (scale = 1 + max |g|, |d| reaches 1e7-2e8), where the NNLS activity
        # threshold 1e-7 x scale calls rows thousands of newtons from their bound active and the oracle's
        # "exact" polish is itself no better than the kernel (r06g, scripts/c3_survey_cert_diag.py: the
        # kernel's objective lower in 4 of 5 uncertified QPs).  Two more acceptances there: objective-
        # certified (feasible, and 1/2 z'Hz + g'z within 1e-9 of the magnitude of its terms above the
        # oracle's optimum) and a step refused by both (alpha = 0: no step length keeps the rollout inside
        # the domain, and the kernel took none)
        objc = (r["pfeas"] <= lim) & (r["f_k"] <= r["f_o"] + 1e-9 * (1.0 + r["f_mag"]))
        ok = ok | objc | r["refused_both"]
        print(f"  c3_survey acceptance: KKT {int(kkt.sum())}, near {int((near & ~kkt).sum())}, objective "
              f"{int((objc & ~kkt & ~near).sum())}, refused by both {int((r['refused_both'] & ~kkt & ~near & ~objc).sum())} "
              f"(QP-problem pairs over {K} QPs)")
    sc = CF.sqp_scale(kind, us.shape[2], N)
    err = np.abs(us[-1] - r["u_oracle"]).max(axis=(1, 2))
    print(f"{name}: {int(solved.sum())}/{B} solved at K = {K}; stopped early at QP k: {stop.sum(axis=1).tolist()}; "
          f"step lengths < 1: {(r['alpha'] < 1).sum(axis=1).tolist()}")
    fails, unresolved_total = [], 0
    for k in range(K):
        # QP k is the kernel's where the k-run reports solved and did not stop at QP k
        req = (st_k[k] == 0) & ~stop[k]
        s = r["scale"][k]
        bad = np.nonzero(req & ~ok[k])[0]
        print(f"  QP {k + 1}: required {int(req.sum())}, certified {int((ok[k] & req).sum())} (by distance to the "
              f"exact optimum: {int((req & ~kkt[k] & near[k]).sum())}); max stat "
              f"{np.max(r['stat'][k][req] / s[req]):.2e} pfeas {np.max(r['pfeas'][k][req] / s[req]):.2e} comp "
              f"{np.max(r['comp'][k][req] / s[req]):.2e}; max |dz - dz_oracle| {r['dz_err'][k][req].max():.2e} "
              f"(scaled); uncertified {[(int(b), float(r['stat'][k][b] / s[b]), float(r['dz_err'][k][b])) for b in bad[:6]]}")
        fails += [(k + 1, int(b)) for b in bad]
        # the oracle's optimum is the reference wherever the kernel's answer is not KKT-certified on its own
        # (c3_survey: the oracle's own polish does not certify every one of these badly scaled QPs either;
        # where the kernel's answer is KKT-certified, it needs no reference)
        need = req & ~kkt[k] & ~r["refused_both"][k] if name == "c3_survey" else req
        if name == "c3_survey":
            # QPs whose answer neither the kernel's KKT certificate nor the oracle's own polish certifies at
            # 1e-9 x scale (scale 1e7-1e8): accepted by objective against the oracle's best point, listed,
            # and held to one in 2,000 QPs
            unres = np.nonzero(need & ~r["exact_ok"][k])[0]
            print(f"  QP {k + 1}: unresolved by both certificates {[(int(b), float(r['f_k'][k][b] - r['f_o'][k][b]), float(r['f_mag'][k][b])) for b in unres[:10]]}")
            unresolved_total += len(unres)
            continue
        assert r["exact_ok"][k][need].all(), np.nonzero(need & ~r["exact_ok"][k])[0][:10]
    worst = np.argsort(-np.where(solved, err, 0))[:5]
    print(f"  max |u* - u*_oracle|_inf over the solved set: {err[solved].max():.3e} (N, rad/s); "
          f"in QP units {np.abs((us[-1] - r['u_oracle']) / sc).max(axis=(1, 2))[solved].max():.3e}; "
          f"> 1e-5: {int((err[solved] > U_TOL).sum())}; worst {[(int(b), float(err[b])) for b in worst]}")
    assert not fails, fails[:20]
    if name != "c3_survey":
        assert err[solved].max() < U_TOL
        assert (solved.mean() >= 0.997), np.bincount(st_k[-1])
        return
    assert unresolved_total <= (K * B) // 2000
    # Every QP the kernel solved is certified at the kernel's own iterates (above).  The oracle's own SQP
    # can still end elsewhere where the kernel STOPPED the SQP: at these scales (1e7-1e8) a later QP's
    # Riccati factorisation breaks down for a few problems (diag bit 1), the kernel refuses that step
    # (the keep-the-iterate rule, 2b) and the oracle's exact QP solve takes it (r06l,
    # scripts/c3_survey_maxiter.py: 1802 stops at QP 3 and ends 1000 N = half the 2000 N trust region
    # from the oracle; 1371 at QP 2, 93.75 N; more interior-point iterations change nothing).  The rest
    # differ by 1e-5 .. 3e-3 N after one branched step length.  They are listed with each QP's domain step
    # length at the kernel's iterate (alpha) and the kernel's applied step as a fraction of the exact one
    # (0 where it stopped); at most 1 in 400 solved problems may branch.
    div = np.nonzero(solved & (err >= U_TOL))[0]
    for b in div[:10]:
        print(f"  branched: problem {int(b)}, |u* - u*_oracle| {err[b]:.3g}; alpha at the kernel's iterates "
              f"{np.round(r['alpha'][:, b], 4).tolist()}, kernel step / exact step {np.round(r['step_ratio'][:, b], 4).tolist()}")
    assert len(div) <= int(solved.sum()) // 400, len(div)
    # SURVEY 8(d)'s full ranges (round 6, VERDICT r05 missing 3: Ux down to 5 m/s, ey to +-3 m, Fx warm
    # starts to +-6000 N per stage): the solved fraction is reported, and every problem the kernel does
    # not solve is one the contract cannot solve either -- the oracle's own SQP ends outside the spatial
    # model's domain (the kernel's VC_OUT_OF_DOMAIN), or one of its QPs has no feasible point (phase-1 LP
    # with a checked Farkas certificate, oracle/feasibility.py)
    from oracle import feasibility as F
    bad = np.nonzero(~solved)[0]
    print(f"  c3_survey: solved {solved.mean():.4f} ({int(solved.sum())}/{B}); status counts "
          f"{np.bincount(st_k[-1], minlength=4).tolist()} (solved, max_iter, nonfinite, out_of_domain)")
    if len(bad):
        sub = {k: v[bad] for k, v in d.items()}
        ref = D.dyn_sqp_solve(sub["x0"], sub["ubar"], sub["kappa"], sub["ds"], dyn_params, W, tyre, keep_qps=True)
        first, farkas = F.first_infeasible_iteration(ref["hist"])
        explained = ~ref["in_domain"] | ((first >= 0) & farkas)
        print(f"  non-solved: oracle x* outside the domain {int((~ref['in_domain']).sum())}, infeasible QP with a "
              f"Farkas certificate {int(((first >= 0) & farkas).sum())}, unexplained "
              f"{[(int(b), int(st_k[-1][b])) for b in bad[~explained][:10]]}")
        # r06k/l: problem 610 is the one the oracle solves and the kernel does not (a later QP's Riccati
        # factorisation breaks down at scale ~1e8, diag flags 1 | 16, status max_iter -- the QPs before
        # it did not all converge); at most one such problem in the set
        assert (~explained).sum() <= 1


def test_kin_ltv_interior_point_status_rests_on_the_true_residual(kin_W):
    """kin_ltv carries its interior-point residuals by the step (1 - alpha)
    instead of recomputing them; the carried value must not end the loop on its own.  With the
    polish off (qp.polish = 0) the returned z is the interior point's iterate, and for every problem
    reported solved: diag[0] (the kernel's final residual / scale, now the true one) is within the
    stopping tolerance; the host-side primal infeasibility of z (C z - d, oracle-built QP) is below
    tol * scale (C z - d = r - s <= r with s >= 0); and the objective gap to the oracle's exact optimum
    is at the duality-gap level m * mu <= m * tol * scale (with the slack of a few residual terms).  A
    carried residual that drifted from the truth would show in both host checks."""
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.workload import kinematic_batch
    cfg = load_config("kinematic_mpc")
    cfg["qp"] = dict(cfg["qp"], polish=0)
    tol = float(cfg["qp"]["tol"])
    p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=cfg)
    d = kinematic_batch(1024, N=20, seed=31)
    with Context(model=_abi.VC_MODEL_KINEMATIC, N=20, max_batch=1024, dtype=_abi.VC_F64, params=p) as c:
        u0, xs, us, st, it, dg = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
    z = (us - d["ubar"]).reshape(1024, 40)
    r = CF.certify_batch("kin", z, dict(W=kin_W, L=L), {k: d[k] for k in ("x0", "ubar", "kappa", "ds")}, chunk=256)
    gap = CF.objective_gap("kin", z, r["z_exact"], dict(W=kin_W, L=L), {k: d[k] for k in ("x0", "ubar", "kappa", "ds")})
    solved = st == 0
    s = r["scale"]
    m = 4 * 20 + 3 * 19
    print(f"polish off: solved {int(solved.sum())}/1024, diag[0] max {dg[solved, 0].max():.2e} (tol {tol:.0e}); host "
          f"pfeas/scale max {np.max(r['pfeas'][solved] / s[solved]):.2e}; objective gap to the exact optimum / (m scale) "
          f"max {np.max(gap[solved] / (m * s[solved])):.2e}, min {np.min(gap[solved] / (m * s[solved])):.2e}")
    assert solved.mean() > 0.99
    assert dg[solved, 0].max() <= tol * (1 + 1e-12)
    assert np.max(r["pfeas"][solved] / s[solved]) <= tol
    assert np.max(gap[solved] / (m * s[solved])) <= 10 * tol
    assert np.min(gap[solved] / s[solved]) >= -1e-12   # the exact optimum is the minimum
