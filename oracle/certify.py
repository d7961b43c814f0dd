"""KKT certificates of the kernels' answers over whole batches (TEST INFRASTRUCTURE ONLY).

Only tests/ may import this module.  It never runs inside the product path.

Every QP the build solves is strictly convex: the proximal term prox ||dz||^2 makes H positive
definite.  So a point z that satisfies the KKT conditions of the oracle-built QP

    stat  = ||H z + g + C' lam||_inf      (stationarity)
    pfeas = max(C z - d)_+               (primal feasibility)
    dfeas = max(-lam)_+                  (dual feasibility)
    comp  = max |lam_i (d_i - C_i z)|    (complementarity)

to rounding level IS the unique optimum.  The kernels do not return multipliers, so they are
recovered here.  The rows with slack <= act_tol * scale are the candidate active set A.  lam_A
is the nonnegative least-squares solution of C_A' lam = -(H z + g) (scipy.optimize.nnls, one
problem at a time).  Then all four residuals are computed.  This checks the kernel's own claim
of optimality independently of its certificate.  The round-4 early polish certified C4 problem
23921 9e-3 off the optimum: its stationarity residual here is ~1e-1, not ~1e-12.

The oracle's exact answer to the same QP comes from oracle/qp.py's active-set polish (equality-
constrained KKT solves, accepted only when primal and dual feasible to 1e-12).  It is seeded
with the active set the multipliers above identify.  The seed only saves active-set changes.
The polish result is certified on its own, and the optimum is unique, so the answer does not
depend on the seed.  A polish that does not certify falls back to the oracle's full interior
point (pdip_batch) on that problem.  The tests also run the fully independent oracle
(pdip_batch + polish from z = 0) on a strided sample, and require the two to agree.

Batches are cut into chunks that a process pool works through ("spawn": the workers never see
the parent's HIP state).  The QP data of a chunk are built by the oracle restatements
(ltv_qp.kin_qp, dyn_sqp.dyn_qp, casc_sqp.casc_qp) in the worker.
"""
from __future__ import annotations

import os

import numpy as np

ACT_TOL = 1e-7      # candidate active rows: slack <= ACT_TOL * scale
CHUNK = 1024


def qp_scale(g, d):
    """The interior point's scale (oracle/qp.py pdip_batch; the kernels use the same rule)."""
    return 1.0 + np.maximum(np.abs(g).max(axis=1), np.abs(d).max(axis=1))


def certify(H, g, C, d, z, act_tol=ACT_TOL):
    """KKT residuals of z[B, n] for the QPs (H, g, C, d), multipliers recovered by NNLS.
    Returns dict of [B] arrays stat, pfeas, dfeas, comp, scale, nact and lam[B, m]."""
    from scipy.optimize import nnls

    H, g, C, d, z = (np.asarray(a, np.float64) for a in (H, g, C, d, z))
    B, m = d.shape
    scale = qp_scale(g, d)
    r = np.einsum("bij,bj->bi", H, z) + g
    slack = d - np.einsum("bmi,bi->bm", C, z)
    lam = np.zeros((B, m))
    stat = np.abs(r).max(axis=1)
    nact = np.zeros(B, np.int64)
    for b in range(B):
        if not np.isfinite(z[b]).all():
            stat[b] = np.inf
            continue
        act = np.nonzero(slack[b] <= act_tol * scale[b])[0]
        nact[b] = len(act)
        if len(act) == 0:
            continue
        M = C[b, act].T
        la, _ = nnls(M, -r[b], maxiter=50 * M.shape[1] + 100)
        lam[b, act] = la
        stat[b] = np.abs(r[b] + M @ la).max()
    pfeas = np.maximum(-slack, 0.0).max(axis=1)
    dfeas = np.maximum(-lam, 0.0).max(axis=1)
    comp = np.abs(lam * slack).max(axis=1)
    return dict(stat=stat, pfeas=pfeas, dfeas=dfeas, comp=comp, scale=scale, nact=nact, lam=lam)


def kkt_ok(cert, tol=1e-9):
    """[B] every residual of the certificate within tol * scale."""
    lim = tol * cert["scale"]
    return ((cert["stat"] <= lim) & (cert["pfeas"] <= lim) & (cert["dfeas"] <= lim) & (cert["comp"] <= lim))


def exact(H, g, C, d, seed_lam=None, seed_z=None):
    """The oracle's exact optimum of each QP (oracle/qp.py): the active-set polish seeded with
    the rows where seed_lam > 0, or the full interior point + polish where that does not
    certify.  Returns z[B, n], ok[B] (certified by the polish's own KKT test), how[B]
    (0 seeded polish, 1 interior point + polish, -1 none)."""
    from .qp import pdip_batch, polish

    H, g, C, d = (np.asarray(a, np.float64) for a in (H, g, C, d))
    B, n = g.shape
    z = np.zeros((B, n))
    ok = np.zeros(B, bool)
    how = np.full(B, -1, np.int64)
    todo = []
    for b in range(B):
        if seed_lam is None:
            todo.append(b)
            continue
        # lam > s picks the seed rows: seeded rows get s = 0, lam = 1
        act = seed_lam[b] > 0.0
        zs = seed_z[b] if seed_z is not None else np.zeros(n)
        zp, _, good = polish(H[b], g[b], C[b], d[b], zs, act.astype(np.float64), np.zeros(len(act)))
        if good:
            z[b], ok[b], how[b] = zp, True, 0
        else:
            todo.append(b)
    if todo:
        idx = np.array(todo)
        zi, lam, s, _, done, _ = pdip_batch(H[idx], g[idx], C[idx], d[idx], tol=1e-13)
        for j, b in enumerate(idx):
            zp, _, good = polish(H[b], g[b], C[b], d[b], zi[j], lam[j], s[j])
            z[b], ok[b] = (zp, True) if good else (zi[j], bool(done[j]))
            how[b] = 1 if ok[b] else -1
    return z, ok, how


# ---- process pool ------------------------------------------------------------------------
def workers():
    """Single-threaded worker processes to use: the box's per-GPU CPU share (OMP_NUM_THREADS,
    16 on the GPU boxes, whose affinity shows the whole machine), else the affinity mask."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    n = min(aff, int(omp)) if omp.isdigit() and int(omp) > 0 else aff
    return max(1, min(n, 16))


def pool_map(fn, jobs, nproc=None):
    """map(fn, jobs) over a spawned process pool (serial for one job or one worker)."""
    nproc = workers() if nproc is None else nproc
    if nproc <= 1 or len(jobs) <= 1:
        return [fn(j) for j in jobs]
    import multiprocessing as mp
    with mp.get_context("spawn").Pool(min(nproc, len(jobs))) as pool:
        return pool.map(fn, jobs, chunksize=1)


def _limit_threads():
    try:
        from threadpoolctl import threadpool_limits
        return threadpool_limits(limits=1)
    except ImportError:  # pragma: no cover
        import contextlib
        return contextlib.nullcontext()


def _qp_data(job):
    kind = job["kind"]
    if kind == "kin":
        from . import ltv_qp as Q
        D = Q.kin_qp(job["x0"], job["ubar"], job["kappa"], job["ds"], job["L"], job["W"], x_ws=job.get("x_ws"))
    elif kind == "dyn":
        from . import dyn_sqp as DS
        D = DS.dyn_qp(job["x0"], job["ubar"], job["kappa"], job["ds"], job["p"], job["W"], job["tyre"])
    elif kind == "casc":
        from . import casc_sqp as CS
        D = CS.casc_qp(job["x0"], job["ubar"], job["kappa"], job["ds"], job["p"], job["W"], job["tyre"])
    else:
        raise ValueError(kind)
    return D["H"], D["g"], D["C"], D["d"]


def _chunk_worker(job):
    """One chunk: build the QPs at job's ubar, certify job['z'] and compute the oracle's exact
    optimum (seeded by the certificate's multipliers); without job['z'] the unseeded oracle."""
    with _limit_threads():
        H, g, C, d = _qp_data(job)
        out = {}
        if job.get("z") is not None:
            cert = certify(H, g, C, d, job["z"])
            zx, okx, how = exact(H, g, C, d, seed_lam=cert["lam"], seed_z=job["z"])
            out.update({k: cert[k] for k in ("stat", "pfeas", "dfeas", "comp", "scale", "nact")})
        else:
            zx, okx, how = exact(H, g, C, d)
        out.update(z_exact=zx, exact_ok=okx, exact_how=how)
        return out


def sqp_scale(kind, H_, N):
    """[H_, 2] physical units per unit of the QP variable dz: Fx / S on every stage, and Fy / S
    on the cascaded point-mass stages (oracle/dyn_sqp.py step 3, casc_sqp.py step 3)."""
    sc = np.ones((H_, 2))
    sc[:, 0] = 1000.0
    if kind == "casc":
        sc[N:, 1] = 1000.0
    return sc


def _predictor(job):
    if job["kind"] == "dyn":
        from . import dyn_sqp as DS
        return DS.dyn_predict, None
    from . import casc_sqp as CS
    W = job["W"]
    return (lambda x0_, u_, k_, ds_, p_, t_: CS.casc_predict(x0_, u_, k_, ds_, p_, W, t_)), CS.casc_in_domain


def _sqp_worker(job):
    """One chunk of an SQP batch (dyn / casc).  job['us'] = the kernel's iterates [K+1, B, H, 2]
    (u_0 = the warm start, u_k = the kernel run with sqp_iters = k), job['stop'] [K, B] = the
    kernel stopped the SQP at QP k (diag bit 16 of the k-run).

    For every k: the QP at the kernel's u_{k-1} is built by the oracle, its exact optimum dz_o
    computed, the step length alpha of the contract's domain test (oracle/dyn_sqp.py
    domain_step) taken at dz_o, and the kernel's step dz_k = (u_k - u_{k-1}) / (alpha scale)
    certified.  Then the oracle's own SQP is run: the QPs at ITS iterates, solved exactly (seeded
    by the kernel's active sets), with the same domain and stopping rules (dyn_sqp_solve /
    casc_sqp_solve); u_oracle = its last iterate."""
    from .dyn_sqp import domain_step
    with _limit_threads():
        us, stop = job["us"], job["stop"]
        K = us.shape[0] - 1
        B, H_ = us.shape[1], us.shape[2]
        N = job["W"].get("N", H_)
        sc = sqp_scale(job["kind"], H_, N)
        predict, in_dom = _predictor(job)
        x0, kap, ds = (np.asarray(job[k], np.float64) for k in ("x0", "kappa", "ds"))
        p, tyre = job["p"], job["tyre"]
        out = {k: np.zeros((K, B)) for k in ("stat", "pfeas", "dfeas", "comp", "scale", "alpha", "dz_err", "f_k", "f_o",
                                             "f_mag")}
        out["refused_both"] = np.zeros((K, B), bool)
        out["step_ratio"] = np.zeros((K, B))
        out["exact_ok"] = np.zeros((K, B), bool)
        uo = np.array(us[0], np.float64, copy=True)
        stopped_o = np.zeros(B, bool)
        for k in range(1, K + 1):
            # (a) the kernel's k-th QP, at the kernel's own iterate
            jk = dict(job, ubar=us[k - 1])
            H, g, C, d = _qp_data(jk)
            # seeded: certify the full step first (alpha = 1 is the rule), its multipliers seed the oracle
            z1 = ((us[k] - us[k - 1]) / sc).reshape(B, -1)
            cert1 = certify(H, g, C, d, z1)
            dz_o, ok_o, _ = exact(H, g, C, d, seed_lam=cert1["lam"], seed_z=z1)
            du_o = dz_o.reshape(B, H_, 2) * sc
            alpha = domain_step(x0, us[k - 1], du_o, kap, ds, p, tyre, predict, in_domain=in_dom)
            with np.errstate(divide="ignore", invalid="ignore"):
                zk = np.where(alpha[:, None] > 0, z1 / np.where(alpha > 0, alpha, 1.0)[:, None], z1)
            cert = certify(H, g, C, d, zk)
            for key in ("stat", "pfeas", "dfeas", "comp", "scale"):
                out[key][k - 1] = cert[key]
            out["alpha"][k - 1] = alpha
            out["exact_ok"][k - 1] = ok_o
            out["dz_err"][k - 1] = np.abs(zk - dz_o).max(axis=1)
            # the QP objective 1/2 z'Hz + g'z at the kernel's step and at the oracle's optimum, and the
            # magnitude of its terms at the optimum (what fp64 rounding of f is relative to)
            hz = np.einsum("bij,bj->bi", H, dz_o)
            out["f_k"][k - 1] = 0.5 * np.einsum("bi,bij,bj->b", zk, H, zk) + np.einsum("bi,bi->b", g, zk)
            out["f_o"][k - 1] = 0.5 * np.einsum("bi,bi->b", dz_o, hz) + np.einsum("bi,bi->b", g, dz_o)
            out["f_mag"][k - 1] = 0.5 * np.einsum("bi,bij,bj->b", np.abs(dz_o), np.abs(H), np.abs(dz_o)) + \
                np.einsum("bi,bi->b", np.abs(g), np.abs(dz_o))
            # no step length keeps the rollout in the domain for the oracle's step (alpha = 0) and the
            # kernel took none either: that QP's answer is not applied by the contract
            out["refused_both"][k - 1] = (alpha == 0) & (np.abs(z1).max(axis=1) == 0)
            # the kernel's applied step against the oracle's optimum of the same QP, as a step length:
            # |z1|_inf / |dz_o|_inf (1 = full step, 1/2^j a cut-back; compared with alpha, the domain test's)
            with np.errstate(divide="ignore", invalid="ignore"):
                out["step_ratio"][k - 1] = np.abs(z1).max(axis=1) / np.abs(dz_o).max(axis=1)
            # (b) the oracle's own SQP iterate
            if k == 1:
                zo, oko = dz_o, ok_o
            else:
                Ho, go, Co, do = _qp_data(dict(job, ubar=uo))
                co = certify(Ho, go, Co, do, zk)
                zo, oko, _ = exact(Ho, go, Co, do, seed_lam=co["lam"], seed_z=zk)
                stopped_o |= ~oko
            zo = np.where(stopped_o[:, None], 0.0, zo)
            duo = zo.reshape(B, H_, 2) * sc
            ao = domain_step(x0, uo, duo, kap, ds, p, tyre, predict, in_domain=in_dom)
            uo = np.where(((ao > 0) & ~stopped_o)[:, None, None], uo + ao[:, None, None] * duo, uo)
        out["u_oracle"] = uo
        out["stopped_oracle"] = stopped_o
        return out


def _gap_worker(job):
    with _limit_threads():
        H, g, C, d = _qp_data(job)
        q = lambda z: 0.5 * np.einsum("bi,bij,bj->b", z, H, z) + np.einsum("bi,bi->b", g, z)
        return q(job["z"]) - q(job["z_ref"])


def objective_gap(kind, z, z_ref, common, per_problem, chunk=CHUNK, nproc=None):
    """[B] q(z) - q(z_ref) of the oracle-built QPs (q = 1/2 z'Hz + g'z)."""
    B = len(z)
    jobs = []
    for lo in range(0, B, chunk):
        hi = min(B, lo + chunk)
        j = dict(common, kind=kind, z=np.ascontiguousarray(z[lo:hi]), z_ref=np.ascontiguousarray(z_ref[lo:hi]))
        j.update({k: np.ascontiguousarray(v[lo:hi]) for k, v in per_problem.items()})
        jobs.append(j)
    return np.concatenate(pool_map(_gap_worker, jobs, nproc))


def certify_sqp_batch(kind, us, stop, common, per_problem, chunk=256, nproc=None):
    """certify every QP of an SQP batch (see _sqp_worker); us [K+1, B, H, 2], stop [K, B]."""
    B = us.shape[1]
    jobs = []
    for lo in range(0, B, chunk):
        hi = min(B, lo + chunk)
        j = dict(common, kind=kind, us=np.ascontiguousarray(us[:, lo:hi]), stop=np.ascontiguousarray(stop[:, lo:hi]))
        j.update({k: np.ascontiguousarray(v[lo:hi]) for k, v in per_problem.items()})
        jobs.append(j)
    res = pool_map(_sqp_worker, jobs, nproc)
    out = {}
    for k in res[0]:
        ax = 0 if res[0][k].ndim == 1 or k == "u_oracle" or k == "stopped_oracle" else 1
        out[k] = np.concatenate([r[k] for r in res], axis=ax)
    return out


def certify_batch(kind, z, common, per_problem, chunk=CHUNK, nproc=None, independent_every=0):
    """Certify z[B, n] against the QPs built from per_problem arrays (dict of [B, ...]) and
    common settings (W, L / p, tyre).  independent_every = k > 0: the unseeded oracle also runs
    on every k-th problem.  Returns dict of [B] arrays (see _chunk_worker; z_indep / indep_ok
    only on the sampled problems, index array `indep_idx`)."""
    B = len(z) if z is not None else len(next(iter(per_problem.values())))
    jobs = []
    for lo in range(0, B, chunk):
        hi = min(B, lo + chunk)
        j = dict(common, kind=kind, z=None if z is None else np.ascontiguousarray(z[lo:hi]))
        j.update({k: np.ascontiguousarray(v[lo:hi]) for k, v in per_problem.items()})
        jobs.append(j)
    res = pool_map(_chunk_worker, jobs, nproc)
    out = {k: np.concatenate([r[k] for r in res]) for k in res[0] if k not in ("z_indep", "indep_ok")}
    if independent_every > 0:
        idx = np.arange(0, B, independent_every)
        sub = {k: np.ascontiguousarray(v[idx]) for k, v in per_problem.items()}
        ij = []
        for lo in range(0, len(idx), max(1, chunk // 4)):
            hi = min(len(idx), lo + max(1, chunk // 4))
            j = dict(common, kind=kind, z=None)
            j.update({k: v[lo:hi] for k, v in sub.items()})
            ij.append(j)
        r2 = pool_map(_chunk_worker, ij, nproc)
        out["indep_idx"] = idx
        out["z_indep"] = np.concatenate([r["z_exact"] for r in r2])
        out["indep_ok"] = np.concatenate([r["exact_ok"] for r in r2])
    return out
