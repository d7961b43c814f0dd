"""CPU study of the kinematic polish's equality solve (csrc/kin_ltv.hip, phase 2): augmented-
Lagrangian passes (nu += R e, the shipped rule) against conjugate gradients on the same multiplier
system preconditioned with R (KIN_POLISH_CG), on the C2 workload's final active sets.  Counts the
triangular-solve pairs each needs to bring the active rows' violation below 1e-14 scale, from the
exact multipliers perturbed by a relative `eps` (the interior point's accuracy at its tolerance)
and from zero.
usage: python scripts/polish_cg_study.py [B] [eps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]
from oracle import ltv_qp as Q  # noqa: E402
from vcmpc.config import load_config  # noqa: E402
from vcmpc.workload import kinematic_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
eps = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-6
AL_RHO, MAXIT = float(os.environ.get("AL_RHO", "1e4")), 60
# NU_TOL > 0: the equality solve also runs until the multiplier step R e is below NU_TOL scale
NU_TOL = float(os.environ.get("NU_TOL", "0"))

d = kinematic_batch(B, seed=int(os.environ.get("SEED", "31")))
W = Q.kin_weights(load_config("kinematic_mpc"))
L = 2.5  # kinematic_car.yaml l
sol = Q.kin_ltv_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], L, W)
N = d["ubar"].shape[1]
n, nb = 2 * N, 4 * N
rng = np.random.default_rng(5)


def passes(H, g, C, dd, lam, mode, start):
    scale = 1.0 + max(np.abs(g).max(), np.abs(dd).max())
    hmax = max(np.diag(H).max(), 1.0)
    act = lam > 1e-12 * (1.0 + np.abs(lam).max())
    # box rows fix variables; state rows become equality rows of the free part
    fixed = np.zeros(n, bool)
    zfix = np.zeros(n)
    for r in np.where(act[:nb])[0]:
        i = np.argmax(np.abs(C[r]))
        fixed[i] = True
        zfix[i] = dd[r] * np.sign(C[r, i])
    rows = np.where(act[nb:])[0] + nb
    if len(rows) == 0:
        return 0, 0
    F = ~fixed
    Cf = C[rows][:, F]
    b = dd[rows] - C[rows][:, fixed] @ zfix[fixed]
    gf = g[F] + H[np.ix_(F, fixed)] @ zfix[fixed]
    rho = AL_RHO * hmax / (Cf ** 2).sum(1)
    M = H[np.ix_(F, F)] + Cf.T @ (rho[:, None] * Cf)
    Lc = np.linalg.cholesky(M)
    solve = lambda v: np.linalg.solve(Lc.T, np.linalg.solve(Lc, v))  # noqa: E731
    nu_star = lam[rows]
    nu = np.zeros_like(nu_star) if start == "zero" else nu_star * (1 + eps * rng.standard_normal(len(rows)))
    z = solve(-gf - Cf.T @ (nu - rho * b))
    e = Cf @ z - b
    k = 1
    if mode == "al":
        while np.abs(e).max() > 1e-14 * scale and k < MAXIT:
            nu = nu + rho * e
            z = solve(-gf - Cf.T @ (nu - rho * b))
            e = Cf @ z - b
            k += 1
    else:
        r = e.copy()
        p = rho * r
        rz = r @ p
        while np.abs(r).max() > 1e-14 * scale and k < MAXIT:
            zq = solve(Cf.T @ p)
            q = Cf @ zq
            al = rz / (p @ q)
            nu, z, r = nu + al * p, z - al * zq, r - al * q
            k += 1
            zt = rho * r
            rzn = r @ zt
            p, rz = zt + rzn / rz * p, rzn
        e = Cf @ z - b
    return k, len(rows), np.abs(e).max() / scale, np.abs(nu - nu_star).max() / (1 + np.abs(nu_star).max())


for start in ("ipm", "zero"):
    res = {}
    for mode in ("al", "cg"):
        out = [passes(sol["H"][i], sol["g"][i], sol["C"][i], sol["d"][i], sol["lam"][i], mode, start) for i in range(B)]
        res[mode] = [o for o in out if o[1] > 0]
    k_al = np.array([o[0] for o in res["al"]])
    k_cg = np.array([o[0] for o in res["cg"]])
    m = np.array([o[1] for o in res["al"]])
    print(f"start {start} (eps {eps:g}): {len(m)} of {B} problems with active state rows (rows mean {m.mean():.1f} max {m.max()})")
    print(f"  AL passes mean {k_al.mean():.2f} max {k_al.max()}   CG solves mean {k_cg.mean():.2f} max {k_cg.max()}")
    print(f"  final violation AL max {max(o[2] for o in res['al']):.1e} CG max {max(o[2] for o in res['cg']):.1e}; "
          f"multiplier error AL max {max(o[3] for o in res['al']):.1e} CG max {max(o[3] for o in res['cg']):.1e}")
    worst = np.argsort(k_al)[::-1][:5]
    print("  worst AL problems (AL passes / CG solves / rows):", [(int(k_al[j]), int(k_cg[j]), int(m[j])) for j in worst])


# ---- the kernel's whole polish from the interior point's own guess (lambda > s at tol 1e-10):
# rounds of one active-set change, each with its equality solve by AL passes or CG (<= 16 solves)
from oracle.qp import pdip_batch  # noqa: E402

tol = float(os.environ.get("IPM_TOL", "1e-10"))
zi, lami, si, iti, *_ = pdip_batch(sol["H"], sol["g"], sol["C"], sol["d"], tol=tol)
# the iterate one interior-point step before the last (same deterministic iteration, stopped early)
lamp, sp = np.zeros_like(lami), np.zeros_like(si)
for kk in np.unique(iti):
    sel = iti == kk
    _, l1, s1, *_ = pdip_batch(sol["H"][sel], sol["g"][sel], sol["C"][sel], sol["d"][sel], tol=tol, max_iter=int(kk) - 1)
    lamp[sel], sp[sel] = l1, s1
exact = sol["lam"] > 1e-12 * (1 + np.abs(sol["lam"]).max(1, keepdims=True))
guesses = {"lam > s": lami > si,
           # Tapia indicators (El-Bakry, Tapia, Zhang 1994): an active row's slack goes to zero
           # superlinearly while its multiplier settles; an inactive row's the other way round
           "tapia": (lami / lamp) > (si / sp)}
# Tapia where the last step decides it (ratios a factor TF apart), lambda > s where it does not
# (a step that barely moved either leaves both ratios at 1)
lr, sr = lami / lamp, si / sp
for TF in [float(x) for x in os.environ.get("TAPIA_F", "1.5,2,4").split(",")]:
    guesses[f"hyb{TF:g}"] = np.where(lr > TF * sr, True, np.where(sr > TF * lr, False, lami > si))
# strict indicators: a side is called active only if its multiplier held (ratio >= 1 - TS) while its
# slack dropped (ratio <= TS), inactive the other way round; lambda > s otherwise
for TS in [float(x) for x in os.environ.get("TAPIA_S", "").split(",") if x]:
    guesses[f"strict{TS:g}"] = np.where((lr >= 1 - TS) & (sr <= TS), True, np.where((sr >= 1 - TS) & (lr <= TS), False, lami > si))
for name, act in guesses.items():
    wrong = (act != exact).sum(1)
    print(f"guess {name:8s}: problems with a misclassified row {int((wrong > 0).sum())} of {B}, rows {int(wrong.sum())}")


def polish_sim(H, g, C, dd, lam, s, mode, rounds_max=10, act0=None, zx=None):
    scale = 1.0 + max(np.abs(g).max(), np.abs(dd).max())
    hmax = max(np.diag(H).max(), 1.0)
    ptol = 1e-9 * scale
    act = (lam > s) if act0 is None else act0.copy()
    total = 0
    for rnd in range(rounds_max):
        fixed = np.zeros(n, bool)
        zfix = np.zeros(n)
        for r in np.where(act[:nb])[0]:
            i = np.argmax(np.abs(C[r]))
            fixed[i] = True
            zfix[i] = dd[r] * np.sign(C[r, i])
        rows = np.where(act[nb:])[0] + nb
        F = ~fixed
        Cf = C[rows][:, F]
        b = dd[rows] - C[rows][:, fixed] @ zfix[fixed]
        gf = g[F] + H[np.ix_(F, fixed)] @ zfix[fixed]
        rho = AL_RHO * hmax / np.maximum((Cf ** 2).sum(1), 1e-300)
        M = H[np.ix_(F, F)] + Cf.T @ (rho[:, None] * Cf)
        Lc = np.linalg.cholesky(M)
        solve = lambda v: np.linalg.solve(Lc.T, np.linalg.solve(Lc, v))  # noqa: E731
        nu = lam[rows].copy()
        z = solve(-gf - Cf.T @ (nu - rho * b))
        e = Cf @ z - b
        k = 1
        if len(rows):
            if mode == "al":
                while (np.abs(e).max() > 1e-14 * scale or np.abs(rho * e).max() > NU_TOL * scale) and k < 16:
                    nu = nu + rho * e
                    z = solve(-gf - Cf.T @ (nu - rho * b))
                    e = Cf @ z - b
                    k += 1
            else:
                r = e.copy()
                p = rho * r
                rz = r @ p
                while (np.abs(r).max() > 1e-14 * scale or np.abs(rho * r).max() > NU_TOL * scale) and k < 16:
                    zq = solve(Cf.T @ p)
                    q = Cf @ zq
                    pq = p @ q
                    if not pq > 0:
                        break
                    al = rz / pq
                    nu, z, r = nu + al * p, z - al * zq, r - al * q
                    k += 1
                    zt = rho * r
                    rzn = r @ zt
                    p, rz = zt + rzn / rz * p, rzn
                e = Cf @ z - b
        total += k
        zp = zfix.copy()
        zp[F] = z
        lamf = np.zeros(len(dd))
        lamf[rows] = nu
        grad = H @ zp + g + C[nb:].T @ lamf[nb:]
        # box multipliers from the gradient (active box rows), state-row multipliers nu
        for r in np.where(act[:nb])[0]:
            i = np.argmax(np.abs(C[r]))
            lamf[r] = -grad[i] * np.sign(C[r, i])
        dv = np.where(act, -lamf, -np.inf)
        pv = np.where(act, -np.inf, C @ zp - dd)
        if dv.max() <= ptol and pv.max() <= ptol:
            ok = np.abs(e).max() <= ptol if len(rows) else True
            return rnd + 1, total, ok, np.abs(zp - zx).max() if (ok and zx is not None) else 0.0
        if dv.max() > ptol:
            act[np.argmax(dv)] = False
        else:
            act[np.argmax(pv)] = True
    return rounds_max, total, False, 0.0


for gname, mode in [("lam > s", "al"), ("lam > s", "cg"), ("tapia", "cg")] + [(k, "cg") for k in guesses if k.startswith(("hyb", "strict"))]:
    out = np.array([polish_sim(sol["H"][i], sol["g"][i], sol["C"][i], sol["d"][i], lami[i], si[i], mode,
                               act0=guesses[gname][i], zx=sol["z"][i]) for i in range(B)])
    print(f"polish from the interior point at tol {tol:g} [{gname}, {mode}]: rounds mean {out[:, 0].mean():.2f} max {out[:, 0].max():.0f}, "
          f"solves mean {out[:, 1].mean():.2f} max {out[:, 1].max():.0f}, certified {out[:, 2].mean():.3f}, "
          f"certified but |z - z*| > 1e-6: {int((out[:, 3] > 1e-6).sum())} (max {out[:, 3].max():.1e})")
    worst = np.argsort(out[:, 1])[::-1][:6]
    print("  most solves (problem, rounds, solves):", [(int(j), int(out[j, 0]), int(out[j, 1])) for j in worst])
