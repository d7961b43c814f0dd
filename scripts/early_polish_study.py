"""CPU cost model of trying the kinematic polish before the interior point's final tolerance
(csrc/kin_ltv.hip): for each C2 problem, the interior-point iterations to reach tol T, whether the
polish (Tapia/lambda > s first guess, CG equality solves, scripts/polish_cg_study.py) certifies from
there within R rounds, and the resulting cycle estimate with the measured section costs
(profiles/r04/sec_r04r.txt); a failed attempt resumes the interior point to the final tolerance.
usage: python scripts/early_polish_study.py [B] [R]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("TAPIA_F", "1.02")
os.environ.setdefault("NU_TOL", "1e-10")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
R = int(sys.argv[2]) if len(sys.argv) > 2 else 2
src = open(os.path.join(ROOT, "scripts", "polish_cg_study.py")).read().split("for start in")[0]
g = {"__file__": os.path.join(ROOT, "scripts", "polish_cg_study.py")}
sys.argv = ["x", str(B)]
exec(compile(src, "study", "exec"), g)
src2 = open(os.path.join(ROOT, "scripts", "polish_cg_study.py")).read()
exec(src2[src2.index("def polish_sim"):src2.index("for gname, mode")], g)
from oracle.qp import pdip_batch  # noqa: E402

sol, polish_sim = g["sol"], g["polish_sim"]
H, gg, C, d = sol["H"], sol["g"], sol["C"], sol["d"]
C_IT, C_FIX, C_ROUND, C_SOLVE = 23.4e3, 55e3, 19.5e3, 5.2e3


def state_at(tol):
    z, lam, s, it, *_ = pdip_batch(H, gg, C, d, tol=tol)
    lp, sp = np.zeros_like(lam), np.zeros_like(s)
    for k in np.unique(it):
        sel = it == k
        _, l1, s1, *_ = pdip_batch(H[sel], gg[sel], C[sel], d[sel], tol=tol, max_iter=int(k) - 1)
        lp[sel], sp[sel] = l1, s1
    lr, sr = lam / lp, s / sp
    act = np.where(lr > 1.02 * sr, True, np.where(sr > 1.02 * lr, False, lam > s))
    out = np.array([polish_sim(H[i], gg[i], C[i], d[i], lam[i], s[i], "cg", rounds_max=R, act0=act[i]) for i in range(B)])
    return it, out


it_f, pol_f = state_at(1e-10)
base = C_FIX + it_f * C_IT + pol_f[:, 0] * C_ROUND + pol_f[:, 1] * C_SOLVE
print(f"final tol 1e-10: iters mean {it_f.mean():.2f} max {it_f.max()}, certified {pol_f[:, 2].mean():.4f}, "
      f"model cycles mean {base.mean():.0f} max {base.max():.0f}")
for T in (3e-10, 1e-9, 3e-9, 1e-8, 3e-8, 1e-7):
    it_T, pol_T = state_at(T)
    ok = pol_T[:, 2].astype(bool)
    cost = np.where(ok, C_FIX + it_T * C_IT + pol_T[:, 0] * C_ROUND + pol_T[:, 1] * C_SOLVE,
                    C_FIX + it_f * C_IT + (pol_T[:, 0] + pol_f[:, 0]) * C_ROUND + (pol_T[:, 1] + pol_f[:, 1]) * C_SOLVE)
    print(f"try at {T:g}: iters there mean {it_T.mean():.2f} max {it_T.max()}, certified {ok.mean():.4f} "
          f"(rounds <= {R}), model cycles mean {cost.mean():.0f} max {cost.max():.0f} "
          f"({100 * (cost.max() / base.max() - 1):+.1f} % max, {100 * (cost.mean() / base.mean() - 1):+.1f} % mean)")
    top = np.argsort(cost)[::-1][:4]
    print("    costliest (problem, iters at T, certified at T, iters final, cycles):",
          [(int(b), int(it_T[b]), bool(ok[b]), int(it_f[b]), int(cost[b])) for b in top])
