"""CPU replay of the kinematic obstacle loop's non-solved steps (captured on the GPU by
scripts/kin_lost_capture.py): for each lost / failing vehicle, its failing steps' first QP is
rebuilt with the oracle (oracle/ltv_qp.py kin_qp, multiple shooting at the captured warm start)
and its constraint set decided by a phase-1 LP (oracle/feasibility.py) -- with the controller's
trust region and without it -- and the state iterate that the step linearises at is summarised
(delta / v of the plan and of its defect rollout, eps range, the first-stage defect).

    python scripts/kin_lost_replay.py gpurun_out/kin_lost/seed5_N50.npz [--max 6]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--max", type=int, default=6)
    ap.add_argument("--sqp", action="store_true", help="also run the oracle SQP step (10 iterations)")
    a = ap.parse_args()
    from oracle import feasibility as FE
    from oracle import kin_sqp as KS
    from oracle import ltv_qp as Q
    from vcmpc.config import load_config
    from vcmpc.controllers.kinematic_mpc import kin_qp_block
    from vcmpc.environment import Track
    tr = Track.load("ippodromo")
    obs = [(o.s, o.ey, o.radius) for o in tr.obstacles]
    for f in a.files:
        z = np.load(f)
        N = int(z["N"])
        cfg = load_config("kinematic_mpc")
        cfg["obstacles"] = True
        cfg["horizon"] = N
        qp = kin_qp_block(cfg)
        W = Q.kin_weights(cfg)
        W.update(trust_a=qp["trust_a"], trust_w=qp["trust_w"])
        W["obstacles"] = obs
        Wn = dict(W, trust_a=0.0, trust_w=0.0)
        print(f"== {f}: seed {int(z['seed'])}, N {N}, qp {qp}")
        for j, b in enumerate(z["vehicles"]):
            fails = np.nonzero(z["FAIL"][:, j])[0]
            ey = z["X"][:, j, 3]
            print(f"-- vehicle {b}: {len(fails)} non-solved, max |ey| {np.abs(ey).max():.2f}, "
                  f"first failing steps {fails[:12].tolist()}")
            for k in fails[:a.max]:
                x0 = z["X"][k, j][None]
                ub = z["UB"][k, j][None]
                xb = z["XB"][k, j][None]
                kap, ds = z["KAP"][k, j][None], z["DS"][k, j][None]
                qd = Q.kin_qp(x0, ub, kap, ds, 2.5, W, x_ws=xb)
                qn = Q.kin_qp(x0, ub, kap, ds, 2.5, Wn, x_ws=xb)
                p_tr = FE.phase1(qd["C"][0], qd["d"][0])
                p_nt = FE.phase1(qn["C"][0], qn["d"][0])
                xv = (qd["xbar"] + qd["e"])[0]
                blocking = ""
                if not p_tr["feasible"] and p_tr["y"] is not None:
                    y = p_tr["y"]
                    top = np.argsort(y)[-4:][::-1]
                    m_in = 4 * N
                    names = []
                    for r in top:
                        if y[r] <= 0:
                            continue
                        if r < m_in:
                            names.append(f"u{r // 4}{'aaww'[r % 4]}{'+-+-'[r % 4]}")
                        else:
                            kk, t = divmod(r - m_in, 3)
                            names.append(f"x{kk + 1}{['v>=', 'd<=', 'd>='][t]}")
                    blocking = " blocking rows " + ",".join(names)
                print(f"   step {k:3d}: x0 v {x0[0, 0]:.2f} d {x0[0, 1]:+.3f} s {x0[0, 2]:.1f} ey {x0[0, 3]:+.2f} "
                      f"ep {x0[0, 4]:+.3f} | plan d [{xb[0, 1:, 1].min():+.3f},{xb[0, 1:, 1].max():+.3f}] "
                      f"ep [{xb[0, :, 4].min():+.2f},{xb[0, :, 4].max():+.2f}] | x+e d [{xv[1:, 1].min():+.3f},"
                      f"{xv[1:, 1].max():+.3f}] | e1 {np.abs(qd['e'][0, 1]).max():.2e} | feasible: trust "
                      f"{p_tr['feasible']} (t {p_tr['t']:.2e}), no trust {p_nt['feasible']} (t {p_nt['t']:.2e})"
                      + blocking)
                if a.sqp:
                    r = KS.kin_sqp_solve(x0, ub, kap, ds, 2.5, W, 10, x_ws=xb)
                    print("      oracle SQP: alpha", [float(h["alpha"][0]) for h in r["hist"]],
                          "qp_ok", [bool(h["qp_ok"][0]) for h in r["hist"]],
                          "restart", bool(r["hist"][0].get("restart", [False])[0]))


if __name__ == "__main__":
    main()
