"""Certification diagnostics on the GPU box: solve a bench-size set, certify every answer against
the oracle-built QP (oracle/certify.py), and dump the worst problems (inputs, kernel answer,
diag flags, oracle optimum) to gpurun_out/cert_<set>.npz for study on the CPU.

    python scripts/cert_diag.py c4_bench [--solver 0] [--top 20]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd"), os.path.join(ROOT, "tests")]


def main():
    from oracle import certify as CF
    from oracle import ltv_qp as Q
    from test_gpu_certify import _kin_ctx, _kin_set
    from vcmpc.config import load_config
    ap = argparse.ArgumentParser()
    ap.add_argument("set")
    ap.add_argument("--solver", type=int, default=0)
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    N, d = _kin_set(a.set)
    B = len(d["x0"])
    W = Q.kin_weights(load_config("kinematic_mpc"))
    with _kin_ctx(N, B, a.solver) as c:
        u0, xs, us, st, it, dg = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
    z = (us - d["ubar"]).reshape(B, 2 * N)
    r = CF.certify_batch("kin", z, dict(W=W, L=2.5), {k: d[k] for k in ("x0", "ubar", "kappa", "ds")}, chunk=2048)
    err = np.abs(z - r["z_exact"]).max(axis=1)
    order = np.argsort(-err)[:a.top]
    flags = dg[:, 2].astype(int)
    print(f"{a.set}: B={B}, solved {(st == 0).mean():.5f}; err > 1e-5: {int((err > 1e-5).sum())}, > 1e-7: "
          f"{int((err > 1e-7).sum())}; flags histogram {dict(zip(*np.unique(flags, return_counts=True)))}")
    print("unpolished solved problems:", int(((flags & 4) == 0).sum()), " their max err", float(err[(flags & 4) == 0].max(initial=0)))
    for b in order:
        print(f"  {int(b)}: err {err[b]:.3e} stat/scale {r['stat'][b] / r['scale'][b]:.2e} status {st[b]} iters {it[b]} "
              f"diag res {dg[b, 0]:.2e} mu {dg[b, 1]:.2e} flags {flags[b]} rounds {int(dg[b, 3])} nact {r['nact'][b]}")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", f"cert_{a.set}.npz"), idx=order, err=err[order],
             z=z[order], z_exact=r["z_exact"][order], diag=dg[order], iters=it[order], status=st[order],
             **{k: d[k][order] for k in ("x0", "ubar", "kappa", "ds")})


if __name__ == "__main__":
    main()
