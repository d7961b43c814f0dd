"""The C3 survey-range problems whose first QP the certificate did not certify (r06f,
tests/test_gpu_certify.py::test_sqp_batch_every_qp_certified[c3_survey]): the kernel's first
step against the oracle's exact optimum of the same QP, the step lengths each rollout allows
(oracle/dyn_sqp.py domain_step) and the QP objective at each point.

    python scripts/c3_survey_cert_diag.py [--probs 1106 1201 ...] [--out f.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vehicle-control_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--probs", type=int, nargs="*", default=None, help="problem indices (default: all, report the uncertified)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from oracle import certify as CF
    from oracle import dyn_sqp as D
    from oracle import models as M
    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.workload import dynamic_batch

    B = 4096
    d = {k: v.astype(np.float64) for k, v in dynamic_batch(B, N=40, seed=31, ranges="survey").items()}
    cfg = load_config("dynamic_mpc")
    ck = dict(cfg, qp=dict(cfg["qp"], sqp_iters=1))
    p = M.dyn_params_from_config(load_config("dynamic_car"))
    params = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=ck, tyre="linear")
    with Context(model=_abi.VC_MODEL_DYNAMIC, N=40, max_batch=B, dtype=_abi.VC_F64, params=params) as c:
        u0, xs, u1, st, it, dg = c.solve(d["x0"], d["kappa"], d["ds"], d["ubar"].copy(), diag=True)
    idx = np.arange(B) if args.probs is None else np.array(args.probs)
    W = D.dyn_weights(cfg)
    sub = {k: v[idx] for k, v in d.items()}
    Q = D.dyn_qp(sub["x0"], sub["ubar"], sub["kappa"], sub["ds"], p, W, "linear")
    H, g, C, dd = Q["H"], Q["g"], Q["C"], Q["d"]
    sc = CF.sqp_scale("dyn", 40, 40)
    z1 = ((u1[idx] - sub["ubar"]) / sc).reshape(len(idx), -1)
    cert1 = CF.certify(H, g, C, dd, z1)
    zo, oko, how = CF.exact(H, g, C, dd, seed_lam=cert1["lam"], seed_z=z1)
    ao = D.domain_step(sub["x0"], sub["ubar"], zo.reshape(len(idx), 40, 2) * sc, sub["kappa"], sub["ds"], p, "linear",
                       D.dyn_predict)
    f = lambda z: 0.5 * np.einsum("bi,bij,bj->b", z, H, z) + np.einsum("bi,bi->b", g, z)
    rep = []
    for j, b in enumerate(idx):
        # the step length that explains the kernel's applied step best
        cands = [0.0] + [2.0 ** -i for i in range(8)]
        errs = [np.abs(z1[j] - a * zo[j]).max() for a in cands]
        ak = cands[int(np.argmin(errs))]
        zk = z1[j] / ak if ak > 0 else z1[j]
        ck1 = CF.certify(H[j:j + 1], g[j:j + 1], C[j:j + 1], dd[j:j + 1], zk[None])
        ok_alpha_o = CF.kkt_ok(CF.certify(H[j:j + 1], g[j:j + 1], C[j:j + 1], dd[j:j + 1],
                                          (z1[j] / ao[j] if ao[j] > 0 else z1[j])[None]))[0]
        ok_alpha_k = CF.kkt_ok(ck1)[0]
        if args.probs is None and ok_alpha_o:
            continue
        rep.append(dict(problem=int(b), status=int(st[b]), diag=dg[b].tolist(), alpha_oracle=float(ao[j]),
                        alpha_kernel_best=ak, err_at_alpha_kernel=float(min(errs)), cert_ok_alpha_oracle=bool(ok_alpha_o),
                        cert_ok_alpha_kernel=bool(ok_alpha_k), dz_err_alpha_kernel=float(np.abs(zk - zo[j]).max()),
                        f_kernel=float(f(zk[None])[0]), f_oracle=float(f(zo[j][None])[0]), exact_ok=bool(oko[j]),
                        stat=float(ck1["stat"][0] / ck1["scale"][0]), pfeas=float(ck1["pfeas"][0] / ck1["scale"][0]),
                        comp=float(ck1["comp"][0] / ck1["scale"][0]), scale=float(ck1["scale"][0])))
    out = dict(n_checked=int(len(idx)), uncertified_at_oracle_alpha=rep)
    print(json.dumps(out, indent=1))
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
