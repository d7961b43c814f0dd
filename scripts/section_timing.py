"""Per-section cycle counts of the fused kernel (timing build: make -C
vehicle-control_amd/csrc timing).  Run with VCMPC_LIB pointing at
libvcmpc_timing.so.  Prints mean s_memtime cycles per problem for each section,
and per interior-point iteration."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))
os.environ.setdefault("VCMPC_LIB", os.path.join(ROOT, "vehicle-control_amd", "vcmpc", "libvcmpc_timing.so"))
from vcmpc import Context, _abi, make_params  # noqa: E402
from vcmpc.config import load_config  # noqa: E402
from vcmpc.workload import kinematic_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
tol = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-10
names = ["S1 rollout", "setup", "resid", "build", "chol", "solve", "pol fact", "polish", "out", "S2 jac", "S3 sens", "S4 hess",
         "pol AL", "AL passes", "upd rounds", "upd cyc", "drop rounds", "early fail", "carry rm", "carry add", "r0 change"]
dev = torch.device("cuda:0")
d = kinematic_batch(B, seed=31)
t = {k: torch.from_numpy(v).to(dev) for k, v in d.items()}
p = make_params(kin_car=load_config("kinematic_car"), kin_mpc=load_config("kinematic_mpc"))
p.qp.tol = tol
with Context(N=20, max_batch=B, params=p) as c:
    B_, N = B, 20
    xbar = torch.empty((B, N + 1, 6), dtype=torch.float64, device=dev)
    u0 = torch.empty((B, 2), dtype=torch.float64, device=dev)
    st = torch.empty((B,), dtype=torch.int32, device=dev)
    it = torch.empty((B,), dtype=torch.int32, device=dev)
    diag = torch.zeros((B, 4 + len(names)), dtype=torch.float64, device=dev)
    ptrs = [C for C in (t["x0"], t["kappa"], t["ds"], xbar, t["ubar"].clone(), u0, st, it, diag)]
    import ctypes as C
    for _ in range(2):
        ub = t["ubar"].clone()
        rc = c.lib.vc_solve_diag(c._h, B, *[C.c_void_p(x.data_ptr()) for x in
                                            (t["x0"], t["kappa"], t["ds"], xbar, ub, u0, st, it, diag)],
                                 _abi.VC_DEVICE_PTRS)
        assert rc == 0
        c.synchronize()
    dg = diag.cpu().numpy()
    its = it.cpu().numpy().astype(float)
    cyc = dg[:, 4:]
    # pol fact (slot 6) and pol AL (12) are parts of polish (7); slot 13 counts AL passes
    tot = cyc[:, :12].sum(1) - cyc[:, 6]
    print(f"B={B} tol={tol:g}: solved {(st.cpu().numpy() == 0).mean():.4f} iters mean {its.mean():.2f} max {its.max():.0f} "
          f"polish rounds mean {dg[:, 3].mean():.2f}")
    print(f"  total stamped cycles/problem: mean {tot.mean():.0f}  max {tot.max():.0f}")
    for i, nm in enumerate(names):
        per_it = cyc[:, i].sum() / max(its.sum(), 1) if nm in ("resid", "build", "chol", "solve") else float("nan")
        print(f"  {nm:10s} mean {cyc[:, i].mean():10.0f}  ({100 * cyc[:, i].mean() / tot.mean():5.1f} %)  per IPM iter {per_it:9.0f}"
              f"   slowest problem {cyc[tot.argmax(), i]:10.0f}")
    # the launch ends with its slowest problem (one wave per SIMD at B = 1024): where the tail comes from
    order = np.argsort(tot)[::-1]
    print(f"  total cycles percentiles p50 {np.percentile(tot, 50):.0f} p90 {np.percentile(tot, 90):.0f} "
          f"p99 {np.percentile(tot, 99):.0f} max {tot.max():.0f}")
    for b in order[:6]:
        print(f"  slow problem {b}: total {tot[b]:.0f} iters {its[b]:.0f} polish rounds {dg[b, 3]:.0f} "
              + " ".join(f"{nm}={cyc[b, i]:.0f}" for i, nm in enumerate(names) if cyc[b, i] > 0))
    for k in range(int(its.min()), int(its.max()) + 1):
        sel = its == k
        if sel.any():
            print(f"  iters {k:2d}: {sel.sum():4d} problems, total cycles mean {tot[sel].mean():.0f} max {tot[sel].max():.0f}")
    ef = cyc[:, names.index("early fail")] > 0
    if ef.any():
        rm, ad = cyc[ef, names.index("carry rm")], cyc[ef, names.index("carry add")]
        print(f"  failed early attempts: {int(ef.sum())}; final set vs the early factor: drops 0 in {int((rm == 0).sum())}, "
              f"adds <= 1 / 2 / 3 with no drop: {int(((rm == 0) & (ad <= 1)).sum())} / {int(((rm == 0) & (ad <= 2)).sum())} / "
              f"{int(((rm == 0) & (ad <= 3)).sum())}; slowest such problems: "
              + ", ".join(f"{int(b)} (rm {int(cyc[b, names.index('carry rm')])}, add {int(cyc[b, names.index('carry add')])})"
                          for b in order if ef[b])[:400])
    r0 = cyc[:, names.index("r0 change")].astype(int)
    if (r0 > 0).any():
        kinds = ["box add", "row add", "drop"]
        tap = ["undecided", "active", "inactive"]
        from collections import Counter
        rows = Counter()
        for b in np.nonzero(r0 > 0)[0]:
            c = r0[b] - 1
            rows[(kinds[c % 3], tap[c // 3], "early fail" if ef[b] else "early ok")] += 1
        print("  early attempts that changed a constraint in round 0 (kind, changed side's Tapia state, outcome): "
              + "; ".join(f"{k}: {v}" for k, v in sorted(rows.items())))
        print("  early-fail problems' first change: " + ", ".join(f"{int(b)}: {kinds[(r0[b] - 1) % 3]} / {tap[(r0[b] - 1) // 3]}"
                                                          for b in np.nonzero(ef)[0]))
    if os.environ.get("SEC_DUMP"):  # per-problem arrays for offline tail analysis
        np.savez(os.environ["SEC_DUMP"], cyc=cyc, its=its, rounds=dg[:, 3], tot=tot)
