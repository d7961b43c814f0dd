#!/usr/bin/env python3
"""Benchmark: batched MPC solves/s on MI355X (BASELINE.json metric).

One step = one fused predict -> linearize -> condense -> interior-point solve of
every problem of this rank's batch (vc_solve, csrc/kin_ltv.hip), inputs resident
in HBM.  Default workload: BASELINE config 2 -- B = 1024 kinematic-bicycle
problems, N = 20, fp64, per GPU.  With --gpus N under torchrun each rank solves
its own batch (weak scaling, no data-path collective); rank 0 prints one JSON line.

The same line carries, under "c3", BASELINE config 3 -- B = 4096 dynamic-bicycle
(linear tyre) single-track NMPC problems per GPU, N = 40, 3 SQP iterations, solved in fp64
(vc_solve on a dynamic context, csrc/st_sqp.hip: the kernel that meets the 1e-5 parity bar,
and the faster one) -- measured the same way; it is a secondary workload, not `value`.
The fp32 condensed kernel BASELINE config 3 names (csrc/dyn_sqp.hip) is measured beside it under
"c3_f32" (it misses the 1e-5 bar -- fp32 QP-data floor, DESIGN 2b -- and is slower than the fp64
kernel; --no-c3-f32 skips it), and "c3_survey" runs the fp64 C3 leg on SURVEY 8(d)'s full sampler
ranges (Ux down to 5 m/s, ey to +-3 m, Fx warm starts to +-6000 N).  Under "c5": BASELINE config 5 -- the closed-loop
Monte-Carlo, 8192 vehicles x 500 steps on ippodromo (horizon -> NMPC solve -> fp64
plant, all on the device, vc_simulate), vehicles sharded over the ranks.  Under
"cascaded": the reference's cascaded NMPC (20 single-track + 40 point-mass stages,
config/controllers/cascaded.yaml), B = 4096 per GPU, fp64
(csrc/casc_ric.hip, stagewise Riccati).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--c3-batch B3]
                    [--c5-vehicles V] [--c5-steps S] [--no-c3] [--no-c5] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP64_VALU_PEAK_TFS = 78.6      # MI355X FP64 vector (spec), SURVEY 8(d)
N_HORIZON, NX, NU = 20, 6, 2
# Compulsory HBM bytes per solve: in x0 + kappa + ds + ubar, out
# u* + x* + u0 (fp64) + status + iters.
BYTES_PER_SOLVE = (NX + N_HORIZON + N_HORIZON + N_HORIZON * NU) * 8 + \
                  (N_HORIZON * NU + (N_HORIZON + 1) * NX + NU) * 8 + 8
# Algorithmic fp64 FLOPs of the fused kernel (DESIGN.md "Arithmetic"): forward
# sweep (rollout, Jacobians, rank-1 Hessian build) once, then per interior-point
# iteration the normal-matrix build sum_r w_r g_r g_r' over the lower-triangular
# constraint rows, an n^3/3 Cholesky, two triangular-solve pairs and the
# mat-vecs; the polish costs about one iteration per round.
N_DEC = NU * N_HORIZON
NC_ROWS = 2 * (N_HORIZON - 1)
FLOP_SWEEP = N_HORIZON * (2 * N_DEC * N_DEC + 200) + 3 * 2 * N_DEC * N_DEC
FLOP_ITER = (2 * N_DEC * sum(2 * (1 + r % (N_HORIZON - 1)) for r in range(NC_ROWS))  # build
             + N_DEC ** 3 // 3 + 2 * 2 * N_DEC * N_DEC                                  # Cholesky, 2 solves
             + 4 * (2 * NC_ROWS * N_DEC) + 2 * 2 * N_DEC * N_DEC)                       # mat-vecs
FP64_VALU_PEAK = 78.6  # TFLOP/s
# newest committed PMC summary first (scripts/pmc_profile.sh -> scripts/pmc_summary.py)
PMC_SUMMARIES = [os.path.join(ROOT, "profiles", r, "pmc_summary.json") for r in ("r06", "r05", "r04")]
PMC_SUMMARY = next((p for p in PMC_SUMMARIES if os.path.exists(p)), PMC_SUMMARIES[0])

# ---- C3: dynamic single-track SQP (fp32, N = 40) ------------------------------------
C3_N, C3_NX = 40, 8
FP32_PEAK_TFS = 157.3          # MI355X FP32 vector = FP32 MFMA (MI355X_MICROARCH.md)
# compulsory bytes: in x0 + kappa + ds + ubar, out u* + x* (N columns) + u0 (fp32) + status + iters
C3_BYTES_PER_SOLVE = (C3_NX + 2 * C3_N + 2 * C3_N) * 4 + (2 * C3_N + C3_N * C3_NX + 2) * 4 + 8
C3_n = 2 * C3_N
# Algorithmic fp32 FLOPs: per interior-point iteration the normal-matrix
# build sum_k V_k' W_k V_k over the triangular stage blocks (7 basis rows, columns < 2k),
# the blocked Cholesky with the augmented inverse (~ n^3), two explicit-inverse solves
# (2 x 2 n^2) and the forward/adjoint G passes (3 + 3 x 2 x 5 x sum_k 2k); per SQP
# iteration the rollout + dual-number Jacobians (~ 40 RK4 evaluations x 9 directions x
# ~300 flops) and the condensing (80 columns x 39 stages x 7 x 7 x 2).
C3_G_NNZ = sum(2 * k for k in range(1, C3_N))                      # nonzeros of one G row set
C3_FLOP_ITER = (sum(2 * (2 * k) * 7 * 7 + (2 * k) ** 2 * 7 for k in range(1, C3_N))  # build: W V, then V'(W V) half
                + C3_n ** 3 + 2 * 2 * 2 * C3_n * C3_n                         # factor + 2 solves
                + 6 * 2 * 5 * C3_G_NNZ)                                       # G passes
C3_FLOP_SQP = 4 * (C3_N - 1) * 9 * 300 + C3_n * (C3_N - 1) * 7 * 7 * 2


# ---- roctx ranges: one per timed leg, so a rocprofv3 --kernel-trace --marker-trace pass can be
# split per leg (scripts/leg_stats.py -> profiles/<round>/kernel_leg_stats_*.csv): the same kernel
# runs in several legs (kin_ltv_kernel<20> in C2 and C4, st_sqp_kernel<60> at 5 and 40 SQP
# iterations, casc_ric at 3 and 40), and a per-grid average mixes them
_ROCTX = None


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        import ctypes
        _ROCTX = False
        for name in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so.4", "libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                _ROCTX = lib
                break
            except (OSError, AttributeError):
                continue
    return _ROCTX


def leg_push(name):
    lib = _roctx()
    if lib:
        lib.roctxRangePushA(("leg:" + name).encode())


def leg_pop():
    lib = _roctx()
    if lib:
        lib.roctxRangePop()


def c3_bytes(N, word):
    """Compulsory HBM bytes per single-track solve: in x0 + kappa + ds + ubar, out u* + x*
    (N columns) + u0, + status + iters."""
    return (C3_NX + 2 * N + 2 * N) * word + (2 * N + N * C3_NX + 2) * word + 8


def st_flops(ipm_iters_total, N, sqp_iters=3):
    """Algorithmic fp64 FLOPs of one stagewise-Riccati SQP solve (csrc/st_sqp.hip):
    per interior-point iteration the Riccati factorisation (per stage T = P [A B] 7x8x6, the
    45 stage-Hessian entries x 6, the 28 + 14 Schur / gain entries: ~1.7 K FLOP), two LQ
    solves (backward + forward sweeps, ~0.45 K FLOP per stage each) and the adjoint residual
    sweep (~0.1 K), plus the stage-local rows (~1 K per stage: 12 rows, barrier Hessian,
    residuals, two step computations); per SQP iteration the RK4 rollout (~1.2 K FLOP per
    stage), the dual-number Jacobians (4 seed pairs x 3 x 1.2 K) and stage functions
    (5 x 2 x 0.25 K)."""
    per_stage_iter = 2 * (56 * 6 + 45 * 7 + 28 * 6 + 14 * 2) + 2 * 450 + 100 + 1000
    per_stage_sqp = 1200 + 4 * 3 * 1200 + 5 * 2 * 250
    return ipm_iters_total * N * per_stage_iter + (sqp_iters + 1) * N * per_stage_sqp


def c3_flops(pdip_iters_total, sqp_iters=3, polish_rounds=2):
    """fp32 FLOPs of one C3 solve given its total interior-point iterations."""
    return (sqp_iters * C3_FLOP_SQP + (pdip_iters_total + sqp_iters * polish_rounds) * C3_FLOP_ITER
            + C3_N * 4 * 300)


def pmc_traffic(batch, kernel="kin_ltv_kernel<20>"):
    """HBM bytes per launch from the committed rocprofv3 PMC passes (FETCH_SIZE +
    WRITE_SIZE, scripts/pmc_profile.sh -> scripts/pmc_summary.py) when they were taken at
    this batch (one 64-lane workgroup per problem: grid = 64 B threads)."""
    try:
        with open(PMC_SUMMARY) as f:
            p = json.load(f)
        # FETCH_SIZE counts half the bytes of a read on gfx950 (MI355X guide; calibrated for this
        # kernel's 8 B-per-lane loads too: scripts/pmc_calibrate.sh, profiles/r05/pmc_calibration_r05y.txt,
        # FETCH_SIZE = 0.500 and WRITE_SIZE = 1.000 of a known byte count), so reads count twice
        return p[f"{kernel} grid={64 * batch}"]["derived"]["traffic_bytes_per_launch_fetch_x2"]
    except (OSError, ValueError, KeyError):
        return None


def pmc_mfma(batch, kernel="kin_ltv_kernel<20>"):
    """The matrix-core share of one launch, from the committed PMC pass at this batch
    (profiles/<round>/pmc_summary.json, scripts/pmc_summary.py):
      flops_per_launch = SQ_INSTS_VALU_MFMA_MOPS_F64 x 512 (v_mfma_f64_16x16x4_f64 = 2,048 FLOP,
                         counted as 4 MOPS of 512), equal to SQ_INSTS_MFMA x 2,048 here (the only
                         MFMA the kernel issues);
      busy_frac        = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x cycles of the launch), SIMDs = 256 CUs x 4,
                         cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums GRBM over the 8 XCDs; MI355X guide,
                         DVFS note) -- BUSY_CYCLES counts SIMD cycles, 64 per v_mfma_f64_16x16x4_f64
                         (463,596 MFMAs, 29.67 M busy cycles at C2, r05);
      peak             = the dense fp64 matrix rate, 78.6 TFLOP/s (16x16x4 f64 = 2,048 FLOP per 64 cycles
                         per SIMD x 1,024 SIMDs x 2.4 GHz), the same number as the fp64 vector peak."""
    try:
        with open(PMC_SUMMARY) as f:
            p = json.load(f)
        e = p[f"{kernel} grid={64 * batch}"]
    except (OSError, ValueError, KeyError):
        return None
    c = e["counters_per_dispatch"]
    flops = float(c.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0)) * 512.0 + float(c.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0)) * 512.0
    cyc = float(c["GRBM_GUI_ACTIVE"]) / 8.0
    busy = float(c["SQ_VALU_MFMA_BUSY_CYCLES"])
    return {"flops_per_launch": flops, "flops_per_solve": flops / batch, "mfma_insts_per_launch": float(c["SQ_INSTS_MFMA"]),
            "busy_cycles_per_launch": busy, "launch_cycles": cyc, "simds": 1024,
            "busy_frac": busy / (1024.0 * cyc), "peak": FP64_VALU_PEAK, "unit": "TFLOP/s",
            "source": os.path.relpath(PMC_SUMMARY, ROOT),
            "valu_insts_per_launch": float(c["SQ_INSTS_VALU"])}


def _mfma_live(m, kern_ms):
    """pmc_mfma's counters priced on this run's live kernel time (the rocprof pass's own
    duration gives busy_frac; achieved / frac use the timed launches)."""
    if m is None:
        return None
    a = m["flops_per_launch"] / (kern_ms / 1e3) / 1e12
    return dict(m, achieved=a, frac=a / m["peak"],
                note="matrix-core FLOP per launch from SQ_INSTS_VALU_MFMA_MOPS_F64 x 512 (= SQ_INSTS_MFMA x 2048); "
                     "busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) of the PMC pass; "
                     "achieved / frac on the live kernel_ms")


class _Skip(Exception):
    """a leg switched off on the command line"""


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024, help="problems per GPU (config 2: 1024)")
    ap.add_argument("--seed", type=int, default=31)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=1024, help="problems in the CPU-baseline sample")
    ap.add_argument("--c3-batch", type=int, default=4096, help="C3 problems per GPU (config 3: 4096)")
    ap.add_argument("--no-c3", action="store_true", help="skip the secondary C3 measurement")
    ap.add_argument("--no-c3-f32", action="store_true",
                    help="skip C3 through the fp32 condensed kernel (BASELINE config 3's named dtype)")
    ap.add_argument("--no-c3-survey", action="store_true",
                    help="skip C3 on SURVEY 8(d)'s full sampler ranges (Ux ~ U(5, 22), ey ~ U(-3, 3), Fx ~ U(-6000, 6000))")
    ap.add_argument("--c5-vehicles", type=int, default=C5_VEHICLES, help="C5 vehicles in total (config 5: 8192)")
    ap.add_argument("--c5-steps", type=int, default=C5_STEPS, help="C5 closed-loop steps (config 5: 500)")
    ap.add_argument("--no-c5", action="store_true", help="skip the secondary C5 closed-loop measurement")
    ap.add_argument("--casc-batch", type=int, default=4096, help="cascaded NMPC problems per GPU")
    ap.add_argument("--no-casc", action="store_true", help="skip the cascaded (point-mass tail) measurement")
    ap.add_argument("--c4-total", type=int, default=C4_TOTAL,
                    help="C4 problems in total, split into contiguous shards over the ranks (config 4: 65536)")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 sharded measurement")
    ap.add_argument("--no-kin-legs", action="store_true",
                    help="skip the stagewise kinematic legs (N = 20 Riccati, N = 50 = kinematic.yaml)")
    ap.add_argument("--latency-calls", type=int, default=200,
                    help="single-vehicle drop-in latency: timed command + drive steps per controller")
    ap.add_argument("--no-latency", action="store_true", help="skip the single-vehicle latency legs")
    ap.add_argument("--no-converged", action="store_true",
                    help="skip the converged-setting legs (40 SQP iterations): a PMC pass then averages the "
                         "st_sqp<60> / casc_ric dispatches of the bench-setting legs only (same kernel, same grid)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU work: each rank only takes its C2/C4/C5 shards and runs the counter "
                         "collective over gloo (tests the launcher and the rank logic on a CPU host)")
    return ap.parse_args()


def cpu_baseline(batch, sample):
    """The numpy oracle (oracle/ltv_qp.py + oracle/qp.py) on one host thread, on the
    first `sample` problems of this rank's workload: the build's CPU 'port' of the
    reference path (the reference's CasADi/IPOPT cannot run)."""
    from threadpoolctl import threadpool_limits

    from oracle import ltv_qp as Q
    from vcmpc.config import load_config
    W = Q.kin_weights(load_config("kinematic_mpc"))
    d = {k: v[:sample] for k, v in batch.items()}
    with threadpool_limits(limits=1):
        t0 = time.perf_counter()
        Q.kin_ltv_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], 2.5, W)
        dt = time.perf_counter() - t0
    cpu = cpu_model()
    return {"value": len(d["x0"]) / dt, "unit": "solves/s", "cores": 1, "kind": "port",
            "sample": f"{len(d['x0'])} problems of the C2 workload, one oracle pass (PDIP + active-set polish, "
                      f"numpy fp64, 1 thread) in {dt:.2f} s on {cpu}; a stand-in for the reference's "
                      f"CasADi/IPOPT path, which cannot run here"}


def usable_cpus():
    """(cores, source): the CPU cores this process may use.  A cgroup CPU quota (cpu.max,
    cgroup v2; cpu.cfs_quota_us, v1) wins; else the box's per-GPU CPU share that the pool
    exports as OMP_NUM_THREADS (16 on the GPU boxes, whose affinity mask shows the whole
    machine); else the affinity mask."""
    import math
    aff = len(os.sched_getaffinity(0))
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            txt = open(path).read().split()
        except OSError:
            continue
        try:
            if path.endswith("cpu.max") and txt[0] != "max":
                return min(aff, max(1, math.floor(int(txt[0]) / int(txt[1])))), f"cgroup {path} = {' '.join(txt)}"
            if path.endswith("cfs_quota_us") and int(txt[0]) > 0:
                per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
                return min(aff, max(1, int(txt[0]) // per)), f"cgroup {path} = {txt[0]} / {per}"
        except (ValueError, IndexError, OSError):
            continue
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        return min(aff, int(omp)), (f"no cgroup CPU quota; OMP_NUM_THREADS={omp} (the pool's per-GPU CPU share; "
                                    f"affinity shows {aff})")
    return aff, "no cgroup CPU quota; sched_getaffinity"


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def _oracle_chunk(job):
    """Pool worker: one oracle pass over a chunk of C2 ("kin") or C3 ("c3") problems, one thread."""
    from threadpoolctl import threadpool_limits

    from vcmpc.config import load_config
    if job is None:  # warm-up: imports only
        from oracle import dyn_sqp, ltv_qp  # noqa: F401
        return 0.0
    kind, chunk = job
    with threadpool_limits(limits=1):
        if kind == "kin":
            from oracle import ltv_qp as Q
            W = Q.kin_weights(load_config("kinematic_mpc"))
            Q.kin_ltv_solve(chunk["x0"], chunk["ubar"], chunk["kappa"], chunk["ds"], 2.5, W)
        else:
            from oracle import dyn_sqp as D
            from oracle import models as M
            W = D.dyn_weights(load_config("dynamic_mpc"))
            p = M.dyn_params_from_config(load_config("dynamic_car"))
            D.dyn_sqp_solve(chunk["x0"], chunk["ubar"], chunk["kappa"], chunk["ds"], p, W, "linear")
    return float(len(chunk["x0"]))


def cpu_baseline_all_cores(batch, sample, kind="kin", per_worker=None):
    """SURVEY 8(d)'s second CPU figure: the oracle pass with one single-threaded process per
    usable core (usable_cpus()), each on its own chunk of the workload.  Spawned children
    (fresh interpreters, no forked HIP state); interpreter start-up and imports are excluded
    by a warm-up map before the timed one.  per_worker: problems per process (default: the
    sample split evenly)."""
    import multiprocessing as mp

    import numpy as np
    workers, source = usable_cpus()
    n_total = len(batch["x0"])
    sample = min(sample if per_worker is None else per_worker * workers, n_total)
    d = {k: np.asarray(v[:sample], np.float64) for k, v in batch.items()}
    parts = np.array_split(np.arange(sample), workers)
    chunks = [(kind, {k: np.ascontiguousarray(v[p]) for k, v in d.items()}) for p in parts if len(p)]
    with mp.get_context("spawn").Pool(len(chunks)) as pool:
        pool.map(_oracle_chunk, [None] * len(chunks), chunksize=1)
        t0 = time.perf_counter()
        done = sum(pool.map(_oracle_chunk, chunks, chunksize=1))
        dt = time.perf_counter() - t0
    what = "C2 kinematic LTV-QP (PDIP + active-set polish)" if kind == "kin" else \
        "C3 single-track SQP (3 SQP iterations, complex-step linearisation + exact QPs)"
    return {"value": done / dt, "unit": "solves/s", "cores": len(chunks), "kind": "port",
            "usable_cores": workers, "usable_cores_source": source, "nproc": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0)), "cpu_model": cpu_model(),
            "sample": f"{int(done)} problems of the {what} workload split over {len(chunks)} single-threaded "
                      f"numpy-oracle processes (one per usable core), {dt:.2f} s wall; the oracle stands in "
                      f"for the reference's CasADi/IPOPT path, which cannot run here"}


def cpu_baseline_c3(data, sample):
    """The fp64 numpy oracle of the SQP contract (oracle/dyn_sqp.py, 3 exact QPs per
    solve), one host thread, on the first `sample` problems of the C3 workload."""
    from threadpoolctl import threadpool_limits

    from oracle import dyn_sqp as D
    from oracle import models as M
    from vcmpc.config import load_config
    W = D.dyn_weights(load_config("dynamic_mpc"))
    p = M.dyn_params_from_config(load_config("dynamic_car"))
    d = {k: v[:sample].astype("float64") for k, v in data.items()}
    with threadpool_limits(limits=1):
        t0 = time.perf_counter()
        D.dyn_sqp_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], p, W, "linear")
        dt = time.perf_counter() - t0
    return {"value": len(d["x0"]) / dt, "unit": "solves/s", "cores": 1, "kind": "port",
            "sample": f"{len(d['x0'])} problems of the C3 workload, one oracle pass (3 SQP iterations of "
                      f"complex-step linearisation + exact QP, numpy fp64, 1 thread) in {dt:.2f} s"}


def run_c3(args, dev, stream, rank, dist, steps, f64=False, N=C3_N, cfg_name="dynamic_mpc", qp=None, leg="c3",
           ranges="traces"):
    """Secondary measurement: BASELINE config 3 on this rank (weak scaling).  f64=True runs
    the same workload through the fp64 stagewise-Riccati kernel (csrc/st_sqp.hip); with
    N = 60 / cfg_name = "singletrack_mpc" it is the reference's own single-track horizon.
    ranges="survey": SURVEY 8(d)'s C3 sampler ranges as written (vcmpc/workload.py dynamic_batch)."""
    import numpy as np
    import torch

    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.workload import dynamic_batch

    B = args.c3_batch
    draw = {}
    data = dynamic_batch(B, N=N, seed=args.seed + 104729 * rank, ranges=ranges, stats=draw)
    tdt = torch.float64 if f64 else torch.float32
    t = {k: torch.from_numpy(v).to(dev, tdt) for k, v in data.items()}
    ubar0 = t["ubar"].clone()
    cfg = load_config(cfg_name)
    cfg["qp"] = dict(cfg["qp"], **(qp or {}))
    params = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=cfg, tyre="linear")
    ctx = Context(model=_abi.VC_MODEL_DYNAMIC, N=N, max_batch=B, dtype=_abi.VC_F64 if f64 else _abi.VC_F32,
                  device=dev.index, params=params)
    ctx.set_stream(stream.cuda_stream)
    xbar = torch.empty((B, N, C3_NX), dtype=tdt, device=dev)
    u0 = torch.empty((B, 2), dtype=tdt, device=dev)
    status = torch.empty((B,), dtype=torch.int32, device=dev)
    iters = torch.empty((B,), dtype=torch.int32, device=dev)

    def step(ev=None):
        t["ubar"].copy_(ubar0)
        if ev is not None:
            ev[0].record(stream)
        ctx.solve(t["x0"], t["kappa"], t["ds"], t["ubar"], xbar, u0, status, iters)
        if ev is not None:
            ev[1].record(stream)

    step()
    torch.cuda.synchronize(dev)
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    dist.barrier()
    torch.cuda.synchronize(dev)
    leg_push(leg)
    t0 = time.perf_counter()
    for i in range(steps):
        step(events[i])
    torch.cuda.synchronize(dev)
    leg_pop()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    st, it = status.cpu().numpy(), iters.cpu().numpy()
    solves, elapsed_max, kern_ms_max = dist.aggregate(float(B * steps), elapsed, kern_ms, dev)
    ctx.close()
    sqp = int(cfg["qp"]["sqp_iters"])
    if f64:
        flops = st_flops(float(it.mean()), N, sqp)
        word, kern, peak, bpsolve = 8, f"st_sqp_kernel<{N}, linear>", FP64_VALU_PEAK, c3_bytes(N, 8)
    else:
        flops = c3_flops(float(it.mean()))
        word, kern, peak, bpsolve = 4, "dyn_sqp_kernel<40, linear>", FP32_PEAK_TFS, C3_BYTES_PER_SOLVE
    dname = "fp64" if f64 else "fp32"
    out = {"metric": f"MPC solves/sec (batched, N={N}, {sqp} SQP iterations, prox {cfg['qp']['prox']})",
           "value": solves / elapsed_max,
           "unit": "solves/s", "steps": steps, "ms_per_step": elapsed_max / steps * 1e3,
           "dtype": "f64" if f64 else "f32",
           "config": {"workload": f"C3 dynamic-bicycle (linear tyre) single-track NMPC via SQP, B={B} per GPU, "
                                  f"N={N}, {dname}" + ("" if cfg_name == "dynamic_mpc" else f", {cfg_name}.yaml"),
                      "batch_per_gpu": B, "horizon": N},
           "roofline": {"bound": "fp64" if f64 else "fp32", "kernel": kern, "kernel_ms": kern_ms,
                        "flops_per_solve": flops, "achieved": flops * B / (kern_ms / 1e3) / 1e12,
                        "peak": peak, "unit": "TFLOP/s",
                        "frac": flops * B / (kern_ms / 1e3) / 1e12 / peak,
                        "hbm": {"bytes_per_solve": bpsolve,
                                "achieved": bpsolve * B / (kern_ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS,
                                "unit": "GB/s"}},
           "solver": {"solved_frac": float((st == 0).mean()), "pdip_iters_mean": float(it.mean()),
                      "pdip_iters_max": int(it.max()),
                      "status_counts": {str(int(k)): int(v) for k, v in zip(*np.unique(st, return_counts=True))}}}
    if ranges == "survey":
        out["config"]["workload"] += (" -- SURVEY 8(d) sampler ranges: Ux ~ U(5, 22), ey ~ U(-3, 3), Fx warm start "
                                      "~ U(-6000, 6000) N per stage; warm starts outside the spatial model's domain "
                                      f"re-drawn ({draw.get('redrawn', 0)} of {draw.get('drawn', 0)} drawn)")
    return out, data


# ---- cascaded NMPC: N = 20 single-track + M = 40 point-mass stages, fp64 ----
CA_N, CA_M = 20, 40
CA_H, CA_n = CA_N + CA_M, 2 * (CA_N + CA_M)
# compulsory bytes: in x0 + kappa + ds + ubar, out u* + x* (H columns) + u0 (fp64) + status + iters
CA_BYTES_PER_SOLVE = (8 + 2 * CA_H + 2 * CA_H) * 8 + (2 * CA_H + 8 * CA_H + 2) * 8 + 8
# algorithmic fp64 FLOPs per interior-point iteration: the stage-block normal matrix
# sum_k V_k' W_k V_k (7 basis rows, columns < 2k + 2: W V then the lower half of V' (W V)),
# n^3/3 Cholesky, 2 x 2 triangular solves, 6 forward/adjoint passes over the condensed rows;
# per SQP iteration the rollout + dual-number Jacobians and the condensing
CA_G_NNZ = 5 * sum(2 * k for k in range(1, CA_N)) + 2 * sum(2 * (CA_N + m) for m in range(CA_M))
CA_FLOP_ITER = (sum(2 * (2 * k + 2) * 7 * 7 + (2 * k + 2) ** 2 * 7 for k in range(CA_H))
                + CA_n ** 3 // 3 + 4 * CA_n * CA_n + 6 * 2 * CA_G_NNZ)
CA_FLOP_SQP = (CA_N - 1) * 10 * 4 * 400 + (CA_M - 1) * 7 * 60 + CA_n * (CA_N * 8 * 8 + CA_M * 5 * 5) * 2


# the SQP setting that reproduces IPOPT's recorded solutions (tests/test_gpu_replay.py)
CONVERGED_QP = {"prox": 0.01, "sqp_iters": 40}


def run_casc(args, dev, stream, rank, dist, steps, qp=None, leg="cascaded"):
    """Cascaded NMPC (horizon_pm = 40) on this rank, B problems per GPU, fp64."""
    import numpy as np
    import torch

    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.workload import cascaded_batch

    B = args.casc_batch
    data = cascaded_batch(B, seed=args.seed + 15485863 * rank)
    t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
    ubar0 = t["ubar"].clone()
    cfg = load_config("cascaded_mpc")
    cfg["qp"] = dict(cfg["qp"], **(qp or {}))
    params = make_params(dyn_car=load_config("dynamic_car"), dyn_mpc=cfg, tyre="fiala")
    ctx = Context(model=_abi.VC_MODEL_CASCADED, N=CA_N, max_batch=B, dtype=_abi.VC_F64, device=dev.index,
                  params=params)
    ctx.set_stream(stream.cuda_stream)
    xbar = torch.empty((B, CA_H, 8), dtype=torch.float64, device=dev)
    u0 = torch.empty((B, 2), dtype=torch.float64, device=dev)
    status = torch.empty((B,), dtype=torch.int32, device=dev)
    iters = torch.empty((B,), dtype=torch.int32, device=dev)

    def step(ev=None):
        t["ubar"].copy_(ubar0)
        if ev is not None:
            ev[0].record(stream)
        ctx.solve(t["x0"], t["kappa"], t["ds"], t["ubar"], xbar, u0, status, iters)
        if ev is not None:
            ev[1].record(stream)

    step()
    torch.cuda.synchronize(dev)
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    dist.barrier()
    torch.cuda.synchronize(dev)
    leg_push(leg)
    t0 = time.perf_counter()
    for i in range(steps):
        step(events[i])
    torch.cuda.synchronize(dev)
    leg_pop()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    st, it = status.cpu().numpy(), iters.cpu().numpy()
    solves, elapsed_max, kern_ms_max = dist.aggregate(float(B * steps), elapsed, kern_ms, dev)
    ctx.close()
    # stagewise Riccati kernel (csrc/casc_ric.hip): st_sqp's per-stage count over the H stages
    # (the point-mass stages are cheaper: an upper estimate)
    sqp = int(cfg["qp"]["sqp_iters"])
    flops = st_flops(float(it.mean()), CA_H, sqp)
    out = {"metric": f"MPC solves/sec (batched, N=20 single-track + 40 point-mass stages, {sqp} SQP iterations, "
                     f"prox {cfg['qp']['prox']})",
           "value": solves / elapsed_max, "unit": "solves/s", "steps": steps,
           "ms_per_step": elapsed_max / steps * 1e3, "dtype": "f64",
           "config": {"workload": f"cascaded NMPC (config/controllers/cascaded.yaml), B={B} per GPU, "
                                  f"H={CA_N}+{CA_M}, fp64, Fiala tyre", "batch_per_gpu": B, "horizon": CA_H},
           "roofline": {"bound": "fp64", "kernel": "casc_ric_kernel<20, 40, fiala>", "kernel_ms": kern_ms,
                        "flops_per_solve": flops, "achieved": flops * B / (kern_ms / 1e3) / 1e12,
                        "peak": FP64_VALU_PEAK, "unit": "TFLOP/s",
                        "frac": flops * B / (kern_ms / 1e3) / 1e12 / FP64_VALU_PEAK,
                        "hbm": {"bytes_per_solve": CA_BYTES_PER_SOLVE,
                                "achieved": CA_BYTES_PER_SOLVE * B / (kern_ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS,
                                "unit": "GB/s"}},
           "solver": {"solved_frac": float((st == 0).mean()), "pdip_iters_mean": float(it.mean()),
                      "pdip_iters_max": int(it.max())}}
    return out, data


def cpu_baseline_casc(data, sample):
    """The fp64 numpy oracle of the cascaded SQP contract (oracle/casc_sqp.py), one thread."""
    from threadpoolctl import threadpool_limits

    from oracle import casc_sqp as CS
    from oracle import models as M
    from vcmpc.config import load_config
    W = CS.casc_weights(load_config("cascaded_mpc"))
    p = M.dyn_params_from_config(load_config("dynamic_car"))
    d = {k: v[:sample] for k, v in data.items()}
    with threadpool_limits(limits=1):
        t0 = time.perf_counter()
        CS.casc_sqp_solve(d["x0"], d["ubar"], d["kappa"], d["ds"], p, W, "fiala")
        dt = time.perf_counter() - t0
    return {"value": len(d["x0"]) / dt, "unit": "solves/s", "cores": 1, "kind": "port",
            "sample": f"{len(d['x0'])} problems of the cascaded workload, one oracle pass (3 SQP iterations of "
                      f"complex-step linearisation + exact QP, numpy fp64, 1 thread) in {dt:.2f} s"}


C5_VEHICLES, C5_STEPS = 8192, 500
C4_TOTAL = 65536
def c4_shard(total, rank, world, seed):
    """This rank's contiguous C4 shard [lo, hi) of `total` kinematic problems;
    vcmpc.workload.c4_shard, shared with tests/test_gpu_certify.py."""
    from vcmpc.workload import c4_shard as shard_of
    return shard_of(total, rank, world, seed, N=N_HORIZON)


def run_c4(args, dev, stream, rank, world, dist, steps, leg="c4"):
    """BASELINE config 4: 65536 kinematic LTV-MPC problems (N = 20, fp64) in total, one
    contiguous shard per rank (8192 per GPU at 8 GPUs), no data-path collective; `value`
    = all problems / the slowest rank's time (strong scaling over the fixed 65536)."""
    import numpy as np
    import torch

    from vcmpc import Context, _abi
    from vcmpc.config import load_config
    lo, hi, data = c4_shard(args.c4_total, rank, world, args.seed)
    B = hi - lo
    t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
    ubar0 = t["ubar"].clone()
    ctx = Context(model=_abi.VC_MODEL_KINEMATIC, N=N_HORIZON, max_batch=B, device=dev.index,
                  kin_car=load_config("kinematic_car"), kin_mpc=load_config("kinematic_mpc"))
    ctx.set_stream(stream.cuda_stream)
    xbar = torch.empty((B, N_HORIZON + 1, NX), dtype=torch.float64, device=dev)
    u0 = torch.empty((B, NU), dtype=torch.float64, device=dev)
    status = torch.empty((B,), dtype=torch.int32, device=dev)
    iters = torch.empty((B,), dtype=torch.int32, device=dev)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        ctx.solve_from(t["x0"], t["kappa"], t["ds"], ubar0, t["ubar"], xbar, u0, status, iters)
        if ev is not None:
            ev[1].record(stream)

    step()
    torch.cuda.synchronize(dev)
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    dist.barrier()
    torch.cuda.synchronize(dev)
    leg_push(leg)
    t0 = time.perf_counter()
    for i in range(steps):
        step(events[i])
    torch.cuda.synchronize(dev)
    leg_pop()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    st, it = status.cpu().numpy(), iters.cpu().numpy()
    solves, elapsed_max, kern_ms_max = dist.aggregate(float(B * steps), elapsed, kern_ms, dev)
    solved, _, _ = dist.aggregate(float((st == 0).sum()), 0.0, 0.0, dev)
    ctx.close()
    return {"metric": "MPC solves/sec (batched, N=20), C4 problem set sharded over the ranks",
            "value": solves / elapsed_max, "unit": "solves/s", "steps": steps,
            "ms_per_step": elapsed_max / steps * 1e3, "kernel": "kin_ltv_kernel<20>", "kernel_ms": kern_ms,
            "kernel_ms_max": kern_ms_max, "dtype": "f64", "scaling": "strong",
            "config": {"workload": f"C4 kinematic-bicycle LTV-MPC, {args.c4_total} problems in total, N={N_HORIZON}, "
                                   f"fp64, contiguous shards", "total_batch": args.c4_total,
                       "batch_per_gpu_rank0": B, "parallelism": f"dp{world} (contiguous shards, no collective "
                                                                f"on the data path)"},
            "solver": {"solved_frac": solved / args.c4_total, "iters_mean_rank0": float(it.mean()),
                       "iters_max_rank0": int(it.max())}}


def run_kin_leg(args, dev, stream, rank, dist, steps, N, solver, B, leg="kin"):
    """A kinematic LTV-MPC leg beside C2: the stagewise-Riccati kernel (csrc/kin_ric.hip) at
    BASELINE's N = 20 (solver = 1, vs the condensed kin_ltv.hip of `value`) and at the
    reference's own horizon N = 50 (config/controllers/kinematic.yaml:2)."""
    import numpy as np
    import torch

    from vcmpc import Context, _abi
    from vcmpc.config import load_config, make_params
    from vcmpc.workload import kinematic_batch
    data = kinematic_batch(B, N=N, seed=args.seed + 7919 * rank + N)
    t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
    ubar0 = t["ubar"].clone()
    cfg = load_config("kinematic_mpc")
    cfg["qp"] = dict(cfg.get("qp") or {}, solver=solver)
    params = make_params(kin_car=load_config("kinematic_car"), kin_mpc=cfg)
    ctx = Context(model=_abi.VC_MODEL_KINEMATIC, N=N, max_batch=B, device=dev.index, params=params)
    ctx.set_stream(stream.cuda_stream)
    xbar = torch.empty((B, N + 1, NX), dtype=torch.float64, device=dev)
    u0 = torch.empty((B, NU), dtype=torch.float64, device=dev)
    status = torch.empty((B,), dtype=torch.int32, device=dev)
    iters = torch.empty((B,), dtype=torch.int32, device=dev)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        ctx.solve_from(t["x0"], t["kappa"], t["ds"], ubar0, t["ubar"], xbar, u0, status, iters)
        if ev is not None:
            ev[1].record(stream)

    step()
    torch.cuda.synchronize(dev)
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    dist.barrier()
    torch.cuda.synchronize(dev)
    leg_push(leg)
    t0 = time.perf_counter()
    for i in range(steps):
        step(events[i])
    torch.cuda.synchronize(dev)
    leg_pop()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    st, it = status.cpu().numpy(), iters.cpu().numpy()
    solves, elapsed_max, _ = dist.aggregate(float(B * steps), elapsed, kern_ms, dev)
    ctx.close()
    kern = "kin_ric_kernel" if (solver == 1 or N != N_HORIZON) else "kin_ltv_kernel"
    return {"metric": f"MPC solves/sec (batched, N={N})", "value": solves / elapsed_max, "unit": "solves/s",
            "steps": steps, "ms_per_step": elapsed_max / steps * 1e3, "kernel": f"{kern}<{N}>", "kernel_ms": kern_ms,
            "dtype": "f64",
            "config": {"workload": f"kinematic-bicycle LTV-MPC, B={B} per GPU, N={N}, fp64, stagewise Riccati "
                                   f"interior point + active-set polish", "batch_per_gpu": B, "horizon": N},
            "solver": {"solved_frac": float((st == 0).mean()), "iters_mean": float(it.mean()),
                       "iters_max": int(it.max())}}


def dry_run(args):
    """--dry-run: the multi-rank control flow without a GPU -- gloo process group from the
    launcher's environment, every rank's C2 batch / C4 and C5 shards, the counter
    collective, and rank 0's JSON line (tests/test_dist.py drives it through `launch`)."""
    from vcmpc import dist
    from vcmpc.workload import shard
    rank, local, world = dist.init("gloo")
    lo4, hi4, d4 = c4_shard(args.c4_total, rank, world, args.seed)
    lo5, hi5 = shard(args.c5_vehicles, rank, world)
    solves, elapsed_max, _ = dist.aggregate(float(args.batch + (hi4 - lo4)), 0.1 * (rank + 1), 0.0)
    c4_first = float(d4["x0"][0, 0])
    rows = [None] * world
    import torch.distributed as tdist
    if tdist.is_initialized():
        tdist.all_gather_object(rows, (rank, local, lo4, hi4, lo5, hi5, c4_first))
    else:
        rows = [(rank, local, lo4, hi4, lo5, hi5, c4_first)]
    if rank == 0:
        print(json.dumps({"metric": "dry-run", "n_gpus": world, "solves": solves, "elapsed_max": elapsed_max,
                          "ranks": rows}), flush=True)
    dist.shutdown()


def cpu_baseline_c5(x0, track, sample_vehicles=8, sample_steps=8):
    """The oracle closed loop (oracle/dyn_sqp.py SQP + oracle/models.py fp64 RK4 plant +
    oracle/track.py curvature), one host thread, on the first vehicles of the C5 job."""
    import numpy as np
    from threadpoolctl import threadpool_limits

    from oracle import dyn_sqp as D
    from oracle import models as M
    from vcmpc.config import load_config
    from vcmpc.workload import C5_MPC_DT
    cfg = load_config("dynamic_mpc")
    W = D.dyn_weights(cfg)
    p = M.dyn_params_from_config(load_config("dynamic_car"))
    B, N = sample_vehicles, C3_N
    x = np.array(x0[:B], np.float64)
    xbar = np.ones((B, N, C3_NX)); xbar[..., 0] += 3
    ubar = np.zeros((B, N, 2))
    with threadpool_limits(limits=1):
        t0 = time.perf_counter()
        for _ in range(sample_steps):
            ds = np.empty((B, N)); kap = np.empty((B, N))
            for b in range(B):
                ds[b], kap[b] = D.dyn_horizon_params(x[b], xbar[b].T, C5_MPC_DT, N, track.k_periodic)
            r = D.dyn_sqp_solve(x, ubar, kap, ds, p, W, "fiala")
            ubar, xbar = r["u_star"], r["x_star"]
            x = M.dyn_transition(x, r["u0"], track.k_periodic(x[:, 4]), 0.05, p, "fiala")
        dt = time.perf_counter() - t0
    return {"value": B * sample_steps / dt, "unit": "vehicle-steps/s", "cores": 1, "kind": "port",
            "sample": f"{B} vehicles x {sample_steps} closed-loop steps of the C5 job through the oracle "
                      f"(horizon + 3-iteration SQP + RK4 plant, numpy fp64, 1 thread) in {dt:.2f} s"}


def run_c5(args, dev, stream, rank, world, dist):
    """BASELINE config 5: closed-loop Monte-Carlo, 8192 vehicles x 500 steps on ippodromo,
    dynamic-bicycle (Fiala) NMPC N = 40 + fp64 RK4 plant, all on the device (vc_simulate).
    The 8192 vehicles are split into contiguous shards over the ranks (strong scaling)."""
    import numpy as np
    import torch

    from vcmpc import _abi
    from vcmpc.config import load_config
    from vcmpc.environment import Track
    from vcmpc.models import DynamicCar
    from vcmpc.simulation import BatchedRacingSimulator
    from vcmpc.workload import C5_MPC_DT, closed_loop_states, shard

    track = Track.load("ippodromo")
    x_all = closed_loop_states(args.c5_vehicles, track.length, seed=args.seed)
    lo, hi = shard(args.c5_vehicles, rank, world)
    B, K = hi - lo, args.c5_steps
    cfg = load_config("dynamic_mpc")
    cfg["mpc_dt"] = C5_MPC_DT
    car = DynamicCar(load_config("dynamic_car"), track, tyre="fiala")
    sim = BatchedRacingSimulator(car, cfg, track, batch=B, device=dev.index)
    sim.ctx.set_stream(stream.cuda_stream)
    sim.reset(x_all[lo:hi])
    sim.run(3, log=False)                      # warm-up (module load, first-touch)
    sim.reset(x_all[lo:hi])
    sim._init_warm_start(args.seed)
    sim.nfail.zero_()
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    dist.barrier()
    torch.cuda.synchronize(dev)
    leg_push("c5")
    t0 = time.perf_counter()
    ev[0].record(stream)
    log_x, _, nfail = sim.ctx.simulate(sim.x, sim.xbar, sim.ubar, K, sim.mpc_dt, sim.dt, log=True, nfail=sim.nfail)
    ev[1].record(stream)
    torch.cuda.synchronize(dev)
    leg_pop()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    gpu_ms = ev[0].elapsed_time(ev[1])
    ey = log_x[:, :, 5].abs()
    on_track = float((ey.max(dim=0).values < track.width / 2).double().mean())
    max_ey = float(ey.max())
    progress = float((log_x[-1, :, 4] - log_x[0, :, 4]).mean())
    nf = float(nfail.sum())
    del log_x
    vsteps, elapsed_max, gpu_ms_max = dist.aggregate(float(B * K), elapsed, gpu_ms, dev)
    out = {"metric": "closed-loop vehicle-steps/s (N=40 NMPC solve + fp64 plant per vehicle-step)",
           "value": vsteps / elapsed_max, "unit": "vehicle-steps/s", "solves_per_s": vsteps / elapsed_max,
           "steps": K, "ms_per_step": elapsed_max / K * 1e3, "gpu_ms_total": gpu_ms_max,
           "dtype": ("f64" if sim.ctx.dtype == _abi.VC_F64 else "f32") + " solve, f64 plant",
           "scaling": "strong",
           "config": {"workload": f"C5 closed loop on ippodromo: {args.c5_vehicles} vehicles x {K} steps (dt 0.05 s), "
                                  f"dynamic-bicycle (Fiala) single-track NMPC N={C3_N}, mpc_dt {C5_MPC_DT}, "
                                  f"3 SQP iterations", "vehicles_total": args.c5_vehicles, "vehicles_per_gpu": B,
                      "horizon": C3_N, "parallelism": f"dp{world} (contiguous vehicle shards)"},
           "closed_loop_rank0": {"on_track_frac": on_track, "max_abs_ey": max_ey, "mean_progress_m": progress,
                                 "nonsolved_frac": nf / (B * K)}}
    return out, x_all, track


# the reference's only published numbers: per-step wall time of command + drive for ONE vehicle
# (simulation/racing.py:231-233, CasADi/IPOPT + HSL MA27 on one unrecorded CPU thread; medians of
# experiments/data/*/*_elapsed.npy)
RECORDED_IPOPT_MEDIAN_MS = {"singletrack_n50": 55.7, "singletrack_n60": 75.4, "cascaded_n20_m15": 33.4,
                            "cascaded_n20_m35": 39.3}


def run_latency(args, dev):
    """Single-vehicle latency of the drop-in controllers: one command(state) + car.drive(action)
    per step (racing.py:231-233 / kinracing.py:283-290), host pointers, one vehicle, closed loop on
    ippodromo; median / p90 / mean over `calls` steps after 20 warm-up steps.  Config: the
    reference's own controller yamls (kinematic N = 20 and kinematic.yaml's N = 50, obstacles off;
    single-track N = 50 / 60 = the recorded singletrack runs; cascaded 20 + 15 / 20 + 40)."""
    import numpy as np

    from vcmpc.config import load_config
    from vcmpc.controllers import CascadedMPC, KinematicMPC
    from vcmpc.environment import Track
    from vcmpc.models import DynamicCar, DynamicPointMass, KinematicCar
    track = Track.load("ippodromo")
    calls = args.latency_calls

    def kin(N):
        cfg = load_config("kinematic_mpc")
        cfg["horizon"], cfg["obstacles"] = N, False
        car = KinematicCar(load_config("kinematic_car"), track)
        car.state = car.create_state(v=5.0, s=1.0)
        return car, KinematicMPC(car, cfg)

    def dyn(cfg_name, N, M=None):
        cfg = load_config(cfg_name)
        cfg["horizon"], cfg["obstacles"] = N, False
        if M is not None:
            cfg["horizon_pm"] = M
        car = DynamicCar(load_config("dynamic_car"), track, tyre="fiala")
        car.state = car.create_state(Ux=8.0, s=1.0)
        return car, CascadedMPC(car, DynamicPointMass(load_config("dynamic_car"), track), cfg)

    legs = {"kinematic_n20": lambda: kin(20), "kinematic_n50": lambda: kin(50),
            "singletrack_n50": lambda: dyn("singletrack_mpc", 50), "singletrack_n60": lambda: dyn("singletrack_mpc", 60),
            "cascaded_n20_m15": lambda: dyn("cascaded_mpc", 20, 15), "cascaded_n20_m35": lambda: dyn("cascaded_mpc", 20, 35),
            "cascaded_n20_m40": lambda: dyn("cascaded_mpc", 20, 40)}
    out = {}
    for name, make in legs.items():
        try:
            np.random.seed(31)
            car, mpc = make()
            ts, solved = [], 0
            for i in range(20 + calls):
                t0 = time.perf_counter()
                a = mpc.command(car.state)
                car.drive(a)
                dt = time.perf_counter() - t0
                if i >= 20:
                    ts.append(dt)
                    solved += int(np.asarray(mpc.status).reshape(-1)[0] == 0)
            ts = np.array(ts) * 1e3
            out[name] = {"median_ms": float(np.median(ts)), "p90_ms": float(np.percentile(ts, 90)),
                         "mean_ms": float(ts.mean()), "calls": calls, "solved_frac": solved / calls,
                         "s_end_m": float(car.state.values[2 if name.startswith("kin") else 4])}
            if name in RECORDED_IPOPT_MEDIAN_MS:
                out[name]["recorded_ipopt_median_ms"] = RECORDED_IPOPT_MEDIAN_MS[name]
        except Exception as e:  # reported, never fatal
            out[name] = {"error": f"{type(e).__name__}: {e}"}
    out["note"] = ("one vehicle, command(state) + drive(action) per step through the drop-in controllers "
                   "(host numpy in/out, H2D + one solve launch + D2H per command; drive = the device plant "
                   "step), closed loop on ippodromo from s = 1 m; recorded_ipopt_median_ms = the reference's "
                   "recorded CasADi/IPOPT medians (experiments/data, unrecorded CPU) -- historical context, "
                   "not a same-host comparison; cascaded_n20_m40 (cascaded.yaml's shape) has no recorded "
                   "counterpart among the recorded runs' horizons")
    return out


def main():
    args = parse()
    from vcmpc import dist
    if dist.needs_launch(args.gpus):
        # `bench.py --gpus N` outside torchrun: start N ranks of this same command (one
        # process per GPU, LOCAL_RANK = GPU index) before anything touches the GPU
        sys.exit(dist.launch([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], args.gpus))
    if args.dry_run:
        return dry_run(args)
    import numpy as np
    import torch

    from vcmpc import Context, _abi
    from vcmpc.config import load_config
    from vcmpc.workload import kinematic_batch

    rank, local, world = dist.env_rank()
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init("nccl", dev)

    B = args.batch
    data = kinematic_batch(B, N=N_HORIZON, seed=args.seed + 7919 * rank)
    t = {k: torch.from_numpy(v).to(dev) for k, v in data.items()}
    ubar0 = t["ubar"].clone()
    ctx = Context(model=_abi.VC_MODEL_KINEMATIC, N=N_HORIZON, max_batch=B, device=local,
                  kin_car=load_config("kinematic_car"), kin_mpc=load_config("kinematic_mpc"))
    # a dedicated stream: the default torch stream is the null stream (handle 0),
    # which vc_set_stream would read as "the context's own stream"
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    xbar = torch.empty((B, N_HORIZON + 1, NX), dtype=torch.float64, device=dev)
    u0 = torch.empty((B, NU), dtype=torch.float64, device=dev)
    status = torch.empty((B,), dtype=torch.int32, device=dev)
    iters = torch.empty((B,), dtype=torch.int32, device=dev)

    def step(ev=None):
        # every step solves the same problems from the same warm start: vc_solve_from reads it from
        # ubar0 (left unchanged) and writes u* to t["ubar"] (ABI 13; round 5 restored it with a
        # 328 KB device copy before each in-place vc_solve, 4 % of the step)
        if ev is not None:
            ev[0].record(stream)
        ctx.solve_from(t["x0"], t["kappa"], t["ds"], ubar0, t["ubar"], xbar, u0, status, iters)
        if ev is not None:
            ev[1].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    dist.barrier()
    torch.cuda.synchronize(dev)
    leg_push("c2")
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(events[i])
    torch.cuda.synchronize(dev)
    leg_pop()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    st = status.cpu().numpy()
    it = iters.cpu().numpy()
    # polish rounds per problem (untimed diagnostic call on the same problems): each round is a
    # normal-matrix build + factorisation + solves, the work of one interior-point iteration
    t["ubar"].copy_(ubar0)
    dg = ctx.solve(t["x0"], t["kappa"], t["ds"], t["ubar"], xbar, u0, status, iters, diag=True)[5]
    polish_rounds = float(dg[:, 3].double().mean().item())
    # PCIe-inclusive rate of the host-pointer path (VC_HOST_PTRS: H2D, solve, D2H)
    # -- reported beside `value`, never as it (DESIGN.md "Measurement")
    ctx.set_stream(None)
    host = {k: v.copy() for k, v in data.items()}
    ctx.solve(host["x0"], host["kappa"], host["ds"], host["ubar"].copy())
    reps = max(3, min(args.steps, 10))
    th = time.perf_counter()
    for _ in range(reps):
        ctx.solve(host["x0"], host["kappa"], host["ds"], host["ubar"].copy())
    host_rate = B * reps / (time.perf_counter() - th)
    solves, elapsed_max, kern_ms_max = dist.aggregate(float(B * args.steps), elapsed, kern_ms, dev)
    c4 = None
    if not args.no_c4:
        try:
            c4 = run_c4(args, dev, stream, rank, world, dist, max(3, args.steps // 4))
        except Exception as e:  # the headline line must still print
            c4 = {"error": f"{type(e).__name__}: {e}"}
    kin_legs = {}
    if not args.no_kin_legs:
        for name, N, solver in (("c2_riccati", N_HORIZON, 1), ("kinematic_n50", 50, 1)):
            try:
                kin_legs[name] = run_kin_leg(args, dev, stream, rank, dist, max(3, args.steps // 4), N, solver, B, leg=name)
            except Exception as e:
                kin_legs[name] = {"error": f"{type(e).__name__}: {e}"}
    c3 = c3_data = c3f = c3s = st60 = st60c = None
    if not args.no_c3:
        # C3 on its parity path: the fp64 stagewise-Riccati kernel meets the 1e-5 bar and is the
        # faster one; the fp32 condensed kernel BASELINE names is reported beside it (c3_f32, a
        # measured precision floor above 1e-5: DESIGN 2b)
        try:
            c3, c3_data = run_c3(args, dev, stream, rank, dist, max(3, args.steps // 4), f64=True)
        except Exception as e:  # the headline line must still print
            c3 = {"error": f"{type(e).__name__}: {e}"}
        if c3 is not None and "error" not in c3:
            c3["dtype_note"] = ("BASELINE config 3 names fp32; C3 runs in fp64 (the reference's own NLP "
                                "precision): the fp32 condensed kernel (csrc/dyn_sqp.hip) cannot meet the "
                                "1e-5 bar -- its QP data, linearised over 40 RK4 stages in fp32, already "
                                "carries errors that condition numbers of 1e4-1e6 amplify past 1e-5 (DESIGN "
                                "2b: 1.4e-5 .. 2.5e-3 measured) -- and it is slower (196 K vs 377 K solves/s, "
                                "r03); measured beside it under c3_f32")
        if not args.no_c3_f32:
            try:
                c3f, _ = run_c3(args, dev, stream, rank, dist, max(3, args.steps // 4), leg="c3_f32")
            except Exception as e:
                c3f = {"error": f"{type(e).__name__}: {e}"}
        if not args.no_c3_survey:
            try:
                c3s, _ = run_c3(args, dev, stream, rank, dist, max(3, args.steps // 4), f64=True, leg="c3_survey",
                                ranges="survey")
            except Exception as e:
                c3s = {"error": f"{type(e).__name__}: {e}"}
        try:
            st60, _ = run_c3(args, dev, stream, rank, dist, max(3, args.steps // 4), f64=True, N=60,
                             cfg_name="singletrack_mpc", leg="singletrack_n60_f64")
        except Exception as e:
            st60 = {"error": f"{type(e).__name__}: {e}"}
        # what a reference-equivalent answer costs: the converged SQP setting of the replay against
        # IPOPT's recorded solutions (tests/test_gpu_replay.py: prox 0.01, 40 SQP iterations)
        try:
            if args.no_converged:
                raise _Skip()
            st60c, _ = run_c3(args, dev, stream, rank, dist, 2, f64=True, N=60, cfg_name="singletrack_mpc",
                              qp=CONVERGED_QP, leg="singletrack_n60_converged")
        except _Skip:
            pass
        except Exception as e:
            st60c = {"error": f"{type(e).__name__}: {e}"}
    ca = ca_data = cac = None
    if not args.no_casc:
        try:
            ca, ca_data = run_casc(args, dev, stream, rank, dist, max(2, args.steps // 8))
        except Exception as e:
            ca = {"error": f"{type(e).__name__}: {e}"}
        try:
            if args.no_converged:
                raise _Skip()
            cac, _ = run_casc(args, dev, stream, rank, dist, 2, qp=CONVERGED_QP, leg="cascaded_converged")
        except _Skip:
            pass
        except Exception as e:
            cac = {"error": f"{type(e).__name__}: {e}"}
    c5 = c5_aux = None
    if not args.no_c5:
        try:
            c5, *c5_aux = run_c5(args, dev, stream, rank, world, dist)
        except Exception as e:
            c5 = {"error": f"{type(e).__name__}: {e}"}

    lat = None
    if world == 1 and not args.no_latency:
        lat = run_latency(args, dev)

    if rank == 0:
        value = solves / elapsed_max
        achieved = BYTES_PER_SOLVE * B / (kern_ms / 1e3) / 1e9
        flops = FLOP_SWEEP + (float(it.mean()) + polish_rounds) * FLOP_ITER  # + the polish rounds
        flops_F = 0.42e6 + (float(it.mean()) + polish_rounds) * 0.28e6
        out = {
            "metric": "MPC solves/sec (batched, N=20)",
            "value": value,
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (seeded C2 sampler, vcmpc/workload.py: SURVEY 8(d)'s x0 / kappa / ubar "
                     "distributions; per-stage ds_n = 0.03 vbar_n + 0.5 from the warm start's speed "
                     "prediction, kinematic_mpc.py:178-182; problems whose warm-start rollout drops to "
                     "v <= 1 m/s or reaches |epsi| >= 1.2 rad are re-drawn)"),
            "config": {"workload": f"C2 kinematic-bicycle LTV-MPC, B={B} per GPU, N={N_HORIZON}, fp64",
                       "batch_per_gpu": B, "global_batch": B * world, "horizon": N_HORIZON,
                       "parallelism": f"dp{world} (independent shards)"},
            # the binding roofline is fp64 compute ("not HBM").  The kernel's fp64 work
            # splits between the VALU and the matrix cores: the v_mfma_f64_16x16x4_f64 tiles (the
            # normal-matrix build C'DC and the blocked factorisation's trailing updates) execute
            # 0.93 MFLOP per solve -- as much as the whole structure-exploiting count (r05 PMC,
            # `mfma` below; a tile pads its triangle, so part of that is padding).  Both units peak
            # at 78.6 TFLOP/s in fp64 on MI355X, so that is the peak.  `frac` prices SURVEY 8(d)'s
            # dense count F = 0.42 M + (iterations + polish rounds) x 0.28 M FLOP per solve; the
            # structure-exploiting count and the matrix-core share are reported beside it
            "roofline": {"bound": "fp64", "achieved": flops_F * B / (kern_ms / 1e3) / 1e12, "peak": FP64_VALU_PEAK,
                         "unit": "TFLOP/s", "frac": flops_F * B / (kern_ms / 1e3) / 1e12 / FP64_VALU_PEAK,
                         "traffic": pmc_traffic(B),
                         "traffic_unit": f"HBM bytes/launch (rocprofv3 2 x FETCH_SIZE + WRITE_SIZE: the gfx950 read correction, calibrated for 8 B/lane in profiles/r05/pmc_calibration_r05y.txt; {os.path.relpath(PMC_SUMMARY, ROOT)})",
                         "kernel": "kin_ltv_kernel<20>", "kernel_ms": kern_ms, "flops_per_solve": flops_F,
                         "flops_note": "SURVEY 8(d) F: 0.42 MFLOP sweep + (IPM iterations + polish rounds) x 0.28 MFLOP; a polish round (normal-matrix build + factorisation + solves) is priced as one iteration",
                         "polish_rounds_mean": polish_rounds,
                         "count": "dense-equivalent: F prices the dense condensing GEMM and dense C'DC the "
                                  "kernel does not execute; the executed (structure-exploiting) count is "
                                  "`structured`",
                         "structured": {"flops_per_solve": flops,
                                        "achieved": flops * B / (kern_ms / 1e3) / 1e12,
                                        "frac": flops * B / (kern_ms / 1e3) / 1e12 / FP64_VALU_PEAK,
                                        "note": "the build's structure-exploiting count (triangular rows, "
                                                "n^3/3 Cholesky): sweep + (IPM iterations + 1) x iteration"},
                         "mfma": _mfma_live(pmc_mfma(B), kern_ms),
                         "hbm": {"achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": achieved / HBM_PEAK_GBS, "algorithmic_bytes": BYTES_PER_SOLVE * B,
                                 "bytes_per_solve": BYTES_PER_SOLVE}},
            "host_ptr_solves_per_s": host_rate,
            "solver": {"solved_frac": float((st == 0).mean()), "iters_mean": float(it.mean()),
                       "iters_max": int(it.max())},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(data, min(args.cpu_sample, B))
            try:
                out["cpu_baseline_all_cores"] = cpu_baseline_all_cores(data, min(args.cpu_sample, B))
            except Exception as e:  # reported, never fatal: the GPU numbers stand alone
                out["cpu_baseline_all_cores"] = {"error": repr(e)}
            if c3_data is not None and "error" not in c3:
                c3["cpu_baseline"] = cpu_baseline_c3(c3_data, 8)
                try:
                    c3["cpu_baseline_all_cores"] = cpu_baseline_all_cores(c3_data, 0, kind="c3", per_worker=8)
                except Exception as e:
                    c3["cpu_baseline_all_cores"] = {"error": repr(e)}
            if ca_data is not None and "error" not in ca:
                ca["cpu_baseline"] = cpu_baseline_casc(ca_data, 4)
            if c5_aux and "error" not in c5:
                from oracle.track import load_track
                otrack = load_track(os.path.join(ROOT, "vehicle-control_amd", "config", "tracks", "ippodromo.yaml"))
                c5["cpu_baseline"] = cpu_baseline_c5(c5_aux[0], otrack)
        out.update(kin_legs)
        if c4 is not None:
            out["c4"] = c4
        if c3 is not None:
            out["c3"] = c3
        if c3f is not None:
            out["c3_f32"] = c3f
        if c3s is not None:
            out["c3_survey"] = c3s
        if st60 is not None:
            out["singletrack_n60_f64"] = st60
        if st60c is not None:
            out["singletrack_n60_converged"] = st60c
        if ca is not None:
            out["cascaded"] = ca
        if cac is not None:
            out["cascaded_converged"] = cac
        if c5 is not None:
            out["c5"] = c5
        if lat is not None:
            out["latency"] = lat
        print(json.dumps(out), flush=True)
    ctx.close()
    dist.shutdown()


if __name__ == "__main__":
    main()
