"""CPU: the multi-GPU path's host logic at world size 2 over gloo -- rank discovery
from the torchrun environment, contiguous sharding of the batch, and the one
collective (sum of solves, max of elapsed / kernel time) -- as bench.py runs it
over RCCL on the GPU box."""
import os
import socket

import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "vehicle-control_amd"))
    from vcmpc import dist
    from vcmpc.workload import kinematic_batch, shard
    r, local, w = dist.init("gloo")
    B_total = 1000
    lo, hi = shard(B_total, r, w)
    d = kinematic_batch(hi - lo, seed=31 + 7919 * r)
    solves, elapsed, kern = dist.aggregate(float(hi - lo), 0.5 + r, 0.1 * (r + 1))
    dist.barrier()
    dist.shutdown()
    q.put((r, lo, hi, d["x0"].shape[0], solves, elapsed, kern))


@pytest.mark.timeout(120)
def test_two_rank_sharding_and_counter_reduce():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    (r0, lo0, hi0, n0, s0, e0, k0), (r1, lo1, hi1, n1, s1, e1, k1) = res
    assert (lo0, hi0, lo1, hi1) == (0, 500, 500, 1000) and n0 == n1 == 500
    assert s0 == s1 == 1000.0           # solves summed over ranks
    assert e0 == e1 == 1.5              # elapsed: max over ranks
    assert abs(k0 - 0.2) < 1e-12 and abs(k1 - 0.2) < 1e-12


@pytest.mark.timeout(240)
def test_bench_launcher_two_ranks_dry_run():
    """`bench.py --gpus 2` outside torchrun starts two ranks itself (vcmpc.dist.launch,
    the path the driver's `bench.py --gpus N` takes without a torchrun environment);
    --dry-run keeps the GPU out: each rank joins the gloo group, takes its C4 / C5
    shards, and rank 0 prints one JSON line with n_gpus = 2."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run",
                        "--c4-total", "20000"], env=env, capture_output=True, text=True, timeout=220)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    ranks = sorted(out["ranks"])
    assert [x[0] for x in ranks] == [0, 1] and [x[1] for x in ranks] == [0, 1]   # LOCAL_RANK = rank
    assert (ranks[0][2], ranks[0][3], ranks[1][2], ranks[1][3]) == (0, 10000, 10000, 20000)
    assert (ranks[0][4], ranks[0][5], ranks[1][4], ranks[1][5]) == (0, 4096, 4096, 8192)
    assert out["solves"] == 2 * 1024 + 20000 and abs(out["elapsed_max"] - 0.2) < 1e-12


def test_c4_shards_are_world_size_independent():
    """The C4 problem set is the same 65536 problems at every world size: rank r's shard
    at world w equals the matching slice of the one-rank set (chunked seeding)."""
    import importlib.util
    import numpy as np
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    total = 20000
    _, _, full = bench.c4_shard(total, 0, 1, 31)
    assert full["x0"].shape == (total, 6)
    for world in (2, 3, 8):
        for r in range(world):
            lo, hi, d = bench.c4_shard(total, r, world, 31)
            for k in full:
                np.testing.assert_array_equal(d[k], full[k][lo:hi])
