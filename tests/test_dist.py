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
