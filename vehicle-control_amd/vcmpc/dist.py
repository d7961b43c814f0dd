"""One process per GPU: rank discovery and the throughput-counter collective.

The solve path shards embarrassingly: each rank owns a contiguous
batch range and no data crosses GPUs.  The only collective is the end-of-run
reduction of a few counters (solves: sum; elapsed: max) -- RCCL over xGMI on the
GPU box (backend "nccl" is RCCL on ROCm), gloo in the CPU tests.
"""
from __future__ import annotations

import os


def env_rank():
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def needs_launch(nprocs: int) -> bool:
    """True when `nprocs` > 1 ranks were asked for but this process is not one of them
    (no WORLD_SIZE from torchrun or from `launch`)."""
    return nprocs > 1 and "WORLD_SIZE" not in os.environ


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(argv, nprocs: int, port: int | None = None, timeout: float | None = None) -> int:
    """Run `argv` (a full command, e.g. [sys.executable, "bench.py", ...]) as `nprocs`
    single-node ranks -- the torchrun environment (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR = 127.0.0.1, MASTER_PORT) set per child -- and return
    the first non-zero exit code (0 when every rank succeeded).  The children are
    started with subprocess (never exec) and the caller must not have touched the GPU:
    each rank binds its own device by LOCAL_RANK.  If a rank fails, the others are
    terminated so a collective cannot wait forever on the missing peer."""
    import subprocess
    import time
    port = port or _free_port()
    procs = []
    for r in range(nprocs):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs),
                   LOCAL_WORLD_SIZE=str(nprocs), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(list(argv), env=env))
    t0 = time.monotonic()
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        if timeout is not None and time.monotonic() - t0 > timeout and live:
            for q in live:
                q.kill()
            rc = rc or 124
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


def init(backend: str, device=None):
    """Initialise torch.distributed from the torchrun environment (world > 1 only)."""
    import torch.distributed as dist
    rank, local, world = env_rank()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return rank, local, world


def barrier():
    import torch.distributed as dist
    if dist.is_initialized():
        dist.barrier()


def aggregate(solves: float, elapsed_s: float, kernel_ms: float, device=None):
    """Sum of solves, max of elapsed and kernel time over ranks (a 3-float payload)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return solves, elapsed_s, kernel_ms
    s = torch.tensor([solves], dtype=torch.float64, device=device)
    m = torch.tensor([elapsed_s, kernel_ms], dtype=torch.float64, device=device)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    return float(s[0]), float(m[0]), float(m[1])


def shutdown():
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()
