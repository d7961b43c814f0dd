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
