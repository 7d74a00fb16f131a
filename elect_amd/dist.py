"""Multi-GPU plumbing: one process per GPU, stripes partitioned by bytes, no
collective on the data path (stripes are independent).  The only
cross-rank traffic is the timing handshake (barrier, max over ranks, and the
per-rank records rank 0 prints), and it runs over gloo on the host: no RCCL
communicator is ever created, so an 8-rank run has no RCCL init to fail.

Rendezvous comes from torch.distributed.run's env (MASTER_ADDR=127.0.0.1).
Ranks map to devices by LOCAL_RANK.  More ranks than visible devices is an
error unless ELECT_BENCH_SHARE_GPU=1 (or the older ELECT_BENCH_BACKEND=gloo),
which rehearses an N-rank run with ranks sharing one GPU.
"""
from __future__ import annotations

import os
from datetime import timedelta

import torch

from .batch import partition_by_bytes


def share_devices() -> bool:
    return os.environ.get("ELECT_BENCH_SHARE_GPU") == "1" or os.environ.get("ELECT_BENCH_BACKEND") == "gloo"


def env_world() -> tuple[int, int, int]:
    """(world, rank, local_rank) from the launcher's environment (1, 0, 0 if unset)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def setup(device_type: str = "cuda"):
    """Select this rank's device and, if WORLD_SIZE > 1, join the gloo group.
    Returns (world, rank, device_index)."""
    world, rank, local = env_world()
    if device_type == "cuda":
        ndev = torch.cuda.device_count()  # counts devices without initialising HIP
        if ndev < 1:
            raise RuntimeError("no HIP device visible")
        if local >= ndev:
            if not share_devices():
                raise RuntimeError(f"local rank {local} has no device of its own ({ndev} visible); "
                                   "set ELECT_BENCH_SHARE_GPU=1 to rehearse with ranks sharing devices")
            local %= ndev
        torch.cuda.set_device(local)
    if world > 1 and not torch.distributed.is_initialized():
        torch.distributed.init_process_group("gloo", timeout=timedelta(minutes=10))
    return world, rank, local


def barrier(world: int) -> None:
    if world > 1:
        torch.distributed.barrier()


def max_over_ranks(x: float, world: int, device_type: str = "cuda") -> float:
    """Max of a host scalar over ranks (gloo; device_type kept for callers)."""
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def gather(obj, world: int) -> list:
    """Every rank's obj, in rank order, on every rank (gloo, host objects)."""
    if world == 1:
        return [obj]
    out = [None] * world
    torch.distributed.all_gather_object(out, obj)
    return out


def shard(sizes, world: int, rank: int):
    """This rank's contiguous, byte-balanced block of independent stripes."""
    return partition_by_bytes(sizes, world, rank)


def teardown(world: int) -> None:
    if world > 1 and torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
