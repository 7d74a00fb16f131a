"""Multi-GPU plumbing: one process per GPU, stripes partitioned by bytes, no
collective on the data path (stripes are independent).  The only
cross-rank traffic is the timing handshake (barrier + max over ranks).

Backend: "nccl" (RCCL on ROCm) for HIP devices, "gloo" for CPU ranks (tests).
Rendezvous comes from torch.distributed.run's env (MASTER_ADDR=127.0.0.1).
"""
from __future__ import annotations

import os

import torch

from .batch import partition_by_bytes


def backend() -> str:
    """nccl (RCCL) across GPUs; ELECT_BENCH_BACKEND=gloo lets several ranks share
    one GPU to rehearse the multi-rank flow (timing handshake over the host)."""
    return os.environ.get("ELECT_BENCH_BACKEND", "nccl")


def setup(device_type: str = "cuda"):
    """Init the process group if WORLD_SIZE > 1.  Returns (world, rank, device_index)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if device_type == "cuda" and backend() == "gloo":
        local %= max(1, torch.cuda.device_count())  # rehearsal: ranks may share a device
    if world > 1 and not torch.distributed.is_initialized():
        if device_type == "cuda" and backend() == "nccl":
            torch.cuda.set_device(local)
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            if device_type == "cuda":
                torch.cuda.set_device(local)
            torch.distributed.init_process_group("gloo")
    elif device_type == "cuda":
        torch.cuda.set_device(local)
    return world, rank, local


def barrier(world: int) -> None:
    if world > 1:
        torch.distributed.barrier()


def max_over_ranks(x: float, world: int, device_type: str = "cuda") -> float:
    if world == 1:
        return x
    on_gpu = device_type == "cuda" and backend() == "nccl"
    t = torch.tensor([x], dtype=torch.float64, device="cuda" if on_gpu else "cpu")
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def shard(sizes, world: int, rank: int):
    """This rank's contiguous, byte-balanced block of independent stripes."""
    return partition_by_bytes(sizes, world, rank)


def teardown(world: int) -> None:
    if world > 1 and torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
