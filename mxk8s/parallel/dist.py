"""Process-group plumbing: one process per GPU, RCCL (``nccl`` backend) over xGMI.

Reads the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*).
Single-process runs never create a process group; every helper degrades to a
no-op so the same code path serves n = 1.  CPU tests use ``gloo``.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def world_info() -> tuple[int, int, int]:
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_distributed(backend: str = "nccl", device: torch.device | None = None,
                     timeout_s: float = 600.0) -> bool:
    """Initialise the default process group if WORLD_SIZE > 1.  Returns True if
    a group is (now) active."""
    world, rank, _ = world_info()
    if world <= 1:
        return False
    if dist.is_initialized():
        return True
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    kwargs = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
    if backend == "nccl" and device is not None:
        # binds the communicator to this rank's GPU up front (eager RCCL init)
        kwargs["device_id"] = device
    dist.init_process_group(**kwargs)
    return True


def active() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def barrier() -> None:
    if active():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def max_over_ranks(x: float, device: torch.device | None = None) -> float:
    if not active():
        return float(x)
    dev = device if (device is not None and dist.get_backend() == "nccl") else torch.device("cpu")
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, device: torch.device | None = None) -> float:
    if not active():
        return float(x)
    dev = device if (device is not None and dist.get_backend() == "nccl") else torch.device("cpu")
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
