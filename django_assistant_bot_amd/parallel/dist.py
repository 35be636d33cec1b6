"""Process-group bootstrap: one process per GPU, ``torch.distributed`` over RCCL (backend "nccl" on
ROCm) for GPU collectives on xGMI, gloo for CPU tests.  Reads RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT from the environment (torchrun convention).

The reference has no collective library at all; its fan-out is Celery/HTTP.  The
engine keeps Celery/HTTP as the control plane and uses these groups for the data plane:
  * ``world``  -- DP replicas of the RAG pipeline and the sharded vector index (all-gather merge);
  * ``tp``     -- tensor-parallel generator groups (two all-reduces per layer).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def env_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", 0))))


def force_group() -> bool:
    """``DAB_FORCE_GROUP=1``: form the process group even for a world of one rank, so every
    collective branch (RCCL device-tensor all_gather / all_to_all / gather / barrier, the node's
    control broadcasts) runs on a single GPU exactly as it does at 8."""
    return os.environ.get("DAB_FORCE_GROUP", "") not in ("", "0")


def grouped() -> bool:
    return dist.is_available() and dist.is_initialized()


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def init(backend: str | None = None, device_type: str | None = None, timeout_s: int = 600) -> DistInfo:
    """Initialise the default group when WORLD_SIZE > 1, or at any world size under
    ``DAB_FORCE_GROUP`` (idempotent).  GPU ranks bind cuda:LOCAL_RANK."""
    rank, world, local = env_world()
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cuda":
        # more ranks than GPUs (a multi-rank rehearsal on a 1-GPU box, with DAB_DIST_BACKEND=gloo:
        # RCCL refuses two ranks on one device) wrap around; one rank per GPU otherwise
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if backend is None:
        backend = os.environ.get("DAB_DIST_BACKEND") or ("nccl" if device_type == "cuda" else "gloo")
    if (world > 1 or force_group()) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1 and "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(_free_port())
        kw = {}
        if backend == "nccl":
            kw["device_id"] = device
        attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT")
        if attempt is not None and os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True":
            # restarted by torch.distributed.run after a rank fault: the agent's store outlives the
            # failed group, so every key of this attempt (group addresses, RCCL unique ids) gets its
            # own prefix instead of meeting the dead group's entries
            base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world, False,
                                 timeout=datetime.timedelta(seconds=timeout_s))
            kw["store"] = dist.PrefixStore(f"dab/attempt_{attempt}", base)
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return DistInfo(rank, world, local, device, backend if dist.is_initialized() else "none")


def barrier(info: DistInfo | None = None) -> None:
    if dist.is_available() and dist.is_initialized():
        if info is not None and info.backend == "nccl":
            dist.barrier(device_ids=[info.local_rank])
        else:
            dist.barrier()


def tp_groups(tp_size: int):
    """Consecutive ranks form tensor-parallel groups (one xGMI-connected node: any grouping is one hop).
    Returns (my_group, my_tp_rank, dp_rank)."""
    rank, world, _ = env_world()
    if tp_size <= 1:
        return None, 0, rank
    assert world % tp_size == 0, "WORLD_SIZE must be a multiple of the TP size"
    mine = None
    for start in range(0, world, tp_size):
        ranks = list(range(start, start + tp_size))
        g = dist.new_group(ranks)
        if rank in ranks:
            mine = g
    return mine, rank % tp_size, rank // tp_size


def max_over_ranks(value: float, device) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_floats(value: float, device) -> list[float]:
    """Every rank's ``value``, in rank order, on every rank (one all_gather; [value] without a group)."""
    if not (dist.is_available() and dist.is_initialized()):
        return [value]
    t = torch.tensor([value], dtype=torch.float64, device=device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]


def broadcast_int(value: int, group=None, device=None) -> int:
    """``value`` of the group's first rank on every rank of ``group`` (the world when None): keeps
    host-side decisions that depend on a rank's own clock (open-loop arrivals) identical across the
    ranks of a tensor-parallel engine, whose schedulers must see the same requests at the same step."""
    if not (dist.is_available() and dist.is_initialized()):
        return value
    src = dist.get_global_rank(group, 0) if group is not None else 0
    t = torch.tensor([value], dtype=torch.int64, device=device)
    dist.broadcast(t, src=src, group=group)
    return int(t.item())


def shutdown() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
