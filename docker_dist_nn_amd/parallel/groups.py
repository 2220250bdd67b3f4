"""Process mesh for PP x DP: one OS process (rank) per GPU.

Rank layout: ``rank = replica * pp + stage`` -- each data-parallel replica is one complete
pipeline of ``pp`` consecutive ranks. On an MI355X node every GPU pair has a direct xGMI link,
so the mapping only has to keep the groups regular.

Groups created (all ranks call ``new_group`` in the same order, as torch requires):
  * per replica, TWO pipeline groups -- one that only carries forward activations
    (stage s -> s+1) and one that only carries backward gradients (s+1 -> s). Keeping the
    directions on separate communicators (separate RCCL streams) means a blocked send in one
    direction can never stall a receive in the other, which is what makes posting every
    receive of a step up front deadlock-free without grouping sends and receives.
  * per stage, one data-parallel group over the replicas (gradient all-reduce).

Backend: ``nccl`` (= RCCL on ROCm, over xGMI) for GPU tensors, ``gloo`` for CPU runs/tests.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class Mesh:
    rank: int
    world: int
    pp: int
    dp: int
    stage: int
    replica: int
    pipe_ranks: list[int] = field(default_factory=list)
    fwd_group: Optional[object] = None
    bwd_group: Optional[object] = None
    dp_group: Optional[object] = None
    dp_ranks: list[int] = field(default_factory=list)
    backend: str = "gloo"

    @property
    def prev_rank(self) -> Optional[int]:
        return self.pipe_ranks[self.stage - 1] if self.stage > 0 else None

    @property
    def next_rank(self) -> Optional[int]:
        return self.pipe_ranks[self.stage + 1] if self.stage + 1 < self.pp else None


def init_distributed(backend: str = "auto", timeout_s: float = 600.0) -> tuple[int, int, str]:
    """Initialise torch.distributed from torchrun env vars (RANK/WORLD_SIZE/MASTER_*)."""
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size(), dist.get_backend()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if backend == "auto":
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    kwargs = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
    if backend == "nccl":
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        kwargs["device_id"] = torch.device("cuda", local)
    dist.init_process_group(**kwargs)
    return rank, world, backend


def build_mesh(pp: int, dp: int) -> Mesh:
    rank, world = dist.get_rank(), dist.get_world_size()
    if pp * dp != world:
        raise ValueError(f"pp({pp}) x dp({dp}) must equal world size {world}")
    backend = dist.get_backend()
    stage, replica = rank % pp, rank // pp
    m = Mesh(rank, world, pp, dp, stage, replica, backend=backend)
    for r in range(dp):
        ranks = list(range(r * pp, (r + 1) * pp))
        fg = dist.new_group(ranks) if pp > 1 else None
        bg = dist.new_group(ranks) if pp > 1 else None
        if r == replica:
            m.pipe_ranks, m.fwd_group, m.bwd_group = ranks, fg, bg
    for s in range(pp):
        ranks = [r * pp + s for r in range(dp)]
        g = dist.new_group(ranks) if dp > 1 else None
        if s == stage:
            m.dp_group, m.dp_ranks = g, ranks
    return m
