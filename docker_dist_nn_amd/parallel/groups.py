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
  * per link (stage s <-> s+1 of a replica), TWO 2-rank groups: the forward channel and the
    backward channel of the native RCCL step (parallel/native_step.py, ``streams`` form).
    RCCL orders the kernels of one communicator, so a channel with one sender and one receiver
    per communicator is what lets a receive run concurrently with the same rank's send in the
    same direction.
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
    # link channels of the native RCCL step: from/to the previous / next stage
    link_f_in: Optional[object] = None
    link_f_out: Optional[object] = None
    link_b_in: Optional[object] = None
    link_b_out: Optional[object] = None
    # this rank's groups in global creation order (communicator warm-up without deadlock)
    member_groups: list = field(default_factory=list)

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
            if fg is not None:
                m.member_groups += [fg, bg]
    for r in range(dp):
        for s in range(pp - 1):
            a, b = r * pp + s, r * pp + s + 1
            lf = dist.new_group([a, b])
            lb = dist.new_group([a, b])
            if rank == a:
                m.link_f_out, m.link_b_in = lf, lb
            elif rank == b:
                m.link_f_in, m.link_b_out = lf, lb
            if rank in (a, b):
                m.member_groups += [lf, lb]
    for s in range(pp):
        ranks = [r * pp + s for r in range(dp)]
        g = dist.new_group(ranks) if dp > 1 else None
        if s == stage:
            m.dp_group, m.dp_ranks = g, ranks
            if g is not None:
                m.member_groups.append(g)
    return m
