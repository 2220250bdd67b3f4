"""Trainer._pick_pipe's auto transport rules without a GPU: a schedule with
per-micro-batch weight gradients (zb, 1f1b_w) has no native multi-rank step, so DNN_PIPE=auto
must pick the message transport for it instead of building a relayed IPC pipe that needs one."""
import types

import pytest
import torch

from docker_dist_nn_amd.engine import trainer as tmod


@pytest.mark.parametrize("schedule", ["zb", "1f1b_w"])
def test_auto_transport_falls_back_for_per_micro_wgrad_schedules(monkeypatch, schedule):
    made = []
    monkeypatch.setattr(tmod, "DistPipe", lambda mesh, st: made.append("dist") or "dist-pipe")
    monkeypatch.setattr(tmod, "IpcPipe",
                        lambda *a, **k: pytest.fail("auto built an IPC pipe for " + schedule))
    monkeypatch.setenv("DNN_PIPE", "auto")
    tr = tmod.Trainer.__new__(tmod.Trainer)
    tr.device = torch.device("cuda", 0)  # only .type is read before the transport choice
    tr.schedule = schedule
    tr._peers_mappable = lambda mesh: True
    mesh = types.SimpleNamespace(pp=3, dp=1, backend="nccl")
    assert tr._pick_pipe(mesh, None, "bf16") == "dist-pipe"
    assert made == ["dist"] and schedule in tr.transport_reason


def _queue_check_worker(rank, world, port, out):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DNN_PIPE="auto",
                      DNN_IPC_RELAYS="2", DNN_IPC_VERIFY="0", GPU_MAX_HW_QUEUES="6")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    closed = []

    class FakeIpc:  # rank 1 carries 3 relay duties (4 + 3 > 6 queues), rank 0 none
        def __init__(self, mesh, st, relays):
            self.duties = [object()] * (3 if rank == 1 else 0)
            self.k = relays

        def close(self):
            closed.append(rank)

    tmod.IpcPipe = FakeIpc
    tmod.DistPipe = lambda mesh, st: "dist-pipe"
    tr = tmod.Trainer.__new__(tmod.Trainer)
    tr.device = torch.device("cuda", 0)
    tr.schedule = "1f1b_lh"
    tr._peers_mappable = lambda mesh: True
    mesh = types.SimpleNamespace(pp=2, dp=1, backend="nccl")
    got = tr._pick_pipe(mesh, None, "bf16")
    with open(f"{out}/r{rank}", "w") as f:
        f.write(f"{got if isinstance(got, str) else 'ipc'}|{bool(closed)}|{tr.transport_reason}")
    dist.barrier()
    dist.destroy_process_group()


def test_queue_check_is_agreed_across_ranks(tmp_path):
    """with an explicit DNN_IPC_RELAYS the ranks carry different relay duty
    counts; the hardware-queue check must fall back on EVERY rank when the busiest rank does
    not fit, or the ranks that keep IPC write into relay slots the others freed."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_queue_check_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    res = [(tmp_path / f"r{r}").read_text().split("|") for r in range(2)]
    assert all(r[0] == "dist-pipe" and r[1] == "True" for r in res), res
    assert all("busiest rank" in r[2] for r in res), res
