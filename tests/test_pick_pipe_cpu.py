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
