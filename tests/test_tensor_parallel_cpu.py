"""Tensor parallelism (parallel/tensor.py: Megatron column / row splits) on CPU with gloo
(127.0.0.1): a TP group trained on a replicated batch must reproduce the single-process
trainer from the same initial weights (only fp32 summation order differs)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from docker_dist_nn_amd import MLPSpec
from docker_dist_nn_amd.data import synthetic_mnist
from docker_dist_nn_amd.engine import OptimConfig, Trainer
from docker_dist_nn_amd.parallel.tensor import TensorParallelMLP, layer_modes


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(rows):
    x, y = synthetic_mnist(rows, seed=11)
    return torch.from_numpy(x), torch.from_numpy(y)


OPT = OptimConfig(lr=0.1, momentum=0.9, weight_decay=1e-4)


def _worker(rank, world, port, spec, rows, steps, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tp = TensorParallelMLP(MLPSpec.parse(spec), rows=rows, tp=world, rank=rank,
                           device=torch.device("cpu"), optim=OPT)
    x, y = _batch(rows)
    losses = []
    for _ in range(steps):
        tp.set_batch(x, y)
        tp.step()
        losses.append(tp.loss())
    ws = tp.full_weights()
    if rank == 0:
        for k, (w, b) in enumerate(ws):
            np.save(os.path.join(out_dir, f"w{k}.npy"), w)
            np.save(os.path.join(out_dir, f"b{k}.npy"), b)
        np.save(os.path.join(out_dir, "loss.npy"), np.array(losses))
    dist.barrier()
    dist.destroy_process_group()


def test_layer_modes():
    assert layer_modes(1) == ["rep"]
    assert layer_modes(2) == ["col", "row"]
    assert layer_modes(3) == ["col", "row", "rep"]
    assert layer_modes(4) == ["col", "row", "col", "row"]


@pytest.mark.parametrize("spec,world", [("784-128-64-32-10", 2), ("784-96-10", 2),
                                        ("784-64-48-10", 4), ("784-256-128-64-10", 4)])
def test_tensor_parallel_matches_single_process(spec, world):
    rows, steps = 256, 3
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), spec, rows, steps, d),
                           nprocs=world, join=True, start_method="fork")
        tr = Trainer(MLPSpec.parse(spec), micro_batch=rows, num_micro=1, optim=OPT,
                     device=torch.device("cpu"))
        x, y = _batch(rows)
        xb = torch.zeros(rows, tr.stages[0].x_in.shape[1], dtype=torch.bfloat16)
        xb[:, :x.shape[1]] = x.to(torch.bfloat16)
        ref_loss = []
        for _ in range(steps):
            tr.set_batch(xb, y)
            tr.step()
            ref_loss.append(tr.loss())
        for k, (w, b) in tr.local_weights().items():
            np.testing.assert_allclose(np.load(os.path.join(d, f"w{k}.npy")), w,
                                       rtol=2e-3, atol=2e-4)
            np.testing.assert_allclose(np.load(os.path.join(d, f"b{k}.npy")), b,
                                       rtol=2e-3, atol=2e-4)
        np.testing.assert_allclose(np.load(os.path.join(d, "loss.npy")), ref_loss, rtol=1e-3)
