"""Data-parallel step on the GPU path (native segment replay) with two ranks sharing cuda:0
(gloo: RCCL needs one GPU per rank, which a one-GPU box does not have). Covers the deferred
update (per-layer forward segments F{j}.L{i}, split optimizer segments O{a}-{b} / OADV): the
ranks must reproduce a single-process trainer on the same global batch."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SPEC = "784-512-256-128-10"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(rows):
    from docker_dist_nn_amd.data import synthetic_mnist

    x, y = synthetic_mnist(rows, seed=9)
    xt = torch.zeros(rows, 832, dtype=torch.bfloat16)
    xt[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    return xt, torch.from_numpy(y).to(torch.int32)


def _worker(rank, world, port, optim, defer, steps, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DNN_DP_DEFER=defer)
    import torch.distributed as dist

    from docker_dist_nn_amd import MLPSpec
    from docker_dist_nn_amd.engine import OptimConfig, Trainer
    from docker_dist_nn_amd.parallel.groups import build_mesh

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mesh = build_mesh(1, world)
    tr = Trainer(MLPSpec.parse(SPEC), micro_batch=1024, num_micro=1, mesh=mesh, device=dev,
                 optim=OptimConfig(name=optim, lr=0.05 if optim == "sgd" else 1e-3))
    assert tr.native_exec
    xt, yt = _batch(1024 * world)
    xs, ys = xt[rank * 1024:(rank + 1) * 1024].to(dev), yt[rank * 1024:(rank + 1) * 1024].to(dev)
    for _ in range(steps):
        tr.set_batch(xs, ys)
        tr.step()
    for k, (w, _b) in tr.local_weights().items():
        np.save(os.path.join(out_dir, f"w{k}_r{rank}.npy"), w)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("optim,defer", [("sgd", "1"), ("adam", "1"), ("sgd", "0")])
def test_dp2_native_matches_single_process(dev, optim, defer):
    from docker_dist_nn_amd import MLPSpec
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    world, steps = 2, 3
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), optim, defer, steps, d),
                           nprocs=world, join=True, start_method="spawn")
        tr = Trainer(MLPSpec.parse(SPEC), micro_batch=1024, num_micro=world, device=dev,
                     optim=OptimConfig(name=optim, lr=0.05 if optim == "sgd" else 1e-3))
        xt, yt = _batch(1024 * world)
        for _ in range(steps):
            tr.set_batch(xt.to(dev), yt.to(dev))
            tr.step()
        for k, (w, _b) in tr.local_weights().items():
            for r in range(world):
                got = np.load(os.path.join(d, f"w{k}_r{r}.npy"))
                np.testing.assert_allclose(got, w, rtol=2e-3, atol=2e-4)


def _pp_worker(rank, world, port, pipe, steps, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DNN_PIPE=pipe)
    import torch.distributed as dist

    from docker_dist_nn_amd import MLPSpec
    from docker_dist_nn_amd.engine import OptimConfig, Trainer
    from docker_dist_nn_amd.parallel.comm import DistPipe, IpcPipe
    from docker_dist_nn_amd.parallel.groups import build_mesh

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mesh = build_mesh(world, 1)
    tr = Trainer(MLPSpec.parse(SPEC), micro_batch=512, num_micro=4, mesh=mesh, device=dev,
                 schedule="1f1b", optim=OptimConfig(lr=0.05))
    assert isinstance(tr.pipe, IpcPipe if pipe == "ipc" else DistPipe)
    xt, yt = _batch(2048)
    for _ in range(steps):
        tr.set_batch(xt.to(dev) if tr.first else None, yt.to(dev) if tr.last else None)
        tr.step()
    torch.cuda.synchronize()
    for k, (w, _b) in tr.local_weights().items():
        np.save(os.path.join(out_dir, f"{pipe}_w{k}.npy"), w)
    dist.barrier()
    dist.destroy_process_group()


def test_pp2_ipc_pipe_bitwise_equals_rccl_path(dev):
    """Two pipeline stages as two processes on cuda:0: activations/gradients through IPC-mapped
    peer buffers + stream-ordered flags (DNN_PIPE=ipc) give bit-identical weights to the
    message-passing transport over 3 steps x 4 micro-batches."""
    world, steps = 2, 3
    with tempfile.TemporaryDirectory() as d:
        for pipe in ("rccl", "ipc"):  # "rccl" runs DistPipe (gloo-staged on one GPU)
            mp.start_processes(_pp_worker, args=(world, _free_port(), pipe, steps, d),
                               nprocs=world, join=True, start_method="spawn")
        for k in range(4):
            a = np.load(os.path.join(d, f"rccl_w{k}.npy"))
            b = np.load(os.path.join(d, f"ipc_w{k}.npy"))
            assert np.array_equal(a, b), k
