"""Multi-process pipeline + data parallel on CPU (gloo): the distributed engine must reproduce
the single-process trainer on the same global batch. Ranks rendezvous on 127.0.0.1."""
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

SPEC = "784-128-64-32-10"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_batch(rows):
    x, y = synthetic_mnist(rows, seed=5)
    xt = torch.zeros(rows, 832, dtype=torch.bfloat16)
    xt[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    return xt, torch.from_numpy(y)


def _worker(rank, world, port, pp, dp, mb, nm, sched, steps, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from docker_dist_nn_amd.parallel.groups import build_mesh

    mesh = build_mesh(pp, dp)
    spec = MLPSpec.parse(SPEC)
    tr = Trainer(spec, micro_batch=mb, num_micro=nm, schedule=sched, mesh=mesh,
                 optim=OptimConfig(lr=0.1, momentum=0.9), device=torch.device("cpu"))
    R = mb * nm
    xt, yt = _global_batch(R * dp)
    xs, ys = xt[mesh.replica * R:(mesh.replica + 1) * R], yt[mesh.replica * R:(mesh.replica + 1) * R]
    losses = []
    for _ in range(steps):
        tr.set_batch(xs if tr.first else None, ys if tr.last else None)
        tr.step()
        losses.append(tr.loss())
    for k, (w, b) in tr.local_weights().items():
        np.save(os.path.join(out_dir, f"w{k}_r{mesh.replica}.npy"), w)
    if tr.last is not None:
        np.save(os.path.join(out_dir, f"loss_r{mesh.replica}.npy"), np.array(losses))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("pp,dp,sched,defer", [(2, 2, "1f1b", "1"), (4, 1, "zb", "1"),
                                               (1, 2, "1f1b", "1"), (1, 2, "1f1b", "0"),
                                               (2, 2, "zb", "1"), (2, 4, "1f1b", "1"),
                                               (1, 8, "1f1b", "1")])
def test_distributed_matches_single_process(pp, dp, sched, defer, monkeypatch):
    """defer = DNN_DP_DEFER: the data-parallel update of the later layers is applied behind
    the next step's forward (parallel/pipeline.dp_split) or at the end of the step."""
    monkeypatch.setenv("DNN_DP_DEFER", defer)
    mb, nm, steps = 128, 4, 3
    world = pp * dp
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), pp, dp, mb, nm, sched, steps, d),
                           nprocs=world, join=True, start_method="fork")
        spec = MLPSpec.parse(SPEC)
        tr = Trainer(spec, micro_batch=mb, num_micro=nm * dp, optim=OptimConfig(lr=0.1, momentum=0.9),
                     device=torch.device("cpu"))
        xt, yt = _global_batch(mb * nm * dp)
        ref_losses = []
        for _ in range(steps):
            tr.set_batch(xt, yt)
            tr.step()
            ref_losses.append(tr.loss())
        ref_w = tr.local_weights()
        for k, (w, _) in ref_w.items():
            for r in range(dp):  # every replica holds identical weights
                got = np.load(os.path.join(d, f"w{k}_r{r}.npy"))
                np.testing.assert_allclose(got, w, rtol=1e-4, atol=2e-5)
        # per-replica loss is the mean over that replica's shard; their mean is the global one
        lr_ = np.mean([np.load(os.path.join(d, f"loss_r{r}.npy")) for r in range(dp)], axis=0)
        np.testing.assert_allclose(lr_, ref_losses, rtol=1e-4)


def test_dp_buckets_cover_every_layer_once_in_contiguous_runs():
    from types import SimpleNamespace as NS

    from docker_dist_nn_amd.parallel.pipeline import dp_buckets

    def stage(dims):
        pad = lambda d: (d + 63) // 64 * 64  # noqa: E731
        return NS(geoms=[NS(kp=pad(a), np_=pad(b)) for a, b in zip(dims, dims[1:])])

    for dims, first in [([784, 512, 256, 128, 10], 0), ([784, 8192, 8192, 10], 1),
                        ([784] + [1024] * 7 + [10], 1), ([784, 10], 0)]:
        b = dp_buckets(stage(dims))
        assert b[0] == [first]  # the largest gradient is all-reduced first, alone
        flat = sorted(i for bk in b for i in bk)
        assert flat == list(range(len(dims) - 1))
        for bk in b:
            assert bk == list(range(bk[0], bk[-1] + 1))  # one contiguous flat range each
    assert dp_buckets(stage([784, 512, 256, 128, 10])) == [[0], [1, 2, 3]]


def test_dp_split_balances_gradient_bytes():
    from types import SimpleNamespace as NS

    from docker_dist_nn_amd.parallel.pipeline import dp_split

    def stage(dims):
        pad = lambda d: (d + 63) // 64 * 64  # noqa: E731
        return NS(geoms=[NS(kp=pad(a), np_=pad(b)) for a, b in zip(dims, dims[1:])])

    assert dp_split(stage([784, 512, 256, 128, 10])) == 1  # layer 0 holds 71 %
    assert dp_split(stage([784] + [1024] * 7 + [10])) == 4
    assert dp_split(stage([784, 8192, 8192, 10])) == 2
    assert dp_split(stage([784, 10])) == 0  # one layer: nothing to defer


def test_relay_assignment_balances_duties():
    from docker_dist_nn_amd.parallel.comm import relay_assignment, relay_parts

    a = relay_assignment(4, 2, 2)
    assert len(a) == 12  # 3 boundaries x 2 directions x 2 replicas
    load = {}
    for (src, dst, _), rl in a.items():
        assert len(rl) == 2 and src not in rl and dst not in rl and len(set(rl)) == 2
        for r in rl:
            load[r] = load.get(r, 0) + 1
    assert sum(load.values()) == 24 and max(load.values()) <= 4  # 3 per rank on average
    b = relay_parts(4096, 8192, 2)
    assert b[0] == 4096 and b[-1] == 8192 and all(x % 8 == 0 for x in b)
    assert sorted(b) == b
