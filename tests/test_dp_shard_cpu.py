"""Sharded data parallelism (Trainer(dp_reduce="shard"), parallel/pipeline.GradSync): bf16
reduce-scatter of each gradient bucket, the optimizer on this rank's 1/dp piece, bf16
all-gather of the updated weights. Multi-process on CPU (gloo, 127.0.0.1): the result must
match single-process training within the bf16 rounding of the exchanged gradients, every
replica must hold identical weights, and the gathered optimizer state must be whole."""
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


def _optim(name):
    return OptimConfig(name=name, lr=0.1 if name == "sgd" else 2e-3, momentum=0.9)


def _worker(rank, world, port, pp, dp, mb, nm, steps, opt, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from docker_dist_nn_amd.parallel.groups import build_mesh

    mesh = build_mesh(pp, dp)
    tr = Trainer(MLPSpec.parse(SPEC), micro_batch=mb, num_micro=nm, schedule="1f1b", mesh=mesh,
                 optim=_optim(opt), device=torch.device("cpu"), dp_reduce="shard")
    assert tr.dp_reduce == "shard" and tr.stages[0].params.sharded
    R = mb * nm
    xt, yt = _global_batch(R * dp)
    sl = slice(mesh.replica * R, (mesh.replica + 1) * R)
    for _ in range(steps):
        tr.set_batch(xt[sl] if tr.first else None, yt[sl] if tr.last else None)
        tr.step()
    for k, (w, b) in tr.local_weights().items():  # gathers master + optimizer state
        np.save(os.path.join(out_dir, f"w{k}_r{mesh.replica}.npy"), w)
    p = tr.stages[0].params
    for s in range(len(p.state)):
        ws, _ = p.export_state(s)
        for i, w in enumerate(ws):
            np.save(os.path.join(out_dir, f"s{s}_{tr.stages[0].l0 + i}_r{mesh.replica}.npy"), w)
    # the shard pieces tile each bucket exactly once over the replicas
    for e0, e1 in p.shard_buckets:
        assert (e1 - e0) % dp == 0 and p.shard_piece(e0, e1)[0] == e0 + mesh.replica * (e1 - e0) // dp
    dist.barrier()
    dist.destroy_process_group()


def _reference(mb, nm, dp, steps, opt):
    tr = Trainer(MLPSpec.parse(SPEC), micro_batch=mb, num_micro=nm * dp, optim=_optim(opt),
                 device=torch.device("cpu"))
    xt, yt = _global_batch(mb * nm * dp)
    for _ in range(steps):
        tr.set_batch(xt, yt)
        tr.step()
    return tr


@pytest.mark.parametrize("pp,dp,opt", [(1, 2, "sgd"), (2, 2, "sgd"), (1, 4, "adam"),
                                       (2, 2, "adam")])
def test_sharded_dp_matches_single_process(pp, dp, opt):
    mb, nm, steps = 128, 2, 3
    world = pp * dp
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), pp, dp, mb, nm, steps, opt, d),
                           nprocs=world, join=True, start_method="fork")
        ref = _reference(mb, nm, dp, steps, opt)
        for k, (w, _) in ref.local_weights().items():
            got = [np.load(os.path.join(d, f"w{k}_r{r}.npy")) for r in range(dp)]
            for g in got[1:]:  # replicas are identical after the all-gathers
                assert np.array_equal(g, got[0])
            if opt == "sgd":  # bf16 gradient exchange: ~2^-9 relative per step
                np.testing.assert_allclose(got[0], w, rtol=2e-2, atol=3e-4)
            else:
                # Adam normalises each element's step: where the replicas' gradients nearly
                # cancel, bf16 rounding can change that step by up to lr (the step size)
                bad = np.abs(got[0] - w) > 3e-4 + 2e-2 * np.abs(w)
                assert bad.mean() < 5e-3, bad.mean()
                assert np.abs(got[0] - w).max() <= 2 * 2e-3 * steps
        p = ref.stages[0].params
        for s in range(len(p.state)):
            ws, _ = p.export_state(s)
            for k, w in enumerate(ws):
                got = np.load(os.path.join(d, f"s{s}_{k}_r0.npy")) if os.path.exists(
                    os.path.join(d, f"s{s}_{k}_r0.npy")) else None
                if got is not None:  # bf16 gradient sums: ~0.2 % per step, compounding
                    assert np.linalg.norm(got - w) <= 3e-2 * np.linalg.norm(w) + 1e-9


def test_shard_layout_pads_layers_to_dp_pieces():
    from docker_dist_nn_amd.engine.stage import StageParams, LayerGeom

    spec = MLPSpec.parse("784-100-10")
    geoms = [LayerGeom(i, spec.layers[i]) for i in range(2)]
    for dp in (2, 3, 8):
        p = StageParams(geoms, torch.device("cpu"), shard=(dp, dp - 1))
        for i in range(2):
            e0, e1 = p.layer_grad_range(i)
            assert (e1 - e0) % (64 * dp) == 0
            p0, p1 = p.shard_piece(e0, e1)
            assert p1 == e1 and p1 - p0 == (e1 - e0) // dp
        assert p.grad_piece.numel() * dp == p.numel
