"""The gloo plan interpreter (parallel/plan_interp.py) on CPU tensors: sends / receives on the
link channels, an RCCL group, and the three DP collectives with the native plan's addressing
(reduce-scatter into a piece, in-place all-gather), against plain torch results. The GPU test
(tests/test_dist_gpu.py) runs it on the real NativeStep op lists."""
import contextlib
import os
import socket
from types import SimpleNamespace as NS

import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from docker_dist_nn_amd.parallel import plan_interp as pi
    from docker_dist_nn_amd.parallel.groups import build_mesh
    from docker_dist_nn_amd.parallel.native_step import (ALL_GATHER, ALLREDUCE, GROUP,
                                                         NCCL_BF16, NCCL_F32, REC, RECV,
                                                         REDUCE_SCATTER, SEND, WAIT)

    dist.init_process_group("gloo", rank=rank, world_size=world)
    mesh = build_mesh(2, 2)  # ranks 0,1 = replica 0; 2,3 = replica 1
    comms, groups = pi.interp_groups(mesh)
    x = torch.arange(32, dtype=torch.float32) + 100 * rank      # hop buffers
    g16 = (torch.arange(64, dtype=torch.float32) * (rank + 1)).to(torch.bfloat16)
    piece = torch.zeros(32, dtype=torch.bfloat16)
    shadow = (torch.arange(64, dtype=torch.float32) + 1000 * mesh.replica).to(torch.bfloat16)
    bias = torch.full((8,), float(rank + 1))
    f = lambda t, off=0: t.data_ptr() + off * t.element_size()  # noqa: E731
    ops = []
    if mesh.stage == 0:  # send rows [0,8) forward, receive rows [8,16) back, one group
        ops.append(dict(kind=GROUP, stream=1, ops=[
            dict(kind=SEND, stream=1, comm=comms["f_out"], a=f(x), count=8, dtype=NCCL_F32,
                 gpeer=mesh.next_rank, tag=("f", 0, 0)),
            dict(kind=RECV, stream=1, comm=comms["b_in"], a=f(x, 8), count=8, dtype=NCCL_F32,
                 gpeer=mesh.next_rank, tag=("b", 0, 0))]))
    else:
        ops.append(dict(kind=RECV, stream=4, comm=comms["f_in"], a=f(x, 16), count=8,
                        dtype=NCCL_F32, gpeer=mesh.prev_rank, tag=("f", 0, 0)))
        ops.append(dict(kind=REC, stream=4, event=0))
        ops.append(dict(kind=WAIT, stream=2, event=0))
        ops.append(dict(kind=SEND, stream=2, comm=comms["b_out"], a=f(x, 24), count=8,
                        dtype=NCCL_F32, gpeer=mesh.prev_rank, tag=("b", 0, 0)))
    d = mesh.dp
    ops.append(dict(kind=REDUCE_SCATTER, stream=3, comm=comms["dp"], a=f(g16),
                    b=f(piece), count=64 // d, dtype=NCCL_BF16))
    ops.append(dict(kind=ALLREDUCE, stream=3, comm=comms["dp"], a=f(bias), count=8,
                    dtype=NCCL_F32))
    c = 64 // d
    ops.append(dict(kind=ALL_GATHER, stream=3, comm=comms["dp"], a=f(shadow, mesh.replica * c),
                    b=f(shadow), count=c, dtype=NCCL_BF16))
    st = NS(device=torch.device("cpu"), x=x, g16=g16, piece=piece, shadow=shadow, bias=bias,
            params=NS(set_lr=lambda lr: None, optim=NS(lr=0.1), step_count=0))
    it = pi.PlanInterpreter.__new__(pi.PlanInterpreter)
    it.ns, it.groups, it.timeout = NS(st=st, ops=ops), groups, 30
    it.stages = [st]
    it.mem = pi.stage_memory(st)
    it.stream = None
    it.queues = {}
    for o in ops:
        it.queues.setdefault(o["stream"], []).append(o)
    torch.cuda.synchronize = lambda *a: None
    torch.cuda.stream = lambda s: contextlib.nullcontext()
    it.run_step()
    torch.save({"x": x, "piece": piece, "shadow": shadow, "bias": bias},
               os.path.join(out, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_interpreter_moves_the_plan_bytes(tmp_path):
    mp.start_processes(_worker, args=(4, _port(), str(tmp_path)), nprocs=4, join=True,
                       start_method="spawn")
    r = [torch.load(tmp_path / f"r{k}.pt", weights_only=True) for k in range(4)]
    for s0, s1 in ((0, 1), (2, 3)):
        assert torch.equal(r[s1]["x"][16:24], torch.arange(8.0) + 100 * s0)   # forward hop
        assert torch.equal(r[s0]["x"][8:16], torch.arange(24.0, 32.0) + 100 * s1)  # backward
    for rank in range(4):
        stage, replica = rank % 2, rank // 2
        peers = [stage, stage + 2]
        full = sum((torch.arange(64, dtype=torch.float32) * (p + 1)).to(torch.bfloat16).float()
                   for p in peers)
        assert torch.equal(r[rank]["piece"].float(), full[replica * 32:(replica + 1) * 32]
                           .to(torch.bfloat16).float())
        assert torch.equal(r[rank]["bias"], torch.full((8,), float(sum(p + 1 for p in peers))))
        want = torch.cat([(torch.arange(32, dtype=torch.float32) + 1000 * q).to(torch.bfloat16)
                          for q in range(2)])
        assert torch.equal(r[rank]["shadow"][:32], want[:32])
        assert torch.equal(r[rank]["shadow"][32:], (torch.arange(32, 64, dtype=torch.float32)
                                                    + 1000).to(torch.bfloat16))
