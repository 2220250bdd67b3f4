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
    shard = defer == "shard"  # sharded DP (bf16 reduce-scatter / all-gather) instead
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      DNN_DP_DEFER="1" if shard else defer)
    import torch.distributed as dist

    from docker_dist_nn_amd import MLPSpec
    from docker_dist_nn_amd.engine import OptimConfig, Trainer
    from docker_dist_nn_amd.parallel.groups import build_mesh

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mesh = build_mesh(1, world)
    tr = Trainer(MLPSpec.parse(SPEC), micro_batch=1024, num_micro=1, mesh=mesh, device=dev,
                 optim=OptimConfig(name=optim, lr=0.05 if optim == "sgd" else 1e-3),
                 dp_reduce="shard" if shard else "allreduce")
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


@pytest.mark.parametrize("optim,defer", [("sgd", "1"), ("adam", "1"), ("sgd", "0"),
                                         ("sgd", "shard")])
def test_dp2_native_matches_single_process(dev, optim, defer):
    """defer "shard": sharded DP on the GPU kernels (pack / unpack / piece update), gloo
    collectives; matches within the bf16 rounding of the exchanged gradients."""
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
                if defer == "shard":
                    np.testing.assert_allclose(got, w, rtol=2e-2, atol=5e-4)
                else:
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


def _native_worker(rank, world, port, native_dist, steps, nm, out_dir, relays=0, tag=None,
                   graph=False, fault="", plan="streams"):
    # every stream of a plan that waits on a flag needs a hardware queue of its own (HIP
    # multiplexes streams beyond GPU_MAX_HW_QUEUES onto shared queues, where one blocked wait
    # would stall the others): 4 plan streams + the relay duties + the default stream
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DNN_PIPE="ipc",
                      DNN_NATIVE_DIST=native_dist, DNN_IPC_RELAYS=str(relays),
                      GPU_MAX_HW_QUEUES="8", DNN_FAULT_NATIVE_STEP=fault, DNN_IPC_PLAN=plan)
    tag = native_dist if tag is None else tag
    import time

    import torch.distributed as dist

    from docker_dist_nn_amd import MLPSpec
    from docker_dist_nn_amd.engine import OptimConfig, Trainer
    from docker_dist_nn_amd.parallel.groups import build_mesh

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mesh = build_mesh(world, 1)
    tr = Trainer(MLPSpec.parse(SPEC), micro_batch=256, num_micro=nm, mesh=mesh, device=dev,
                 schedule="1f1b", optim=OptimConfig(name="sgd", lr=0.05, momentum=0.9))
    assert (tr.native_step is not None) == (native_dist == "1" and not fault)
    assert (tr.native_fallback is not None) == bool(fault)
    xt, yt = _batch(256 * nm)
    xd, yd = xt.to(dev), yt.to(dev)
    host = []
    done = 0
    if graph:  # one eager warm-up step + the capture's executed step, then replays
        tr.set_batch(xd if tr.first else None, yd if tr.last else None)
        tr.capture(warmup=1)
        done = 2
    for _ in range(steps - done):
        tr.set_batch(xd if tr.first else None, yd if tr.last else None, zero_copy=not graph)
        t0 = time.perf_counter()
        tr.step()
        host.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    for k, (w, _b) in tr.local_weights().items():
        np.save(os.path.join(out_dir, f"n{tag}_w{k}.npy"), w)
    np.save(os.path.join(out_dir, f"n{tag}_host_r{rank}.npy"), np.array(host))
    if tr.last is not None:
        np.save(os.path.join(out_dir, f"n{tag}_loss.npy"), np.array([tr.loss()]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,nm", [(2, 4), (4, 6)])
def test_native_multirank_step_bitwise_equals_python(dev, world, nm):
    """The native multi-rank step (parallel/native_step.py: ONE StepPlan call per step, xGMI
    peer-copy transport) gives bit-identical weights and loss to the op-by-op Python executor
    over the same transport; ranks = processes sharing cuda:0. Also bounds the host time of a
    native step (the plan enqueues everything; no per-op Python)."""
    steps = 4
    with tempfile.TemporaryDirectory() as d:
        for native_dist in ("0", "1"):
            mp.start_processes(_native_worker,
                               args=(world, _free_port(), native_dist, steps, nm, d),
                               nprocs=world, join=True, start_method="spawn")
        for k in range(4):
            a = np.load(os.path.join(d, f"n0_w{k}.npy"))
            b = np.load(os.path.join(d, f"n1_w{k}.npy"))
            assert np.array_equal(a, b), k
        assert np.array_equal(np.load(os.path.join(d, "n0_loss.npy")),
                              np.load(os.path.join(d, "n1_loss.npy")))
        host = [np.median(np.load(os.path.join(d, f"n1_host_r{r}.npy"))[1:])
                for r in range(world)]
        print("native host s/step per rank:", host)
        assert max(host) < 2e-3, host


def test_native_step_construction_fault_falls_back_on_every_rank(dev):
    """One rank cannot build its native step (injected fault): the ranks agree over the world
    group and ALL run the Python executor (mixing the two would post hops on different
    communicators), training bit for bit like an all-Python run."""
    world, steps, nm = 3, 3, 4
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_native_worker, args=(world, _free_port(), "0", steps, nm, d),
                           nprocs=world, join=True, start_method="spawn")
        mp.start_processes(_native_worker, args=(world, _free_port(), "1", steps, nm, d, 0,
                                                 "f", False, "1"),
                           nprocs=world, join=True, start_method="spawn")
        for k in range(4):
            assert np.array_equal(np.load(os.path.join(d, f"n0_w{k}.npy")),
                                  np.load(os.path.join(d, f"nf_w{k}.npy"))), k
        assert np.array_equal(np.load(os.path.join(d, "n0_loss.npy")),
                              np.load(os.path.join(d, "nf_loss.npy")))


@pytest.mark.parametrize("world,relays", [(3, 1), (4, 2)])
def test_relayed_ipc_hops_bitwise_equal_direct(dev, world, relays):
    """Relayed xGMI hops (DNN_IPC_RELAYS, parallel/comm.relay_assignment): every hop's rows
    striped over the direct copy and `relays` two-hop copies through other ranks' staging
    slots and relay streams give bit-identical training to direct hops (ranks = processes
    sharing cuda:0; the data moved is the same, only its route differs)."""
    steps, nm = 3, 4
    with tempfile.TemporaryDirectory() as d:
        for k, tag in ((0, "direct"), (relays, "relay")):
            mp.start_processes(_native_worker,
                               args=(world, _free_port(), "1", steps, nm, d, k, tag),
                               nprocs=world, join=True, start_method="spawn")
        for k in range(4):
            a = np.load(os.path.join(d, f"ndirect_w{k}.npy"))
            b = np.load(os.path.join(d, f"nrelay_w{k}.npy"))
            assert np.array_equal(a, b), k
        assert np.array_equal(np.load(os.path.join(d, "ndirect_loss.npy")),
                              np.load(os.path.join(d, "nrelay_loss.npy")))


@pytest.mark.parametrize("world,relays,nm", [(2, 0, 4), (4, 0, 4), (4, 2, 8), (4, "auto", 4)])
def test_native_multirank_step_graph_capture(dev, world, relays, nm):
    """The native multi-rank step (IPC hops: device step-number flag kernels) captured into a
    HIP graph and replayed gives bit-identical training to eager plan runs, and a replayed
    step costs the host only the graph launch. Relayed hops included (capture
    now records the slotted single-stream form, Trainer.capture). pp4 x 8 micro-batches with
    2 relays: the host time per replayed rank-step stays under 100 us."""
    steps = 6
    with tempfile.TemporaryDirectory() as d:
        for tag, graph in (("eager", False), ("graph", True)):
            mp.start_processes(_native_worker,
                               args=(world, _free_port(), "1", steps, nm, d, relays, tag,
                                     graph),
                               nprocs=world, join=True, start_method="spawn")
        for k in range(4):
            a = np.load(os.path.join(d, f"neager_w{k}.npy"))
            b = np.load(os.path.join(d, f"ngraph_w{k}.npy"))
            assert np.array_equal(a, b), k
        assert np.array_equal(np.load(os.path.join(d, "neager_loss.npy")),
                              np.load(os.path.join(d, "ngraph_loss.npy")))
        host = [float(np.median(np.load(os.path.join(d, f"ngraph_host_r{r}.npy"))))
                for r in range(world)]
        print(f"graph replay host us/step per rank (pp{world}, {nm} micro-batches, relays "
              f"{relays}):", [round(h * 1e6, 1) for h in host])
        assert max(host) < 1e-4, host


@pytest.mark.parametrize("world,relays", [(3, 1), (4, "auto")])
def test_ipc_slotted_plan_bitwise_equals_streams(dev, world, relays):
    """The slotted IPC form (DNN_IPC_PLAN=slotted: one stream per rank in logical-clock order)
    trains bit for bit like the multi-stream form, relays included."""
    steps, nm = 3, 4
    with tempfile.TemporaryDirectory() as d:
        for plan in ("streams", "slotted"):
            mp.start_processes(_native_worker,
                               args=(world, _free_port(), "1", steps, nm, d, relays, plan,
                                     False, "", plan),
                               nprocs=world, join=True, start_method="spawn")
        for k in range(4):
            assert np.array_equal(np.load(os.path.join(d, f"nstreams_w{k}.npy")),
                                  np.load(os.path.join(d, f"nslotted_w{k}.npy"))), k


def test_step_plan_rccl_allreduce_one_rank(dev):
    """The StepPlan's RCCL entry points bind to torch's librccl and drive the communicator
    torch created (world of one rank: all-reduce is a copy), on a plan-owned stream."""
    import torch.distributed as dist

    from docker_dist_nn_amd.parallel.native_step import (ALLREDUCE, NCCL_F32, REC, WAIT,
                                                         comm_ptr, torch_rccl_path)
    from docker_dist_nn_amd.utils.native import native

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        t = torch.ones(1, device=dev)
        dist.all_reduce(t)
        n = native()
        n.nccl_load(torch_rccl_path())
        comm = comm_ptr(dist.group.WORLD, dev)
        assert n.nccl_comm_info(comm) == (1, 0)
        x = torch.arange(4096, dtype=torch.float32, device=dev)
        ref = x.clone()
        plan = n.StepPlan(2, 2)
        plan.add(kind=REC, stream=0, event=0)
        plan.add(kind=WAIT, stream=1, event=0)
        plan.add(kind=ALLREDUCE, stream=1, comm=comm, a=x.data_ptr(), count=x.numel(),
                 dtype=NCCL_F32)
        plan.run(torch.cuda.current_stream(dev).cuda_stream)
        plan.run(torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        assert torch.equal(x, ref) and plan.seq == 2 and plan.comm_error() == 0
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("optim", ["sgd", "adam"])
def test_native_sharded_dp_one_rank_equals_python(dev, optim, monkeypatch):
    """The sharded-DP step (bf16 reduce-scatter of each weight bucket, piece update, bf16
    all-gather, fp32 bias all-reduce: parallel/native_step._sharded_update) as ONE StepPlan
    call on RCCL equals the Python executor's sharded step bitwise -- on a DP group of one
    rank (the only RCCL group a one-GPU box can form; a piece is then the whole bucket)."""
    import torch.distributed as dist

    from docker_dist_nn_amd import MLPSpec
    from docker_dist_nn_amd.engine import OptimConfig, Trainer
    from docker_dist_nn_amd.parallel.groups import Mesh

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        xt, yt = _batch(2048)
        xd, yd = xt.to(dev), yt.to(dev)
        out = {}
        for nd in ("0", "1"):
            monkeypatch.setenv("DNN_NATIVE_DIST", nd)
            mesh = Mesh(0, 1, 1, 1, 0, 0, dp_group=dist.group.WORLD, dp_ranks=[0],
                        backend="nccl")
            tr = Trainer(MLPSpec.parse(SPEC), micro_batch=1024, num_micro=2, mesh=mesh,
                         device=dev, dp_reduce="shard",
                         optim=OptimConfig(name=optim, lr=0.05 if optim == "sgd" else 1e-3,
                                           momentum=0.9))
            assert tr.stages[0].params.sharded
            assert (tr.native_step is not None) == (nd == "1")
            for _ in range(3):
                tr.set_batch(xd, yd, zero_copy=True)
                tr.step()
            torch.cuda.synchronize(dev)
            out[nd] = (tr.local_weights(), tr.loss())
        for k, (w, b) in out["0"][0].items():
            assert np.array_equal(w, out["1"][0][k][0]), k
            assert np.array_equal(b, out["1"][0][k][1]), k
        assert out["0"][1] == out["1"][1]
    finally:
        dist.destroy_process_group()


def _tp_worker(rank, world, port, spec, rows, steps, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from docker_dist_nn_amd import MLPSpec
    from docker_dist_nn_amd.engine import OptimConfig
    from docker_dist_nn_amd.parallel.tensor import TensorParallelMLP

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tp = TensorParallelMLP(MLPSpec.parse(spec), rows=rows, tp=world, rank=rank, device=dev,
                           optim=OptimConfig(lr=0.05, momentum=0.9))
    xt, yt = _batch(rows)
    for _ in range(steps):
        tp.set_batch(xt[:, :784].float(), yt)
        tp.step()
    ws = tp.full_weights()
    if rank == 0:
        for k, (w, b) in enumerate(ws):
            np.save(os.path.join(out_dir, f"tp_w{k}.npy"), w)
        np.save(os.path.join(out_dir, "tp_loss.npy"), np.array([tp.loss()]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_tensor_parallel_gpu_matches_single_process(dev, world):
    """Megatron column/row tensor parallelism (parallel/tensor.py) on the gfx950 kernels --
    ranks = processes sharing cuda:0, gloo all-reduces -- reproduces single-GPU training."""
    from docker_dist_nn_amd import MLPSpec
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    rows, steps = 1024, 3
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_tp_worker, args=(world, _free_port(), SPEC, rows, steps, d),
                           nprocs=world, join=True, start_method="spawn")
        tr = Trainer(MLPSpec.parse(SPEC), micro_batch=rows, num_micro=1, device=dev,
                     optim=OptimConfig(lr=0.05, momentum=0.9))
        xt, yt = _batch(rows)
        for _ in range(steps):
            tr.set_batch(xt.to(dev), yt.to(dev))
            tr.step()
        for k, (w, _b) in tr.local_weights().items():
            np.testing.assert_allclose(np.load(os.path.join(d, f"tp_w{k}.npy")), w,
                                       rtol=1e-2, atol=1e-3)
        np.testing.assert_allclose(np.load(os.path.join(d, "tp_loss.npy"))[0], tr.loss(),
                                   rtol=1e-2)


def _interp_worker(rank, world, port, pp, mode, boundary, dp_reduce, use_interp, steps, nm,
                   out_dir, tag):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DNN_DP_DEFER="0")
    import torch.distributed as dist

    from docker_dist_nn_amd import MLPSpec
    from docker_dist_nn_amd.engine import OptimConfig, Trainer
    from docker_dist_nn_amd.parallel.groups import build_mesh
    from docker_dist_nn_amd.parallel.native_step import NativeStep
    from docker_dist_nn_amd.parallel.plan_interp import PlanInterpreter, interp_groups

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mesh = build_mesh(pp, world // pp)
    mb = 256
    tr = Trainer(MLPSpec.parse(SPEC), micro_batch=mb, num_micro=nm, mesh=mesh, device=dev,
                 schedule="1f1b_lh", boundary=boundary, dp_reduce=dp_reduce,
                 optim=OptimConfig(name="sgd", lr=0.05, momentum=0.9))
    assert tr.native_step is None  # gloo: the Python executor, unless interpreted below
    it = None
    if use_interp:
        comms, groups = interp_groups(mesh)
        ns = NativeStep(tr.executor, mesh, "rccl", comms=comms, mode=mode, build_only=True)
        it = PlanInterpreter(ns, groups, timeout_s=60)
    rows = mb * nm
    xt, yt = _batch(rows * mesh.dp)
    xs = xt[mesh.replica * rows:(mesh.replica + 1) * rows].to(dev)
    ys = yt[mesh.replica * rows:(mesh.replica + 1) * rows].to(dev)
    for _ in range(steps):
        tr.set_batch(xs if tr.first else None, ys if tr.last else None)
        if it is None:
            tr.step()
        else:
            for st in tr.stages:
                st.begin_step()
            it.run_step()
    torch.cuda.synchronize()
    for k, (w, b) in tr.local_weights().items():
        if mesh.replica == 0:
            np.save(os.path.join(out_dir, f"{tag}_w{k}.npy"), w)
            np.save(os.path.join(out_dir, f"{tag}_b{k}.npy"), b)
    if tr.last is not None and mesh.replica == 0:
        np.save(os.path.join(out_dir, f"{tag}_loss.npy"), np.array([tr.loss()]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("pp,world,mode,boundary,dp_reduce", [
    (2, 4, "streams", "bf16", "shard"),
    (2, 4, "slotted", "fp8", "allreduce"),
    (4, 4, "streams", "fp8", "allreduce"),
    (3, 3, "slotted", "bf16", "allreduce"),
])
def test_rccl_plan_interpreted_bitwise_equals_python(dev, pp, world, mode, boundary, dp_reduce):
    """The EXACT op list of the native RCCL step (NativeStep._build: streams or slotted form,
    link-channel sends / receives, RCCL groups, sharded reduce-scatter into grad_piece + e0/d and
    in-place all-gather, fp8 two-part hops), executed by the gloo plan interpreter
    (parallel/plan_interp.py) on processes sharing cuda:0, trains bit for bit like the
    op-by-op Python executor: every pointer, count, peer and event edge of the plan is right."""
    steps, nm = 3, 2 * pp
    with tempfile.TemporaryDirectory() as d:
        for use, tag in ((False, "py"), (True, "plan")):
            mp.start_processes(_interp_worker,
                               args=(world, _free_port(), pp, mode, boundary, dp_reduce, use,
                                     steps, nm, d, tag),
                               nprocs=world, join=True, start_method="spawn")
        for k in range(4):
            for wb in ("w", "b"):
                a = np.load(os.path.join(d, f"py_{wb}{k}.npy"))
                b = np.load(os.path.join(d, f"plan_{wb}{k}.npy"))
                assert np.array_equal(a, b), (wb, k)
        assert np.array_equal(np.load(os.path.join(d, "py_loss.npy")),
                              np.load(os.path.join(d, "plan_loss.npy")))


def _verify_worker(rank, world, port, pipe, fault, relays, steps, out_dir, tag):
    # one GPU, `world` processes: IPC hops between processes sharing cuda:0, gloo collectives;
    # the first IPC step is verified against the message transport (Python executor over gloo)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DNN_PIPE=pipe,
                      DNN_IPC_VERIFY="1", DNN_FAULT_IPC_VERIFY=fault,
                      DNN_IPC_RELAYS=str(relays), GPU_MAX_HW_QUEUES="8")
    import torch.distributed as dist

    from docker_dist_nn_amd import MLPSpec
    from docker_dist_nn_amd.engine import OptimConfig, Trainer
    from docker_dist_nn_amd.parallel.groups import build_mesh

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mesh = build_mesh(world, 1)
    tr = Trainer(MLPSpec.parse(SPEC), micro_batch=256, num_micro=4, mesh=mesh, device=dev,
                 schedule="1f1b", optim=OptimConfig(name="sgd", lr=0.05, momentum=0.9))
    xt, yt = _batch(1024)
    for _ in range(steps):
        tr.set_batch(xt.to(dev) if tr.first else None, yt.to(dev) if tr.last else None)
        tr.step()
    torch.cuda.synchronize()
    for k, (w, _b) in tr.local_weights().items():
        np.save(os.path.join(out_dir, f"{tag}_w{k}.npy"), w)
    with open(os.path.join(out_dir, f"{tag}_transport_r{rank}.txt"), "w") as f:
        f.write(f"{tr.transport}\n{tr.transport_reason}\n")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,relays", [(2, 0), (4, 2)])
def test_ipc_first_step_verification_and_fallback(dev, world, relays):
    """The verified IPC transport (engine/trainer.py _verify_first_step): the first step runs
    on the IPC plan and, from the same state, on the fallback transport; with agreeing weights
    the job stays on IPC, with a corrupted IPC result on ONE rank every rank falls back. Either
    way training equals a message-transport-only run bit for bit, and every rank records the
    same transport and reason."""
    steps = 3
    with tempfile.TemporaryDirectory() as d:
        for tag, pipe, fault in (("ref", "rccl", ""), ("ok", "ipc", ""),
                                 ("fault", "ipc", "1")):
            mp.start_processes(_verify_worker,
                               args=(world, _free_port(), pipe, fault, relays, steps, d, tag),
                               nprocs=world, join=True, start_method="spawn")
        for k in range(4):
            ref = np.load(os.path.join(d, f"ref_w{k}.npy"))
            for tag in ("ok", "fault"):
                assert np.array_equal(ref, np.load(os.path.join(d, f"{tag}_w{k}.npy"))), (tag, k)
        for tag, want in (("ok", "ipc"), ("fault", "gloo")):
            got = {open(os.path.join(d, f"{tag}_transport_r{r}.txt")).read()
                   for r in range(world)}
            assert len(got) == 1, got
            transport, reason = got.pop().split("\n")[:2]
            assert transport == want, (tag, transport, reason)
            assert ("verified" in reason) if tag == "ok" else ("differed" in reason), reason


def test_uncached_buffers_freed_with_their_last_view(dev):
    """utils/devmem.py: an uncached receive / relay buffer lives as long as any tensor view of
    it and is freed when the last one dies (they used to be pinned until exit)."""
    import gc

    from docker_dist_nn_amd.utils.devmem import live_buffers, uncached_zeros

    gc.collect()
    n0 = live_buffers()
    t = uncached_zeros((64, 128), torch.bfloat16, dev)
    v = t[3:5]
    del t
    gc.collect()
    assert live_buffers() == n0 + 1  # the view keeps the allocation
    v.fill_(1.5)
    torch.cuda.synchronize(dev)
    assert float(v.float().sum()) == 1.5 * 2 * 128
    del v
    gc.collect()
    assert live_buffers() == n0
