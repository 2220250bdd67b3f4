"""Replicated-stage (fan) pipelines on the GPU: processes sharing cuda:0 (gloo), the EXACT op
list of the native fan step (fan.FanNativeStep: slotted RCCL groups on the boundary
communicators, DP buckets of the replicated stages) executed by the gloo plan interpreter
trains bit for bit like the op-by-op Python executor (FanPipe)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SPEC = "784-256-128-64-10"


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, dist_, reps, M, dp_reduce, use_interp, steps, out_dir, tag,
            place=None, ipc=False, graph=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DNN_DP_DEFER="0")
    import torch.distributed as dist

    from docker_dist_nn_amd import MLPSpec
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig
    from docker_dist_nn_amd.engine.fan_trainer import FanTrainer
    from docker_dist_nn_amd.parallel.fan import FanLayout, FanNativeStep, build_fan_mesh
    from docker_dist_nn_amd.parallel.plan_interp import PlanInterpreter

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lay = FanLayout(tuple(dist_), tuple(reps), place)
    mesh = build_fan_mesh(lay)
    mb = 256
    tr = FanTrainer(MLPSpec.parse(SPEC), lay, mesh, micro_batch=mb, num_micro=M, device=dev,
                    dp_reduce=dp_reduce, optim=OptimConfig(name="sgd", lr=0.05, momentum=0.9),
                    ipc_rehearsal=ipc)
    assert (tr.native_step is None) == (ipc != "native")  # gloo: the Python executor
    it = None
    if ipc and ipc != "native":  # the IPC fan plan: real peer copies + flags, the DP buckets over gloo
        groups = {"dp": mesh.dp_group} if mesh.dp_group is not None else {}
        ns = FanNativeStep(tr.executor, mesh, tr.sched, comms={k: k for k in groups},
                           build_only=True, ipc=tr.ipc_pipe)
        assert ns.transport == "ipc" and ns.mode == "fan-ipc-slotted"
        it = PlanInterpreter(ns, groups, timeout_s=60)
    elif use_interp and lay.colocated:  # boundary-indexed communicators (co-located plan)
        names = {f"f{b}": g for b, g in mesh.bnd_f.items()}
        names.update({f"b{b}": g for b, g in mesh.bnd_b.items()})
        names.update({f"dp{s_}": g for s_, g in mesh.dp_groups.items()})
        ns = FanNativeStep(tr.executor, mesh, tr.sched, comms={k: k for k in names},
                           build_only=True)
        assert ns.mode == "fan-slotted-colocated"
        it = PlanInterpreter(ns, names, timeout_s=60)
    elif use_interp:
        names = {"f_in": mesh.fwd_in, "f_out": mesh.fwd_out, "b_in": mesh.bwd_in,
                 "b_out": mesh.bwd_out, "dp": mesh.dp_group}
        comms = {k: k for k, g in names.items() if g is not None}
        groups = {k: g for k, g in names.items() if g is not None}
        ns = FanNativeStep(tr.executor, mesh, tr.sched, comms=comms, build_only=True)
        it = PlanInterpreter(ns, groups, timeout_s=60)
    x, y = synthetic_mnist(mb * M, seed=3)
    xt = torch.zeros(mb * M, 832, dtype=torch.bfloat16)
    xt[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xt, yt = xt.to(dev), torch.from_numpy(y).to(dev)
    done = 0
    if graph:  # the capture executes one real step; the rest are replays
        tr.set_global_batch(xt, yt)
        tr.capture(warmup=0)
        assert tr.graph_nodes > 0
        done = 1
    for _ in range(steps - done):
        tr.set_global_batch(xt, yt)
        if it is None:
            tr.step()
        else:
            for st in tr.stages:
                st.begin_step()
            it.run_step()
    torch.cuda.synchronize()
    bounds = np.cumsum([0] + list(dist_))
    for k, (w, b) in tr.local_weights().items():
        s = int(np.searchsorted(bounds, k, side="right")) - 1
        if mesh.replica_at(s) == 0:
            np.save(os.path.join(out_dir, f"{tag}_w{k}.npy"), w)
            np.save(os.path.join(out_dir, f"{tag}_b{k}.npy"), b)
    if tr.last is not None:
        np.save(os.path.join(out_dir, f"{tag}_loss{mesh.replica_at(lay.S - 1)}.npy"),
                np.array([tr.loss()]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("dist_,reps,M,dp_reduce", [([1, 3], [3, 1], 7, "allreduce"),
                                                    ([2, 2], [1, 3], 6, "shard"),
                                                    ([1, 1, 2], [2, 1, 2], 5, "allreduce")])
def test_fan_plan_interpreted_bitwise_equals_python(dev, dist_, reps, M, dp_reduce):
    world, steps = sum(reps), 3
    with tempfile.TemporaryDirectory() as d:
        for use, tag in ((False, "py"), (True, "plan")):
            mp.start_processes(_worker, args=(world, _port(), dist_, reps, M, dp_reduce, use,
                                              steps, d, tag),
                               nprocs=world, join=True, start_method="spawn")
        for k in range(4):
            for wb in ("w", "b"):
                a = np.load(os.path.join(d, f"py_{wb}{k}.npy"))
                b = np.load(os.path.join(d, f"plan_{wb}{k}.npy"))
                assert np.array_equal(a, b), (wb, k)
        for q in range(reps[-1]):
            assert np.array_equal(np.load(os.path.join(d, f"py_loss{q}.npy")),
                                  np.load(os.path.join(d, f"plan_loss{q}.npy")))


@pytest.mark.timeout(300)
def test_bench_runs_the_fan_layout(tmp_path):
    """bench.py at N = 4 (four ranks sharing cuda:0 over gloo, launched by torch.distributed.run
    as the driver launches it) runs the replicated-stage layout the planner picks for the
    headline model at the default batch (tests/test_fan_cpu.py) -- 3 layers on three GPUs, the
    classifier layer on one -- through the ladder (at a small batch here), and reports it with
    a uniform pipeline grid's prediction beside it."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DNN_FORCE_DEVICE="0", DNN_DIST_BACKEND="gloo", TMPDIR=str(tmp_path))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "4", "--master-addr", "127.0.0.1",
                        "--master-port", str(_port()), os.path.join(root, "bench.py"),
                        "--gpus", "4", "--steps", "3", "--warmup", "1", "--batch", "4096",
                        "--parallelism", "fan:3x3,1x1", "--no-dp-compare"],
                       env=env, stdout=subprocess.PIPE, stderr=None, text=True, timeout=280,
                       cwd=root)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["value"] > 0 and out["n_gpus"] == 4
    assert out["config"]["parallelism"] == "fan3x3,1x1", out["config"]
    assert out["config"]["stage_gpus"] == [3, 1]
    assert out["ladder"]["rung"] == "default"
    assert out["ladder"]["attempts"][0]["rung"] == "default"
    assert 0 < out["last_loss"] < 10
    # the literal grid is measured after the fan number (--no-dp-compare skips only DP)
    assert out["uniform_pipeline"]["value"] > 0, out["uniform_pipeline"]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("reps,place,M,dp_reduce", [([2, 1], ((0, 1), (1,)), 6, "allreduce"),
                                                    ([3, 1], ((0, 1, 2), (2,)), 7, "shard")])
def test_colocated_fan_bitwise_equals_separate_gpus(dev, reps, place, M, dp_reduce):
    """The light last stage co-located with the heavy stage's last replica (its hops to that
    replica become device copies, the others fan in over the boundary communicator) trains bit
    for bit like the same layout with the light stage on a rank of its own."""
    dist_, steps = [3, 1], 3
    with tempfile.TemporaryDirectory() as d:
        for pl, tag in ((None, "sep"), (place, "colo")):
            world = sum(reps) if pl is None else len({x for p in pl for x in p})
            mp.start_processes(_worker, args=(world, _port(), dist_, reps, M, dp_reduce, False,
                                              steps, d, tag, pl),
                               nprocs=world, join=True, start_method="spawn")
        for k in range(4):
            for wb in ("w", "b"):
                a = np.load(os.path.join(d, f"sep_{wb}{k}.npy"))
                b = np.load(os.path.join(d, f"colo_{wb}{k}.npy"))
                assert np.array_equal(a, b), (wb, k)
        assert np.array_equal(np.load(os.path.join(d, "sep_loss0.npy")),
                              np.load(os.path.join(d, "colo_loss0.npy")))


@pytest.mark.timeout(400)
def test_bench_colocated_fan_with_uniform_and_dp_measured(tmp_path):
    """bench.py at N = 4 (four ranks sharing cuda:0 over gloo, through the ladder) on the
    co-located layout fan:3x4,1x1@3 -- then, as comparisons inside the deadline, the literal
    uniform grid (pp4) and data parallelism, all in ONE JSON line."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DNN_FORCE_DEVICE="0", DNN_DIST_BACKEND="gloo", TMPDIR=str(tmp_path))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "4", "--master-addr", "127.0.0.1",
                        "--master-port", str(_port()), os.path.join(root, "bench.py"),
                        "--gpus", "4", "--steps", "3", "--warmup", "1", "--batch", "4096",
                        "--parallelism", "fan:3x4,1x1@3"],
                       env=env, stdout=subprocess.PIPE, stderr=None, text=True, timeout=380,
                       cwd=root)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["value"] > 0 and out["n_gpus"] == 4
    cfg = out["config"]
    assert cfg["parallelism"] == "fan3x4,1x1@3" and cfg["stage_place"] == [[0, 1, 2, 3], [3]]
    u, dp = out["uniform_pipeline"], out["dp_only"]
    assert u["value"] > 0 and u["parallelism"] == "pp4", u
    assert dp["value"] > 0 and dp["parallelism"] == "dp4", dp
    assert out["ladder"]["seconds"] < 540
    assert [a["rung"] for a in out["ladder"]["compare_attempts"]] == ["uniform", "dp-native"]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("dist_,reps,M,dp_reduce", [([3, 1], [3, 1], 7, "allreduce"),
                                                    ([2, 2], [1, 3], 6, "shard")])
def test_fan_ipc_plan_bitwise_equals_python(dev, dist_, reps, M, dp_reduce):
    """the fan step on the xGMI peer-write transport -- the EXACT op list of
    FanNativeStep's IPC form (one stream, copies into IPC-mapped L2-uncached receive rows +
    step-numbered flags + per-peer acks) with real device copies / flags between processes
    sharing cuda:0 -- trains bit for bit like the Python executor over gloo, for three steps
    (the acks of one step gate the writes of the next)."""
    world, steps = sum(reps), 3
    with tempfile.TemporaryDirectory() as d:
        for ipc, tag in ((False, "py"), (True, "ipc")):
            mp.start_processes(_worker, args=(world, _port(), dist_, reps, M, dp_reduce, False,
                                              steps, d, tag, None, ipc),
                               nprocs=world, join=True, start_method="spawn")
        for k in range(4):
            for wb in ("w", "b"):
                a = np.load(os.path.join(d, f"py_{wb}{k}.npy"))
                b = np.load(os.path.join(d, f"ipc_{wb}{k}.npy"))
                assert np.array_equal(a, b), (wb, k)
        for q in range(reps[-1]):
            assert np.array_equal(np.load(os.path.join(d, f"py_loss{q}.npy")),
                                  np.load(os.path.join(d, f"ipc_loss{q}.npy")))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("dist_,M", [([3, 1], 4), ([1, 1, 2], 5)])
def test_fan_ipc_native_step_graph_capture(dev, dist_, M):
    """the IPC fan plan as the rank's real StepPlan (device step-number flags,
    per-peer acks, peer copies in clock order on one stream) -- eager, and captured into a HIP
    graph and replayed -- trains bit for bit like the Python executor. One replica per stage:
    on one GPU the ranks cannot open an RCCL DP group (one rank per GPU), so replicated stages
    are rehearsed through the plan interpreter above."""
    reps, steps = [1] * len(dist_), 4
    world = len(dist_)
    with tempfile.TemporaryDirectory() as d:
        for ipc, graph, tag in ((False, False, "py"), ("native", False, "eager"),
                                ("native", True, "graph")):
            mp.start_processes(_worker, args=(world, _port(), dist_, reps, M, "allreduce", False,
                                              steps, d, tag, None, ipc, graph),
                               nprocs=world, join=True, start_method="spawn")
        for tag in ("eager", "graph"):
            for k in range(4):
                for wb in ("w", "b"):
                    a = np.load(os.path.join(d, f"py_{wb}{k}.npy"))
                    b = np.load(os.path.join(d, f"{tag}_{wb}{k}.npy"))
                    assert np.array_equal(a, b), (tag, wb, k)
            assert np.array_equal(np.load(os.path.join(d, "py_loss0.npy")),
                                  np.load(os.path.join(d, f"{tag}_loss0.npy")))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("reps,place,M,dp_reduce", [([2, 1], ((0, 1), (1,)), 6, "allreduce"),
                                                    ([3, 1], ((0, 1, 2), (2,)), 7, "shard")])
def test_colocated_fan_plan_interpreted_bitwise_equals_python(dev, reps, place, M, dp_reduce):
    """The native step of a co-located layout -- the EXACT op list FanNativeStep builds for the
    rank hosting a heavy-stage replica AND the light stage (both workers' segments on one
    stream in slot order, the hops between them as device copies, the others in per-slot
    groups on the boundary communicators, each worker's DP buckets) -- run by the gloo plan
    interpreter trains bit for bit like the Python executor (processes sharing cuda:0)."""
    dist_, steps = [3, 1], 3
    world = len({x for p in place for x in p})
    with tempfile.TemporaryDirectory() as d:
        for use, tag in ((False, "py"), (True, "plan")):
            mp.start_processes(_worker, args=(world, _port(), dist_, reps, M, dp_reduce, use,
                                              steps, d, tag, place),
                               nprocs=world, join=True, start_method="spawn")
        for k in range(4):
            for wb in ("w", "b"):
                a = np.load(os.path.join(d, f"py_{wb}{k}.npy"))
                b = np.load(os.path.join(d, f"plan_{wb}{k}.npy"))
                assert np.array_equal(a, b), (wb, k)
        assert np.array_equal(np.load(os.path.join(d, "py_loss0.npy")),
                              np.load(os.path.join(d, "plan_loss0.npy")))

