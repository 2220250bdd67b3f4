"""Headline benchmark: samples/sec (whole node) of MNIST-FCNN training on N MI355X GPUs.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 it is launched
by ``torch.distributed.run`` with one rank per GPU (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in the
env, RCCL over xGMI). W untimed warm-up steps, then EXACTLY K timed steps bracketed by a barrier
+ device synchronize on both sides; the max elapsed time over ranks is used; rank 0 prints one
JSON line.

Model: BASELINE.json config "784-512-256-128-10 MNIST FCNN bf16" (random init, synthetic
MNIST-shaped data resident in HBM). One step = forward + backward + SGD update of the global
batch (bf16 operands, fp32 accumulation/master weights), on our own gfx950 kernels.

Parallel layout (the metric is "... at 1/2/4/8-stage pipeline"):
  * ``--parallelism pipeline`` (default): N = 1 is the single-GPU step; for N > 1 the deepest
    pipeline that divides N and fits the layers, data parallel over the rest
    (planner.pipeline_layout: pp2, pp4, pp4dp2 at 2/4/8 GPUs for this model), one stage per
    GPU, the layer split chosen by the planner's hop/compute model, 1F1B micro-batching, and
    the native multi-rank step (parallel/native_step.py: one C++ call per step, RCCL P2P on
    per-direction communicators, DP buckets on their own stream);
  * after the pipeline number, the same N GPUs also run pure data parallelism (``dp_only`` in
    the JSON; ``--no-dp-compare`` skips it);
  * ``ppS`` / ``dpN`` / ``ppSdpD`` force a layout; ``best`` lets the planner pick.
Weak scaling: every GPU contributes ``--batch`` rows per step.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

# Multi-rank steps run several busy streams per rank: the IPC plan 4 + its relay duties
# (~7 at pp4dp2 with 2 relays), the RCCL fallback plan built next to it for the first-step
# verification 6 (parallel/native_step.py), torch's and RCCL's own. HIP multiplexes streams
# onto GPU_MAX_HW_QUEUES hardware queues (default 4) in order, so two streams sharing a queue
# would serialise a spinning wait in one direction with the work that releases it. Give every
# stream its own queue (set before the HIP runtime initialises; <= 32 by pool policy). The box
# exports GPU_MAX_HW_QUEUES=4 (HIP's default), so raise it rather than setdefault; one-GPU
# rehearsals (DNN_FORCE_DEVICE: many ranks share one GPU) keep what the caller set.
if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not os.environ.get("DNN_FORCE_DEVICE"):
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 24:
        os.environ["GPU_MAX_HW_QUEUES"] = "24"

import torch  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from docker_dist_nn_amd import NAMED_MODELS, MLPSpec  # noqa: E402
from docker_dist_nn_amd import ladder, switches  # noqa: E402
from docker_dist_nn_amd.faults import FaultInjector  # noqa: E402
from docker_dist_nn_amd.data import DeviceDataset, synthetic_mnist  # noqa: E402
from docker_dist_nn_amd.engine import OptimConfig, Trainer  # noqa: E402
from docker_dist_nn_amd.parallel.fan import FanLayout, parse_fan  # noqa: E402
from docker_dist_nn_amd.parallel.planner import Planner, parse_parallelism  # noqa: E402

METRIC = "samples/sec (whole node) MNIST FCNN training at 1/2/4/8-stage pipeline"
# BASELINE.md publishes no number for this metric on this model: vs_baseline is null. The only
# published training throughput of the reference is centralized Keras on a DIFFERENT model
# (784-32-16-10, batch 32, 54,000 samples in ~5 s/epoch on Colab CPU; notebook
# …ipynb:302-361); it is reported as a labelled reference frame, not as vs_baseline.
KERAS_REF_SAMPLES_PER_S = 10_800.0
MODEL_LABEL = {"mnist-fcnn": "784-512-256-128-10 MNIST FCNN",
               "mlp8": "784-1024x7-10 MLP (8 Linear)", "mlp7": "784-1024x6-10 MLP",
               "wide": "784-8192-8192-10 MLP"}


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="mnist-fcnn")
    ap.add_argument("--batch", type=int, default=65536,
                    help="rows per GPU per step (global batch = batch x N)")
    ap.add_argument("--parallelism", default="pipeline")
    ap.add_argument("--schedule", default="auto",
                    help="pipeline schedule; auto = 1f1b_lh (latency-hiding 1F1B) for pipelines "
                         "across GPUs, 1f1b for single-process (loopback) pipelines")
    ap.add_argument("--micro", type=int, default=0, help="micro-batch rows (0 = planner)")
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--optimizer", default="sgd", choices=["sgd", "adam", "adamw"])
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="replay the step as a HIP graph (1 GPU, or N > 1 with the native step). "
                         "auto (default): N > 1 on the IPC transport, kept only if its timed "
                         "steps beat eager ones (the host enqueue of a rank's plan is ~3 us per "
                         "op eager, ~0.4 us per node replayed: profiles/r3_host). The captured "
                         "plan is the slotted single-stream form, deadlock-free whatever order "
                         "the graph executor picks (profiles/r4_multirank); the ladder's later "
                         "rungs run with --graph off")
    ap.add_argument("--graph-copies", type=int, default=2,
                    help="alternate between this many instantiations of the step graph")
    ap.add_argument("--boundary", default="bf16", choices=["bf16", "fp8"],
                    help="pipeline hop format: bf16 (default) or e4m3 rows + fp32 row scales "
                         "(half the xGMI bytes; opt-in, reduced-precision hops)")
    ap.add_argument("--dp-reduce", default="shard", choices=["allreduce", "shard"],
                    help="data-parallel gradient exchange: bf16 reduce-scatter + sharded "
                         "optimizer + bf16 all-gather (default) or fp32 all-reduce")
    ap.add_argument("--no-dp-compare", action="store_true",
                    help="N > 1: skip the data-parallel-only comparison run")
    ap.add_argument("--seed", type=int, default=0)
    return ap.parse_args(argv)


def _plan(a, spec, n, world, text):
    # the relayed IPC transport the trainer picks first on an RCCL job (engine/trainer.py
    # _pick_pipe); a run that falls back to RCCL reports it in "transport"
    kr = switches.get("DNN_IPC_RELAYS")
    relays = ("plan" if kr == "auto" else int(kr)) \
        if switches.get("DNN_PIPE") in ("auto", "ipc") and n > 1 else 0
    planner = Planner.calibrated(spec, relays=relays,
                                 dp_grad_bytes=2.0 if a.dp_reduce == "shard" else 4.0)
    loopback = world == 1
    fan = parse_fan(text)
    if fan is not None:  # 'fan:1x1,2x7' (layers x GPUs per stage), 'fan:1,7' (GPUs only) or
        # 'fan:3x4,1x1@3' (the last stage co-located on rank 3)
        dist_, reps, place = fan
        if not reps or FanLayout(tuple([1] * len(reps)), tuple(reps), place).world != n:
            raise SystemExit(f"--parallelism {text}: the layout must use {n} GPUs")
        if not dist_:
            from docker_dist_nn_amd.parallel.planner import compositions

            dist_ = max(compositions(len(spec.layers), len(reps)),
                        key=lambda d: planner.evaluate_fan(spec, d, reps, a.batch,
                                                           place=place).samples_per_s)
        return planner.evaluate_fan(spec, dist_, reps, a.batch, place=place)
    pp, dp = parse_parallelism("pipeline" if text == "uniform" else text, n, loopback=loopback)
    if pp is None:
        if text == "best":
            return planner.best(spec, n, a.batch)
        if n == 1:
            return planner.evaluate(spec, 1, 1, a.batch)
        if text == "uniform" or loopback:  # the literal ppS x dpD grid (BASELINE's layouts)
            return planner.pipeline_layout(spec, n, a.batch)
        # the pipeline the planner scores best over every layer split and every split of
        # the GPUs into per-stage replica groups (parallel/fan.py; equal counts = ppS x dpD)
        return planner.best_fan(spec, n, a.batch)
    rows = a.batch * (1 if loopback else pp)  # loopback: every stage on the one GPU
    return planner.evaluate(spec, pp, dp, rows, loopback=loopback)


def _uniform_prediction(a, spec, n, world):
    if n < 2 or a.parallelism not in ("pipeline", "auto"):
        return None
    p = _plan(a, spec, n, world, "uniform")
    return {"parallelism": p.parallelism, "layer_distribution": p.distribution,
            "planner_predicted": round(p.samples_per_s, 1)}


def first_step_guard(tr, one_step, dev, timeout_s):
    """Run the first multi-rank step under a watchdog: if it has not completed on the device
    within ``timeout_s`` (a cross-rank hang: a hop or collective whose partner never comes),
    print this rank's plan and exit non-zero instead of hanging the job. The process exits
    with os._exit (no exec, nothing re-launched)."""
    import threading

    done = threading.Event()

    def watch():
        if not done.wait(timeout_s):
            ns = tr.native_step
            rank = os.environ.get("RANK", "?")
            print(f"[bench] rank {rank}: first step not done after {timeout_s:.0f} s; "
                  f"transport {tr.transport}, plan "
                  f"{ns.describe() if ns is not None else 'python executor'}",
                  file=sys.stderr, flush=True)
            if ns is not None:
                print(ns.trace(), file=sys.stderr, flush=True)
            os._exit(3)

    th = threading.Thread(target=watch, daemon=True)
    th.start()
    one_step()
    torch.cuda.synchronize(dev)
    done.set()
    th.join()


def measure(a, spec, n, world, dev, text):
    """Build the trainer for one layout, W warm-up + K timed steps; returns the JSON fields."""
    plan = _plan(a, spec, n, world, text)
    fan = plan.reps is not None and (len(set(plan.reps)) > 1 or plan.colocated)
    lay = FanLayout(tuple(plan.distribution), tuple(plan.reps), plan.place) if fan else None
    if fan and world != lay.world:
        raise SystemExit(f"fan layout {plan.parallelism} needs {lay.world} ranks")
    if plan.reps is not None and not fan:  # equal replica counts: the uniform ppS x dpD grid
        plan.dp = plan.reps[0]
        plan.reps = None
    mb = a.micro or plan.micro_batch
    if fan:  # replicated-stage pipeline (parallel/fan.py): nm = the GLOBAL micro-batch count
        rows = nm = None
        nm = max(1, plan.micro_batch * plan.num_micro // mb)
        if mb * nm != plan.micro_batch * plan.num_micro or mb % 64:
            raise SystemExit(f"batch {plan.micro_batch * plan.num_micro} must split into "
                             "micro-batches of a multiple of 64")
    else:
        rows = a.batch * (1 if world == 1 else plan.pp)  # rows per replica per step
        nm = max(1, rows // mb)
        if mb * nm != rows or mb % 64:
            raise SystemExit(f"batch {rows} must split into micro-batches of a multiple of 64")
    mesh = None
    if fan:
        from docker_dist_nn_amd.data import FanDataset
        from docker_dist_nn_amd.engine.fan_trainer import FanTrainer
        from docker_dist_nn_amd.parallel.fan import build_fan_mesh

        mesh = build_fan_mesh(lay)
        sched = "fan"
        tr = FanTrainer(spec, lay, mesh, micro_batch=mb, num_micro=nm,
                        optim=OptimConfig(name=a.optimizer, lr=a.lr), device=dev, seed=a.seed,
                        dp_reduce=a.dp_reduce)
        data = FanDataset(tr.input_micros, mb, dev,
                          kp=tr.stages[0].x_in.shape[1] if tr.first else None, seed=a.seed,
                          inputs=tr.first is not None, labels=tr.last is not None,
                          label_micros=tr.label_micros)
        global_batch = mb * nm
    else:
        if world > 1:
            from docker_dist_nn_amd.parallel.groups import build_mesh

            mesh = build_mesh(plan.pp, plan.dp)
            # communicator set-up happens at a group's first collective: do it here, outside
            # the W warm-up steps and the timed region
            t = torch.ones(1024, device=dev)
            for g in (mesh.fwd_group, mesh.bwd_group, mesh.dp_group, None):
                torch.distributed.all_reduce(t, group=g)
            torch.cuda.synchronize(dev)
        sched = a.schedule
        if sched == "auto":
            sched = "1f1b_lh" if world > 1 and plan.pp > 1 else "1f1b"
        tr = Trainer(spec, micro_batch=mb, num_micro=nm, distribution=plan.distribution,
                     pp=plan.pp, dp=plan.dp, schedule=sched,
                     optim=OptimConfig(name=a.optimizer, lr=a.lr),
                     device=dev, seed=a.seed, mesh=mesh, boundary=a.boundary,
                     dp_reduce=a.dp_reduce)
        replica = mesh.replica if mesh else 0
        x, y = synthetic_mnist(max(60000, 2 * rows), seed=a.seed + 1000 * replica)
        data = DeviceDataset(x, y, rows, dev,
                             kp=tr.stages[0].x_in.shape[1] if tr.first else None)
        global_batch = rows * plan.dp

    # --graph: the step as a HIP graph (one GPU, or a native multi-rank step: opt-in, the
    # plan's flag waits are kernels so the whole rank step -- hops included -- is captured)
    use_graph = a.graph == "on" and (world == 1 or tr.native_step is not None)
    step_i = 0
    rank = int(os.environ.get("RANK", "0"))
    injector = FaultInjector()  # DNN_FAULT (the ladder's tests): stage = global rank
    beat = ladder.Throttled(5.0)

    def one_step():
        nonlocal step_i
        injector.maybe_inject(rank, step_i)
        xb, yb = data.batch(step_i)
        tr.set_batch(xb if tr.first else None, yb if tr.last else None, zero_copy=True)
        tr.step()
        step_i += 1
        beat(f"step {step_i}")

    ladder.heartbeat("trainer built")
    if world > 1:  # the first multi-rank step is bounded: a hang prints the plan and exits
        first_step_guard(tr, one_step, dev, float(switches.get("DNN_FIRST_STEP_TIMEOUT")))
        ladder.heartbeat("first step done")
    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)

    def timed(k):  # seconds for k steps, max over ranks (every rank gets the same value)
        barrier()
        t = time.perf_counter()
        for _ in range(k):
            one_step()
        barrier()
        t = torch.tensor([time.perf_counter() - t], device=dev, dtype=torch.float64)
        if world > 1:
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        return float(t.item())

    graph_trial = None
    if use_graph:
        xb, yb = data.batch(0)
        tr.set_batch(xb if tr.first else None, yb if tr.last else None)
        tr.capture(copies=a.graph_copies)
    elif a.graph == "auto" and world > 1 and tr.transport == "ipc" and \
            tr.native_step is not None and not fan:
        # (fan plans hold their replicated stages' RCCL all-reduce: they stay eager)
        # the relayed IPC plan is hundreds of ops per rank: replayed as a graph when that
        # measures faster (RCCL plans stay eager: capturing RCCL calls is not validated here)
        eager_s = timed(3)
        xb, yb = data.batch(0)
        tr.set_batch(xb if tr.first else None, yb if tr.last else None)
        tr.capture(copies=a.graph_copies)
        graph_s = timed(3)
        use_graph = graph_s < 0.98 * eager_s
        graph_trial = {"eager_ms": round(eager_s / 3 * 1e3, 4),
                       "graph_ms": round(graph_s / 3 * 1e3, 4), "kept": use_graph}
        if not use_graph:
            tr.release_graph()
    for _ in range(a.warmup):
        one_step()

    # DNN_BENCH_STEP_EVENTS=1 (diagnosis): a HIP event before every timed step and after the
    # last, so the JSON carries the per-step GPU times of the timed window
    evs = [] if switches.get("DNN_BENCH_STEP_EVENTS") == "1" else None
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        if evs is not None:
            evs.append(torch.cuda.Event(enable_timing=True))
            evs[-1].record()
        one_step()
    if evs is not None:
        evs.append(torch.cuda.Event(enable_timing=True))
        evs[-1].record()
    host_s = time.perf_counter() - t0  # enqueue time of the K steps (no sync inside)
    tr.flush()  # the last step's deferred DP update belongs to the timed region
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    loss = tr.loss()
    if world > 1 and fan:  # the last stage's replicas hold shares of the global mean loss
        lt = torch.tensor([loss if loss is not None else 0.0], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(lt)
        loss = float(lt.item())
    elif world > 1:  # the last stage of replica 0 owns the loss; rank 0 prints
        lt = torch.tensor([loss if loss is not None else -1.0], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(lt, op=torch.distributed.ReduceOp.MAX)
        loss = float(lt.item())
    value = global_batch * a.steps / elapsed
    out = {
        "value": round(value, 1), "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "global_batch": global_batch,
        "parallelism": plan.parallelism + ("-loopback" if world == 1 and plan.pp > 1 else ""),
        "layer_distribution": plan.distribution, "micro_batch": mb, "num_micro": nm,
        "stage_gpus": plan.reps if fan else None,
        "stage_place": [list(p) for p in plan.place] if fan and plan.colocated else None,
        "schedule": sched if plan.pp > 1 else "none",
        "transport": tr.transport, "transport_reason": tr.transport_reason,
        "native_step": tr.native_step is not None or world == 1,
        "rccl_plan": tr.native_step.mode if tr.native_step is not None else None,
        "native_fallback": tr.native_fallback,
        "boundary": tr.boundary,
        "dp_reduce": tr.dp_reduce if (plan.dp > 1 or (fan and max(plan.reps) > 1)) else None,
        "hip_graph": use_graph, "graph_copies": a.graph_copies if use_graph else 0,
        "graph_trial": graph_trial, "host_ms_per_step": round(host_s / a.steps * 1e3, 4),
        "step_ms": ([round(e0.elapsed_time(e1), 4) for e0, e1 in zip(evs, evs[1:])]
                    if evs else None),
        "loss": loss, "planner_predicted": round(plan.samples_per_s, 1),
    }
    del tr, data
    gc.collect()
    torch.cuda.empty_cache()
    return out


def measure_tp(a, spec, n, world, dev):
    """--parallelism tpN: Megatron column/row tensor parallelism over all N ranks
    (parallel/tensor.py) on ONE replicated batch of --batch rows (opt-in; not the pipeline
    metric's layout)."""
    from docker_dist_nn_amd.parallel.tensor import TensorParallelMLP

    tp = int(a.parallelism[2:])
    if world != tp:
        raise SystemExit(f"--parallelism tp{tp} needs WORLD_SIZE={tp}")
    rank = int(os.environ.get("RANK", "0"))
    m = TensorParallelMLP(spec, rows=a.batch, tp=tp, rank=rank, device=dev,
                          optim=OptimConfig(name=a.optimizer, lr=a.lr), seed=a.seed)
    x, y = synthetic_mnist(a.batch, seed=a.seed + 1000)
    m.set_batch(torch.from_numpy(x), torch.from_numpy(y))
    for _ in range(a.warmup):
        m.step()
    torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        m.step()
    torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(t.item())
    return {"value": round(a.batch * a.steps / elapsed, 1),
            "ms_per_step": round(elapsed / a.steps * 1e3, 4), "global_batch": a.batch,
            "parallelism": f"tp{tp}", "layer_distribution": [len(spec.layers)],
            "micro_batch": a.batch, "num_micro": 1, "schedule": "none",
            "transport": "rccl" if torch.distributed.get_backend() == "nccl" else "gloo",
            "transport_reason": "tensor parallel collectives",
            "native_step": False, "rccl_plan": None, "boundary": "bf16", "dp_reduce": None,
            "hip_graph": False,
            "graph_copies": 0, "loss": m.loss(), "planner_predicted": None,
            "native_fallback": None}


DP_ONLY_KEYS = ("parallelism", "global_batch", "transport", "native_step", "dp_reduce")


def _summary(d, keys):
    return {"value": d["value"], "ms_per_step": d["ms_per_step"],
            **{k: d["config"].get(k) for k in keys}}


def supervise(a, argv) -> int:
    """WORLD_SIZE > 1: this process is the rank's supervisor (ladder.py). It never touches the
    GPU; every attempt runs ``bench.py`` again as a fresh child per rank (new rendezvous port),
    climbing the fallback ladder until one attempt succeeds on every rank. Then, while the time
    left allows, two comparisons run the same way: the literal uniform ppS x dpD pipeline of
    BASELINE.json (when the main layout was a replicated-stage "fan" pipeline) and pure data
    parallelism. Rank 0 prints the one JSON line, with every attempt (rung, exit codes, last
    heartbeat of a stalled child) listed -- also when the job is ended by SIGTERM
    (ladder.OneLine), so a bench the driver stops at its deadline still reports.

    Time: a failing rung costs at most a child's start-up + the first-step guard
    (DNN_FIRST_STEP_TIMEOUT, 30 s) or a heartbeat stall (DNN_LADDER_STALL, 60 s); past
    DNN_LADDER_BUDGET (360 s) only the last rung is tried; a comparison starts only if 1.5 x the
    main attempt's time + 30 s is left; nothing runs past DNN_LADDER_DEADLINE (540 s from
    start) -- inside a 600-second driver window."""
    t_start = time.monotonic()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ["WORLD_SIZE"])
    base = [sys.executable, "-u", os.path.abspath(__file__),
            *(sys.argv[1:] if argv is None else argv)]
    st = {"res": None, "rung": None, "attempts": [], "extra": {}}
    sup = None
    spec = NAMED_MODELS.get(a.model) or MLPSpec.parse(a.model)

    def entry_json(key, e):
        if e is None:
            return None
        if "skipped" in e:
            return {"value": None, **e}
        d = e["result"]
        if d is None:
            return {"value": None, "error": "every rung failed"}
        if key == "uniform_pipeline":
            return {**_summary(d, ("parallelism", "layer_distribution", "transport",
                                   "rccl_plan")),
                    "planner_predicted": d.get("planner_predicted")}
        return _summary(d, DP_ONLY_KEYS)

    def build(reason):
        attempts = list(sup.attempts) if sup is not None else []
        if st["res"] is None:
            out = {"metric": METRIC, "value": None, "unit": "samples/s", "n_gpus": world,
                   "steps": a.steps, "warmup": a.warmup, "higher_is_better": True,
                   "error": ("terminated before any rung succeeded" if reason else
                             "every rung of the fallback ladder failed"),
                   "ladder": {"attempts": attempts}}
        else:
            out = dict(st["res"])
            n_main = len(st["attempts"])
            for key in ("uniform_pipeline", "dp_only"):
                e = st["extra"].get(key)
                if e is not None:  # measured (or skipped) over the child's prediction
                    out[key] = {**(out.get(key) or {}), **entry_json(key, e)}
                elif reason and key in st["pending"]:
                    out[key] = {**(out.get(key) or {}), "value": None, "skipped": "terminated"}
            out["ladder"] = {"rung": st["rung"], "attempts": st["attempts"],
                             "compare_attempts": attempts[n_main:]}
        out["ladder"]["seconds"] = round(time.monotonic() - t_start, 1)
        if reason:
            out["terminated"] = reason
        return out

    line = ladder.OneLine(rank, build)
    line.install_sigterm()  # before the Supervisor's handler, which chains to it
    sup = ladder.Supervisor(lambda r: [*base, *r.args, "--no-dp-compare"], rank=rank,
                            world=world, stall=float(switches.get("DNN_LADDER_STALL")),
                            startup=float(switches.get("DNN_LADDER_STARTUP")),
                            deadline=t_start + float(switches.get("DNN_LADDER_DEADLINE")))
    is_fan = False
    if a.parallelism.startswith("tp"):
        rungs = [ladder.Rung("default")]
    else:
        # the planner runs on the CPU: the supervisor knows whether the default layout is a
        # replicated-stage pipeline without touching the GPU
        if not a.parallelism.startswith("dp"):
            p = _plan(a, spec, world, world, a.parallelism)
            is_fan = p.reps is not None and (len(set(p.reps)) > 1 or p.colocated)
        rungs = ladder.bench_rungs(world, dp_only=a.parallelism.startswith("dp"), fan=is_fan)
    st["pending"] = []
    res, rung = sup.climb(rungs, budget_s=float(switches.get("DNN_LADDER_BUDGET")))
    st.update(res=res, rung=rung.name if rung else None, attempts=list(sup.attempts))
    if res is not None:
        lay = res["config"]["parallelism"]
        items = []
        # the literal BASELINE grid, measured, when the main number came from a fan layout
        if is_fan and lay.startswith("fan"):
            items.append(("uniform_pipeline", ladder.uniform_rungs()))
        if not a.no_dp_compare and not lay.startswith(("dp", "tp")):
            items.append(("dp_only", ladder.bench_rungs(world, dp_only=True)))
        st["pending"] = [k for k, _ in items]
        need = 1.5 * sup.attempts[-1]["seconds"] + 30
        sup.comparisons(items, need, on_done=lambda k, e: st["extra"].__setitem__(k, e))
    line.emit()
    return 0 if res is not None else 1


def main(argv=None):
    a = parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus != world and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if world > 1 and not ladder.is_child() and switches.get("DNN_LADDER") == "1":
        return supervise(a, argv)
    ladder.heartbeat("start")
    n = max(a.gpus, world)
    spec = NAMED_MODELS.get(a.model) or MLPSpec.parse(a.model)

    # DNN_FORCE_DEVICE / DNN_DIST_BACKEND exist only to rehearse the multi-rank path on a
    # one-GPU box (several gloo ranks sharing cuda:0); real runs use one GPU per rank + RCCL.
    local = int(switches.get("DNN_FORCE_DEVICE") or os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        from docker_dist_nn_amd.parallel.groups import init_distributed

        init_distributed(switches.get("DNN_DIST_BACKEND"))
        ladder.heartbeat("rendezvous done")

    if a.parallelism.startswith("tp"):
        m = measure_tp(a, spec, n, world, dev)
    else:
        m = measure(a, spec, n, world, dev, a.parallelism)
    uniform = _uniform_prediction(a, spec, n, world)
    if world > 1 and not ladder.is_child() and m["parallelism"].startswith("fan"):
        # without the ladder (DNN_LADDER=0): the literal grid measured in-process too
        u = measure(a, spec, n, world, dev, "uniform")
        uniform = {**(uniform or {}), "value": u["value"], "ms_per_step": u["ms_per_step"],
                   "parallelism": u["parallelism"], "layer_distribution": u["layer_distribution"],
                   "transport": u["transport"], "rccl_plan": u["rccl_plan"]}
    dp_only = None
    if world > 1 and not a.no_dp_compare and not m["parallelism"].startswith(("dp", "tp")):
        d = measure(a, spec, n, world, dev, f"dp{n}")
        dp_only = {k: d[k] for k in ("value", "ms_per_step", "parallelism", "global_batch",
                                     "transport", "native_step", "dp_reduce")}
    out = {
        "metric": METRIC,
        "value": m["value"],
        "unit": "samples/s",
        "n_gpus": n,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": m["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "reference_frame": {
            "label": "vs Keras 784-32-16-10 CPU training (different model, BASELINE.md)",
            "samples_per_s": KERAS_REF_SAMPLES_PER_S,
            "ratio": round(m["value"] / KERAS_REF_SAMPLES_PER_S, 1)},
        "dtype": "bf16",
        "data": "synthetic (MNIST-shaped 784-feature inputs, teacher labels; random-init weights)",
        "config": {
            "model": MODEL_LABEL.get(a.model, spec.describe()),
            "global_batch": m["global_batch"],
            "seq_len": None,
            **{k: m.get(k) for k in ("parallelism", "layer_distribution", "stage_gpus",
                                 "stage_place",
                                 "micro_batch", "num_micro",
                                 "schedule", "transport", "transport_reason", "native_step",
                                 "rccl_plan",
                                 "boundary", "dp_reduce", "hip_graph", "graph_copies")},
            "optimizer": a.optimizer,
        },
        # EXECUTED FLOPs (no dgrad of the first layer: models/mlp.py)
        "model_tflops": round(spec.flops_per_sample_train() * m["value"] / 1e12, 1),
        "last_loss": None if m["loss"] is None else round(m["loss"], 5),
        "planner_predicted": m["planner_predicted"],
        "host_ms_per_step": m.get("host_ms_per_step"),
        **({"step_ms": m["step_ms"]} if m.get("step_ms") else {}),
        "graph_trial": m.get("graph_trial"),
        "dp_only": dp_only,
        # the literal uniform ppS x dpD grid of BASELINE.json: predicted by the same planner,
        # measured too after a fan layout's number (the supervisor's comparison; in-process
        # without the ladder)
        "uniform_pipeline": uniform,
        "native_fallback": m["native_fallback"],  # why the Python executor ran, if it did
        "switches": switches.active(),  # non-default DNN_* switches of this run
    }
    rank = int(os.environ.get("RANK", "0"))
    if ladder.is_child():
        out["ladder_rung"] = os.environ.get(ladder.RUNG_ENV)
    if rank == 0 and not ladder.write_result(out):
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
