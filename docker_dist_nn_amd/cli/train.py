"""Pipelined training CLI: ``python -m docker_dist_nn_amd.cli.train`` (single process) or
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 -m
docker_dist_nn_amd.cli.train ...`` (one rank per GPU, PP x DP).

This is the distributed version of the reference's centralized recipes
(/root/reference/scripts/generate_mnist_pytorch.py:35-52, notebook …ipynb:274-285): softmax
cross-entropy on the last layer's logits, mini-batch optimizer steps; the trained weights are
exported in the reference's neuron-JSON format with the notebook's ``inference_metrics``
block (accuracy / weighted precision, recall, F1 / latency, …ipynb:493-506).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time
from typing import Optional

import numpy as np

if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not os.environ.get("DNN_FORCE_DEVICE"):
    # one hardware queue per stream (see bench.py); the box exports 4, so raise it
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 24:  # see bench.py
        os.environ["GPU_MAX_HW_QUEUES"] = "24"

import torch  # noqa: E402

log = logging.getLogger("train")


def prepare_data(examples, synthetic: int, input_dim: int, seed: int):
    from ..data import synthetic_mnist

    if synthetic or examples is None or len(examples) == 0 or (examples.labels < 0).all():
        n = synthetic or 60000
        x, y = synthetic_mnist(n, seed=seed, dim=input_dim)
        return x, y, "synthetic"
    if examples.dim != input_dim:
        raise ValueError(f"inputs have {examples.dim} features but the model expects {input_dim}")
    return examples.x, examples.labels, "inputs"


def _batches(x, y, rows: int, kp: int, device, epoch_seed: int):
    n = x.shape[0]
    order = np.random.default_rng(epoch_seed).permutation(n)
    for s in range(0, n, rows):
        idx = order[s:s + rows]
        xb = torch.zeros(rows, kp, dtype=torch.bfloat16)
        xb[:len(idx), :x.shape[1]] = torch.from_numpy(x[idx]).to(torch.bfloat16)
        yb = torch.full((rows,), -1, dtype=torch.int32)
        yb[:len(idx)] = torch.from_numpy(y[idx].astype(np.int32))
        yield xb.to(device), yb.to(device), len(idx)


def evaluate(ws, bs, acts, x, y, device, batch: int = 65536) -> dict:
    from ..config import LayerWeights
    from ..engine.inference import InferenceEngine
    from ..metrics import classification_report

    layers = [LayerWeights(w, b, a) for w, b, a in zip(ws, bs, acts)]
    eng = InferenceEngine([layers], device, expected_input=layers[0].in_dim, max_rows=batch)
    t0 = time.time()
    out = eng.predict(x)
    dt = time.time() - t0
    rep = classification_report(y, out.argmax(1), n_classes=out.shape[1])
    rep.update(total_latency_sec=dt, avg_latency_per_sample_sec=dt / max(1, len(x)))
    return rep


def train_model(mc, examples, a, distribution, random_init: bool):
    """Local (single-process) training used by ``run_grpc_fcnn.py --train``."""
    from ..engine import OptimConfig, Trainer
    from ..metrics import MetricsWriter

    spec = mc.spec()
    dev = torch.device("cpu") if getattr(a, "device", "auto") == "cpu" or \
        not torch.cuda.is_available() else torch.device("cuda", 0)
    x, y, src = prepare_data(examples, a.synthetic, spec.in_dim, a.seed)
    pp = sum(1 for d in distribution if d)
    tr = Trainer(spec, micro_batch=a.micro_batch, num_micro=a.num_micro_batches, pp=pp,
                 distribution=distribution, schedule=a.schedule,
                 optim=OptimConfig(name=a.optimizer, lr=a.lr, momentum=a.momentum),
                 device=dev, seed=a.seed)
    if not random_init:
        tr.load_weights([L.weight for L in mc.layers], [L.bias for L in mc.layers])
    mw = MetricsWriter(getattr(a, "metrics", None))
    rows = a.micro_batch * a.num_micro_batches
    kp = tr.stages[0].x_in.shape[1]
    step, t0, loss = 0, time.time(), None
    for ep in range(max(1, a.epochs)):
        for xb, yb, n in _batches(x, y, rows, kp, dev, a.seed + ep):
            tr.set_batch(xb, yb)
            tr.step()
            step += 1
            if step % 50 == 0 or (a.steps and step >= a.steps):
                loss = tr.loss()
                mw.write("train", step=step, loss=loss, samples_per_s=step * rows / (time.time() - t0))
            if a.steps and step >= a.steps:
                break
        if a.steps and step >= a.steps:
            break
        loss = tr.loss()
        log.info(f"Epoch {ep + 1}, Loss: {loss:.5f} ({src} data, {step} steps)")
    loss = tr.loss()
    elapsed = time.time() - t0
    ww = tr.local_weights()
    ws = [ww[i][0] for i in range(len(spec.layers))]
    bs = [ww[i][1] for i in range(len(spec.layers))]
    metrics = evaluate(ws, bs, [l.activation for l in spec.layers], x, y, dev)
    report = {"steps": step, "final_loss": loss, "train_seconds": elapsed,
              "samples_per_s": step * rows / max(elapsed, 1e-9), "data": src,
              "inference_metrics": metrics}
    mw.write("done", **{k: v for k, v in report.items() if k != "inference_metrics"})
    mw.close()
    return ws, bs, report


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Pipelined PP x DP MLP training on MI355X")
    ap.add_argument("--model", default="mnist-fcnn", help="named model or widths '784-512-10'")
    ap.add_argument("--config", default=None, help="reference model JSON to start from")
    ap.add_argument("--inputs", default=None, help="reference inputs JSON with labels")
    ap.add_argument("--synthetic", type=int, default=60000)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--optimizer", choices=["sgd", "adam", "adamw"], default="sgd")
    ap.add_argument("--momentum", type=float, default=0.0)
    ap.add_argument("--weight-decay", type=float, default=0.0)
    ap.add_argument("--micro-batch", type=int, default=4096)
    ap.add_argument("--num-micro-batches", type=int, default=1)
    ap.add_argument("--pp", type=int, default=0, help="pipeline stages (0 = planner)")
    ap.add_argument("--layer-distribution", default=None)
    ap.add_argument("--schedule", choices=["gpipe", "1f1b", "1f1b_lh", "1f1b_w", "zb"], default="1f1b")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--save", default=None, help="export trained model JSON (reference format)")
    ap.add_argument("--checkpoint-dir", default=None)
    ap.add_argument("--checkpoint-every", type=int, default=0)
    ap.add_argument("--resume", action="store_true")
    ap.add_argument("--metrics", default=None, help="JSONL metrics path ({rank} expands)")
    ap.add_argument("--trace", default=None, help="chrome trace of the last step ({rank})")
    ap.add_argument("--watchdog", type=float, default=None,
                    help="seconds without step progress before the rank dumps its stacks and "
                         "exits (default: 300 for multi-rank jobs, off for one process; 0 = off)")
    ap.add_argument("--dp-reduce", default="allreduce", choices=["allreduce", "shard"],
                    help="data-parallel gradients: fp32 all-reduce + replicated optimizer, or "
                         "bf16 reduce-scatter + sharded optimizer + bf16 weight all-gather")
    ap.add_argument("--check-every", type=int, default=20,
                    help="steps between loss finiteness / RCCL async-error checks")
    return ap


def main(argv: Optional[list[str]] = None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    a = build_parser().parse_args(argv)
    from .. import checkpoint as ckpt
    from ..config import load_model_config
    from ..data import load_examples
    from ..engine import OptimConfig, Trainer
    from ..engine.trainer import default_distribution
    from ..faults import FaultInjector, Watchdog, check_finite
    from ..metrics import MetricsWriter
    from ..models.mlp import NAMED_MODELS, MLPSpec
    from ..profiler import StepProfiler

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    mc = load_model_config(a.config) if a.config else None
    spec = mc.spec() if mc else (NAMED_MODELS.get(a.model) or MLPSpec.parse(a.model))
    if a.device == "cpu" or not torch.cuda.is_available():
        dev = torch.device("cpu")
    else:
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(dev)
    mesh = None
    if world > 1:
        from ..parallel.groups import build_mesh, init_distributed

        init_distributed("nccl" if dev.type == "cuda" else "gloo")
    pp = a.pp or (world if world <= len(spec.layers) else 1)
    if world > 1 and world % pp:
        raise SystemExit(f"--pp {pp} does not divide world size {world}")
    dp = world // pp if world > 1 else 1  # single process: pp stages on one device (loopback)
    dist_ = json.loads(a.layer_distribution) if a.layer_distribution else \
        (mc.layer_distribution if mc and mc.layer_distribution and
         sum(1 for d in mc.layer_distribution if d) == pp else default_distribution(spec, pp))
    if world > 1:
        mesh = build_mesh(pp, dp)
    tr = Trainer(spec, micro_batch=a.micro_batch, num_micro=a.num_micro_batches, pp=pp, dp=dp,
                 distribution=dist_, schedule=a.schedule, mesh=mesh, device=dev, seed=a.seed,
                 optim=OptimConfig(name=a.optimizer, lr=a.lr, momentum=a.momentum,
                                   weight_decay=a.weight_decay), dp_reduce=a.dp_reduce)
    start_step = 0
    if a.resume and a.checkpoint_dir and os.path.exists(os.path.join(a.checkpoint_dir, "meta.json")):
        # any layout: weights AND optimizer state are stored per layer (re-partition is exact)
        start_step = ckpt.restore_trainer(a.checkpoint_dir, tr)
        log.info(f"resumed from {a.checkpoint_dir} at step {start_step} "
                 f"(saved layout {ckpt.read_meta(a.checkpoint_dir)['layer_distribution']}, "
                 f"now {list(dist_)})")
    elif mc is not None:
        tr.load_weights([L.weight for L in mc.layers], [L.bias for L in mc.layers])

    replica = mesh.replica if mesh else 0
    ex = load_examples(a.inputs) if a.inputs else None
    x, y, src = prepare_data(ex, 0 if ex is not None else a.synthetic, spec.in_dim, a.seed)
    rows = a.micro_batch * a.num_micro_batches
    shard = slice(replica, None, dp)  # each replica sees a disjoint strided shard
    x, y = x[shard], y[shard]
    kp = (spec.in_dim + 63) // 64 * 64  # the FIRST stage's padded input width (on every rank)
    mw = MetricsWriter(a.metrics.format(rank=rank) if a.metrics else None, rank)
    prof = StepProfiler(tr.executor, rank, enabled=bool(a.trace))
    if a.watchdog is None:  # on by default wherever a peer can hang us
        a.watchdog = 300.0 if world > 1 else 0.0
    wd = Watchdog(a.watchdog, name=f"rank{rank}").start() if a.watchdog else None
    faults = FaultInjector()
    sid = tr.stages[0].stage_index
    step, t0 = start_step, time.time()
    done = False
    barrier = torch.distributed.barrier if world > 1 else None

    def comm_healthy() -> bool:
        """No RCCL async error and no timed-out IPC flag wait on ANY rank (a timed-out wait
        lets the step consume rows that never arrived): agreed over the world group."""
        bad = 0.0
        if tr.native_step is not None:
            bad = 1.0 if tr.native_step.comm_error() else 0.0
        if world > 1:
            t = torch.tensor([bad], device=dev if torch.distributed.get_backend() == "nccl"
                             else "cpu")
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            bad = float(t.item())
        return bad == 0.0

    def save(step_):
        # never commit a checkpoint built from a step whose hops failed
        if not comm_healthy():
            raise RuntimeError(f"rank {rank}: communication error or flag-wait timeout before "
                               f"the step-{step_} checkpoint; not committing it")
        ckpt.save_trainer(a.checkpoint_dir, tr, step_, barrier=barrier, is_writer=replica == 0,
                          extra={"seed": a.seed, "rows_per_step": rows, "dp": dp})

    per_epoch = -(-x.shape[0] // rows)
    if a.steps and start_step >= a.steps:
        done = True
    for ep in range(max(1, a.epochs)):
        if done:
            break
        if (ep + 1) * per_epoch <= start_step:
            continue  # epoch fully consumed before the checkpoint
        skip = max(0, start_step - ep * per_epoch)
        for bi, (xb, yb, _) in enumerate(_batches(x, y, rows, kp, dev, a.seed + ep)):
            if bi < skip:
                continue  # resume: the batch order is seeded per epoch, skip what was trained
            faults.maybe_inject(sid, step, tr.stages[0])
            tr.set_batch(xb if tr.first else None, yb if tr.last else None)
            tr.step()
            step += 1
            if wd:
                wd.beat(f"step {step}")
            if a.trace:
                prof.collect()
            if a.check_every and step % a.check_every == 0:
                if tr.native_step is not None:  # RCCL async errors of this rank's comms
                    err = tr.native_step.comm_error()
                    if err:
                        raise RuntimeError(f"rank {rank}: RCCL async error {err} at step {step}")
                loss = tr.loss()
                check_finite(loss)
                mw.write("train", step=step, loss=loss,
                         samples_per_s=(step - start_step) * rows * dp / (time.time() - t0))
            if a.checkpoint_dir and a.checkpoint_every and step % a.checkpoint_every == 0:
                save(step)
            if a.steps and step >= a.steps:
                done = True
                break
        if tr.last is not None:
            log.info(f"Epoch {ep + 1}, Loss: {tr.loss():.5f}")
        if done:
            break
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    elapsed = time.time() - t0
    if wd:
        wd.stop()
    if a.trace and prof.steps:
        prof.chrome_trace(a.trace.format(rank=rank))
        log.info(f"step profile: {StepProfiler.summarize(prof.steps[-1])}")
    tr.flush()
    if a.checkpoint_dir:
        save(step)
    rate = (step - start_step) * rows * dp / max(elapsed, 1e-9)
    mw.write("done", step=step, samples_per_s=rate, loss=tr.loss())
    mw.close()
    if a.save:
        if world > 1:
            torch.distributed.barrier()
            if rank == 0 and a.checkpoint_dir:
                ckpt.export_json(a.checkpoint_dir, a.save, wrapped=False)
        else:
            from ..weights_io import export_model_json

            ww = tr.local_weights()
            export_model_json(a.save, [ww[i][0] for i in range(len(spec.layers))],
                              [ww[i][1] for i in range(len(spec.layers))],
                              [l.activation for l in spec.layers], layer_distribution=dist_)
    if rank == 0:
        print(json.dumps({"steps": step, "samples_per_s": rate, "loss": tr.loss(),
                          "parallelism": f"pp{pp}dp{dp}", "data": src}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
