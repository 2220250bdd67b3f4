"""``run_grpc_fcnn.py`` -- bring up the distributed FCNN, optionally train it, serve, tear down.

Reference contract kept (/root/reference/src/run_grpc_fcnn.py:257-363):
  * flags ``--config`` / ``--inputs`` with the same script-relative defaults;
  * the model file's ``layers`` + ``layer_distribution`` (default ``[1]``) define the stages;
    the notebook's ``{"model": ...}`` form is accepted too;
  * the stage mapping (names ``layer_container_<i>``, ports ``5100+100*i+1``, expected input
    dims, 0-layer stages skipped) and the per-stage weight files
    ``cache/neuron_configs/<name>_neurons_config.json`` (``{"layer_1": [...]}``);
  * log lines "Loaded model config from: ...", "Layer distribution: ...",
    "Distributed FCNN setup completed in X seconds.", then block until Ctrl+C and tear down.
What changes: a stage is a GPU process (``--mode ranks``, RCCL hops) or an in-process stage
(``--mode local``) running gfx950 kernels instead of a Docker container running NumPy, the
gRPC ingress on port 5101 speaks the reference protocol, and ``--train`` trains the model
first with the pipelined engine (new flags are additive).
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

SCRIPT_DIR_DEFAULT = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "src")
log = logging.getLogger("run_grpc_fcnn")


def build_parser(script_dir: str) -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(
        description="Run a distributed FCNN on MI355X stages (reference-compatible CLI).")
    ap.add_argument("--config", type=str,
                    default=os.path.join(script_dir, "../config/mnist_model(10).json"),
                    help="Path to the model configuration JSON file")
    ap.add_argument("--inputs", type=str,
                    default=os.path.join(script_dir, "../config/example_inputs/mnist_examples_5.json"),
                    help="Path to the example inputs JSON file")
    # additive flags
    ap.add_argument("--mode", choices=["auto", "local", "ranks", "workers"], default="auto",
                    help="ranks: one process per stage/GPU (RCCL); local: all stages in-process; "
                         "workers: one gRPC stage process per stage on the reference's env "
                         "contract (grpc_node.py), chained over gRPC")
    ap.add_argument("--device", default="auto", help="auto | cpu | cuda")
    ap.add_argument("--port", type=int, default=5101)
    ap.add_argument("--layer-distribution", type=str, default=None,
                    help="override, e.g. '[1,1,1]'")
    ap.add_argument("--cache-dir", type=str, default=os.path.join(script_dir, "cache/neuron_configs"))
    ap.add_argument("--hop-timeout", type=float, default=10.0,
                    help="per-hop deadline of the stage chain (reference: 10 s, grpc_node.py:133)")
    ap.add_argument("--run-for", type=float, default=0.0,
                    help="serve this many seconds then shut down (0 = until Ctrl+C)")
    ap.add_argument("--no-serve", action="store_true", help="exit after setup/training")
    ap.add_argument("--train", action="store_true", help="train before serving")
    ap.add_argument("--model", type=str, default=None,
                    help="model spec for a random-init model when --config does not exist")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--steps", type=int, default=0, help="train steps (overrides --epochs)")
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--optimizer", choices=["sgd", "adam", "adamw"], default="sgd")
    ap.add_argument("--momentum", type=float, default=0.0)
    ap.add_argument("--micro-batch", type=int, default=256)
    ap.add_argument("--num-micro-batches", type=int, default=1)
    ap.add_argument("--schedule", choices=["gpipe", "1f1b", "1f1b_lh", "1f1b_w", "zb"], default="1f1b")
    ap.add_argument("--synthetic", type=int, default=0,
                    help="train on N synthetic MNIST-shaped samples instead of --inputs")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--save", type=str, default=None, help="write the (trained) model JSON here")
    ap.add_argument("--checkpoint-dir", type=str, default=None)
    ap.add_argument("--metrics", type=str, default=None, help="JSONL metrics stream path")
    return ap


def _device(name: str):
    import torch

    if name == "cpu" or (name == "auto" and not torch.cuda.is_available()):
        return torch.device("cpu")
    return torch.device("cuda", 0)


def train_ranks(mc, a, distribution, random_init: bool, n_st: int):
    """``--train`` with one rank per non-empty stage (reference: one container per stage,
    /root/reference/src/run_grpc_fcnn.py:83-155): the pipelined trainer (cli/train.py) under
    launch.spawn_ranks -- RCCL hops on GPUs, gloo with ``--device cpu`` -- exporting the
    trained model from its committed checkpoint; returns (weights, biases, report)."""
    import tempfile

    from ..config import load_model_config
    from ..launch import spawn_ranks
    from ..weights_io import export_model_json

    with tempfile.TemporaryDirectory(prefix="fcnn_train_") as tmp:
        args = ["--layer-distribution", json.dumps(list(distribution)), "--pp", str(n_st),
                "--lr", str(a.lr), "--optimizer", a.optimizer, "--momentum", str(a.momentum),
                "--micro-batch", str(a.micro_batch),
                "--num-micro-batches", str(a.num_micro_batches), "--schedule", a.schedule,
                "--seed", str(a.seed), "--epochs", str(a.epochs), "--steps", str(a.steps),
                "--checkpoint-dir", os.path.join(tmp, "ckpt"),
                "--save", os.path.join(tmp, "trained.json"),
                "--device", "cpu" if a.device == "cpu" else "auto"]
        if random_init:
            args += ["--model", "-".join(str(w) for w in mc.spec().widths)]
        else:
            cfg = os.path.join(tmp, "start.json")
            export_model_json(cfg, [L.weight for L in mc.layers], [L.bias for L in mc.layers],
                              [L.activation for L in mc.layers],
                              layer_distribution=list(distribution))
            args += ["--config", cfg]
        if a.synthetic:
            args += ["--synthetic", str(a.synthetic)]
        elif os.path.exists(a.inputs):
            args += ["--inputs", os.path.abspath(a.inputs)]
        if a.metrics:
            args += ["--metrics", a.metrics]
        log.info(f"training with {n_st} ranks (one per stage): {' '.join(args)}")
        t0 = time.time()
        job = spawn_ranks("docker_dist_nn_amd.cli.train", args, n_st,
                          names=[f"train_stage{i}" for i in range(n_st)])
        try:
            codes = job.wait()
        finally:
            job.terminate()
        if any(codes):
            raise RuntimeError(f"training ranks exited with {codes}")
        out = load_model_config(os.path.join(tmp, "trained.json"))
    report = {"ranks": n_st, "train_seconds": time.time() - t0,
              "layer_distribution": list(distribution)}
    return [L.weight for L in out.layers], [L.bias for L in out.layers], report


def main(argv: Optional[list[str]] = None, script_dir: str = SCRIPT_DIR_DEFAULT) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    a = build_parser(script_dir).parse_args(argv)
    start_time = time.time()

    from ..config import ModelConfig, LayerWeights, load_model_config
    from ..data import load_examples
    from ..models.mlp import MLPSpec
    from ..partition import calculate_layer_mappings, plan_stages

    # ---- model config ----------------------------------------------------------------------
    try:
        if not os.path.exists(a.config) and a.model:
            spec = MLPSpec.parse(a.model)
            mc = ModelConfig([LayerWeights(np.zeros((l.out_dim, l.in_dim), np.float32),
                                           np.zeros(l.out_dim, np.float32), l.activation, l.type,
                                           l.out_dim) for l in spec.layers],
                             [len(spec.layers)], source=a.model)
            random_init = True
        else:
            mc = load_model_config(a.config)
            random_init = False
        distribution = json.loads(a.layer_distribution) if a.layer_distribution else mc.distribution
        log.info(f"Loaded model config from: {a.config if not random_init else a.model}")
        log.info(f"Layer distribution: {distribution}")
    except FileNotFoundError:
        log.error(f"Configuration file not found: {a.config}")
        return 1
    except (KeyError, json.JSONDecodeError, ValueError) as e:
        log.error(f"Error loading or parsing config file {a.config}: {e}")
        return 1

    # ---- inputs (input dim, and training data for --train) ----------------------------------
    examples = None
    try:
        examples = load_examples(a.inputs)
        log.info(f"Loaded example inputs from: {a.inputs}")
    except FileNotFoundError:
        if not (a.train and a.synthetic):
            log.error(f"Inputs file not found: {a.inputs}")
            return 1
    except (json.JSONDecodeError, ValueError, RuntimeError) as e:
        log.error(f"Error parsing inputs file {a.inputs}: {e}")
        return 1
    input_dim = 0
    if examples is not None and len(examples) and not examples.raw_list:
        input_dim = examples.outer_len  # reference rule: len(examples[0]["input"])
    if input_dim == 0:
        input_dim = mc.layers[0].in_dim
        log.warning("Could not determine initial input dimension from example inputs; "
                    f"using the model's first-layer width {input_dim}.")

    # ---- stage mapping (reference semantics) ------------------------------------------------
    try:
        layer_stub = [{"nodes": L.out_dim, "neurons": []} for L in mc.layers]
        mappings = calculate_layer_mappings(layer_stub, distribution,
                                            [{"input": [0.0] * input_dim}])
        plans = plan_stages(len(mc.layers), distribution)
    except (ValueError, IndexError) as e:
        log.error(f"Error calculating layer mappings: {e}")
        return 1

    # ---- optional training -----------------------------------------------------------------
    if a.train:
        import torch

        from .train import train_model

        n_st = len(plans)
        ranks = n_st > 1 and (a.mode == "ranks" or (
            a.mode == "auto" and a.device != "cpu" and torch.cuda.device_count() >= n_st))
        try:
            if ranks:  # one process (GPU) per non-empty stage, like the reference's containers
                ws, bs, report = train_ranks(mc, a, distribution, random_init, n_st)
            else:
                ws, bs, report = train_model(mc, examples, a, distribution, random_init)
        except (ValueError, RuntimeError) as e:
            log.error(f"Training failed: {e}")
            return 1
        for L, w, b in zip(mc.layers, ws, bs):
            L.weight, L.bias = w, b
        log.info(f"Training finished: {report}")
        if a.save:
            from ..weights_io import export_model_json

            export_model_json(a.save, ws, bs, [L.activation for L in mc.layers],
                              layer_distribution=distribution, wrapped=True,
                              inference_metrics=report.get("inference_metrics"))
            log.info(f"Saved trained model to {a.save}")

    # ---- per-stage weight files (reference format) -------------------------------------------
    from ..utils.native import native

    os.makedirs(a.cache_dir, exist_ok=True)
    stage_entries = []
    for p in plans:
        m = mappings[p.container]
        layers = mc.layers[p.layer_start:p.layer_end]
        path = os.path.join(a.cache_dir, f"{m['container_name']}_neurons_config.json")
        native().write_neuron_json(path, [np.ascontiguousarray(L.weight, np.float32) for L in layers],
                                   [np.ascontiguousarray(L.bias, np.float32) for L in layers],
                                   [L.activation for L in layers],
                                   [L.type or "hidden" for L in layers], [], True)
        stage_entries.append({"name": m["container_name"], "port": m["listen_port"],
                              "expected_input": m["expected_input"], "neurons_file": path,
                              "out_dim": layers[-1].out_dim, "next_nodes": m["next_nodes"]})
    if a.no_serve:
        log.info(f"Distributed FCNN setup completed in {time.time() - start_time:.3f} seconds.")
        return 0

    # ---- bring-up ---------------------------------------------------------------------------
    import torch

    n_st = len(plans)
    mode = a.mode
    if mode == "auto":
        mode = "ranks" if (n_st > 1 and a.device != "cpu" and torch.cuda.device_count() >= n_st) \
            else "local"
    job = server = None
    rc = 0

    def _term(signum, frame):  # SIGTERM behaves like Ctrl+C: always tear the ranks down
        raise KeyboardInterrupt
    import signal

    signal.signal(signal.SIGTERM, _term)
    try:
        if mode == "local":
            from ..engine.inference import InferenceEngine
            from ..serve.ingress import serve

            dev = _device(a.device)
            eng = InferenceEngine([mc.layers[p.layer_start:p.layer_end] for p in plans], dev,
                                  expected_input=input_dim, names=[s["name"] for s in stage_entries])
            server = serve(eng.predict, port=a.port, name=stage_entries[0]["name"])
        elif mode == "workers":
            from ..launch import spawn_workers, wait_for_port
            from ..weights_io import stage_files_from_model

            envs = stage_files_from_model(mc, a.cache_dir, input_dim, distribution)
            order = sorted(envs)
            port_of = {}
            for k, ci in enumerate(order):  # base port --port, +100 per stage (5101, 5201, ...)
                port_of[str(envs[ci]["LISTEN_PORT"])] = str(a.port + 100 * k)
            stage_envs = []
            for k, ci in enumerate(order):
                e = dict(envs[ci])
                e["LISTEN_PORT"] = port_of[e["LISTEN_PORT"]]
                # containers resolved each other by name on the Docker network; local stage
                # processes are on 127.0.0.1
                e["NEXT_NODES"] = json.dumps([{"host": "127.0.0.1",
                                               "port": port_of.get(str(n["port"]), str(n["port"]))}
                                              for n in json.loads(e["NEXT_NODES"])])
                e["DNN_HOP_TIMEOUT"] = str(a.hop_timeout)
                e["DNN_WORKER_DEVICE"] = "cpu" if a.device == "cpu" else "auto"
                e["LOCAL_RANK"] = str(k)
                stage_envs.append(e)
            job = spawn_workers("docker_dist_nn_amd.serve.worker", stage_envs,
                                names=[s["name"] for s in stage_entries], pid_dir=a.cache_dir)
            for e in stage_envs:  # every stage must listen (the reference probed stage 0 only)
                if not wait_for_port(int(e["LISTEN_PORT"]), timeout=120.0, alive=job.alive):
                    job.poll()
                    raise RuntimeError(f"stage {e['CONTAINER_NAME']} did not start listening "
                                       f"on port {e['LISTEN_PORT']}")
        else:
            from ..launch import spawn_ranks, wait_for_port

            plan_path = os.path.join(a.cache_dir, "chain_plan.json")
            json.dump({"stages": stage_entries, "port": a.port, "hop_timeout": a.hop_timeout,
                       "device": "cpu" if a.device == "cpu" else "auto"}, open(plan_path, "w"))
            job = spawn_ranks("docker_dist_nn_amd.serve.chain", ["--plan", plan_path], n_st,
                              devices=list(range(n_st)) if a.device != "cpu" else None,
                              names=[s["name"] for s in stage_entries])
            if not wait_for_port(a.port, timeout=120.0, alive=job.alive):
                job.poll()
                raise RuntimeError(f"first stage did not start listening on port {a.port}")
        log.info(f"Distributed FCNN setup completed in {time.time() - start_time:.3f} seconds.")
        log.info(f"{n_st} stage(s) running ({mode} mode). Press Ctrl+C to shut down.")
        # readiness marker for orchestration: every stage is up (the reference only probed
        # stage 0 and ignored the result, run_grpc_fcnn.py:319)
        with open(os.path.join(a.cache_dir, "chain_ready.json"), "w") as f:
            json.dump({"mode": mode, "port": a.port, "stages": [s["name"] for s in stage_entries],
                       "pid": os.getpid()}, f)
        t0 = time.time()
        reported = set()
        while not a.run_for or time.time() - t0 < a.run_for:
            time.sleep(0.2)
            if job is not None and mode == "workers":
                # independent stage servers, like the reference's containers: a dead stage is
                # reported (its upstream answers UNAVAILABLE "Failed to forward request to
                # ..."), the others keep serving
                for r, pr in enumerate(job.procs):
                    if pr.poll() is not None and r not in reported:
                        reported.add(r)
                        log.error(f"stage {job.names[r]} exited with code {pr.returncode}")
            elif job is not None:
                job.poll()  # RCCL ranks: one dead rank breaks the communicators -> fail fast
    except KeyboardInterrupt:
        log.info("Shutdown signal received (Ctrl+C).")
    except Exception as e:  # noqa: BLE001
        log.error(f"An unexpected error occurred during setup/runtime: {e}")
        rc = 1
    finally:
        signal.signal(signal.SIGTERM, signal.SIG_IGN)  # a second signal must not cut teardown
        signal.signal(signal.SIGINT, signal.SIG_IGN)
        log.info("Shutting down and cleaning up stages...")
        if server is not None:
            server.stop(grace=1.0)
        if job is not None:
            job.terminate()
        log.info("Shutdown complete.")
    return rc


if __name__ == "__main__":
    sys.exit(main())
