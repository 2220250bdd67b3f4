"""``run_grpc_inference.py`` -- batched inference client (reference-compatible).

Same CLI as /root/reference/src/run_grpc_inference.py:218-252 (positional ``input_index``,
``--inputs``, ``--port``, ``--timeout``, ``--batch-size``) and the same log lines
("Batch i/n completed in X seconds (k examples).", "Total inference time: X seconds",
"Correct predictions: A out of N", "Inference process completed."). Differences:
  * requests/responses are (de)serialised in C++ (no Python row lists), and the server has no
    4 MiB cap, so the default single batch of 60,000 examples works;
  * ``input_index`` mode reports "out of 1" instead of the whole file size (§2.7 #3);
  * additive: ``--local CONFIG`` runs the engine in-process (no server), ``--host``,
    ``--metrics-json`` (accuracy, weighted P/R/F1, latency percentiles like the notebook).
"""
from __future__ import annotations

import argparse
import json
import logging
import math
import os
import sys
import time
from typing import Optional

import numpy as np

SCRIPT_DIR_DEFAULT = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "src")
log = logging.getLogger("run_grpc_inference")


def build_parser(script_dir: str) -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Run inference on a distributed FCNN via gRPC.")
    ap.add_argument("input_index", type=int, nargs="?",
                    help="Index of the input example to use (default: all examples).")
    ap.add_argument("--inputs", type=str, default=os.path.join(
        script_dir, "../config/example_inputs/mnist_examples_60000.json"))
    ap.add_argument("--port", type=int, default=5101)
    ap.add_argument("--timeout", type=float, default=10.0)
    ap.add_argument("--batch-size", type=int, default=None)
    ap.add_argument("--host", type=str, default="127.0.0.1")
    ap.add_argument("--local", type=str, default=None,
                    help="model config JSON: run the MI355X engine in-process, no server")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--metrics-json", type=str, default=None)
    return ap


def main(argv: Optional[list[str]] = None, script_dir: str = SCRIPT_DIR_DEFAULT) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    a = build_parser(script_dir).parse_args(argv)
    from ..data import load_examples
    from ..metrics import LatencyStats, classification_report

    try:
        ex = load_examples(a.inputs)
    except FileNotFoundError:
        log.error(f"Inputs file not found: {a.inputs}")
        return 1
    except (json.JSONDecodeError, ValueError, RuntimeError) as e:
        log.error(f"Error parsing inputs file {a.inputs}: {e}")
        return 1
    if len(ex) == 0:
        log.warning(f"No 'examples' found in {a.inputs}.")
        log.error("No examples loaded, cannot run inference.")
        return 1
    x, labels = ex.x, ex.labels
    if a.input_index is not None:
        if not 0 <= a.input_index < len(ex):
            log.error(f"Input index {a.input_index} is out of range (0-{len(ex) - 1}).")
            return 1
        x, labels = x[a.input_index:a.input_index + 1], labels[a.input_index:a.input_index + 1]
    num_examples = len(x)

    if a.local:
        import torch

        from ..config import load_model_config
        from ..engine.inference import InferenceEngine

        mc = load_model_config(a.local)
        dev = torch.device("cpu") if a.device == "cpu" or not torch.cuda.is_available() \
            else torch.device("cuda", 0)
        eng = InferenceEngine([mc.layers], dev, expected_input=mc.layers[0].in_dim)

        def call(batch):
            return eng.predict(batch)
    else:
        import grpc

        from ..serve.ingress import LayerClient

        address = f"{a.host}:{a.port}"
        try:
            client = LayerClient(address, timeout=a.timeout, wait_ready=a.timeout / 2)
        except grpc.FutureTimeoutError:
            log.error(f"Timeout waiting for gRPC channel to {address} to become ready.")
            return 1

        def call(batch):
            return client.process(batch)

    def run_batch(batch):
        t0 = time.monotonic()
        try:
            out = call(batch)
            return out, time.monotonic() - t0
        except Exception as e:  # noqa: BLE001
            el = time.monotonic() - t0
            code = getattr(e, "code", None)
            details = getattr(e, "details", None)
            if callable(code):
                log.error(f"Batch gRPC call failed after {el:.4f}s: {code()} - {details()}")
            else:
                log.error(f"Unexpected batch error after {el:.4f}s: {e}")
            return None, el

    correct = 0
    preds = np.full(num_examples, -1, dtype=np.int64)
    lat = LatencyStats()
    total_start = time.monotonic()
    if a.batch_size is None or a.batch_size >= num_examples:
        out, el = run_batch(x)
        lat.add(el)
        if out is not None and out.size:
            preds[:] = out.argmax(1)
            correct = int((preds == labels).sum())
        log.info(f"Batch inference completed in {el:.4f} seconds for {num_examples} examples.")
    else:
        nb = math.ceil(num_examples / a.batch_size)
        for b in range(nb):
            s, e = b * a.batch_size, min((b + 1) * a.batch_size, num_examples)
            out, el = run_batch(x[s:e])
            lat.add(el)
            if out is not None and out.size:
                preds[s:e] = out.argmax(1)
                correct += int((preds[s:e] == labels[s:e]).sum())
            log.info(f"Batch {b + 1}/{nb} completed in {el:.4f} seconds ({e - s} examples).")
    total = time.monotonic() - total_start
    log.info(f"Total inference time: {total:.4f} seconds")
    log.info(f"Correct predictions: {correct} out of {num_examples}")
    if (labels >= 0).any():
        rep = classification_report(labels[labels >= 0], preds[labels >= 0])
        log.info(f"Accuracy: {rep['accuracy']:.4f}, Precision: {rep['precision']:.4f}, "
                 f"Recall: {rep['recall']:.4f}, F1 Score: {rep['f1_score']:.4f}")
    else:
        rep = {}
    summ = lat.summary()
    if summ:
        log.info(f"Batch latency p50 {summ['p50_s'] * 1e3:.3f} ms, p90 {summ['p90_s'] * 1e3:.3f} ms, "
                 f"p99 {summ['p99_s'] * 1e3:.3f} ms; {num_examples / max(total, 1e-12):.1f} samples/s")
    if a.metrics_json:
        with open(a.metrics_json, "w") as f:
            json.dump({**rep, "total_latency_sec": total,
                       "avg_latency_per_sample_sec": total / num_examples, "latency": summ,
                       "correct": correct, "num_examples": num_examples}, f)
    log.info("Inference process completed.")
    return 0


if __name__ == "__main__":
    sys.exit(main())
