"""BASELINE config 5: inference-chain batch=1 latency (p50/p90/p99), 8 stages.

Two measurements on one MI355X:
  * engine: ``InferenceEngine.predict`` on an 8-stage 784-1024x7-10 chain (stages in-process,
    whole forward replayed as one HIP graph per row bucket) -- host->device->host included;
  * grpc: the same engine behind the reference-protocol gRPC ingress, timed from a client on
    127.0.0.1 (what run_grpc_inference.py sees; the reference measured p50 4.3 ms for 3 CPU
    stages).
Prints one JSON line per measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from docker_dist_nn_amd.config import LayerWeights  # noqa: E402
from docker_dist_nn_amd.engine.inference import InferenceEngine  # noqa: E402


def pct(ts):
    a = np.asarray(ts) * 1e3
    return {"p50_ms": round(float(np.percentile(a, 50)), 4),
            "p90_ms": round(float(np.percentile(a, 90)), 4),
            "p99_ms": round(float(np.percentile(a, 99)), 4), "n": len(ts)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=500)
    ap.add_argument("--widths", default="784," + ",".join(["1024"] * 7) + ",10")
    ap.add_argument("--rows", type=int, default=1)
    a = ap.parse_args()
    dims = [int(x) for x in a.widths.split(",")]
    rng = np.random.default_rng(0)
    layers = [LayerWeights(rng.standard_normal((dims[i + 1], dims[i])) / np.sqrt(dims[i]),
                           rng.standard_normal(dims[i + 1]) * 0.1,
                           "softmax" if i == len(dims) - 2 else "relu")
              for i in range(len(dims) - 1)]
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    eng = InferenceEngine([[l] for l in layers], dev, expected_input=dims[0])
    x = rng.random((a.rows, dims[0]))
    for _ in range(50):
        eng.predict(x)
    ts = []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        eng.predict(x)
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"metric": "inference chain latency", "path": "engine", "stages": len(layers),
                      "rows": a.rows, "model": "-".join(map(str, dims)), **pct(ts)}), flush=True)

    from docker_dist_nn_amd.launch import free_port
    from docker_dist_nn_amd.serve.ingress import LayerClient, serve

    port = free_port()
    server = serve(eng.predict, port=port)
    c = LayerClient(f"127.0.0.1:{port}", timeout=10, wait_ready=10)
    for _ in range(50):
        c.process(x)
    ts = []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        c.process(x)
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"metric": "inference chain latency", "path": "grpc", "stages": len(layers),
                      "rows": a.rows, "model": "-".join(map(str, dims)), **pct(ts)}), flush=True)
    c.close()
    server.stop(0)


if __name__ == "__main__":
    main()
