"""Bulk inference throughput -- the reference's own measured quantity.

The reference times ``run_grpc_inference.py`` over its 60,000-example inference set
(/root/reference/src/run_grpc_inference.py:162-216; the set is the notebook's 10 % split tiled
x10, …ipynb:257-266) and reports "Total inference time". SURVEY §6 records ~5.7 k samples/s
through its 3-container CPU chain and ~13.2 k samples/s for centralised Keras.

Measured here, for each model (one stage per layer, as layer_distribution [1, 1, ...]):
  * device: the whole chain's forward on device-resident bf16 inputs (HIP graph per bucket),
    samples/s of the GPU alone;
  * predict: ``InferenceEngine.predict`` on 60,000 fp64 host examples (pinned staging, H2D,
    pack, forward, D2H) -- what an in-process client sees;
  * grpc: the same 60,000 examples through the reference-protocol gRPC ingress in batches of
    --grpc-batch rows (what the unmodified reference client sees; protobuf fp64 rows).
Random-init weights, synthetic MNIST-shaped inputs. One JSON line per measurement."""
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
from docker_dist_nn_amd.data import synthetic_mnist  # noqa: E402
from docker_dist_nn_amd.engine.inference import InferenceEngine  # noqa: E402

MODELS = {"notebook 784-32-16-10": [784, 32, 16, 10],
          "mnist-fcnn 784-512-256-128-10": [784, 512, 256, 128, 10],
          "mlp8 784-1024x7-10": [784] + [1024] * 7 + [10]}


def engine_for(dims, dev):
    rng = np.random.default_rng(0)
    layers = [LayerWeights(rng.standard_normal((dims[i + 1], dims[i])) / np.sqrt(dims[i]),
                           rng.standard_normal(dims[i + 1]) * 0.1,
                           "softmax" if i == len(dims) - 2 else "relu")
              for i in range(len(dims) - 1)]
    return InferenceEngine([[l] for l in layers], dev, expected_input=dims[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--examples", type=int, default=60000)
    ap.add_argument("--grpc-batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    x, _ = synthetic_mnist(a.examples, seed=1)
    x = x.astype(np.float64)
    for name, dims in MODELS.items():
        eng = engine_for(dims, dev)
        n = len(dims) - 1
        # device-resident forward over one 65536-row bucket
        R = 65536
        eng.predict(x[:R] if a.examples >= R else np.resize(x, (R, dims[0])))
        rows = eng._bucket(R)
        torch.cuda.synchronize()
        for _ in range(3):
            eng._forward_padded(rows)
        eng._stream.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 50
        with torch.cuda.stream(eng._stream):
            s.record()
            for _ in range(it):
                eng._forward_padded(rows)
            e.record()
        e.synchronize()
        ms = s.elapsed_time(e) / it
        print(json.dumps({"metric": "inference samples/s", "path": "device", "model": name,
                          "stages": n, "rows": R, "ms": round(ms, 4),
                          "samples_per_s": round(R / ms * 1e3, 1)}), flush=True)
        # host fp64 -> predict -> host, the whole 60k set
        eng.predict(x)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            eng.predict(x)
            ts.append(time.perf_counter() - t0)
        t = float(np.median(ts))
        print(json.dumps({"metric": "inference samples/s", "path": "predict", "model": name,
                          "stages": n, "examples": a.examples, "total_s": round(t, 5),
                          "samples_per_s": round(a.examples / t, 1)}), flush=True)
        # the reference client's path: gRPC ingress, fp64 protobuf rows, batched
        from docker_dist_nn_amd.launch import free_port
        from docker_dist_nn_amd.serve.ingress import LayerClient, serve

        port = free_port()
        server = serve(eng.predict, port=port)
        c = LayerClient(f"127.0.0.1:{port}", timeout=60, wait_ready=10)
        c.process(x[:a.grpc_batch])
        ts = []
        for _ in range(max(1, a.reps // 2)):
            t0 = time.perf_counter()
            for r0 in range(0, a.examples, a.grpc_batch):
                c.process(x[r0:r0 + a.grpc_batch])
            ts.append(time.perf_counter() - t0)
        t = float(np.median(ts))
        print(json.dumps({"metric": "inference samples/s", "path": "grpc", "model": name,
                          "stages": n, "examples": a.examples, "batch": a.grpc_batch,
                          "total_s": round(t, 4), "samples_per_s": round(a.examples / t, 1)}),
              flush=True)
        c.close()
        server.stop(0)


if __name__ == "__main__":
    main()
