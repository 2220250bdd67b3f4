"""Serving engine on the GPU: HIP-graph row buckets vs the fp64 stage-worker oracle, mixed
activations (incl. a hidden row-softmax), batch-1 latency, and --train through the compat CLI."""
import os
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

from docker_dist_nn_amd.config import LayerWeights
from docker_dist_nn_amd.cpu_ref import model_forward
from docker_dist_nn_amd.engine.inference import InferenceEngine

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _layers(dims, acts, seed=0):
    rng = np.random.default_rng(seed)
    return [LayerWeights(rng.standard_normal((dims[i + 1], dims[i])) / np.sqrt(dims[i]),
                         rng.standard_normal(dims[i + 1]) * 0.1, acts[i]) for i in range(len(acts))]


@pytest.mark.parametrize("rows", [1, 3, 8, 63, 64, 500, 4096])
def test_engine_matches_fp64(dev, rows):
    L = _layers([784, 512, 256, 128, 10], ["relu", "sigmoid", "relu", "softmax"])
    eng = InferenceEngine([L[:2], L[2:]], dev, expected_input=784)
    x = np.random.default_rng(rows).random((rows, 784))
    out = eng.predict(x)
    np.testing.assert_allclose(out, model_forward(L, x), atol=1e-2)
    out2 = eng.predict(x)  # graph replay path
    np.testing.assert_array_equal(out, out2)


def test_hidden_softmax_and_linear_output(dev):
    L = _layers([100, 64, 32], ["softmax", "linear"])
    eng = InferenceEngine([L], dev, expected_input=100)
    for rows in (70, 2):  # MFMA path and the serving-size GEMV path
        x = np.random.default_rng(rows).random((rows, 100))
        np.testing.assert_allclose(eng.predict(x), model_forward(L, x), rtol=2e-2, atol=2e-2)


def test_batch1_latency_8_stage_chain(dev):
    L = _layers([784] + [1024] * 7 + [10], ["relu"] * 7 + ["softmax"])
    eng = InferenceEngine([[l] for l in L], dev, expected_input=784)
    x = np.random.default_rng(2).random((1, 784))
    for _ in range(20):
        eng.predict(x)
    ts = []
    for _ in range(200):
        t0 = time.perf_counter()
        eng.predict(x)
        ts.append(time.perf_counter() - t0)
    p50 = float(np.percentile(ts, 50)) * 1e3
    print(f"8-stage batch-1 p50 latency {p50:.3f} ms")
    assert p50 < 4.3  # reference chain p50 (3 stages): 4.3 ms


def test_compat_cli_trains_on_gpu(tmp_path):
    out = tmp_path / "trained.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "src", "run_grpc_fcnn.py"),
                        "--config", str(tmp_path / "none.json"), "--model", "784-128-64-10",
                        "--inputs", str(tmp_path / "none_inputs.json"), "--train",
                        "--synthetic", "8192", "--micro-batch", "1024", "--epochs", "3",
                        "--lr", "0.2", "--save", str(out), "--no-serve",
                        "--cache-dir", str(tmp_path / "c")],
                       capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stdout + r.stderr
    import json
    doc = json.load(open(out))
    assert doc["inference_metrics"]["accuracy"] > 0.3
    assert len(doc["model"]["layers"]) == 3
