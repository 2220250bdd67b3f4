"""BASELINE config 5 through the RANK chain: batch=1 latency (p50/p90/p99) of an 8-stage
784-1024x7-10 inference chain brought up by run_grpc_fcnn.py --mode ranks (one process per
stage, serve/chain.py) and queried by the reference-protocol client on 127.0.0.1 -- the path
the reference measured (p50 4.3 ms over 3 CPU stages).

With fewer GPUs than stages (the one-GPU pool) every stage runs on cuda:0 and the hops go
through host memory over gloo (``rehearsal``: DNN_FORCE_DEVICE=0, DNN_DIST_BACKEND=gloo); on an
8-GPU node each stage has its own GPU and the hops are RCCL. One JSON line.

Usage: python bench/chain_latency.py [--iters 500] [--rows 1] [--stages 8]"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=500)
    ap.add_argument("--rows", type=int, default=1)
    ap.add_argument("--stages", type=int, default=8)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--log", default=None, help="write the servers' log here")
    a = ap.parse_args()
    import torch

    from docker_dist_nn_amd.data import write_examples
    from docker_dist_nn_amd.launch import free_port
    from docker_dist_nn_amd.serve.ingress import LayerClient
    from docker_dist_nn_amd.weights_io import export_model_json

    dims = [784] + [a.width] * (a.stages - 1) + [10]
    rng = np.random.default_rng(0)
    ws = [rng.standard_normal((dims[i + 1], dims[i])) / np.sqrt(dims[i]) for i in range(a.stages)]
    bs = [rng.standard_normal(dims[i + 1]) * 0.1 for i in range(a.stages)]
    n_gpu = torch.cuda.device_count() if torch.cuda.is_available() else 0
    rehearsal = n_gpu < a.stages
    env = dict(os.environ, PYTHONPATH=ROOT)
    if rehearsal:
        # every stage on cuda:0: 8 processes x the default 4 hardware queues each oversubscribe
        # the GPU's queue slots, and the scheduler's queue rotation put ~13 ms outliers into
        # the p99 (profiles/r4_chain: 13.7 ms at 4 queues, 0.75 ms at 2); one real GPU per
        # stage has no such sharing
        env.update(DNN_FORCE_DEVICE="0", DNN_DIST_BACKEND="gloo",
                   GPU_MAX_HW_QUEUES=os.environ.get("DNN_REHEARSAL_HW_QUEUES", "2"))
    with tempfile.TemporaryDirectory() as d:
        cfg = os.path.join(d, "model.json")
        export_model_json(cfg, ws, bs, ["relu"] * (a.stages - 1) + ["softmax"],
                          layer_distribution=[1] * a.stages)
        x = rng.random((64, 784))
        inp = os.path.join(d, "inputs.json")
        write_examples(inp, x, np.zeros(64, dtype=np.int64))
        port = free_port()
        p = subprocess.Popen([sys.executable, os.path.join(ROOT, "src", "run_grpc_fcnn.py"),
                              "--config", cfg, "--inputs", inp, "--port", str(port),
                              "--mode", "ranks", "--device", "cuda" if n_gpu else "cpu",
                              "--cache-dir", os.path.join(d, "cache"), "--run-for", "600"],
                             env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        ok = True
        try:
            c = LayerClient(f"127.0.0.1:{port}", timeout=30, wait_ready=180)
            q = x[:a.rows]
            print("servers ready", file=sys.stderr, flush=True)
            for _ in range(50):
                c.process(q)
            print("warm-up done", file=sys.stderr, flush=True)
            ts = []
            for i in range(a.iters):
                t0 = time.perf_counter()
                c.process(q)
                ts.append(time.perf_counter() - t0)
                if (i + 1) % 100 == 0:  # progress (a long run must not look hung)
                    print(f"{i + 1} requests, p50 so far {np.median(ts) * 1e3:.3f} ms",
                          file=sys.stderr, flush=True)
            c.close()
        except Exception:
            ok = False
            raise
        finally:
            p.terminate()
            try:
                log, _ = p.communicate(timeout=60)
            except subprocess.TimeoutExpired:
                p.kill()
                log, _ = p.communicate()
            if a.log:
                with open(a.log, "w") as f:
                    f.write(log or "")
            if not ok:
                print((log or "")[-6000:], file=sys.stderr, flush=True)
    fast = "device-side chain" in (log or "")
    import re
    m = re.search(r"predict latency over (\d+) requests: p50 ([\d.]+) ms p90 ([\d.]+) ms "
                  r"p99 ([\d.]+) ms", log or "")
    inner = ({"requests": int(m.group(1)), "p50_ms": float(m.group(2)),
              "p90_ms": float(m.group(3)), "p99_ms": float(m.group(4))} if m else None)
    t = np.asarray(ts) * 1e3
    print(json.dumps({"metric": "inference chain latency", "path": "rank chain (grpc ingress)",
                      "stages": a.stages, "rows": a.rows, "model": "-".join(map(str, dims)),
                      "transport": ("device-side chain: IPC slots + flags (serve/fastpath.py)"
                                    if fast else "gloo via host" if rehearsal else "rccl") +
                                   (", one-GPU rehearsal: every stage on cuda:0"
                                    if rehearsal else ""),
                      "gpu_max_hw_queues": env.get("GPU_MAX_HW_QUEUES"),
                      "persistent_stages": env.get("DNN_CHAIN_PERSIST", "1") == "1",
                      # rank 0's predict() alone (request in -> logits out, no gRPC): the
                      # device-side chain's own latency, warm-up requests included
                      "chain_only": inner,
                      "p50_ms": round(float(np.percentile(t, 50)), 4),
                      "p90_ms": round(float(np.percentile(t, 90)), 4),
                      "p99_ms": round(float(np.percentile(t, 99)), 4), "n": len(ts),
                      "reference_p50_ms": 4.3}), flush=True)


if __name__ == "__main__":
    main()
