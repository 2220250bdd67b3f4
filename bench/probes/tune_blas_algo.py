"""In-step choice of the hipBLASLt algorithm for every GEMM the tuned table routes to the
library: the heuristic's candidates 0..N-1 are each timed inside the real training step
(bench/tune.py step_ms) and the fastest is stored as ``blas_algo`` (kept at 0 unless another
wins by > 0.5 %). Deterministic at run time: the table names the algorithm.

Usage: python bench/tune_blas_algo.py --configs 65536:mnist-fcnn,16384:wide [--algos 8]"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from docker_dist_nn_amd import MLPSpec, NAMED_MODELS  # noqa: E402
from docker_dist_nn_amd.data import synthetic_mnist  # noqa: E402
from docker_dist_nn_amd.ops import tuning  # noqa: E402
from tune import signatures, step_ms  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="65536:mnist-fcnn,65536:mlp8,16384:wide")
    ap.add_argument("--algos", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=tuning.TABLE_PATH)
    a = ap.parse_args()
    os.environ.pop("DNN_BLAS", None)
    dev = torch.device("cuda")
    with open(a.out if os.path.exists(a.out) else tuning.TABLE_PATH) as f:
        doc = json.load(f)
    table = tuning._load()
    table.clear()
    table.update(doc["entries"])
    for cfg in a.configs.split(","):
        rows, model = cfg.split(":")
        R = int(rows)
        spec = NAMED_MODELS.get(model) or MLPSpec.parse(model)
        kp0 = (spec.layers[0].in_dim + 63) // 64 * 64
        xs, ys = synthetic_mnist(min(R, 65536), seed=3)
        reps_rows = -(-R // len(xs))
        x = torch.zeros(R, kp0, dtype=torch.bfloat16)
        x[:, :xs.shape[1]] = torch.from_numpy(xs).to(torch.bfloat16).repeat(reps_rows, 1)[:R]
        y = torch.from_numpy(ys).repeat(reps_rows)[:R].to(torch.int32)
        x, y = x.to(dev), y.to(dev)
        for (op, M, N, K, _) in signatures(spec, R):
            k = tuning.key(op, M, N, K)
            e = table.get(k)
            if not e or not e.get("blas"):
                continue
            res = []
            for alg in range(a.algos):
                e["blas_algo"] = alg
                try:
                    res.append((step_ms(spec, R, x, y, dev, a.steps, a.reps), alg))
                except (ValueError, RuntimeError) as err:
                    print(json.dumps({"sig": k, "algo": alg, "err": str(err)[:80]}), flush=True)
            base = [r for r in res if r[1] == 0]
            best = min(res)
            if base and best[0] < base[0][0] * 0.995:
                e["blas_algo"] = best[1]
            else:
                e.pop("blas_algo", None)
            print(json.dumps({"sig": k, "times": [[alg, round(t, 4)] for t, alg in res],
                              "chosen": e.get("blas_algo", 0)}), flush=True)
        doc["entries"] = dict(table)
        doc["date"] = time.strftime("%Y-%m-%d")
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
