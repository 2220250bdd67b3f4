"""GEMM micro-benchmark: our gfx950 MFMA kernels vs hipBLASLt (torch.matmul) on the shapes of
the benchmark models. Prints one JSON line per (shape, op). Random bf16 data (guide §5.4
rule 25: never time zero-filled operands)."""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402


def timeit(fn, iters=50, warmup=5):
    for _ in range(warmup):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def run(M, K, N, iters):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    dz = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    splits = ops.pick_splits(N, K, M)
    slabs = torch.empty(splits, N, K, device=dev)
    flop = 2.0 * M * N * K
    res = []
    cases = {
        "fwd": (lambda: ops.linear_fwd(x, w, b, y, "relu"),
                lambda: torch.relu(torch.addmm(b.to(torch.bfloat16), x, w.t()))),
        "dgrad": (lambda: ops.linear_dgrad(dz, w, dx, x, "relu"),
                  lambda: (dz @ w) * (x > 0)),
        "wgrad": (lambda: ops.linear_wgrad(dz, x, slabs, splits),
                  lambda: dz.t().float() @ x.float() if False else dz.t() @ x),
    }
    for name, (ours, theirs) in cases.items():
        t_ours = timeit(ours, iters)
        t_ref = timeit(theirs, iters)
        res.append({"shape": [M, K, N], "op": name, "ours_us": round(t_ours, 2),
                    "ours_tflops": round(flop / t_ours / 1e6, 1),
                    "hipblaslt_us": round(t_ref, 2),
                    "hipblaslt_tflops": round(flop / t_ref / 1e6, 1),
                    "splits": splits if name == "wgrad" else 1,
                    "tiles": list(ops.pick_tiles(*((N, K) if name == "wgrad" else
                                                   (M, N if name == "fwd" else K)), splits
                                                 if name == "wgrad" else 1))})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--shapes", default="65536x832x512,65536x512x256,65536x256x128,"
                    "65536x128x64,65536x1024x1024,16384x832x8192,16384x8192x8192,8192x8192x8192")
    a = ap.parse_args()
    for s in a.shapes.split(","):
        M, K, N = map(int, s.split("x"))
        for r in run(M, K, N, a.iters):
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
