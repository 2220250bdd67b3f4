"""Raster group (group_m: row tiles per group of the XCD-aware walk) of the wide model's
16384x8192x8192 GEMMs on the tuned stage code 11, interleaved reps. One JSON line per row.
Usage: python bench/probes/wide_raster.py"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ, MNMAJ  # noqa: E402


def timed(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    R = K = N = 8192
    R = 16384
    x = torch.randn(R, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    dz = torch.randn(R, N, device=dev, generator=g).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    y = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(R, K, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * R * K * N
    gms = (1, 2, 4, 8, 16, 32)
    for op in ("fwd", "dgrad"):
        fns = {}
        for gm in gms:
            if op == "fwd":
                fns[gm] = (lambda gm=gm: ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=R, N=N,
                                                  K=K, bias=b, act="relu", tiles=(256, 256),
                                                  stages=11, group_m=gm))
            else:
                fns[gm] = (lambda gm=gm: ops.gemm(dz, w, dx, layout_a=KMAJ, layout_b=MNMAJ, M=R,
                                                  N=K, K=N, aux=x, act="relu", tiles=(256, 256),
                                                  stages=11, group_m=gm))
        for f in fns.values():
            f()
        res = {gm: [] for gm in gms}
        for _ in range(4):
            for gm in gms:
                res[gm].append(timed(fns[gm]))
        for gm in gms:
            print(json.dumps({"op": op, "group_m": gm, "us": [round(t, 1) for t in res[gm]],
                              "best_tflops": round(fl / min(res[gm]) / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
