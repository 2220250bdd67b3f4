"""Stage code 13 (4-wave 256x256, 128x128 per wave) against code 11 (8-wave) on the 256x256
GEMMs of the BASELINE models: bitwise comparison of the outputs (same k order per element, so
they must match exactly) and interleaved timings. One JSON line per GEMM.
Usage: python bench/probes/rp4_ab.py [--reps 3] [--iters 20]"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ, MNMAJ  # noqa: E402

# (name, op, rows, K (layer input), N (layer output), splits)
SHAPES = [
    ("wide fwd", "fwd", 16384, 8192, 8192, 1),
    ("wide dgrad", "dgrad", 16384, 8192, 8192, 1),
    ("wide wgrad", "wgrad", 16384, 8192, 8192, 1),
    ("wide fwd0", "fwd", 16384, 832, 8192, 1),
    ("mlp8 fwd", "fwd", 65536, 1024, 1024, 1),
    ("mlp8 dgrad", "dgrad", 65536, 1024, 1024, 1),
    ("mlp8 wgrad", "wgrad", 65536, 1024, 1024, 8),
    ("head fwd0", "fwd", 65536, 832, 512, 1),
]


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for name, op, R, K, N, splits in SHAPES:
        if a.only and a.only not in name:
            continue
        x = torch.randn(R, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
        dz = torch.randn(R, N, device=dev, generator=g).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        outs = {}

        def make(stages):
            if op == "fwd":
                y = torch.zeros(R, N, device=dev, dtype=torch.bfloat16)
                outs[stages] = y
                return lambda: ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=R, N=N, K=K,
                                        bias=b, act="relu", tiles=(256, 256), stages=stages)
            if op == "dgrad":
                dx = torch.zeros(R, K, device=dev, dtype=torch.bfloat16)
                outs[stages] = dx
                return lambda: ops.gemm(dz, w, dx, layout_a=KMAJ, layout_b=MNMAJ, M=R, N=K, K=N,
                                        aux=x, act="relu", tiles=(256, 256), stages=stages)
            sl = torch.zeros(splits, N, K, device=dev)
            outs[stages] = sl
            return lambda: ops.gemm(dz, x, sl, layout_a=MNMAJ, layout_b=MNMAJ, M=N, N=K, K=R,
                                    k_total=R, splits=splits, tiles=(256, 256), stages=stages)

        f11, f13 = make(11), make(13)
        f11()
        f13()
        torch.cuda.synchronize()
        same = bool(torch.equal(outs[11], outs[13]))
        maxdiff = float((outs[11].float() - outs[13].float()).abs().max())
        t11, t13 = [], []
        for _ in range(a.reps):
            t11.append(timed(f11, a.iters))
            t13.append(timed(f13, a.iters))
        fl = 2.0 * R * K * N
        print(json.dumps({"gemm": name, "bitwise_equal": same, "max_abs_diff": maxdiff,
                          "code11_us": [round(t, 1) for t in t11],
                          "code13_us": [round(t, 1) for t in t13],
                          "code11_tflops": round(fl / min(t11) / 1e6, 1),
                          "code13_tflops": round(fl / min(t13) / 1e6, 1)}), flush=True)
        del outs, x, w, dz
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
