"""A/B of the persistent-workgroup GEMM (gemm_persist.hip) against the one-tile-per-workgroup
kernel (gemm.hip) on the GEMMs of the BASELINE models, isolated (HIP-event timed). Prints one
JSON line per (GEMM, tile, form). The step-level effect is measured by bench.py with
DNN_GEMM_PERSIST=0/1.

Usage: python bench/persist_ab.py [--iters 20] [--shapes headline|wide|all]"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ, MNMAJ  # noqa: E402
from stage_sweep import timeit  # noqa: E402

# (name, op, rows, in, out, tiles, wgrad splits)
HEADLINE = [
    ("fwd1", "fwd", 65536, 832, 512, [(256, 256), (128, 128), (256, 128)], 0),
    ("fwd2", "fwd", 65536, 512, 256, [(256, 64), (256, 128), (128, 128)], 0),
    ("fwd3", "fwd", 65536, 256, 128, [(64, 64), (128, 64), (256, 64), (128, 128)], 0),
    ("dgrad2", "dgrad", 65536, 512, 256, [(256, 64), (128, 128), (256, 128)], 0),
    ("dgrad3", "dgrad", 65536, 256, 128, [(256, 64), (128, 64)], 0),
    ("wgrad1", "wgrad", 65536, 832, 512, [(128, 128), (256, 128), (128, 256)], 6),
    ("wgrad2", "wgrad", 65536, 512, 256, [(128, 64), (128, 128)], 8),
]
WIDE = [
    ("wide_fwd", "fwd", 16384, 8192, 8192, [(256, 256), (128, 128)], 0),
    ("wide_dgrad", "dgrad", 16384, 8192, 8192, [(256, 256), (128, 128)], 0),
    ("wide_wgrad", "wgrad", 16384, 8192, 8192, [(256, 256), (128, 128)], 1),
    ("mlp8_fwd", "fwd", 65536, 1024, 1024, [(256, 256), (128, 128)], 0),
]


def run(name, op, R, K, N, tiles, splits, iters, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(R, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    dz = torch.randn(R, N, device=dev, generator=g).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    flops = 2.0 * R * K * N
    for tile in tiles:
        for persist in (0, -1, 1 << 30):  # classic / persistent / direct epilogue only
            if op == "fwd":
                y = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
                fn = lambda: ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=R, N=N, K=K,  # noqa
                                      bias=b, act="relu", tiles=tile, persist=persist)
            elif op == "dgrad":
                dx = torch.empty(R, K, device=dev, dtype=torch.bfloat16)
                cs = torch.empty(-(-R // tile[0]), K, device=dev)
                fn = lambda: ops.gemm(dz, w, dx, layout_a=KMAJ, layout_b=MNMAJ, M=R, N=K, K=N,  # noqa
                                      aux=x, act="relu", tiles=tile, colsum=cs, persist=persist)
            else:
                slabs = torch.empty(max(splits, 1), N, K, device=dev)
                fn = lambda: ops.gemm(dz, x, slabs, layout_a=MNMAJ, layout_b=MNMAJ, M=N, N=K,  # noqa
                                      K=R, k_total=R, splits=max(splits, 1), tiles=tile,
                                      persist=persist)
            try:
                us = timeit(fn, iters)
            except Exception as e:  # unsupported combination: record and go on
                print(json.dumps({"gemm": name, "tile": tile, "persist": persist,
                                  "error": str(e)[:120]}), flush=True)
                continue
            print(json.dumps({"gemm": name, "op": op, "M": R, "K": K, "N": N, "tile": tile,
                              "splits": splits, "persist": persist, "us": round(us, 2),
                              "tflops": round(flops / us / 1e6, 1)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default="all", choices=["headline", "wide", "all"])
    a = ap.parse_args()
    dev = torch.device("cuda")
    shapes = {"headline": HEADLINE, "wide": WIDE, "all": HEADLINE + WIDE}[a.shapes]
    for s in shapes:
        run(*s, a.iters, dev)


if __name__ == "__main__":
    main()
