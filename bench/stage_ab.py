"""A/B of GEMM LDS-ring forms on the benchmark models' shapes, interleaved rounds in ONE process
(guide §5.4 rule 24), random bf16 operands. Prints one JSON line per (case, variant) with the
median / min us over rounds, and checks every variant's output bitwise against the first.

Variants are (tile, stages): stages 2 = the 2-deep ring, 3 = 3-deep, 5 = asymmetric ring
(A 3 deep, B 2 deep: csrc/kernels/gemm_tile.hpp mma_tile_asym), 6 / 7 = register-prefetched
2- / 3-deep ring (mma_tile_rp), 9 / 10 = the same with the register-direct epilogue, 8 = ping-pong (256x256), 12-14 = 32-deep k-steps.

Usage: python bench/stage_ab.py [--rounds 7] [--cases f0,d1,w0,...]"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops.kernels import KMAJ, MNMAJ  # noqa: E402

DEV = torch.device("cuda")


def rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


def case_fwd(M, K, N, variants):
    x, w = rnd(M, K), rnd(N, K, scale=0.05)
    b = torch.randn(N, device=DEV)
    outs = {v: torch.empty(M, N, device=DEV, dtype=torch.bfloat16) for v in variants}

    def run(v):
        (bm, bn), st = v
        ops.gemm(x, w, outs[v], layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, bias=b, act="relu",
                 tiles=(bm, bn), stages=st)
    return run, outs, 2.0 * M * N * K


def case_dgrad(M, K, N, variants):
    """dX[M][N] = dZ[M][K] . W[K][N] read through the transposed shadow W^T [N][K] (KMAJ x
    KMAJ), ReLU derivative from the activation aux [M][N], bias-gradient column sums."""
    dz, wt, aux = rnd(M, K), rnd(N, K, scale=0.05), rnd(M, N)
    outs = {v: torch.empty(M, N, device=DEV, dtype=torch.bfloat16) for v in variants}
    cs = {v: torch.empty(-(-M // v[0][0]), N, device=DEV) for v in variants}

    def run(v):
        (bm, bn), st = v
        ops.gemm(dz, wt, outs[v], layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, aux=aux,
                 act="relu", tiles=(bm, bn), stages=st, colsum=cs[v])
    return run, outs, 2.0 * M * N * K


def case_wgrad(R, M, N, splits, variants):
    """dW[M][N] = dZ[R][M]^T . X[R][N] (MNMAJ x MNMAJ), fp32 split-K slabs."""
    dz, x = rnd(R, M), rnd(R, N)
    outs = {v: torch.empty(splits, M, N, device=DEV) for v in variants}

    def run(v):
        (bm, bn), st = v
        ops.gemm(dz, x, outs[v], layout_a=MNMAJ, layout_b=MNMAJ, M=M, N=N, K=0, k_total=R,
                 splits=splits, tiles=(bm, bn), stages=st)
    return run, outs, 2.0 * M * N * R


T256, T128, T12864 = (256, 256), (128, 128), (128, 64)
TS = [(T256, 9), ((256, 128), 9), ((256, 128), 11), (T128, 9), (T128, 11), (T12864, 9)]
BIG = [(T256, 2), (T256, 9), (T256, 11)]
WG = [(T128, 2), (T128, 9), (T128, 11)]
CASES = {
    "f0": lambda: case_fwd(65536, 832, 512, BIG),
    "f1": lambda: case_fwd(65536, 512, 256, BIG),
    "d1": lambda: case_dgrad(65536, 256, 512, BIG),
    "w0": lambda: case_wgrad(65536, 512, 832, 18, WG),
    "w1": lambda: case_wgrad(65536, 256, 512, 64, WG),
    "w2": lambda: case_wgrad(65536, 128, 256, 64, [((64, 64), 2), ((64, 64), 6), ((64, 64), 9),
                                                    (T12864, 6), (T12864, 9)]),
    "m8f": lambda: case_fwd(65536, 1024, 1024, BIG),
    "m8d": lambda: case_dgrad(65536, 1024, 1024, BIG),
    "m8w": lambda: case_wgrad(65536, 1024, 1024, 8, [(T128, 9), (T128, 11)]),
    "wide": lambda: case_fwd(16384, 8192, 8192, [(T256, 2), (T256, 9), (T256, 11)]),
    # tile sweep of the register-direct form on the headline's thin GEMMs
    "f0t": lambda: case_fwd(65536, 832, 512, TS),
    "f1t": lambda: case_fwd(65536, 512, 256, TS),
    "d1t": lambda: case_dgrad(65536, 256, 512, TS),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cases", default="f0,f1,d1,w0,w1,w2,m8f,m8d,m8w,wide")
    a = ap.parse_args()
    for name in a.cases.split(","):
        variants = None
        run, outs, flop = CASES[name]()
        variants = list(outs)
        times = {v: [] for v in variants}
        for v in variants:  # warm-up + correctness
            run(v)
        torch.cuda.synchronize()
        ref = outs[variants[0]]
        same = {v: bool(torch.equal(outs[v], ref)) for v in variants}
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(a.rounds):
            for v in variants:
                s.record()
                for _ in range(a.iters):
                    run(v)
                e.record()
                torch.cuda.synchronize()
                times[v].append(s.elapsed_time(e) / a.iters * 1e3)
        for v in variants:
            med = statistics.median(times[v])
            print(json.dumps({"case": name, "tile": list(v[0]), "stages": v[1],
                              "us_median": round(med, 2), "us_min": round(min(times[v]), 2),
                              "tflops": round(flop / med / 1e6, 1),
                              "bitwise_equal_first": same[v]}), flush=True)


if __name__ == "__main__":
    main()
