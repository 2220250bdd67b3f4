"""Time GEMM epilogue variants of the wide / mlp8 steps in isolation (HIP events, interleaved):
the forward 784->8192 and the logits dgrad 10->8192 with and without the transposed second
output (``ct``, K-major weight gradients), and the 1024x1024 forward/dgrad in both forms.

    python bench/ct_ab.py [--iters 20]   -> one JSON line per case (median us)
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ  # noqa: E402


def timed(fn, iters):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(iters)]
    for _ in range(3):
        fn()
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    t = sorted(s.elapsed_time(e) * 1e3 for s, e in ev)
    return t[len(t) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*s, scale=1.0):
        return (torch.randn(*s, device=dev, generator=g) * scale).to(torch.bfloat16)

    cases = {}
    # wide forward 784 -> 8192 (K padded 832), 16384 rows: y (+ y^T)
    R, K, N = 16384, 832, 8192
    x, w, b = rnd(R, K), rnd(N, K, scale=0.05), torch.randn(N, device=dev)
    y = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
    yt = torch.empty(N, R, device=dev, dtype=torch.bfloat16)
    for name, ct in (("fwd832x8192", None), ("fwd832x8192+ct", yt)):
        cases[name] = lambda ct=ct: ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=R, N=N, K=K,
                                             bias=b, act="relu", tiles=(256, 256), ct=ct)
    # wide logits dgrad 10 (64 padded) -> 8192 with the relu' of the stored activation
    dz, wt2, aux = rnd(R, 64), rnd(8192, 64, scale=0.05), rnd(R, N)
    dx = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
    for name, ct in (("dgrad64x8192", None), ("dgrad64x8192+ct", yt)):
        cases[name] = lambda ct=ct: ops.gemm(dz, wt2, dx, layout_a=KMAJ, layout_b=KMAJ, M=R,
                                             N=N, K=64, aux=aux, act="relu", tiles=(128, 64),
                                             ct=ct)
    # mlp8 1024 x 1024 at 65536 rows: forward and dgrad (W^T operand), both forms
    R2 = 65536
    x2, w2, b2, a2 = rnd(R2, 1024), rnd(1024, 1024, scale=0.03), torch.randn(1024, device=dev), \
        rnd(R2, 1024)
    y2 = torch.empty(R2, 1024, device=dev, dtype=torch.bfloat16)
    for pers in (0, -1):
        cases[f"fwd1024_p{pers}"] = lambda pers=pers: ops.gemm(
            x2, w2, y2, layout_a=KMAJ, layout_b=KMAJ, M=R2, N=1024, K=1024, bias=b2, act="relu",
            tiles=(256, 256), persist=pers)
        cases[f"dgrad1024_p{pers}"] = lambda pers=pers: ops.gemm(
            x2, w2, y2, layout_a=KMAJ, layout_b=KMAJ, M=R2, N=1024, K=1024, aux=a2, act="relu",
            tiles=(256, 256), persist=pers)
    res = {k: [] for k in cases}
    for _ in range(3):  # interleaved rounds
        for k, fn in cases.items():
            res[k].append(timed(fn, a.iters))
    for k, v in res.items():
        print(json.dumps({"case": k, "us": round(sorted(v)[1], 2), "all": [round(t, 2) for t in v]}))


if __name__ == "__main__":
    main()
