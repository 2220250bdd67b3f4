"""Pipeline-depth x tile sweep of the GEMMs of one MNIST-FCNN training step (and of the wider
benchmark models): time of every (op, shape) under NS = 2/3/4 LDS stages and each legal tile.
Prints one JSON line per measurement; used to set ops.kernels.STAGES / the tile policy.
Random bf16 operands (never time zero-filled data)."""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ, MNMAJ  # noqa: E402

TILES = [(128, 128), (128, 64), (64, 128), (64, 64), (256, 256), (256, 128), (128, 256),
         (256, 64)]


def timeit(fn, iters, warmup=5):
    for _ in range(warmup):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def layers(model: str):
    dims = [int(d) for d in model.split("-")]
    pad = [((d + 63) // 64) * 64 for d in dims]
    return list(zip(pad[:-1], pad[1:]))  # (Kp, Np) per layer


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--model", default="784-512-256-128-10")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--stages", default="2", help="pipeline depths of 4-wave tiles, e.g. 234")
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    R = a.rows
    rnd = lambda *s: torch.randn(*s, device=dev, generator=g).to(torch.bfloat16)  # noqa: E731
    for li, (K, N) in enumerate(layers(a.model)):
        x, w, dz = rnd(R, K), rnd(N, K) * 0.05, rnd(R, N)
        y = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(R, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(N, device=dev)
        flop = 2.0 * R * N * K
        for op in a.ops.split(","):
            if op == "dgrad" and li == 0:
                continue  # the first layer's input gradient is never computed
            for (bm, bn) in TILES:
                cands = [1]
                if op == "wgrad" and N % bm == 0 and K % bn == 0:
                    t = (N // bm) * (K // bn)
                    cands = sorted({max(1, min(R // 64, round(k * 256 / t)))
                                    for k in (1, 2, 3, 4, 6)})
                depths = (2,) if max(bm, bn) == 256 else tuple(int(d) for d in a.stages)
                for ns, splits in [(ns, sp) for ns in depths for sp in cands]:
                    if op == "fwd":
                        if R % bm or N % bn:
                            continue
                        fn = lambda: ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=R, N=N,  # noqa: E731,E501
                                              K=K, bias=b, act="relu", tiles=(bm, bn), stages=ns)
                    elif op == "dgrad":
                        if R % bm or K % bn:
                            continue
                        fn = lambda: ops.gemm(dz, w, dx, layout_a=KMAJ, layout_b=MNMAJ, M=R,  # noqa: E731,E501
                                              N=K, K=N, aux=x, act="relu", tiles=(bm, bn),
                                              stages=ns)
                    else:
                        if N % bm or K % bn:
                            continue
                        slabs = torch.empty(splits, N, K, device=dev)
                        fn = lambda: ops.gemm(dz, x, slabs, layout_a=MNMAJ, layout_b=MNMAJ,  # noqa: E731,E501
                                              M=N, N=K, K=R, k_total=R, splits=splits,
                                              tiles=(bm, bn), stages=ns)
                    us = timeit(fn, a.iters)
                    print(json.dumps({"layer": li, "op": op, "M": R, "K": K, "N": N,
                                      "tile": [bm, bn], "stages": ns, "splits": splits,
                                      "us": round(us, 2), "tflops": round(flop / us / 1e6, 1)}),
                          flush=True)


if __name__ == "__main__":
    main()
