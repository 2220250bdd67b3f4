"""Run ONE GEMM configuration repeatedly (for rocprofv3 --pmc counter collection).
Example: python bench/one_gemm.py --op fwd --M 65536 --K 832 --N 512 --tile 128x128 --stages 2"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ, MNMAJ  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="fwd", choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--M", type=int, default=65536, help="batch rows")
    ap.add_argument("--K", type=int, default=832, help="layer input width (padded)")
    ap.add_argument("--N", type=int, default=512, help="layer output width (padded)")
    ap.add_argument("--tile", default="128x128")
    ap.add_argument("--stages", type=int, default=2)
    ap.add_argument("--splits", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--group-m", type=int, default=0)
    a = ap.parse_args()
    bm, bn = map(int, a.tile.split("x"))
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    R, K, N = a.M, a.K, a.N
    x = torch.randn(R, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    dz = torch.randn(R, N, device=dev, generator=g).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    if a.op == "fwd":
        y = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
        fn = lambda: ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=R, N=N, K=K, bias=b,  # noqa: E731,E501
                              act="relu", tiles=(bm, bn), stages=a.stages, group_m=a.group_m)
    elif a.op == "dgrad":
        dx = torch.empty(R, K, device=dev, dtype=torch.bfloat16)
        fn = lambda: ops.gemm(dz, w, dx, layout_a=KMAJ, layout_b=MNMAJ, M=R, N=K, K=N, aux=x,  # noqa: E731,E501
                              act="relu", tiles=(bm, bn), stages=a.stages, group_m=a.group_m)
    else:
        slabs = torch.empty(a.splits, N, K, device=dev)
        fn = lambda: ops.gemm(dz, x, slabs, layout_a=MNMAJ, layout_b=MNMAJ, M=N, N=K, K=R,  # noqa: E731,E501
                              k_total=R, splits=a.splits, tiles=(bm, bn), stages=a.stages, group_m=a.group_m)
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
