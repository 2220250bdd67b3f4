"""Fused classifier tail (csrc/kernels/mlp_tail.hip) vs the four unfused kernels it replaces
(fwd L-2, fwd L-1 + softmax CE, dgrad L-1, dgrad L-2), isolated, HIP-event timed.
Usage: python bench/tail_ab.py [--rows 65536] [--k3 256 --n3 128 --n4 64 --classes 10]"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from stage_sweep import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--k3", type=int, default=256)
    ap.add_argument("--n3", type=int, default=128)
    ap.add_argument("--n4", type=int, default=64)
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda")
    R, k3, n3, n4, nc = a.rows, a.k3, a.n3, a.n4, a.classes
    g = torch.Generator(device=dev).manual_seed(0)
    bf, f32 = torch.bfloat16, torch.float32
    x = torch.relu(torch.randn(R, k3, device=dev, generator=g)).to(bf)
    w3 = (torch.randn(n3, k3, device=dev, generator=g) / k3 ** 0.5).to(bf)
    w4 = torch.zeros(n4, n3, device=dev, dtype=bf)
    w4[:nc] = (torch.randn(nc, n3, device=dev, generator=g) / n3 ** 0.5).to(bf)
    b3, b4 = torch.zeros(n3, device=dev), torch.zeros(n4, device=dev)
    lab = torch.randint(0, nc, (R,), device=dev, generator=g, dtype=torch.int32)
    h3, dz3 = (torch.empty(R, n3, device=dev, dtype=bf) for _ in range(2))
    dz4 = torch.empty(R, n4, device=dev, dtype=bf)
    dz2 = torch.empty(R, k3, device=dev, dtype=bf)
    nb = ops.tail_blocks(R)
    loss, corr = torch.zeros(nb, device=dev), torch.zeros(nb, device=dev, dtype=torch.int32)
    cs4, cs3, cs2 = (torch.zeros(nb, c, device=dev) for c in (n4, n3, k3))

    def fused():
        ops.mlp_tail(x, w3, b3, w4, b4, lab, h3, dz4, dz3, dz2, nc, 1.0 / R, loss_part=loss,
                     correct=corr, cs4=cs4, cs3=cs3, cs2=cs2)

    nx = R // ops.xent_tiles(R, n4)[0]
    lx, cx = torch.zeros(nx, device=dev), torch.zeros(nx, device=dev, dtype=torch.int32)
    c4 = torch.zeros(nx, n4, device=dev)
    c3 = torch.zeros(R // ops.dgrad_tiles(R, n3, n4)[0], n3, device=dev, dtype=f32)
    c2 = torch.zeros(R // ops.dgrad_tiles(R, k3, n3)[0], k3, device=dev, dtype=f32)

    def unfused():
        ops.linear_fwd(x, w3, b3, h3, act="relu")
        ops.linear_fwd_xent(h3, w4, b4, dz4, lab, nc, 1.0 / R, lx, cx, colsum=c4)
        ops.linear_dgrad(dz4, w4, dz3, y_prev=h3, act_prev="relu", colsum=c3)
        ops.linear_dgrad(dz3, w3, dz2, y_prev=x, act_prev="relu", colsum=c2)

    nbytes = 2 * R * (k3 + n3 + n4 + n3 + k3)
    for name, fn in (("unfused", unfused), ("fused", fused), ("unfused", unfused),
                     ("fused", fused)):
        us = timeit(fn, a.iters)
        print(json.dumps({"variant": name, "rows": R, "k3": k3, "n3": n3, "n4": n4,
                          "us": round(us, 2), "TBps": round(nbytes / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
