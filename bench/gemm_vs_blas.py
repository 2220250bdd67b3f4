"""Each GEMM of a BASELINE model's training step against hipBLASLt and the HBM floor.

For every fwd / dgrad / wgrad of the step (tuned tile, fused epilogue, via ops.linear_*), this
prints our time next to:
  * ``blas_us``: torch.mm (hipBLASLt) of the same product, bf16 in and out, no epilogue: what
    the library takes for the bare product (our wgrad writes fp32 split-K slabs instead);
  * ``hbm_us``: the bytes the fused op must move at least once (operands + aux + output) over
    the measured device-to-device copy bandwidth -- the memory floor.
One JSON line per GEMM. Usage: python bench/gemm_vs_blas.py [--model 784-512-256-128-10]"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import kernels as K_  # noqa: E402
from stage_sweep import layers, timeit  # noqa: E402


def copy_bw(dev, nbytes=1 << 30):
    a = torch.empty(nbytes // 2, dtype=torch.bfloat16, device=dev)
    b = torch.empty_like(a)
    us = timeit(lambda: b.copy_(a), 10)
    return 2 * nbytes / us / 1e6  # TB/s (read + write)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="784-512-256-128-10")
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    R = a.rows
    bw = copy_bw(dev)
    print(json.dumps({"copy_TBps": round(bw, 3)}), flush=True)
    g = torch.Generator(device=dev).manual_seed(0)
    L = layers(a.model)
    for i, (Kp, Np) in enumerate(L):
        last = i == len(L) - 1
        x = torch.randn(R, Kp, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(Np, Kp, device=dev, generator=g) * 0.05).to(torch.bfloat16)
        dz = torch.randn(R, Np, device=dev, generator=g).to(torch.bfloat16)
        b = torch.randn(Np, device=dev)
        fl = 2.0 * R * Kp * Np
        rows = []
        if not last:  # the last layer runs the fused linear+CE tile (fixed geometry)
            y = torch.empty(R, Np, device=dev, dtype=torch.bfloat16)
            ours = timeit(lambda: K_.linear_fwd(x, w, b, y, act="relu"), a.iters)
            blas = timeit(lambda: torch.mm(x, w.t(), out=y), a.iters)
            rows.append(("fwd", ours, blas, 2 * (R * Kp + Np * Kp + R * Np)))
        if i > 0:
            dx = torch.empty(R, Kp, device=dev, dtype=torch.bfloat16)
            bm = K_.dgrad_tiles(R, Kp, Np)[0]
            cs = torch.empty(-(-R // bm), Kp, device=dev)
            ours = timeit(lambda: K_.linear_dgrad(dz, w, dx, y_prev=x, act_prev="relu",
                                                  colsum=cs), a.iters)
            blas = timeit(lambda: torch.mm(dz, w, out=dx), a.iters)
            rows.append(("dgrad", ours, blas, 2 * (R * Np + Np * Kp + 2 * R * Kp)))
        bm, bn, s = K_.wgrad_config(Np, Kp, R)
        slabs = torch.empty(s, Np, Kp, device=dev)
        ours = timeit(lambda: K_.linear_wgrad(dz, x, slabs, splits=s), a.iters)
        blas = timeit(lambda: torch.mm(dz.t(), x), a.iters)
        rows.append(("wgrad", ours, blas, 2 * (R * Np + R * Kp) + 4 * s * Np * Kp))
        for op, ours, blas, nbytes in rows:
            print(json.dumps({"layer": i, "op": op, "shape": [R, Kp, Np], "ours_us": round(ours, 2),
                              "blas_us": round(blas, 2), "hbm_us": round(nbytes / bw / 1e6, 2),
                              "ours_tflops": round(fl / ours / 1e6, 1),
                              "blas_tflops": round(fl / blas / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
