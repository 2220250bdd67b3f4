"""Where a dgrad's time goes beyond its product: the same K-major x K-major GEMM (W^T shadow,
tuned 256x256 code 11) with each epilogue piece on and off -- bare bf16 store, + the ReLU
derivative (1-bit fragment mask, or the stored activation), + the bias-gradient column sums
-- against the forward of the same shape (bias + ReLU). Interleaved reps, one JSON line each.
Usage: python bench/probes/dgrad_epi.py"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ  # noqa: E402
from docker_dist_nn_amd.ops.kernels import FragMask  # noqa: E402


def timed(fn, iters=20):
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
    for (R, K, N, tile, code) in ((65536, 1024, 1024, (256, 256), 11),
                                  (65536, 512, 256, (256, 256), 9)):
        # dgrad: dx[R][K] = dz[R][N] . W[N][K], read through W^T [K][N] (K-major)
        dz = torch.randn(R, N, device=dev, generator=g).to(torch.bfloat16)
        wt = (torch.randn(K, N, device=dev, generator=g) * 0.05).to(torch.bfloat16)
        y = torch.relu(torch.randn(R, K, device=dev, generator=g)).to(torch.bfloat16)
        dx = torch.empty(R, K, device=dev, dtype=torch.bfloat16)
        cs = torch.empty(R // tile[0], K, device=dev)
        fm = FragMask.alloc(R, K, tile, dev)
        xin = torch.randn(R, N, device=dev, generator=g).to(torch.bfloat16)
        b = torch.randn(K, device=dev)
        kw = dict(layout_a=KMAJ, layout_b=KMAJ, M=R, N=K, K=N, tiles=tile, stages=code)
        # the forward of the same GEMM shape writes the fragment mask the dgrad reads
        ops.gemm(xin, wt, dx, bias=b, act="relu", mask_out=fm, **kw)
        cases = {
            "fwd bias+relu": lambda: ops.gemm(xin, wt, dx, bias=b, act="relu", **kw),
            "bare": lambda: ops.gemm(dz, wt, dx, **kw),
            "mask": lambda: ops.gemm(dz, wt, dx, act="relu", mask_in=fm, **kw),
            "aux": lambda: ops.gemm(dz, wt, dx, aux=y, act="relu", **kw),
            "colsum": lambda: ops.gemm(dz, wt, dx, colsum=cs, **kw),
            "mask+colsum": lambda: ops.gemm(dz, wt, dx, act="relu", mask_in=fm, colsum=cs, **kw),
            "aux+colsum": lambda: ops.gemm(dz, wt, dx, aux=y, act="relu", colsum=cs, **kw),
        }
        for f in cases.values():
            f()
        res = {k: [] for k in cases}
        for _ in range(4):
            for k, f in cases.items():
                res[k].append(timed(f))
        for k, v in res.items():
            print(json.dumps({"shape": [R, K, N], "tile": tile, "code": code, "case": k,
                              "us": [round(t, 1) for t in v], "best": round(min(v), 1)}),
                  flush=True)
        del dz, wt, y, dx, cs, fm, xin
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
