"""Operand-layout A/B for the three GEMMs of a Linear layer, interleaved in one process
(guide §5.4 rule 24): what does a transposed copy of an operand buy?

  fwd    Y[M][N]  = X[M][K] . W[N][K]^T          KMAJ x KMAJ (always)
  dgrad  dX[M][K] = dZ[M][N] . W[N][K]           KMAJ x MNMAJ (W as stored)
                                                 KMAJ x KMAJ  (a transposed copy W^T[K][N])
  wgrad  dW[N][K] = dZ[M][N]^T . X[M][K]         MNMAJ x MNMAJ (as stored)
                                                 KMAJ x KMAJ  (transposed dZ^T, X^T)

Random bf16 data (rule 25). Prints one JSON line per (shape, variant) with the median and min
over rounds, plus hipBLASLt (torch) for the same product as a yardstick.
Example: python bench/layout_ab.py --shapes 16384x8192x8192,65536x1024x1024"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ, MNMAJ  # noqa: E402


def timer(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="16384x8192x8192,65536x1024x1024,65536x832x512")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--splits", type=int, default=0, help="wgrad split-K (0 = model)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    for shp in a.shapes.split(","):
        M, K, N = map(int, shp.split("x"))
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
        dz = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
        wt, xt, dzt = w.t().contiguous(), x.t().contiguous(), dz.t().contiguous()
        b = torch.randn(N, device=dev)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        bm_w, bn_w, sp = ops.wgrad_config(N, K, M)
        sp = a.splits or sp
        slabs = torch.empty(sp, N, K, device=dev)
        t_fwd = ops.pick_tiles(M, N)
        t_dg = ops.pick_tiles(M, K)
        v = {}
        for st in (2, 8):
            if t_fwd == (256, 256) or st == 2:
                v[f"fwd_s{st}"] = lambda st=st: ops.gemm(
                    x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, bias=b, act="relu",
                    tiles=t_fwd if st == 2 else (256, 256), stages=st)
            v[f"dgrad_mn_s{st}"] = lambda st=st: ops.gemm(
                dz, w, dx, layout_a=KMAJ, layout_b=MNMAJ, M=M, N=K, K=N, aux=x, act="relu",
                tiles=t_dg if st == 2 else (256, 256), stages=st)
            v[f"dgrad_kt_s{st}"] = lambda st=st: ops.gemm(
                dz, wt, dx, layout_a=KMAJ, layout_b=KMAJ, M=M, N=K, K=N, aux=x, act="relu",
                tiles=t_dg if st == 2 else (256, 256), stages=st)
        for tl in ((256, 256), (256, 128)):
            tn = f"{tl[0]}x{tl[1]}"
            v[f"fwd_p{tn}"] = lambda tl=tl: ops.gemm(
                x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, bias=b, act="relu",
                tiles=tl, stages=2, persist=-1)
            v[f"dgrad_kt_p{tn}"] = lambda tl=tl: ops.gemm(
                dz, wt, dx, layout_a=KMAJ, layout_b=KMAJ, M=M, N=K, K=N, aux=x, act="relu",
                tiles=tl, stages=2, persist=-1)
        v["wgrad_mnmn"] = lambda: ops.gemm(dz, x, slabs, layout_a=MNMAJ, layout_b=MNMAJ, M=N, N=K,
                                           K=M, k_total=M, splits=sp, tiles=(bm_w, bn_w))
        v["wgrad_kk"] = lambda: ops.gemm(dzt, xt, slabs, layout_a=KMAJ, layout_b=KMAJ, M=N, N=K,
                                         K=M, k_total=M, splits=sp, tiles=(bm_w, bn_w))
        v["wgrad_kmn"] = lambda: ops.gemm(dzt, x, slabs, layout_a=KMAJ, layout_b=MNMAJ, M=N, N=K,
                                          K=M, k_total=M, splits=sp, tiles=(bm_w, bn_w))
        v["blas_fwd"] = lambda: torch.mm(x, wt, out=y)
        v["blas_dgrad"] = lambda: torch.mm(dz, w, out=dx)
        gw = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        v["blas_wgrad"] = lambda: torch.mm(dzt, x, out=gw)
        for fn in v.values():
            fn()
        torch.cuda.synchronize()
        res = {k: [] for k in v}
        for _ in range(a.rounds):
            for k, fn in v.items():
                res[k].append(timer(fn, a.iters))
        flop = 2.0 * M * N * K
        for k, ts in res.items():
            ts.sort()
            med = ts[len(ts) // 2]
            print(json.dumps({"shape": [M, K, N], "variant": k, "median_us": round(med, 2),
                              "min_us": round(ts[0], 2),
                              "tflops": round(flop / med / 1e6, 1),
                              "wgrad_cfg": [bm_w, bn_w, sp] if k.startswith("wgrad") else None}),
                  flush=True)


if __name__ == "__main__":
    main()
