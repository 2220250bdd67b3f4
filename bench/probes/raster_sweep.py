"""Raster-order (group_m) sweep of the large-GEMM shapes vs hipBLASLt (torch.matmul).
One JSON line per (shape, op, group_m)."""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ, MNMAJ  # noqa: E402
from stage_sweep import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for (R, K, N) in [(16384, 8192, 8192), (16384, 832, 8192), (65536, 832, 512)]:
        x = torch.randn(R, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
        dz = torch.randn(R, N, device=dev, generator=g).to(torch.bfloat16)
        y = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(R, K, device=dev, dtype=torch.bfloat16)
        slab = torch.empty(1, N, K, device=dev)
        flop = 2.0 * R * N * K
        it = max(3, min(30, int(3e12 / flop)))
        ref = {"fwd": lambda: torch.mm(x, w.t()), "dgrad": lambda: torch.mm(dz, w),
               "wgrad": lambda: torch.mm(dz.t(), x)}
        for op in ("fwd", "dgrad", "wgrad"):
            t_ref = timeit(ref[op], it)
            for (tile, ns, gm) in [((256, 256), 2, 4), ((256, 64), 2, 4), ((128, 128), 2, 4)]:
                if op == "fwd":
                    fn = lambda: ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=R, N=N, K=K,  # noqa: E731,E501
                                          tiles=tile, group_m=gm, stages=ns)
                elif op == "dgrad":
                    fn = lambda: ops.gemm(dz, w, dx, layout_a=KMAJ, layout_b=MNMAJ, M=R, N=K,  # noqa: E731,E501
                                          K=N, tiles=tile, group_m=gm, stages=ns)
                else:
                    if K % tile[1] or N % tile[0]:
                        continue
                    fn = lambda: ops.gemm(dz, x, slab, layout_a=MNMAJ, layout_b=MNMAJ, M=N,  # noqa: E731,E501
                                          N=K, K=R, tiles=tile, group_m=gm, stages=ns)
                t = timeit(fn, it)
                print(json.dumps({"shape": [R, K, N], "op": op, "group_m": gm, "tile": tile, "ns": ns, "us": round(t, 1),
                                  "tflops": round(flop / t / 1e6, 1),
                                  "hipblaslt_tflops": round(flop / t_ref / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
