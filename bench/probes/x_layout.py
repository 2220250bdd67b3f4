"""Layer-0 GEMMs of the headline step (65536 rows, 832 padded inputs, 512 outputs) with the
input stored row-major X[rows][832] (today) or transposed X^T[832][rows] (a dataset layout
choice), and dZ0 row-major or transposed: the forward and the weight gradient per operand
layout, stage code and split count, isolated with cold operands (a 256 MiB buffer is streamed
between launches). One JSON line per configuration. Usage: python bench/probes/x_layout.py"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ, MNMAJ  # noqa: E402


def cold(f, junk, junk2, n=15):
    ts = []
    for _ in range(n):
        junk2.copy_(junk)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        f()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 1), round(ts[0], 1)


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    R, K, N = 65536, 832, 512
    x = torch.randn(R, K, device=dev, generator=g).to(torch.bfloat16)
    xt = x.t().contiguous()
    dz = torch.randn(R, N, device=dev, generator=g).to(torch.bfloat16)
    dzt = dz.t().contiguous()
    w = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16)
    b = torch.zeros(N, device=dev)
    y = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
    junk = torch.empty(64 << 20, device=dev)
    junk2 = torch.empty_like(junk)
    ref = None
    for name, a, la in (("fwd X", x, KMAJ), ("fwd XT", xt, MNMAJ)):
        for tile, code in (((256, 256), 9), ((256, 256), 11), ((256, 128), 9)):
            def f():
                ops.gemm(a, w, y, layout_a=la, layout_b=KMAJ, M=R, N=N, K=K, bias=b, act="relu",
                         tiles=tile, stages=code)
            try:
                f()
            except Exception as e:  # noqa: BLE001
                print(json.dumps({"op": name, "tile": tile, "code": code, "err": str(e)[:90]}),
                      flush=True)
                continue
            torch.cuda.synchronize()
            if ref is None:
                ref = y.clone()
            same = bool(torch.equal(ref, y))
            med, mn = cold(f, junk, junk2)
            print(json.dumps({"op": name, "tile": tile, "code": code, "cold_us_median": med,
                              "cold_us_min": mn, "bitwise_vs_first": same}), flush=True)
    ref = None
    for name, a, la, bb, lb in (("wgrad dZ,X", dz, MNMAJ, x, MNMAJ),
                                ("wgrad dZ,XT", dz, MNMAJ, xt, KMAJ),
                                ("wgrad dZT,XT", dzt, KMAJ, xt, KMAJ),
                                ("wgrad dZT,X", dzt, KMAJ, x, MNMAJ)):
        for tile, code in (((128, 128), 9), ((128, 128), 11), ((256, 128), 9), ((256, 256), 9)):
            for splits in (12, 18, 24):
                sl = torch.empty(splits, N, K, device=dev)

                def f():
                    ops.gemm(a, bb, sl, layout_a=la, layout_b=lb, M=N, N=K, K=R, k_total=R,
                             splits=splits, tiles=tile, stages=code)
                try:
                    f()
                except Exception as e:  # noqa: BLE001
                    print(json.dumps({"op": name, "tile": tile, "code": code, "splits": splits,
                                      "err": str(e)[:90]}), flush=True)
                    continue
                med, mn = cold(f, junk, junk2)
                print(json.dumps({"op": name, "tile": tile, "code": code, "splits": splits,
                                  "cold_us_median": med, "cold_us_min": mn}), flush=True)
                del sl


if __name__ == "__main__":
    main()
