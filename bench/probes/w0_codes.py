"""The headline's layer-0 weight gradient (512x832 over 65536 rows, both operands MN-major,
fp32 split-K slabs) over tile x stage code x split count, isolated, with cold operands (a
256 MiB buffer is streamed between launches, as the step's other kernels do to the caches).
One JSON line per configuration. Usage: python bench/probes/w0_codes.py"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import MNMAJ  # noqa: E402


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    R, K, N = 65536, 832, 512
    x = torch.randn(R, K, device=dev, generator=g).to(torch.bfloat16)
    dz = torch.randn(R, N, device=dev, generator=g).to(torch.bfloat16)
    junk = torch.empty(64 << 20, device=dev)
    junk2 = torch.empty_like(junk)
    for tile, code in (((128, 128), 9), ((128, 128), 11), ((128, 128), 6), ((256, 128), 11),
                       ((128, 64), 9), ((256, 256), 11)):
        for splits in (12, 18, 24, 36):
            sl = torch.empty(splits, N, K, device=dev)

            def f():
                ops.gemm(dz, x, sl, layout_a=MNMAJ, layout_b=MNMAJ, M=N, N=K, K=R, k_total=R,
                         splits=splits, tiles=tile, stages=code)
            try:
                f()
            except Exception as e:  # noqa: BLE001
                print(json.dumps({"tile": tile, "code": code, "splits": splits,
                                  "err": str(e)[:80]}), flush=True)
                continue
            ts = []
            for _ in range(15):
                junk2.copy_(junk)  # evict the operands from L2 / the Infinity Cache
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                f()
                e.record()
                e.synchronize()
                ts.append(s.elapsed_time(e) * 1e3)
            ts.sort()
            print(json.dumps({"tile": tile, "code": code, "splits": splits,
                              "cold_us_median": round(ts[len(ts) // 2], 1),
                              "cold_us_min": round(ts[0], 1)}), flush=True)
            del sl


if __name__ == "__main__":
    main()
