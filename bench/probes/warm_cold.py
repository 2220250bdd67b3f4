"""Headline-step GEMMs isolated with cold operands (a 256 MiB buffer streamed between launches:
operands come from HBM, as in the step) and warm ones (back-to-back launches: operands in the
Infinity Cache / L2): the gap is what a latency-hiding change (deeper in-flight loads, an L2
prefetch) could win at best. One JSON line per GEMM. Usage: python bench/probes/warm_cold.py"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ, MNMAJ  # noqa: E402


def timed(f, flush, n=15):
    ts = []
    for _ in range(n):
        if flush is not None:
            flush()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        f()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 1)


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    R = 65536
    bf = torch.bfloat16
    x = torch.randn(R, 832, device=dev, generator=g).to(bf)
    w0 = torch.randn(512, 832, device=dev, generator=g).to(bf)
    h0 = torch.randn(R, 512, device=dev, generator=g).to(bf).relu_()
    w1t = torch.randn(256, 512, device=dev, generator=g).to(bf)  # dgrad B operand [K=256][N=512]
    w1 = torch.randn(256, 512, device=dev, generator=g).to(bf)
    dz1 = torch.randn(R, 256, device=dev, generator=g).to(bf)
    dz0 = torch.randn(R, 512, device=dev, generator=g).to(bf)
    b0 = torch.zeros(512, device=dev)
    b1 = torch.zeros(256, device=dev)
    y0 = torch.empty(R, 512, device=dev, dtype=bf)
    y1 = torch.empty(R, 256, device=dev, dtype=bf)
    sl0 = torch.empty(18, 512, 832, device=dev)
    sl1 = torch.empty(64, 256, 512, device=dev)
    junk = torch.empty(64 << 20, device=dev)
    junk2 = torch.empty_like(junk)
    cases = {
        "fwd0 784->512": lambda: ops.gemm(x, w0, y0, layout_a=KMAJ, layout_b=KMAJ, M=R, N=512,
                                          K=832, bias=b0, act="relu", tiles=(256, 256), stages=9),
        "fwd1 512->256": lambda: ops.gemm(h0, w1, y1, layout_a=KMAJ, layout_b=KMAJ, M=R, N=256,
                                          K=512, bias=b1, act="relu", tiles=(256, 256), stages=9),
        "dgrad1 256->512": lambda: ops.gemm(dz1, w1t, dz0, layout_a=KMAJ, layout_b=MNMAJ, M=R,
                                            N=512, K=256, aux=h0, act="relu", tiles=(256, 256),
                                            stages=9),
        "W0 512x832 s18": lambda: ops.gemm(dz0, x, sl0, layout_a=MNMAJ, layout_b=MNMAJ, M=512,
                                           N=832, K=R, k_total=R, splits=18, tiles=(128, 128),
                                           stages=9),
        "W1 256x512 s64": lambda: ops.gemm(dz1, h0, sl1, layout_a=MNMAJ, layout_b=MNMAJ, M=256,
                                           N=512, K=R, k_total=R, splits=64, tiles=(128, 128),
                                           stages=9),
    }
    for name, f in cases.items():
        try:
            f()
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"op": name, "err": str(e)[:100]}), flush=True)
            continue
        cold = timed(f, lambda: junk2.copy_(junk))
        warm = timed(f, None)
        print(json.dumps({"op": name, "cold_us": cold, "warm_us": warm}), flush=True)


if __name__ == "__main__":
    main()
