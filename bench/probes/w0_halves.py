"""Feasibility of splitting the headline's layer-0 weight gradient and the next step's layer-0
forward into two output halves (the half the next forward needs first, then the other half
beside that forward): isolated times of the full GEMMs and of their halves over split counts
and tiles, plus the two halves run concurrently on two streams. One JSON line per row.
Usage: python bench/probes/w0_halves.py"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ, MNMAJ  # noqa: E402


def timed(fn, iters=30):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return round(s.elapsed_time(e) * 1e3 / iters, 2)


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    R, K, N = 65536, 832, 512
    x = torch.randn(R, K, device=dev, generator=g).to(torch.bfloat16)
    dz = torch.randn(R, N, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    y = torch.empty(R, N, device=dev, dtype=torch.bfloat16)

    def wg(M, splits, tile, stages, col0=0):
        sl = torch.empty(splits, M, K, device=dev)
        a = dz[:, col0:col0 + M]
        return lambda: ops.gemm(a, x, sl, layout_a=MNMAJ, layout_b=MNMAJ, M=M, N=K, K=R,
                                k_total=R, splits=splits, tiles=tile, stages=stages)

    print(json.dumps({"op": "W0 full", "splits": 18, "tile": [128, 128],
                      "us": timed(wg(512, 18, (128, 128), 9))}), flush=True)
    for tile in ((128, 128), (128, 64), (256, 256), (64, 64)):
        for splits in (18, 27, 36, 54, 72):
            try:
                us = timed(wg(256, splits, tile, 9))
            except Exception as e:  # noqa: BLE001
                us = str(e)[:60]
            print(json.dumps({"op": "W0 half", "splits": splits, "tile": list(tile), "us": us}),
                  flush=True)

    def fw(n0, n, tile, stages):
        return lambda: ops.gemm(x, w[n0:n0 + n], y[:, n0:n0 + n], layout_a=KMAJ, layout_b=KMAJ,
                                M=R, N=n, K=K, bias=b[n0:n0 + n], act="relu", tiles=tile,
                                stages=stages)

    print(json.dumps({"op": "fwd0 full", "us": timed(fw(0, 512, (256, 256), 9))}), flush=True)
    for tile, st in (((256, 256), 9), ((256, 256), 11), ((256, 128), 11), ((128, 128), 11)):
        print(json.dumps({"op": "fwd0 half", "tile": list(tile), "stages": st,
                          "us": timed(fw(0, 256, tile, st))}), flush=True)
    # the overlap: W0 second half (36 splits) beside the forward's first half
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    f_w, f_f = wg(256, 36, (128, 128), 9, 256), fw(0, 256, (256, 256), 9)

    def both():
        ev = torch.cuda.Event()
        ev.record()
        s1.wait_event(ev)
        s2.wait_event(ev)
        with torch.cuda.stream(s1):
            f_w()
        with torch.cuda.stream(s2):
            f_f()
        torch.cuda.current_stream().wait_stream(s1)
        torch.cuda.current_stream().wait_stream(s2)

    print(json.dumps({"op": "W0 half(36) || fwd0 half", "us": timed(both)}), flush=True)
    print(json.dumps({"op": "W0 half(36) then fwd0 half",
                      "us": timed(lambda: (f_w(), f_f()))}), flush=True)


if __name__ == "__main__":
    main()
