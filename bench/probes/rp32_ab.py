"""A/B of the 32-deep register-prefetched ring (stage codes 20 / 21, gemm_tile.hpp
mma_tile_rp32) against stage code 9 on the headline's big GEMMs, with COLD operands (a 512 MiB
buffer is rewritten between repetitions, so inputs come from HBM as in the step), HIP-event
timing, the variants interleaved. Also checks every output bitwise against code 9.

  python bench/probes/rp32_ab.py --reps 15 > gpurun_out/rp32_ab.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ, MNMAJ  # noqa: E402


def cases(dev, g):
    R = 65536
    bf = torch.bfloat16

    def rnd(*shape, s=1.0):
        return (torch.randn(*shape, device=dev, generator=g) * s).to(bf)

    x0 = rnd(R, 832)
    w0 = rnd(512, 832, s=0.05)
    b0 = torch.randn(512, device=dev, generator=g)
    h0 = torch.relu(rnd(R, 512))
    w1 = rnd(256, 512, s=0.05)
    b1 = torch.randn(256, device=dev, generator=g)
    dz1 = rnd(R, 256)
    w1t = w1.t().contiguous()  # [512][256]: the dgrad's K-major W^T shadow
    dz0 = rnd(R, 512)
    out = {}

    def fwd0(code, tiles=(256, 256)):
        y = out.setdefault(("f0", code), torch.empty(R, 512, device=dev, dtype=bf))
        ops.gemm(x0, w0, y, layout_a=KMAJ, layout_b=KMAJ, M=R, N=512, K=832, bias=b0,
                 act="relu", tiles=tiles, stages=code)
        return y

    def fwd1(code, tiles=(256, 256)):
        y = out.setdefault(("f1", code), torch.empty(R, 256, device=dev, dtype=bf))
        ops.gemm(h0, w1, y, layout_a=KMAJ, layout_b=KMAJ, M=R, N=256, K=512, bias=b1,
                 act="relu", tiles=tiles, stages=code)
        return y

    def dgrad1(code, tiles=(256, 256)):
        y = out.setdefault(("d1", code), torch.empty(R, 512, device=dev, dtype=bf))
        ops.gemm(dz1, w1t, y, layout_a=KMAJ, layout_b=KMAJ, M=R, N=512, K=256, aux=h0,
                 act="relu", tiles=tiles, stages=code)
        return y

    def wgrad0(code, tiles=(128, 128)):
        y = out.setdefault(("w0", code), torch.empty(18, 512, 832, device=dev))
        ops.gemm(dz0, x0, y, layout_a=MNMAJ, layout_b=MNMAJ, M=512, N=832, K=R, k_total=R,
                 splits=18, tiles=tiles, stages=code)
        return y

    def wgrad1(code, tiles=(128, 128)):
        y = out.setdefault(("w1", code), torch.empty(64, 256, 512, device=dev))
        ops.gemm(dz1, h0, y, layout_a=MNMAJ, layout_b=MNMAJ, M=256, N=512, K=R, k_total=R,
                 splits=64, tiles=tiles, stages=code)
        return y

    return {"fwd0 784->512": fwd0, "fwd1 512->256": fwd1, "dgrad1 256->512": dgrad1,
            "W0 512x832 s18": wgrad0, "W1 256x512 s64": wgrad1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--codes", default="9,20,21")
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    cs = cases(dev, g)
    codes = [int(c) for c in a.codes.split(",")]
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    for name, fn in cs.items():
        times = {c: [] for c in codes}
        ref = None
        for c in codes:  # warm-up + bitwise check
            y = fn(c)
            torch.cuda.synchronize()
            if ref is None:
                ref = y.clone()
            elif not torch.equal(ref, y):
                print(json.dumps({"case": name, "code": c, "bitwise_equal": False}), flush=True)
        for _ in range(a.reps):
            for c in codes:
                flush.fill_(1)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn(c)
                e1.record()
                torch.cuda.synchronize()
                times[c].append(e0.elapsed_time(e1) * 1e3)
        for c in codes:
            v = sorted(times[c])
            print(json.dumps({"case": name, "code": c, "us_median": round(v[len(v) // 2], 2),
                              "us_min": round(v[0], 2)}), flush=True)


if __name__ == "__main__":
    main()
