"""128x512 tiles (8 waves of 64x128, stage code 9): one 128-row panel against the whole 512-wide
weight, so the 65536-row input is read once instead of once per 256-column tile. The headline's
fwd 784->512 and dgrad 256->512 against their tuned 256x256 tiles, cold operands (a 256 MiB
buffer streamed between launches), bitwise against the incumbent. One JSON line per case.
The 128x512 tile was removed after this measurement: apply profiles/r6_headline/tile_128x512.patch
and rebuild to run it again."""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ  # noqa: E402


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
    R = 65536
    junk = torch.empty(64 << 20, device=dev)
    junk2 = torch.empty_like(junk)
    # fwd 784->512: X [R][832], W [512][832]
    x = torch.randn(R, 832, device=dev, generator=g).to(torch.bfloat16)
    w0 = (torch.randn(512, 832, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    b0 = torch.randn(512, device=dev, generator=g)
    # dgrad 256->512: dZ1 [R][256], W1^T [512][256], H0 [R][512] (ReLU derivative), colsum
    dz1 = torch.randn(R, 256, device=dev, generator=g).to(torch.bfloat16)
    w1t = (torch.randn(512, 256, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    h0 = torch.relu(torch.randn(R, 512, device=dev, generator=g)).to(torch.bfloat16)
    cases = []
    for tile in ((256, 256), (128, 512)):
        y = torch.empty(R, 512, device=dev, dtype=torch.bfloat16)
        cases.append(("fwd 784->512", tile, y, None, lambda y=y, tile=tile: ops.gemm(
            x, w0, y, layout_a=KMAJ, layout_b=KMAJ, M=R, N=512, K=832, bias=b0, act="relu",
            tiles=tile, stages=9)))
    for tile in ((256, 256), (128, 512)):
        y = torch.empty(R, 512, device=dev, dtype=torch.bfloat16)
        cs = torch.zeros(R // tile[0], 512, device=dev)
        cases.append(("dgrad 256->512", tile, y, cs, lambda y=y, cs=cs, tile=tile: ops.gemm(
            dz1, w1t, y, layout_a=KMAJ, layout_b=KMAJ, M=R, N=512, K=256, aux=h0, act="relu",
            tiles=tile, colsum=cs, stages=9)))
    ref = {}
    for name, tile, y, cs, f in cases:
        try:
            f()
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"op": name, "tile": tile, "err": str(e)[:120]}), flush=True)
            continue
        torch.cuda.synchronize()
        same = None
        if name in ref:
            same = bool(torch.equal(ref[name][0], y))
            if cs is not None:
                same = same and bool(torch.allclose(ref[name][1].sum(0), cs.sum(0), rtol=1e-3,
                                                    atol=1e-2))
        else:
            ref[name] = (y.clone(), None if cs is None else cs.clone())
        med, mn = cold(f, junk, junk2)
        print(json.dumps({"op": name, "tile": list(tile), "code": 9, "cold_us_median": med,
                          "cold_us_min": mn, "equal_to_256x256": same}), flush=True)


if __name__ == "__main__":
    main()
