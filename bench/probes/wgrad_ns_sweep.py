"""Split-K wgrad GEMM: pipeline depth x tile x split count sweep (the in-step tuner only tries
depth 2 for wgrad). Isolated HIP-event timing; confirm winners in-step (bench/tune.py)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import MNMAJ  # noqa: E402
from stage_sweep import timeit  # noqa: E402

dev = torch.device("cuda")
shapes = [(65536, 832, 512), (65536, 512, 256), (65536, 1024, 1024)]
cands = [((128, 128), 2), ((128, 128), 3), ((128, 128), 4), ((256, 128), 2), ((256, 128), 3),
         ((128, 256), 2), ((128, 256), 3), ((128, 64), 3), ((128, 64), 4), ((64, 128), 3)]
for (R, K, N) in shapes:
    dz = torch.randn(R, N, device=dev).to(torch.bfloat16)
    x = torch.randn(R, K, device=dev).to(torch.bfloat16)
    for tile, ns in cands:
        if N % tile[0]:
            continue
        nt = (N // tile[0]) * -(-K // tile[1])
        for mult in (1, 2, 3, 4):
            s = max(1, round(mult * 256 / nt))
            slabs = torch.empty(s, N, K, device=dev)
            try:
                us = timeit(lambda: ops.gemm(dz, x, slabs, layout_a=MNMAJ, layout_b=MNMAJ, M=N,
                                             N=K, K=R, k_total=R, splits=s, tiles=tile,
                                             stages=ns), 10)
            except (ValueError, RuntimeError) as e:
                print(json.dumps({"shape": [R, K, N], "tile": tile, "ns": ns, "err": str(e)[:60]}))
                break
            print(json.dumps({"shape": [R, K, N], "tile": tile, "ns": ns, "splits": s,
                              "us": round(us, 1)}), flush=True)
