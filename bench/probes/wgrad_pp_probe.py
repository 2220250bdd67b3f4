"""Ping-pong 256x256 form (gemm_pp.hip, MN-major operands) on the headline's 512x832 weight
gradient: the whole output (one partial column tile) and the 768-wide bulk alone, over split
counts, against the tuned 128x128 split-K kernel. Isolated HIP-event timing."""
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
R, K, N = 65536, 832, 512
dz = torch.randn(R, N, device=dev).to(torch.bfloat16)
x = torch.randn(R, K, device=dev).to(torch.bfloat16)
for KK, label in ((832, "full"), (768, "bulk768")):
    for s in (16, 24, 32, 42, 48, 64):
        slabs = torch.empty(s, N, KK, device=dev)
        for tile, st in (((256, 256), 8), ((256, 256), 2), ((128, 128), 2)):
            try:
                us = timeit(lambda: ops.gemm(dz, x, slabs, layout_a=MNMAJ, layout_b=MNMAJ, M=N,
                                             N=KK, K=R, k_total=R, splits=s, tiles=tile,
                                             stages=st), 10)
                print(json.dumps({"n": label, "splits": s, "tile": tile, "stages": st,
                                  "us": round(us, 1)}), flush=True)
            except (ValueError, RuntimeError) as e:
                print(json.dumps({"n": label, "splits": s, "tile": tile, "err": str(e)[:80]}))
