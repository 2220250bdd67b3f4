"""Per-tile fixed cost vs per-k-step cost of the forward GEMM: time the fwd of M x N at several
K and fit T = a + b*K per tile config (a = prologue + epilogue + launch, b = main loop)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ  # noqa: E402
from stage_sweep import timeit  # noqa: E402

dev = torch.device("cuda")
M, N = 65536, 512
Ks = [832, 1664, 3328, 6656]
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(M, Ks[-1], device=dev, generator=g).to(torch.bfloat16)
w = torch.randn(N, Ks[-1], device=dev, generator=g).to(torch.bfloat16) * 0.05
y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
b = torch.randn(N, device=dev)
for tile in [(256, 256), (256, 64), (128, 128), (64, 128)]:
    ts = []
    for K in Ks:
        xs, ws = x[:, :K], w[:, :K]
        ts.append(timeit(lambda: ops.gemm(xs, ws, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K,
                                          bias=b, act="relu", tiles=tile), 20))
    bb, aa = np.polyfit(Ks, ts, 1)
    tiles = (M // tile[0]) * (N // tile[1])
    print(json.dumps({"tile": tile, "us": [round(t, 1) for t in ts], "fixed_us": round(aa, 1),
                      "us_per_64k": round(bb * 64, 3), "tiles": tiles,
                      "tflops_at_K832": round(2 * M * N * 832 / ts[0] / 1e6, 1),
                      "tflops_loop": round(2 * M * N * 64 / (bb * 64) / 1e6, 1)}), flush=True)
