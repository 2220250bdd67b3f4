"""Large GEMMs of the BASELINE models, isolated: hipBLASLt (torch.mm, no epilogue) vs our
256x256 one-tile kernel (stages 2), the ping-pong form (stages 8, gemm_pp.hip) and smaller tiles."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops import KMAJ, MNMAJ  # noqa: E402
from stage_sweep import timeit  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
SHAPES = [("fwd", 16384, 8192, 8192), ("dgrad", 16384, 8192, 8192), ("fwd", 65536, 832, 512),
          ("fwd", 65536, 1024, 1024), ("dgrad", 65536, 1024, 1024), ("fwd", 65536, 512, 256)]
for op, R, K, N in SHAPES:
    x = torch.randn(R, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    dz = torch.randn(R, N, device=dev, generator=g).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    y = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(R, K, device=dev, dtype=torch.bfloat16)
    if op == "fwd":
        ref = lambda: torch.mm(x, w.t(), out=y)  # noqa: E731  hipBLASLt, no epilogue
    else:
        ref = lambda: torch.mm(dz, w, out=dx)  # noqa: E731
    us = timeit(ref, 10 if K * N > 1e7 else 30)
    print(json.dumps({"op": op, "M": R, "K": K, "N": N, "tile": "hipblaslt", "stages": 0,
                      "us": round(us, 2), "tflops": round(2.0 * R * K * N / us / 1e6, 1)}),
          flush=True)
    for tile, ns in [((256, 256), 2), ((256, 256), 8), ((256, 64), 2), ((128, 128), 2)]:
        if op == "fwd":
            fn = lambda: ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=R, N=N, K=K,  # noqa
                                  bias=b, act="relu", tiles=tile, stages=ns)
        else:
            fn = lambda: ops.gemm(dz, w, dx, layout_a=KMAJ, layout_b=MNMAJ, M=R, N=K, K=N,  # noqa
                                  aux=x, act="relu", tiles=tile, stages=ns)
        us = timeit(fn, 10 if K * N > 1e7 else 30)
        print(json.dumps({"op": op, "M": R, "K": K, "N": N, "tile": tile, "stages": ns,
                          "us": round(us, 2), "tflops": round(2.0 * R * K * N / us / 1e6, 1)}),
              flush=True)
