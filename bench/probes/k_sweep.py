"""Per-k-step cost vs fixed (prologue + epilogue) cost of the forward GEMM: time M x N x K for a
sweep of K at the headline's M = 65536, N = 512 (and M = 32768: one tile per CU), per stage code.
The slope over K is the steady-state k-step time, the intercept the per-tile overhead."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops.kernels import KMAJ  # noqa: E402

dev = torch.device("cuda")
codes = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "2,6,5").split(",")]
for M in (65536, 32768):
    for K in (64, 128, 256, 512, 832, 1664, 3328):
        N = 512
        x = (torch.randn(M, K, device=dev) * 0.1).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        res = {}
        for st in codes:
            def run():
                ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, bias=b,
                         act="relu", tiles=(256, 256), stages=st)
            run()
            torch.cuda.synchronize()
            ts = []
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(5):
                s.record()
                for _ in range(20):
                    run()
                e.record()
                torch.cuda.synchronize()
                ts.append(s.elapsed_time(e) / 20 * 1e3)
            res[st] = round(statistics.median(ts), 2)
        print(json.dumps({"M": M, "N": N, "K": K, "us": res}), flush=True)
