"""Per-k-step cost vs fixed (prologue + epilogue) cost of the forward GEMM: time M x N x K for a
sweep of K at the headline's M = 65536, N = 512, per (tile, stage code, persistent) variant.
The slope over K is the steady-state k-step time, the intercept the per-tile overhead.
Usage: python bench/probes/k_sweep.py [--ks 64,832,3328] [--variants 256x256:2:0,256x256:6:0]"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops.kernels import KMAJ  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ks", default="64,128,256,512,832,1664,3328")
ap.add_argument("--ms", default="65536")
ap.add_argument("--n", type=int, default=512)
ap.add_argument("--variants", default="256x256:2:0,256x256:6:0,256x256:5:0")
ap.add_argument("--f32", action="store_true", help="fp32 output (no bias/act)")
a = ap.parse_args()
dev = torch.device("cuda")
variants = []
for v in a.variants.split(","):
    t, st, pe = v.split(":")
    bm, bn = (int(x) for x in t.split("x"))
    variants.append(((bm, bn), int(st), int(pe)))
for M in (int(m) for m in a.ms.split(",")):
    for K in (int(k) for k in a.ks.split(",")):
        N = a.n
        x = (torch.randn(M, K, device=dev) * 0.1).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        y = torch.empty(M, N, device=dev, dtype=torch.float32 if a.f32 else torch.bfloat16)
        res = {}
        for (tile, st, pe) in variants:
            def run():
                if a.f32:
                    ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, tiles=tile,
                             stages=st, persist=pe)
                else:
                    ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, bias=b,
                             act="relu", tiles=tile, stages=st, persist=pe)
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
            res[f"{tile[0]}x{tile[1]}:{st}:{pe}"] = round(statistics.median(ts), 2)
        print(json.dumps({"M": M, "N": N, "K": K, "f32": a.f32, "us": res}), flush=True)
