"""Does a concurrent streaming read of the input (a prefetch into the Infinity Cache) speed up
the headline's first-layer forward on a COLD input? Four 65536x832 bf16 inputs (436 MB, more
than the 256 MB Infinity Cache) are used round-robin so each forward starts cold, as in the
training step where every step reads a new batch. Variants, alternating, HIP events around the
forward on the main stream:
  cold      forward alone
  warm      prefetch completed before the forward (upper bound)
  pf<B>     prefetch with B workgroups on a second stream, started with the forward
  pfnt<B>   the same with non-temporal loads

Build (CPU): python bench/probes/prefetch_probe.py --build
Run (GPU):   python bench/probes/prefetch_probe.py"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
LIB = os.path.join(HERE, "build", "prefetch_probe.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--iters", type=int, default=40)
    a = ap.parse_args()
    if a.build:
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                        os.path.join(HERE, "prefetch_probe.hip"), "-o", LIB], check=True)
        print("built", LIB)
        return
    import torch

    sys.path.insert(0, ROOT)
    from docker_dist_nn_amd import ops

    dev = torch.device("cuda")
    lib = ctypes.CDLL(LIB)
    M, K, N = 65536, 832, 512
    xs = [torch.randn(M, K, device=dev).to(torch.bfloat16) for _ in range(4)]
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    b = torch.zeros(N, device=dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    sink = torch.zeros(1, device=dev, dtype=torch.int32)
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()

    def pf(x, blocks, nt, stream):
        rc = lib.prefetch_launch(ctypes.c_void_p(x.data_ptr()), ctypes.c_long(x.numel() * 2),
                                 blocks, nt, ctypes.c_void_p(sink.data_ptr()),
                                 ctypes.c_void_p(stream.cuda_stream))
        assert rc == 0

    variants = ["cold", "warm", "pf64", "pf128", "pf256", "pfnt128"]
    res = {v: [] for v in variants}
    it = 0
    for rep in range(a.iters):
        for v in variants:
            x = xs[it % 4]
            it += 1
            if v == "warm":
                pf(x, 256, 0, main_s)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            if v.startswith("pf"):
                nt = v.startswith("pfnt")
                blocks = int(v[4:] if nt else v[2:])
                side.wait_event(e0)
                pf(x, blocks, int(nt), side)
            ops.linear_fwd(x, w, b, y, act="relu")
            e1.record(main_s)
            main_s.wait_stream(side)
            torch.cuda.synchronize()
            if rep >= 3:
                res[v].append(e0.elapsed_time(e1) * 1e3)
    out = {v: round(sorted(t)[len(t) // 2], 2) for v, t in res.items()}
    print(json.dumps({"shape": [M, N, K], "median_us": out}), flush=True)


if __name__ == "__main__":
    main()
