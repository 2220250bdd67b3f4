"""Where the fused classifier tail's time goes: the kernel (csrc/kernels/mlp_tail.hip) is built
into separate probe libraries with parts removed (-DDNN_TAIL_PROBE bits: 1 = no bias-gradient
column sums, 2 = no global stores, 4 = no softmax) and timed against the full kernel over a
rows sweep, HIP-event timed, alternating variants.

Build (CPU, here): python bench/probes/tail_probe.py --build
Run (GPU box):     python bench/probes/tail_probe.py [--rows 16384,32768,65536,131072]"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "build")
VARIANTS = (0, 1, 2, 4, 7)


def lib_path(v: int) -> str:
    return os.path.join(OUT, f"tail_probe_{v}.so")


def build() -> None:
    os.makedirs(OUT, exist_ok=True)
    for v in VARIANTS:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
               "-shared", "-fno-slp-vectorize", f"-I{ROOT}/csrc", f"-I{ROOT}/csrc/kernels",
               f"-DDNN_TAIL_PROBE={v}", os.path.join(HERE, "tail_probe.hip"), "-o", lib_path(v)]
        subprocess.run(cmd, check=True)
        print("built", lib_path(v))


class TailParams(ctypes.Structure):  # csrc/kernels/mlp_tail.hpp, field for field
    P, L, I, F = ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_float
    _fields_ = [("X", P), ("ldx", L), ("W3", P), ("ldw3", L), ("b3", P), ("W4", P), ("ldw4", L),
                ("b4", P), ("labels", P), ("H3", P), ("ldh3", L), ("DZ4", P), ("lddz4", L),
                ("DZ3", P), ("lddz3", L), ("DZ2", P), ("lddz2", L), ("loss_part", P),
                ("correct", P), ("cs4", P), ("ld_cs4", L), ("cs3", P), ("ld_cs3", L),
                ("cs2", P), ("ld_cs2", L), ("M", I), ("K3", I), ("N3", I), ("N4", I),
                ("n_cls", I), ("scale", F), ("act3", I), ("act2", I)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--rows", default="16384,32768,65536,131072")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    if a.build:
        return build()
    import torch

    sys.path.insert(0, ROOT)
    from docker_dist_nn_amd import ops

    dev = torch.device("cuda")
    libs = {v: ctypes.CDLL(lib_path(v)) for v in VARIANTS}
    bf = torch.bfloat16
    k3, n3, n4, nc = 256, 128, 64, 10
    relu = 1  # Act code of ReLU (csrc/kernels/common.hpp)
    for R in (int(r) for r in a.rows.split(",")):
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.relu(torch.randn(R, k3, device=dev, generator=g)).to(bf)
        w3 = (torch.randn(n3, k3, device=dev, generator=g) / k3 ** 0.5).to(bf)
        w4 = torch.zeros(n4, n3, device=dev, dtype=bf)
        w4[:nc] = (torch.randn(nc, n3, device=dev, generator=g) / n3 ** 0.5).to(bf)
        b3, b4 = torch.zeros(n3, device=dev), torch.zeros(n4, device=dev)
        lab = torch.randint(0, nc, (R,), device=dev, generator=g, dtype=torch.int32)
        h3, dz3 = (torch.empty(R, n3, device=dev, dtype=bf) for _ in range(2))
        dz4 = torch.empty(R, n4, device=dev, dtype=bf)
        dz2 = torch.empty(R, k3, device=dev, dtype=bf)
        nb = ops.tail_blocks(R)
        loss, corr = torch.zeros(nb, device=dev), torch.zeros(nb, device=dev, dtype=torch.int32)
        cs4, cs3, cs2 = (torch.zeros(nb, c, device=dev) for c in (n4, n3, k3))
        P = lambda t: t.data_ptr()  # noqa: E731
        prm = TailParams(P(x), k3, P(w3), k3, P(b3), P(w4), n3, P(b4), P(lab), P(h3), n3,
                         P(dz4), n4, P(dz3), n3, P(dz2), k3, P(loss), P(corr), P(cs4), n4,
                         P(cs3), n3, P(cs2), k3, R, k3, n3, n4, nc, 1.0 / R, relu, relu)
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        res = {v: [] for v in VARIANTS}
        for rep in range(3):
            for v in VARIANTS:
                fn = libs[v].tail_probe_launch
                for _ in range(5):
                    assert fn(ctypes.byref(prm), stream) == 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn(ctypes.byref(prm), stream)
                e1.record()
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) * 1e3 / a.iters)
        print(json.dumps({"rows": R, "us": {str(v): round(min(t), 2) for v, t in res.items()},
                          "legend": "0 full, 1 no colsum, 2 no stores, 4 no softmax, 7 none"}),
              flush=True)


if __name__ == "__main__":
    main()
