"""Per-workgroup phase timeline of one-tile GEMM kernels (GemmParams::timeline, s_memrealtime
at 100 MHz): where a tile's time goes -- launch skew, ring prologue, main loop, epilogue -- for
the headline forward / dgrad / wgrad shapes, per stage code. Prints medians over workgroups (us)
and the kernel span.

Usage: python bench/probes/gemm_timeline.py [--variants 256x256:2,256x256:6]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops.kernels import KMAJ, MNMAJ  # noqa: E402

dev = torch.device("cuda")


def rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


EPI = 0  # --epi-probe


def fwd(M, K, N):
    x, w, b = rnd(M, K, scale=0.1), rnd(N, K, scale=0.05), torch.randn(N, device=dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    return lambda tile, st, tl: ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K,
                                         bias=b, act="relu", tiles=tile, stages=st, timeline=tl,
                                         epi_probe=EPI)


def fwd_mask(M, K, N):
    """fwd with the fragment-order ReLU mask written too (DNN_RELU_MASK=2)."""
    x, w, b = rnd(M, K, scale=0.1), rnd(N, K, scale=0.05), torch.randn(N, device=dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    masks = {}

    def run(tile, st, tl):
        m = masks.setdefault(tile, ops.FragMask.alloc(M, N, tile, dev))
        return ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, bias=b,
                        act="relu", tiles=tile, stages=st, timeline=tl, mask_out=m)
    return run


def dgrad_mask(M, K, N):
    """dgrad with the ReLU derivative from a fragment-order mask instead of the activation."""
    dz, wt = rnd(M, K, scale=0.1), rnd(N, K, scale=0.05)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    masks = {}

    def run(tile, st, tl):
        m = masks.get(tile)
        if m is None:
            m = masks[tile] = ops.FragMask.alloc(M, N, tile, dev)
            m.buf.random_(0, 256)
        return ops.gemm(dz, wt, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, act="relu",
                        tiles=tile, stages=st, timeline=tl, mask_in=m)
    return run


def fwd32(M, K, N):
    x, w = rnd(M, K, scale=0.1), rnd(N, K, scale=0.05)
    y = torch.empty(M, N, device=dev)
    return lambda tile, st, tl: ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K,
                                         tiles=tile, stages=st, timeline=tl)


def wgrad(R, M, N, splits):
    dz, x = rnd(R, M), rnd(R, N)
    out = torch.empty(splits, M, N, device=dev)
    return lambda tile, st, tl: ops.gemm(dz, x, out, layout_a=MNMAJ, layout_b=MNMAJ, M=M, N=N,
                                         K=0, k_total=R, splits=splits, tiles=tile, stages=st,
                                         timeline=tl)


def dgrad(M, K, N):
    """dX = dZ . W with the W^T shadow (both K-major), ReLU derivative from the stored
    activation (the headline's dgrad 256 -> 512)."""
    dz, wt, h = rnd(M, K, scale=0.1), rnd(N, K, scale=0.05), rnd(M, N)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    return lambda tile, st, tl: ops.gemm(dz, wt, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N,
                                         K=K, aux=h, act="relu", tiles=tile, stages=st,
                                         timeline=tl, epi_probe=EPI)


CASES = {"f0": lambda: fwd(65536, 832, 512), "f1": lambda: fwd(65536, 512, 256),
         "d1": lambda: dgrad(65536, 256, 512), "d1s": lambda: dgrad(8192, 256, 512),
         "f0k": lambda: fwd_mask(65536, 832, 512), "d1k": lambda: dgrad_mask(65536, 256, 512),
         "f0s": lambda: fwd(8192, 832, 512), "f0m": lambda: fwd(32768, 832, 512),
         "f0f32": lambda: fwd32(65536, 832, 512), "f0sf32": lambda: fwd32(8192, 832, 512),
         "w0": lambda: wgrad(65536, 512, 832, 18), "m8f": lambda: fwd(65536, 1024, 1024)}


def q(v, f):
    v = sorted(v)
    return v[min(len(v) - 1, int(f * len(v)))]


ap = argparse.ArgumentParser()
ap.add_argument("--cases", default="f0,f1,w0,m8f")
ap.add_argument("--variants", default="256x256:2,256x256:6")
ap.add_argument("--wvariants", default="128x128:2,128x128:6")
ap.add_argument("--epi-probe", type=int, default=0,
                help="GemmParams::epi_probe bits for the register-direct epilogue (1: no stores, "
                     "2: no bias loads); outputs are wrong, only the phases are timed")
ap.add_argument("--cold", action="store_true",
                help="evict the Infinity Cache (write 1 GiB) before the timed run: operands "
                     "come from HBM, as inside the training step")
a = ap.parse_args()
EPI = a.epi_probe
flush = torch.empty(1 << 29, dtype=torch.bfloat16, device=dev) if a.cold else None
tl = torch.zeros(4 * 65536, dtype=torch.int64, device=dev)
for name in a.cases.split(","):
    run = CASES[name]()
    for v in (a.wvariants if name.startswith("w") else a.variants).split(","):
        t, st = v.split(":")
        tile = tuple(int(x) for x in t.split("x"))
        for _ in range(3):
            run(tile, int(st), None)
        tl.zero_()
        if flush is not None:
            flush.fill_(1.0)
        torch.cuda.synchronize()
        run(tile, int(st), tl)
        torch.cuda.synchronize()
        d = tl.view(-1, 4).cpu()
        d = d[d[:, 3] > 0].double() / 100.0  # us
        t0 = d[:, 0].min()
        start, pro, loop, epi = (d[:, 0] - t0), (d[:, 1] - d[:, 0]), (d[:, 2] - d[:, 1]), \
            (d[:, 3] - d[:, 2])
        print(json.dumps({
            "case": name, "cold": bool(a.cold), "epi_probe": EPI, "tile": list(tile), "stages": int(st), "wgs": int(d.shape[0]),
            "span_us": round(float(d[:, 3].max() - t0), 2),
            "start_us_p10_p50_p90": [round(float(q(start.tolist(), f)), 2) for f in (.1, .5, .9)],
            "prologue_us_med": round(float(q(pro.tolist(), .5)), 2),
            "loop_us_med": round(float(q(loop.tolist(), .5)), 2),
            "epilogue_us_med": round(float(q(epi.tolist(), .5)), 2),
            "epilogue_us_p10_p90": [round(float(q(epi.tolist(), f)), 2) for f in (.1, .9)],
            "loop_us_p10_p90": [round(float(q(loop.tolist(), f)), 2) for f in (.1, .9)],
            "wg_total_us_med": round(float(q((d[:, 3] - d[:, 0]).tolist(), .5)), 2)}),
            flush=True)
