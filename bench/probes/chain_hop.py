"""Device-side cost of one hop of the serving chain, without processes or Python between the
stages: one process, one stream per stage, stage k's stream holds chain_recv (spin on its
input flag) -> chain_gemv_send (its 1024x1024 layer straight into stage k+1's slot); stage 0
is fed by a chain_signal from the host stream and the last stage's flag is waited for by
chain_wait. Every request's kernels are enqueued before the first one is released, as in the
multi-process chain, and the request is timed with HIP events from the release to the last
flag. The slope over the stage count is the per-hop device latency (flag propagation + kernel
dispatch + GEMV); the multi-process rehearsal's chain_only latency minus this is host time.

Usage: python bench/probes/chain_hop.py [--stages 1,2,4,8] [--iters 200]"""
from __future__ import annotations

import argparse
import json
import os
import sys

# one hardware queue per stage stream (the box exports 4: with stages + the host stream
# sharing queues, a spinning receive would sit in front of the signal that releases it)
os.environ["GPU_MAX_HW_QUEUES"] = "16"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from docker_dist_nn_amd.utils.devmem import uncached_zeros  # noqa: E402
from docker_dist_nn_amd.utils.native import native  # noqa: E402


def run(n, dev, S, iters, W=1024, rows=1, form=1):
    """form 1: one kernel per hop (receive folded into chain_gemv_send); 2: chain_recv +
    chain_gemv_send; 3: chain_recv + gemv + chain_send."""
    flags = [uncached_zeros((64,), torch.int32, dev) for _ in range(S + 1)]  # [0] in, [2:4] hdr
    slots = [uncached_zeros((8, W), torch.bfloat16, dev) for _ in range(S + 1)]
    xl = [torch.zeros(8, W, dtype=torch.bfloat16, device=dev) for _ in range(S)]
    lh = [torch.zeros(4, dtype=torch.int32, device=dev) for _ in range(S)]
    err = [torch.zeros(4, dtype=torch.int32, device=dev) for _ in range(S + 1)]
    ctr = [torch.zeros(4, dtype=torch.int32, device=dev) for _ in range(S)]
    out = [torch.zeros(8, W, dtype=torch.bfloat16, device=dev) for _ in range(S)]
    w = [(torch.randn(W, W, device=dev) * 0.03).to(torch.bfloat16) for _ in range(S)]
    b = [torch.zeros(W, device=dev) for _ in range(S)]
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    host = torch.cuda.Stream(dev)
    rb = W * 2
    ts = []
    for it in range(1, iters + 1):
        for k in range(S):
            s = streams[k].cuda_stream
            fk, fn = flags[k].data_ptr(), flags[k + 1].data_ptr()
            if form == 1:
                n.chain_gemv_send(s, slots[k].data_ptr(), W, w[k].data_ptr(), W,
                                  b[k].data_ptr(), 1, rows, W, W, 0, slots[k + 1].data_ptr(), W,
                                  fn + 8, fk + 8, err[k].data_ptr(), k, 0, 0, 0, fn, it, 0,
                                  ctr[k].data_ptr(), 1.0, in_flag=fk)
                continue
            n.chain_recv(s, fk, slots[k].data_ptr(), rb, fk + 8, xl[k].data_ptr(), rb,
                         lh[k].data_ptr(), rows, rb, err[k].data_ptr(), it, 0, 1.0)
            if form == 2:
                n.chain_gemv_send(s, xl[k].data_ptr(), W, w[k].data_ptr(), W, b[k].data_ptr(),
                                  1, rows, W, W, 0, slots[k + 1].data_ptr(), W, fn + 8,
                                  lh[k].data_ptr(), err[k].data_ptr(), k, 0, 0, 0, fn, it, 0,
                                  ctr[k].data_ptr(), 1.0)
            else:
                n.gemv_bf16(xl[k].data_ptr(), W, w[k].data_ptr(), W, b[k].data_ptr(),
                            out[k].data_ptr(), W, rows, W, W, 1, 0, s)
                n.chain_send(s, out[k].data_ptr(), rb, slots[k + 1].data_ptr(), rb, rows, rb,
                             fn + 8, lh[k].data_ptr(), err[k].data_ptr(), k, 0, 0, 0, fn, it,
                             0, 1.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(host)
        n.chain_signal(host.cuda_stream, flags[0].data_ptr(), it)
        n.chain_wait(host.cuda_stream, flags[S].data_ptr(), it, err[S].data_ptr(), 1.0)
        e1.record(host)
        torch.cuda.synchronize(dev)
        if int(err[S][0]):
            raise RuntimeError(f"request {it} did not reach the end of the chain")
        ts.append(e0.elapsed_time(e1))
    t = np.asarray(ts[10:]) * 1e3
    return {"stages": S, "kernels_per_hop": form, "p50_us": round(float(np.percentile(t, 50)), 2),
            "p90_us": round(float(np.percentile(t, 90)), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stages", default="1,2,4,8")
    ap.add_argument("--iters", type=int, default=60)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n = native()
    for form in (1, 2, 3):
        for S in (int(v) for v in a.stages.split(",")):
            try:
                r = run(n, dev, S, a.iters, form=form)
            except RuntimeError as e:  # a request timed out (1 s): next form
                print(json.dumps({"stages": S, "kernels_per_hop": form, "error": str(e)}),
                      flush=True)
                break
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
