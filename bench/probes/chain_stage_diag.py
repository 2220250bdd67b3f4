"""Diagnose the persistent stage kernel (chain_stage_run) on one GPU: launch it with a given
workgroup count, feed requests from the host, and print the kernel's control words after each
(or after a timeout). Usage: python bench/probes/chain_stage_diag.py [--wg 64] [--K 1024]"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from docker_dist_nn_amd.utils.devmem import uncached_zeros  # noqa: E402
from docker_dist_nn_amd.utils.native import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--wg", type=int, default=0)
    ap.add_argument("--K", type=int, default=1024)
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--requests", type=int, default=4)
    ap.add_argument("--dedicated", type=int, default=1)
    ap.add_argument("--ctl", default="host", choices=["host", "device"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = native()
    K, N, nslot = a.K, a.N, 4
    f_in = uncached_zeros((64,), torch.int32, dev)
    f_out = uncached_zeros((64,), torch.int32, dev)
    f_ack = uncached_zeros((16,), torch.int32, dev)
    f_prod = uncached_zeros((16,), torch.int32, dev)
    slots_in = uncached_zeros((nslot, 8, K), torch.bfloat16, dev)
    slots_out = uncached_zeros((nslot, 8, N), torch.bfloat16, dev)
    sync = torch.zeros(2 * nslot + 4, dtype=torch.int32, device=dev)
    hp, dp = n.host_alloc_mapped(64)
    ctl = np.ctypeslib.as_array((ctypes.c_uint32 * 16).from_address(hp))
    dctl = uncached_zeros((16,), torch.int32, dev)
    stop_p = dp if a.ctl == "host" else dctl.data_ptr()
    w = (torch.randn(N, K) * 0.05).to(torch.bfloat16).to(dev)
    b = torch.randn(N).to(dev)
    if a.dedicated:
        sp = n.stream_create_dedicated()
        s = torch.cuda.ExternalStream(sp, device=dev)
    else:
        s = torch.cuda.Stream(dev)
    torch.cuda.synchronize()

    def state(tag):
        print(f"[{tag}] f_in {f_in[:nslot].tolist()} hdr {f_in[16:16 + 2 * nslot].tolist()} "
              f"f_out {f_out[:nslot].tolist()} out_hdr {f_out[16:16 + 2 * nslot].tolist()} "
              f"prod_ack {int(f_prod[0])} sync {sync.tolist()} ctl {ctl[:4].tolist()} "
              f"dctl {dctl[:4].tolist()}",
              flush=True)

    wg = n.chain_stage_run(s.cuda_stream, f_in.data_ptr(), f_in.data_ptr() + 64,
                           slots_in.data_ptr(), K, f_prod.data_ptr(), w.data_ptr(), K,
                           b.data_ptr(), 1, N, K, 0, slots_out.data_ptr(), 8 * N * 2, N,
                           f_out.data_ptr() + 64, 2, f_out.data_ptr(), f_ack.data_ptr(), stop_p,
                           stop_p + 4, sync.data_ptr(), 0, 1, 1, nslot, 8, 3.0, 1.0, a.wg)
    print(f"launched {wg} workgroups", flush=True)
    side = torch.cuda.Stream(dev)
    torch.cuda.set_stream(side)
    time.sleep(0.2)
    state("after launch")
    x = (torch.randn(8, K) * 0.5).to(torch.bfloat16).to(dev)
    for seq in range(1, a.requests + 1):
        slot = seq % nslot
        slots_in[slot].copy_(x)
        f_in[16 + 2 * slot:18 + 2 * slot] = torch.tensor([0, 2], dtype=torch.int32, device=dev)
        torch.cuda.current_stream().synchronize()
        f_in[slot] = seq
        torch.cuda.current_stream().synchronize()
        t0 = time.monotonic()
        while int(f_out[slot]) != seq and time.monotonic() - t0 < 2.0:
            time.sleep(1e-3)
        ok = int(f_out[slot]) == seq
        print(f"request {seq}: {'served' if ok else 'NOT served'} in "
              f"{(time.monotonic() - t0) * 1e3:.2f} ms", flush=True)
        state(f"req {seq}")
        if ok:
            ref = torch.relu(x[:2].float() @ w.float().t() + b)
            print("  max err vs fp32", float((slots_out[slot, :2].float() - ref).abs().max()),
                  flush=True)
        f_ack[0] = seq
        torch.cuda.current_stream().synchronize()
    ctl[0] = 1
    dctl[0] = 1
    t0 = time.monotonic()
    s.synchronize()
    print(f"stopped in {(time.monotonic() - t0) * 1e3:.1f} ms", flush=True)
    state("end")


if __name__ == "__main__":
    main()
