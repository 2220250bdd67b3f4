"""Diagnose native IPC pipeline steps with relayed hops on ONE GPU (ranks = processes sharing
cuda:0): every rank logs each completed step; a rank that makes no progress for `--stall`
seconds dumps its flag block (read on a fresh stream) and exits.

    python bench/relay_diag.py --world 3 --relays 1 --hwq 8 --out gpurun_out/relay
"""
from __future__ import annotations

import argparse
import os
import socket
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _worker(rank, a, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DNN_PIPE="ipc",
                      DNN_IPC_RELAYS=str(a.relays), GPU_MAX_HW_QUEUES=str(a.hwq))
    import torch.distributed as dist

    from docker_dist_nn_amd import MLPSpec
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer
    from docker_dist_nn_amd.parallel.groups import build_mesh

    log = open(os.path.join(a.out, f"diag_w{a.world}_k{a.relays}_r{rank}.log"), "w")

    def say(*x):
        print(f"[{time.time():.3f}]", *x, file=log, flush=True)

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=a.world)
    mesh = build_mesh(a.world, 1)
    tr = Trainer(MLPSpec.parse("784-512-256-128-10"), micro_batch=a.mb, num_micro=a.nm,
                 mesh=mesh, device=dev, schedule="1f1b", optim=OptimConfig(lr=0.05))
    say("built", "native" if tr.native_step is not None else "python",
        "duties", getattr(tr.pipe, "duties", None),
        "streams", 4 + len(getattr(tr.pipe, "duties", [])))
    x, y = synthetic_mnist(a.mb * a.nm, seed=1)
    xb = torch.zeros(a.mb * a.nm, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xd, yd = xb.to(dev), torch.from_numpy(y).to(dev)
    last = [time.time()]

    def watch():
        while True:
            time.sleep(1)
            if time.time() - last[0] > a.stall:
                s = torch.cuda.Stream(dev)
                with torch.cuda.stream(s):
                    f = tr.pipe.flags.to("cpu", non_blocking=False)
                say("STALL flags", f.tolist(), "seq", tr.pipe.seq)
                os._exit(3)

    threading.Thread(target=watch, daemon=True).start()
    host = []
    for step in range(a.steps):
        tr.set_batch(xd if tr.first else None, yd if tr.last else None, zero_copy=True)
        t0 = time.perf_counter()
        tr.step()  # host time of the enqueue only: the plan must never wait on the GPU
        host.append(time.perf_counter() - t0)
        torch.cuda.synchronize(dev)
        last[0] = time.time()
        say("step", step, "ok", f"host_us {host[-1] * 1e6:.1f}")
    if len(host) > 2:
        say("median host us per step", round(sorted(host[1:])[len(host[1:]) // 2] * 1e6, 1))
    dist.barrier()
    say("done")
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=3)
    ap.add_argument("--relays", type=int, default=1)
    ap.add_argument("--hwq", type=int, default=8)
    ap.add_argument("--mb", type=int, default=256)
    ap.add_argument("--nm", type=int, default=4)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--stall", type=float, default=20.0)
    ap.add_argument("--out", default="gpurun_out/relay")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(_worker, args=(a, port), nprocs=a.world, join=True, start_method="spawn")
    print("ok", a.world, a.relays)


if __name__ == "__main__":
    main()
