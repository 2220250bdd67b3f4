"""Can two ranks share ONE GPU in an RCCL communicator on this pool? (If so, the fan step's
real RCCL plan can be rehearsed on one GPU.) Two processes on cuda:0: init, all_reduce,
send/recv; prints one JSON line per rank."""
import json
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    out = {"rank": rank}
    try:
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", 0))
        t = torch.full((1024,), float(rank + 1), device="cuda")
        dist.all_reduce(t)
        torch.cuda.synchronize()
        out["all_reduce"] = float(t[0])
        if rank == 0:
            dist.send(torch.arange(8, device="cuda", dtype=torch.float32), 1)
        else:
            r = torch.empty(8, device="cuda")
            dist.recv(r, 0)
            torch.cuda.synchronize()
            out["recv"] = r.tolist()
        dist.destroy_process_group()
        out["ok"] = True
    except Exception as e:  # noqa: BLE001
        out["error"] = repr(e)[:300]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    port = int(sys.argv[1]) if len(sys.argv) > 1 else 29611
    mp.start_processes(worker, args=(2, port), nprocs=2, join=True, start_method="spawn")
