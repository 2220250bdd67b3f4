"""Why did capturing RCCL send/recv into a HIP graph crash the process? (VERDICT r3 #4,
profiles/r3_host/README.md: a StepPlan SEND+RECV to self on a one-rank communicator, captured
with GraphExec, took the process down.)

Each case runs in a child process of its own (a crash ends only that child), with
NCCL_DEBUG=WARN so RCCL says what it rejects. The cases separate the suspects:

  eager_self      the StepPlan group SEND+RECV to self, no capture (control)
  torch_allreduce torch.cuda.graph capture of dist.all_reduce on the same 1-rank communicator
                  (RCCL under torch's own capture)
  plan_self       the r3 crash: StepPlan group SEND+RECV to self captured by GraphExec
  plan_self_torch the same plan captured inside torch.cuda.graph (torch's capture path)
  plan_self_warm  plan_self after one eager run of the same plan (RCCL's lazy per-peer
                  connection set-up then happens outside the capture)
  plan_fork_signal  a 2-stream StepPlan with only a SIGNAL kernel on the side stream captured
                  (the plan's own fork / join under capture, no RCCL)
  plan_group_only   GSTART + GEND with nothing inside, captured (RCCL group calls alone)
  plan_send_only    the warm plan with the SEND alone inside the group (no matching RECV
                  issued under capture: only whether the capture call itself crashes)

Round-4 box run: eager_self ok; torch_allreduce "ok" but its graph is EMPTY (a 1-rank
all-reduce launches nothing), so it proves nothing; plan_self_warm segfaults inside
StepPlan.run under capture after the eager run succeeded. RCCL plans therefore stay eager.

Output: one JSON line per case {case, rc, ok, stderr_tail}. One GPU.
Usage: python bench/probes/rccl_capture.py
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# least to most likely to crash: a crash ends the probe (nothing more runs on the GPU after it)
CASES = ["eager_self", "torch_allreduce", "plan_fork_signal", "plan_group_only",
         "plan_send_only", "plan_self_warm", "plan_self_torch", "plan_self"]


def child(case: str) -> None:
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from docker_dist_nn_amd.parallel.native_step import (GEND, GSTART, NCCL_U8, RECV, SEND,
                                                         comm_ptr, torch_rccl_path)
    from docker_dist_nn_amd.utils.native import native

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n = native()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    t = torch.ones(1 << 10, device=dev)
    dist.all_reduce(t)
    torch.cuda.synchronize()
    if case == "torch_allreduce":
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.graph(g, stream=s):
            dist.all_reduce(t)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        print(f"replayed ok, t[0]={float(t[0])}", flush=True)
        dist.destroy_process_group()
        return
    if case == "plan_fork_signal":
        from docker_dist_nn_amd.parallel.native_step import SIGNAL
        flag = torch.zeros(4, dtype=torch.int32, device=dev)
        p = n.StepPlan(2, 1)
        p.add(kind=SIGNAL, stream=1, a=flag.data_ptr(), delta=0)
        s = torch.cuda.Stream(dev)
        g = n.GraphExec()
        g.begin_capture(s.cuda_stream)
        try:
            p.run(s.cuda_stream)
        finally:
            g.end_capture()
        g.replay(s.cuda_stream)
        torch.cuda.synchronize()
        print(f"fork/signal plan captured ({g.num_nodes} nodes) and replayed", flush=True)
        dist.destroy_process_group()
        return
    n.nccl_load(torch_rccl_path())
    comm = comm_ptr(dist.group.WORLD, dev)
    if case in ("plan_group_only", "plan_send_only"):
        buf = torch.zeros(4096, dtype=torch.uint8, device=dev)
        p = n.StepPlan(2, 1)
        p.add(kind=GSTART, stream=1)
        if case == "plan_send_only":
            p.add(kind=SEND, stream=1, comm=comm, a=buf.data_ptr(), count=buf.numel(),
                  dtype=NCCL_U8, peer=0)
        p.add(kind=GEND, stream=1)
        s = torch.cuda.Stream(dev)
        g = n.GraphExec()
        print("capturing", flush=True)
        g.begin_capture(s.cuda_stream)
        try:
            p.run(s.cuda_stream)
        finally:
            g.end_capture()
        print(f"captured {g.num_nodes} nodes (not replayed)", flush=True)
        dist.destroy_process_group()
        return
    buf = torch.arange(4096, dtype=torch.int32, device=dev).view(torch.uint8)
    rb = torch.zeros_like(buf)
    p = n.StepPlan(2, 1)
    p.add(kind=GSTART, stream=1)
    p.add(kind=SEND, stream=1, comm=comm, a=buf.data_ptr(), count=buf.numel(), dtype=NCCL_U8,
          peer=0)
    p.add(kind=RECV, stream=1, comm=comm, a=rb.data_ptr(), count=rb.numel(), dtype=NCCL_U8,
          peer=0)
    p.add(kind=GEND, stream=1)
    s = torch.cuda.Stream(dev)
    if case in ("eager_self", "plan_self_warm"):
        p.run(s.cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(rb, buf), "eager self send/recv moved the wrong bytes"
        print("eager ok", flush=True)
        if case == "eager_self":
            dist.destroy_process_group()
            return
        rb.zero_()
    if case in ("plan_self", "plan_self_warm"):
        g = n.GraphExec()
        print("capturing", flush=True)
        g.begin_capture(s.cuda_stream)
        try:
            p.run(s.cuda_stream)
        finally:
            g.end_capture()
        print(f"captured {g.num_nodes} nodes", flush=True)
        g.replay(s.cuda_stream)
    else:  # plan_self_torch
        g = torch.cuda.CUDAGraph()
        s.wait_stream(torch.cuda.current_stream())
        print("capturing (torch)", flush=True)
        with torch.cuda.graph(g, stream=s):
            p.run(s.cuda_stream)
        print("captured", flush=True)
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(rb, buf), "replayed self send/recv moved the wrong bytes"
    print("replay ok", flush=True)
    dist.destroy_process_group()


def main() -> None:
    port = 29650
    for case in CASES:
        port += 1
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   NCCL_DEBUG="WARN")
        try:
            r = subprocess.run([sys.executable, __file__, "--child", case], env=env,
                               capture_output=True, text=True, timeout=120)
            rc, out, err = r.returncode, r.stdout, r.stderr
        except subprocess.TimeoutExpired as e:
            rc, out, err = "timeout", (e.stdout or b"").decode(), (e.stderr or b"").decode()
        print(json.dumps({"case": case, "rc": rc, "ok": rc == 0,
                          "stdout_tail": out.strip().splitlines()[-3:],
                          "stderr_tail": err.strip().splitlines()[-12:]}), flush=True)
        if rc == "timeout" or (isinstance(rc, int) and (rc < 0 or rc >= 124)):
            print(json.dumps({"stopped_after": case}), flush=True)
            break


if __name__ == "__main__":
    if len(sys.argv) == 3 and sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        main()
