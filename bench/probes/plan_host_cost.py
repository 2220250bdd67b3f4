"""Host cost of each StepPlan op kind (bench for VERDICT r2 item 7: host time per rank-step):
a plan of 128 ops of one kind is run 50 times and the host time of StepPlan.run is divided per
op. Kinds: REC+WAIT event pairs, SIGNAL / WAITV flag kernels, COPY kernels, SEG replays of a
one-kernel segment, RCCL SEND+RECV to self in a group (1-rank communicator), and the
standalone costs of hipGraph replay for comparison. One GPU, one process.
Usage: python bench/probes/plan_host_cost.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.parallel.native_step import (COPY, GEND, GSTART, NCCL_U8, REC,  # noqa
                                                     RECV, SEG, SEND, SIGNAL, WAIT, WAITV,
                                                     comm_ptr, torch_rccl_path)
from docker_dist_nn_amd.utils.native import native  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
n = native()
N, REPS = 128, 50
stream = torch.cuda.current_stream(dev).cuda_stream


def _median_us(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(REPS):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    t.sort()
    return t[len(t) // 2] * 1e6


GRAPH = {}


def host_us(plan, name=None):
    """Host us of plan.run; with a name, also of replaying the plan captured as a hipGraph
    (GRAPH[name] = (us, nodes))."""
    us = _median_us(lambda: plan.run(stream))
    if name:
        try:
            g = n.GraphExec()
            s = torch.cuda.Stream(dev)
            with torch.cuda.stream(s):
                g.begin_capture(s.cuda_stream)
                plan.run(s.cuda_stream)
                g.end_capture()
            torch.cuda.synchronize()
            GRAPH[name] = (_median_us(lambda: g.replay(stream)), g.num_nodes)
        except Exception as e:  # noqa: BLE001 -- report, keep measuring
            GRAPH[name] = (repr(e)[:120], 0)
    return us


res = {}
empty = n.StepPlan(2, 1)
base = host_us(empty)
res["empty_plan_us"] = round(base, 2)

p = n.StepPlan(2, N)
for k in range(N):
    p.add(kind=REC, stream=1, event=k)
    p.add(kind=WAIT, stream=0, event=k)
res["rec_wait_pair_us"] = round((host_us(p, "rec_wait") - base) / N, 3)

flags = torch.zeros(4 * N, dtype=torch.int32, device=dev)
p = n.StepPlan(1, 1)
for k in range(N):
    p.add(kind=SIGNAL, stream=0, a=flags.data_ptr() + 16 * k, delta=0)
res["signal_us"] = round((host_us(p, "signal") - base) / N, 3)

p = n.StepPlan(1, 1)
for k in range(N):  # flag already >= target: returns at once
    p.add(kind=WAITV, stream=0, a=flags.data_ptr() + 16 * k, delta=-1000)
res["waitv_us"] = round((host_us(p) - base) / N, 3)

src = torch.zeros(1 << 16, dtype=torch.uint8, device=dev)
dst = torch.zeros_like(src)
p = n.StepPlan(1, 1)
for k in range(N):
    p.add(kind=COPY, stream=0, a=src.data_ptr(), b=dst.data_ptr(), count=src.numel())
res["copy_64k_us"] = round((host_us(p) - base) / N, 3)

ctr = torch.zeros(1, dtype=torch.int32, device=dev)
prog = n.Program()
n.record_begin(prog)
prog.mark("K")
ops.step_advance(ctr)
n.record_end()
prog.close()
p = n.StepPlan(1, 1)
for k in range(N):
    p.add(kind=SEG, stream=0, prog=prog, seg="K")
res["seg_one_kernel_us"] = round((host_us(p, "seg") - base) / N, 3)

# eager kernel launch through the Python op (for scale)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N * 10):
    ops.step_advance(ctr)
res["python_op_launch_us"] = round((time.perf_counter() - t0) / (N * 10) * 1e6, 3)
torch.cuda.synchronize()

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29611")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
try:
    t = torch.ones(1, device=dev)
    dist.all_reduce(t)
    n.nccl_load(torch_rccl_path())
    comm = comm_ptr(dist.group.WORLD, dev)
    buf = torch.zeros(1 << 16, dtype=torch.uint8, device=dev)
    rb = torch.zeros_like(buf)
    p = n.StepPlan(2, 1)
    for k in range(N):
        p.add(kind=GSTART, stream=1)
        p.add(kind=SEND, stream=1, comm=comm, a=buf.data_ptr(), count=4096, dtype=NCCL_U8,
              peer=0)
        p.add(kind=RECV, stream=1, comm=comm, a=rb.data_ptr(), count=4096, dtype=NCCL_U8,
              peer=0)
        p.add(kind=GEND, stream=1)
    res["rccl_group_send_recv_us"] = round((host_us(p) - base) / N, 3)  # (capturing it crashed)
finally:
    dist.destroy_process_group()
res["graph_replay"] = {k: {"us": v[0], "nodes": v[1],
                           "us_per_op": round(v[0] / N, 3) if isinstance(v[0], float) else None}
                       for k, v in GRAPH.items()}
print(json.dumps(res), flush=True)
