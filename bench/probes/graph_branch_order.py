"""Does a HIP graph run its independent branches concurrently? (the captured
relayed-IPC rank step stalled, profiles/r3_ipc/README.md.)

One process, one GPU. N streams are forked from a capture stream; branch 0 spins on a flag
(chain_wait, 2 s timeout -> error word instead of a hang), branches 1..N-2 do a trivial signal
of their own, branch N-1 sets the flag. Run eagerly (every stream on its own hardware queue:
GPU_MAX_HW_QUEUES is raised before HIP starts) the branches overlap and branch 0 sees the flag.
If the graph executor maps the branches onto fewer internal streams than there are branches,
or launches them in one topological order, branch 0 can run ahead of branch N-1 on a shared
stream and only its timeout ends it -- exactly the shape of the relayed IPC step, whose relay
duty streams spin on flags that other branches (and other ranks) release.

For N in 2, 3, 4, 6, 8, 12 and both capture orders (waiting branch enqueued first / last),
each graph is replayed 3 times. Output: one JSON line per case; err 1 = the wait timed out.
Usage: python bench/probes/graph_branch_order.py
"""
from __future__ import annotations

import json
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "24")  # before HIP initialises (eager reference)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from docker_dist_nn_amd.utils.native import native  # noqa: E402

TIMEOUT_S = 2.0


def enqueue(n, s0, streams, buf, wait_first):
    """Fork every stream from s0, branch 0 waits on buf[0], branch N-1 signals it, join."""
    flag, err = buf.data_ptr(), buf.data_ptr() + 4 * 16
    ev = torch.cuda.Event()
    ev.record(s0)
    for s in streams:
        s.wait_event(ev)
    last = len(streams) - 1
    order = list(range(len(streams))) if wait_first else list(range(len(streams)))[::-1]
    for i in order:
        s = streams[i]
        if i == 0:
            n.chain_wait(s.cuda_stream, flag, 1, err, TIMEOUT_S)
        elif i == last:
            n.chain_signal(s.cuda_stream, flag, 1)
        else:  # a branch of its own that releases nothing anyone waits for
            n.chain_signal(s.cuda_stream, flag + 4 * (32 + i), 1)
    for s in streams:
        e = torch.cuda.Event()
        e.record(s)
        s0.wait_event(e)


def main():
    n = native()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    buf = torch.zeros(128, dtype=torch.int32, device=dev)
    s0 = torch.cuda.Stream(dev)
    pool = [torch.cuda.Stream(dev) for _ in range(12)]
    for nb in (2, 3, 4, 6, 8, 12):
        streams = pool[:nb]
        for wait_first in (True, False):
            buf.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            enqueue(n, s0, streams, buf, wait_first)
            torch.cuda.synchronize()
            eager = {"err": int(buf[16].item()), "ms": round((time.perf_counter() - t0) * 1e3, 2)}
            g = n.GraphExec()
            buf.zero_()
            torch.cuda.synchronize()
            s0.wait_stream(torch.cuda.current_stream())
            g.begin_capture(s0.cuda_stream)
            try:
                enqueue(n, s0, streams, buf, wait_first)
            finally:
                g.end_capture()
            runs = []
            for _ in range(3):
                buf.zero_()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                g.replay(s0.cuda_stream)
                s0.synchronize()
                runs.append({"err": int(buf[16].item()),
                             "ms": round((time.perf_counter() - t0) * 1e3, 2)})
            print(json.dumps({"branches": nb,
                              "capture_order": "wait first" if wait_first else "signal first",
                              "nodes": g.num_nodes, "eager": eager, "graph_replays": runs}),
                  flush=True)


if __name__ == "__main__":
    main()
