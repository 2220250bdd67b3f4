"""Interpreter of a rank's native StepPlan op list over ``torch.distributed`` (gloo).

The RCCL native step (parallel/native_step.py) can only run across ranks with one GPU per
rank, which a one-GPU box does not have. This interpreter executes the EXACT op list
``NativeStep._build`` produces for RCCL -- the same recorded segments, the same device
addresses, byte counts, peers, communicators and the same stream / event structure -- with
every RCCL operation mapped onto gloo on host copies of the addressed bytes:

  SEG            replay of the recorded segment on the device (one torch stream)
  SEND / RECV    isend / irecv of ``count`` elements at address ``a`` to / from the op's peer on
                 the gloo group standing in for its communicator
  GROUP          all members posted together, retired when all completed
  ALLREDUCE      in-place sum over the group;  REDUCE_SCATTER ``a`` (count x group size) -> ``b``;
  ALL_GATHER     ``a`` (count) -> ``b`` (count x group size)
  REC / WAIT     host-side event flags between the plan's streams
  COPY / SIGNAL / WAITV   (IPC plans) the real device ops on the interpreter's stream: a peer
                 copy into an IPC-mapped buffer, a flag store / wait at step number + delta
                 (processes sharing one GPU map each other's memory)

Streams are interpreted cooperatively (each advances while its head op can), so a plan whose
streams block each other shows up as an interpreter stall (a timeout naming the stream heads),
and the data an op moves is the data the GPU plan would move: a wrong offset, count or peer
breaks bitwise equality with the Python executor (tests/test_dist_gpu.py).
"""
from __future__ import annotations

import threading
import time
from typing import Optional

import torch
import torch.distributed as dist

from .native_step import (ALL_GATHER, ALLREDUCE, COPY, ESIZE, GROUP, NCCL_BF16, NCCL_F32,
                          NCCL_U8, REC, RECV, REDUCE_SCATTER, SEG, SEND, SIGNAL, WAIT, WAITV)

DTYPES = {NCCL_BF16: torch.bfloat16, NCCL_F32: torch.float32, NCCL_U8: torch.uint8}


class DeviceMemory:
    """Device address -> tensor view, over a set of contiguous device tensors."""

    def __init__(self, tensors):
        self.ranges = []
        seen = set()
        for t in tensors:
            if not isinstance(t, torch.Tensor) or \
                    not t.is_contiguous() or t.numel() == 0 or t.data_ptr() in seen:
                continue
            seen.add(t.data_ptr())
            self.ranges.append((t.data_ptr(), t.numel() * t.element_size(), t))

    def view(self, addr: int, count: int, dtype: int) -> torch.Tensor:
        nbytes = count * ESIZE[dtype]
        for base, size, t in self.ranges:
            if base <= addr and addr + nbytes <= base + size:
                flat = t.reshape(-1).view(torch.uint8)
                return flat[addr - base:addr - base + nbytes].view(DTYPES[dtype])
        raise KeyError(f"address {addr:#x} (+{nbytes} B) is in no registered device buffer")


def stage_memory(st) -> DeviceMemory:
    ts = list(vars(st).values()) + list(vars(st.params).values())
    for v in list(ts):
        if isinstance(v, (list, tuple)):
            ts += [x for x in v if isinstance(x, torch.Tensor)]
        elif isinstance(v, dict):
            ts += [x for x in v.values() if isinstance(x, torch.Tensor)]
    return DeviceMemory(ts)


class _Done:
    """Completion of a gloo work: gloo's send / receive works report is_completed() only after
    wait(), so a helper thread waits and the interpreter polls the flag."""

    def __init__(self, work):
        self.work, self.err = work, None
        self.ev = threading.Event()
        threading.Thread(target=self._run, daemon=True).start()

    def _run(self):
        try:
            self.work.wait()
        except Exception as e:  # surfaced by the interpreter
            self.err = e
        self.ev.set()

    def done(self) -> bool:
        if self.ev.is_set() and self.err is not None:
            raise self.err
        return self.ev.is_set()


class PlanInterpreter:
    """``groups``: communicator handle (the names NativeStep was built with) -> gloo group."""

    def __init__(self, ns, groups: dict, timeout_s: float = 120.0):
        self.ns, self.groups, self.timeout = ns, groups, timeout_s
        # a co-located fan rank's plan addresses every hosted worker's buffers
        self.stages = list(getattr(ns, "stages_all", None) or [ns.st])
        self.mem = DeviceMemory([])
        for st in self.stages:
            self.mem.ranges += stage_memory(st).ranges
        self.stream = torch.cuda.current_stream(ns.st.device)
        self.queues: dict[int, list] = {}
        for o in ns.ops:
            self.queues.setdefault(o["stream"], []).append(o)

    # ---- one op ------------------------------------------------------------------------------
    def _host(self, addr, count, dtype):
        return self.mem.view(addr, count, dtype).cpu()

    def _start(self, o):
        """Post an RCCL-mapped op; returns a list of (work, finish callback)."""
        k = o["kind"]
        g = self.groups[o["comm"]]
        if k in (SEND, RECV):
            tag = 1 if o["tag"][0] == "f" else 2
            if k == SEND:
                torch.cuda.synchronize()
                buf = self._host(o["a"], o["count"], o["dtype"])
                return [(dist.isend(buf, dst=o["gpeer"], group=g, tag=tag), None)]
            buf = torch.empty(o["count"], dtype=DTYPES[o["dtype"]])
            dst = self.mem.view(o["a"], o["count"], o["dtype"])
            return [(dist.irecv(buf, src=o["gpeer"], group=g, tag=tag),
                     lambda: dst.copy_(buf))]
        torch.cuda.synchronize()
        n = dist.get_world_size(g)
        if k == ALLREDUCE:
            buf = self._host(o["a"], o["count"], o["dtype"])
            dst = self.mem.view(o["a"], o["count"], o["dtype"])
            return [(dist.all_reduce(buf, group=g, async_op=True), lambda: dst.copy_(buf))]
        if k == REDUCE_SCATTER:
            src = self._host(o["a"], o["count"] * n, o["dtype"])
            out = torch.empty(o["count"], dtype=DTYPES[o["dtype"]])
            dst = self.mem.view(o["b"], o["count"], o["dtype"])
            return [(dist.reduce_scatter_tensor(out, src, group=g, async_op=True),
                     lambda: dst.copy_(out))]
        if k == ALL_GATHER:
            src = self._host(o["a"], o["count"], o["dtype"])
            out = torch.empty(o["count"] * n, dtype=DTYPES[o["dtype"]])
            dst = self.mem.view(o["b"], o["count"] * n, o["dtype"])
            return [(dist.all_gather_into_tensor(out, src, group=g, async_op=True),
                     lambda: dst.copy_(out))]
        raise ValueError(f"op kind {k} is not an RCCL op")

    # ---- one step ------------------------------------------------------------------------------
    def run_step(self) -> None:
        ns = self.ns
        for st in self.stages:
            st.params.set_lr(st.params.optim.lr)
        ipc = getattr(ns, "ipc", None)
        nat = None
        if ipc is not None or any(o["kind"] == COPY for q in self.queues.values() for o in q):
            from ..utils.native import native

            nat = native()  # device copies: IPC hops, and a co-located rank's local hops
        seq = 0
        if ipc is not None:
            ipc.seq += 1
            seq = ipc.seq
        head = {s: 0 for s in self.queues}
        events: set = set()
        inflight: dict[int, list] = {}
        t0 = time.monotonic()
        with torch.cuda.stream(self.stream):
            while any(head[s] < len(q) for s, q in self.queues.items()):
                progress = False
                for s, q in self.queues.items():
                    while head[s] < len(q):
                        o = q[head[s]]
                        k = o["kind"]
                        if s in inflight:
                            works = inflight[s]
                            if not all(w.done() for w, _ in works):
                                break
                            for _, fin in works:
                                if fin is not None:
                                    fin()
                            del inflight[s]
                        elif k == SEG:
                            o["prog"].run([o["seg"]], self.stream.cuda_stream)
                        elif k == COPY:
                            nat.copy_async(o["b"], o["a"], o["count"], self.stream.cuda_stream)
                        elif k == SIGNAL:
                            nat.signal_u32(self.stream.cuda_stream, o["a"], seq + o["delta"])
                        elif k == WAITV:
                            nat.wait_geq_u32(self.stream.cuda_stream, o["a"], seq + o["delta"])
                        elif k == REC:
                            events.add(o["event"])
                        elif k == WAIT:
                            if o["event"] not in events:
                                break
                        elif k == GROUP:
                            inflight[s] = [(_Done(w), f) for m in o["ops"]
                                           for w, f in self._start(m)]
                            continue
                        else:
                            inflight[s] = [(_Done(w), f) for w, f in self._start(o)]
                            continue
                        head[s] += 1
                        progress = True
                if not progress:
                    if time.monotonic() - t0 > self.timeout:
                        heads = {s: (q[head[s]]["kind"], q[head[s]].get("tag") or
                                     q[head[s]].get("seg") or q[head[s]].get("event"))
                                 for s, q in self.queues.items() if head[s] < len(q)}
                        raise RuntimeError(f"plan interpreter stalled: {heads}")
                    time.sleep(0.0005)
        torch.cuda.synchronize()
        for st in self.stages:
            st.params.step_count += 1


def interp_groups(mesh, names: Optional[dict] = None) -> tuple[dict, dict]:
    """(comms, groups) for NativeStep(..., comms=comms) + PlanInterpreter(groups): the link
    channels and the DP group of a gloo mesh."""
    comms, groups = {}, {}
    for name in ("f_in", "f_out", "b_in", "b_out"):
        g = getattr(mesh, "link_" + name)
        if g is not None:
            comms[name] = name
            groups[name] = g
    if mesh.dp_group is not None:
        comms["dp"] = "dp"
        groups["dp"] = mesh.dp_group
    return comms, groups
