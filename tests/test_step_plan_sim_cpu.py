"""Deadlock-freedom of the native multi-rank step plans (parallel/native_step.py) on the CPU.

Every rank's StepPlan op list is built exactly as on a GPU (NativeStep._build over the real
schedule and IpcPipe flag / relay layout), with fake device addresses instead of buffers, and
then executed by a small event simulator with HIP stream semantics: per-stream FIFO order,
hipStreamWaitValue32 (WAITV) blocks until the flag word reaches the step's sequence number,
hipStreamWriteValue32 (SIGNAL) sets it, events (REC / WAIT) order streams of one rank, and
every plan run forks its side streams from the caller's stream and joins them back. A plan
set that can stall on some interleaving shows up as a simulator state in which no stream can
make progress. This covers layouts the one-GPU pool cannot run (8 ranks, relayed hops).
"""
from types import SimpleNamespace as NS

import pytest

from docker_dist_nn_amd.parallel import native_step as nsmod
from docker_dist_nn_amd.parallel.comm import IpcPipe, relay_assignment, relay_parts
from docker_dist_nn_amd.parallel.pipeline import schedule_ops


class FakeTensor:
    def __init__(self, base, rows, cols, esize=2):
        self.base, self.rows, self.cols, self.esize = base, rows, cols, esize

    def __getitem__(self, sl):
        return FakeTensor(self.base + sl.start * self.cols * self.esize, sl.stop - sl.start,
                          self.cols, self.esize)

    def data_ptr(self):
        return self.base

    def numel(self):
        return self.rows * self.cols

    def element_size(self):
        return self.esize

    def stride(self, d):
        return self.cols if d == 0 else 1


def _addr(rank, key):
    keys = ["x_in", "grad_out", "output", "dx_send", "flags"] + [f"relay{i}" for i in range(16)]
    return (rank + 1) << 40 | (keys.index(key) + 1) << 32


def _build_rank(rank, pp, dp, nm, mb, k, width, sched):
    stage, replica = rank % pp, rank // pp
    mesh = NS(rank=rank, pp=pp, dp=dp, stage=stage, replica=replica,
              prev_rank=rank - 1 if stage > 0 else None,
              next_rank=rank + 1 if stage + 1 < pp else None)
    rows = mb * nm
    st = NS(nm=nm, mb=mb, boundary="bf16", _has_w=True, _o_native=True,
            _prog=NS(segments=lambda: {"FINO", "W"}),
            params=NS(sharded=False, grad=FakeTensor(_addr(rank, "output") + (1 << 31), 1, 1, 4),
                      layer_grad_range=lambda i: (i * 4096, (i + 1) * 4096)),
            geoms=[NS(np_=64, kp=64), NS(np_=64, kp=64)],
            x_in=FakeTensor(_addr(rank, "x_in"), rows, width),
            grad_out=FakeTensor(_addr(rank, "grad_out"), rows, width),
            output=FakeTensor(_addr(rank, "output"), rows, width),
            dx_send=FakeTensor(_addr(rank, "dx_send"), rows, width),
            rows_of=lambda j: slice(j * mb, (j + 1) * mb))
    assign = relay_assignment(pp, dp, k) if k else {}
    ipc = NS(k=k, nm=nm, seq=0)
    ipc.duties = [(h[0], h[1], h[2], rl.index(rank) + 1) for h, rl in assign.items()
                  if rank in rl]
    ipc.ackf = 2 * nm * (k + 1)
    ipc.ackb = ipc.ackf + 1
    for f in ("fidx", "bidx", "ridx"):
        setattr(ipc, f, getattr(IpcPipe, f).__get__(ipc))
    ipc.flags = FakeTensor(_addr(rank, "flags"), 1, 1, 4)
    ipc.row_bytes_f = ipc.row_bytes_b = width * 2
    b = relay_parts(0, mb, k)
    ipc.part_max = max(y - x for x, y in zip(b, b[1:]))
    ipc.relay_bufs = [(FakeTensor(_addr(rank, f"relay{d}"), 1, 1, 1), width * 2)
                      for d in range(len(ipc.duties))]

    def peer(r):
        if r is None:
            return None
        return {"x_in": _addr(r, "x_in"), "grad_out": _addr(r, "grad_out"),
                "flags": _addr(r, "flags")}

    ipc.prev, ipc.next = peer(mesh.prev_rank), peer(mesh.next_rank)

    def duty_index(r, hop):
        return [h for h, rl in assign.items() if r in rl].index(hop)

    ipc.relay_out = {"f": [], "b": []}
    for d, pr in (("f", mesh.next_rank), ("b", mesh.prev_rank)):
        if pr is None:
            continue
        for r in assign.get((rank, pr, d), []):
            di = duty_index(r, (rank, pr, d))
            ipc.relay_out[d].append({"buf": _addr(r, f"relay{di}"), "flags": _addr(r, "flags"),
                                     "d": di})
    ipc.relay_dst = [{"buf": _addr(dst, "x_in" if d == "f" else "grad_out"),
                      "flags": _addr(dst, "flags")} for _s, dst, d, _p in ipc.duties]
    ex = NS(stages=[st], ops=[schedule_ops(sched, pp, nm, stage)])
    ns = nsmod.NativeStep.__new__(nsmod.NativeStep)
    ns.ex, ns.mesh, ns.st, ns.transport, ns.ipc = ex, mesh, st, "ipc", ipc
    ns.dp, ns.sharded = dp, False
    ns.comm_f = ns.comm_b = ns.comm_dp = 0
    ns._ev, ns.ops = 0, []
    ns._build()
    return ns.ops, 4 + len(ipc.duties)


def simulate(pp, dp, nm, k, steps=3, sched="1f1b", mb=64, width=64):
    """Runs `steps` plan executions of every rank; returns the number of ops executed or
    raises AssertionError with the blocked stream heads on a deadlock."""
    world = pp * dp
    mem = {}
    queues = {}  # (rank, stream) -> list of (kind, payload, step)
    arrivals = {}  # collective key -> set of ranks whose stream reached it
    for r in range(world):
        ops, ns = _build_rank(r, pp, dp, nm, mb, k, width, sched)
        n_coll = 0
        for o in ops:  # collectives: a barrier over the stage's DP group, in program order
            if o["kind"] == nsmod.ALLREDUCE:
                o["coll"] = n_coll
                n_coll += 1
        for s in range(1, steps + 1):
            queues.setdefault((r, 0), []).append(("FORK", None, s))
            for i in range(1, ns):
                queues.setdefault((r, i), []).append(("WFORK", None, s))
            for o in ops:
                queues.setdefault((r, o["stream"]), []).append(("OP", o, s))
            for i in range(1, ns):
                queues[(r, i)].append(("JREC", i, s))
                queues[(r, 0)].append(("JWAIT", i, s))
    fork, join, ev = {}, {}, {}
    heads = {q: 0 for q in queues}
    done = 0
    while True:
        progress = False
        for (r, si), q in queues.items():
            while heads[(r, si)] < len(q):
                kind, o, s = q[heads[(r, si)]]
                if kind == "FORK":
                    fork[r] = s
                elif kind == "WFORK":
                    if fork.get(r, 0) < s:
                        break
                elif kind == "JREC":
                    join[(r, o)] = s
                elif kind == "JWAIT":
                    if join.get((r, o), 0) < s:
                        break
                else:
                    kd = o["kind"]
                    if kd == nsmod.WAITV:
                        if mem.get(o["a"], 0) < s + o.get("delta", 0):
                            break
                    elif kd == nsmod.SIGNAL:
                        mem[o["a"]] = s + o.get("delta", 0)
                    elif kd == nsmod.REC:
                        ev[(r, o["event"])] = s
                    elif kd == nsmod.WAIT:
                        if ev.get((r, o["event"]), 0) < s:
                            break
                    elif kd == nsmod.ALLREDUCE:
                        key = (r % pp, s, o["coll"])
                        arrivals.setdefault(key, set()).add(r)
                        if len(arrivals[key]) < dp:
                            break
                    # SEG / COPY complete immediately
                heads[(r, si)] += 1
                done += 1
                progress = True
        if all(heads[q] == len(v) for q, v in queues.items()):
            return done
        if not progress:
            blocked = {q: queues[q][heads[q]] for q in queues if heads[q] < len(queues[q])}
            raise AssertionError(f"deadlock: {blocked}")


@pytest.mark.parametrize("pp,dp,k", [(2, 1, 0), (3, 1, 0), (4, 1, 0), (3, 1, 1), (4, 1, 2),
                                     (4, 2, 0), (4, 2, 2), (8, 1, 2), (2, 4, 2), (4, 2, 6)])
def test_ipc_plans_deadlock_free(pp, dp, k):
    assert simulate(pp, dp, nm=2 * pp, k=k) > 0


@pytest.mark.parametrize("sched", ["gpipe", "1f1b"])
def test_ipc_relay_plans_deadlock_free_per_schedule(sched):
    assert simulate(4, 2, nm=8, k=2, sched=sched) > 0


def test_relay_stripes_reach_every_row_once():
    """Every consumer row of every micro-batch is written by exactly one COPY (direct or
    relayed), for every hop of a pp4 x dp2 mesh with 2 relays."""
    pp, dp, nm, mb, k, width = 4, 2, 4, 64, 2, 64
    rb = width * 2
    writes = {}
    for r in range(pp * dp):
        ops, _ = _build_rank(r, pp, dp, nm, mb, k, width, "1f1b")
        for o in ops:
            if o["kind"] == nsmod.COPY and (o["b"] >> 32) & 0xff in (1, 2):  # x_in / grad_out
                for row in range(o["count"] // rb):
                    key = (o["b"] >> 32, (o["b"] & 0xffffffff) // rb + row)
                    writes[key] = writes.get(key, 0) + 1
    assert set(writes.values()) == {1}
    # (pp - 1) boundaries x 2 directions x dp replicas x all rows
    assert len(writes) == (pp - 1) * 2 * dp * nm * mb
