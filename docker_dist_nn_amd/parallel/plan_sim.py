"""Timed discrete-event simulator of multi-rank StepPlans (parallel/native_step.py).

Every rank's plan is the op list ``NativeStep._build`` produces (the exact list a GPU run
enqueues); the simulator executes all ranks' lists with the semantics the GPU runtime and RCCL
give them, and a duration per op:

* streams: FIFO per (rank, stream); each plan run forks its side streams from stream 0 and
  joins them back (``StepPlan::run``); REC / WAIT are event edges between a rank's streams;
* RCCL point-to-point: SEND and RECV are blocking rendezvous per (communicator, src, dst)
  channel, matched in FIFO order; a transfer starts when both sides have posted it and takes
  ``p2p_time(op)``;
* GROUP (``ncclGroupStart/End``): its SEND / RECV members progress concurrently; the group is
  one kernel and retires when its last member has;
* collectives (ALLREDUCE / REDUCE_SCATTER / ALL_GATHER): a barrier over every rank that uses
  the communicator, matched in program order per communicator;
* IPC hops: SIGNAL sets a flag word to the step number (+ delta), WAITV blocks until it is
  reached, COPY is a kernel;
* ``serial_rccl=True``: at most ONE RCCL kernel (op or group) per rank is resident at a time
  -- the strictest co-residency assumption: a posted RCCL op holds the rank's RCCL slot until
  it retires, and a RCCL op at the head of another stream waits for the slot (granted in the
  order the ops became ready). A plan that only works when several RCCL kernels of a rank run
  concurrently deadlocks here.

``simulate`` returns per-rank finish times and per-op timings, or raises :class:`Deadlock`
with the blocked stream heads. The tests (tests/test_step_plan_sim_cpu.py) check deadlock
freedom of every BASELINE layout and the steady-state period of the pipelines.
"""
from __future__ import annotations

import heapq
import itertools
from dataclasses import dataclass, field
from typing import Callable, Optional

from .native_step import (ALL_GATHER, ALLREDUCE, COPY, GROUP, RECV, REC, REDUCE_SCATTER, SEG,
                          SEND, SIGNAL, WAIT, WAITV)

RCCL_KINDS = (SEND, RECV, ALLREDUCE, REDUCE_SCATTER, ALL_GATHER, GROUP)
COLL_KINDS = (ALLREDUCE, REDUCE_SCATTER, ALL_GATHER)
KIND_NAMES = {SEG: "SEG", SEND: "SEND", RECV: "RECV", ALLREDUCE: "ALLREDUCE",
              REDUCE_SCATTER: "REDUCE_SCATTER", ALL_GATHER: "ALL_GATHER", COPY: "COPY",
              SIGNAL: "SIGNAL", WAITV: "WAITV", REC: "REC", WAIT: "WAIT", GROUP: "GROUP"}


class Deadlock(AssertionError):
    pass


@dataclass
class RankPlan:
    ops: list
    n_streams: int


@dataclass
class Result:
    finish: dict                      # rank -> time its last stream retired its last op
    step_end: dict                    # (rank, step) -> time the step's join completed
    seg_times: dict = field(default_factory=dict)   # (rank, step, seg) -> (start, end)
    xfer_times: list = field(default_factory=list)  # (src, dst, start, end, step)

    @property
    def makespan(self) -> float:
        return max(self.finish.values()) if self.finish else 0.0


def _default_seg(rank, seg):
    return 1.0


def _default_p2p(op):
    return 1.0


def _default_coll(op):
    return 1.0


def simulate(plans: dict, steps: int = 2, *, seg_time: Callable = _default_seg,
             p2p_time: Callable = _default_p2p, coll_time: Callable = _default_coll,
             copy_time: Optional[Callable] = None, serial_rccl: bool = False) -> Result:
    """plans: rank -> RankPlan. Runs ``steps`` executions of every plan."""
    copy_time = copy_time or (lambda op: 0.0)
    # per (rank, stream) program: ("FORK"|"WFORK"|"JREC"|"JWAIT"|"OP", payload, step)
    prog = {}
    for r, rp in plans.items():
        for s in range(1, steps + 1):
            prog.setdefault((r, 0), []).append(("FORK", None, s))
            for i in range(1, rp.n_streams):
                prog.setdefault((r, i), []).append(("WFORK", None, s))
            for o in rp.ops:
                prog.setdefault((r, o["stream"]), []).append(("OP", o, s))
            for i in range(1, rp.n_streams):
                prog[(r, i)].append(("JREC", i, s))
                prog[(r, 0)].append(("JWAIT", i, s))
            prog[(r, 0)].append(("END", None, s))
    # collective members: every rank whose plan uses the communicator
    members = {}
    for r, rp in plans.items():
        for o in rp.ops:
            for m in ([o] + list(o.get("ops", []))):
                if m["kind"] in COLL_KINDS:
                    members.setdefault(m["comm"], set()).add(r)

    head = {q: 0 for q in prog}
    ready_t = {q: 0.0 for q in prog}
    fork, joinrec, events, flags = {}, {}, {}, {}
    waiters: dict = {}          # key -> list of queues blocked on it
    chan_posts: dict = {}       # (comm, src, dst) -> [ (kind, rank, time, token) ] unmatched
    coll_seq: dict = {}         # (rank, comm) -> collectives issued so far
    coll_arr: dict = {}         # (comm, idx, step) -> {rank: (time, token)}
    pending: dict = {}          # token -> [remaining members, max end, queue]
    rccl_busy: dict = {}        # rank -> token holding the RCCL slot
    rccl_wait: dict = {}        # rank -> heap of (time, seq, queue)
    posted = set()              # queues whose head RCCL op is posted (waiting for partners)
    res = Result({}, {})
    heap: list = []
    seq = itertools.count()
    tokens = itertools.count()

    def push(t, q):
        heapq.heappush(heap, (t, next(seq), q))

    def block(key, q):
        waiters.setdefault(key, []).append(q)

    def wake(key, t):
        for q in waiters.pop(key, []):
            push(max(t, ready_t[q]), q)

    def advance(q, t):
        head[q] += 1
        ready_t[q] = t
        push(t, q)

    def retire_member(tok, t_end):
        ent = pending[tok]
        ent[0] -= 1
        ent[1] = max(ent[1], t_end)
        if ent[0] == 0:
            q = ent[2]
            r = q[0]
            del pending[tok]
            posted.discard(q)
            if rccl_busy.get(r) == tok:
                del rccl_busy[r]
                if rccl_wait.get(r):
                    tw, _, qw = heapq.heappop(rccl_wait[r])
                    push(max(tw, ent[1]), qw)
            advance(q, ent[1])

    def post_p2p(m, r, t, tok, step):
        if m["kind"] == SEND:
            key, other = (m["comm"], r, m["gpeer"]), RECV
        else:
            key, other = (m["comm"], m["gpeer"], r), SEND
        lst = chan_posts.setdefault(key, [])
        # FIFO: the oldest unmatched post of the opposite kind matches
        for i, (k2, r2, t2, tok2, m2) in enumerate(lst):
            if k2 == other:
                del lst[i]
                start = max(t, t2)
                end = start + p2p_time(m if m["kind"] == SEND else m2)
                src = r if m["kind"] == SEND else r2
                dst = r2 if m["kind"] == SEND else r
                res.xfer_times.append((src, dst, start, end, step))
                retire_member(tok, end)
                retire_member(tok2, end)
                return
            break  # the oldest post has the same kind: queue behind it
        lst.append((m["kind"], r, t, tok, m))

    def post_coll(m, r, t, tok, step):
        idx = coll_seq.get((r, m["comm"]), 0)
        coll_seq[(r, m["comm"])] = idx + 1
        key = (m["comm"], idx, step)
        arr = coll_arr.setdefault(key, {})
        arr[r] = (t, tok)
        if len(arr) == len(members[m["comm"]]):
            end = max(v[0] for v in arr.values()) + coll_time(m)
            for _, (_, tk) in arr.items():
                retire_member(tk, end)
            del coll_arr[key]

    def post_rccl(o, q, t, step):
        r = q[0]
        mem = o["ops"] if o["kind"] == GROUP else [o]
        tok = next(tokens)
        pending[tok] = [len(mem), t, q]
        if serial_rccl:
            rccl_busy[r] = tok
        for m in mem:
            if m["kind"] in (SEND, RECV):
                post_p2p(m, r, t, tok, step)
            else:
                post_coll(m, r, t, tok, step)

    for q in prog:
        push(0.0, q)
    while heap:
        t, _, q = heapq.heappop(heap)
        t = max(t, ready_t[q])
        if head[q] >= len(prog[q]) or q in posted:
            continue
        r, si = q
        kind, o, s = prog[q][head[q]]
        if kind == "FORK":
            fork[r] = (s, t)
            wake(("fork", r, s), t)
            advance(q, t)
        elif kind == "WFORK":
            f = fork.get(r)
            if f is None or f[0] < s:
                block(("fork", r, s), q)
                continue
            advance(q, max(t, f[1]))
        elif kind == "JREC":
            joinrec[(r, o, s)] = t
            wake(("join", r, o, s), t)
            advance(q, t)
        elif kind == "JWAIT":
            tj = joinrec.get((r, o, s))
            if tj is None:
                block(("join", r, o, s), q)
                continue
            advance(q, max(t, tj))
        elif kind == "END":
            res.step_end[(r, s)] = t
            advance(q, t)
        else:
            k = o["kind"]
            if k == SEG:
                d = seg_time(r, o["seg"])
                res.seg_times[(r, s, o["seg"])] = (t, t + d)
                advance(q, t + d)
            elif k == COPY:
                advance(q, t + copy_time(o))
            elif k == REC:
                events[(r, o["event"])] = (s, t)
                wake(("ev", r, o["event"], s), t)
                advance(q, t)
            elif k == WAIT:
                e = events.get((r, o["event"]))
                if e is None or e[0] < s:
                    block(("ev", r, o["event"], s), q)
                    continue
                advance(q, max(t, e[1]))
            elif k == SIGNAL:
                v = s + o.get("delta", 0)
                flags[o["a"]] = (v, t)
                wake(("flag", o["a"]), t)
                advance(q, t)
            elif k == WAITV:
                f = flags.get(o["a"], (0, 0.0))  # flag words start at 0
                if f[0] < s + o.get("delta", 0):
                    block(("flag", o["a"]), q)
                    continue
                advance(q, max(t, f[1]))
            elif k in RCCL_KINDS:
                if serial_rccl and r in rccl_busy:
                    heapq.heappush(rccl_wait.setdefault(r, []), (t, next(seq), q))
                    continue
                posted.add(q)
                post_rccl(o, q, t, s)
            else:
                raise ValueError(f"unknown op kind {k}")
    undone = {q: prog[q][head[q]] for q in prog if head[q] < len(prog[q])}
    if undone:
        def show(v):
            kind, o, s = v
            if kind != "OP":
                return (kind, s)
            return (KIND_NAMES[o["kind"]], s, o.get("seg") or o.get("tag") or o.get("peer"))
        raise Deadlock("deadlock: " + ", ".join(f"r{q[0]}/s{q[1]}: {show(v)}"
                                                for q, v in sorted(undone.items())))
    for q in prog:
        res.finish[q[0]] = max(res.finish.get(q[0], 0.0), ready_t[q])
    return res

