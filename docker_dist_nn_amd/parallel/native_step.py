"""Native multi-rank training step: the whole step of a rank as ONE C++ call.

The Python executor (pipeline.PipelineExecutor._run_op) walks the schedule op by op and issues
every pipeline hop and DP bucket through torch.distributed. For a rank that owns one stage this
module instead compiles the SAME schedule once into a ``StepPlan`` (csrc/runtime/step_plan.hpp)
of recorded-segment replays, RCCL calls on communicators torch created (or xGMI peer copies +
stream flags), and event edges between streams.

RCCL hops, two plan forms (``DNN_RCCL_PLAN``; both checked by the timed plan simulator,
parallel/plan_sim.py, and by the gloo plan interpreter, parallel/plan_interp.py):

* ``streams`` (default): one channel per hop direction and link. Every link of a pipeline has
  two private 2-rank communicators (forward, backward: groups.Mesh.link_*), and a rank drives
  each of its (up to four) channels on a stream of its own:

      stream 0  compute: F{j}, B{j}, W, FIN*, O / FINO segments
      stream 1  forward sends   (F(j) -> next stage, after F{j})
      stream 2  backward sends  (B(j) -> previous stage, after B{j})
      stream 3  data-parallel buckets
      stream 4  forward receives: every receive of the step posted at step start
      stream 5  backward receives: likewise

  A channel has exactly one sender and one receiver and carries its micro-batches in FIFO
  order, so the hop-in of micro-batch j+1 runs while j is computed and while j's hop-out
  drains: a micro-batch costs max(compute, hop in, hop out) in steady state
  (planner.Planner). It needs every stream on its own hardware queue (checked) and the
  channels' RCCL kernels co-resident (each is a few workgroups; nothing else spins).
* ``slotted``: safe even if at most ONE RCCL kernel of a rank is resident at a time. All RCCL
  work of a rank is on ONE stream: the replica's pipeline is laid out on a global logical
  clock (every compute op at the earliest time its inputs allow, one clock slot per hop), and
  at slot t every rank issues one ncclGroupStart/End holding all transfers of slot t -- whose
  partners are in the partner's slot-t group by construction -- then the DP collectives in
  one fixed order. Group t of every rank can complete once all groups < t have, whatever the
  kernel residency, at the price of hop-ins that wait for the previous hop-outs.

``auto`` picks ``streams`` when GPU_MAX_HW_QUEUES gives each of its streams a queue, else
``slotted`` (2 streams). DP buckets (pipeline.dp_buckets: largest layer first) are reduced
while the remaining weight-gradient GEMMs run, then the update waits for them.

Per step the host does: lr scalar refresh, one ``StepPlan.run``. No Python per hop, no host
synchronisation, and the plan forks/joins its streams from the caller's stream, so the whole
step can be captured into a HIP graph.

Reference: the stage chain /root/reference/src/grpc_node.py:120-135 (one synchronous RPC per
hop) and its spawn/topology /root/reference/src/run_grpc_fcnn.py:199-248.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from ..utils.native import native
from .. import switches
from .comm import relay_parts
from .pipeline import dp_buckets, schedule_ops

(SEG, SEND, RECV, ALLREDUCE, REDUCE_SCATTER, ALL_GATHER, COPY, SIGNAL, WAITV, REC, WAIT,
 GSTART, GEND) = range(13)
GROUP = 100  # plan-builder only: {"ops": [SEND / RECV ...]} -> GSTART, members, GEND
NCCL_BF16, NCCL_F32, NCCL_U8 = 9, 7, 1
MAIN, FWD, BWD, DPS, FRECV, BRECV = 0, 1, 2, 3, 4, 5
COMM = 1  # slotted plans: the rank's one RCCL stream
# keys StepPlan.add accepts (the op dicts also carry simulator-only keys: gpeer, tag)
PLAN_KEYS = ("kind", "stream", "prog", "seg", "comm", "a", "b", "count", "dtype", "peer",
             "delta", "event")
ESIZE = {NCCL_BF16: 2, NCCL_F32: 4, NCCL_U8: 1}


def torch_rccl_path() -> str:
    """The librccl torch loaded (its communicators live in that instance)."""
    return os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")


def comm_ptr(group, device) -> int:
    """ncclComm_t of a torch process group (created eagerly by a collective if needed)."""
    be = group._get_backend(device)
    p = int(be._comm_ptr())
    if not p:
        raise RuntimeError("process group has no RCCL communicator yet")
    return p


class NativeStep:
    """Builds and runs the StepPlan of one rank. ``transport``: "rccl" (RCCL P2P on the link
    communicators) or "ipc" (an IpcPipe's mapped peer buffers and flags).

    ``comms`` (tests: plan simulator / gloo interpreter): name -> communicator handle for
    "f_in" / "f_out" / "b_in" / "b_out" (the link channels) and "dp", instead of the RCCL
    communicators of the mesh's process groups; with ``build_only`` no StepPlan is created
    (``self.ops`` is the op list a GPU run would enqueue)."""

    def __init__(self, executor, mesh, transport: str, ipc=None, comms: Optional[dict] = None,
                 mode: Optional[str] = None, build_only: bool = False):
        if len(executor.stages) != 1:
            raise ValueError("native multi-rank step: one stage per rank")
        st = executor.stages[0]
        if st._prog is None or not st._has_w or not st._o_native:
            raise ValueError("native multi-rank step needs a recorded stage (compile_native)")
        self.ex, self.mesh, self.st = executor, mesh, st
        self.transport = transport
        self.ipc = ipc
        self.dp = mesh.dp if mesh is not None else 1
        self.sharded = st.params.sharded
        self.pp = mesh.pp if mesh is not None else 1
        hwq = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
        mode = mode or switches.get("DNN_RCCL_PLAN" if transport == "rccl" else "DNN_IPC_PLAN")
        if mode == "auto":
            mode = "streams" if hwq >= 6 else "slotted"
        if mode not in ("streams", "slotted"):
            raise ValueError(f"plan form must be auto | streams | slotted, got {mode!r}")
        # "ipc": one stream per direction and relay duty; "ipc-slotted": everything on ONE
        # stream in global logical-clock order (_build_ipc_slotted)
        self.mode = mode if transport == "rccl" else ("ipc-slotted" if mode == "slotted"
                                                      else "ipc")
        self.comms = dict(comms or {})
        if comms is None and not build_only:
            self.n = native()
            dev = st.device
            if transport == "rccl" or self.dp > 1 or self.sharded:
                self.n.nccl_load(torch_rccl_path())
            if transport == "rccl" and self.pp > 1:
                for name in ("f_in", "f_out", "b_in", "b_out"):
                    g = getattr(mesh, "link_" + name)
                    if g is not None:
                        self.comms[name] = comm_ptr(g, dev)
            if self.dp > 1 or self.sharded:
                self.comms["dp"] = comm_ptr(mesh.dp_group, dev)
            self._check_comm_ranks()
        self._ev = 0
        self.ops: list[dict] = []
        self._build()
        if self.mode == "ipc-slotted":
            self.n_streams = 1
        elif self.transport == "ipc":
            self.n_streams = 4 + (len(ipc.duties) if ipc is not None else 0)
        else:
            self.n_streams = 6 if self.mode == "streams" else 2
        if build_only:
            return
        # streams of a plan block on flags / peers: each needs its own hardware queue (HIP maps
        # streams beyond GPU_MAX_HW_QUEUES onto shared queues, where one blocked wait stalls
        # the streams behind it -- a cross-rank deadlock); stream 0 is the caller's
        if self.n_streams > hwq:
            raise RuntimeError(f"native step needs {self.n_streams} hardware queues, "
                               f"GPU_MAX_HW_QUEUES={hwq}: set it (before the GPU is "
                               f"initialised) to >= {self.n_streams}")
        self.n = native()
        self.plan = self.n.StepPlan(self.n_streams, max(1, self._ev))
        for o in flatten(self.ops):
            self.plan.add(**{k: v for k, v in o.items() if k in PLAN_KEYS})

    # ---- communicators ---------------------------------------------------------------------
    def _link_peer(self, other_rank: int) -> int:
        """Rank of ``other_rank`` inside a 2-rank link communicator (group ranks follow the
        global rank order: the lower rank is 0)."""
        return 0 if other_rank < self.mesh.rank else 1

    def _check_comm_ranks(self) -> None:
        """The offsets of the plan assume comm rank == position in the group: 0/1 on a link
        (lower global rank first), the replica index on the DP communicator."""
        n, m = self.n, self.mesh
        for name, comm in self.comms.items():
            size, rank = n.nccl_comm_info(comm)
            want = (self.dp, m.replica) if name == "dp" else \
                (2, 0 if name in ("f_out", "b_in") else 1)
            if (size, rank) != want:
                raise RuntimeError(f"communicator {name}: (size, rank) = {(size, rank)}, "
                                   f"the plan assumes {want}")

    # ---- plan construction -------------------------------------------------------------
    def _event(self) -> int:
        self._ev += 1
        return self._ev - 1

    def _edge(self, src: int, dst: int) -> None:
        """Stream ``dst`` waits for everything enqueued on ``src`` so far."""
        e = self._event()
        self.ops.append(dict(kind=REC, stream=src, event=e))
        self.ops.append(dict(kind=WAIT, stream=dst, event=e))

    def _seg(self, name: str, stream: int = MAIN) -> None:
        self.ops.append(dict(kind=SEG, stream=stream, prog=self.st._prog, seg=name))

    def _rows(self, t: torch.Tensor, j: int) -> tuple[int, int]:
        r = self.st.rows_of(j)
        v = t[r]
        return v.data_ptr(), v.numel()

    def _hop_bufs(self, direction: str, inbound: bool):
        """(tensor, dtype) pieces of one hop message: bf16 rows, or (fp8 boundary) e4m3 rows
        then their fp32 row scales -- the same order on both sides."""
        st = self.st
        if st.boundary == "fp8":
            if inbound:
                q, sc = (st.q_in, st.s_in) if direction == "f" else (st.q_gin, st.s_gin)
            else:
                q, sc = (st.q_out, st.s_out) if direction == "f" else (st.q_dx, st.s_dx)
            return [(q, NCCL_U8), (sc, NCCL_F32)]
        if inbound:
            return [(st.x_in if direction == "f" else st.grad_out, NCCL_BF16)]
        return [(st.output if direction == "f" else st.dx_send, NCCL_BF16)]

    def _p2p(self, kind: int, direction: str, j: int, stream: int) -> list[dict]:
        """The RCCL op(s) of micro-batch j's hop in ``direction`` ("f"/"b"); kind SEND (my
        output to the neighbour) or RECV (the neighbour's output into my buffer)."""
        m = self.mesh
        inbound = kind == RECV
        if direction == "f":
            other = m.prev_rank if inbound else m.next_rank
            name = "f_in" if inbound else "f_out"
        else:
            other = m.next_rank if inbound else m.prev_rank
            name = "b_in" if inbound else "b_out"
        out = []
        for part, (t, dt) in enumerate(self._hop_bufs(direction, inbound)):
            ptr, cnt = self._rows(t, j)
            out.append(dict(kind=kind, stream=stream, comm=self.comms.get(name, 0), a=ptr,
                            count=cnt, dtype=dt, peer=self._link_peer(other), gpeer=other,
                            tag=(direction, j, part)))
        return out

    def _peer_order(self, stage: int, op_kind: str) -> list[int]:
        """Micro-batches in the order stage ``stage`` executes its ``op_kind`` ops (= the order
        it sends that direction's messages)."""
        return [j for op, j in schedule_ops(self.ex.kind, self.pp, self.st.nm, stage)
                if op == op_kind]

    def _recv_ipc(self, direction: str, j: int) -> None:
        """The producer's copies + flags: wait on the compute stream."""
        p = self.ipc
        base = p.flags.data_ptr()
        for part in range(p.k_in[direction] + 1):  # the direct stripe and every relayed one
            idx = p.fidx(j, part) if direction == "f" else p.bidx(j, part)
            self.ops.append(dict(kind=WAITV, stream=MAIN, a=base + 4 * idx, delta=0))

    def _send_ipc(self, direction: str, j: int, stream: Optional[int] = None) -> None:
        """``stream`` None: the direction's send stream, ordered after the compute so far;
        else that stream as it is (the slotted form: everything on MAIN)."""
        st = self.st
        t = st.output if direction == "f" else st.dx_send
        if stream is None:
            s = FWD if direction == "f" else BWD
            self._edge(MAIN, s)
        else:
            s = stream
        ptr, cnt = self._rows(t, j)
        p = self.ipc
        peer = p.next if direction == "f" else p.prev
        if j == 0:  # the peer finished reading that buffer in the previous step (ack)
            ack = p.ackf if direction == "f" else p.ackb
            self.ops.append(dict(kind=WAITV, stream=s, a=p.flags.data_ptr() + 4 * ack,
                                 delta=-1))
        dst_base = peer["x_in"] if direction == "f" else peer["grad_out"]
        row_bytes = p.row_bytes_f if direction == "f" else p.row_bytes_b
        r = st.rows_of(j)
        k = p.k_out[direction]  # this hop's relays (per hop: comm.relay_plan)
        bounds = relay_parts(r.start, r.stop, k)
        for part in range(k + 1):  # stripe 0 direct, stripe q via relay q - 1
            a0, a1 = bounds[part], bounds[part + 1]
            src = ptr + (a0 - r.start) * row_bytes
            if part == 0:
                self.ops.append(dict(kind=COPY, stream=s, a=src, b=dst_base + a0 * row_bytes,
                                     count=(a1 - a0) * row_bytes))
                idx = p.fidx(j, 0) if direction == "f" else p.bidx(j, 0)
                self.ops.append(dict(kind=SIGNAL, stream=s, a=peer["flags"] + 4 * idx,
                                     delta=0))
            else:
                rel = p.relay_out[direction][part - 1]
                slot = rel["buf"] + j * rel["part_max"] * row_bytes
                self.ops.append(dict(kind=COPY, stream=s, a=src, b=slot,
                                     count=(a1 - a0) * row_bytes))
                self.ops.append(dict(kind=SIGNAL, stream=s,
                                     a=rel["flags"] + 4 * p.ridx(rel["d"], j), delta=0))

    def _wgrad_update(self, dps: int) -> None:
        st = self.st
        segs = st._prog.segments()
        if self.dp <= 1 and not self.sharded:
            self._seg("W")
            if "FINO" in segs:
                self._seg("FINO")
            else:
                self._seg("FIN")
                self._seg("O")
            return
        p = st.params
        if self.sharded:
            self._sharded_update(dps)
            return
        for bucket in dp_buckets(st):
            for i in bucket:
                self._seg(f"W{i}")
            a, b = bucket[0], bucket[-1]
            self._seg(f"FIN{a}" if a == b else f"FIN{a}-{b}")
            e0, _ = p.layer_grad_range(a)
            _, e1 = p.layer_grad_range(b)
            self._edge(MAIN, dps)
            self.ops.append(dict(kind=ALLREDUCE, stream=dps, comm=self.comms.get("dp", 0),
                                 a=p.grad.data_ptr() + 4 * e0, count=e1 - e0, dtype=NCCL_F32))
        self._edge(dps, MAIN)
        self._seg("O")

    def _sharded_update(self, dps: int) -> None:
        """Sharded DP (pipeline.GradSync shard): per bucket, W segments -> FIN -> bf16 pack on
        the compute stream, then the bucket's bf16 reduce-scatter on the DP stream (overlapping
        the next bucket's wgrads). Per bucket again: unpack + update of this rank's piece, then
        the bf16 all-gather of the piece's shadow weights; the W^T refresh waits for all.
        Offsets: replica r's piece of bucket [e0, e1) is grad_piece[e0/d : e1/d] (every weight
        is padded to d equal aligned pieces, StageParams.shard_piece)."""
        st = self.st
        p = st.params
        dpc = self.comms.get("dp", 0)
        buckets = []
        for bucket in dp_buckets(st):
            a, b = bucket[0], bucket[-1]
            e0, _ = p.layer_grad_range(a)
            _, e1 = p.layer_grad_range(b)
            buckets.append((a, b, e0, e1))
        p.shard_buckets = [(e0, e1) for _, _, e0, e1 in buckets]
        d = p.dp
        for (a, b, e0, e1), bucket in zip(buckets, dp_buckets(st)):
            for i in bucket:
                self._seg(f"W{i}")
            self._seg(f"FIN{a}" if a == b else f"FIN{a}-{b}")
            self._seg(f"SP{a}-{b}")
            self._edge(MAIN, dps)
            self.ops.append(dict(kind=REDUCE_SCATTER, stream=dps, comm=dpc,
                                 a=p.grad16.data_ptr() + 2 * e0,
                                 b=p.grad_piece.data_ptr() + 2 * (e0 // d),
                                 count=(e1 - e0) // d, dtype=NCCL_BF16))
        # every bias gradient (fp32, a few KB): all-reduced, then updated on every rank
        self.ops.append(dict(kind=ALLREDUCE, stream=dps, comm=dpc,
                             a=p.grad.data_ptr() + 4 * p.bias_lo, count=p.numel - p.bias_lo,
                             dtype=NCCL_F32))
        self._edge(dps, MAIN)
        self._seg("SB")
        for a, b, e0, e1 in buckets:
            self._seg(f"SU{a}-{b}")
            self._edge(MAIN, dps)
            p0, _ = p.shard_piece(e0, e1)
            self.ops.append(dict(kind=ALL_GATHER, stream=dps, comm=dpc,
                                 a=p.shadow.data_ptr() + 2 * p0, b=p.shadow.data_ptr() + 2 * e0,
                                 count=(e1 - e0) // d, dtype=NCCL_BF16))
        if p.optim.name != "sgd":
            self._seg("OADV")
        self._edge(dps, MAIN)
        self._seg("T")

    def _check_w(self, ops) -> None:
        for k, (op, j) in enumerate(ops):
            nxt = ops[k + 1][0] if k + 1 < len(ops) else None
            if op == "W" and (j >= 0 or nxt != "O"):
                raise ValueError("native multi-rank step: batched W followed by O only")

    def _build(self) -> None:
        self._check_w(self.ex.ops[0])
        if self.mode == "ipc-slotted":
            self._build_ipc_slotted()
        elif self.transport == "ipc":
            self._build_ipc()
        elif self.mode == "slotted":
            self._build_slotted()
        else:
            self._build_streams()

    def _build_ipc(self) -> None:
        m = self.mesh
        has_prev = m is not None and m.prev_rank is not None
        has_next = m is not None and m.next_rank is not None
        for op, j in self.ex.ops[0]:
            if op == "F":
                if has_prev:
                    self._recv_ipc("f", j)
                self._seg(f"F{j}")
                if has_next:
                    self._send_ipc("f", j)
            elif op == "B":
                if has_next:
                    self._recv_ipc("b", j)
                self._seg(f"B{j}")
                if has_prev:
                    self._send_ipc("b", j)
            elif op == "W":
                self._wgrad_update(DPS)
        self._release_acks()
        self._relay_duties()

    def _release_acks(self) -> None:
        p = self.ipc  # release the buffers I receive into for the next step
        if p.prev is not None:
            self.ops.append(dict(kind=SIGNAL, stream=MAIN, a=p.prev["flags"] + 4 * p.ackf,
                                 delta=0))
        if p.next is not None:
            self.ops.append(dict(kind=SIGNAL, stream=MAIN, a=p.next["flags"] + 4 * p.ackb,
                                 delta=0))

    def _collect(self, fn, *args) -> list[dict]:
        """The ops ``fn(*args)`` would append, returned instead of appended."""
        saved, self.ops = self.ops, []
        try:
            fn(*args)
            return self.ops
        finally:
            self.ops = saved

    def _build_ipc_slotted(self) -> None:
        """IPC hops on ONE stream, in the replica's global logical-clock order (logical_times:
        the clock the slotted RCCL form uses; every replica runs the same clock). At slot t a
        rank enqueues, in this order: (0) its sends of slot t (copy + flag per stripe), (1)
        its relay duties of slot t (wait for the stripe, copy it on, raise the consumer's
        flag), (2) its receive waits of slot t, (3) its compute of slot t. A wait of slot t is
        released only by sends / relays of slot t, which every rank enqueues before its own
        waits of slot t, and sends wait on nothing but the previous step's acks -- so the
        plan completes whatever order an executor runs independent work in, and a captured
        graph of it is a single chain (the multi-stream relayed plan stalled
        when captured). The price: copies and relays serialise with this rank's compute."""
        m, st, p = self.mesh, self.st, self.ipc
        kind, pp, nm = self.ex.kind, self.pp, st.nm
        T = logical_times(kind, pp, nm)
        my_t = T[m.stage]
        has_prev, has_next = m.prev_rank is not None, m.next_rank is not None
        entries = []  # (slot, order, ops)

        def msg_slots(src_stage: int, opname: str):
            """(slot, j) of every message stage ``src_stage`` sends after its ``opname``."""
            for k, (op, j) in enumerate(schedule_ops(kind, pp, nm, src_stage)):
                if op == opname:
                    yield T[src_stage][k] + 1, j

        for idx, (op, j) in enumerate(self.ex.ops[0]):
            if op not in ("F", "B"):
                continue
            d = op.lower()
            entries.append((my_t[idx], 3, [dict(kind=SEG, stream=MAIN, prog=st._prog,
                                                seg=f"{op}{j}")]))
            if (d == "f" and has_next) or (d == "b" and has_prev):
                entries.append((my_t[idx] + 1, 0, self._collect(self._send_ipc, d, j, MAIN)))
        for d, has, src, opname in (("f", has_prev, m.stage - 1, "F"),
                                    ("b", has_next, m.stage + 1, "B")):
            if has:
                for t, j in msg_slots(src, opname):
                    entries.append((t, 2, self._collect(self._recv_ipc, d, j)))
        for dd, (src, _dst, direction, _part) in enumerate(p.duties):
            for t, j in msg_slots(src % pp, "F" if direction == "f" else "B"):
                entries.append((t, 1, self._relay_op(dd, j, MAIN)))
        for _, _, ops in sorted(entries, key=lambda e: (e[0], e[1])):
            self.ops += ops
        self._wgrad_update(MAIN)
        self._release_acks()

    def _build_streams(self) -> None:
        """One stream per hop channel; every receive of the step posted at its start (the rows
        of every micro-batch have their own buffer slice, and the previous step's readers of
        them all precede the plan's fork)."""
        m, st = self.mesh, self.st
        fp8 = st.boundary == "fp8"
        has_prev, has_next = m.prev_rank is not None, m.next_rank is not None
        ev_in = {}
        for direction, has, stream, src in (("f", has_prev, FRECV, m.stage - 1),
                                            ("b", has_next, BRECV, m.stage + 1)):
            if not has:
                continue
            for j in self._peer_order(src, "F" if direction == "f" else "B"):
                self.ops += self._p2p(RECV, direction, j, stream)
                ev_in[(direction, j)] = e = self._event()
                self.ops.append(dict(kind=REC, stream=stream, event=e))
        for op, j in self.ex.ops[0]:
            if op in ("F", "B"):
                d = op.lower()
                if (d == "f" and has_prev) or (d == "b" and has_next):
                    self.ops.append(dict(kind=WAIT, stream=MAIN, event=ev_in[(d, j)]))
                    if fp8:
                        self._seg(f"DQF{j}" if d == "f" else f"DQB{j}")
                self._seg(f"{op}{j}")
                if (d == "f" and has_next) or (d == "b" and has_prev):
                    if fp8:
                        self._seg(f"QF{j}" if d == "f" else f"QB{j}")
                    s = FWD if d == "f" else BWD
                    self._edge(MAIN, s)
                    self.ops += self._p2p(SEND, d, j, s)
            elif op == "W":
                self._wgrad_update(DPS)

    def _build_slotted(self) -> None:
        """All RCCL work on ONE stream, grouped per slot of the replica's logical clock (see
        the module docstring); the DP collectives follow in bucket order. Host enqueue order
        follows the clock too -- group t after the compute at t-1 whose output it sends, the
        compute at t after the groups holding its inputs -- so every WAIT is enqueued after
        the REC it names (an event wait binds to the last record enqueued before it)."""
        m, st = self.mesh, self.st
        fp8 = st.boundary == "fp8"
        sends, recvs = slot_messages(self.ex.kind, self.pp, st.nm, m.stage)
        my_t = logical_times(self.ex.kind, self.pp, st.nm)[m.stage]
        has_prev, has_next = m.prev_rank is not None, m.next_rank is not None
        produced_at, consumed = {}, {}
        group_ev = {}
        for t in sorted(recvs):
            group_ev[t] = self._event()
            for msg in recvs[t]:
                consumed[msg] = group_ev[t]
        entries = []  # (time, 0 = comm group / 1 = compute, ops)
        for idx, (op, j) in enumerate(self.ex.ops[0]):
            if op not in ("F", "B"):
                continue
            d, ops = op.lower(), []
            if (d, j) in consumed:
                ops.append(dict(kind=WAIT, stream=MAIN, event=consumed[(d, j)]))
                if fp8:
                    ops.append(dict(kind=SEG, stream=MAIN, prog=st._prog,
                                    seg=f"DQF{j}" if d == "f" else f"DQB{j}"))
            ops.append(dict(kind=SEG, stream=MAIN, prog=st._prog, seg=f"{op}{j}"))
            if (d == "f" and has_next) or (d == "b" and has_prev):
                if fp8:
                    ops.append(dict(kind=SEG, stream=MAIN, prog=st._prog,
                                    seg=f"QF{j}" if d == "f" else f"QB{j}"))
                produced_at[(d, j)] = e = self._event()
                ops.append(dict(kind=REC, stream=MAIN, event=e))
            entries.append((my_t[idx], 1, ops))
        for t in sorted(set(sends) | set(recvs)):
            ops, members = [], []
            for d, j in sends.get(t, []):
                ops.append(dict(kind=WAIT, stream=COMM, event=produced_at[(d, j)]))
                members += self._p2p(SEND, d, j, COMM)
            for d, j in recvs.get(t, []):
                members += self._p2p(RECV, d, j, COMM)
            ops.append(dict(kind=GROUP, stream=COMM, ops=members, tag=("slot", t)))
            if t in group_ev:
                ops.append(dict(kind=REC, stream=COMM, event=group_ev[t]))
            entries.append((t, 0, ops))
        for _, _, ops in sorted(entries, key=lambda e: (e[0], e[1])):
            self.ops += ops
        self._wgrad_update(COMM)

    def _relay_duties(self) -> None:
        """My relay work for other ranks' hops, one stream per duty (a duty's stripes arrive
        in micro-batch order, and separate streams keep one hop from blocking another):
        wait for the producer's stripe j in my slot -> copy it into the consumer's rows ->
        raise the consumer's stripe flag."""
        for d in range(len(self.ipc.duties)):
            for j in range(self.st.nm):
                self.ops += self._relay_op(d, j, 4 + d)

    def _relay_op(self, d: int, j: int, stream: int) -> list[dict]:
        """Duty d's stripe of micro-batch j: wait for it in my slot, copy it into the
        consumer's rows, raise the consumer's stripe flag."""
        p, st = self.ipc, self.st
        (_src, _dst, direction, part), dst_ptrs = p.duties[d], p.relay_dst[d]
        buf, rb = p.relay_bufs[d]
        k, pm = p.layout.duty_k[d], p.duty_part_max[d]
        r = st.rows_of(j)  # every stage shares the micro-batch row layout
        bounds = relay_parts(r.start, r.stop, k)
        a0, a1 = bounds[part], bounds[part + 1]
        idx = p.fidx(j, part) if direction == "f" else p.bidx(j, part)
        return [dict(kind=WAITV, stream=stream, a=p.flags.data_ptr() + 4 * p.ridx(d, j),
                     delta=0),
                dict(kind=COPY, stream=stream, a=buf.data_ptr() + j * pm * rb,
                     b=dst_ptrs["buf"] + a0 * rb, count=(a1 - a0) * rb),
                dict(kind=SIGNAL, stream=stream, a=dst_ptrs["flags"] + 4 * idx, delta=0)]

    # ---- execution -----------------------------------------------------------------------
    def run(self, stream: int) -> None:
        p = self.st.params
        p.set_lr(p.optim.lr)
        if self.transport == "ipc":
            self.plan.seq = self.ipc.seq  # one sequence space with the Python IpcPipe
        self.plan.run(stream)
        if self.transport == "ipc":
            self.ipc.seq = self.plan.seq
        p.step_count += 1

    def comm_error(self) -> int:
        """RCCL async error of any communicator of the plan, or -1 if a flag wait (IPC hop)
        timed out (DNN_FLAG_TIMEOUT seconds)."""
        rc = self.plan.comm_error()
        if rc == 0 and self.transport == "ipc" and self.plan.flag_timeouts():
            return -1
        return rc

    def describe(self) -> dict:
        kinds = {}
        for o in flatten(self.ops):
            kinds[o["kind"]] = kinds.get(o["kind"], 0) + 1
        names = ["SEG", "SEND", "RECV", "ALLREDUCE", "REDUCE_SCATTER", "ALL_GATHER", "COPY",
                 "SIGNAL", "WAITV", "REC", "WAIT", "GSTART", "GEND"]
        return {"transport": self.transport, "mode": self.mode, "ops": len(self.ops),
                "streams": self.n_streams,
                "by_kind": {names[k]: v for k, v in sorted(kinds.items())}}

    def trace(self) -> str:
        """The plan as text, one op per line (DNN_PLAN_TRACE dumps / hang diagnostics)."""
        names = {SEG: "SEG", SEND: "SEND", RECV: "RECV", ALLREDUCE: "ALLREDUCE",
                 REDUCE_SCATTER: "REDUCE_SCATTER", ALL_GATHER: "ALL_GATHER", COPY: "COPY",
                 SIGNAL: "SIGNAL", WAITV: "WAITV", REC: "REC", WAIT: "WAIT", GROUP: "GROUP"}
        out = []
        for i, o in enumerate(self.ops):
            extra = o.get("seg") or o.get("tag") or o.get("event", "")
            if o["kind"] == GROUP:
                extra = [(names[x["kind"]], x.get("gpeer"), x.get("tag")) for x in o["ops"]]
            elif o["kind"] in (SEND, RECV):
                extra = (o.get("gpeer"), o.get("tag"), o["count"])
            out.append(f"{i:4d} s{o['stream']} {names[o['kind']]:14s} {extra}")
        return "\n".join(out)


def flatten(ops: list) -> list:
    """GROUP entries -> GSTART, members, GEND (what StepPlan.add takes)."""
    out = []
    for o in ops:
        if o["kind"] == GROUP:
            out.append(dict(kind=GSTART, stream=o["stream"]))
            out += o["ops"]
            out.append(dict(kind=GEND, stream=o["stream"]))
        else:
            out.append(o)
    return out


def logical_times(kind: str, pp: int, nm: int) -> list[list[int]]:
    """Global logical clock of a replica's pipeline for the slotted plan: compute op k of
    stage s runs at the earliest slot after its predecessor on the stage and TWO slots after
    the op producing its input on the neighbour (the slot between carries the hop)."""
    lists = [schedule_ops(kind, pp, nm, s) for s in range(pp)]
    when = {}  # (stage, op, j) -> time
    t = [[None] * len(lst) for lst in lists]
    remaining = sum(len(lst) for lst in lists)
    while remaining:
        progress = False
        for s, lst in enumerate(lists):
            for k, (op, j) in enumerate(lst):
                if t[s][k] is not None:
                    continue
                prev = t[s][k - 1] if k else -1
                if prev is None:
                    break
                ready = prev + 1
                dep = None
                if op == "F" and s > 0:
                    dep = when.get((s - 1, "F", j), "x")
                elif op == "B" and s < pp - 1:
                    dep = when.get((s + 1, "B", j), "x")
                if dep == "x":
                    break
                if dep is not None:
                    ready = max(ready, dep + 2)
                t[s][k] = ready
                when[(s, op, j)] = ready
                remaining -= 1
                progress = True
        if not progress:
            raise RuntimeError("logical_times: inconsistent schedules")
    return t


def slot_messages(kind: str, pp: int, nm: int, stage: int):
    """Slot -> [(direction, j)] of the messages stage ``stage`` sends / receives in the
    slotted plan: F(j) leaves stage s in the slot after its compute; B(j) likewise."""
    t = logical_times(kind, pp, nm)
    lists = [schedule_ops(kind, pp, nm, s) for s in range(pp)]
    sends, recvs = {}, {}
    for s, lst in enumerate(lists):
        for k, (op, j) in enumerate(lst):
            if op == "F" and s < pp - 1:
                slot, dst = t[s][k] + 1, s + 1
            elif op == "B" and s > 0:
                slot, dst = t[s][k] + 1, s - 1
            else:
                continue
            msg = (op.lower(), j)
            if s == stage:
                sends.setdefault(slot, []).append(msg)
            if dst == stage:
                recvs.setdefault(slot, []).append(msg)
    return sends, recvs


def native_step_supported(executor, mesh) -> Optional[str]:
    """None if the executor's step can run as a NativeStep, else the reason it cannot."""
    if mesh is None:
        return "single process (the loopback plan covers it)"
    if len(executor.stages) != 1:
        return "several stages in one process"
    st = executor.stages[0]
    if st.device.type != "cuda":
        return "CPU stage"
    if st._prog is None or not st._has_w or not st._o_native:
        return "stage not recorded"
    if executor.hooks["before_op"] or executor.hooks["after_op"] or executor.lr_fn is not None:
        return "per-op hooks / lr schedule"
    ops = executor.ops[0]
    for k, (op, j) in enumerate(ops):
        if op == "W" and (j >= 0 or k + 1 >= len(ops) or ops[k + 1][0] != "O"):
            return "per-micro-batch weight gradients"
    if (mesh.dp > 1 or st.params.sharded) and mesh.backend != "nccl":
        return "data-parallel group is not RCCL"
    return None
