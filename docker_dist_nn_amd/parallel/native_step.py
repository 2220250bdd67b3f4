"""Native multi-rank training step: the whole step of a rank as ONE C++ call.

The Python executor (pipeline.PipelineExecutor._run_op) walks the schedule op by op and issues
every pipeline hop and DP bucket through torch.distributed. For a rank that owns one stage this
module instead compiles the SAME schedule once into a ``StepPlan`` (csrc/runtime/step_plan.hpp)
of recorded-segment replays, RCCL calls on the communicators torch already created (or xGMI
peer copies + stream flags), and event edges between four streams:

  stream 0  compute (the caller's stream): F{j}, B{j}, W{i}, FIN*, O / FINO segments
  stream 1  forward hops:   recv F(j) from the previous stage, send F(j) to the next
  stream 2  backward hops:  recv B(j) from the next stage,     send B(j) to the previous
  stream 3  data-parallel gradient all-reduce buckets

Each direction keeps its own FIFO in micro-batch order on its own communicator (the fwd / bwd
process groups of parallel/groups.py), so a blocked transfer in one direction never stalls the
other and no send/recv grouping is needed; compute waits only for the receive it consumes.
DP buckets (pipeline.dp_buckets: largest layer first) are all-reduced on stream 3 while the
remaining weight-gradient GEMMs run, then the update waits for all of them.

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
from .comm import relay_parts
from .pipeline import dp_buckets

SEG, SEND, RECV, ALLREDUCE, REDUCE_SCATTER, ALL_GATHER, COPY, SIGNAL, WAITV, REC, WAIT = range(11)
NCCL_BF16, NCCL_F32, NCCL_U8 = 9, 7, 1
MAIN, FWD, BWD, DPS = 0, 1, 2, 3


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
    """Builds and runs the StepPlan of one rank. ``transport``: "rccl" (RCCL P2P on the fwd /
    bwd groups) or "ipc" (an IpcPipe's mapped peer buffers and flags)."""

    def __init__(self, executor, mesh, transport: str, ipc=None):
        if len(executor.stages) != 1:
            raise ValueError("native multi-rank step: one stage per rank")
        st = executor.stages[0]
        if st._prog is None or not st._has_w or not st._o_native:
            raise ValueError("native multi-rank step needs a recorded stage (compile_native)")
        self.ex, self.mesh, self.st = executor, mesh, st
        self.transport = transport
        self.ipc = ipc
        self.n = native()
        dev = st.device
        self.dp = mesh.dp if mesh is not None else 1
        self.sharded = st.params.sharded
        if transport == "rccl" or self.dp > 1 or self.sharded:
            self.n.nccl_load(torch_rccl_path())
        self.comm_f = self.comm_b = self.comm_dp = 0
        if transport == "rccl" and mesh.pp > 1:
            self.comm_f = comm_ptr(mesh.fwd_group, dev)
            self.comm_b = comm_ptr(mesh.bwd_group, dev)
        if self.dp > 1 or self.sharded:
            self.comm_dp = comm_ptr(mesh.dp_group, dev)
        self._ev = 0
        self.ops: list[tuple] = []
        self._build()
        n_streams = 4 + (len(ipc.duties) if transport == "ipc" and ipc is not None else 0)
        # streams of a plan block on flags / peers: each needs its own hardware queue (HIP maps
        # streams beyond GPU_MAX_HW_QUEUES onto shared queues, where one blocked wait stalls
        # the streams behind it -- a cross-rank deadlock); stream 0 is the caller's
        hwq = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
        if n_streams > hwq:
            raise RuntimeError(f"native step needs {n_streams} hardware queues, "
                               f"GPU_MAX_HW_QUEUES={hwq}: set it (before the GPU is "
                               f"initialised) to >= {n_streams}")
        self.plan = self.n.StepPlan(n_streams, max(1, self._ev))
        for o in self.ops:
            self.plan.add(**o)

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

    def _recv(self, direction: str, j: int) -> None:
        st, m = self.st, self.mesh
        if st.boundary == "fp8":  # e4m3 rows then fp32 row scales, then unpack on compute
            s = FWD if direction == "f" else BWD
            peer = m.stage - 1 if direction == "f" else m.stage + 1
            q, sc = (st.q_in, st.s_in) if direction == "f" else (st.q_gin, st.s_gin)
            for t, dt in ((q, NCCL_U8), (sc, NCCL_F32)):
                ptr, cnt = self._rows(t, j)
                self.ops.append(dict(kind=RECV, stream=s,
                                     comm=self.comm_f if s == FWD else self.comm_b,
                                     a=ptr, count=cnt, dtype=dt, peer=peer))
            self._edge(s, MAIN)
            self._seg(f"DQF{j}" if direction == "f" else f"DQB{j}")
            return
        t = st.x_in if direction == "f" else st.grad_out
        if self.transport == "ipc":  # the producer's copies + flags: wait on the compute stream
            p = self.ipc
            base = p.flags.data_ptr()
            for part in range(p.k + 1):  # the direct stripe and every relayed one
                idx = p.fidx(j, part) if direction == "f" else p.bidx(j, part)
                self.ops.append(dict(kind=WAITV, stream=MAIN, a=base + 4 * idx, delta=0))
            return
        ptr, cnt = self._rows(t, j)
        s = FWD if direction == "f" else BWD
        peer = m.stage - 1 if direction == "f" else m.stage + 1
        self.ops.append(dict(kind=RECV, stream=s, comm=self.comm_f if s == FWD else self.comm_b,
                             a=ptr, count=cnt, dtype=NCCL_BF16, peer=peer))
        self._edge(s, MAIN)

    def _send(self, direction: str, j: int) -> None:
        st, m = self.st, self.mesh
        if st.boundary == "fp8":
            s = FWD if direction == "f" else BWD
            self._seg(f"QF{j}" if direction == "f" else f"QB{j}")
            self._edge(MAIN, s)
            peer = m.stage + 1 if direction == "f" else m.stage - 1
            q, sc = (st.q_out, st.s_out) if direction == "f" else (st.q_dx, st.s_dx)
            for t, dt in ((q, NCCL_U8), (sc, NCCL_F32)):
                ptr, cnt = self._rows(t, j)
                self.ops.append(dict(kind=SEND, stream=s,
                                     comm=self.comm_f if s == FWD else self.comm_b,
                                     a=ptr, count=cnt, dtype=dt, peer=peer))
            return
        t = st.output if direction == "f" else st.dx_send
        s = FWD if direction == "f" else BWD
        self._edge(MAIN, s)
        ptr, cnt = self._rows(t, j)
        if self.transport == "ipc":
            p = self.ipc
            peer = p.next if direction == "f" else p.prev
            if j == 0:  # the peer finished reading that buffer in the previous step (ack)
                ack = p.ackf if direction == "f" else p.ackb
                self.ops.append(dict(kind=WAITV, stream=s, a=p.flags.data_ptr() + 4 * ack,
                                     delta=-1))
            dst_base = peer["x_in"] if direction == "f" else peer["grad_out"]
            row_bytes = p.row_bytes_f if direction == "f" else p.row_bytes_b
            r = st.rows_of(j)
            bounds = relay_parts(r.start, r.stop, p.k)
            for part in range(p.k + 1):  # stripe 0 direct, stripe q via relay q - 1
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
                    slot = rel["buf"] + j * p.part_max * row_bytes
                    self.ops.append(dict(kind=COPY, stream=s, a=src, b=slot,
                                         count=(a1 - a0) * row_bytes))
                    self.ops.append(dict(kind=SIGNAL, stream=s,
                                         a=rel["flags"] + 4 * p.ridx(rel["d"], j), delta=0))
            return
        peer = m.stage + 1 if direction == "f" else m.stage - 1
        self.ops.append(dict(kind=SEND, stream=s, comm=self.comm_f if s == FWD else self.comm_b,
                             a=ptr, count=cnt, dtype=NCCL_BF16, peer=peer))

    def _wgrad_update(self) -> None:
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
            self._sharded_update()
            return
        for bucket in dp_buckets(st):
            for i in bucket:
                self._seg(f"W{i}")
            a, b = bucket[0], bucket[-1]
            self._seg(f"FIN{a}" if a == b else f"FIN{a}-{b}")
            e0, _ = p.layer_grad_range(a)
            _, e1 = p.layer_grad_range(b)
            self._edge(MAIN, DPS)
            self.ops.append(dict(kind=ALLREDUCE, stream=DPS, comm=self.comm_dp,
                                 a=p.grad.data_ptr() + 4 * e0, count=e1 - e0, dtype=NCCL_F32))
        self._edge(DPS, MAIN)
        self._seg("O")

    def _sharded_update(self) -> None:
        """Sharded DP (pipeline.GradSync shard): per bucket, W segments -> FIN -> bf16 pack on
        the compute stream, then the bucket's bf16 reduce-scatter on the DP stream (overlapping
        the next bucket's wgrads). Per bucket again: unpack + update of this rank's piece, then
        the bf16 all-gather of the piece's shadow weights; the W^T refresh waits for all."""
        st = self.st
        p = st.params
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
            self._edge(MAIN, DPS)
            self.ops.append(dict(kind=REDUCE_SCATTER, stream=DPS, comm=self.comm_dp,
                                 a=p.grad16.data_ptr() + 2 * e0,
                                 b=p.grad_piece.data_ptr() + 2 * (e0 // d),
                                 count=(e1 - e0) // d, dtype=NCCL_BF16))
        # every bias gradient (fp32, a few KB): all-reduced, then updated on every rank
        self.ops.append(dict(kind=ALLREDUCE, stream=DPS, comm=self.comm_dp,
                             a=p.grad.data_ptr() + 4 * p.bias_lo, count=p.numel - p.bias_lo,
                             dtype=NCCL_F32))
        self._edge(DPS, MAIN)
        self._seg("SB")
        for a, b, e0, e1 in buckets:
            self._seg(f"SU{a}-{b}")
            self._edge(MAIN, DPS)
            p0, _ = p.shard_piece(e0, e1)
            self.ops.append(dict(kind=ALL_GATHER, stream=DPS, comm=self.comm_dp,
                                 a=p.shadow.data_ptr() + 2 * p0, b=p.shadow.data_ptr() + 2 * e0,
                                 count=(e1 - e0) // d, dtype=NCCL_BF16))
        if p.optim.name != "sgd":
            self._seg("OADV")
        self._edge(DPS, MAIN)
        self._seg("T")

    def _build(self) -> None:
        m, st = self.mesh, self.st
        ops = self.ex.ops[0]
        has_prev = m is not None and m.prev_rank is not None
        has_next = m is not None and m.next_rank is not None
        for k, (op, j) in enumerate(ops):
            nxt = ops[k + 1][0] if k + 1 < len(ops) else None
            if op == "F":
                if has_prev:
                    self._recv("f", j)
                self._seg(f"F{j}")
                if has_next:
                    self._send("f", j)
            elif op == "B":
                if has_next:
                    self._recv("b", j)
                self._seg(f"B{j}")
                if has_prev:
                    self._send("b", j)
            elif op == "W":
                if j >= 0 or nxt != "O":
                    raise ValueError("native multi-rank step: batched W followed by O only")
                self._wgrad_update()
            elif op == "O":
                pass  # emitted with the batched W
        if self.transport == "ipc":  # release the buffers I receive into for the next step
            p = self.ipc
            if p.prev is not None:
                self.ops.append(dict(kind=SIGNAL, stream=MAIN, a=p.prev["flags"] + 4 * p.ackf,
                                     delta=0))
            if p.next is not None:
                self.ops.append(dict(kind=SIGNAL, stream=MAIN, a=p.next["flags"] + 4 * p.ackb,
                                     delta=0))
            self._relay_duties()

    def _relay_duties(self) -> None:
        """My relay work for other ranks' hops, one stream per duty (a duty's stripes arrive
        in micro-batch order, and separate streams keep one hop from blocking another):
        wait for the producer's stripe j in my slot -> copy it into the consumer's rows ->
        raise the consumer's stripe flag."""
        p, st = self.ipc, self.st
        for d, ((src, dst, direction, part), dst_ptrs) in enumerate(zip(p.duties, p.relay_dst)):
            stream = 4 + d
            buf, rb = p.relay_bufs[d]
            for j in range(st.nm):
                r = st.rows_of(j)  # every stage shares the micro-batch row layout
                bounds = relay_parts(r.start, r.stop, p.k)
                a0, a1 = bounds[part], bounds[part + 1]
                self.ops.append(dict(kind=WAITV, stream=stream,
                                     a=p.flags.data_ptr() + 4 * p.ridx(d, j), delta=0))
                self.ops.append(dict(kind=COPY, stream=stream,
                                     a=buf.data_ptr() + j * p.part_max * rb,
                                     b=dst_ptrs["buf"] + a0 * rb, count=(a1 - a0) * rb))
                idx = p.fidx(j, part) if direction == "f" else p.bidx(j, part)
                self.ops.append(dict(kind=SIGNAL, stream=stream, a=dst_ptrs["flags"] + 4 * idx,
                                     delta=0))

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
        for o in self.ops:
            kinds[o["kind"]] = kinds.get(o["kind"], 0) + 1
        names = ["SEG", "SEND", "RECV", "ALLREDUCE", "REDUCE_SCATTER", "ALL_GATHER", "COPY",
                 "SIGNAL", "WAITV", "REC", "WAIT"]
        return {"transport": self.transport, "ops": len(self.ops),
                "by_kind": {names[k]: v for k, v in sorted(kinds.items())}}


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
