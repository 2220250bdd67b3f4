"""Pipeline transports: how micro-batch activations / gradients move between stages.

The reference forwarded every request through a fresh gRPC channel, re-serialising fp64 rows
at every hop (/root/reference/src/grpc_node.py:120-135). Here a hop is a bf16 row slice of a
pre-allocated step buffer, moved by:

* :class:`DistPipe` -- ``torch.distributed`` P2P. With the ``nccl`` backend that is RCCL
  send/recv over the direct xGMI link between the two GPUs, issued on RCCL's own stream with
  event ordering against the compute stream (``isend`` waits for the producing kernel, the
  consumer's stream waits on ``irecv``), so transfers overlap compute of other micro-batches.
  Every receive of a step is posted at step start on a direction-private communicator (see
  groups.py), so data lands as soon as the producer sends it. With ``gloo`` it runs on CPU
  tensors (tests) or stages GPU tensors through host memory (``staged=True``, one-GPU
  multi-rank rehearsals).
* :class:`IpcPipe` -- xGMI peer writes (``DNN_PIPE=ipc``): each rank maps its neighbours'
  receive buffers and flag words through IPC handles (csrc/runtime/p2p.cpp). A hop is one
  device-to-device copy straight into the consumer's input rows plus a stream-ordered flag
  write; the consumer's stream waits on the flag (hipStreamWaitValue32) -- no RCCL kernel, no
  host round trip.
* :class:`LoopbackPipe` -- all stages in one process on one device: the next stage's input
  buffer IS the previous stage's output buffer (and likewise for gradients), so a hop costs
  nothing; used to run/verify S-stage pipelines on a single GPU or CPU.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .groups import Mesh


class LoopbackPipe:
    """Zero-copy hops between stages living in the same process and device."""

    def __init__(self, stages):
        self.stages = stages
        for a, b in zip(stages, stages[1:]):
            if a.output.shape != b.x_in.shape or a.device != b.device:
                raise ValueError("loopback stages must share device and boundary width")
            b.x_in = b.x_buf = a.output  # activations: producer writes the consumer's input
            a.dz[-1] = b.dx_send        # gradients: consumer writes the producer's dZ
            # ... and the consumer's first dgrad epilogue emits the producer's bias-gradient
            # partials (column sums of that dZ): no boundary colsum kernel per micro-batch
            a.fuse_boundary_colsum(b)

    def begin_step(self):
        pass

    def recv_fwd(self, stage, j):
        pass

    def send_fwd(self, stage, j):
        pass

    def recv_bwd(self, stage, j):
        pass

    def send_bwd(self, stage, j):
        pass

    def end_step(self):
        pass


class DistPipe:
    """P2P transport between the ranks of one pipeline (one stage per rank)."""

    def __init__(self, mesh: Mesh, stage, staged: Optional[bool] = None):
        self.mesh = mesh
        self.stage = stage
        dev_is_gpu = stage.device.type == "cuda"
        self.staged = staged if staged is not None else (dev_is_gpu and mesh.backend == "gloo")
        self._recv_f: dict[int, object] = {}
        self._recv_b: dict[int, object] = {}
        self._sends: list = []
        self._host = {}

    def _buf(self, key, t):
        b = self._host.get(key)
        if b is None or b.shape != t.shape:
            b = torch.empty(t.shape, dtype=t.dtype, pin_memory=torch.cuda.is_available())
            self._host[key] = b
        return b

    def _irecv(self, t, src, group, key):
        if self.staged:
            h = self._buf(key, t)
            w = dist.irecv(h, src=src, group=group)
            return (w, h, t)
        return (dist.irecv(t, src=src, group=group), None, None)

    def _finish_recv(self, rec):
        w, h, t = rec
        w.wait()
        if h is not None:
            t.copy_(h, non_blocking=False)

    def _isend(self, t, dst, group, key):
        if self.staged:
            h = self._buf(key, t)
            h.copy_(t)  # synchronous D2H: the kernel that produced t has finished
            self._sends.append(dist.isend(h, dst=dst, group=group))
        else:
            self._sends.append(dist.isend(t, dst=dst, group=group))

    def begin_step(self):
        m, s = self.mesh, self.stage
        fp8 = s.boundary == "fp8"
        # post every receive of the step now, in micro-batch order, per direction channel
        # (fp8 boundary: the e4m3 rows, then their scales -- the same order on both sides)
        if m.prev_rank is not None:
            for j in range(s.nm):
                r = s.rows_of(j)
                bufs = (s.q_in[r], s.s_in[r]) if fp8 else (s.x_in[r],)
                self._recv_f[j] = [self._irecv(b, m.prev_rank, m.fwd_group, ("rf", j, k))
                                   for k, b in enumerate(bufs)]
        if m.next_rank is not None:
            for j in range(s.nm):
                r = s.rows_of(j)
                bufs = (s.q_gin[r], s.s_gin[r]) if fp8 else (s.grad_out[r],)
                self._recv_b[j] = [self._irecv(b, m.next_rank, m.bwd_group, ("rb", j, k))
                                   for k, b in enumerate(bufs)]

    def recv_fwd(self, stage, j):
        if self.mesh.prev_rank is not None:
            for rec in self._recv_f.pop(j):
                self._finish_recv(rec)
            if stage.boundary == "fp8":
                stage.unpack_fwd(j)

    def send_fwd(self, stage, j):
        if self.mesh.next_rank is not None:
            r = stage.rows_of(j)
            if stage.boundary == "fp8":
                stage.pack_fwd(j)
                bufs = (stage.q_out[r], stage.s_out[r])
            else:
                bufs = (stage.output[r],)
            for k, b in enumerate(bufs):
                self._isend(b, self.mesh.next_rank, self.mesh.fwd_group, ("sf", j, k))

    def recv_bwd(self, stage, j):
        if self.mesh.next_rank is not None:
            for rec in self._recv_b.pop(j):
                self._finish_recv(rec)
            if stage.boundary == "fp8":
                stage.unpack_bwd(j)

    def send_bwd(self, stage, j):
        if self.mesh.prev_rank is not None:
            r = stage.rows_of(j)
            if stage.boundary == "fp8":
                stage.pack_bwd(j)
                bufs = (stage.q_dx[r], stage.s_dx[r])
            else:
                bufs = (stage.dx_send[r],)
            for k, b in enumerate(bufs):
                self._isend(b, self.mesh.prev_rank, self.mesh.bwd_group, ("sb", j, k))

    def end_step(self):
        for w in self._sends:
            w.wait()
        self._sends.clear()
        if self._recv_f or self._recv_b:
            raise RuntimeError("step ended with unconsumed pipeline receives")


def relay_assignment(pp: int, dp: int, k: int) -> dict:
    """Relay ranks of every directed pipeline hop of a pp x dp mesh (rank = replica * pp +
    stage, parallel/groups.build_mesh): {(src, dst, "f" | "b"): [k relay ranks]}. A hop's rows
    are striped over the direct link and k two-link paths src -> relay -> dst, so one hop
    draws on k + 1 of the source's xGMI links instead of one. Relays are picked least-loaded
    first (then by distance from the source), so duties spread over the node; the result is
    a pure function of (pp, dp, k): every rank computes the same table."""
    world = pp * dp
    hops = []
    for r in range(dp):
        for s in range(pp - 1):
            a, b = r * pp + s, r * pp + s + 1
            hops += [(a, b, "f"), (b, a, "b")]
    if k and world - 2 < k:
        raise ValueError(f"{k} relays per hop need >= {k + 2} ranks (world {world})")
    load = [0] * world
    out = {}
    for src, dst, d in hops:
        cands = sorted((x for x in range(world) if x not in (src, dst)),
                       key=lambda x: (load[x], (x - src) % world))
        out[(src, dst, d)] = cands[:k]
        for x in cands[:k]:
            load[x] += 1
    return out


def relay_plan(pp: int, dp: int, hop_bytes, dp_bytes=None, max_k: int = 6,
               max_duties: int = 6, relay_eff: float = 0.8) -> dict:
    """Relay ranks of every directed pipeline hop, chosen PER HOP from a load model of the
    node's directed xGMI links (each GPU pair has its own link both ways):

    * a hop src -> dst of boundary b moves ``hop_bytes[b]`` per step; with k relays its rows
      are striped over k + 1 paths -- the direct link and src -> r -> dst for each relay -- so
      each path carries 1/(k + 1) of the bytes, a relayed path's two links at 1/relay_eff (the
      relay re-reads the stripe from its HBM and adds a hop of latency);
    * data-parallel traffic (``dp_bytes[s]`` per step for the stage-s gradient exchange of a
      ring over the replicas) loads the links between replicas of a stage;
    * widest hops first (two passes), each hop takes the relay count k <= ``max_k`` that
      minimises its own transfer time -- the most loaded link on any of its paths, given
      everything else on the links -- adding relays least-loaded first, each extra relay kept
      only if it saves >= 2 % (a relay costs a stream on its rank and HBM traffic there); a
      rank takes at most ``max_duties`` relay duties.

    The wide boundary of a pipeline (e.g. 784-512-... at pp4: 512 columns after stage 0, 4x
    the 128-column one) thus gets more paths than the narrow ones, instead of the uniform
    ``relay_assignment`` k. Returns {(src, dst, "f" | "b"): [relay ranks]} -- a pure function
    of its arguments: every rank computes the same table. Rank = replica * pp + stage."""
    world = pp * dp
    hops = []  # (src, dst, direction, bytes)
    for r in range(dp):
        for s in range(pp - 1):
            a, b = r * pp + s, r * pp + s + 1
            hops += [(a, b, "f", float(hop_bytes[s])), (b, a, "b", float(hop_bytes[s]))]
    load = {}

    def add(link, v):
        load[link] = load.get(link, 0.0) + v

    if dp_bytes is not None and dp > 1:
        for s in range(pp):
            ring = [r * pp + s for r in range(dp)]
            for i, a in enumerate(ring):
                b = ring[(i + 1) % dp]
                if a != b:
                    add((a, b), float(dp_bytes[s]))
    relays = {(h[0], h[1], h[2]): [] for h in hops}
    duties = [0] * world

    def contribution(h, rl, sign):
        src, dst, _d, nb = h
        frac = nb / (len(rl) + 1)
        add((src, dst), sign * frac)
        for x in rl:
            add((src, x), sign * frac / relay_eff)
            add((x, dst), sign * frac / relay_eff)

    def hop_time(h, rl):  # h's most loaded link once its stripes are on (h not in `load`)
        src, dst, _d, nb = h
        frac = nb / (len(rl) + 1)
        t = load.get((src, dst), 0.0) + frac
        for x in rl:
            t = max(t, load.get((src, x), 0.0) + frac / relay_eff,
                    load.get((x, dst), 0.0) + frac / relay_eff)
        return t

    for h in hops:
        contribution(h, [], +1)
    order = sorted(hops, key=lambda h: (-h[3], h[0], h[1]))
    for _ in range(2):
        for h in order:
            key = (h[0], h[1], h[2])
            contribution(h, relays[key], -1)
            for x in relays[key]:
                duties[x] -= 1
            best_rl, best_t = [], hop_time(h, [])
            rl = []
            while len(rl) < max_k:
                cands = [x for x in range(world) if x not in (h[0], h[1]) and x not in rl and
                         duties[x] < max_duties]
                if not cands:
                    break
                x = min(cands, key=lambda x: (max(load.get((h[0], x), 0.0),
                                                  load.get((x, h[1]), 0.0)), duties[x],
                                              (x - h[0]) % world))
                rl = rl + [x]
                t = hop_time(h, rl)
                if t < best_t * 0.98:
                    best_rl, best_t = list(rl), t
            relays[key] = best_rl
            for x in best_rl:
                duties[x] += 1
            contribution(h, best_rl, +1)
    return relays


def relay_link_loads(pp: int, dp: int, table: dict, hop_bytes, dp_bytes=None,
                     relay_eff: float = 0.8) -> dict:
    """Per-hop transfer cost under ``table``: {(src, dst, dir): bytes-equivalent of the most
    loaded link on any of the hop's paths} (the planner's effective hop bandwidth)."""
    load = {}

    def add(link, v):
        load[link] = load.get(link, 0.0) + v

    hops = {}
    for r in range(dp):
        for s in range(pp - 1):
            a, b = r * pp + s, r * pp + s + 1
            hops[(a, b, "f")] = hops[(b, a, "b")] = float(hop_bytes[s])
    if dp_bytes is not None and dp > 1:
        for s in range(pp):
            ring = [r * pp + s for r in range(dp)]
            for i, a in enumerate(ring):
                b = ring[(i + 1) % dp]
                if a != b:
                    add((a, b), float(dp_bytes[s]))
    for (src, dst, d), nb in hops.items():
        rl = table.get((src, dst, d), [])
        frac = nb / (len(rl) + 1)
        add((src, dst), frac)
        for x in rl:
            add((src, x), frac / relay_eff)
            add((x, dst), frac / relay_eff)
    out = {}
    for (src, dst, d), nb in hops.items():
        rl = table.get((src, dst, d), [])
        links = [(src, dst)] + [l for x in rl for l in ((src, x), (x, dst))]
        out[(src, dst, d)] = max(load[l] for l in links)
    return out


class RelayLayout:
    """One rank's view of a relay table (relay_plan / relay_assignment): stripe counts of its
    own hops, its relay duties, the flag-block indices and the relay slot sizes. The flag block
    reserves kmax + 1 stripe flags per micro-batch and direction (kmax = the table's largest
    k), so every rank computes every peer's flag indices without knowing the peer's hops."""

    def __init__(self, table: dict, me: int, prev: Optional[int], nxt: Optional[int], nm: int,
                 mb: int):
        self.table = table
        self.nm, self.mb = nm, mb
        self.kmax = max((len(v) for v in table.values()), default=0)
        hk = lambda h: len(table.get(h, []))  # noqa: E731
        self.k_in = {"f": hk((prev, me, "f")) if prev is not None else 0,
                     "b": hk((nxt, me, "b")) if nxt is not None else 0}
        self.k_out = {"f": hk((me, nxt, "f")) if nxt is not None else 0,
                      "b": hk((me, prev, "b")) if prev is not None else 0}
        # my duties, in table order: (src, dst, direction, stripe index), their hops' k
        self.duties = [(h[0], h[1], h[2], rl.index(me) + 1) for h, rl in table.items()
                       if me in rl]
        self.duty_k = [hk((d[0], d[1], d[2])) for d in self.duties]
        self.ackf = 2 * nm * (self.kmax + 1)
        self.ackb = self.ackf + 1
        self.n_flags = self.ackf + 2 + len(self.duties) * nm

    def fidx(self, j: int, p: int = 0) -> int:
        return j * (self.kmax + 1) + p

    def bidx(self, j: int, p: int = 0) -> int:
        return self.nm * (self.kmax + 1) + j * (self.kmax + 1) + p

    def ridx(self, d: int, j: int) -> int:
        return self.ackf + 2 + d * self.nm + j

    def part_max(self, k: int) -> int:
        """Rows of the largest stripe of a micro-batch split k + 1 ways."""
        b = relay_parts(0, self.mb, k)
        return max(y - x for x, y in zip(b, b[1:]))

    def duty_index(self, r: int, hop) -> int:
        """Index of ``hop`` among rank r's duties (the slot it relays that hop into)."""
        return [h for h, rl in self.table.items() if r in rl].index(hop)


def relay_parts(r0: int, r1: int, k: int) -> list[int]:
    """Row bounds of the k + 1 stripes of rows [r0, r1) (stripe 0 = the direct link)."""
    n = r1 - r0
    return [r0 + (n * p // (k + 1)) // 8 * 8 for p in range(k + 1)] + [r1]


def _cpu_group():
    """A gloo group over the world for small host-side agreements (works whatever the default
    backend is)."""
    import torch.distributed as dist

    global _CPU_GROUP
    if _CPU_GROUP is None:
        _CPU_GROUP = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" \
            else dist.group.WORLD
    return _CPU_GROUP


_CPU_GROUP = None


class IpcPipe:
    """Pipeline hops as direct writes into IPC-mapped peer buffers (one stage per rank).

    Per rank, a small int32 flag block: ``f[j]`` (activation j of step s has landed in my
    input rows), ``b[j]`` (gradient j has landed in my grad_out rows), ``ack_f`` / ``ack_b``
    (my consumer / producer finished reading the buffers I write into, for step s). Flags
    carry the step sequence number s = 1, 2, ... so nothing is ever reset:

      send_fwd(j): wait ack_f >= s-1 (consumer done with step s-1) -> copy output rows j into
                   the consumer's x_in rows j -> consumer.f[j] = s
      recv_fwd(j): wait f[j] >= s
      send_bwd / recv_bwd: the same with dx_send -> producer's grad_out and b[j]
      end_step:   producer.ack_f... i.e. tell the previous rank its writes into my x_in may
                  resume (prev.ack_f = s) and the next rank likewise (next.ack_b = s)

    All waits/signals are stream-ordered on the compute stream: the signal follows the copy,
    the acks follow every kernel of the step that reads the buffers (wgrad included).

    ``relays`` = k > 0 (native step only, parallel/native_step.py): every hop's rows are
    striped over the direct link and k relay ranks (relay_assignment). Stripe p >= 1 is copied
    into a relay rank's staging slot, whose own relay stream waits for it, copies it into the
    consumer's rows and raises the consumer's per-stripe flag; the consumer waits for all k + 1
    stripe flags. The consumer's end-of-step ack also covers the relay slots (it follows the
    relay copies it waited for). Flag block: [f[j][p], b[j][p], ack_f, ack_b, relay[d][j]]."""

    def __init__(self, mesh: Mesh, stage, relays: int = 0, uncached: bool = True):
        import torch.distributed as dist

        from ..utils.native import native

        if stage.device.type != "cuda":
            raise ValueError("IpcPipe needs GPU stages")
        self.n = native()
        self.mesh = mesh
        self.stage = stage
        nm = stage.nm
        self.nm = nm
        me = mesh.rank
        world = dist.get_world_size()
        # relays: k (the same count on every hop, relay_assignment) or a per-hop table
        # (relay_plan); RelayLayout = this rank's stripes, duties and flag indices
        if isinstance(relays, dict):
            assign = relays
        else:
            k = int(relays)
            assign = relay_assignment(mesh.pp, mesh.dp, k) if k else {}
        self.table = assign
        self.layout = lay = RelayLayout(assign, me, mesh.prev_rank, mesh.next_rank, nm,
                                        stage.mb)
        self.k = lay.kmax
        self.k_in, self.k_out = lay.k_in, lay.k_out
        # my relay duties, in table order: (src, dst, direction, stripe index)
        self.duties = lay.duties
        self.ackf, self.ackb = lay.ackf, lay.ackb
        # Every rank takes part in every collective below even when its local part failed
        # (it sends an error marker instead), and all ranks raise together: one rank raising
        # between two collectives would leave the others blocked in the second one.
        err = None
        mine = {}
        try:
            self.flags = torch.zeros(lay.n_flags, dtype=torch.int32, device=stage.device)
            if uncached:  # the buffers peers write into (see utils/devmem.py)
                self._uncached_recv(stage)
            # destination rows have the source's width: my output == the consumer's input, my
            # dx_send == the producer's grad_out
            self.row_bytes_f = stage.output.stride(0) * stage.output.element_size()
            self.row_bytes_b = (stage.dx_send.stride(0) * stage.dx_send.element_size()
                                if stage.dx_send is not None else 0)
            # rows of a relay slot per micro-batch: the largest stripe of that duty's hop
            self.duty_part_max = [lay.part_max(k) for k in lay.duty_k]
        except Exception as e:  # noqa: BLE001 -- agreed on below
            err = e
            self.row_bytes_f = self.row_bytes_b = 0
        everyone_rb = [None] * world
        dist.all_gather_object(everyone_rb, (self.row_bytes_f, self.row_bytes_b))
        # a relay slot holds one stripe of one micro-batch of the hop's rows
        self.relay_bufs = []
        if err is None:
            try:
                for (src, dst, d, _p), pm in zip(self.duties, self.duty_part_max):
                    rb = everyone_rb[src][0] if d == "f" else everyone_rb[src][1]
                    shape = (nm * pm * rb,)
                    buf = (self._uc(shape, torch.uint8) if uncached else
                           torch.zeros(shape, dtype=torch.uint8, device=stage.device))
                    self.relay_bufs.append((buf, rb))
                torch.cuda.synchronize(stage.device)
                mine = {"x_in": self.n.ipc_export(stage.x_in.data_ptr()),
                        "grad_out": self.n.ipc_export(stage.grad_out.data_ptr()),
                        "flags": self.n.ipc_export(self.flags.data_ptr()),
                        "relay": [self.n.ipc_export(b.data_ptr()) for b, _ in self.relay_bufs]}
            except Exception as e:  # noqa: BLE001
                err = e
        if err is not None:
            mine = {"error": repr(err)}
        everyone = [None] * world
        dist.all_gather_object(everyone, mine)
        bad = [(r, e["error"]) for r, e in enumerate(everyone) if "error" in e]
        if bad:
            raise RuntimeError(f"IPC transport unavailable: {bad}")
        self.seq = 0
        try:
            self.prev = self._peer(everyone, mesh.prev_rank)
            self.next = self._peer(everyone, mesh.next_rank)
            imp = lambda r, key: self.n.ipc_import(*everyone[r][key])  # noqa: E731

            # my hops' relays: where stripe p >= 1 goes (the relay's slot holds, per
            # micro-batch, the largest stripe of this hop)
            self.relay_out = {"f": [], "b": []}
            for d, peer in (("f", mesh.next_rank), ("b", mesh.prev_rank)):
                if peer is None:
                    continue
                pm = lay.part_max(self.k_out[d])
                for r in assign.get((me, peer, d), []):
                    di = lay.duty_index(r, (me, peer, d))
                    self.relay_out[d].append({
                        "buf": self.n.ipc_import(*everyone[r]["relay"][di]),
                        "flags": imp(r, "flags"), "d": di, "part_max": pm})
            # my duties' consumers: where my relay slots go
            self.relay_dst = [{"buf": imp(dst, "x_in" if d == "f" else "grad_out"),
                               "flags": imp(dst, "flags")} for _s, dst, d, _p in self.duties]
        except Exception as e:  # noqa: BLE001
            err = e
        failed = torch.tensor([1 if err is not None else 0], dtype=torch.int32)
        dist.all_reduce(failed, op=dist.ReduceOp.MAX, group=_cpu_group())
        if int(failed.item()):
            raise RuntimeError(f"IPC transport unavailable (peer mapping failed on a rank; "
                               f"here: {err!r})")

    def close(self) -> None:
        """Drop what only this transport uses -- relay slots, the flag block, peer mappings --
        when the job falls back to another transport (they were pinned for the
        life of the process). The re-homed receive buffers stay: the stage's recorded programs
        read them whatever the transport. Uncached memory is freed when its last tensor view
        dies (utils/devmem.py)."""
        self.relay_bufs = []
        self.relay_out = {"f": [], "b": []}
        self.relay_dst = []
        self.prev = self.next = None
        self.flags = None

    def _uc(self, shape, dtype):
        from ..utils.devmem import uncached_zeros

        return uncached_zeros(shape, dtype, self.stage.device)

    def _uncached_recv(self, st) -> None:
        """Re-home this stage's receive buffers (x_in of a non-first stage, grad_out = dz[-1] of
        a non-last stage) in L2-uncached memory. Before any launch is recorded (the recorded
        programs then bind the new addresses)."""
        if st._prog is not None:
            raise RuntimeError("receive buffers must be re-homed before compile_native")
        if self.mesh.prev_rank is not None:
            st.x_buf = self._uc(tuple(st.x_buf.shape), st.x_buf.dtype)
            st.x_in = st.x_buf
        if self.mesh.next_rank is not None:
            st.dz[-1] = self._uc(tuple(st.dz[-1].shape), st.dz[-1].dtype)

    def fidx(self, j: int, p: int = 0) -> int:
        return self.layout.fidx(j, p)

    def bidx(self, j: int, p: int = 0) -> int:
        return self.layout.bidx(j, p)

    def ridx(self, d: int, j: int) -> int:
        return self.layout.ridx(d, j)

    def _peer(self, everyone, rank):
        if rank is None:
            return None
        d = everyone[rank]
        imp = lambda k: self.n.ipc_import(*d[k])  # noqa: E731
        return {"x_in": imp("x_in"), "grad_out": imp("grad_out"), "flags": imp("flags")}

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.stage.device).cuda_stream

    def _flag(self, base: int, i: int) -> int:
        return base + 4 * i

    def begin_step(self):
        if self.k:
            raise RuntimeError("relayed IPC hops run in the native step only "
                               "(parallel/native_step.py)")
        self.seq += 1

    def recv_fwd(self, stage, j):
        if self.prev is not None:
            self.n.wait_geq_u32(self._stream(), self._flag(self.flags.data_ptr(), self.fidx(j)),
                                self.seq)

    def send_fwd(self, stage, j):
        if self.next is None:
            return
        s = self._stream()
        if j == 0:  # the consumer finished every read of its x_in for the previous step
            self.n.wait_geq_u32(s, self._flag(self.flags.data_ptr(), self.ackf), self.seq - 1)
        r = stage.rows_of(j)
        src = stage.output[r]
        off = r.start * self.row_bytes_f
        self.n.copy_async(self.next["x_in"] + off, src.data_ptr(), src.numel() * src.element_size(), s)
        self.n.signal_u32(s, self._flag(self.next["flags"], self.fidx(j)), self.seq)

    def recv_bwd(self, stage, j):
        if self.next is not None:
            self.n.wait_geq_u32(self._stream(), self._flag(self.flags.data_ptr(), self.bidx(j)),
                                self.seq)

    def send_bwd(self, stage, j):
        if self.prev is None:
            return
        s = self._stream()
        if j == 0:
            self.n.wait_geq_u32(s, self._flag(self.flags.data_ptr(), self.ackb), self.seq - 1)
        r = stage.rows_of(j)
        src = stage.dx_send[r]
        off = r.start * self.row_bytes_b
        self.n.copy_async(self.prev["grad_out"] + off, src.data_ptr(),
                          src.numel() * src.element_size(), s)
        self.n.signal_u32(s, self._flag(self.prev["flags"], self.bidx(j)), self.seq)

    def end_step(self):
        s = self._stream()
        if self.prev is not None:  # my x_in is free for the previous rank's next step
            self.n.signal_u32(s, self._flag(self.prev["flags"], self.ackf), self.seq)
        if self.next is not None:  # my grad_out is free for the next rank's next step
            self.n.signal_u32(s, self._flag(self.next["flags"], self.ackb), self.seq)
