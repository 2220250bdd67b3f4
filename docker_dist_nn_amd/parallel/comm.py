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
        # post every receive of the step now, in micro-batch order, per direction channel
        if m.prev_rank is not None:
            for j in range(s.nm):
                self._recv_f[j] = self._irecv(s.x_in[s.rows_of(j)], m.prev_rank, m.fwd_group,
                                              ("rf", j))
        if m.next_rank is not None:
            for j in range(s.nm):
                self._recv_b[j] = self._irecv(s.grad_out[s.rows_of(j)], m.next_rank,
                                              m.bwd_group, ("rb", j))

    def recv_fwd(self, stage, j):
        if self.mesh.prev_rank is not None:
            self._finish_recv(self._recv_f.pop(j))

    def send_fwd(self, stage, j):
        if self.mesh.next_rank is not None:
            self._isend(stage.output[stage.rows_of(j)], self.mesh.next_rank, self.mesh.fwd_group,
                        ("sf", j))

    def recv_bwd(self, stage, j):
        if self.mesh.next_rank is not None:
            self._finish_recv(self._recv_b.pop(j))

    def send_bwd(self, stage, j):
        if self.mesh.prev_rank is not None:
            self._isend(stage.dx_send[stage.rows_of(j)], self.mesh.prev_rank,
                        self.mesh.bwd_group, ("sb", j))

    def end_step(self):
        for w in self._sends:
            w.wait()
        self._sends.clear()
        if self._recv_f or self._recv_b:
            raise RuntimeError("step ended with unconsumed pipeline receives")
