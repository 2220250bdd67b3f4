"""Training front-end of a replicated-stage ("fan") pipeline (parallel/fan.py).

Each rank owns replica ``mesh.replica`` of stage ``mesh.stage``: the stage's layers, the rows of
its own micro-batches (j = replica, replica + r_s, ...), fan-in / fan-out hops to the replicas
of the neighbouring stages, and -- when the stage has several replicas -- a gradient exchange
over the stage's own DP group. The step is the full-batch update of ``micro_batch x
num_micro`` rows, the same math as one process training on the whole batch (the reference's
centralized recipe, /root/reference/scripts/generate_mnist_pytorch.py:35-52, distributed over
a layout the reference's layer_distribution chain, /root/reference/src/run_grpc_fcnn.py:199-248,
cannot express).
"""
from __future__ import annotations

from typing import Optional

import torch

from ..models.mlp import MLPSpec
from ..parallel.fan import (FanIpcPipe, FanLayout, FanMesh, FanPipe, fan_schedule,
                             gather_rows, stage_costs)
from ..parallel.pipeline import GradSync, PipelineExecutor
from ..partition import plan_stages
from .stage import OptimConfig, Stage
from .trainer import Trainer, _any_rank, _warm_groups
from .. import switches


class _RankSteps:
    """The Python step of a rank hosting several workers (co-located fan layout): each
    worker's stage has an executor of its own (its own DP group), and the rank runs every
    compute op of its workers in the schedule's rank order (FanSchedule.rank_ops: one GPU, one
    compute stream), then each stage's batched weight gradient and update."""

    def __init__(self, execs: dict, order: list, pipe):
        self.execs, self.order, self.pipe = execs, order, pipe
        self.stages = [ex.stages[0] for _, ex in sorted(execs.items())]
        self.native_step = None
        self.capturing = False

    def run_step(self) -> None:
        if self.native_step is not None:  # the co-located slotted RCCL plan (fan.FanNativeStep)
            for st in self.stages:
                st.begin_step()
            self.native_step.run(torch.cuda.current_stream(self.stages[0].device).cuda_stream)
            return
        self.pipe.begin_step()
        for ex in self.execs.values():
            st = ex.stages[0]
            st.begin_step()
            if st.params.fused_layers:  # one-split wgrads update in their epilogue
                st.params.set_lr(ex.lr_fn() if ex.lr_fn else st.params.optim.lr)
        for s, op, jj in self.order:
            ex = self.execs[s]
            ex._run_op(ex.stages[0], op, jj, None)
        for s, ex in sorted(self.execs.items(), reverse=True):
            st = ex.stages[0]
            ex._run_op(st, "W", -1, "O")
            ex._run_op(st, "O", -1, None)
        self.pipe.end_step()

    def flush(self) -> None:
        for ex in self.execs.values():
            ex.flush()

    def xstep_join(self) -> None:
        pass


class FanTrainer(Trainer):
    def __init__(self, spec: MLPSpec, layout: FanLayout, mesh: FanMesh, *, micro_batch: int,
                 num_micro: int, optim: Optional[OptimConfig] = None,
                 device: Optional[torch.device] = None, seed: int = 0,
                 dp_reduce: str = "allreduce", native_exec: Optional[bool] = None,
                 hop_cost: float = 0.0, ipc_rehearsal: bool = False):
        """``ipc_rehearsal`` (one-GPU tests: ranks sharing a GPU over gloo): set up the IPC
        transport (``self.ipc_pipe``) whatever the backend, for a test that runs the IPC fan
        plan through the plan interpreter; the Python executor keeps the gloo FanPipe.
        ``ipc_rehearsal="native"``: the IPC fan plan as the rank's real StepPlan (eager or
        captured, Trainer.capture) -- layouts without replicated stages only, since a DP
        group's buckets are RCCL calls and RCCL runs one rank per GPU."""
        if sum(layout.dist) != len(spec.layers):
            raise ValueError(f"fan layout {layout.dist} does not cover {len(spec.layers)} layers")
        layout.check_directions(num_micro)
        self.spec, self.mesh, self.layout = spec, mesh, layout
        self.device = device or (torch.device("cuda", torch.cuda.current_device())
                                 if torch.cuda.is_available() else torch.device("cpu"))
        workers = mesh.workers or [(mesh.stage, mesh.replica)]
        s, q = workers[0]
        r = layout.reps[s]
        self.pp, self.dp = layout.S, r
        self.plans = plan_stages(len(spec.layers), list(layout.dist))
        self.distribution = list(layout.dist)
        self.schedule = "fan"
        self.micro_batch, self.num_micro = micro_batch, num_micro
        self.global_batch = micro_batch * num_micro
        self.optim = optim or OptimConfig()
        if dp_reduce not in ("allreduce", "shard"):
            raise ValueError(f"dp_reduce must be allreduce | shard, got {dp_reduce!r}")
        self.dp_reduce = dp_reduce if max(layout.reps[w] for w, _ in workers) > 1 \
            else "allreduce"
        self.local = layout.local_micros(s, q, num_micro)
        f, b = stage_costs(spec, layout.dist)
        self.sched = fan_schedule(layout, num_micro, f, b, hop_cost)
        stages = {}
        for ws, wq in workers:
            wr = layout.reps[ws]
            p = self.plans[ws]
            st = Stage(spec, p.layer_start, p.layer_end, micro_batch=micro_batch,
                       num_micro=len(layout.local_micros(ws, wq, num_micro)),
                       device=self.device, global_batch=self.global_batch, optim=self.optim,
                       wgrad="batched", stage_index=ws, num_stages=layout.S,
                       dp_shard=(wr, wq) if self.dp_reduce == "shard" and wr > 1 else None)
            st.params.init_default(seed)
            stages[ws] = st
        self.stages = [stages[k] for k in sorted(stages)]
        self.pipe = FanPipe(mesh, stages if len(stages) > 1 else stages[s], self.sched)
        if native_exec is None:
            native_exec = self.device.type == "cuda"
        # xGMI peer writes (FanIpcPipe) on RCCL jobs, like the uniform pipeline's DNN_PIPE=auto:
        # set up before the stage records its launches (the receive buffers move to uncached
        # memory); verified bitwise against the RCCL plan on the first step
        self._ipc_verify = None
        self._fallback_step = None
        ipc, ipc_why = None, None
        self.ipc_pipe = None
        if ipc_rehearsal:
            self.ipc_pipe = FanIpcPipe(mesh, stages[s], self.sched)
        mode = switches.get("DNN_PIPE")
        if mesh.backend == "nccl" and self.device.type == "cuda" and native_exec and \
                not layout.colocated and mode in ("auto", "ipc") and \
                switches.get("DNN_NATIVE_DIST") != "0":
            if mode == "ipc" or self._peers_mappable(mesh):
                try:
                    ipc = FanIpcPipe(mesh, stages[s], self.sched)  # errors agreed inside
                except RuntimeError as e:
                    if mode == "ipc":
                        raise
                    ipc_why = f"IPC set-up failed: {e}"[:200]
            else:
                ipc_why = "a GPU pair of the plan has no peer access"
        self.boundary = "bf16"
        execs = {}
        for ws, wq in workers:
            wr = layout.reps[ws]
            sync = GradSync(mesh.dp_groups.get(ws), wr,
                            shard=self.dp_reduce == "shard") if wr > 1 else None
            ex = PipelineExecutor([stages[ws]], self.pipe, "1f1b", layout.S, [ws], sync)
            ex.ops = [self.sched.local_ops(ws, wq)]
            execs[ws] = ex
            if wr == 1:  # the gradient is complete where it is produced: update in the epilogue
                stages[ws].enable_fused_wgrad_update()
        if len(workers) == 1:
            self.executor = execs[s]
        else:
            order = [(ws, op, layout.local_index(ws, j)) for ws, op, j in
                     self.sched.rank_ops(mesh.rank)]
            self.executor = _RankSteps(execs, order, self.pipe)
        self.native_exec = bool(native_exec)
        if self.native_exec:
            for st in self.stages:
                st.compile_native()
        self.native_step = None
        self.native_fallback = None
        self.transport = "rccl" if mesh.backend == "nccl" else mesh.backend
        self.transport_reason = (f"fan layout {layout.describe()}: fan-in / fan-out P2P "
                                 f"({self.transport}), Python executor" +
                                 (", co-located hops as device copies" if len(workers) > 1
                                  else ""))
        if mesh.backend == "nccl" and self.native_exec and \
                switches.get("DNN_NATIVE_DIST") != "0":
            # the rank's whole step as one StepPlan call (fan.FanNativeStep, slotted RCCL form;
            # a co-located rank runs all its workers in it); agreed over the world like the
            # uniform mesh's native step (trainer.py)
            from ..parallel.fan import FanNativeStep

            _warm_groups(mesh, self.device)
            err = None
            try:
                self.native_step = FanNativeStep(self.executor, mesh, self.sched)
            except Exception as e:
                err = e
            if _any_rank(self.native_step is None, self.device):
                self.native_fallback = repr(err) if err is not None else "another rank"
                self.native_step = None
            else:
                self.executor.native_step = self.native_step
                self.transport_reason = (f"fan layout {layout.describe()}: slotted RCCL plan "
                                         "(one group per clock slot), native step")
            if ipc is not None:
                ipc_step, err = None, None
                try:
                    if self.native_step is None:
                        raise RuntimeError("no RCCL plan to verify the IPC plan against")
                    ipc_step = FanNativeStep(self.executor, mesh, self.sched, ipc=ipc)
                except Exception as e:
                    err = e
                if _any_rank(ipc_step is None, self.device):
                    ipc.close()
                    ipc_why = f"IPC fan plan unavailable ({err!r} here)"[:200]
                else:
                    # the first step runs on IPC, then from the same state on the RCCL plan;
                    # IPC stays only if every rank's weights agree bit for bit
                    # (Trainer._verify_first_step, the uniform pipeline's protocol)
                    self._fallback_step = self.native_step
                    self.native_step = ipc_step
                    self.executor.native_step = ipc_step
                    self.executor.pipe = ipc
                    self._ipc_verify = (ipc, self.pipe)
                    self.pipe = ipc
                    self.transport = "ipc"
                    self.transport_reason = (
                        f"fan layout {layout.describe()}: ipc, peer copies + flags in clock "
                        "order on one stream (verification pending: first step)")
            if ipc_why is not None and self.transport != "ipc":
                self.transport_reason += f"; IPC not used: {ipc_why}"
        if ipc_rehearsal == "native":
            from ..parallel.fan import FanNativeStep

            if max(layout.reps) > 1 or layout.colocated:
                raise ValueError("native IPC fan rehearsal: one replica per stage (DP buckets "
                                 "are RCCL calls, one rank per GPU)")
            self.native_step = FanNativeStep(self.executor, mesh, self.sched, comms={},
                                             ipc=self.ipc_pipe)
            self.executor.native_step = self.native_step
            self.executor.pipe = self.pipe = self.ipc_pipe
            self.transport = "ipc"
        self._graph = None
        self._graphs = []
        self._stream = None
        self.graph_nodes = 0
        self.steps_done = 0

    @property
    def input_micros(self) -> list:
        """Global micro-batches whose INPUT rows this rank holds (its stage-0 replica's)."""
        q = next((wq for ws, wq in (self.mesh.workers or [(self.mesh.stage,
                                                            self.mesh.replica)]) if ws == 0),
                 None)
        return [] if q is None else self.layout.local_micros(0, q, self.num_micro)

    @property
    def label_micros(self) -> list:
        """Global micro-batches whose LABELS this rank holds (its last-stage replica's)."""
        S = self.layout.S
        q = next((wq for ws, wq in (self.mesh.workers or [(self.mesh.stage,
                                                            self.mesh.replica)])
                  if ws == S - 1), None)
        return [] if q is None else self.layout.local_micros(S - 1, q, self.num_micro)

    def set_global_batch(self, x: Optional[torch.Tensor], labels: Optional[torch.Tensor]):
        """The GLOBAL batch (all micro-batches); this rank keeps its own micro-batches' rows
        (its first-stage replica: inputs; its last-stage replica: labels)."""
        mb = self.micro_batch
        xs = gather_rows(x, [slice(j * mb, (j + 1) * mb) for j in self.input_micros]) \
            if self.first is not None else None
        ys = gather_rows(labels, [slice(j * mb, (j + 1) * mb) for j in self.label_micros]) \
            if self.last is not None else None
        self.set_batch(xs, ys)

    def loss(self) -> Optional[float]:
        """This replica's share of the global mean loss (the replicas' shares add up)."""
        if self.last is None:
            return None
        return self.last.loss_sum() / self.global_batch
