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
from ..parallel.fan import FanLayout, FanMesh, FanPipe, fan_rows, fan_schedule, gather_rows, \
    stage_costs
from ..parallel.pipeline import GradSync, PipelineExecutor
from ..partition import plan_stages
from .stage import OptimConfig, Stage
from .trainer import Trainer, _any_rank, _warm_groups
from .. import switches


class FanTrainer(Trainer):
    def __init__(self, spec: MLPSpec, layout: FanLayout, mesh: FanMesh, *, micro_batch: int,
                 num_micro: int, optim: Optional[OptimConfig] = None,
                 device: Optional[torch.device] = None, seed: int = 0,
                 dp_reduce: str = "allreduce", native_exec: Optional[bool] = None,
                 hop_cost: float = 0.0):
        if sum(layout.dist) != len(spec.layers):
            raise ValueError(f"fan layout {layout.dist} does not cover {len(spec.layers)} layers")
        self.spec, self.mesh, self.layout = spec, mesh, layout
        self.device = device or (torch.device("cuda", torch.cuda.current_device())
                                 if torch.cuda.is_available() else torch.device("cpu"))
        s, q = mesh.stage, mesh.replica
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
        self.dp_reduce = dp_reduce if r > 1 else "allreduce"
        self.local = layout.local_micros(s, q, num_micro)
        p = self.plans[s]
        st = Stage(spec, p.layer_start, p.layer_end, micro_batch=micro_batch,
                   num_micro=len(self.local), device=self.device,
                   global_batch=self.global_batch, optim=self.optim, wgrad="batched",
                   stage_index=s, num_stages=layout.S,
                   dp_shard=(r, q) if self.dp_reduce == "shard" else None)
        st.params.init_default(seed)
        self.stages = [st]
        f, b = stage_costs(spec, layout.dist)
        self.sched = fan_schedule(layout, num_micro, f, b, hop_cost)
        self.pipe = FanPipe(mesh, st, self.sched)
        self.boundary = "bf16"
        sync = GradSync(mesh.dp_group, r, shard=self.dp_reduce == "shard") if r > 1 else None
        self.executor = PipelineExecutor(self.stages, self.pipe, "1f1b", layout.S, [s], sync)
        self.executor.ops = [self.sched.local_ops(s, q)]
        if r == 1:  # the gradient is complete where it is produced: update in the epilogue
            st.enable_fused_wgrad_update()
        if native_exec is None:
            native_exec = self.device.type == "cuda"
        self.native_exec = bool(native_exec)
        if self.native_exec:
            st.compile_native()
        self.native_step = None
        self.native_fallback = None
        self.transport = "rccl" if mesh.backend == "nccl" else mesh.backend
        self.transport_reason = (f"fan layout {layout.describe()}: fan-in / fan-out P2P "
                                 f"({self.transport}), Python executor")
        if mesh.backend == "nccl" and self.native_exec and \
                switches.get("DNN_NATIVE_DIST") != "0":
            # the rank's whole step as one StepPlan call (fan.FanNativeStep, slotted RCCL form);
            # agreed over the world like the uniform mesh's native step (trainer.py)
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
        self._ipc_verify = None
        self._fallback_step = None
        self._graph = None
        self._graphs = []
        self._stream = None
        self.graph_nodes = 0
        self.steps_done = 0

    def set_global_batch(self, x: Optional[torch.Tensor], labels: Optional[torch.Tensor]):
        """The GLOBAL batch (all micro-batches); this rank keeps its own micro-batches' rows
        (first stage: inputs, last stage: labels)."""
        s, q = self.mesh.stage, self.mesh.replica
        rows = fan_rows(self.layout, s, q, self.num_micro, self.micro_batch)
        xs = gather_rows(x, rows) if self.first is not None else None
        ys = gather_rows(labels, rows) if self.last is not None else None
        self.set_batch(xs, ys)

    def loss(self) -> Optional[float]:
        """This replica's share of the global mean loss (the replicas' shares add up)."""
        if self.last is None:
            return None
        return self.last.loss_sum() / self.global_batch
