"""Training front-end: builds stages for a PP x DP layout and runs steps.

Two modes:

* local (``mesh=None``): every pipeline stage lives in this process on one device, joined by
  zero-copy loopback hops. ``pp=1`` is the single-GPU path; its whole step -- all GEMMs, the
  fused loss, wgrad reductions and the optimizer, ~20 kernels -- can be captured once into a
  HIP graph (:meth:`capture`) and replayed with a single launch per step.
* distributed (``mesh`` given): this rank owns stage ``mesh.stage`` of replica
  ``mesh.replica``; hops are RCCL send/recv and gradients are all-reduced over the stage's DP
  group, bucketed per layer and overlapped with the remaining weight-gradient GEMMs.

The micro-batching / schedule replaces the reference's one-request-at-a-time synchronous chain
(/root/reference/src/grpc_node.py:120-135); training itself is the reference's centralized
recipe (/root/reference/scripts/generate_mnist_pytorch.py:35-52: logits -> softmax CE ->
backward -> optimizer step) distributed over the stages.
"""
from __future__ import annotations

import os

from typing import Optional, Sequence

import numpy as np
import torch

from ..models.mlp import MLPSpec
from ..parallel.comm import DistPipe, IpcPipe, LoopbackPipe
from ..parallel.groups import Mesh
from ..parallel.pipeline import GradSync, PipelineExecutor
from ..partition import balanced_distribution, plan_stages
from ..utils.native import native
from .stage import OptimConfig, Stage
from .. import switches


def default_distribution(spec: MLPSpec, pp: int) -> list[int]:
    """Balanced contiguous split by per-layer training FLOPs."""
    return balanced_distribution([l.flops_per_sample_train for l in spec.layers], pp)


def _warm_groups(mesh: Mesh, device) -> None:
    """Make sure the RCCL communicators of this rank's groups exist (one tiny collective each,
    in global group-creation order: two ranks sharing groups meet them in the same order, so
    the warm-up cannot deadlock) before their handles are taken."""
    import torch.distributed as dist

    t = torch.zeros(1, device=device)
    groups = mesh.member_groups or [g for g in (mesh.fwd_group, mesh.bwd_group, mesh.dp_group)
                                    if g is not None]
    for g in groups:
        dist.all_reduce(t, group=g)
    torch.cuda.synchronize(device)


def _any_rank(flag: bool, device) -> bool:
    """True on every rank if ``flag`` is true on any rank (MAX all-reduce, world group)."""
    import torch.distributed as dist

    t = torch.tensor([1.0 if flag else 0.0],
                     device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return bool(t.item() > 0)


class Trainer:
    def __init__(self, spec: MLPSpec, *, micro_batch: int, num_micro: int = 1, pp: int = 1,
                 dp: int = 1, distribution: Optional[Sequence[int]] = None,
                 schedule: str = "1f1b", optim: Optional[OptimConfig] = None,
                 device: Optional[torch.device] = None, seed: int = 0,
                 mesh: Optional[Mesh] = None, wgrad: Optional[str] = None,
                 native_exec: Optional[bool] = None, boundary: str = "bf16",
                 dp_reduce: str = "allreduce"):
        self.spec = spec
        self.mesh = mesh
        self.device = device or (torch.device("cuda", torch.cuda.current_device())
                                 if torch.cuda.is_available() else torch.device("cpu"))
        if mesh is not None:
            pp, dp = mesh.pp, mesh.dp
        self.pp, self.dp = pp, dp
        dist_ = list(distribution) if distribution is not None else default_distribution(spec, pp)
        self.plans = plan_stages(len(spec.layers), dist_)
        if len(self.plans) != pp:
            raise ValueError(f"layer_distribution {dist_} has {len(self.plans)} non-empty "
                             f"stages but pp={pp}")
        self.distribution = dist_
        self.schedule = schedule
        self.micro_batch, self.num_micro = micro_batch, num_micro
        self.global_batch = micro_batch * num_micro * dp
        self.optim = optim or OptimConfig()
        wmode = wgrad or ("per_micro" if schedule in ("1f1b_w", "zb") else "batched")
        # data-parallel gradient exchange: "allreduce" (fp32 all-reduce, replicated optimizer)
        # or "shard" (bf16 reduce-scatter -> optimizer on this rank's 1/dp piece -> bf16
        # all-gather of the weights; pipeline.GradSync)
        if dp_reduce not in ("allreduce", "shard"):
            raise ValueError(f"dp_reduce must be allreduce | shard, got {dp_reduce!r}")
        # (a DP group of one rank -- mesh.dp_group set with dp == 1 -- runs the sharded path
        # with one piece per bucket: the single-GPU check of its native plan)
        self.dp_reduce = dp_reduce if (mesh is not None and mesh.dp_group is not None) \
            else "allreduce"
        shard = (mesh.dp, mesh.replica) if self.dp_reduce == "shard" else None
        mk = lambda p: Stage(spec, p.layer_start, p.layer_end, micro_batch=micro_batch,
                             num_micro=num_micro, device=self.device,
                             global_batch=self.global_batch, optim=self.optim, wgrad=wmode,
                             stage_index=p.stage, num_stages=pp, dp_shard=shard)
        if boundary not in ("bf16", "fp8"):
            raise ValueError(f"boundary must be bf16 | fp8, got {boundary!r}")
        self.boundary = boundary if (mesh is not None and pp > 1) else "bf16"
        self._ipc_verify = None  # set by _pick_pipe while the first IPC step is unverified
        self._fallback_step = None
        self.transport_reason = "loopback (one process)"
        if mesh is None:
            if boundary == "fp8" and pp > 1:
                raise ValueError("the fp8 boundary is a multi-rank hop format (loopback stages "
                                 "share their buffers; there is no hop to compress)")
            if dp != 1:
                raise ValueError("data parallelism needs a distributed mesh (one rank per GPU)")
            self.stages = [mk(p) for p in self.plans]
            for st in self.stages:
                st.params.init_default(seed)
            self.pipe = LoopbackPipe(self.stages)
            ids = [p.stage for p in self.plans]
            sync = None
        else:
            st = mk(self.plans[mesh.stage])
            st.params.init_default(seed)
            self.stages = [st]
            if boundary == "fp8" and mesh.pp > 1:  # e4m3 rows + fp32 row scales on the hops
                if switches.get("DNN_PIPE") == "ipc":
                    raise ValueError("the fp8 boundary runs on the message transport (rccl/gloo)")
                st.enable_fp8_boundary(mesh.prev_rank is not None, mesh.next_rank is not None)
            self.pipe = self._pick_pipe(mesh, st, boundary)
            ids = [mesh.stage]
            sync = (GradSync(mesh.dp_group, mesh.dp, shard=self.dp_reduce == "shard")
                    if mesh.dp > 1 or self.dp_reduce == "shard" else None)
        self.executor = PipelineExecutor(self.stages, self.pipe, schedule, pp, ids, sync)
        # one-split weight gradients update their weights in the GEMM epilogue (no DP: the
        # gradient is complete where it is produced)
        if mesh is None or (mesh.dp == 1 and self.dp_reduce != "shard"):
            for st in self.stages:
                st.enable_fused_wgrad_update()
        # native step executor: record each stage's launches once, replay from C++ (after the
        # pipe has aliased loopback buffers, so the recorded pointers are the final ones)
        if native_exec is None:
            native_exec = (self.device.type == "cuda" and
                           switches.get("DNN_NATIVE_EXEC") != "0")
        self.native_exec = bool(native_exec)
        if self.native_exec:
            for st in self.stages:
                st.compile_native()
        # native multi-rank step (parallel/native_step.py): the rank's whole step -- segment
        # replays, RCCL hops / xGMI peer copies, DP buckets -- as ONE C++ call per step
        self.native_step = None
        self.native_fallback = None
        self.transport = ("loopback" if mesh is None else
                          "ipc" if isinstance(self.pipe, IpcPipe) else
                          "rccl" if mesh.backend == "nccl" else mesh.backend)
        if mesh is not None and self.native_exec and \
                switches.get("DNN_NATIVE_DIST") != "0":
            from ..parallel.native_step import NativeStep, native_step_supported

            why = native_step_supported(self.executor, mesh)
            err = None
            if mesh.backend == "nccl":  # every rank (group collectives): before any handle
                _warm_groups(mesh, self.device)
            if why is None and self.transport in ("rccl", "ipc"):
                try:
                    if str(mesh.rank) in switches.get("DNN_FAULT_NATIVE_STEP").split(","):
                        raise RuntimeError("injected native-step construction fault")
                    self.native_step = NativeStep(self.executor, mesh, self.transport,
                                                  ipc=self.pipe if self.transport == "ipc"
                                                  else None)
                    if self._ipc_verify is not None and mesh.backend == "nccl":
                        # the verified IPC step's fallback: the RCCL plan, built up front, in
                        # the `slotted` form -- correct whatever the RCCL kernel residency, so
                        # the first step needs no co-residency assumption
                        self._fallback_step = NativeStep(self.executor, mesh, "rccl",
                                                         mode="slotted")
                except Exception as e:  # agreed on below: every rank falls back together
                    err = e
            # A rank running the native step and one running the Python executor would post
            # their hops on different communicators: all ranks agree (one collective over the
            # world group) and, if any rank could not build its native step (an error, or a
            # configuration it does not support), all of them use the Python executor instead
            # of failing or deadlocking the job.
            if _any_rank(self.native_step is None, self.device) and \
                    (self.native_step is not None or err is not None):
                import sys
                print(f"[trainer] rank {mesh.rank}: native multi-rank step unavailable "
                      f"({err!r} on this rank); every rank uses the Python executor",
                      file=sys.stderr, flush=True)
                self.native_fallback = repr(err) if err is not None else "another rank"
                self.native_step = None
            if self.native_step is not None:
                self.executor.native_step = self.native_step
            elif self._ipc_verify is not None:
                # DNN_PIPE=auto picked IPC but the native step is unavailable (a schedule it
                # does not support, hooks, a construction error): the message transport
                # (this must not raise for auto)
                self._use_fallback_pipe("IPC needs the native multi-rank step "
                                        f"({self.native_fallback or why})")
            elif isinstance(self.pipe, IpcPipe) and self.pipe.k:
                # relayed IPC hops exist only in the native step: name the cause here instead
                # of failing inside the first Python-executor step
                raise RuntimeError(
                    f"DNN_IPC_RELAYS={self.pipe.k} needs the native multi-rank step on every "
                    f"rank, which is unavailable ({self.native_fallback or why}); run with "
                    f"DNN_IPC_RELAYS=0 or fix the native step")
        if self._ipc_verify is not None and self.native_step is None:
            # the IPC step cannot be verified without the native step: message transport
            self._use_fallback_pipe("IPC needs the native multi-rank step "
                                    f"({self.native_fallback or 'native step disabled'})")
        self._graph = None
        self._stream = None
        self.graph_nodes = 0
        self.steps_done = 0

    # ---- pipeline transport --------------------------------------------------------------
    def _pick_pipe(self, mesh, st, boundary):
        """The hop transport of this rank (all ranks decide alike).

        DNN_PIPE=rccl: RCCL P2P (DistPipe). DNN_PIPE=ipc: xGMI peer writes into IPC-mapped,
        L2-uncached receive buffers with ``DNN_IPC_RELAYS`` relay stripes per hop (IpcPipe).
        DNN_PIPE=auto (default): IPC with relays (the planner's link model: a hop then draws
        on k + 1 xGMI links) on a real multi-GPU RCCL job, when every GPU can map its peers --
        VERIFIED on the first step: that step runs on both transports from the same state and
        the weights must agree bit for bit on every rank (``_verify_first_step``), else the job
        stays on RCCL. The chosen transport and the reason are in ``transport_reason``."""
        self._ipc_verify = None  # (ipc pipe, fallback pipe) while the first step is pending
        self._fallback_step = None
        mode = switches.get("DNN_PIPE")
        if mode not in ("auto", "ipc", "rccl"):
            raise ValueError(f"DNN_PIPE must be auto | ipc | rccl, got {mode!r}")
        if mode == "rccl" or self.device.type != "cuda" or mesh.pp < 2:
            self.transport_reason = ("DNN_PIPE=rccl" if mode == "rccl" else
                                     "no pipeline hops" if mesh.pp < 2 else "CPU ranks")
            return DistPipe(mesh, st)
        if boundary == "fp8":
            if mode == "ipc":
                raise ValueError("the fp8 boundary runs on the message transport (rccl/gloo)")
            self.transport_reason = "fp8 boundary (message transport)"
            return DistPipe(mesh, st)
        if mode == "auto" and mesh.backend != "nccl":
            self.transport_reason = f"{mesh.backend} ranks (auto picks IPC on RCCL jobs)"
            return DistPipe(mesh, st)
        if mode == "auto" and not self._peers_mappable(mesh):
            self.transport_reason = "a GPU pair of the plan has no peer access"
            return DistPipe(mesh, st)
        if mode == "auto" and self.schedule in ("1f1b_w", "zb"):
            self.transport_reason = (f"schedule {self.schedule} (per-micro-batch weight "
                                     "gradients: no native step, so no IPC)")
            return DistPipe(mesh, st)
        kr = switches.get("DNN_IPC_RELAYS")
        world = mesh.pp * mesh.dp
        hwq = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
        if kr == "auto":  # per-hop relay counts from the directed-link load model
            k = self.relay_table(mesh, max_duties=max(0, min(6, hwq - 6)))
        else:
            k = int(kr)
        verify = switches.get("DNN_IPC_VERIFY")
        verify = mode == "auto" if verify == "auto" else verify == "1"
        try:
            ipc = IpcPipe(mesh, st, relays=k)
        except RuntimeError as e:  # raised on every rank together (comm.IpcPipe)
            if mode == "ipc":
                raise
            self.transport_reason = f"IPC set-up failed: {e}"[:300]
            return DistPipe(mesh, st)
        # Every rank reaches this point (all earlier exits are agreed), and the queue check
        # must be agreed too: with an explicit DNN_IPC_RELAYS=k ranks carry different relay
        # duty counts, and a rank that fell back alone would free relay slots its peers have
        # mapped and still write into. Decide on the busiest rank's count.
        if mode == "auto":
            import torch.distributed as dist

            from ..parallel.comm import _cpu_group

            tt = torch.tensor([len(ipc.duties), -hwq], dtype=torch.int64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=_cpu_group())
            most_duties, least_hwq = int(tt[0].item()), -int(tt[1].item())
            if 4 + most_duties > least_hwq:
                ipc.close()
                self.transport_reason = (f"IPC plan needs {4 + most_duties} hardware queues on "
                                         f"its busiest rank, GPU_MAX_HW_QUEUES={least_hwq}")
                return DistPipe(mesh, st)
        kdesc = (f"{k} relays per hop" if isinstance(k, int) else
                 "per-hop relays " + "/".join(str(len(v)) for h, v in sorted(k.items())
                                              if h[2] == "f" and h[0] < mesh.pp))
        self.transport_reason = (f"ipc, {kdesc}" +
                                 (" (verification pending: first step)" if verify else ""))
        if verify:
            self._ipc_verify = (ipc, DistPipe(mesh, st))
        return ipc

    def relay_table(self, mesh, max_duties: int = 6) -> dict:
        """comm.relay_plan for this job: per step, every boundary hop moves rows x padded
        width x 2 bytes each way and every stage's DP group exchanges its bf16 gradient and
        weights; the same table on every rank (a pure function of the layout)."""
        from ..models.mlp import round_up
        from ..parallel.comm import relay_plan

        rows = self.micro_batch * self.num_micro
        hop_bytes = [rows * round_up(self.spec.layers[p.layer_end - 1].out_dim, 64) * 2
                     for p in self.plans[:-1]]
        dp_bytes = [2 * (mesh.dp - 1) / mesh.dp * 2 *
                    sum(l.params for l in self.spec.layers[p.layer_start:p.layer_end])
                    for p in self.plans]
        return relay_plan(mesh.pp, mesh.dp, hop_bytes, dp_bytes=dp_bytes,
                          max_k=min(6, mesh.pp * mesh.dp - 2), max_duties=max_duties)

    def _peers_mappable(self, mesh) -> bool:
        """Every rank can map every other rank's GPU (one rank per GPU on one node; a relay can
        be any rank), agreed over the world."""
        import torch.distributed as dist

        from ..parallel.comm import _cpu_group

        n = native()
        ndev = torch.cuda.device_count()
        me = self.device.index if self.device.index is not None else torch.cuda.current_device()
        devs = [None] * dist.get_world_size()
        dist.all_gather_object(devs, me, group=_cpu_group())
        ok = all(n.can_access_peer(me, d) for d in devs if d is not None and d < ndev) and \
            len(set(devs)) == len(devs)  # ranks sharing a GPU: not a multi-GPU job
        t = torch.tensor([0 if ok else 1], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=_cpu_group())
        return int(t.item()) == 0

    def _use_fallback_pipe(self, why: str) -> None:
        ipc, fb = self._ipc_verify
        self._ipc_verify = None
        ipc.close()
        self.pipe = fb
        self.executor.pipe = fb
        self.transport = "rccl" if self.mesh.backend == "nccl" else self.mesh.backend
        self.native_step = self._fallback_step
        self.executor.native_step = self._fallback_step
        self._fallback_step = None
        mode = getattr(self.native_step, "mode", None) if self.native_step is not None else None
        self.transport_reason = (f"{self.transport}{', ' + mode if mode else ''} "
                                 f"(IPC not used: {why})")[:300]

    def _state_tensors(self) -> list:
        out = []
        for st in self.stages:
            p = st.params
            out += [p.master, p.shadow, *p.state, *p.wt.values()]
            for name in ("lr_dev", "step_dev"):
                t = getattr(p, name, None)
                if isinstance(t, torch.Tensor):
                    out.append(t)
        return out

    def _verify_first_step(self) -> None:
        """Run the first step on the IPC plan, then from the same state on the fallback
        transport; keep IPC only if every rank's weights agree bit for bit (the two move the
        same bytes) and no flag wait timed out. The fallback's step is the one kept."""
        import sys

        import torch.distributed as dist

        from ..parallel.comm import _cpu_group

        state = self._state_tensors()
        snap = [t.clone() for t in state]
        counts = [st.params.step_count for st in self.stages]
        # a stalled IPC plan must report well inside bench.py's first-step bound; steady state
        # keeps the long flag-wait timeout
        plan = self.native_step.plan if self.native_step is not None else None
        long_timeout = plan.wait_timeout if plan is not None else None
        if plan is not None:
            plan.wait_timeout = float(switches.get("DNN_VERIFY_FLAG_TIMEOUT"))
        try:
            self.executor.run_step()  # IPC
            torch.cuda.synchronize(self.device)
        finally:
            if plan is not None:
                plan.wait_timeout = long_timeout
        ipc_state = [t.clone() for t in state]
        timeouts = self.native_step.comm_error() if self.native_step is not None else 0
        if str(self.mesh.rank) in switches.get("DNN_FAULT_IPC_VERIFY").split(","):
            ipc_state[0].view(-1)[0] += 1.0  # injected corruption (tests the fallback branch)
        for t, v in zip(state, snap):
            t.copy_(v)
        for st, c in zip(self.stages, counts):
            st.params.step_count = c
        ipc_ns, ipc_pipe = self.native_step, self.pipe
        fb = self._ipc_verify[1]
        self.executor.native_step = self._fallback_step
        self.executor.pipe = fb
        self.executor.run_step()  # fallback transport, same state and batch
        torch.cuda.synchronize(self.device)
        same = timeouts == 0 and all(torch.equal(a, b) for a, b in zip(ipc_state, state))
        t = torch.tensor([0 if same else 1], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=_cpu_group())
        if int(t.item()) == 0:
            self.executor.native_step = ipc_ns
            self.executor.pipe = ipc_pipe
            self._ipc_verify = None
            self._fallback_step = None
            self.transport_reason = self.transport_reason.replace(
                "(verification pending: first step)",
                "(first step verified bitwise against the fallback transport)")
        else:
            self._use_fallback_pipe("the first step's weights differed from the fallback "
                                    "transport's on a rank" if timeouts == 0 else
                                    "a flag wait timed out in the first step")
            print(f"[trainer] rank {self.mesh.rank}: {self.transport_reason}", file=sys.stderr,
                  flush=True)

    # -------------------------------------------------------------------------------------
    @property
    def first(self) -> Optional[Stage]:
        return self.stages[0] if self.stages[0].first else None

    @property
    def last(self) -> Optional[Stage]:
        return self.stages[-1] if self.stages[-1].last else None

    def set_batch(self, x: Optional[torch.Tensor], labels: Optional[torch.Tensor],
                  zero_copy: bool = False) -> None:
        """x: this replica's [rows][Kp] bf16 inputs; labels: [rows] int32 (-1 = padding).

        ``zero_copy`` (eager mode only): the first stage reads ``x`` in place -- e.g. a row
        slice of an HBM-resident dataset -- instead of copying it into its input buffer."""
        if self.first is not None:
            if x is None:
                raise ValueError("first stage needs inputs")
            st = self.first
            if zero_copy and self._graph is None and x.shape == st.x_buf.shape and \
                    x.dtype == st.x_buf.dtype and x.device == st.x_buf.device and \
                    x.stride(1) == 1 and x.data_ptr() % 16 == 0 and len(self.stages) == 1:
                st.bind_input(x)
            else:
                st.bind_input(st.x_buf)  # never write through an alias of a previous batch
                st.x_in.copy_(x)
        if self.last is not None:
            if labels is None:
                raise ValueError("last stage needs labels")
            st = self.last
            if zero_copy and self._graph is None and labels.shape == st.labels_buf.shape and \
                    labels.dtype == st.labels_buf.dtype and \
                    labels.device == st.labels_buf.device and labels.is_contiguous():
                st.bind_labels(labels)
            else:
                st.bind_labels(st.labels_buf)
                st.labels.copy_(labels)

    def step(self) -> None:
        if self._graph is not None:
            cur = torch.cuda.current_stream(self.device)
            for st in self.stages:  # the captured update reads the learning rate from device
                st.params.set_lr(st.params.optim.lr)
            self._stream.wait_stream(cur)  # inputs (and lr) written on the caller's stream
            # alternate between identical instantiations: relaunching the SAME exec before its
            # previous launch retired makes the host wait (measured ~130 us idle per step)
            g = self._graphs[self.steps_done % len(self._graphs)]
            g.replay(self._stream.cuda_stream)
            cur.wait_stream(self._stream)
            for st in self.stages:  # the captured update advanced the device step counter
                st.params.step_count += 1
        elif self._ipc_verify is not None:
            self._verify_first_step()
        else:
            self.executor.run_step()
        self.steps_done += 1

    def capture(self, warmup: int = 1, copies: int = 2) -> None:
        """Capture one full training step into a HIP graph (local mode, GPU only).

        Every buffer is allocated up front, so replay touches fixed pointers. The capture runs
        on a private stream (the legacy null stream cannot be captured); replay is ordered
        against the caller's stream with events. Capturing executes the step once for real."""
        if self.device.type != "cuda" or (self.mesh is not None and self.native_step is None):
            raise RuntimeError("graph capture needs the local GPU path or a native "
                               "multi-rank step (parallel/native_step.py)")
        if self._ipc_verify is not None:
            # never capture (and replay) an unverified relayed-IPC plan: the first
            # step runs the verification, which may switch the transport
            self.step()
            if self.mesh is not None and self.native_step is None:
                raise RuntimeError("graph capture needs a native multi-rank step; the IPC "
                                   "verification fell back to the Python executor")
        ns = self.native_step
        if ns is not None and ns.mode == "ipc":
            # the multi-stream IPC plan spins on flags in branches that other branches (and
            # other ranks) release; a graph executor may order independent branches any way
            # it likes (the captured relayed step stalled: VERDICT r3 #4). The slotted form is
            # ONE stream in global clock order, so its graph is a single chain that completes
            # whatever the executor does (parallel/native_step._build_ipc_slotted).
            from ..parallel.native_step import NativeStep

            self.native_step = NativeStep(self.executor, self.mesh, "ipc", ipc=self.pipe,
                                          mode="slotted")
            self.executor.native_step = self.native_step
        cur = torch.cuda.current_stream(self.device)
        # an eager step before the capture may have left its cross-step side-stream tail (the
        # reduce + update of layers 1..L-1) running: order the capture after it, and start the
        # cross-step chain afresh when eager steps resume
        self.executor.xstep_join()
        self.executor._xprimed = False
        self._stream = torch.cuda.Stream(self.device)
        self._stream.wait_stream(cur)
        if self.first is not None and self.first.x_in.data_ptr() != self.first.x_buf.data_ptr():
            self.first.x_in = self.first.x_buf  # a graph needs the fixed input buffer
        graphs = []
        self.executor.capturing = True  # single-stream plan: the graph serialises anyway
        with torch.cuda.stream(self._stream):
            for _ in range(warmup):
                self.executor.run_step()
            self._stream.synchronize()
            counts = [st.params.step_count for st in self.stages]
            for _ in range(max(1, copies)):
                g = native().GraphExec()
                g.begin_capture(self._stream.cuda_stream)
                try:
                    self.executor.run_step()
                finally:
                    g.end_capture()
                graphs.append(g)
            graphs[0].replay(self._stream.cuda_stream)  # capture itself executes nothing
        for st, c in zip(self.stages, counts):  # `copies` captures, ONE executed step
            st.params.step_count = c + 1
        cur.wait_stream(self._stream)
        self._graphs = graphs
        self._graph = graphs[0]
        self.graph_nodes = graphs[0].num_nodes
        torch.cuda.synchronize(self.device)
        ns = self.native_step
        if ns is not None:  # captures advanced only the host mirror of the step number
            ns.plan.sync_seq()
            if ns.ipc is not None:
                ns.ipc.seq = ns.plan.seq

    def release_graph(self) -> None:
        self._graph = None
        self._graphs = []
        ns = self.native_step
        if ns is not None:  # replays advanced the device step number only
            torch.cuda.synchronize(self.device)
            ns.plan.sync_seq()
            if ns.ipc is not None:
                ns.ipc.seq = ns.plan.seq

    # -------------------------------------------------------------------------------------
    def loss(self) -> Optional[float]:
        """Mean loss of the last step (this replica's share scaled to the global batch)."""
        if self.last is None:
            return None
        return self.last.loss_sum() / (self.micro_batch * self.num_micro)

    def correct(self) -> Optional[int]:
        return None if self.last is None else int(self.last.correct.sum().item())

    def load_weights(self, weights: Sequence[np.ndarray], biases: Sequence[np.ndarray]) -> None:
        for st in self.stages:
            st.params.load(weights[st.l0:st.l1], biases[st.l0:st.l1])

    def flush(self) -> None:
        """Complete every deferred data-parallel update (parallel/pipeline.dp_split): call
        before reading weights or ending a timed region; training steps need not."""
        self.executor.flush()

    def gather_sharded(self) -> None:
        """Sharded DP: make the fp32 master weights and optimizer state whole on every rank
        (each rank updates only its pieces); before export / checkpoint."""
        if self.dp_reduce == "shard":
            for st in self.stages:
                st.params.gather_full(self.mesh.dp_group)

    def local_weights(self) -> dict[int, tuple[np.ndarray, np.ndarray]]:
        self.flush()
        self.gather_sharded()
        out = {}
        for st in self.stages:
            ws, bs = st.params.export()
            for k, (w, b) in enumerate(zip(ws, bs)):
                out[st.l0 + k] = (w, b)
        return out

    def flops_per_step(self) -> float:
        """Model FLOPs of one global step across all ranks (padding excluded)."""
        return float(self.spec.flops_per_sample_train()) * self.global_batch
