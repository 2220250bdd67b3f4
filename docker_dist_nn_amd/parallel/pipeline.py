"""Executes pipeline schedules (csrc/runtime/schedule.cpp) over stages and transports.

For a rank that owns one stage, the schedule's op list runs in order:

  F(j): recv activation j -> stage.forward(j) -> send activation j
  B(j): recv gradient  j -> stage.backward(j) -> send gradient j
  W(j): stage.wgrad(j)            (W(-1): one batch-contraction GEMM per layer over all rows)
  O   : finalize grads -> data-parallel all-reduce -> fused optimizer

When the step ends with a batched W, the weight gradients are produced layer by layer from the
last layer backwards and each layer's gradient bucket is all-reduced asynchronously (RCCL
stream) while the next layer's wgrad GEMM runs -- the DP traffic overlaps compute.

For several stages in ONE process (loopback), ops of all stages are interleaved in a
dependency-respecting order (F(s,j) after F(s-1,j); B(s,j) after B(s+1,j)), which both runs
S-stage pipelines on one device and checks that the schedules are deadlock-free.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import torch
import torch.distributed as dist

from ..utils.native import native
from .. import switches


def schedule_ops(kind: str, num_stages: int, num_micro: int, stage: int):
    n = native()
    out = []
    for op in n.make_schedule(kind, num_stages, num_micro, stage):
        out.append(({n.OpKind.FWD: "F", n.OpKind.BWD: "B", n.OpKind.WGRAD: "W",
                     n.OpKind.OPT: "O"}[op.kind], op.micro))
    return out


class GradSync:
    """Bucketed, asynchronous gradient all-reduce over the data-parallel group.

    ``shard=True``: sharded data parallelism instead (StageParams.shard_piece): per bucket a
    bf16 reduce-scatter of the gradient, the optimizer on this rank's piece only, and a bf16
    all-gather of the updated shadow weights -- half the bytes of the fp32 all-reduce."""

    def __init__(self, group, world: int, shard: bool = False):
        self.group = group
        self.world = world
        self.shard = shard
        self._works = []

    def reduce_scatter(self, p, e0: int, e1: int):
        """Async bf16 reduce-scatter of bucket [e0, e1) of p.grad16 into p.grad_piece."""
        d = self.world
        w = dist.reduce_scatter_tensor(p.grad_piece[e0 // d:e1 // d], p.grad16[e0:e1],
                                       group=self.group, async_op=True)
        self._works.append(w)
        return w

    def all_gather_shadow(self, p, e0: int, e1: int):
        p0, p1 = p.shard_piece(e0, e1)
        w = dist.all_gather_into_tensor(p.shadow[e0:e1], p.shadow[p0:p1], group=self.group,
                                        async_op=True)
        self._works.append(w)
        return w

    def launch(self, flat_grad, start: int, end: int):
        """Async all-reduce of flat_grad[start:end]; returns the work handle (also kept for
        wait())."""
        if self.world <= 1 and not self.shard:
            return None
        w = dist.all_reduce(flat_grad[start:end], group=self.group, async_op=True)
        self._works.append(w)
        return w

    def wait(self) -> None:
        for w in self._works:
            w.wait()
        self._works.clear()

    def wait_one(self, w) -> None:
        """Order the current stream after one bucket's all-reduce (others stay in flight)."""
        if w is not None:
            w.wait()
            self._works = [x for x in self._works if x is not w]


def dp_split(st) -> int:
    """Layer split s of a stage for the deferred data-parallel update: layers [0, s) are
    all-reduced and updated at the end of the step; layers [s, L) are all-reduced behind the
    NEXT step's forward of [0, s) and updated just before that forward reaches layer s. The
    split puts about half the gradient bytes on each side (first layer range holding >= 50 %);
    0 = no split (one layer)."""
    L = len(st.geoms)
    if L < 2:
        return 0
    size = [st.geoms[i].np_ * st.geoms[i].kp + st.geoms[i].np_ for i in range(L)]
    tot, cum = sum(size), 0
    for i in range(L - 1):
        cum += size[i]
        if 2 * cum >= tot:
            return i + 1
    return L - 1


def dp_buckets(st, cap_bytes: int = 4 << 20) -> list[list[int]]:
    """Data-parallel gradient buckets of a stage, in launch order.

    The largest layer's gradient goes first and alone: its all-reduce -- the longest on the
    xGMI ring -- then overlaps every other layer's wgrad GEMM. The remaining layers are merged
    into runs of consecutive layer indices (a contiguous range of the flat gradient, so one
    RCCL call and one reduce launch each), last layers first, up to ``cap_bytes`` of fp32
    gradient per bucket: few, larger collectives instead of one latency-bound call per layer.
    """
    L = len(st.geoms)
    size = [4 * (st.geoms[i].np_ * st.geoms[i].kp + st.geoms[i].np_) for i in range(L)]
    big = max(range(L), key=lambda i: size[i])
    out = [[big]]
    run: list[int] = []
    for i in range(L - 1, -1, -1):
        if i == big or (run and (run[0] - 1 != i or sum(size[j] for j in run) + size[i] >
                                 cap_bytes)):
            if run:
                out.append(sorted(run))
            run = []
            if i == big:
                continue
        run.insert(0, i)
    if run:
        out.append(sorted(run))
    return out


class PipelineExecutor:
    def __init__(self, stages: Sequence, pipe, kind: str, num_stages: int,
                 stage_ids: Sequence[int], grad_sync: Optional[GradSync] = None,
                 lr_fn: Optional[Callable[[], float]] = None):
        self.stages = list(stages)
        self.pipe = pipe
        self.kind = kind
        self.S = num_stages
        self.stage_ids = list(stage_ids)
        self.grad_sync = grad_sync
        self.lr_fn = lr_fn
        self.ops = [schedule_ops(kind, num_stages, st.nm, sid)
                    for st, sid in zip(self.stages, self.stage_ids)]
        self.hooks: dict[str, list[Callable]] = {"before_op": [], "after_op": []}
        # concurrent wgrad streams in native single-process plans (DNN_WGRAD_STREAMS)
        self.wgrad_streams = int(switches.get("DNN_WGRAD_STREAMS"))
        self._side = None
        # deferred data-parallel update (DNN_DP_DEFER=0 disables): see dp_split
        self.defer = (grad_sync is not None and grad_sync.world > 1 and
                      not grad_sync.shard and switches.get("DNN_DP_DEFER") != "0")
        self._split = {id(st): (dp_split(st) if self.defer else 0) for st in self.stages}
        self._pending = {}  # id(stage) -> (work of layers [s, L), s)
        self._works = {}    # id(stage) -> [work of [0, s), work of [s, L)] this step

    # ---------------------------------------------------------------------------------------
    def _run_op(self, st, op, j, next_op=None):
        for h in self.hooks["before_op"]:
            h(st, op, j)
        if op == "F":
            self.pipe.recv_fwd(st, j)
            pend = self._pending.pop(id(st), None)
            if pend is not None:  # first forward of the step: finish last step's update
                work, sp = pend
                st.forward_layers(j, 0, sp)
                self.grad_sync.wait_one(work)
                st.update_then_forward(j, sp, self.lr_fn() if self.lr_fn else None)
            else:
                st.forward(j)
            self.pipe.send_fwd(st, j)
        elif op == "B":
            self.pipe.recv_bwd(st, j)
            st.backward(j)
            self.pipe.send_bwd(st, j)
        elif op == "W":
            if j < 0 and next_op == "O":
                self._wgrad_finalize_overlapped(st)
            else:
                st.wgrad(j)
        elif op == "O":
            sp = self._split.get(id(st), 0)
            if sp:
                self._optimizer_deferred(st, sp)
                return self._after(st, op, j)
            if self.grad_sync is not None and self.grad_sync.shard:
                self._sharded_update(st)
                return self._after(st, op, j)
            if not getattr(st, "_finalized", False):
                st.finalize_grads()
                if self.grad_sync is not None:
                    self.grad_sync.launch(st.params.grad, 0, st.params.numel)
            if self.grad_sync is not None:
                self.grad_sync.wait()
            st._finalized = False
            st.optimizer_step(self.lr_fn() if self.lr_fn else None)
        self._after(st, op, j)

    def _after(self, st, op, j):
        for h in self.hooks["after_op"]:
            h(st, op, j)

    def _shard_buckets(self, st) -> list[tuple[list[int], int, int]]:
        """(layers, e0, e1) of every DP bucket of a sharded stage, in launch order."""
        out = []
        for bucket in dp_buckets(st):
            e0, _ = st.params.layer_grad_range(bucket[0])
            _, e1 = st.params.layer_grad_range(bucket[-1])
            out.append((bucket, e0, e1))
        st.params.shard_buckets = [(e0, e1) for _, e0, e1 in out]
        return out

    def _sharded_update(self, st) -> None:
        """O of a sharded stage: (buckets reduce-scattered in _wgrad_finalize_overlapped, or
        now for per-micro-batch W schedules) -> unpack + update this rank's piece of every
        bucket -> all-gather the bf16 shadow -> refresh W^T."""
        gs, p = self.grad_sync, st.params
        buckets = self._shard_buckets(st)
        if not getattr(st, "_finalized", False):
            st.finalize_grads()
            for _, e0, e1 in buckets:
                p.shard_pack(e0, e1)
                gs.reduce_scatter(p, e0, e1)
            gs.launch(p.grad, p.bias_lo, p.numel)
        gs.wait()
        st._finalized = False
        lr = self.lr_fn() if self.lr_fn else None
        for _, e0, e1 in buckets:
            st.shard_update(e0, e1, lr)
        st.bias_update(lr)
        if p.optim.name != "sgd":  # the step's one device-counter advance (Adam)
            if p.device.type == "cuda":
                from .. import ops

                ops.step_advance(p.step_dev)
        p.step_count += 1
        for _, e0, e1 in buckets:
            gs.all_gather_shadow(p, e0, e1)
        gs.wait()
        p.refresh_t()

    def _optimizer_deferred(self, st, sp: int) -> None:
        """O with a deferred split: all-reduce [0, sp) must be done -> update it now; the
        [sp, L) all-reduce stays in flight until the next step's first forward (or flush)."""
        L = len(st.geoms)
        works = self._works.pop(id(st), None)
        if works is None or not getattr(st, "_finalized", False):  # per-micro W schedules
            st.finalize_grads()
            a0, a1 = st.params.layers_range(0, sp)
            b0, b1 = st.params.layers_range(sp, L)
            works = [self.grad_sync.launch(st.params.grad, a0, a1),
                     self.grad_sync.launch(st.params.grad, b0, b1)]
        st._finalized = False
        self.grad_sync.wait_one(works[0])
        st.update_layers(0, sp, self.lr_fn() if self.lr_fn else None, advance=False)
        self._pending[id(st)] = (works[1], sp)

    def flush(self) -> None:
        """Apply every deferred update now (end of training / before reading weights)."""
        self.xstep_join()
        for st in self.stages:
            pend = self._pending.pop(id(st), None)
            if pend is not None:
                work, sp = pend
                self.grad_sync.wait_one(work)
                st.update_layers(sp, len(st.geoms), self.lr_fn() if self.lr_fn else None,
                                 advance=True)

    def _wgrad_finalize_overlapped(self, st):
        """Batched W: per layer (last first) wgrad -> reduce -> async bucket all-reduce. Without
        a DP group there is nothing to overlap: all wgrads, then ONE reduce launch."""
        if self.grad_sync is None or (self.grad_sync.world <= 1 and not self.grad_sync.shard):
            for i in range(len(st.geoms) - 1, -1, -1):
                st.wgrad_layer(i)
            st.finalize_grads()
            st._finalized = True
            return
        sp = self._split.get(id(st), 0)
        if sp:  # deferred update: [0, sp) first (needed at O), then [sp, L)
            L = len(st.geoms)
            works = []
            for a, b in ((0, sp), (sp, L)):
                st.wgrad_finalize(list(reversed(range(a, b))))  # one native call per bucket
                e0, e1 = st.params.layers_range(a, b)
                works.append(self.grad_sync.launch(st.params.grad, e0, e1))
            self._works[id(st)] = works
            st._finalized = True
            return
        if self.grad_sync.shard:  # bf16 reduce-scatter per bucket, overlapping later wgrads
            for bucket, e0, e1 in self._shard_buckets(st):
                for i in bucket:
                    st.wgrad_layer(i)
                st.finalize_grads(bucket)
                st.params.shard_pack(e0, e1)
                self.grad_sync.reduce_scatter(st.params, e0, e1)
            p = st.params  # every bias gradient: one small fp32 all-reduce
            self.grad_sync.launch(p.grad, p.bias_lo, p.numel)
            st._finalized = True
            return
        for bucket in dp_buckets(st):
            for i in bucket:
                st.wgrad_layer(i)
            st.finalize_grads(bucket)  # one reduce launch per bucket
            a, _ = st.params.layer_grad_range(bucket[0])
            _, b = st.params.layer_grad_range(bucket[-1])
            self.grad_sync.launch(st.params.grad, a, b)  # contiguous flat range
        st._finalized = True

    def _native_plan(self):
        """For an all-native loopback step (one process, no DP, batched wgrad, SGD): the
        schedule's op order as (stage, segment) pairs, computed once by a dry traversal of
        the same dispatch rules as _run_op. None when any op needs the Python path."""
        if getattr(self, "_plan", False) is not False:
            return self._plan
        from .comm import LoopbackPipe

        self._plan = None
        if switches.get("DNN_NATIVE_PLAN") == "0":  # per-op replay (A/B, host cost)
            return None
        if not isinstance(self.pipe, LoopbackPipe) or self.grad_sync is not None or \
                self.hooks["before_op"] or self.hooks["after_op"] or self.lr_fn is not None:
            return None
        if any(st._prog is None or not st._has_w or not st._o_native for st in self.stages):
            return None
        mode = switches.get("DNN_BW_OVERLAP")
        # small steps are host-bound: every fork / join is an event record + wait (~6-8 us of
        # host time each), more than the overlap can win back on GEMMs of a few thousand rows
        if mode in ("1", "5") and len(self.stages) == 1 and \
                self.stages[0].rows >= int(switches.get("DNN_BW_OVERLAP_MIN_ROWS")):
            ov = self._overlap_plan(self.stages[0], mode)
            if ov is not None:
                self._plan = ov
                return ov
        order = []
        self._traverse(lambda s, op, j, nxt: order.append((s, op, j, nxt)))
        plan = []
        for s, op, j, nxt in order:
            st = self.stages[s]
            if op in ("F", "B"):
                plan.append((st, f"{op}{j}"))
            elif op == "W":
                if j >= 0:
                    return None
                if nxt == "O":  # as _wgrad_finalize_overlapped without a DP group
                    L = len(st.geoms)
                    if self.wgrad_streams > 1 and L > 1:
                        # the biggest layer's wgrad on the main stream, the rest concurrently
                        # on the side stream (independent GEMMs; small ones alone leave the
                        # chip idle), joined before the one reduction launch
                        big = max(range(L), key=lambda i: st.geoms[i].np_ * st.geoms[i].kp)
                        plan.append((None, "@fork"))
                        plan += [(st, f"W{i}", 1) for i in range(L - 1, -1, -1) if i != big]
                        plan.append((st, f"W{big}"))
                        plan.append((None, "@join"))
                    else:  # one segment: a grouped launch when the layers share a tile
                        plan.append((st, "W"))
                    plan.append((st, "FIN"))
                    plan.append((st, "#finalized"))
                else:
                    plan.append((st, "W"))
            elif op == "O":
                if (st, "#finalized") not in plan:
                    plan.append((st, "FIN"))
                plan.append((st, "O"))
        # a stage's whole-step reduction followed by its SGD update: one fused launch (FINO)
        # when recorded (Stage.fused_fin_sgd_ok); nothing of that stage runs in between
        fused = []
        for e in plan:
            st, seg = e[0], e[1]
            if seg == "O" and st is not None and "FINO" in st._prog.segments():
                k = max(i for i, f in enumerate(fused) if f[0] is st and f[1] == "FIN")
                fused[k] = (st, "FINO") + tuple(fused[k][2:])
                continue
            fused.append(e)
        self._plan = [(e[0], e[1], e[2] if len(e) > 2 else 0) for e in fused
                      if not e[1].startswith("#")]
        return self._plan

    def _overlap_plan(self, st, mode: str = "1"):
        """Single stage, one micro-batch: each layer's weight-gradient GEMM runs on the side
        stream while the main stream computes the next dgrad (wgrad_i needs dZ_i, which is
        ready before dgrad_i starts), so a memory-bound dgrad and a wgrad fill each other's
        tails. Ends with a join, the first layer's wgrad and the gradient reduction/update.

        Mode "5" (opt-in): the small wgrads on the side stream, W1 and W0 on the main stream.
        The other variants measured over rounds 2-5 (one fork with every side wgrad under the
        dgrads or under W0, W1 first on the side, fork elision, a delay kernel instead of event
        packets, stream priorities, an early join, a workgroup cap on the side reduction) lost
        or tied and were removed in round 6 (profiles/r6_prune)."""
        segs = st._prog.segments()
        if st.nm != 1 or not st.first or not st.last or "W0" not in segs:
            return None
        L = len(st.geoms)
        fused = st.params.fused_layers  # their wgrad also UPDATES W_i and W_i^T
        # auto: on unless a layer updates in its wgrad epilogue (the wide model: there the
        # side-stream update of layers 1.. competes with the fused W1; profiles/r3b_fino)
        sf = switches.get("DNN_SPLIT_FINO")
        split = ((sf == "1" or (sf == "auto" and not fused)) and L > 1 and
                 f"FINO1-{L - 1}" in segs and "FINO0-0" in segs and 0 not in fused)
        if mode == "5" and L >= 3 and not fused:
            # one fork: the small wgrads (L-1 .. 2) on the side under the dgrads; W1 on the
            # main stream right after the last dgrad, then W0 -- so W1 and W0 never share the
            # chip whatever the dgrads cost (with the fragment-mask dgrad the default plan lets
            # W0 start before W1: profiles/r4_timeline)
            plan = self._mode5_head(st, L) + [(st, "W1", 0)]
            if split:
                return plan + [(None, "@fork", 0), (st, f"FINO1-{L - 1}", 1), (st, "W0", 0),
                               (st, "FINO0-0", 0), (None, "@join", 0)]
            plan += [(st, "W0", 0), (None, "@join", 0)]
            plan.append((st, "FINO", 0) if "FINO" in segs else (st, "FIN", 0))
            if "FINO" not in segs:
                plan.append((st, "O", 0))
            return plan
        plan = [(st, "F0", 0), (None, "@fork", 0)]
        for i in range(L - 1, 0, -1):
            if i in fused:  # dgrad_i reads the old W_i^T: the updating wgrad_i starts after it
                plan += [(st, f"B0.L{i}", 0), (None, "@fork", 0), (st, f"W{i}", 1)]
            else:
                plan += [(st, f"W{i}", 1), (st, f"B0.L{i}", 0), (None, "@fork", 0)]
        if plan[-1][1] == "@fork" and not split:
            plan = plan[:-1]
        if split:
            # the side stream reduces + updates layers 1..L-1 (their wgrads are done; the fork
            # above orders it after the last dgrad, the last reader of their W^T) while the
            # main stream runs W0; then only layer 0's reduction + update is left at the end
            if plan[-1][1] != "@fork":
                plan.append((None, "@fork", 0))
            plan += [(st, f"FINO1-{L - 1}", 1), (st, "W0", 0)]
            return plan + [(st, "FINO0-0", 0), (None, "@join", 0)]
        plan += [(st, "W0", 0), (None, "@join", 0)]
        plan.append((st, "FINO", 0) if "FINO" in segs else (st, "FIN", 0))
        if "FINO" not in segs:
            plan.append((st, "O", 0))
        return plan

    @staticmethod
    def _mode5_head(st, L: int):
        """Forward, then the small wgrads W{L-1} .. W2 on the side stream and every dgrad on
        the main stream (overlap mode 5). W_i reads dZ_i, which the dgrad of layer i+1
        (B0.L{i+1}) writes -- or the forward F0, when i = L-1 or when the classifier tail
        already ran that dgrad (an empty segment). So before each side W_i whose dZ comes from
        a real dgrad, that dgrad is placed on the main stream and a fresh fork orders the side
        stream after it (a single fork after F0 let W_i race the dgrad producing its
        input for L >= 5, or L = 4 without the tail)."""
        plan = [(st, "F0", 0)]
        emitted, fork_due = set(), True
        for i in range(L - 1, 1, -1):
            src = i + 1  # the dgrad writing dZ_i (none for the last layer: F0 does)
            if src <= L - 1 and src not in emitted:
                plan.append((st, f"B0.L{src}", 0))
                emitted.add(src)
                if st._prog.segment_size(f"B0.L{src}") > 0:
                    fork_due = True  # the side stream must wait for this dgrad
            if fork_due:
                plan.append((None, "@fork", 0))
                fork_due = False
            plan.append((st, f"W{i}", 1))
        plan += [(st, f"B0.L{i}", 0) for i in range(L - 1, 0, -1) if i not in emitted]
        return plan

    def _loopback_step_plan(self, plan):
        """Several stages in one process (loopback): run each stage on ITS OWN stream, with an
        event edge per micro-batch hop (F(s, j) after F(s-1, j); B(s, j) after B(s+1, j)).
        Stages then execute concurrently on the one GPU like a real pipeline, instead of the
        whole schedule serialised on one stream: micro-batch GEMMs are small (a 4-stage,
        16-micro-batch step at 65536 rows runs 4096-row GEMMs) and fill the chip only together.
        Built once into a StepPlan (csrc/runtime/step_plan.hpp): one C++ call per step."""
        from .native_step import REC, SEG, WAIT

        S = len(self.stages)
        idx = {id(st): k for k, st in enumerate(self.stages)}
        ev = {}
        ops = []

        def event(key):
            ev[key] = len(ev)
            return ev[key]

        for st, seg, si in plan:
            if st is None or si:
                return None  # fork/join side streams: keep the single-stream plan
            s = idx[id(st)]
            kind, j = seg[0], seg[1:]
            if kind in "FB" and j.isdigit():
                j = int(j)
                dep = ("F", s - 1, j) if kind == "F" else ("B", s + 1, j)
                if dep in ev:
                    ops.append(dict(kind=WAIT, stream=s, event=ev[dep]))
                ops.append(dict(kind=SEG, stream=s, prog=st._prog, seg=seg))
                ops.append(dict(kind=REC, stream=s, event=event((kind, s, j))))
            else:
                ops.append(dict(kind=SEG, stream=s, prog=st._prog, seg=seg))
        sp = native().StepPlan(S, max(1, len(ev)))
        for o in ops:
            sp.add(**o)
        return sp

    def run_step(self) -> None:
        ns = getattr(self, "native_step", None)
        if ns is not None:  # one C++ call: parallel/native_step.py
            for st in self.stages:
                st.begin_step()
            ns.run(torch.cuda.current_stream(self.stages[0].device).cuda_stream)
            return
        self.pipe.begin_step()
        for st in self.stages:
            st.begin_step()
            if st.params.fused_layers:
                # one-split wgrads apply SGD in their epilogue (W, before O): they read the
                # device lr, so this step's rate must be there before any W
                st.params.set_lr(self.lr_fn() if self.lr_fn else st.params.optim.lr)
        plan = self._native_plan()
        if plan is not None and len(self.stages) > 1 and not getattr(self, "capturing", False) \
                and switches.get("DNN_LOOPBACK_STREAMS") == "1":
            if getattr(self, "_lb_plan", False) is False:
                self._lb_plan = self._loopback_step_plan(plan)
            if self._lb_plan is not None:
                for st in self.stages:
                    st.params.set_lr(st.params.optim.lr)
                self._lb_plan.run(torch.cuda.current_stream(self.stages[0].device).cuda_stream)
                for st in self.stages:
                    st.params.step_count += 1
                self.pipe.end_step()
                return
        if plan is not None and len(self.stages) == 1 and \
                not getattr(self, "capturing", False):
            if getattr(self.stages[0], "h0_double", False):
                self.stages[0].flip_h0()
            if switches.get("DNN_XSTEP") == "1":
                plan = self._xstep_plan(plan)
        if plan is not None:
            dev = self.stages[0].device
            if getattr(self, "_xprimed", False) and any(
                    float(st.params.optim.lr) != getattr(st.params, "_lr_cur", None)
                    for st in self.stages):
                # the previous step's side-stream update still reads lr_dev: a new rate is
                # written only after it
                self.xstep_join()
            for st in self.stages:
                st.params.set_lr(st.params.optim.lr)
            if self._side is None and (self.wgrad_streams > 1 or
                                       any(e[1] == "@fork" for e in plan)):
                self._side = torch.cuda.Stream(dev)
            main = cur = torch.cuda.current_stream(dev)
            native().run_plan([(st._prog if st is not None else None, seg, si)
                               for st, seg, si in plan],
                              main.cuda_stream,
                              self._side.cuda_stream if self._side is not None else 0,
                              switches.get("DNN_EVENT_FENCE") == "device", id(self))
            for st in self.stages:
                st.params.step_count += 1
            self.pipe.end_step()
            return
        if len(self.stages) == 1:
            st, ops = self.stages[0], self.ops[0]
            for k, (op, j) in enumerate(ops):
                nxt = ops[k + 1][0] if k + 1 < len(ops) else None
                self._run_op(st, op, j, nxt)
        else:
            self._run_interleaved()
        self.pipe.end_step()

    def _xstep_plan(self, plan):
        """Cross-step overlap of a single-stage overlap plan (DNN_XSTEP=1): the step no longer
        ends with a join of the side stream. The side stream marks "w" after its last weight
        gradient and "end" after its last op (the reduce + update of layers 1..L-1); the NEXT
        step waits for "w" before its layer-0 forward (which overwrites the activation those
        weight gradients read) and for "end" only before its layer-1 forward (which needs the
        updated W_1). So the next step's first GEMM runs beside this step's side-stream tail
        instead of after it. Bitwise the same step (only the join moves); applied only to plans
        of the form [F0, ..., side W's, ..., main FINO0-0, @join] (split reduction)."""
        if getattr(self, "_xplan_src", None) is plan:
            out = self._xplan
        else:
            out = None
            st = self.stages[0]
            L = len(st.geoms)
            side_w = [k for k, e in enumerate(plan) if e[2] == 1 and e[1].startswith("W")]
            if (plan and plan[0][1] == "F0" and plan[-1][1] == "@join" and side_w and
                    plan[-2][1] == "FINO0-0" and all(f"F0.L{i}" in st._prog.segments()
                                                     for i in range(L))):
                # with a double-buffered layer-0 activation (DNN_H0_DOUBLE) the layer-0
                # forward writes the buffer the previous step's wgrads do NOT read: no wait
                dbl = getattr(st, "h0_double", False)
                out = ([] if dbl else [(None, "@xwait:w", 0)]) + \
                    [(st, "F0.L0", 0), (None, "@xwait:end", 0)]
                out += [(st, f"F0.L{i}", 0) for i in range(1, L)]
                last_w = side_w[-1]
                for k, e in enumerate(plan[1:-1], start=1):
                    out.append(e)
                    if k == last_w and not dbl:
                        out.append((None, "@xmark:w", 1))
                out.append((None, "@xmark:end", 1))
            self._xplan_src, self._xplan = plan, out
        if out is None:
            return plan
        if not getattr(self, "_xprimed", False):  # nothing recorded yet: no waits this step
            self._xprimed = True
            return [e for e in out if not e[1].startswith("@xwait")]
        self._xpending = True
        return out

    def xstep_join(self) -> None:
        """Order the current stream after the last cross-step side-stream work (before
        reading weights / ending a timed region)."""
        if getattr(self, "_xprimed", False) and self._side is not None:
            st = self.stages[0]
            cur = torch.cuda.current_stream(st.device)
            native().run_plan([(None, "@xwait:end", 0)], cur.cuda_stream,
                              self._side.cuda_stream,
                              switches.get("DNN_EVENT_FENCE") == "device", id(self))

    def _run_interleaved(self):
        self._traverse(lambda s, op, j, nxt: self._run_op(self.stages[s], op, j, nxt))

    def _traverse(self, visit):
        """Walk every stage's op list in a dependency-respecting round-robin order (a
        micro-batch's F after the previous stage's F, its B after the next stage's B)."""
        S = len(self.stages)
        pc = [0] * S
        fdone = [set() for _ in range(S)]
        bdone = [set() for _ in range(S)]
        remaining = sum(len(o) for o in self.ops)
        while remaining:
            progress = False
            for s in range(S):
                ops = self.ops[s]
                while pc[s] < len(ops):
                    op, j = ops[pc[s]]
                    if op == "F" and s > 0 and j not in fdone[s - 1]:
                        break
                    if op == "B" and s < S - 1 and j not in bdone[s + 1]:
                        break
                    nxt = ops[pc[s] + 1][0] if pc[s] + 1 < len(ops) else None
                    visit(s, op, j, nxt)
                    if op == "F":
                        fdone[s].add(j)
                    elif op == "B":
                        bdone[s].add(j)
                    pc[s] += 1
                    remaining -= 1
                    progress = True
                    if op in ("F", "B"):
                        break  # round-robin: give the neighbours a chance
            if not progress:
                raise RuntimeError("pipeline schedule deadlocked (inconsistent op lists)")
