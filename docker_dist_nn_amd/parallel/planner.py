"""Parallel-layout planner: choose (pp, dp, layer_distribution, micro-batching) for N GPUs.

MI355X-first reasoning, encoded as a cost model (all constants overridable):

* compute: a stage's time is its EXECUTED training FLOPs (fwd + dgrad + wgrad, no dgrad for the
  network's first layer) at the step rate measured on one MI355X (``tflops``);
* a pipeline hop moves ``width x 2`` bytes per sample (bf16) forward over the direct xGMI link
  between two GPUs and the same backward on the opposite direction of that link; the native
  step (parallel/native_step.py) runs each direction on its own stream, overlapped with
  compute, so in steady state a micro-batch costs ``max(stage compute, hop in, hop out)``
  (``link_gbps`` = achieved per-direction point-to-point rate; xGMI is 7 links x ~153 GB/s per
  GPU, not all of it reachable by one P2P stream);
* a data-parallel replica exchanges its stage gradient once per step with RCCL's rings over
  the fully connected mesh (``allreduce_gbps`` bus bandwidth), bucketed and about half hidden
  behind the remaining weight-gradient GEMMs: by default as a bf16 reduce-scatter + bf16
  all-gather of the updated weights (sharded optimizer, ``dp_grad_bytes`` = 2), or as an fp32
  all-reduce (``dp_grad_bytes`` = 4).

``pipeline_layout`` is the layout the benchmark runs for N GPUs (the metric is "... at
1/2/4/8-stage pipeline"): the deepest pipeline that divides N and fits the layers, data
parallel over the rest, with the layer split this model scores best -- which weighs boundary
WIDTH (hop bytes) against compute balance, not FLOPs alone. ``best`` searches every
(pp, dp) instead (the data-parallel-only number the benchmark also reports).
"""
from __future__ import annotations

import itertools
import math
from dataclasses import dataclass, field
from typing import Optional

from ..models.mlp import MLPSpec


@dataclass
class Plan:
    pp: int
    dp: int
    distribution: list[int]
    num_micro: int
    micro_batch: int
    step_time_s: float
    samples_per_s: float
    detail: dict = field(default_factory=dict)
    reps: Optional[list] = None  # fan layout: GPUs per stage (parallel/fan.py)

    @property
    def parallelism(self) -> str:
        if self.reps is not None and len(set(self.reps)) > 1:
            return "fan" + ",".join(f"{k}x{r}" for k, r in zip(self.distribution, self.reps))
        if self.reps is not None:  # equal replica counts: the uniform grid
            d = self.reps[0]
            return f"pp{self.pp}" + (f"dp{d}" if d > 1 else "")
        if self.pp == 1:
            return f"dp{self.dp}"
        if self.dp == 1:
            return f"pp{self.pp}"
        return f"pp{self.pp}dp{self.dp}"


def layer_train_flops(spec: MLPSpec) -> list[float]:
    """Executed training FLOPs per sample of each layer (no dgrad for layer 0)."""
    out = []
    for i, l in enumerate(spec.layers):
        out.append((4.0 if i == 0 else 6.0) * l.in_dim * l.out_dim)
    return out


def compositions(n: int, k: int):
    """Every split of n consecutive layers into k non-empty contiguous stages."""
    for cuts in itertools.combinations(range(1, n), k - 1):
        b = (0,) + cuts + (n,)
        yield [b[i + 1] - b[i] for i in range(k)]


# Measured one-GPU training steps on MI355X with the round-2 own-kernel table
# (profiles/r2_own_kernels, profiles/r2_epilogue): widths -> (rows, ms per step).
MEASURED_STEP_MS = {  # round 3: driver BENCH_r03 (headline), profiles/r3b_final4 (others)
    (784, 512, 256, 128, 10): (65536, 0.350),
    (784, 1024, 1024, 1024, 1024, 1024, 1024, 1024, 10): (65536, 2.88),
    (784, 8192, 8192, 10): (16384, 5.96),
}


class Planner:
    # Calibrated on MI355X (one GPU, own kernels, profiles/r2_own_kernels): headline step 0.36 ms
    # at 65536 rows = ~470 executed TFLOP/s; 784-1024x7-10 ~600; 784-8192-8192-10 ~880. The
    # xGMI rates are estimates (the 1-GPU pool cannot time a cross-GPU hop).
    def __init__(self, tflops: float = 550.0, link_gbps: float = 64.0,
                 hop_latency_us: float = 15.0, allreduce_gbps: float = 150.0,
                 step_overhead_us: float = 20.0, boundary_bytes: float = 2.0,
                 dp_grad_bytes: float = 2.0, relays=0, relay_eff: float = 0.8):
        self.rate = tflops * 1e12
        self.link = link_gbps * 1e9
        self.lat = hop_latency_us * 1e-6
        self.ar = allreduce_gbps * 1e9
        self.ovh = step_overhead_us * 1e-6
        self.bb = boundary_bytes  # bytes per boundary element on the wire (bf16 = 2)
        self.gb = dp_grad_bytes   # bytes per parameter per DP collective (shard bf16 = 2)
        # relayed IPC hops: a hop's rows striped over the direct link and k two-link paths,
        # each path worth `relay_eff` of a link (the relay's second copy adds latency and HBM
        # traffic on the relay GPU). relays = k (the same on every hop,
        # comm.relay_assignment) or "plan": per-hop k from the directed-link load model
        # (comm.relay_plan -- what the IPC transport uses with DNN_IPC_RELAYS=auto), each hop
        # costing its most loaded link with every other hop and the DP exchange on the links
        self.relays = relays
        self.relay_eff = relay_eff
        self.hop_bw = self.link * (1.0 + (0 if relays == "plan" else relays) * relay_eff)

    @classmethod
    def calibrated(cls, spec: MLPSpec, **kw) -> "Planner":
        """A planner whose compute rate is this model's MEASURED one-GPU step rate (executed
        FLOPs / step time), when one is on record; else the default rate."""
        m = MEASURED_STEP_MS.get(tuple(spec.widths))
        if m is not None and "tflops" not in kw:
            rows, ms = m
            kw["tflops"] = sum(layer_train_flops(spec)) * rows / (ms * 1e-3) / 1e12
        return cls(**kw)

    def hop_ratios(self, spec: MLPSpec, dist: list[int], dp: int = 1,
                   rows: int = 65536) -> list[float]:
        """Per boundary: seconds per byte of that hop relative to one direct link (1.0 = a
        link of its own; < 1 with relays). With relays == "plan" this is the slowest direction /
        replica of the boundary under comm.relay_plan's table."""
        pp = len(dist)
        widths, g = [], 0
        for k in dist[:-1]:
            g += k
            widths.append(spec.layers[g - 1].out_dim)
        if self.relays != "plan" or pp < 2:
            return [self.link / self.hop_bw] * len(widths)
        from .comm import relay_link_loads, relay_plan

        hb = [rows * w * self.bb for w in widths]
        dpb, g = [], 0
        for k in dist:
            params = sum(l.params for l in spec.layers[g:g + k])
            g += k
            dpb.append(2 * (dp - 1) / max(1, dp) * params * self.gb)
        table = relay_plan(pp, dp, hb, dp_bytes=dpb, max_k=min(6, pp * dp - 2),
                           relay_eff=self.relay_eff)
        loads = relay_link_loads(pp, dp, table, hb, dp_bytes=dpb, relay_eff=self.relay_eff)
        out = [0.0] * len(widths)
        for (src, dst, d), v in loads.items():
            b = min(src, dst) % pp  # boundary between stages b and b + 1
            out[b] = max(out[b], v / hb[b])
        return out

    def _stage_costs(self, spec: MLPSpec, dist: list[int], mb: int, dp: int = 1):
        fl = layer_train_flops(spec)
        ratios = self.hop_ratios(spec, dist, dp, mb)
        comp, hops, g = [], [], 0
        for k in dist:
            comp.append(sum(fl[g:g + k]) * mb / self.rate)
            g += k
            if g < len(spec.layers):
                hops.append(self.lat + mb * spec.layers[g - 1].out_dim * self.bb *
                            ratios[len(hops)] / self.link)
        return comp, hops

    def best_distribution(self, spec: MLPSpec, pp: int, mb: int, dp: int = 1) -> list[int]:
        """The split minimising the slowest stage / hop per micro-batch; among hop-bound ties
        (equal-width boundaries), the one with the most balanced compute."""
        best, best_k = None, (float("inf"), float("inf"))
        for dist in compositions(len(spec.layers), pp):
            comp, hops = self._stage_costs(spec, dist, mb, dp)
            k = (round(max(comp + hops), 12), max(comp))
            if k < best_k:
                best, best_k = dist, k
        return best

    def evaluate(self, spec: MLPSpec, pp: int, dp: int, rows_per_replica: int,
                 micro_batch: Optional[int] = None,
                 distribution: Optional[list[int]] = None, loopback: bool = False) -> Plan:
        L = spec.layers
        if loopback and pp > 1 and not micro_batch:
            # every stage on ONE GPU: the stages overlap only through their streams, so the
            # micro-batch GEMMs must stay big enough to fill the chip: >= 16384 rows measured
            # best (profiles/r2_own_kernels/loopback_micro_ab.jsonl: pp4 0.72 -> 0.59-0.63 ms,
            # pp8 4.55 -> 4.37 ms against 8192-row micro-batches)
            micro_batch = max(16384, rows_per_replica // (2 * pp)) // 64 * 64
            micro_batch = min(micro_batch, rows_per_replica)
        mb = micro_batch or (rows_per_replica if pp == 1 else
                             max(64, rows_per_replica // (4 * pp) // 64 * 64))
        M = max(1, rows_per_replica // mb)
        dist = distribution or (self.best_distribution(spec, pp, mb, dp) if pp > 1
                                else [len(L)])
        comp, hops = self._stage_costs(spec, dist, mb, dp)
        per_micro = max(comp + hops)
        pipe = (M + pp - 1) * per_micro if pp > 1 else comp[0]
        ar, g = 0.0, 0
        for k in dist:
            params = sum(l.params for l in L[g:g + k])
            g += k
            if dp > 1:
                ar = max(ar, 2 * (dp - 1) / dp * params * self.gb / self.ar)
        t = pipe + 0.5 * ar + self.ovh
        detail = {"stage_ms_per_micro": [round(c * 1e3, 4) for c in comp],
                  "hop_ms_per_micro": [round(h * 1e3, 4) for h in hops],
                  "bubble": round((pp - 1) / (M + pp - 1), 3) if pp > 1 else 0.0,
                  "allreduce_ms": round(ar * 1e3, 4)}
        return Plan(pp, dp, dist, M, mb, t, rows_per_replica * dp / t, detail)

    def best(self, spec: MLPSpec, n_gpus: int, rows_per_gpu: int, min_pp: int = 1) -> Plan:
        cands = []
        for pp in range(1, n_gpus + 1):
            if n_gpus % pp or pp > len(spec.layers) or pp < min_pp:
                continue
            dp = n_gpus // pp
            # weak scaling in GPUs: each replica gets rows_per_gpu * pp rows
            cands.append(self.evaluate(spec, pp, dp, rows_per_gpu * pp))
        if not cands:
            raise ValueError(f"no valid layout for {n_gpus} GPUs and {len(spec.layers)} layers")
        return max(cands, key=lambda p: p.samples_per_s)

    # ---- replicated-stage ("fan") pipelines (parallel/fan.py) -----------------------------
    def evaluate_fan(self, spec: MLPSpec, dist: list[int], reps: list[int], rows_per_gpu: int,
                     num_micro: Optional[int] = None) -> Plan:
        """Predicted step of a fan layout: stage s (layers dist[s]) on reps[s] GPUs, micro-batch
        j on replica j % r_s of every stage (parallel/fan.py).

        * compute: a replica of stage s runs ceil(M / r_s) micro-batches of ``c_s`` each;
        * hops: the pair (producer p, consumer c) of boundary b carries the micro-batches with
          j % r_b == p and j % r_{b+1} == c over its own direct xGMI link (every GPU pair of an
          MI355X node has one), forward and backward on the two directions; the slowest pair
          bounds the boundary (``link_gbps`` per direction, ``hop_latency_us`` per message);
        * the pipeline fills and drains once per step: one micro-batch's trip through every
          other stage and hop;
        * a replicated stage exchanges its gradient over its own DP group of r_s GPUs (half
          hidden behind the weight gradients, as ``evaluate``)."""
        from .fan import lcm_reps

        S, N = len(reps), sum(reps)
        L = spec.layers
        G = rows_per_gpu * N
        if num_micro is None:  # ~8 micro-batches per GPU: GEMMs of >= 8192 rows at 65536
            num_micro = max(8 * N, 2 * max(reps))
            while G % num_micro or (G // num_micro) % 64:
                num_micro += 1
                if num_micro > G // 64:
                    num_micro = max(reps)
                    break
        M = num_micro
        mb = G // M
        fl = layer_train_flops(spec)
        comp, g = [], 0
        for k in dist:
            comp.append(sum(fl[g:g + k]) * mb / self.rate)
            g += k
        busy = [math.ceil(M / r) * c for r, c in zip(reps, comp)]
        hops, g = [], 0
        for b in range(S - 1):
            g += dist[b]
            width = L[g - 1].out_dim
            per_msg = self.lat + mb * width * self.bb / self.link
            ra, rb = reps[b], reps[b + 1]
            most = max(sum(1 for j in range(M) if j % ra == p and j % rb == c)
                       for p in range(ra) for c in range(rb))
            hops.append((most * per_msg, per_msg))
        fill = sum(comp) - max(comp) + 2 * sum(h[1] for h in hops)
        pipe = max(busy + [h[0] for h in hops]) + fill
        ar, g = 0.0, 0
        for k, r in zip(dist, reps):
            params = sum(l.params for l in L[g:g + k])
            g += k
            if r > 1:
                ar = max(ar, 2 * (r - 1) / r * params * self.gb / self.ar)
        t = pipe + 0.5 * ar + self.ovh
        detail = {"fan_reps": list(reps), "stage_ms_per_micro": [round(c * 1e3, 4) for c in comp],
                  "stage_busy_ms": [round(x * 1e3, 4) for x in busy],
                  "boundary_link_ms": [round(h[0] * 1e3, 4) for h in hops],
                  "fill_ms": round(fill * 1e3, 4), "allreduce_ms": round(ar * 1e3, 4),
                  "lcm_reps": lcm_reps(reps)}
        plan = Plan(S, 1, list(dist), M, mb, t, G / t, detail)
        plan.reps = list(reps)
        return plan

    def best_fan(self, spec: MLPSpec, n_gpus: int, rows_per_gpu: int,
                 min_stages: int = 2) -> Plan:
        """The best fan layout with at least ``min_stages`` stages over every contiguous layer
        split and every split of the N GPUs (uniform ppS x dpD is the case of equal replica
        counts; a single stage is plain data parallelism)."""
        best = None
        for S in range(min_stages, min(n_gpus, len(spec.layers)) + 1):
            for dist in compositions(len(spec.layers), S):
                for reps in compositions(n_gpus, S):
                    p = self.evaluate_fan(spec, dist, reps, rows_per_gpu)
                    if best is None or p.samples_per_s > best.samples_per_s:
                        best = p
        if best is None:
            raise ValueError(f"no fan layout of >= {min_stages} stages for {n_gpus} GPUs")
        return best

    def pipeline_layout(self, spec: MLPSpec, n_gpus: int, rows_per_gpu: int) -> Plan:
        """The deepest pipeline for N GPUs: pp = largest divisor of N that is <= #layers,
        dp = N / pp (e.g. 784-512-256-128-10: pp2, pp4, pp4dp2 at 2/4/8; 784-8192-8192-10 at
        8: pp2dp4 -- BASELINE.json's configurations)."""
        pp = max(p for p in range(1, n_gpus + 1)
                 if n_gpus % p == 0 and p <= len(spec.layers))
        return self.evaluate(spec, pp, n_gpus // pp, rows_per_gpu * pp)


def parse_parallelism(text: str, n_gpus: int,
                      loopback: bool = False) -> tuple[Optional[int], Optional[int]]:
    """'auto' / 'pipeline' / 'dp' -> (None, None) (the caller picks); 'pp4' / 'dp8' / 'pp2dp4'
    -> explicit degrees. With ``loopback`` (one process), 'ppS' may exceed the GPU count: all S
    stages then run in the one process (loopback channels) -- the pipeline engine without the
    interconnect."""
    if text in ("auto", "pipeline", "best"):
        return None, None
    import re

    m = re.fullmatch(r"(?:pp(\d+))?(?:dp(\d+))?", text)
    if not m or not (m.group(1) or m.group(2)):
        raise ValueError(f"bad --parallelism {text!r}")
    pp = int(m.group(1)) if m.group(1) else None
    dp = int(m.group(2)) if m.group(2) else None
    if pp is None:
        pp = n_gpus // dp
    if dp is None:
        dp = 1 if loopback and n_gpus == 1 else n_gpus // pp
    if loopback and n_gpus == 1 and dp == 1:
        return pp, 1
    if pp * dp != n_gpus:
        raise ValueError(f"--parallelism {text} does not use {n_gpus} GPUs")
    return pp, dp
