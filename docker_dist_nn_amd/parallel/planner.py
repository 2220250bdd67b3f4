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
    place: Optional[tuple] = None  # fan layout with co-located stages: ranks per stage

    @property
    def colocated(self) -> bool:
        return self.place is not None and sum(self.reps) != len({x for p in self.place
                                                                  for x in p})

    @property
    def parallelism(self) -> str:
        if self.colocated:
            from .fan import FanLayout

            lay = FanLayout(tuple(self.distribution), tuple(self.reps), self.place)
            return "fan" + lay.spec_text()[4:]
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


# Measured one-GPU training steps on MI355X (one micro-batch, the single-stage overlap plan):
# widths -> (rows, ms per step). Headline: the driver's BENCH_r05 (0.3286 ms); mlp8 / wide:
# the round-5 end-of-round A/B medians (profiles/r5_tables), re-checked in round 6.
MEASURED_STEP_MS = {
    (784, 512, 256, 128, 10): (65536, 0.3286),
    (784, 1024, 1024, 1024, 1024, 1024, 1024, 1024, 10): (65536, 2.68),
    (784, 8192, 8192, 10): (16384, 5.33),
}


class StageTimes:
    """Measured compute of one pipeline-stage replica per step (bench/planner_calibrate.py,
    ``stage_times_gfx950.json``): layers [a, b) of a model, n micro-batches of
    mb rows through the recorded forward / backward segments, then the batched weight
    gradient and the fused update.

    Per (a, b, mb) the measured n are fit as t = fixed + n * per_micro (least squares: the
    weight gradient and update scale with the rows, so ``fixed`` absorbs only what does not);
    between measured micro-batch sizes both terms are interpolated linearly, outside them
    extrapolated at the nearest size's per-row rate. A range that was not measured (mlp8's
    middle ranges) is the sum of its single layers."""

    def __init__(self, rows):
        self.fit: dict = {}  # (widths, a, b) -> sorted [(mb, fixed_s, per_micro_s)]
        pts: dict = {}
        for widths, a, b, mb, n, ms in rows:
            pts.setdefault((tuple(widths), a, b, mb), []).append((n, ms * 1e-3))
        for (w, a, b, mb), v in pts.items():
            if len(v) == 1:
                n, t = v[0]
                fixed, per = 0.0, t / n
            else:
                k = len(v)
                sx = sum(n for n, _ in v)
                sy = sum(t for _, t in v)
                sxx = sum(n * n for n, _ in v)
                sxy = sum(n * t for n, t in v)
                den = k * sxx - sx * sx
                if den <= 0:  # every point at the same micro-batch count: no fixed term
                    fixed, per = 0.0, sy / sx
                else:
                    per = (k * sxy - sx * sy) / den
                    fixed = (sy - per * sx) / k
                    if fixed < 0.0:  # refit through the origin rather than clamp
                        fixed, per = 0.0, sxy / sxx
            self.fit.setdefault((w, a, b), []).append((mb, fixed, per))
        for v in self.fit.values():
            v.sort()

    @classmethod
    def load(cls, path: Optional[str] = None) -> "StageTimes":
        import json
        import os

        path = path or os.path.join(os.path.dirname(__file__), "stage_times_gfx950.json")
        with open(path) as f:
            return cls(json.load(f)["rows"])

    def has(self, widths) -> bool:
        w = tuple(widths)
        return any(k[0] == w for k in self.fit)

    def _terms(self, w, a, b, mb):
        v = self.fit.get((w, a, b))
        if v is None:
            if b - a <= 1:
                return None
            parts = [self._terms(w, i, i + 1, mb) for i in range(a, b)]
            if any(p is None for p in parts):
                return None
            return sum(p[0] for p in parts), sum(p[1] for p in parts)
        if mb <= v[0][0]:
            m0, f0, p0 = v[0]
            return f0, p0 * mb / m0 if mb < m0 else p0
        if mb >= v[-1][0]:
            m1, f1, p1 = v[-1]
            return f1, p1 * mb / m1
        for (m0, f0, p0), (m1, f1, p1) in zip(v, v[1:]):
            if m0 <= mb <= m1:
                x = (mb - m0) / (m1 - m0)
                return f0 + x * (f1 - f0), p0 + x * (p1 - p0)
        return None

    def step(self, widths, a: int, b: int, mb: int, n: int) -> Optional[float]:
        """Seconds of one replica step of layers [a, b): n micro-batches of mb rows."""
        t = self._terms(tuple(widths), a, b, mb)
        return None if t is None else t[0] + n * t[1]

    def per_micro(self, widths, a: int, b: int, mb: int) -> Optional[float]:
        t = self._terms(tuple(widths), a, b, mb)
        return None if t is None else t[1]


class Planner:
    # Calibrated on MI355X (one GPU, own kernels, profiles/r2_own_kernels): headline step 0.36 ms
    # at 65536 rows = ~470 executed TFLOP/s; 784-1024x7-10 ~600; 784-8192-8192-10 ~880. The
    # xGMI rates are estimates (the 1-GPU pool cannot time a cross-GPU hop).
    def __init__(self, tflops: float = 550.0, link_gbps: float = 64.0,
                 hop_latency_us: float = 15.0, allreduce_gbps: float = 150.0,
                 step_overhead_us: float = 20.0, boundary_bytes: float = 2.0,
                 dp_grad_bytes: float = 2.0, relays=0, relay_eff: float = 0.8,
                 stage_times: Optional[StageTimes] = None,
                 one_gpu_step: Optional[tuple] = None):
        # stage_times: measured replica steps (calibrated planners); one_gpu_step: (rows, s)
        # of the model's own single-stage one-micro-batch step (MEASURED_STEP_MS)
        self.times = stage_times
        self.one_step = one_gpu_step
        self._memo: dict = {}
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
        """A planner on this model's MEASURED one-GPU numbers: the single-stage step
        (MEASURED_STEP_MS: the compute rate, and the data-parallel replica's step) and the
        replica steps of every layer range at every micro-batch size and count
        (stage_times_gfx950.json, round 6). Without measurements: the default FLOP rate."""
        m = MEASURED_STEP_MS.get(tuple(spec.widths))
        if m is not None and "tflops" not in kw:
            rows, ms = m
            kw["tflops"] = sum(layer_train_flops(spec)) * rows / (ms * 1e-3) / 1e12
            kw.setdefault("one_gpu_step", (rows, ms * 1e-3))
        if "stage_times" not in kw:
            try:
                t = StageTimes.load()
                if t.has(spec.widths):
                    kw["stage_times"] = t
            except OSError:
                pass
        return cls(**kw)

    def replica_step(self, spec: MLPSpec, a: int, b: int, mb: int, n: int) -> float:
        key = ("r", tuple(spec.widths), a, b, mb, n)
        v = self._memo.get(key)
        if v is None:
            v = self._memo[key] = self._replica_step(spec, a, b, mb, n)
        return v

    def _replica_step(self, spec: MLPSpec, a: int, b: int, mb: int, n: int) -> float:
        """Compute seconds of one replica of layers [a, b) per step: n micro-batches of mb
        rows, batched weight gradient, update -- measured (StageTimes) when available, the
        FLOP rate otherwise; the model's own one-micro-batch step when that is the case."""
        L = len(spec.layers)
        if (a, b) == (0, L) and n == 1 and self.one_step is not None and \
                mb == self.one_step[0]:
            return self.one_step[1]
        if self.times is not None:
            t = self.times.step(spec.widths, a, b, mb, n)
            if t is not None:
                return t
        return sum(layer_train_flops(spec)[a:b]) * mb * n / self.rate

    def micro_time(self, spec: MLPSpec, a: int, b: int, mb: int) -> float:
        """Seconds one micro-batch of mb rows spends in layers [a, b) (forward + backward)."""
        key = ("m", tuple(spec.widths), a, b, mb)
        v = self._memo.get(key)
        if v is None:
            v = self._memo[key] = self._micro_time(spec, a, b, mb)
        return v

    def _micro_time(self, spec: MLPSpec, a: int, b: int, mb: int) -> float:
        if self.times is not None:
            t = self.times.per_micro(spec.widths, a, b, mb)
            if t is not None:
                return t
        return sum(layer_train_flops(spec)[a:b]) * mb / self.rate

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
        ratios = self.hop_ratios(spec, dist, dp, mb)
        comp, hops, g = [], [], 0
        for k in dist:
            comp.append(self.micro_time(spec, g, g + k, mb))
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
        if pp > 1:
            # the slowest stage's measured fixed part (batched wgrad + update beyond the
            # per-micro-batch rate) ends the step after the pipeline drains
            g, fixed = 0, 0.0
            for k, c in zip(dist, comp):
                fixed = max(fixed, self.replica_step(spec, g, g + k, mb, M) - M * c)
                g += k
            pipe = (M + pp - 1) * per_micro + fixed
        else:
            pipe = self.replica_step(spec, 0, len(L), mb, M)
        ar, g = 0.0, 0
        for k in dist:
            params = sum(l.params for l in L[g:g + k])
            g += k
            if dp > 1:
                ar = max(ar, 2 * (dp - 1) / dp * params * self.gb / self.ar)
        t = pipe + 0.5 * ar + (0.0 if self.one_step is not None and pp == 1 else self.ovh)
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
                     num_micro: Optional[int] = None, place: Optional[tuple] = None) -> Plan:
        """Predicted step of a fan layout: stage s (layers dist[s]) on reps[s] GPUs, micro-batch
        j on replica j % r_s of every stage (parallel/fan.py); ``place`` co-locates stages
        (FanLayout.place: a GPU hosting a replica of two stages runs both).

        * compute: every GPU runs the replica steps of the workers it hosts -- n micro-batches
          of mb rows through the stage's layers, its batched weight gradient and update,
          MEASURED at that micro-batch size and count (StageTimes) when calibrated;
        * hops: micro-batch j crosses boundary b from the GPU of replica j % r_b to the GPU of
          replica j % r_{b+1} (nothing when that is the same GPU: co-location), forward on one
          direction of their direct xGMI link and its gradient back on the other; each
          direction of each GPU pair carries its messages serially (``link_gbps``,
          ``hop_latency_us`` per message) and the busiest one bounds the step with the busiest
          GPU;
        * the pipeline fills and drains once per step: one micro-batch's trip through every
          other stage and hop;
        * a replicated stage exchanges its gradient over its own DP group of r_s GPUs (half
          hidden behind the weight gradients, as ``evaluate``)."""
        from .fan import FanLayout, lcm_reps

        lay = FanLayout(tuple(dist), tuple(reps), place)
        S, N = len(reps), lay.world
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
        lay.check_directions(M)
        mb = G // M
        bounds, g = [], 0
        for k in dist:
            bounds.append((g, g + k))
            g += k
        comp = [self.micro_time(spec, a, b, mb) for a, b in bounds]
        busy: dict = {}
        for s_, (a, b) in enumerate(bounds):
            for q in range(reps[s_]):
                n = len(lay.local_micros(s_, q, M))
                r = lay.rank_of(s_, q)
                busy[r] = busy.get(r, 0.0) + self.replica_step(spec, a, b, mb, n)
        link: dict = {}
        msg = []
        for bnd in range(S - 1):
            width = L[bounds[bnd][1] - 1].out_dim
            per_msg = self.lat + mb * width * self.bb / self.link
            msg.append(per_msg)
            ra, rb = reps[bnd], reps[bnd + 1]
            per = ra * rb // math.gcd(ra, rb)  # the (producer, consumer) pattern repeats
            cnt: dict = {}
            for j in range(min(M, per)):
                key = (j % ra, j % rb)
                cnt[key] = len(range(j, M, per))
            for (p_, c_), n_ in cnt.items():
                src, dst = lay.rank_of(bnd, p_), lay.rank_of(bnd + 1, c_)
                if src != dst:
                    link[(src, dst)] = link.get((src, dst), 0.0) + n_ * per_msg  # forward
                    link[(dst, src)] = link.get((dst, src), 0.0) + n_ * per_msg  # gradient
        fill = sum(comp) - max(comp) + 2 * sum(msg)
        pipe = max(list(busy.values()) + list(link.values())) + fill
        ar = 0.0
        for (a, b), r in zip(bounds, reps):
            if r > 1:
                params = sum(l.params for l in L[a:b])
                ar = max(ar, 2 * (r - 1) / r * params * self.gb / self.ar)
        t = pipe + 0.5 * ar + self.ovh
        detail = {"fan_reps": list(reps), "stage_ms_per_micro": [round(c * 1e3, 4) for c in comp],
                  "gpu_busy_ms": [round(busy[r] * 1e3, 4) for r in range(N)],
                  "busiest_link_ms": round(max(link.values(), default=0.0) * 1e3, 4),
                  "fill_ms": round(fill * 1e3, 4), "allreduce_ms": round(ar * 1e3, 4),
                  "lcm_reps": lcm_reps(reps), "calibrated": self.times is not None}
        if lay.colocated:
            detail["place"] = [list(p) for p in lay.place]
        plan = Plan(S, 1, list(dist), M, mb, t, G / t, detail)
        plan.reps = list(reps)
        plan.place = lay.place if lay.colocated else None
        return plan

    def fan_candidates(self, spec: MLPSpec, n_gpus: int, min_stages: int = 2,
                       colocate: bool = True):
        """(dist, reps, place) of every fan layout on n_gpus GPUs with at least
        ``min_stages`` stages: every contiguous layer split, every split of the GPUs into
        per-stage replica counts, and -- with ``colocate`` -- the last stage with one replica
        placed on the last GPU of the stage before it (the light classifier
        stage beside a heavy replica instead of on a GPU of its own)."""
        from .fan import colocated_place

        L = len(spec.layers)
        for S in range(min_stages, L + 1):
            for dist in compositions(L, S):
                cos = [(False,) * (S - 1)] + ([(False,) * (S - 2) + (True,)] if colocate
                                                else [])
                for co in cos:
                    co = (False,) + tuple(co)
                    if S - sum(co) < 1 or (sum(co) and S - sum(co) < min_stages - 1):
                        continue
                    k = S - sum(co)
                    if k > n_gpus:
                        continue
                    for rr in compositions(n_gpus, k):
                        it = iter(rr)
                        reps = [1 if c else next(it) for c in co]
                        yield dist, reps, (colocated_place(reps, co) if any(co) else None)

    def best_fan(self, spec: MLPSpec, n_gpus: int, rows_per_gpu: int,
                 min_stages: int = 2, colocate: bool = True) -> Plan:
        """The best fan layout with at least ``min_stages`` stages over every contiguous layer
        split, every split of the N GPUs and every co-location of one-replica stages (uniform
        ppS x dpD is the case of equal replica counts; a single stage is plain data
        parallelism)."""
        best = None
        G = rows_per_gpu * n_gpus
        for dist, reps, place in self.fan_candidates(spec, n_gpus, min_stages, colocate):
            # micro-batch count: a few per GPU (bigger GEMMs, fewer messages) up to ~8 (less
            # fill); the measured replica steps decide
            for per_gpu in (1, 2, 4, 8):
                M = max(per_gpu * n_gpus, max(reps))
                if G % M or (G // M) % 64:
                    continue
                try:
                    p = self.evaluate_fan(spec, dist, reps, rows_per_gpu, num_micro=M,
                                          place=place)
                except ValueError:  # a placement whose boundaries run both ways on a rank
                    continue
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
