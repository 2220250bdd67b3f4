"""Parallel-layout planner: choose (pp, dp, layer_distribution, micro-batching) for N GPUs.

MI355X-first reasoning, encoded as a cost model:

* a pipeline hop moves ``rows x width x 2`` bytes of bf16 activations forward and the same
  amount of gradients backward over ONE xGMI link (point-to-point, ~50-64 GB/s per direction
  achieved); per sample that is ``4 * width`` bytes per hop against ``6 * in * out`` FLOPs of
  stage compute, so thin (MNIST-width) layers make a pipeline link-bound long before it is
  compute-bound;
* a data-parallel replica instead moves only its gradients, once per step, with a ring
  all-reduce that RCCL spreads over the fully connected xGMI mesh, overlapped with the
  remaining weight-gradient GEMMs.

The planner evaluates every (pp, dp) with pp * dp = N (pp <= number of layers), the balanced
layer split for each pp, and the 1F1B step time including the bubble, and returns the fastest.
Constants can be overridden from measurements (``Planner(link_gbps=..., tflops=...)``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

from ..models.mlp import MLPSpec
from ..partition import balanced_distribution


@dataclass
class Plan:
    pp: int
    dp: int
    distribution: list[int]
    num_micro: int
    micro_batch: int
    step_time_s: float
    samples_per_s: float

    @property
    def parallelism(self) -> str:
        if self.pp == 1:
            return f"dp{self.dp}"
        if self.dp == 1:
            return f"pp{self.pp}"
        return f"pp{self.pp}dp{self.dp}"


class Planner:
    # Defaults calibrated on MI355X: measured training steps run at 565 (784-512-256-128-10),
    # 730 (784-1024x7-10) and 935 (784-8192-8192-10) model TFLOP/s with no launch gaps
    # (profiles/r1_tiles/configs_vs_torch.jsonl); xGMI P2P and all-reduce rates are
    # conservative estimates (not measurable on the 1-GPU test pool).
    def __init__(self, tflops: float = 700.0, link_gbps: float = 55.0, hop_latency_us: float = 25.0,
                 allreduce_gbps: float = 120.0, step_overhead_us: float = 20.0):
        self.rate = tflops * 1e12
        self.link = link_gbps * 1e9
        self.lat = hop_latency_us * 1e-6
        self.ar = allreduce_gbps * 1e9
        self.ovh = step_overhead_us * 1e-6

    def evaluate(self, spec: MLPSpec, pp: int, dp: int, rows_per_replica: int,
                 micro_batch: Optional[int] = None) -> Plan:
        L = spec.layers
        flops = [l.flops_per_sample_train for l in L]
        dist = balanced_distribution(flops, pp)
        mb = micro_batch or (rows_per_replica if pp == 1 else
                             max(64, rows_per_replica // (4 * pp) // 64 * 64))
        M = max(1, rows_per_replica // mb)
        # per micro-batch stage time and boundary transfer time
        stage_t, bounds, g = [], [], 0
        for k in dist:
            stage_t.append(sum(flops[g:g + k]) * mb / self.rate)
            g += k
            if g < len(L):
                bounds.append(self.lat + mb * L[g - 1].out_dim * 2 / self.link)
        per_micro = max(stage_t + bounds) if bounds else max(stage_t)
        pipe = (M + pp - 1) * per_micro
        # largest stage gradient all-reduce (bucketed, ~half hidden behind wgrad)
        g, ar = 0, 0.0
        for k in dist:
            params = sum(l.params for l in L[g:g + k])
            g += k
            if dp > 1:
                ar = max(ar, 2 * (dp - 1) / dp * params * 4 / self.ar)
        t = pipe + 0.5 * ar + self.ovh
        return Plan(pp, dp, dist, M, mb, t, rows_per_replica * dp / t)

    def best(self, spec: MLPSpec, n_gpus: int, rows_per_gpu: int,
             min_pp: int = 1) -> Plan:
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


def parse_parallelism(text: str, n_gpus: int,
                      loopback: bool = False) -> tuple[Optional[int], Optional[int]]:
    """'auto' -> (None, None); 'pp4' / 'dp8' / 'pp2dp4' -> explicit degrees. With
    ``loopback`` (one process), 'ppS' may exceed the GPU count: all S stages then run in the
    one process (loopback channels) -- the pipeline engine without the interconnect."""
    if text == "auto":
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
