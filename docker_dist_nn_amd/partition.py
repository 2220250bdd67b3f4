"""Topology / partitioner: ``layer_distribution`` -> pipeline stages -> GPU ranks.

:func:`calculate_layer_mappings` reproduces the reference's container mapping contract
(/root/reference/src/run_grpc_fcnn.py:176-252): the sum check and its error text, consecutive
layer slices keyed ``layer_1..layer_k`` per stage, skipping 0-layer stages (also when looking
up the next hop), container names ``layer_container_<i>``, ports ``5100 + 100*i + 1`` and
``expected_input`` = output width of the previous stage's last layer.

:func:`plan_stages` is what the engine uses: one rank (one GPU process) per non-empty stage.
Unlike the reference a leading 0 entry is handled (reference defect #6: KeyError at
run_grpc_fcnn.py:318). :func:`balanced_distribution` finds the contiguous split minimising the
slowest stage (a planner the reference does not have).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass
from typing import Any, Callable, Optional, Sequence

log = logging.getLogger(__name__)

CONTAINER_NAME_PREFIX = "layer_container_"
BASE_PORT_FIRST_LAYER = 5100
BASE_PORT_INCREMENT = 100


def stage_name(i: int) -> str:
    return f"{CONTAINER_NAME_PREFIX}{i}"


def stage_port(i: int) -> int:
    return BASE_PORT_FIRST_LAYER + i * BASE_PORT_INCREMENT + 1


def _input_dim(examples: Sequence[Any]) -> int:
    if examples:
        ex0 = examples[0]
        if isinstance(ex0, dict) and isinstance(ex0.get("input"), list):
            return len(ex0["input"])
    log.warning("Could not determine initial input dimension from example inputs.")
    return 0


def calculate_layer_mappings(layers_config: Sequence[dict], distribution: Sequence[int],
                             input_examples: Sequence[Any]) -> dict[int, dict]:
    """Reference-compatible stage mapping (see module doc)."""
    if sum(distribution) != len(layers_config):
        raise ValueError(
            "Sum of layer_distribution does not match the number of layers in config.")
    mappings: dict[int, dict] = {}
    expected = _input_dim(input_examples)
    g = 0
    n = len(distribution)
    for ci in range(n):
        k = distribution[ci]
        if k == 0:
            log.warning(f"Container {ci} has 0 layers assigned, skipping.")
            continue
        neurons_cfg: dict[str, list] = {}
        out_dim = expected
        for i in range(k):
            if g >= len(layers_config):
                raise IndexError("Layer distribution requests more layers than available in config.")
            lc = layers_config[g]
            neurons_cfg[f"layer_{i + 1}"] = lc.get("neurons", [])
            out_dim = lc.get("nodes", 0)
            g += 1
        nxt = ci + 1
        while nxt < n and distribution[nxt] == 0:
            nxt += 1
        next_nodes = ([{"host": stage_name(nxt), "port": str(stage_port(nxt))}]
                      if nxt < n else [])
        mappings[ci] = {
            "container_name": stage_name(ci),
            "listen_port": stage_port(ci),
            "expected_input": expected,
            "neurons_config": neurons_cfg,
            "next_nodes": next_nodes,
        }
        expected = out_dim
    log.info(f"Calculated mappings for {len(mappings)} containers.")
    return mappings


@dataclass(frozen=True)
class StagePlan:
    stage: int          # pipeline stage index among NON-empty stages (= pipeline rank)
    container: int      # index in layer_distribution (reference container index)
    layer_start: int    # global layer index range [start, end)
    layer_end: int
    name: str
    port: int

    @property
    def num_layers(self) -> int:
        return self.layer_end - self.layer_start


def plan_stages(num_layers: int, distribution: Sequence[int]) -> list[StagePlan]:
    if any(d < 0 for d in distribution):
        raise ValueError("layer_distribution entries must be >= 0")
    if sum(distribution) != num_layers:
        raise ValueError(
            "Sum of layer_distribution does not match the number of layers in config.")
    plans, g = [], 0
    for ci, k in enumerate(distribution):
        if k == 0:
            continue
        plans.append(StagePlan(len(plans), ci, g, g + k, stage_name(ci), stage_port(ci)))
        g += k
    if not plans:
        raise ValueError("layer_distribution assigns no layers")
    return plans


def balanced_distribution(costs: Sequence[float], num_stages: int,
                          comm_cost: Optional[Callable[[int], float]] = None) -> list[int]:
    """Contiguous partition of layer costs into ``num_stages`` non-empty stages minimising the
    slowest stage (+ the cost of its outgoing boundary, ``comm_cost(boundary_layer)``)."""
    L = len(costs)
    if not 1 <= num_stages <= L:
        raise ValueError(f"cannot split {L} layers into {num_stages} non-empty stages")
    pre = [0.0]
    for c in costs:
        pre.append(pre[-1] + c)
    INF = float("inf")
    # best[s][i]: minimal max-stage cost splitting the first i layers into s stages
    best = [[INF] * (L + 1) for _ in range(num_stages + 1)]
    cut = [[0] * (L + 1) for _ in range(num_stages + 1)]
    best[0][0] = 0.0
    for s in range(1, num_stages + 1):
        for i in range(s, L - (num_stages - s) + 1):
            for j in range(s - 1, i):
                stage = pre[i] - pre[j]
                if comm_cost is not None and i < L:
                    stage += comm_cost(i - 1)
                v = max(best[s - 1][j], stage)
                if v < best[s][i]:
                    best[s][i], cut[s][i] = v, j
    dist, i = [], L
    for s in range(num_stages, 0, -1):
        j = cut[s][i]
        dist.append(i - j)
        i = j
    return dist[::-1]
