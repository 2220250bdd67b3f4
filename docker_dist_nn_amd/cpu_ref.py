"""Single-process fp64 NumPy reference paths (BASELINE config 1, the test oracle).

Two forward semantics, both reproduced from the reference's behaviour:

* :func:`stage_forward` -- the stage worker (/root/reference/src/grpc_node.py:62-97): per-layer
  activation from the first neuron, case-sensitive names, ``np.dot(x, W) + b`` with a dimension
  check that raises ``ValueError("(<name>) Layer k: expected input dim d, got x")``, row softmax
  with max subtraction.
* :func:`manual_forward` -- ``scripts/manual_nn.py`` (:23-70): per-neuron dot products,
  case-insensitive activations among relu/softmax/linear (sigmoid falls back to linear there),
  whole-layer softmax only when every neuron of the layer is softmax.

:func:`train_step` is a NumPy fp64 SGD step with softmax cross-entropy, used to pin the
engine's training numerics on tiny models.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from .config import LayerWeights


def activate(values: np.ndarray, func: str) -> np.ndarray:
    if func == "relu":
        return np.maximum(0, values)
    if func == "sigmoid":
        return 1 / (1 + np.exp(-values))
    if func == "softmax":
        e = np.exp(values - np.max(values, axis=-1, keepdims=True))
        return e / np.sum(e, axis=-1, keepdims=True)
    return values


def stage_forward(layers: Sequence[LayerWeights], x: np.ndarray, expected_input_dim: int,
                  name: str = "layer") -> np.ndarray:
    cur = np.asarray(x, dtype=np.float64)
    if cur.ndim == 1:
        cur = cur[None, :]
    expected = expected_input_dim
    for i, L in enumerate(layers):
        if cur.shape[1] != expected:
            raise ValueError(f"({name}) Layer {i + 1}: expected input dim {expected}, "
                             f"got {cur.shape[1]}")
        w = np.asarray(L.weight, dtype=np.float64)
        cur = activate(cur @ w.T + np.asarray(L.bias, dtype=np.float64), L.activation)
        expected = cur.shape[1]
    return cur


def model_forward(layers: Sequence[LayerWeights], x: np.ndarray) -> np.ndarray:
    return stage_forward(layers, x, layers[0].in_dim)


_MANUAL = {"relu": lambda z: max(0.0, z), "linear": lambda z: z}


def manual_forward(network_config: dict, input_vector) -> np.ndarray:
    a = np.array(input_vector, dtype=np.float64)
    for idx, layer in enumerate(network_config["layers"]):
        neurons = layer["neurons"]
        acts = [n.get("activation", "linear") for n in neurons]
        all_softmax = all(x.lower() == "softmax" for x in acts)
        z = []
        for n in neurons:
            w = np.array(n["weights"], dtype=np.float64)
            if len(w) != a.shape[0]:
                raise ValueError(f"Dimension mismatch in layer {idx}: input dimension "
                                 f"{a.shape[0]} does not match number of weights {len(w)}")
            z.append(float(np.dot(a, w) + n["bias"]))
        z = np.array(z)
        if all_softmax:
            e = np.exp(z - np.max(z))
            a = e / e.sum()
        else:
            # a lone softmax neuron is a softmax over one value, i.e. 1.0 (manual_nn.py:8-11)
            a = np.array([1.0 if act.lower() == "softmax"
                          else _MANUAL.get(act.lower(), _MANUAL["linear"])(v)
                          for act, v in zip(acts, z)])
    return a


def train_step(weights: list[np.ndarray], biases: list[np.ndarray], acts: Sequence[str],
               x: np.ndarray, labels: np.ndarray, lr: float) -> float:
    """In-place fp64 SGD step on mean softmax-CE (last layer's activation is the softmax)."""
    hs = [np.asarray(x, dtype=np.float64)]
    for i, (w, b) in enumerate(zip(weights, biases)):
        z = hs[-1] @ w.T + b
        hs.append(z if i == len(weights) - 1 else activate(z, acts[i]))
    logits = hs[-1]
    m = logits.max(1, keepdims=True)
    logp = logits - m - np.log(np.exp(logits - m).sum(1, keepdims=True))
    n = x.shape[0]
    loss = -logp[np.arange(n), labels].mean()
    g = np.exp(logp)
    g[np.arange(n), labels] -= 1.0
    g /= n
    for i in range(len(weights) - 1, -1, -1):
        gw = g.T @ hs[i]
        gb = g.sum(0)
        if i > 0:
            g = g @ weights[i]
            if acts[i - 1] == "relu":
                g = g * (hs[i] > 0)
            elif acts[i - 1] == "sigmoid":
                g = g * hs[i] * (1 - hs[i])
        weights[i] -= lr * gw
        biases[i] -= lr * gb
    return float(loss)
