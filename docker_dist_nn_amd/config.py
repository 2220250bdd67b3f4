"""Model-config / topology schema loading (reference-compatible) and the run configuration.

Accepted model files:

* ``{"layers": [...], "layer_distribution": [...]}`` -- what ``run_grpc_fcnn.py`` reads
  (/root/reference/src/run_grpc_fcnn.py:263-266, schema /root/reference/config/config_sample.json);
* ``{"model": {"layers": [...]}, "inference_metrics": {...}}`` -- what the notebook writes
  (/root/reference/scripts/Centralized_MNIST_Experimentation.ipynb:493-506). The reference
  fails on it with a KeyError (run_grpc_fcnn.py:265); we accept both.
* a per-stage file ``{"layer_1": [neurons], ...}`` (run_grpc_fcnn.py:113-116, grpc_node.py:43-55).

Each neuron is one OUTPUT unit; its ``weights`` (length in_dim) is a row of an nn.Linear
weight ``[out][in]``. The activation of a layer is that of its FIRST neuron
(grpc_node.py:53); mixed activations are reported as a warning.
"""
from __future__ import annotations

import json
import logging
import os
import warnings
from dataclasses import dataclass, field
from typing import Any, Optional, Sequence

import numpy as np

from .models.mlp import LayerSpec, MLPSpec, normalize_activation

log = logging.getLogger(__name__)

DEFAULT_LAYER_DISTRIBUTION = [1]  # run_grpc_fcnn.py:23
NATIVE_PARSE_THRESHOLD = 32 << 20  # bytes; above this the streaming C++ parser is used


@dataclass
class LayerWeights:
    weight: np.ndarray  # [out][in] (float64 from Python json, float32 from the native parser)
    bias: np.ndarray    # [out]
    activation: str = "linear"  # as written in the file (first neuron)
    type: str = ""
    nodes: int = 0      # declared "nodes"
    mixed_activation: bool = False

    @property
    def in_dim(self) -> int:
        return int(self.weight.shape[1]) if self.weight.ndim == 2 else 0

    @property
    def out_dim(self) -> int:
        return int(self.weight.shape[0])


@dataclass
class ModelConfig:
    layers: list[LayerWeights]
    layer_distribution: Optional[list[int]] = None
    wrapped: bool = False
    stage_file: bool = False
    inference_metrics: Optional[dict] = None
    source: str = ""

    @property
    def distribution(self) -> list[int]:
        return list(self.layer_distribution or DEFAULT_LAYER_DISTRIBUTION)

    def spec(self, case_sensitive: bool = True) -> MLPSpec:
        """Validated MLPSpec; raises ValueError on a width mismatch (the reference's
        ``np.dot`` ValueError for the same file, grpc_node.py:83-87)."""
        specs = []
        for i, L in enumerate(self.layers):
            if i and L.in_dim != self.layers[i - 1].out_dim:
                raise ValueError(
                    f"Layer {i + 1}: expected input dim {self.layers[i - 1].out_dim}, "
                    f"got {L.in_dim}")
            specs.append(LayerSpec(L.in_dim, L.out_dim,
                                   normalize_activation(L.activation, case_sensitive),
                                   L.type or ("output" if i == len(self.layers) - 1 else "hidden")))
        return MLPSpec(tuple(specs), name=os.path.basename(self.source) or "config")

    def layer_dicts(self) -> list[dict]:
        """Reference-schema layer dicts (used by the partitioner / stage files)."""
        return [layer_to_dict(L) for L in self.layers]


def neurons_from_arrays(w: np.ndarray, b: np.ndarray, activation: str) -> list[dict]:
    w = np.asarray(w, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return [{"weights": w[j].tolist(), "bias": float(b[j]), "activation": activation}
            for j in range(w.shape[0])]


def layer_to_dict(L: LayerWeights) -> dict:
    return {"type": L.type or "hidden", "nodes": L.nodes or L.out_dim,
            "neurons": neurons_from_arrays(L.weight, L.bias, L.activation)}


def _layer_from_neurons(neurons: Sequence[dict], type_: str = "", nodes: int = 0) -> LayerWeights:
    if not neurons:
        return LayerWeights(np.zeros((0, 0)), np.zeros(0), "linear", type_, nodes)
    try:
        w = np.array([n["weights"] for n in neurons], dtype=np.float64)
    except ValueError as e:
        raise ValueError(f"ragged neuron weights: {e}") from None
    if w.ndim > 2:  # 2-D weight lists are flattened
        w = w.reshape(w.shape[0], -1)
    b = np.array([n.get("bias", 0.0) for n in neurons], dtype=np.float64)
    acts = [n.get("activation", "linear") for n in neurons]
    return LayerWeights(w, b, acts[0], type_, nodes or len(neurons),
                        any(a != acts[0] for a in acts))


def model_config_from_dict(cfg: dict, source: str = "") -> ModelConfig:
    wrapped = False
    metrics = None
    if "layers" not in cfg and isinstance(cfg.get("model"), dict):
        wrapped = True
        metrics = cfg.get("inference_metrics")
        body = cfg["model"]
    else:
        body = cfg
    dist = cfg.get("layer_distribution", body.get("layer_distribution"))
    if "layers" in body:
        layers = [_layer_from_neurons(l.get("neurons", []), l.get("type", ""),
                                      int(l.get("nodes", 0) or 0)) for l in body["layers"]]
        stage_file = False
    else:
        keys = [k for k in body if k.startswith("layer_") and isinstance(body[k], list)]
        if not keys:
            raise KeyError("'layers'")  # the reference's failure for such a file
        keys.sort(key=lambda k: int(k.split("_")[1]))  # grpc_node.py:46
        layers = [_layer_from_neurons(body[k]) for k in keys if body[k]]  # :49 skip empty
        stage_file = True
    out = ModelConfig(layers, list(dist) if dist is not None else None, wrapped, stage_file,
                      metrics, source)
    _warn_mixed(out)
    return out


def _warn_mixed(mc: ModelConfig) -> None:
    for i, L in enumerate(mc.layers):
        if L.mixed_activation:
            warnings.warn(f"layer {i + 1}: neurons have different activations; using the first "
                          f"({L.activation!r}) for the whole layer like the reference stage worker")


def load_model_config(path: str, native_parser: Optional[bool] = None) -> ModelConfig:
    """Load any of the accepted model files. Large files go through the C++ parser."""
    size = os.path.getsize(path)
    use_native = native_parser if native_parser is not None else size > NATIVE_PARSE_THRESHOLD
    if use_native:
        from .utils.native import native

        pm = native().parse_neuron_json(path)
        layers = [LayerWeights(d["weights"], d["bias"], d["activation"], d["type"], d["nodes"],
                               d["mixed_activation"]) for d in pm["layers"]]
        dist = list(pm["layer_distribution"]) if pm["has_distribution"] else None
        mc = ModelConfig(layers, dist, pm["wrapped"], pm["stage_file"], None, path)
        _warn_mixed(mc)
        return mc
    with open(path, "r") as f:
        cfg = json.load(f)
    return model_config_from_dict(cfg, source=path)
