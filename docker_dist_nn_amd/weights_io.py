"""Weight IO in the reference's per-neuron JSON format, plus per-stage files.

* :func:`export_model_json` writes the full model file (``{"layers": ..., "layer_distribution"}``
  or the notebook's ``{"model": ..., "inference_metrics": ...}`` wrapping,
  /root/reference/scripts/Centralized_MNIST_Experimentation.ipynb:464-506);
* :func:`write_stage_files` writes ``<cache>/<layer_container_i>_neurons_config.json`` with
  ``{"layer_1": [...], ...}`` exactly as the reference launcher does for large stages
  (/root/reference/src/run_grpc_fcnn.py:91-127), so the files can be inspected or fed to any
  consumer of the reference format.
Large models use the streaming C++ writer (``_native.write_neuron_json``).
"""
from __future__ import annotations

import json
import os
from typing import Optional, Sequence

import numpy as np

from .config import LayerWeights, ModelConfig, load_model_config, neurons_from_arrays
from .partition import calculate_layer_mappings

NEURON_CONFIG_SIZE_THRESHOLD = 1000  # run_grpc_fcnn.py:91 (env var vs file)
NATIVE_WRITE_THRESHOLD = 4_000_000   # parameters; above this use the C++ writer


def _as_f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def export_model_json(path: str, weights: Sequence[np.ndarray], biases: Sequence[np.ndarray],
                      activations: Sequence[str], layer_distribution: Optional[Sequence[int]] = None,
                      wrapped: bool = False, inference_metrics: Optional[dict] = None,
                      types: Optional[Sequence[str]] = None) -> None:
    n = len(weights)
    types = list(types) if types else ["output" if i == n - 1 else "hidden" for i in range(n)]
    nparams = sum(int(np.asarray(w).size) for w in weights)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    if nparams > NATIVE_WRITE_THRESHOLD and not wrapped:
        from .utils.native import native

        native().write_neuron_json(path, [_as_f32(w) for w in weights],
                                   [_as_f32(b) for b in biases], list(activations), types,
                                   list(layer_distribution or []), False)
        return
    layers = [{"type": types[i], "nodes": int(np.asarray(weights[i]).shape[0]),
               "neurons": neurons_from_arrays(weights[i], biases[i], activations[i])}
              for i in range(n)]
    if wrapped:
        doc = {"model": {"layers": layers}, "inference_metrics": inference_metrics or {}}
        if layer_distribution is not None:
            doc["layer_distribution"] = list(layer_distribution)
    else:
        doc = {"layers": layers}
        if layer_distribution is not None:
            doc["layer_distribution"] = list(layer_distribution)
    with open(path, "w") as f:
        json.dump(doc, f)


def write_stage_files(cache_dir: str, mappings: dict[int, dict],
                      threshold: int = NEURON_CONFIG_SIZE_THRESHOLD) -> dict[int, dict]:
    """Materialise the per-stage neuron configs like the reference launcher.

    Returns, per container index, the env contract a stage process would get
    (run_grpc_fcnn.py:101-126): NEURONS_FILE_CONFIG for configs longer than ``threshold``
    characters, NEURONS_CONFIG inline otherwise.
    """
    os.makedirs(cache_dir, exist_ok=True)
    envs = {}
    for ci, m in mappings.items():
        env = {"CONTAINER_NAME": m["container_name"], "LISTEN_PORT": str(m["listen_port"]),
               "EXPECTED_INPUT_DIM": str(m["expected_input"]),
               "NEXT_NODES": json.dumps(m["next_nodes"])}
        s = json.dumps(m["neurons_config"])
        if len(s) > threshold:
            p = os.path.join(cache_dir, f"{m['container_name']}_neurons_config.json")
            with open(p, "w") as f:
                f.write(s)
            env["NEURONS_FILE_CONFIG"] = p
        else:
            env["NEURONS_CONFIG"] = s
        envs[ci] = env
    return envs


def stage_files_from_model(model: ModelConfig, cache_dir: str, input_dim: int,
                           distribution: Optional[Sequence[int]] = None) -> dict[int, dict]:
    dist = list(distribution or model.distribution)
    examples = [{"input": [0.0] * input_dim}] if input_dim else []
    mappings = calculate_layer_mappings(model.layer_dicts(), dist, examples)
    return write_stage_files(cache_dir, mappings)


def load_stage_env(env: dict) -> list[LayerWeights]:
    """Load a stage's layers from its env contract (grpc_node.py:22-55 semantics)."""
    if "NEURONS_CONFIG" in env:
        cfg = json.loads(env["NEURONS_CONFIG"])
    elif "NEURONS_FILE_CONFIG" in env:
        return load_model_config(env["NEURONS_FILE_CONFIG"]).layers
    else:
        raise RuntimeError("No neuron configuration provided (NEURONS_CONFIG or "
                           "NEURONS_FILE_CONFIG env var).")
    from .config import model_config_from_dict

    return model_config_from_dict(cfg).layers if cfg else []
