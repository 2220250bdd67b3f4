"""Checkpoint / resume (the reference has none: its weights are immutable inputs).

Layout of a checkpoint directory:
  ``meta.json``                       model widths/activations, layer_distribution, step
  ``stage{s}.safetensors``            per pipeline stage (written by DP replica 0): the flat
                                      fp32 master buffer, optimizer state buffers, and each
                                      layer's UNPADDED ``w{L}``/``b{L}`` (global layer index L)
Resume:
  * same layout -> :func:`load_stage` restores master + optimizer state exactly;
  * different layout -> :func:`load_full_weights` reassembles every layer from the shards and
    the trainer re-partitions them (optimizer state restarts).
Export to the reference's neuron-JSON model format: :func:`export_json`.
safetensors only (no pickle); loading never executes code from the file.
"""
from __future__ import annotations

import json
import os
from typing import Optional, Sequence

import numpy as np
import torch
from safetensors.torch import load_file, save_file

from .models.mlp import MLPSpec


def _meta_path(d: str) -> str:
    return os.path.join(d, "meta.json")


def save_stage(d: str, stage, step: int, spec: MLPSpec, distribution: Sequence[int],
               extra: Optional[dict] = None) -> str:
    os.makedirs(d, exist_ok=True)
    p = stage.params
    tensors = {"master": p.master.detach().cpu().contiguous()}
    for k, t in enumerate(p.state):
        tensors[f"state{k}"] = t.detach().cpu().contiguous()
    ws, bs = p.export()
    for k, (w, b) in enumerate(zip(ws, bs)):
        tensors[f"w{stage.l0 + k}"] = torch.from_numpy(np.ascontiguousarray(w))
        tensors[f"b{stage.l0 + k}"] = torch.from_numpy(np.ascontiguousarray(b))
    path = os.path.join(d, f"stage{stage.stage_index}.safetensors")
    save_file(tensors, path, metadata={"step": str(step), "l0": str(stage.l0),
                                       "l1": str(stage.l1), "opt_steps": str(p.step_count),
                                       "optimizer": p.optim.name})
    if stage.stage_index == 0:
        meta = {"widths": spec.widths, "activations": [l.activation for l in spec.layers],
                "layer_distribution": list(distribution), "step": step, **(extra or {})}
        with open(_meta_path(d), "w") as f:
            json.dump(meta, f)
    return path


def read_meta(d: str) -> dict:
    with open(_meta_path(d)) as f:
        return json.load(f)


def load_stage(d: str, stage) -> int:
    """Restore a stage saved with the SAME layout; returns the saved step."""
    path = os.path.join(d, f"stage{stage.stage_index}.safetensors")
    t = load_file(path)
    from safetensors import safe_open

    with safe_open(path, framework="pt") as f:
        md = f.metadata()
    if int(md["l0"]) != stage.l0 or int(md["l1"]) != stage.l1:
        raise ValueError("checkpoint layout differs; use load_full_weights + re-partition")
    p = stage.params
    if t["master"].numel() != p.master.numel():
        raise ValueError("checkpoint geometry mismatch")
    p.master.copy_(t["master"].to(p.master.device))
    for k, s in enumerate(p.state):
        if f"state{k}" in t:
            s.copy_(t[f"state{k}"].to(s.device))
    p.set_step(int(md.get("opt_steps", 0)))
    p.refresh_shadow()
    return int(md["step"])


def load_full_weights(d: str) -> tuple[list[np.ndarray], list[np.ndarray], dict]:
    meta = read_meta(d)
    n = len(meta["widths"]) - 1
    ws: list = [None] * n
    bs: list = [None] * n
    for fn in sorted(os.listdir(d)):
        if fn.startswith("stage") and fn.endswith(".safetensors"):
            t = load_file(os.path.join(d, fn))
            for k, v in t.items():
                if k[0] in "wb" and k[1:].isdigit():
                    (ws if k[0] == "w" else bs)[int(k[1:])] = v.numpy()
    if any(w is None for w in ws) or any(b is None for b in bs):
        raise ValueError(f"checkpoint {d} is missing layers")
    return ws, bs, meta


def export_json(d: str, out_path: str, wrapped: bool = False,
                inference_metrics: Optional[dict] = None) -> None:
    from .weights_io import export_model_json

    ws, bs, meta = load_full_weights(d)
    export_model_json(out_path, ws, bs, meta["activations"],
                      layer_distribution=meta.get("layer_distribution"), wrapped=wrapped,
                      inference_metrics=inference_metrics)
