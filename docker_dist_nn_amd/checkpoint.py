"""Checkpoint / resume (the reference has none: its weights are immutable inputs, and its only
persistence is the notebook's offline JSON export, …ipynb:464-506).

Layout of a checkpoint directory::

  meta.json                          the COMMIT MARKER: model widths/activations,
                                     layer_distribution, step, optimizer, and the exact list of
                                     shard files that make up this checkpoint
  stage{s}.step{N}.safetensors       one shard per pipeline stage (written by DP replica 0):
                                     each layer's UNPADDED ``w{L}`` / ``b{L}`` (global layer
                                     index L) and optimizer state ``s{k}.w{L}`` / ``s{k}.b{L}``

Protocol (crash-safe, layout-independent):

* every shard is written to a temporary name and ``os.replace``-d into place; shard names carry
  the step, so a new save never overwrites a shard the committed ``meta.json`` names;
* after every stage's shard is on disk (the caller's barrier across ranks), the owner of
  stage 0 writes ``meta.json`` the same way -- that replace is the commit -- and then deletes
  every shard the new meta does not name (older steps, stages of an older layout);
* loading reads ONLY the shards named by ``meta.json`` and checks that each carries the
  committed step and the layer range the layout implies. A crash mid-save therefore leaves the
  previous checkpoint intact, and stale shards of an older ``layer_distribution`` can never be
  mixed in.

Everything is stored per layer and unpadded, so a resume onto a different
``layer_distribution`` restores weights AND optimizer state (momentum / Adam moments and the
update counter) exactly: :func:`restore_trainer`. Export to the reference's neuron-JSON model
format: :func:`export_json`. safetensors only (no pickle); loading executes nothing from the
file.
"""
from __future__ import annotations

import glob
import json
import os
import re
from typing import Callable, Optional, Sequence

import numpy as np
import torch
from safetensors import safe_open
from safetensors.torch import load_file, save_file

from .models.mlp import MLPSpec

FORMAT = 2
_SHARD_RE = re.compile(r"^stage(\d+)\.step(\d+)\.safetensors$")


def _meta_path(d: str) -> str:
    return os.path.join(d, "meta.json")


def shard_name(stage_index: int, step: int) -> str:
    return f"stage{stage_index}.step{step}.safetensors"


def _atomic_json(path: str, obj: dict) -> None:
    tmp = f"{path}.tmp.{os.getpid()}"
    with open(tmp, "w") as f:
        json.dump(obj, f)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def save_stage(d: str, stage, step: int, spec: MLPSpec, distribution: Sequence[int],
               extra: Optional[dict] = None) -> str:
    """Write this stage's shard for ``step`` (not yet committed: see :func:`commit`)."""
    del spec, distribution, extra  # recorded by commit()
    os.makedirs(d, exist_ok=True)
    p = stage.params
    tensors = {}
    ws, bs = p.export()
    for k, (w, b) in enumerate(zip(ws, bs)):
        tensors[f"w{stage.l0 + k}"] = torch.from_numpy(np.ascontiguousarray(w))
        tensors[f"b{stage.l0 + k}"] = torch.from_numpy(np.ascontiguousarray(b))
    for s in range(len(p.state)):
        sw, sb = p.export_state(s)
        for k, (w, b) in enumerate(zip(sw, sb)):
            tensors[f"s{s}.w{stage.l0 + k}"] = torch.from_numpy(np.ascontiguousarray(w))
            tensors[f"s{s}.b{stage.l0 + k}"] = torch.from_numpy(np.ascontiguousarray(b))
    path = os.path.join(d, shard_name(stage.stage_index, step))
    tmp = f"{path}.tmp.{os.getpid()}"
    save_file(tensors, tmp, metadata={"step": str(step), "l0": str(stage.l0),
                                      "l1": str(stage.l1), "opt_steps": str(p.step_count),
                                      "optimizer": p.optim.name, "n_state": str(len(p.state))})
    os.replace(tmp, path)
    return path


def commit(d: str, step: int, spec: MLPSpec, distribution: Sequence[int],
           optimizer: str, extra: Optional[dict] = None) -> dict:
    """Publish the shards of ``step`` as THE checkpoint (call once, after every stage's
    :func:`save_stage` finished), then delete every shard it does not name."""
    dist_ = [int(x) for x in distribution]
    n_stages = sum(1 for x in dist_ if x)
    shards = [shard_name(s, step) for s in range(n_stages)]
    missing = [s for s in shards if not os.path.exists(os.path.join(d, s))]
    if missing:
        raise RuntimeError(f"checkpoint commit of step {step}: shards not written: {missing}")
    meta = {"format": FORMAT, "widths": spec.widths,
            "activations": [l.activation for l in spec.layers],
            "layer_distribution": dist_, "step": int(step), "optimizer": optimizer,
            "shards": shards, **(extra or {})}
    _atomic_json(_meta_path(d), meta)
    keep = set(shards)
    for p in glob.glob(os.path.join(d, "stage*.safetensors")):
        if os.path.basename(p) not in keep:
            os.remove(p)
    return meta


def save_trainer(d: str, trainer, step: int, *, barrier: Optional[Callable[[], None]] = None,
                 is_writer: bool = True, extra: Optional[dict] = None) -> None:
    """Checkpoint every stage this process holds; the process holding stage 0 commits after
    ``barrier`` (all ranks must call this; ``is_writer`` False on DP replicas > 0, which only
    take part in the barrier)."""
    trainer.flush()  # deferred DP update of the last step
    gather = getattr(trainer, "gather_sharded", None)
    if gather is not None:  # sharded DP: every rank (collective) makes master / state whole
        gather()
    if is_writer:
        for st in trainer.stages:
            save_stage(d, st, step, trainer.spec, trainer.distribution)
    if barrier is not None:
        barrier()
    if is_writer and trainer.stages[0].stage_index == 0:
        commit(d, step, trainer.spec, trainer.distribution, trainer.optim.name, extra)
    if barrier is not None:
        barrier()  # nobody resumes / exports before the commit is visible


def read_meta(d: str) -> dict:
    with open(_meta_path(d)) as f:
        meta = json.load(f)
    if meta.get("format") != FORMAT or "shards" not in meta:
        if meta.get("format") == 1 or "shards" not in meta:
            raise ValueError(
                f"{d}: format-1 checkpoint (per-stage stage{{s}}.safetensors, no shard list): "
                f"this version reads format {FORMAT} only. Migrate by exporting the weights with "
                f"the version that wrote it (neuron JSON) and starting from that JSON "
                f"(cli/train.py --config), or train from scratch into a fresh directory; "
                f"--resume on this directory would otherwise discard its shards on commit")
        raise ValueError(f"{d}: not a format-{FORMAT} checkpoint (meta format "
                         f"{meta.get('format')!r})")
    return meta


def _shard_ranges(meta: dict) -> list[tuple[int, int]]:
    out, l0 = [], 0
    for n in meta["layer_distribution"]:
        if n:
            out.append((l0, l0 + n))
        l0 += n
    return out


def _read_shard(d: str, meta: dict, s: int) -> tuple[dict, dict]:
    path = os.path.join(d, meta["shards"][s])
    with safe_open(path, framework="pt") as f:
        md = f.metadata()
    l0, l1 = _shard_ranges(meta)[s]
    if int(md["step"]) != int(meta["step"]):
        raise ValueError(f"{path}: shard step {md['step']} != committed step {meta['step']}")
    if (int(md["l0"]), int(md["l1"])) != (l0, l1):
        raise ValueError(f"{path}: shard holds layers [{md['l0']},{md['l1']}) but the "
                         f"committed layout assigns [{l0},{l1})")
    return load_file(path), md


def load_full_state(d: str) -> dict:
    """Every layer's weights, biases and optimizer state from the committed shards:
    ``{"w": [..], "b": [..], "state": [(ws, bs), ...], "opt_steps": n, "meta": meta}``."""
    meta = read_meta(d)
    n = len(meta["widths"]) - 1
    ws: list = [None] * n
    bs: list = [None] * n
    n_state, opt_steps, state = None, None, None
    for s in range(len(meta["shards"])):
        t, md = _read_shard(d, meta, s)
        k_state = int(md.get("n_state", 0))
        if n_state is None:
            n_state, opt_steps = k_state, int(md.get("opt_steps", 0))
            state = [([None] * n, [None] * n) for _ in range(n_state)]
        elif k_state != n_state or int(md.get("opt_steps", 0)) != opt_steps:
            raise ValueError(f"{d}: shards disagree on optimizer state / update count")
        for key, v in t.items():
            m = re.fullmatch(r"(?:s(\d+)\.)?([wb])(\d+)", key)
            if not m:
                continue
            arr, li = v.numpy(), int(m.group(3))
            if m.group(1) is None:
                (ws if m.group(2) == "w" else bs)[li] = arr
            else:
                state[int(m.group(1))][0 if m.group(2) == "w" else 1][li] = arr
    if any(w is None for w in ws) or any(b is None for b in bs):
        raise ValueError(f"checkpoint {d} is missing layers")
    return {"w": ws, "b": bs, "state": state or [], "opt_steps": opt_steps or 0, "meta": meta}


def load_full_weights(d: str) -> tuple[list[np.ndarray], list[np.ndarray], dict]:
    st = load_full_state(d)
    return st["w"], st["b"], st["meta"]


def restore_trainer(d: str, trainer) -> int:
    """Resume ``trainer`` (any layout: the checkpoint's or a new ``layer_distribution``) from
    the committed checkpoint in ``d``: weights, optimizer state and update counter. Optimizer
    state is dropped (with the counter) only if the optimizer kind changed. Returns the step."""
    st = load_full_state(d)
    meta = st["meta"]
    if list(meta["widths"]) != list(trainer.spec.widths):
        raise ValueError(f"checkpoint widths {meta['widths']} != model {trainer.spec.widths}")
    acts = [l.activation for l in trainer.spec.layers]
    if meta.get("activations") is not None and list(meta["activations"]) != acts:
        raise ValueError(f"checkpoint activations {meta['activations']} != model {acts}")
    same_opt = meta.get("optimizer") == trainer.optim.name
    for stage in trainer.stages:
        p = stage.params
        p.load(st["w"][stage.l0:stage.l1], st["b"][stage.l0:stage.l1])
        if same_opt and len(st["state"]) == len(p.state):
            for k, (sw, sb) in enumerate(st["state"]):
                p.load_state(k, sw[stage.l0:stage.l1], sb[stage.l0:stage.l1])
            p.set_step(st["opt_steps"])
        else:
            for s in p.state:
                s.zero_()
            p.set_step(0)
    return int(meta["step"])


def load_stage(d: str, stage) -> int:
    """Restore one stage (weights + optimizer state) from a committed checkpoint of any layout;
    returns the committed step."""
    st = load_full_state(d)
    p = stage.params
    p.load(st["w"][stage.l0:stage.l1], st["b"][stage.l0:stage.l1])
    if st["meta"].get("optimizer") == p.optim.name and len(st["state"]) == len(p.state):
        for k, (sw, sb) in enumerate(st["state"]):
            p.load_state(k, sw[stage.l0:stage.l1], sb[stage.l0:stage.l1])
        p.set_step(st["opt_steps"])
    return int(st["meta"]["step"])


def export_json(d: str, out_path: str, wrapped: bool = False,
                inference_metrics: Optional[dict] = None) -> None:
    from .weights_io import export_model_json

    ws, bs, meta = load_full_weights(d)
    export_model_json(out_path, ws, bs, meta["activations"],
                      layer_distribution=meta.get("layer_distribution"), wrapped=wrapped,
                      inference_metrics=inference_metrics)
