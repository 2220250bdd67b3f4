"""Inputs: the reference's example files and synthetic MNIST-shaped data.

* :func:`load_examples` reads ``{"examples": [{"input": [...], "label": int}, ...]}`` and the
  raw-list form ``{"examples": [[...], ...]}`` (/root/reference/src/run_grpc_inference.py:35-52,
  /root/reference/scripts/manual_nn.py:85). Big files (the default client file holds 60,000
  examples x 784 doubles) go through the streaming C++ parser.
* :func:`synthetic_mnist` makes MNIST-shaped data (784 features in [0,1), 10 classes) whose
  labels come from a fixed random teacher network, so training on it is learnable and loss
  curves are meaningful -- there is no network access for the real MNIST.
* :class:`DeviceDataset` keeps the whole set resident in HBM as padded bf16 (the
  MI355X-first data path: 60k x 832 bf16 is 100 MB of 288 GB) and hands out batches by slicing.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from .models.mlp import round_up

NATIVE_PARSE_THRESHOLD = 16 << 20


@dataclass
class Examples:
    x: np.ndarray         # [n][dim] float32 (nested inputs flattened)
    labels: np.ndarray    # [n] int32, -1 when absent
    outer_len: int = 0    # len(input) of the first example (reference input-dim rule)
    raw_list: bool = False

    def __len__(self) -> int:
        return int(self.x.shape[0])

    @property
    def dim(self) -> int:
        return int(self.x.shape[1]) if self.x.ndim == 2 else 0


def load_examples(path: str, native_parser: Optional[bool] = None) -> Examples:
    size = os.path.getsize(path)
    if native_parser if native_parser is not None else size > NATIVE_PARSE_THRESHOLD:
        from .utils.native import native

        d = native().parse_examples_json(path)
        return Examples(d["x"], d["labels"], d["outer_len"], d["raw_list"])
    with open(path) as f:
        doc = json.load(f)
    return examples_from_list(doc.get("examples", []))


def examples_from_list(examples: list) -> Examples:
    if not examples:
        return Examples(np.zeros((0, 0), np.float32), np.zeros(0, np.int32))
    raw = not isinstance(examples[0], dict)
    xs, ys = [], []
    for ex in examples:
        inp = ex if raw else ex.get("input")
        xs.append(np.asarray(inp, dtype=np.float32).reshape(-1))
        lab = None if raw else ex.get("label")
        ys.append(-1 if lab is None else int(lab))
    first = examples[0] if raw else examples[0].get("input")
    outer = len(first) if isinstance(first, list) else 0
    dims = {x.size for x in xs}
    if len(dims) != 1:
        raise ValueError(f"examples have different input sizes: {sorted(dims)}")
    return Examples(np.stack(xs), np.asarray(ys, np.int32), outer, raw)


def write_examples(path: str, x: np.ndarray, labels: Optional[np.ndarray] = None,
                   raw_list: bool = False) -> None:
    x = np.asarray(x, dtype=np.float64)
    if raw_list:
        doc = {"examples": [row.tolist() for row in x]}
    else:
        doc = {"examples": [{"input": x[i].tolist(),
                             "label": int(labels[i]) if labels is not None else None}
                            for i in range(x.shape[0])]}
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        json.dump(doc, f)


def synthetic_mnist(n: int, seed: int = 0, dim: int = 784, n_classes: int = 10,
                    noise: float = 0.05) -> tuple[np.ndarray, np.ndarray]:
    """MNIST-shaped synthetic data with teacher labels (float32 x in [0,1), int32 labels)."""
    rng = np.random.default_rng(seed)
    teacher_rng = np.random.default_rng(12345)  # fixed teacher across seeds / splits
    t1 = teacher_rng.standard_normal((dim, 64)).astype(np.float32) / np.sqrt(dim)
    t2 = teacher_rng.standard_normal((64, n_classes)).astype(np.float32) / 8.0
    # sparse-ish "images": most pixels dark like MNIST
    x = rng.random((n, dim), dtype=np.float32)
    x *= (rng.random((n, dim), dtype=np.float32) < 0.2)
    h = np.maximum((x - 0.1) @ t1, 0.0)
    logits = h @ t2 + noise * rng.standard_normal((n, n_classes)).astype(np.float32)
    return x, np.argmax(logits, axis=1).astype(np.int32)


def synthetic_digits(n: int, seed: int = 0, dim: int = 784, n_classes: int = 10,
                     noise: float = 0.35) -> tuple[np.ndarray, np.ndarray]:
    """Class-template synthetic MNIST stand-in: each class has a fixed sparse "digit" template
    (shared across seeds / splits); a sample is its class template with per-pixel jitter, a
    random stroke-intensity scale and background noise -- learnable to > 95 % like MNIST, so
    training recipes can be compared on accuracy (no dataset is available offline)."""
    rng = np.random.default_rng(seed)
    trng = np.random.default_rng(4242)
    templates = (trng.random((n_classes, dim)) < 0.15).astype(np.float32)
    templates *= trng.uniform(0.5, 1.0, (n_classes, dim)).astype(np.float32)
    y = rng.integers(0, n_classes, n).astype(np.int32)
    scale = rng.uniform(0.6, 1.2, (n, 1)).astype(np.float32)
    keep = (rng.random((n, dim)) > 0.25).astype(np.float32)  # dropped strokes
    x = templates[y] * scale * keep
    x += noise * rng.random((n, dim), dtype=np.float32) * (rng.random((n, dim)) < 0.3)
    return np.clip(x, 0.0, 1.0).astype(np.float32), y


def tiled_inference_set(x: np.ndarray, y: np.ndarray, frac: float = 0.1, tiles: int = 10):
    """The notebook's 60k inference set: last 10% tiled x10 (…ipynb:257-266)."""
    k = int(round(len(x) * (1 - frac)))
    return np.tile(x[k:], (tiles, 1)), np.tile(y[k:], tiles)


class DeviceDataset:
    """Resident padded-bf16 dataset; ``batch(i)`` returns views, no host traffic per step."""

    def __init__(self, x: np.ndarray, labels: np.ndarray, batch_rows: int,
                 device: torch.device, kp: Optional[int] = None, min_batches: int = 2):
        n, dim = x.shape
        self.dim = dim
        self.kp = kp or round_up(dim, 64)
        self.batch_rows = batch_rows
        nb = max(min_batches, -(-n // batch_rows))
        self.num_batches = nb
        rows = nb * batch_rows
        idx = np.arange(rows) % n  # wrap to fill whole batches
        xt = torch.from_numpy(np.ascontiguousarray(x[idx], dtype=np.float32))
        self.x = torch.zeros(rows, self.kp, dtype=torch.bfloat16, device=device)
        self.x[:, :dim] = xt.to(device=device, dtype=torch.bfloat16)
        self.labels = torch.from_numpy(np.ascontiguousarray(labels[idx], dtype=np.int32)).to(device)

    def batch(self, i: int) -> tuple[torch.Tensor, torch.Tensor]:
        b = i % self.num_batches
        r0 = b * self.batch_rows
        return self.x[r0:r0 + self.batch_rows], self.labels[r0:r0 + self.batch_rows]


class FanDataset:
    """The rows one rank of a replicated-stage pipeline (parallel/fan.py) holds: micro-batch j
    of the global batch is ``synthetic_mnist(mb, seed + 7919 * b + j)`` for alternating batch
    b in {0, 1}, so the first stage's replica of j and the last stage's replica of j -- on
    different ranks -- hold the inputs and labels of the SAME samples without any rank
    generating the whole global batch. ``batch(i)`` returns this rank's rows (its
    micro-batches in local order), resident in HBM like DeviceDataset."""

    def __init__(self, micros, mb: int, device: torch.device, kp: Optional[int] = None,
                 seed: int = 0, inputs: bool = True, labels: bool = True,
                 label_micros=None):
        """``micros``: the global micro-batches whose inputs this rank holds (its first-stage
        replica's); ``label_micros``: those whose labels it holds (its last-stage replica's;
        default ``micros`` -- they differ on a rank hosting co-located stages)."""
        label_micros = micros if label_micros is None else label_micros
        self.batches = []
        for b in range(2):
            xt = yt = None
            if inputs and micros:
                xs = [synthetic_mnist(mb, seed=seed + 7919 * b + j)[0] for j in micros]
                dim = xs[0].shape[1]
                kpp = kp or round_up(dim, 64)
                xt = torch.zeros(len(micros) * mb, kpp, dtype=torch.bfloat16, device=device)
                xt[:, :dim] = torch.from_numpy(np.concatenate(xs)).to(device, torch.bfloat16)
            if labels and label_micros:
                ys = [synthetic_mnist(mb, seed=seed + 7919 * b + j)[1] for j in label_micros]
                yt = torch.from_numpy(np.concatenate(ys)).to(device)
            self.batches.append((xt, yt))

    def batch(self, i: int):
        return self.batches[i % 2]
