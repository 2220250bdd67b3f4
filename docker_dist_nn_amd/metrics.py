"""Metrics: classification quality, latency distributions, and a JSONL metrics stream.

The notebook reports accuracy and weighted precision/recall/F1 (``average='weighted',
zero_division=0``) plus total and per-sample latency, embedded as ``inference_metrics`` in the
exported model (/root/reference/scripts/Centralized_MNIST_Experimentation.ipynb:385-398,
495-502). :func:`classification_report` computes the same numbers without sklearn at runtime;
the reference client's log lines are reproduced in ``run_grpc_inference.py``.
"""
from __future__ import annotations

import json
import os
import time
from dataclasses import dataclass, field
from typing import Optional

import numpy as np


def classification_report(y_true, y_pred, n_classes: Optional[int] = None) -> dict:
    y_true = np.asarray(y_true).astype(np.int64)
    y_pred = np.asarray(y_pred).astype(np.int64)
    n = len(y_true)
    if n == 0:
        return {"accuracy": 0.0, "precision": 0.0, "recall": 0.0, "f1_score": 0.0}
    k = n_classes or int(max(y_true.max(), y_pred.max()) + 1)
    cm = np.zeros((k, k), np.int64)
    np.add.at(cm, (y_true, y_pred), 1)
    tp = np.diag(cm).astype(np.float64)
    support = cm.sum(1).astype(np.float64)
    pred_cnt = cm.sum(0).astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        prec = np.where(pred_cnt > 0, tp / pred_cnt, 0.0)
        rec = np.where(support > 0, tp / support, 0.0)
        f1 = np.where(prec + rec > 0, 2 * prec * rec / (prec + rec), 0.0)
    w = support / support.sum()
    return {"accuracy": float(tp.sum() / n), "precision": float((prec * w).sum()),
            "recall": float((rec * w).sum()), "f1_score": float((f1 * w).sum())}


@dataclass
class LatencyStats:
    samples: list = field(default_factory=list)

    def add(self, seconds: float) -> None:
        self.samples.append(float(seconds))

    def summary(self) -> dict:
        if not self.samples:
            return {}
        a = np.asarray(self.samples)
        return {"n": int(a.size), "mean_s": float(a.mean()), "p50_s": float(np.percentile(a, 50)),
                "p90_s": float(np.percentile(a, 90)), "p99_s": float(np.percentile(a, 99)),
                "min_s": float(a.min()), "max_s": float(a.max())}


class MetricsWriter:
    """Append-only JSONL stream (one record per step/event, rank-tagged)."""

    def __init__(self, path: Optional[str], rank: int = 0):
        self.path = path
        self.rank = rank
        self._f = None
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
            self._f = open(path, "a", buffering=1)

    def write(self, kind: str, **fields) -> None:
        if self._f is None:
            return
        rec = {"ts": time.time(), "rank": self.rank, "kind": kind, **fields}
        self._f.write(json.dumps(rec) + "\n")

    def close(self) -> None:
        if self._f is not None:
            self._f.close()
            self._f = None
