"""Measured GEMM configurations for gfx950 (a tuned-solution table, like a BLAS library's).

``tuned_gfx950.json`` maps a GEMM signature to the fastest (tile, split-K, pipeline depth)
measured on an MI355X by ``bench/tune.py``. The ops consult it first and fall back to the
analytic rules in :mod:`.kernels` for shapes it does not cover. Lookups are deterministic, so a
given shape always runs the same kernel configuration (bitwise-reproducible training).

Signatures (the GEMM as the kernel sees it: C[M][N] = sum over K):
  fwd   : M = rows, N = layer output width, K = layer input width (padded)
  dgrad : M = rows, N = layer input width,  K = layer output width
  wgrad : M = layer output width, N = layer input width, K = rows (split-K contraction)
``DNN_TUNED=0`` disables the table (A/B against the rules); ``DNN_TUNED_TABLE`` reads another
table file (A/B of two tunings).
"""
from __future__ import annotations

import json
import os
from typing import Optional
from .. import switches

TABLE_PATH = (switches.get("DNN_TUNED_TABLE") or
              os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned_gfx950.json"))
_table: Optional[dict] = None


def _load() -> dict:
    global _table
    if _table is None:
        try:
            with open(TABLE_PATH) as f:
                _table = json.load(f).get("entries", {})
        except FileNotFoundError:
            _table = {}
    return _table


def key(op: str, M: int, N: int, K: int) -> str:
    return f"{op}:{M}x{N}x{K}"


def lookup(op: str, M: int, N: int, K: int) -> Optional[dict]:
    """{"tile": [bm, bn], "splits": s, "stages": ns} or None."""
    if switches.get("DNN_TUNED") == "0":
        return None
    return _load().get(key(op, M, N, K))


def reload() -> None:
    global _table
    _table = None
