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
table file (A/B of two tunings). Such a file may be an override table --
``{"base": "default", "override": {signature: entry or null}}`` -- which is the default table
with those entries replaced (null: removed); experiment tables are kept in that form
(``scripts/table_diff.py`` converts full copies).
"""
from __future__ import annotations

import json
import os
from typing import Optional
from .. import switches

DEFAULT_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned_gfx950.json")
TABLE_PATH = switches.get("DNN_TUNED_TABLE") or DEFAULT_PATH
_table: Optional[dict] = None


def load_table(path: str) -> dict:
    """Entries of a table file; an override table is applied on top of the default table."""
    with open(path) as f:
        doc = json.load(f)
    if "override" not in doc:
        return doc.get("entries", {})
    if doc.get("base", "default") != "default":
        raise ValueError(f"{path}: override tables apply to the default table only")
    with open(DEFAULT_PATH) as f:
        entries = dict(json.load(f).get("entries", {}))
    for k, v in doc["override"].items():
        if v is None:
            entries.pop(k, None)
        else:
            entries[k] = v
    return entries


def _load() -> dict:
    global _table
    if _table is None:
        try:
            _table = load_table(TABLE_PATH)
        except FileNotFoundError:
            if TABLE_PATH != DEFAULT_PATH:  # an explicitly requested table must exist
                raise
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
