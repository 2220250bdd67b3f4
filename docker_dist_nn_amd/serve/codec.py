"""Matrix <-> numpy through the native protobuf codec (csrc/runtime/matrix_codec.cpp)."""
from __future__ import annotations

import numpy as np

from ..utils.native import native


def decode(data: bytes) -> np.ndarray:
    """Matrix wire bytes -> float64 [rows][cols] (ValueError on ragged rows)."""
    try:
        return native().decode_matrix(data)
    except (RuntimeError, ValueError) as e:
        raise ValueError(str(e)) from None


def encode(a) -> bytes:
    a = np.asarray(a, dtype=np.float64)
    if a.ndim == 1:
        a = a[None, :]
    return native().encode_matrix(np.ascontiguousarray(a))
