"""Device buffers torch's caching allocator cannot make: L2-uncached memory for the receive side
of xGMI peer writes (csrc/runtime/p2p.hpp alloc_uncached).

A peer GPU's stores land in this GPU's HBM without invalidating its L2s (one per XCD, not
coherent with one another or with the peer), so a buffer that is rewritten remotely every step
and read locally by GEMMs would otherwise risk serving the previous step's rows from L2. The
buffers are wrapped as torch tensors through ``__cuda_array_interface__`` (no copy) and freed at
process exit.
"""
from __future__ import annotations

import atexit
import math

import torch

from .native import native


class _Raw:
    """A device byte range exposed through __cuda_array_interface__ (torch.as_tensor wraps it
    without copying)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1",
                                         "data": (ptr, False), "version": 3, "strides": None}


_LIVE: dict[int, torch.Tensor] = {}


def uncached_zeros(shape, dtype: torch.dtype, device: torch.device) -> torch.Tensor:
    """Zeroed ``shape`` tensor of ``dtype`` on ``device`` in L2-uncached memory."""
    nbytes = math.prod(shape) * torch.empty((), dtype=dtype).element_size()
    with torch.cuda.device(device):
        ptr = native().alloc_uncached(max(16, nbytes))
        raw = torch.as_tensor(_Raw(ptr, max(16, nbytes)), device=device)
    if raw.data_ptr() != ptr:
        raise RuntimeError("uncached buffer was copied instead of wrapped")
    _LIVE[ptr] = raw
    return raw[:nbytes].view(dtype).view(*shape)


@atexit.register
def _free_all() -> None:
    if not _LIVE:
        return
    try:
        torch.cuda.synchronize()
    except Exception:  # noqa: BLE001 -- exiting anyway
        pass
    n = native()
    for ptr in list(_LIVE):
        n.free_device(ptr)
    _LIVE.clear()
