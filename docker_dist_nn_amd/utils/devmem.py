"""Device buffers torch's caching allocator cannot make: L2-uncached memory for the receive side
of xGMI peer writes (csrc/runtime/p2p.hpp alloc_uncached).

A peer GPU's stores land in this GPU's HBM without invalidating its L2s (one per XCD, not
coherent with one another or with the peer), so a buffer that is rewritten remotely every step
and read locally by GEMMs would otherwise risk serving the previous step's rows from L2. The
buffers are wrapped as torch tensors through ``__cuda_array_interface__`` (no copy).

Lifetime: torch keeps the exporting object alive as long as the tensor's storage (every view
included), so the owner below frees the allocation when the last view dies -- an IpcPipe that
is replaced or dropped releases its relay slots instead of pinning them for the life of the
process. Owners still alive at exit are freed by the atexit hook, before the HIP
runtime goes away. ``hipFree`` synchronises the device, so no kernel still reads the buffer.
"""
from __future__ import annotations

import atexit
import math
import weakref

import torch

from .native import native


class _Owner:
    """Owns one uncached allocation; exposed through __cuda_array_interface__ so that
    torch.as_tensor wraps it without copying (and keeps this object alive with the storage)."""

    def __init__(self, ptr: int, nbytes: int):
        self.ptr = ptr
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1",
                                         "data": (ptr, False), "version": 3, "strides": None}
        _LIVE.add(self)

    def free(self) -> None:
        if self.ptr:
            p, self.ptr = self.ptr, 0
            try:
                native().free_device(p)
            except Exception:  # noqa: BLE001 -- interpreter shutdown
                pass

    def __del__(self):
        self.free()


_LIVE: "weakref.WeakSet[_Owner]" = weakref.WeakSet()


def uncached_zeros(shape, dtype: torch.dtype, device: torch.device) -> torch.Tensor:
    """Zeroed ``shape`` tensor of ``dtype`` on ``device`` in L2-uncached memory."""
    nbytes = math.prod(shape) * torch.empty((), dtype=dtype).element_size()
    with torch.cuda.device(device):
        ptr = native().alloc_uncached(max(16, nbytes))
        owner = _Owner(ptr, max(16, nbytes))
        raw = torch.as_tensor(owner, device=device)
    if raw.data_ptr() != ptr:
        owner.free()
        raise RuntimeError("uncached buffer was copied instead of wrapped")
    return raw[:nbytes].view(dtype).view(*shape)


def live_buffers() -> int:
    """Uncached allocations not yet freed (tests)."""
    return sum(1 for o in list(_LIVE) if o.ptr)


@atexit.register
def _free_all() -> None:
    owners = [o for o in list(_LIVE) if o.ptr]
    if not owners:
        return
    try:
        torch.cuda.synchronize()
    except Exception:  # noqa: BLE001 -- exiting anyway
        pass
    for o in owners:
        o.free()
