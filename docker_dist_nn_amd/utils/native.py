"""Loader for the in-tree native extension (``docker_dist_nn_amd._native``).

``torch`` is imported first on purpose: torch ships its own ``libamdhip64.so.7`` and our
extension links against the same SONAME, so loading torch first makes both share ONE HIP
runtime (a second runtime in the process would own separate device contexts).

On a machine with a GPU the extension is mandatory: :func:`native` raises instead of silently
falling back, so a GPU test can never pass on an eager/PyTorch path by accident.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys
import threading

import torch  # noqa: F401  (must precede the extension import, see module doc)
from .. import switches

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def _try_import():
    global _mod, _err
    with _lock:
        if _mod is not None or _err is not None:
            return
        alt = switches.get("DNN_NATIVE_PATH")
        if alt:  # A/B of another build: same module name, different file
            spec = importlib.util.spec_from_file_location("docker_dist_nn_amd._native", alt)
            _mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_mod)
            sys.modules["docker_dist_nn_amd._native"] = _mod
            return
        try:
            _mod = importlib.import_module("docker_dist_nn_amd._native")
        except ImportError as e:  # not built yet
            if switches.get("DNN_AUTOBUILD") == "1":
                try:
                    from .._build import build

                    build()
                    _mod = importlib.import_module("docker_dist_nn_amd._native")
                    return
                except Exception as be:  # pragma: no cover - build env specific
                    _err = RuntimeError(f"native extension missing and build failed: {be}")
                    return
            _err = e


class _SyncDebug:
    """``DNN_SYNC_DEBUG=1``: every native call is followed by a device synchronize, so an
    asynchronous kernel fault is reported at the op that launched it (with its name) instead of
    at some later, unrelated sync. Debug only -- it serialises host and device. Calls made while
    a HIP graph is being captured are not synchronised (sync is illegal during capture)."""

    _NO_SYNC = {"GraphExec", "device_sync"}

    def __init__(self, mod):
        self._mod = mod

    def __getattr__(self, name):
        f = getattr(self._mod, name)
        if name in self._NO_SYNC or not callable(f):
            return f

        def call(*a, **k):
            out = f(*a, **k)
            if not torch.cuda.is_current_stream_capturing():
                try:
                    self._mod.device_sync()
                except RuntimeError as e:
                    raise RuntimeError(f"DNN_SYNC_DEBUG: device error after native.{name}: {e}") \
                        from e
            return out

        return call


_debug = None


def native():
    """Return the native module or raise a loud error explaining why it is unavailable."""
    global _debug
    _try_import()
    if _mod is None:
        raise RuntimeError(
            "docker_dist_nn_amd native extension is not available "
            f"({_err}); build it with `python -m docker_dist_nn_amd._build`")
    if switches.get("DNN_SYNC_DEBUG") == "1":
        if _debug is None:
            _debug = _SyncDebug(_mod)
        return _debug
    return _mod


def native_available() -> bool:
    _try_import()
    return _mod is not None


def native_path() -> str | None:
    _try_import()
    return getattr(_mod, "__file__", None)
