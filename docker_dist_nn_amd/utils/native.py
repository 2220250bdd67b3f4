"""Loader for the in-tree native extension (``docker_dist_nn_amd._native``).

``torch`` is imported first on purpose: torch ships its own ``libamdhip64.so.7`` and our
extension links against the same SONAME, so loading torch first makes both share ONE HIP
runtime (a second runtime in the process would own separate device contexts).

On a machine with a GPU the extension is mandatory: :func:`native` raises instead of silently
falling back, so a GPU test can never pass on an eager/PyTorch path by accident.
"""
from __future__ import annotations

import importlib
import os
import threading

import torch  # noqa: F401  (must precede the extension import, see module doc)

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def _try_import():
    global _mod, _err
    with _lock:
        if _mod is not None or _err is not None:
            return
        try:
            _mod = importlib.import_module("docker_dist_nn_amd._native")
        except ImportError as e:  # not built yet
            if os.environ.get("DNN_AUTOBUILD", "1") == "1":
                try:
                    from .._build import build

                    build()
                    _mod = importlib.import_module("docker_dist_nn_amd._native")
                    return
                except Exception as be:  # pragma: no cover - build env specific
                    _err = RuntimeError(f"native extension missing and build failed: {be}")
                    return
            _err = e


def native():
    """Return the native module or raise a loud error explaining why it is unavailable."""
    _try_import()
    if _mod is None:
        raise RuntimeError(
            "docker_dist_nn_amd native extension is not available "
            f"({_err}); build it with `python -m docker_dist_nn_amd._build`")
    return _mod


def native_available() -> bool:
    _try_import()
    return _mod is not None


def native_path() -> str | None:
    _try_import()
    return getattr(_mod, "__file__", None)
