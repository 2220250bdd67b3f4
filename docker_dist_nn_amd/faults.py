"""Failure detection and fault injection.

The reference's only failure handling is passive: a 10 s per-hop RPC deadline and error-code
propagation (/root/reference/src/grpc_node.py:133-140), plus a readiness probe whose result is
ignored (/root/reference/src/run_grpc_fcnn.py:319). Here:

* :class:`Watchdog` -- a per-rank thread; the training/serving loop calls ``beat()`` every
  step. If no beat arrives within ``timeout`` seconds (a hung collective, a wedged kernel, a
  peer that died mid-send) it logs which phase stalled, dumps every thread's stack and exits
  the process with ``EXIT_WATCHDOG`` so the launcher's fail-fast monitor tears the job down.
  (RCCL's own async error handling + the process-group timeout cover the comm side as well.)
* :class:`FaultInjector` -- ``DNN_FAULT="stage:1,step:3,kind:crash|hang|nan|raise"`` makes the
  matching rank fail at that step, for tests of the detection paths.
* :func:`check_finite` -- NaN/Inf guard on the loss.
"""
from __future__ import annotations

import faulthandler
import logging
import os
import sys
import threading
import time
from dataclasses import dataclass
from typing import Optional
from . import switches

log = logging.getLogger(__name__)

EXIT_WATCHDOG = 86
EXIT_INJECTED = 87


class Watchdog:
    def __init__(self, timeout: float, name: str = "rank", exit_on_fire: bool = True,
                 on_fire=None):
        self.timeout = float(timeout)
        self.name = name
        self.exit_on_fire = exit_on_fire
        self.on_fire = on_fire
        self.phase = "init"
        self.fired = False
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name=f"watchdog-{name}", daemon=True)

    def start(self) -> "Watchdog":
        self._last = time.monotonic()
        self._t.start()
        return self

    def beat(self, phase: str = "") -> None:
        self._last = time.monotonic()
        if phase:
            self.phase = phase

    def stop(self) -> None:
        self._stop.set()

    def _run(self) -> None:
        while not self._stop.wait(min(1.0, self.timeout / 4)):
            idle = time.monotonic() - self._last
            if idle > self.timeout:
                self.fired = True
                log.error(f"[watchdog:{self.name}] no progress for {idle:.1f}s in phase "
                          f"'{self.phase}' (timeout {self.timeout}s)")
                try:
                    faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                except Exception:  # noqa: BLE001
                    pass
                if self.on_fire is not None:
                    self.on_fire(self)
                if self.exit_on_fire:
                    os._exit(EXIT_WATCHDOG)
                return


@dataclass
class FaultSpec:
    stage: int
    step: int
    kind: str


def parse_fault(text: Optional[str]) -> Optional[FaultSpec]:
    if not text:
        return None
    kv = dict(item.split(":", 1) for item in text.split(","))
    kind = kv.get("kind", "crash")
    if kind not in ("crash", "hang", "nan", "raise"):
        raise ValueError(f"unknown fault kind {kind!r}")
    return FaultSpec(int(kv.get("stage", 0)), int(kv.get("step", 0)), kind)


class FaultInjector:
    def __init__(self, spec: Optional[FaultSpec] = None):
        self.spec = spec if spec is not None else parse_fault(switches.get("DNN_FAULT"))

    def maybe_inject(self, stage_index: int, step: int, stage=None) -> None:
        s = self.spec
        if s is None or s.stage != stage_index or s.step != step:
            return
        log.error(f"injecting fault '{s.kind}' at stage {stage_index}, step {step}")
        if s.kind == "crash":
            os._exit(EXIT_INJECTED)
        if s.kind == "hang":
            while True:
                time.sleep(3600)
        if s.kind == "raise":
            raise RuntimeError(f"injected fault at stage {stage_index} step {step}")
        if s.kind == "nan" and stage is not None:
            stage.params.master[0] = float("nan")
            stage.params.refresh_shadow()


def check_finite(value: Optional[float], what: str = "loss") -> None:
    if value is not None and not (value == value and abs(value) != float("inf")):
        raise FloatingPointError(f"non-finite {what}: {value}")
