"""Per-op device timing for pipeline steps, Chrome-trace export and bubble accounting.

The reference only had wall-clock log lines (/root/reference/src/run_grpc_fcnn.py:321-322,
/root/reference/src/run_grpc_inference.py:139-142). :class:`StepProfiler` hooks the pipeline
executor: every schedule op (F/B/W/O of each stage) is bracketed by HIP events on the compute
stream, so after the step the device time of each op, each stage's busy time, and the pipeline
bubble (1 - busy/makespan) are known. ``chrome_trace()`` writes a chrome://tracing /
Perfetto-compatible JSON per rank. For kernel-level detail use
``rocprofv3 --kernel-trace --stats`` (see README "Profiling").
"""
from __future__ import annotations

import json
import os
from typing import Optional

import torch


class _WallEvent:
    """CPU stand-in for a timing event (host wall clock, ms)."""

    def __init__(self):
        import time

        self.t = time.perf_counter()

    def elapsed_time(self, other: "_WallEvent") -> float:
        return (other.t - self.t) * 1e3


class StepProfiler:
    def __init__(self, executor, rank: int = 0, enabled: bool = True):
        self.executor = executor
        self.rank = rank
        self.enabled = enabled
        self.records: list[tuple] = []  # (stage, op, micro, start_event, end_event)
        self._open: dict = {}
        self.steps: list[list[dict]] = []
        if enabled:
            executor.hooks["before_op"].append(self._before)
            executor.hooks["after_op"].append(self._after)

    def _ev(self, stage):
        if stage.device.type != "cuda":
            return _WallEvent()
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream(stage.device))
        return e

    def _before(self, stage, op, j):
        self._open[(stage.stage_index, op, j)] = self._ev(stage)

    def _after(self, stage, op, j):
        s = self._open.pop((stage.stage_index, op, j), None)
        self.records.append((stage.stage_index, op, j, s, self._ev(stage)))

    def collect(self) -> list[dict]:
        """Resolve the events of the last step (synchronizes)."""
        if not self.records:
            return []
        evs = [r for r in self.records if r[3] is not None]
        if evs:
            if not isinstance(evs[0][3], _WallEvent):
                torch.cuda.synchronize()
            t0 = evs[0][3]
        out = []
        for st, op, j, s, e in self.records:
            if s is None:
                out.append({"stage": st, "op": op, "micro": j, "start_ms": 0.0, "dur_ms": 0.0})
            else:
                out.append({"stage": st, "op": op, "micro": j,
                            "start_ms": t0.elapsed_time(s), "dur_ms": s.elapsed_time(e)})
        self.records.clear()
        self.steps.append(out)
        return out

    @staticmethod
    def summarize(ops: list[dict]) -> dict:
        if not ops:
            return {}
        end = max(o["start_ms"] + o["dur_ms"] for o in ops)
        start = min(o["start_ms"] for o in ops)
        span = max(end - start, 1e-9)
        busy: dict[int, float] = {}
        by_op: dict[str, float] = {}
        for o in ops:
            busy[o["stage"]] = busy.get(o["stage"], 0.0) + o["dur_ms"]
            by_op[o["op"]] = by_op.get(o["op"], 0.0) + o["dur_ms"]
        return {"makespan_ms": span, "busy_ms": busy, "op_ms": by_op,
                "bubble": 1.0 - sum(busy.values()) / (len(busy) * span)}

    def chrome_trace(self, path: str, step: int = -1) -> None:
        ops = self.steps[step] if self.steps else []
        names = {"F": "forward", "B": "backward", "W": "wgrad", "O": "optimizer"}
        ev = [{"name": f"{names.get(o['op'], o['op'])} mb{o['micro']}", "ph": "X",
               "pid": self.rank, "tid": o["stage"], "ts": o["start_ms"] * 1e3,
               "dur": o["dur_ms"] * 1e3, "args": {"micro": o["micro"]}} for o in ops]
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
        with open(path, "w") as f:
            json.dump({"traceEvents": ev, "displayTimeUnit": "ms"}, f)
