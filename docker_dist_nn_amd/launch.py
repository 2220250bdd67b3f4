"""Rank launcher: one OS process per GPU (or per CPU rank for gloo runs).

Replaces the reference's Docker orchestration (/root/reference/src/run_grpc_fcnn.py:34-172):
containers on a bridge network become local processes joined by torch.distributed (RCCL over
xGMI for GPUs, gloo on CPU), rendezvous on 127.0.0.1. Fixed reference defects:

* spawn errors are fatal instead of silently skipping a stage (run_grpc_fcnn.py:121-124,149-153);
* the readiness probe's result is checked and every rank must report ready, not only stage 0
  (:157-172, :319);
* any rank that dies tears the whole job down (fail-fast monitor) and is reported with its exit
  code; SIGINT/SIGTERM remove every child process group (the reference removed containers in a
  ``finally``, :329-344).
"""
from __future__ import annotations

import logging
import os
import signal
import socket
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Optional, Sequence

log = logging.getLogger(__name__)

READINESS_CHECK_TIMEOUT = 10.0   # run_grpc_fcnn.py:26
READINESS_CHECK_INTERVAL = 0.5   # run_grpc_fcnn.py:27


def free_port(host: str = "127.0.0.1") -> int:
    s = socket.socket()
    s.bind((host, 0))
    p = s.getsockname()[1]
    s.close()
    return p


def wait_for_port(port: int, timeout: float = READINESS_CHECK_TIMEOUT,
                  interval: float = READINESS_CHECK_INTERVAL, host: str = "127.0.0.1",
                  alive=None) -> bool:
    """TCP readiness probe (same cadence as the reference). ``alive()`` may abort early."""
    t0 = time.monotonic()
    while time.monotonic() - t0 < timeout:
        if alive is not None and not alive():
            return False
        try:
            with socket.create_connection((host, port), timeout=interval):
                return True
        except OSError:
            time.sleep(interval)
    return False


class RankFailure(RuntimeError):
    def __init__(self, rank: int, code: int, name: str = ""):
        super().__init__(f"rank {rank}{' (' + name + ')' if name else ''} exited with code {code}")
        self.rank, self.code, self.name = rank, code, name


@dataclass
class Job:
    procs: list = field(default_factory=list)
    names: list = field(default_factory=list)
    master_port: int = 0

    def poll(self) -> None:
        """Raise RankFailure if any rank has died with a non-zero code."""
        for r, p in enumerate(self.procs):
            rc = p.poll()
            if rc not in (None, 0):
                raise RankFailure(r, rc, self.names[r] if r < len(self.names) else "")

    def alive(self) -> bool:
        return all(p.poll() is None for p in self.procs)

    def wait(self, timeout: Optional[float] = None) -> list[int]:
        t0 = time.monotonic()
        while True:
            self.poll()
            if all(p.poll() is not None for p in self.procs):
                return [p.returncode for p in self.procs]
            if timeout is not None and time.monotonic() - t0 > timeout:
                raise TimeoutError("ranks did not finish in time")
            time.sleep(0.05)

    def terminate(self, grace: float = 5.0) -> None:
        for p in self.procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except (ProcessLookupError, PermissionError):
                    pass
        t0 = time.monotonic()
        for p in self.procs:
            try:
                p.wait(max(0.0, grace - (time.monotonic() - t0)))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
                p.wait()


def spawn_ranks(module: str, args: Sequence[str], nprocs: int,
                devices: Optional[Sequence[int]] = None, env: Optional[dict] = None,
                names: Optional[Sequence[str]] = None, log_dir: Optional[str] = None) -> Job:
    """Start ``python -m module args`` once per rank with the torchrun env contract."""
    port = free_port()
    job = Job(master_port=port, names=list(names or [f"rank{r}" for r in range(nprocs)]))
    base = dict(os.environ)
    base.update(env or {})
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # in-tree package
    base["PYTHONPATH"] = root + (os.pathsep + base["PYTHONPATH"] if base.get("PYTHONPATH") else "")
    try:
        for r in range(nprocs):
            e = dict(base)
            e.update(RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_RANK=str(r),
                     LOCAL_WORLD_SIZE=str(nprocs), MASTER_ADDR="127.0.0.1",
                     MASTER_PORT=str(port), DNN_STAGE_NAME=job.names[r])
            if devices is not None:
                e["LOCAL_RANK"] = str(devices[r])
            out = None
            if log_dir:
                os.makedirs(log_dir, exist_ok=True)
                out = open(os.path.join(log_dir, f"{job.names[r]}.log"), "w")
            p = subprocess.Popen([sys.executable, "-m", module, *args], env=e,
                                 start_new_session=True, stdout=out, stderr=subprocess.STDOUT
                                 if out else None)
            job.procs.append(p)
    except Exception:
        job.terminate()
        raise
    return job


def spawn_workers(module: str, envs: Sequence[dict], names: Optional[Sequence[str]] = None,
                  log_dir: Optional[str] = None, pid_dir: Optional[str] = None) -> Job:
    """Start ``python -m module`` once per stage with that stage's own env contract (the
    reference's per-container environment, run_grpc_fcnn.py:101-126); no rendezvous.
    ``pid_dir``: write ``<name>.pid`` per stage (the container-id analogue)."""
    job = Job(names=list(names or [e.get("CONTAINER_NAME", f"stage{i}")
                                   for i, e in enumerate(envs)]))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    try:
        for i, extra in enumerate(envs):
            e = dict(os.environ)
            e.update(extra)
            e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            e["PYTHONPATH"] = root + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
            out = None
            if log_dir:
                os.makedirs(log_dir, exist_ok=True)
                out = open(os.path.join(log_dir, f"{job.names[i]}.log"), "w")
            job.procs.append(subprocess.Popen([sys.executable, "-m", module], env=e,
                                              start_new_session=True, stdout=out,
                                              stderr=subprocess.STDOUT if out else None))
            if pid_dir:
                with open(os.path.join(pid_dir, f"{job.names[i]}.pid"), "w") as f:
                    f.write(str(job.procs[-1].pid))
    except Exception:
        job.terminate()
        raise
    return job


def install_signal_teardown(job: Job) -> None:
    def handler(signum, frame):
        log.info("Shutdown signal received; tearing down ranks...")
        job.terminate()
        raise KeyboardInterrupt
    signal.signal(signal.SIGTERM, handler)
