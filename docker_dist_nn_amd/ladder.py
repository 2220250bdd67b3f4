"""Fail-safe multi-rank runs: a ladder of transports / plan forms, each attempt in fresh child
processes, so that a job produces a result whatever its first choice does.

The reference has no such thing -- a stage that hangs or dies takes its request down, and the
launcher only logs it (/root/reference/src/run_grpc_fcnn.py:83-155, grpc_node.py:120-140).
Here the first real run of a cross-GPU plan is also the first execution of several mechanisms
(relayed xGMI peer writes, per-link RCCL communicators, co-resident RCCL kernels) that a one-GPU
pool cannot time. A hang or crash in any of them must cost one attempt, not the job.

How it works (``Supervisor``), one supervisor per rank, started by ``torch.distributed.run``:

* the supervisor NEVER touches the GPU (no HIP call: it only imports torch for the c10d
  ``TCPStore``) and never execs; each attempt is a fresh child process per rank
  (``subprocess.Popen``, own session), on a fresh rendezvous port chosen by rank 0 and shared
  through the store;
* each supervisor watches its child: exit code, and a heartbeat file the child touches at every
  phase / step (``DNN_LADDER_HEARTBEAT``); a child silent for ``stall`` seconds is killed;
* every rank's outcome is published under ``attempt/<i>/rc/<rank>``. When ANY rank's child
  fails, every other supervisor kills its own child (whose peers are gone, so it would only
  hang) and publishes "killed". An attempt succeeded iff every rank's child exited 0 -- every
  supervisor reads the same keys, so all agree without another collective;
* on failure all supervisors move to the next rung together; on success rank 0's child has
  written its result (``DNN_LADDER_RESULT``) and rank 0 reports it with the list of attempts.

Rungs of the training benchmark (``bench_rungs``), most capable first:

  1. ``default``       -- the configured transport (DNN_PIPE=auto: relayed IPC, its first step
                          verified against the RCCL ``slotted`` plan);
  2. ``ipc-slotted``   -- relayed IPC on ONE stream per rank in global clock order (no
                          assumption about how streams or kernels are co-scheduled);
  3. ``rccl-slotted``  -- RCCL, one grouped send/recv per logical clock slot (safe with ONE
                          resident RCCL kernel per rank);
  4. ``rccl-streams``  -- RCCL, one stream + communicator per link channel;
  5. ``python``        -- the Python executor over torch.distributed P2P;
  6. ``dp-native`` / ``dp-python`` -- data parallelism only (no pipeline hops at all).

When the default layout is a replicated-stage pipeline (parallel/fan.py) the rungs are
``default`` (its native slotted RCCL step) -> ``fan-python`` -> ``uniform-rccl-slotted`` /
``uniform-python`` (the literal ppS x dpD grid) -> ``dp-native`` / ``dp-python``.
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Callable, Optional, Sequence

HEARTBEAT_ENV = "DNN_LADDER_HEARTBEAT"
RESULT_ENV = "DNN_LADDER_RESULT"
RUNG_ENV = "DNN_LADDER_RUNG"
CHILD_ENV = "DNN_LADDER_CHILD"


@dataclass
class Rung:
    name: str
    env: dict = field(default_factory=dict)     # overrides for the child's environment
    args: list = field(default_factory=list)    # extra command-line arguments (appended)


def uniform_rungs() -> list[Rung]:
    """The literal uniform ppS x dpD grid (bench ``--parallelism uniform``), measured after a
    fan layout's number: its default transport, then the RCCL slotted plan, then the Python
    executor -- eager, like every fallback rung."""
    uni = ["--parallelism", "uniform", "--graph", "off"]
    return [Rung("uniform", {}, uni),
            Rung("uniform-rccl-slotted", {"DNN_PIPE": "rccl", "DNN_RCCL_PLAN": "slotted"}, uni),
            Rung("uniform-python", {"DNN_PIPE": "rccl", "DNN_NATIVE_DIST": "0"}, uni)]


def bench_rungs(n: int, dp_only: bool = False, fan: bool = False) -> list[Rung]:
    """The training benchmark's ladder for ``n`` ranks. ``dp_only``: the layout is already
    data-parallel (no hops), only the executor can fall back. ``fan``: the default layout is
    a replicated-stage pipeline (parallel/fan.py: IPC plan verified against the RCCL slotted
    plan): the RCCL plan alone, its Python executor, then the uniform ppS x dpD grid with its
    own rungs, then data parallelism."""
    # every rung after the first replays eagerly: a failed first attempt may have been the
    # graph replay itself (bench --graph auto)
    eager = ["--graph", "off"]
    dp = [Rung("dp-native", {}, ["--parallelism", f"dp{n}", *eager]),
          Rung("dp-python", {"DNN_NATIVE_DIST": "0"}, ["--parallelism", f"dp{n}", *eager])]
    if dp_only:
        return dp
    if fan:
        uni = ["--parallelism", "uniform", *eager]
        return [Rung("default"),
                Rung("fan-rccl", {"DNN_PIPE": "rccl"}, eager),
                Rung("fan-python", {"DNN_NATIVE_DIST": "0"}, eager),
                Rung("uniform-rccl-slotted", {"DNN_PIPE": "rccl", "DNN_RCCL_PLAN": "slotted"},
                     uni),
                Rung("uniform-python", {"DNN_PIPE": "rccl", "DNN_NATIVE_DIST": "0"}, uni),
                *dp]
    return [Rung("default"),
            Rung("ipc-slotted", {"DNN_IPC_PLAN": "slotted"}, eager),
            Rung("rccl-slotted", {"DNN_PIPE": "rccl", "DNN_RCCL_PLAN": "slotted"}, eager),
            Rung("rccl-streams", {"DNN_PIPE": "rccl", "DNN_RCCL_PLAN": "streams"}, eager),
            Rung("python", {"DNN_PIPE": "rccl", "DNN_NATIVE_DIST": "0"}, eager),
            *dp]


# ---- child side ---------------------------------------------------------------------------
def is_child() -> bool:
    return os.environ.get(CHILD_ENV) == "1"


def heartbeat(phase: str = "") -> None:
    """Tell the supervisor this child is making progress (no-op outside a ladder)."""
    path = os.environ.get(HEARTBEAT_ENV)
    if path:
        try:
            with open(path, "w") as f:
                f.write(f"{time.time():.3f} {phase}\n")
        except OSError:
            pass


class Throttled:
    """Per-step heartbeat that writes at most every ``interval`` seconds (a step loop calls it
    every step; the cost is one clock read)."""

    def __init__(self, interval: float = 5.0):
        self.interval = interval
        self.last = 0.0
        self.on = bool(os.environ.get(HEARTBEAT_ENV))

    def __call__(self, phase: str = "") -> None:
        if self.on:
            t = time.monotonic()
            if t - self.last >= self.interval:
                self.last = t
                heartbeat(phase)


def write_result(obj: dict) -> bool:
    """Child rank 0: hand the result to the supervisor. False outside a ladder."""
    path = os.environ.get(RESULT_ENV)
    if not path:
        return False
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f)
    os.replace(tmp, path)
    return True


def rung_fault(rung: str, spec: str) -> str:
    """``DNN_LADDER_FAULT`` = 'rung=fault;rung=fault' (fault in DNN_FAULT syntax): the fault
    the child of ``rung`` injects (tests of the ladder itself); rung '*' = every rung not named
    on its own."""
    wild = ""
    for item in filter(None, (s.strip() for s in spec.split(";"))):
        name, _, fault = item.partition("=")
        if name.strip() == rung:
            return fault.strip()
        if name.strip() == "*":
            wild = fault.strip()
    return wild


# ---- supervisor side ----------------------------------------------------------------------
def _store(rank: int, world: int):
    """The job's c10d store (CPU only). Under torch.distributed.run the elastic agent hosts it
    on MASTER_PORT; otherwise rank 0 hosts it."""
    from datetime import timedelta

    import torch.distributed as dist

    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ["MASTER_PORT"])
    agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() in ("1", "true")
    master = rank == 0 and not agent
    st = dist.TCPStore(host, port, world if master else None, master,
                       timeout=timedelta(seconds=600), wait_for_workers=False)
    run = os.environ.get("TORCHELASTIC_RUN_ID", "")
    return dist.PrefixStore(f"dnn_ladder/{run}/", st)


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _kill(p: subprocess.Popen) -> None:
    try:
        os.killpg(p.pid, signal.SIGKILL)
    except (ProcessLookupError, PermissionError):
        pass
    try:
        p.wait(30)
    except subprocess.TimeoutExpired:
        pass


class Supervisor:
    """Runs a ladder of attempts on every rank (see the module docstring).

    ``command(rung)`` -> the child's argv. ``stall``: seconds without a heartbeat (or an exit)
    before a child is killed; ``store``: a c10d store shared by the ranks (default: the job's)."""

    def __init__(self, command: Callable[[Rung], Sequence[str]], *, rank: int, world: int,
                 stall: float = 60.0, store=None, workdir: Optional[str] = None,
                 log=None, deadline: Optional[float] = None, startup: float = 120.0):
        self.command = command
        self.rank, self.world = rank, world
        self.stall = float(stall)
        # a child's first heartbeat comes after `import torch` (up to minutes on a cold box):
        # until then it gets max(stall, startup) seconds
        self.startup = max(float(startup), self.stall)
        # time.monotonic() after which no attempt may run on: a running child is killed
        # ("deadline") and climb() tries no further rung -- so a ladder ends inside the
        # driver's own window
        self.deadline = deadline
        self.store = store if store is not None else _store(rank, world)
        self.workdir = workdir or os.path.join(
            os.environ.get("TMPDIR", "/tmp"),
            f"dnn_ladder_{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}")
        os.makedirs(self.workdir, exist_ok=True)
        self.log = log or (lambda msg: print(f"[ladder r{rank}] {msg}", file=sys.stderr,
                                              flush=True))
        self.attempts: list[dict] = []
        self._n = 0  # attempts made (store keys are per attempt index)
        self._child: Optional[subprocess.Popen] = None
        # the launcher ends a job with SIGTERM (torch.distributed.run does when any rank
        # fails): take the current child down with us -- it runs in a session of its own and
        # would otherwise live on, blocked in a rendezvous whose peers are gone
        try:
            prev = signal.getsignal(signal.SIGTERM)

            def _term(signum, frame):
                if self._child is not None and self._child.poll() is None:
                    _kill(self._child)
                if callable(prev):
                    prev(signum, frame)
                raise SystemExit(128 + signum)

            signal.signal(signal.SIGTERM, _term)
        except ValueError:  # not the main thread: the caller handles termination
            pass

    def _key(self, i: int, what: str) -> str:
        return f"attempt/{i}/{what}"

    def _peer_rcs(self, i: int) -> dict:
        out = {}
        for r in range(self.world):
            k = self._key(i, f"rc/{r}")
            if self.store.check([k]):
                out[r] = self.store.get(k).decode()
        return out

    def attempt(self, rung: Rung) -> tuple[bool, Optional[dict]]:
        """One attempt of ``rung`` on every rank; returns (success, rank 0's child's result),
        the same on every rank."""
        i = self._n
        self._n += 1
        if self.rank == 0:
            self.store.set(self._key(i, "port"), str(_free_port()))
        port = self.store.get(self._key(i, "port")).decode()
        hb = os.path.join(self.workdir, f"hb_{i}_{self.rank}")
        res = os.path.join(self.workdir, f"result_{i}.json")
        for path in (hb, res):
            if os.path.exists(path) and (path == hb or self.rank == 0):
                os.remove(path)
        env = dict(os.environ)
        env.update({k: str(v) for k, v in rung.env.items()})
        env.update({"MASTER_PORT": port, "TORCHELASTIC_USE_AGENT_STORE": "False",
                    CHILD_ENV: "1", RUNG_ENV: rung.name, HEARTBEAT_ENV: hb})
        if self.rank == 0:
            env[RESULT_ENV] = res
        else:
            env.pop(RESULT_ENV, None)
        fault = rung_fault(rung.name, os.environ.get("DNN_LADDER_FAULT", ""))
        if fault:
            env["DNN_FAULT"] = fault
        cmd = list(self.command(rung))
        heartbeat_t = time.monotonic()
        started = False  # the child has written a heartbeat of its own
        with open(hb, "w") as f:
            f.write("spawn\n")
        spawn_mt = os.path.getmtime(hb)
        t0 = time.monotonic()
        # the child's stdout goes to stderr: the supervisor's stdout carries only its result
        p = subprocess.Popen(cmd, env=env, start_new_session=True, stdout=sys.stderr.fileno())
        self._child = p
        mine = None      # this rank's outcome: exit code or "stall" / "killed"
        tail = ""
        while True:
            rc = p.poll()
            if mine is None and rc is not None:
                mine = str(rc)
                self.store.set(self._key(i, f"rc/{self.rank}"), mine)
            rcs = self._peer_rcs(i)
            if mine is None:
                failed = [r for r, v in rcs.items() if v != "0" and r != self.rank]
                try:
                    mt = os.path.getmtime(hb)
                    if mt != spawn_mt:
                        started = True
                        heartbeat_t = max(heartbeat_t, time.monotonic() - (time.time() - mt))
                except OSError:
                    pass
                now = time.monotonic()
                stalled = now - heartbeat_t > (self.stall if started else self.startup)
                late = self.deadline is not None and now > self.deadline
                if failed or stalled or late:
                    _kill(p)
                    mine = ("killed" if failed else "deadline" if late and not stalled
                            else "stall")
                    try:
                        with open(hb) as f:
                            tail = f.read().strip()[-200:]
                    except OSError:
                        pass
                    self.store.set(self._key(i, f"rc/{self.rank}"), mine)
                    rcs[self.rank] = mine
            if mine is not None and len(rcs) == self.world:
                break
            time.sleep(0.2)
        ok = all(v == "0" for v in rcs.values())
        result = None
        if ok and self.rank == 0:
            try:
                with open(res) as f:
                    result = json.load(f)
            except (OSError, ValueError) as e:
                ok = False
                rcs[0] = f"no result ({e.__class__.__name__})"
        if self.rank == 0:  # rank 0's view decides whether its result is usable: share it,
            # with the result itself (every supervisor decides the next step from it)
            if ok:
                self.store.set(self._key(i, "result"), json.dumps(result))
            self.store.set(self._key(i, "ok"), "1" if ok else "0")
        ok = self.store.get(self._key(i, "ok")).decode() == "1"
        if ok and self.rank != 0:
            result = json.loads(self.store.get(self._key(i, "result")).decode())
        # every rank has read the outcome before rank 0 (which may host the store) moves on or
        # exits
        self.store.add(self._key(i, "read"), 1)
        if self.rank == 0:
            while self.store.add(self._key(i, "read"), 0) < self.world:
                time.sleep(0.05)
        rec ={"rung": rung.name, "ok": ok, "seconds": round(time.monotonic() - t0, 1),
               "rc": {str(r): rcs[r] for r in sorted(rcs)}}
        if tail and not ok:
            rec["last_heartbeat"] = tail
        self.attempts.append(rec)
        self.log(f"attempt {i} rung {rung.name}: {'ok' if ok else 'FAILED'} {rec['rc']}")
        return ok, result

    def climb(self, rungs: Sequence[Rung],
              budget_s: Optional[float] = None) -> tuple[Optional[dict], Optional[Rung]]:
        """Try ``rungs`` in order until one succeeds; (its result or None, the rung) -- the
        same on every rank."""
        t0 = time.monotonic()
        for k, rung in enumerate(rungs):
            # past the time budget only the last (most conservative) rung is still tried, past
            # the deadline none; every rank measures the same attempts' outcomes but its own
            # clock, so the skip decision is rank 0's, shared through the store
            if (budget_s is not None and k < len(rungs) - 1) or self.deadline is not None:
                key = self._key(self._n, f"skip{k}")
                if self.rank == 0:
                    now = time.monotonic()
                    # a peer whose (own-clock) deadline ended the last attempt ends the ladder
                    # too, even when rank 0's clock has a moment left
                    peer_late = bool(self.attempts) and \
                        "deadline" in self.attempts[-1].get("rc", {}).values()
                    why = ("deadline" if self.deadline is not None and
                           (now > self.deadline or peer_late) else
                           "budget" if budget_s is not None and k < len(rungs) - 1 and
                           now - t0 > budget_s else "")
                    self.store.set(key, why)
                why = self.store.get(key).decode()
                if why:
                    self.log(f"time {why} spent: skipping rung {rung.name}")
                    self.attempts.append({"rung": rung.name, "ok": False, "skipped": why})
                    continue
            ok, result = self.attempt(rung)
            if ok:
                return result, rung
        return None, None

    def seconds_left(self) -> Optional[float]:
        return None if self.deadline is None else self.deadline - time.monotonic()

    def comparisons(self, items: Sequence[tuple[str, Sequence[Rung]]], need_s: float,
                    on_done: Optional[Callable[[str, dict], None]] = None) -> dict:
        """Further measurements after the main one (bench.py: the literal uniform pipeline,
        then data parallelism), each climbing its own rungs -- but only while the deadline
        leaves room for another attempt of ``need_s`` seconds. Rank 0 decides per item and
        every rank reads the decision from the store, so all climb (or skip) together.
        Returns key -> {"result": rank 0's child result or None, "attempts": [...]} or
        {"skipped": "budget", "seconds_left", "seconds_needed"}; ``on_done(key, entry)`` sees
        each entry as soon as it exists (the SIGTERM report uses what is known by then)."""
        out: dict = {}
        for key, rungs in items:
            dk = f"compare/{key}/decision"
            if self.rank == 0:
                left = self.seconds_left()
                self.store.set(dk, "run" if left is None or left > need_s else "skip")
            if self.store.get(dk).decode() == "run":
                n0 = len(self.attempts)
                res, _ = self.climb(rungs)
                out[key] = {"result": res, "attempts": self.attempts[n0:]}
            else:
                out[key] = {"skipped": "budget",
                            "seconds_left": round(self.seconds_left() or 0.0, 1),
                            "seconds_needed": round(need_s, 1)}
            if on_done is not None:
                on_done(key, out[key])
        return out


class OneLine:
    """Rank 0's single JSON line, printed exactly once: when the run completes, or from the
    supervisor's SIGTERM handler with whatever is known by then (the driver ends a bench that
    overruns its window with SIGTERM; a bench killed there must still report its attempts).
    ``build(reason)`` returns the object to print (reason None = normal completion)."""

    def __init__(self, rank: int, build: Callable[[Optional[str]], dict]):
        self.rank, self.build, self.done = rank, build, False

    def emit(self, reason: Optional[str] = None) -> None:
        if self.done or self.rank != 0:
            self.done = True
            return
        self.done = True
        try:
            obj = self.build(reason)
        except Exception as e:  # never lose the line over a formatting problem
            obj = {"value": None, "error": f"report failed: {e!r}", "terminated": reason}
        sys.stdout.write(json.dumps(obj) + "\n")
        sys.stdout.flush()

    def install_sigterm(self) -> None:
        """Print the line on SIGTERM, then exit 128 + 15. Install BEFORE the Supervisor (its
        own handler kills the running child, then chains to this one)."""
        def _term(signum, frame):
            self.emit("terminated")
            raise SystemExit(128 + signum)

        try:
            signal.signal(signal.SIGTERM, _term)
        except ValueError:  # not the main thread
            pass
