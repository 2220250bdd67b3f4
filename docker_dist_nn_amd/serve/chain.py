"""Distributed inference chain: one rank (process / GPU) per non-empty stage.

Reference behaviour (/root/reference/src/grpc_node.py:99-158): stage i computes its layers and
forwards to stage i+1 over a fresh gRPC channel with a 10 s deadline per hop (:130-133); the
last stage's result unwinds back through every hop; a downstream failure keeps its gRPC code
and is reported as "Failed to forward request to <next>" (:136-140). Here:

* rank 0 hosts the gRPC ingress (port 5101, a 10-worker pool like grpc_node.py:169) and
  stage 0; a request becomes a small header tensor (request id, rows, width, status, extra)
  plus the padded bf16 activations, sent rank to rank with torch.distributed (RCCL over xGMI
  on GPUs, gloo on CPU) on a FORWARD group;
* several requests are in flight at once: rank 0 only serialises its own stage's compute
  (shared per-bucket buffers); a sender thread feeds the chain, a receiver thread collects
  results that the LAST rank sends straight back to rank 0 on a separate RETURN group (one
  hop, not S; its own communicator, so a pending receive never blocks a send), and hands each
  to the waiting request by id. Stages 1..S-1 process requests in arrival order, so stage k
  works on request n while stage k-1 already computes request n+1;
* every request waits with a deadline (``--hop-timeout`` x hops, capped by the client's own
  gRPC deadline): a hung or dead downstream stage maps to DEADLINE_EXCEEDED "Failed to
  forward request to layer_container_1: ..." within the deadline, the ingress keeps
  answering, and a late result is dropped by request id instead of being delivered to the
  wrong caller;
* a stage that fails turns the header status into an error code carrying its stage index;
  rank 0 raises ``StageFailure`` -> the reference's gRPC code + details;
* blame on a timeout names the stage that actually stopped: every rank > 0 publishes the id of
  the last request it has PROCESSED (received + computed) to the job's key-value store from a
  background thread, and a payload receive that misses its per-hop deadline publishes an error
  record; when a request's deadline expires, rank 0 blames the first stage that has not
  processed it ("Failed to forward request to layer_container_k", as the reference's hop
  before a dead stage reports it, grpc_node.py:136-140);
* small requests (<= ops.GEMV_MAX_ROWS rows, the batch-1 serving path) travel as ONE fixed-size
  packet per hop (header + rows); larger ones as a packet header then the payload;
* ``STOP`` headers shut the chain down in order.

Run by the launcher: ``python -m docker_dist_nn_amd.serve.chain --plan plan.json``.
Fault injection (tests): ``DNN_FAULT_STAGE=<rank>`` with ``DNN_FAULT_KIND=raise`` (default:
the stage reports INTERNAL) or ``hang`` (the stage stops responding after
``DNN_FAULT_AFTER`` requests, default 0).
"""
from __future__ import annotations

import argparse
from contextlib import nullcontext
import itertools
import json
import logging
import os
import queue
import signal
import threading
import time
from concurrent.futures import Future
from concurrent.futures import TimeoutError as FutureTimeout
from typing import Optional

import grpc
import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from ..config import load_model_config
from ..engine.inference import InferenceStage
from ..models.mlp import round_up
from .ingress import StageFailure, serve
from .. import switches

log = logging.getLogger(__name__)

ST_OK, ST_STOP, ST_VALUE, ST_INTERNAL, ST_DEADLINE = 0, 1, 2, 3, 4
_CODES = {ST_VALUE: grpc.StatusCode.INVALID_ARGUMENT, ST_INTERNAL: grpc.StatusCode.INTERNAL,
          ST_DEADLINE: grpc.StatusCode.DEADLINE_EXCEEDED}
HOP_TIMEOUT_S = 10.0  # grpc_node.py:133
HDR_BYTES = 64  # packet header: 5 int64 (request id, rows bucket, width, status, extra) + pad
PUBLISH_S = 0.02  # progress publication period of ranks > 0


def bucket(rows: int) -> int:
    """Row bucket of a request: serving sizes (<= ops.GEMV_MAX_ROWS) travel and run unpadded
    (GEMV path, csrc/kernels/gemv.hip), larger batches pad to a power of two >= 64."""
    if rows <= ops.GEMV_MAX_ROWS:
        return rows
    b = 64
    while b < rows:
        b *= 2
    return b if rows <= 65536 else round_up(rows, 64)


class ChainRank:
    def __init__(self, stage: InferenceStage, rank: int, world: int, names: list[str],
                 device: torch.device, hop_timeout: float = HOP_TIMEOUT_S):
        self.stage, self.rank, self.world, self.names = stage, rank, world, names
        self.device = device
        self.comm_dev = device if dist.get_backend() == "nccl" else torch.device("cpu")
        self.hop_timeout = float(hop_timeout)
        self.out_pad = round_up(stage.out_dim, 64)
        # groups: every rank calls new_group in the same order
        self.fwd_group = dist.new_group(list(range(world))) if world > 1 else None
        self.ret_group = dist.new_group(sorted({0, world - 1})) if world > 1 else None
        self.compute_lock = threading.Lock()
        self._ids = itertools.count(1)
        self._pending: dict[int, Future] = {}
        self._pending_lock = threading.Lock()
        self._sendq: "queue.Queue" = queue.Queue()
        self._threads: list[threading.Thread] = []
        self.fault_stage = switches.get("DNN_FAULT_STAGE")
        self.fault_kind = switches.get("DNN_FAULT_KIND")
        self.fault_after = int(switches.get("DNN_FAULT_AFTER"))
        self.small = ops.GEMV_MAX_ROWS
        self._packets: dict = {}
        self.store = dist.distributed_c10d._get_default_store() if world > 1 else None
        self.fast = None  # serve/fastpath.FastChain once enable_fast() agreed on it
        # every thread of a chain rank does its GPU work on this non-blocking stream, never on
        # the null stream: a persistent device-chain kernel runs on a blocking stream of its
        # own (serve/fastpath.py), and null-stream work would wait for it to return
        self.work_stream = torch.cuda.Stream(device) if device.type == "cuda" else None
        self._processed = 0
        self._published = 0
        if rank > 0 and world > 1:
            t = threading.Thread(target=self._publisher, name="chain-progress", daemon=True)
            t.start()
        if rank == 0 and world > 1:
            for fn, nm in ((self._sender, "chain-send"), (self._receiver, "chain-recv")):
                t = threading.Thread(target=self._on_work_stream, args=(fn,), name=nm,
                                     daemon=True)
                t.start()
                self._threads.append(t)

    def _on_work_stream(self, fn, *args):
        """Run ``fn`` with this thread's current stream set to the work stream (thread-local)."""
        if self.work_stream is not None:
            torch.cuda.set_stream(self.work_stream)
        return fn(*args)

    # -- transport ----------------------------------------------------------------------------
    def _hdr(self, *vals) -> torch.Tensor:
        return torch.tensor(list(vals), dtype=torch.int64, device=self.comm_dev)

    def _send(self, t: torch.Tensor, dst: int, group) -> None:
        dist.send(t if t.device == self.comm_dev else t.to(self.comm_dev), dst, group=group)

    def _recv_into(self, t: torch.Tensor, src: int, group) -> torch.Tensor:
        if t.device == self.comm_dev:
            dist.recv(t, src, group=group)
            return t
        tmp = torch.empty(t.shape, dtype=t.dtype, device=self.comm_dev)
        dist.recv(tmp, src, group=group)
        t.copy_(tmp)
        return t

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()

    def _packet(self, width: int) -> torch.Tensor:
        """Fixed-size hop packet for activations of ``width`` bf16 columns: header bytes, then
        up to ``small`` rows (reused per width; sends and receives of one rank are serial)."""
        p = self._packets.get(width)
        if p is None:
            p = torch.zeros(HDR_BYTES + self.small * width * 2, dtype=torch.uint8,
                            device=self.comm_dev)
            self._packets[width] = p
        return p

    def _send_msg(self, hdr: list, payload: Optional[torch.Tensor], dst: int, group,
                  width: int) -> None:
        """One packet (header + the rows of a small request), then -- for a request of more
        than ``small`` rows -- the payload as a second message."""
        pk = self._packet(width)
        h = torch.tensor(hdr, dtype=torch.int64)
        pk[:40].copy_(h.view(torch.uint8))
        R = hdr[1]
        if payload is not None and hdr[3] == ST_OK and R <= self.small:
            src = payload.reshape(-1).view(torch.uint8)
            pk[HDR_BYTES:HDR_BYTES + src.numel()].copy_(src)
            payload = None
        self._send(pk, dst, group)
        if payload is not None and hdr[3] == ST_OK:
            self._send(payload, dst, group)

    def _recv_hdr(self, src: int, group, width: int) -> tuple[list, torch.Tensor]:
        pk = self._packet(width)
        dist.recv(pk, src, group=group)
        hdr = pk[:40].cpu().view(torch.int64).tolist()
        return hdr, pk

    def _recv_payload(self, dst: torch.Tensor, src: int, group, timeout_s: float) -> bool:
        """Second message of a large request, bounded by the per-hop deadline. It lands in a
        scratch tensor of its own: after a timeout the receive stays posted, and a late payload
        must not overwrite the shared stage buffer while a later request computes on it
        (ADVICE r3). The caller then stops serving this hop (``loop``)."""
        import datetime

        t = torch.empty(dst.shape, dtype=dst.dtype, device=self.comm_dev)
        w = dist.irecv(t, src, group=group)
        try:
            w.wait(timeout=datetime.timedelta(seconds=timeout_s))
        except RuntimeError:
            return False
        dst.copy_(t)
        return True

    def enable_fast(self) -> str:
        """Collective (every rank): build the device-side chain for serving-size requests
        (serve/fastpath.py). Ranks > 0 start serving it on a thread of their own; the message
        chain keeps carrying larger requests and is the fallback if any rank cannot map its
        peers."""
        from .fastpath import FastChain

        fc = FastChain(self)
        if not fc.ok:
            return fc.why
        self.fast = fc
        if self.rank > 0:
            t = threading.Thread(target=fc.loop, name="chain-fast", daemon=True)
            t.start()
            self._fast_thread = t
        return fc.why

    # -- progress / blame ---------------------------------------------------------------------
    def _publisher(self) -> None:
        """Ranks > 0: the id of the last request this stage processed, to the store."""
        key = f"chain/processed/{self.rank}"
        while True:
            n = self._processed
            if n != self._published:
                try:
                    self.store.set(key, str(n))
                    self._published = n
                except Exception:  # noqa: BLE001 -- the store went away at teardown
                    return
            time.sleep(PUBLISH_S)

    def _progress(self, rank: int) -> int:
        key = f"chain/processed/{rank}"
        try:
            if not self.store.check([key]):
                return 0
            return int(self.store.get(key))
        except Exception:  # noqa: BLE001
            return 0

    def blame(self, rid: int) -> int:
        """The stage a timed-out request is stuck at: the first rank > 0 that has not
        processed it (every rank before it has, so the hop INTO it is where the request
        stopped). Waits one publication period so a healthy stage's counter is current."""
        time.sleep(2 * PUBLISH_S)
        for k in range(1, self.world):
            if self._progress(k) < rid:
                return k
        return self.world - 1

    # -- rank 0 -------------------------------------------------------------------------------
    def predict(self, x: np.ndarray, timeout: Optional[float] = None) -> np.ndarray:
        x = np.asarray(x)
        if x.ndim != 2:
            x = x.reshape(x.shape[0], -1)
        rows, cols = x.shape
        self.stage.check_input_dim(cols)  # ValueError -> INVALID_ARGUMENT
        if self.fast is not None and rows <= self.small:
            return self.fast.predict(x, timeout)
        if self.work_stream is not None:  # (an ingress worker thread: see work_stream)
            torch.cuda.set_stream(self.work_stream)
        R = bucket(rows)
        with self.compute_lock:  # this rank's per-bucket buffers are shared
            buf = self.stage.buffers(R)
            xb = buf["x"]
            xb.zero_()
            ops.pack_bf16(torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(self.device),
                          xb[:rows])
            out = self.stage.forward(R)
            if self.world == 1:
                return out[:rows, :self.stage.out_dim].double().cpu().numpy()
            payload = out.clone()  # the next request may overwrite `out` while this one flies
            self._sync()
        rid = next(self._ids)
        fut: Future = Future()
        with self._pending_lock:
            self._pending[rid] = fut
        self._sendq.put((rid, R, rows, payload))
        limit = self.hop_timeout * (self.world - 1)
        if timeout is not None:
            limit = min(limit, max(0.0, timeout))
        try:
            hdr, res = fut.result(timeout=limit)
        except FutureTimeout:
            with self._pending_lock:
                self._pending.pop(rid, None)
            k = self.blame(rid)
            raise StageFailure(self.names[k], grpc.StatusCode.DEADLINE_EXCEEDED,
                               f"Deadline Exceeded (request {rid} not processed by "
                               f"{self.names[k]} within {limit:.1f} s)") from None
        status = hdr[3]
        if status != ST_OK:
            bad = self.names[hdr[4]] if 0 <= hdr[4] < len(self.names) else "stage"
            raise StageFailure(bad, _CODES.get(status, grpc.StatusCode.INTERNAL),
                               f"stage {bad} failed (status {status})")
        return res[:rows].double().numpy()

    def _sender(self) -> None:
        """Feeds the chain in request order (the only thread sending on the forward group)."""
        while True:
            item = self._sendq.get()
            w = self.out_pad
            if item is None:
                self._send_msg([0, 0, 0, ST_STOP, 0], None, 1, self.fwd_group, w)
                return
            rid, R, rows, payload = item
            self._send_msg([rid, R, payload.shape[1], ST_OK, rows], payload, 1, self.fwd_group,
                           w)

    def _receiver(self) -> None:
        """Collects results from the last rank and completes the waiting requests."""
        last = self.world - 1
        while True:
            hdr = self._recv_into(self._hdr(0, 0, 0, 0, 0), last, self.ret_group).tolist()
            rid, R, n_out, status, extra = hdr
            if status == ST_STOP:
                return
            res = None
            if status == ST_OK:
                res = torch.empty(R, n_out, dtype=torch.float32, device=self.comm_dev)
                self._recv_into(res, last, self.ret_group)
                res = res.cpu()
            elif status == ST_DEADLINE:  # a stage's payload receive timed out: blame its hop
                hdr = [rid, R, n_out, status, extra]
            with self._pending_lock:
                fut = self._pending.pop(rid, None)
            if fut is not None:
                fut.set_result((hdr, res))
            else:
                log.warning(f"dropping the late answer of request {rid} (its caller timed out)")

    def stop_chain(self, timeout: float = 10.0) -> None:
        if self.fast is not None:
            self.fast.stop()
        if self.world > 1:
            self._sendq.put(None)
            for t in self._threads:
                t.join(timeout)

    # -- ranks > 0 ------------------------------------------------------------------------------
    def _maybe_fault(self, served: int) -> None:
        if self.fault_stage != str(self.rank) or served < self.fault_after:
            return
        if self.fault_kind == "hang":
            log.error(f"({self.names[self.rank]}) injected hang")
            while True:
                time.sleep(3600)
        raise RuntimeError("injected fault")

    def loop(self) -> None:
        if self.work_stream is not None:
            torch.cuda.set_stream(self.work_stream)
        prev = self.rank - 1
        last = self.rank == self.world - 1
        in_w = self.stage.in_pad
        served = 0
        while True:
            hdr, pk = self._recv_hdr(prev, self.fwd_group, in_w)
            req, R, width, status, extra = hdr
            if status == ST_STOP:
                if last:
                    self._send(self._hdr(0, 0, 0, ST_STOP, 0), 0, self.ret_group)
                else:
                    self._send_msg([0, 0, 0, ST_STOP, 0], None, self.rank + 1, self.fwd_group,
                                   self.out_pad)
                return
            # the GPU is this request's: a persistent device-chain kernel steps aside
            with (self.fast.paused() if self.fast is not None else nullcontext()):
                if status != ST_OK:  # propagate an upstream failure
                    self._processed = req
                    self._forward_hdr(last, req, R, 0, status, extra)
                    continue
                buf = self.stage.buffers(R)
                if R <= self.small:
                    buf["x"].reshape(-1).view(torch.uint8).copy_(
                        pk[HDR_BYTES:HDR_BYTES + R * width * 2])
                elif not self._recv_payload(buf["x"], prev, self.fwd_group, self.hop_timeout):
                    # the hop is broken: the posted receive would take the next message from
                    # prev (on NCCL the timed-out wait aborts the communicator), so nothing
                    # later on it can be trusted. Report this request, then stop serving; rank 0
                    # blames this stage for every later request from the progress it no longer
                    # publishes.
                    log.error(f"({self.names[self.rank]}) payload of request {req} did not "
                              f"arrive within {self.hop_timeout:.1f} s; the hop from rank {prev} "
                              f"is broken, this stage stops serving")
                    self._forward_hdr(last, req, R, 0, ST_DEADLINE, prev)
                    return
                try:
                    self._maybe_fault(served)
                    out = self.stage.forward(R)
                    if self.comm_dev.type == "cpu":
                        self._sync()
                except ValueError:
                    self._processed = req
                    self._forward_hdr(last, req, R, 0, ST_VALUE, self.rank)
                    continue
                except Exception:  # noqa: BLE001
                    log.exception(f"({self.names[self.rank]}) stage failure")
                    self._processed = req
                    self._forward_hdr(last, req, R, 0, ST_INTERNAL, self.rank)
                    continue
                finally:
                    served += 1
                self._processed = req  # received + computed: what rank 0's blame reads
                if last:
                    self._send(self._hdr(req, R, self.stage.out_dim, ST_OK, 0), 0,
                               self.ret_group)
                    self._send(out[:, :self.stage.out_dim].contiguous(), 0, self.ret_group)
                else:
                    self._send_msg([req, R, out.shape[1], ST_OK, 0], out, self.rank + 1,
                                   self.fwd_group, self.out_pad)

    def _forward_hdr(self, last: bool, req, R, width, status, extra) -> None:
        if last:
            self._send(self._hdr(req, R, width, status, extra), 0, self.ret_group)
        else:
            self._send_msg([req, R, width, status, extra], None, self.rank + 1, self.fwd_group,
                           self.out_pad)


def main(argv: Optional[list[str]] = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--plan", required=True, help="JSON written by run_grpc_fcnn.py")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    plan = json.load(open(a.plan))
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    # a request crosses threads at every hop (ingress worker -> sender -> ... -> receiver ->
    # worker): with the default 5 ms GIL switch interval a hand-off can wait a whole interval
    import sys

    sys.setswitchinterval(1e-4)
    torch.set_num_threads(max(1, min(4, (os.cpu_count() or 8) // max(1, world))))
    use_gpu = plan.get("device", "auto") != "cpu" and torch.cuda.is_available()
    if use_gpu:
        # DNN_FORCE_DEVICE / DNN_DIST_BACKEND=gloo: every stage on one GPU, hops through host
        # memory (one-GPU rehearsals of the rank chain; RCCL needs one GPU per rank)
        local = int(switches.get("DNN_FORCE_DEVICE") or os.environ.get("LOCAL_RANK", rank))
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
        if switches.get("DNN_DIST_BACKEND") == "gloo":
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
    else:
        device = torch.device("cpu")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    st = plan["stages"][rank]
    layers = load_model_config(st["neurons_file"]).layers
    names = [s["name"] for s in plan["stages"]]
    stage = InferenceStage(layers, device, expected_input=st["expected_input"], name=st["name"],
                           is_last=rank == world - 1)
    cr = ChainRank(stage, rank, world, names, device,
                   hop_timeout=plan.get("hop_timeout", HOP_TIMEOUT_S))
    if world > 1 and use_gpu and switches.get("DNN_CHAIN_FAST") == "1":
        why = cr.enable_fast()
        if rank == 0:
            log.info(f"({st['name']}) serving-size requests: {why}")
    log.info(f"({st['name']}) stage ready on {device}: {len(layers)} layer(s), "
             f"expected input dim {st['expected_input']}")
    if rank == 0:
        server = serve(cr.predict, port=plan["port"], name=st["name"],
                       max_workers=plan.get("max_workers", 10))
        done = threading.Event()

        def _stop(signum, frame):
            done.set()
        signal.signal(signal.SIGTERM, _stop)
        signal.signal(signal.SIGINT, _stop)
        done.wait()
        server.stop(grace=1.0)
        cr.stop_chain()
        if any(t.is_alive() for t in cr._threads):  # a stage never answered the STOP
            log.warning(f"({st['name']}) chain did not drain; exiting without teardown")
            logging.shutdown()
            os._exit(0)
    else:
        signal.signal(signal.SIGINT, signal.SIG_IGN)
        cr.loop()
        if cr.fast is not None:  # (a stage hung by fault injection is not waited for)
            cr._fast_thread.join(cr.hop_timeout + 2.0)
    if cr.fast is not None:
        cr.fast.close()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
