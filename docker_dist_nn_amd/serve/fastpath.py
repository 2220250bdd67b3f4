"""Device-side serving chain: serving-size requests (<= ops.GEMV_MAX_ROWS rows) cross the rank
chain with no host hop between stages (SURVEY §5 "fast path for tiny messages").

The reference chain makes one blocking gRPC call per hop (/root/reference/src/grpc_node.py:
120-135) driven by the client's per-batch RPC (/root/reference/src/run_grpc_inference.py:
112-158). The message-passing chain (serve/chain.py) still did a host receive, a device->host
header read and a host send per hop. Here:

* every rank owns NSLOT input slots in L2-uncached memory (utils/devmem.py), IPC-mapped by its
  producer, and a flag block (input flags, slot headers, the consumer's ack, a wait-timeout
  word); rank 0 also owns NSLOT result slots, written by the last rank;
* rank 0 announces each request -- (sequence number, rows) -- in a shared-memory ring on the
  node (``/dev/shm``); every stage's host sees it at once and enqueues, on its own stream,
  ``chain_recv`` (wait for the slot's flag, pull the rows into its cached input buffer, ack
  the producer) -> its GEMV layers -> ``chain_send`` (wait until the consumer freed the slot
  this request reuses, copy the rows into the consumer's slot, write the slot header, release
  the consumer's flag) (csrc/kernels/chain.hip). All stages' kernels are queued before the
  rows arrive, so a hop costs kernel time only;
* rank 0's host does the only host work of a request: H2D of the bf16 rows, its own stage,
  the send, then (second stream) a wait on the result flag, one D2H of header + logits, the
  result slot's ack, an event;
* failures keep the reference's semantics (grpc_node.py:136-158, chain.py blame): a stage that
  raises sends its status instead of rows (INVALID_ARGUMENT / INTERNAL naming it); a stage
  whose input does not arrive within the per-hop deadline (10 s, grpc_node.py:133) sends
  DEADLINE_EXCEEDED naming its producer -- the stage that stopped -- and every later stage
  forwards the status unchanged;
* one-layer stages > 0 run as ONE persistent kernel each (``chain_stage_run``, DNN_CHAIN_PERSIST):
  it polls its input flags itself, takes a request's rows from the slot header the producer
  wrote, and serves request after request with no host work at all -- no announcement read, no
  launch; the host thread only relaunches it after an idle exit and publishes its progress
  counter (coherent host memory) for rank 0's blame. A stage that must use the GPU for
  something else (a message-chain request) pauses it first (``paused``);
* larger requests and any set-up that cannot map its peers keep using the message-passing
  chain (serve/chain.py), which stays the fallback.
"""
from __future__ import annotations

import collections
import contextlib
import ctypes
import logging
import mmap
import os
import socket
import threading
import time
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from .. import ops, switches
from ..utils.native import native

log = logging.getLogger(__name__)

NSLOT = 16          # slots per hop: more than the ingress's 10 workers can have in flight
ANN_SLOTS = 1024    # announcement ring
HDR = 64            # bytes of header in front of a result slot's rows
ST_OK, ST_VALUE, ST_INTERNAL, ST_DEADLINE = 0, 2, 3, 4
# flag block layout (int32 words)
F_IN = 0                    # [NSLOT] input flags (written by the producer)
F_HDR = NSLOT               # [NSLOT][2] input slot headers (status, rows)
F_ACK = 3 * NSLOT           # consumer's ack: last request whose slot it has drained
F_ERR = F_ACK + 1           # this rank's recv-timeout word
F_LHDR = F_ACK + 4          # [2] local copy of the current request's input header
F_RES = F_ACK + 8           # rank 0: [NSLOT] result flags (written by the last rank)
F_WORDS = F_RES + NSLOT + 8
PERSIST_IDLE_S = 1.0   # a persistent stage kernel returns after this long without a request
PERSIST_POLL_S = 5e-4  # its host thread's poll period (progress, stop, pause)


class Announcer:
    """Shared-memory ring on the node: rank 0 writes (seq, rows) of every request, the other
    ranks' hosts read them in order. Layout (int64): [0] last announced seq, [1] stop, then
    ANN_SLOTS entries of (seq, rows). x86 stores are not reordered, and the entry is written
    before the head."""

    def __init__(self, path: str, create: bool, timeout: float = 60.0):
        self.path = path
        size = 8 * (4 + 2 * ANN_SLOTS)
        if create:
            fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o600)
            os.ftruncate(fd, size)
        else:
            t0 = time.monotonic()
            while True:
                try:
                    fd = os.open(path, os.O_RDWR)
                    if os.fstat(fd).st_size >= size:
                        break
                    os.close(fd)
                except FileNotFoundError:
                    pass
                if time.monotonic() - t0 > timeout:
                    raise RuntimeError(f"announcement ring {path} did not appear")
                time.sleep(0.01)
        self._mm = mmap.mmap(fd, size)
        os.close(fd)
        self.a = np.ndarray((4 + 2 * ANN_SLOTS,), dtype=np.int64, buffer=self._mm)
        self.owner = create

    def announce(self, seq: int, rows: int) -> None:
        i = 4 + 2 * (seq % ANN_SLOTS)
        self.a[i + 1] = rows
        self.a[i] = seq
        self.a[0] = seq

    def stop(self) -> None:
        self.a[1] = 1

    def next(self, seq: int) -> Optional[int]:
        """Rows of request ``seq`` once announced; None once the chain stops. Spins while
        requests are flowing, backs off to short sleeps when idle."""
        a = self.a
        spins = 0
        while a[0] < seq:
            if a[1]:
                return None
            spins += 1
            if spins > 20000:
                time.sleep(50e-6)
        i = 4 + 2 * (seq % ANN_SLOTS)
        while a[i] != seq:  # the head is written last; the entry is there
            if a[i] > seq:  # lapped: rank 0 ran a whole ring ahead of this stage
                raise RuntimeError(f"announcement ring overrun at request {seq}")
            if a[1]:
                return None
            time.sleep(0)
        return int(a[i + 1])

    def close(self) -> None:
        try:
            del self.a
            self._mm.close()
        except (BufferError, ValueError):
            pass
        if self.owner:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass


def _ptr(t: torch.Tensor, word: int = 0) -> int:
    return t.data_ptr() + 4 * word


class FastChain:
    """The device-side chain of one rank (see the module docstring). Built collectively by
    every rank of the chain; ``ok`` is agreed (all ranks run the fast path or none)."""

    def __init__(self, cr, ann_dir: str = "/dev/shm"):
        self.cr = cr
        st = cr.stage
        self.rank, self.world = cr.rank, cr.world
        self.dev = cr.device
        self.n = None
        self.ok = False
        self.max_rows = ops.GEMV_MAX_ROWS
        mine: dict = {}
        err = None
        try:
            if self.dev.type != "cuda" or self.world < 2:
                raise RuntimeError("needs GPU stages and >= 2 ranks")
            self.n = native()
            from ..utils.devmem import uncached_zeros

            self.flags = uncached_zeros((F_WORDS,), torch.int32, self.dev)
            self.in_w = st.in_pad
            self.out_w = st.pads[-1]
            self.out_f32 = st.is_last
            if self.rank > 0:
                self.slots = uncached_zeros((NSLOT, self.max_rows, self.in_w), torch.bfloat16,
                                            self.dev)
                self.x_local = torch.zeros(self.max_rows, self.in_w, dtype=torch.bfloat16,
                                           device=self.dev)
            torch.cuda.synchronize(self.dev)
            mine = {"flags": self.n.ipc_export(self.flags.data_ptr()),
                    "in_w": self.in_w, "out_w": self.out_w, "out_dim": st.out_dim,
                    # which GPU: persistent stages sharing one split its workgroup slots
                    "gpu": (socket.gethostname(), str(torch.cuda.get_device_properties(
                        self.dev).uuid))}
            if self.rank > 0:
                mine["slots"] = self.n.ipc_export(self.slots.data_ptr())
        except Exception as e:  # noqa: BLE001 -- agreed on below
            err = e
            mine = {"error": repr(e)}
        everyone = [None] * self.world
        dist.all_gather_object(everyone, mine)
        # rank 0 sizes its result slots by the last stage's output width (the last rank
        # addresses them with the same stride)
        if "error" not in everyone[0] and all("error" not in e for e in everyone):
            try:
                w_last = everyone[-1]["out_w"]
                self.res_w = w_last
                self.res_bytes = HDR + self.max_rows * w_last * 4
                if self.rank == 0:
                    self.res = uncached_zeros((NSLOT, self.res_bytes // 4), torch.int32,
                                              self.dev)
                    torch.cuda.synchronize(self.dev)
                    res_h = self.n.ipc_export(self.res.data_ptr())
                else:
                    res_h = None
            except Exception as e:  # noqa: BLE001
                err = err or e
                res_h = None
        else:
            res_h = None
        res_all = [None] * self.world
        dist.all_gather_object(res_all, {"res": res_h, "error": repr(err) if err else None})
        bad = [(r, e["error"]) for r, e in enumerate(everyone) if "error" in e] + \
              [(r, e["error"]) for r, e in enumerate(res_all) if e["error"]]
        # widths must chain: a producer's padded output is its consumer's padded input
        for r in range(self.world - 1):
            if not bad and everyone[r]["out_w"] != everyone[r + 1]["in_w"]:
                bad.append((r, f"width {everyone[r]['out_w']} -> {everyone[r + 1]['in_w']}"))
        if not bad:  # the ranks on this rank's GPU: the persistent stages that may share it
            self.gpu_share = sum(1 for r in range(self.world)
                                 if everyone[r].get("gpu") == everyone[self.rank].get("gpu"))
        if bad:
            self.why = f"fast path unavailable: {bad}"[:300]
            log.info(self.why)
            self._agree(False)
            return
        ok = True
        try:
            imp = lambda r, k: self.n.ipc_import(*everyone[r][k])  # noqa: E731
            nxt = (self.rank + 1) % self.world
            self.next_flags = imp(nxt, "flags")
            self.prev_flags = imp(self.rank - 1, "flags") if self.rank > 0 else 0
            self._last_flags = imp(self.world - 1, "flags") if self.rank == 0 else 0
            self.n_out = everyone[-1]["out_dim"]
            if self.rank == self.world - 1:
                self.dst = self.n.ipc_import(*res_all[0]["res"])  # rank 0's result slots
            else:
                self.dst = imp(nxt, "slots")
        except Exception as e:  # noqa: BLE001
            log.warning(f"fast path peer mapping failed: {e!r}")
            ok = False
        if not self._agree(ok):
            self.why = "fast path unavailable: peer mapping failed on a rank"
            return
        # the announcement ring: rank 0 creates it, its name travels with a broadcast
        name = [f"{ann_dir}/dnn_chain_{os.getpid()}_{os.environ.get('MASTER_PORT', '0')}"
                if self.rank == 0 else None]
        dist.broadcast_object_list(name, src=0)
        try:
            self.ann = Announcer(name[0], create=self.rank == 0)
            good = True
        except Exception as e:  # noqa: BLE001
            log.warning(f"announcement ring unavailable: {e!r}")
            good = False
        if not self._agree(good):
            self.why = "fast path unavailable: no shared-memory announcement ring"
            return
        self.ack_ptr = _ptr(self.flags, F_ACK)  # this rank's "consumer drained" word
        self.res_flags_ptr = self.next_flags + 4 * F_RES if self.rank == self.world - 1 else 0
        self.stream = torch.cuda.Stream(self.dev)
        # the stage's last layer fused with the send of its hop (chain_gemv_send): not for a
        # softmax output (a row-wise second pass)
        self.fused = (switches.get("DNN_CHAIN_FUSED") == "1" and
                      st.acts[-1] != "softmax")
        self.counter = torch.zeros(4, dtype=torch.int32, device=self.dev)
        self.one_launch = self.fused and switches.get("DNN_CHAIN_ONE_LAUNCH") == "1"
        self.trace = switches.get("DNN_CHAIN_TRACE") == "1"
        self.lat: collections.deque = collections.deque(maxlen=100000)  # rank 0: seconds
        self.host = None  # rank 0: runtime ChainHost (the native request path)
        self.seq = 0
        self.inflight = 0  # rank 0: requests announced and not yet answered (back-pressure)
        self.lock = threading.Lock()
        self.processed = 0
        if self.rank == 0:
            self.res_stream = torch.cuda.Stream(self.dev)
            self.h_in = [torch.zeros(self.max_rows, self.in_w, dtype=torch.bfloat16,
                                     pin_memory=True) for _ in range(NSLOT)]
            self.h_out = [torch.zeros(self.res_bytes // 4, dtype=torch.int32, pin_memory=True)
                          for _ in range(NSLOT)]
            self.x0 = torch.zeros(self.max_rows, self.in_w, dtype=torch.bfloat16,
                                  device=self.dev)
            self.events = [torch.cuda.Event() for _ in range(NSLOT)]
            # one-layer stage 0 on the fused path: the whole request is one native call
            # (runtime/chain_host.cpp), its completion a GIL-free spin
            self.host = (self.n.ChainHost(NSLOT) if self.fused and len(st.layers) == 1 and
                         switches.get("DNN_CHAIN_NATIVE") == "1" else None)
        self.failed = False
        self.persist = self._persist_ok()
        self._setup_doorbell(ann_dir, st)
        if self.persist:
            self._set_persist_state()
        self.ok = True
        self.why = (f"device-side chain ({NSLOT} slots per hop"
                    + (", last layer fused with the send" if self.fused else "")
                    + (", one-layer stages as persistent kernels"
                       if switches.get("DNN_CHAIN_PERSIST") == "1" else "")
                    + (", requests and results through host-memory doorbells"
                       if self.doorbell else "") + ")")
        if self.doorbell and self.rank == 0:  # rank 0's own stage kernel and its runner
            t = threading.Thread(target=self.loop, name="chain-doorbell", daemon=True)
            t.start()
            self._runner = t

    # ---- doorbells (rank 0 <-> host memory) ---------------------------------------------------
    def _setup_doorbell(self, ann_dir: str, st) -> None:
        """DNN_CHAIN_DOORBELL: rank 0's stage is a persistent kernel too, reading each request
        from host memory the ingress thread writes (rows, header, then the flag), and the last
        rank writes results into a host-memory ring shared with rank 0 (a /dev/shm mapping
        page-locked in both processes), which rank 0's thread polls on the CPU. A request then
        costs rank 0 a bf16 conversion, a few stores and a spin: no HIP call at all."""
        self.doorbell = False
        name = [None]
        if self.rank == 0 and switches.get("DNN_CHAIN_DOORBELL") == "1" and \
                self._persist_ok(rank0=True):
            path = f"{ann_dir}/dnn_res_{os.getpid()}_{os.environ.get('MASTER_PORT', '0')}"
            try:
                fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o600)
                os.ftruncate(fd, NSLOT * self.res_bytes + 4096)
                os.close(fd)
                name = [path]
            except OSError as e:
                log.info(f"doorbell result ring unavailable: {e!r}")
        dist.broadcast_object_list(name, src=0)
        if name[0] is None:
            return
        good = True
        try:
            if self.rank in (0, self.world - 1):
                self._open_results(name[0])
            if self.rank == 0:
                self._open_requests()
        except Exception as e:  # noqa: BLE001 -- agreed on below
            log.warning(f"doorbell set-up failed: {e!r}")
            good = False
        self.doorbell = self._agree(good)
        if not self.doorbell:
            self._close_doorbell()
            return
        if self.rank == self.world - 1:  # results go to the shared host ring
            self.dst = self._res_dev
            self.res_flags_ptr = self._res_dev + self._res_flag_off
            self.ack_ptr = self._res_dev + self._res_flag_off + 4 * NSLOT
        if self.rank == 0:
            self.persist = True

    def _open_results(self, path: str) -> None:
        size = NSLOT * self.res_bytes + 4096
        fd = os.open(path, os.O_RDWR)
        try:
            mm = mmap.mmap(fd, size)
        finally:
            os.close(fd)
        self._res_mm, self._res_path, self._res_size = mm, path, size
        self._res_anchor = ctypes.c_char.from_buffer(mm)  # (released before mm.close())
        self._res_host = ctypes.addressof(self._res_anchor)
        self._res_flag_off = NSLOT * self.res_bytes
        self.res_np = np.ndarray((size // 4,), dtype=np.int32, buffer=mm)
        self._res_dev = self.n.host_register(self._res_host, size)

    def _open_requests(self) -> None:
        row_b = self.max_rows * self.in_w * 2
        self._req_rows_off = 0
        self._req_hdr_off = NSLOT * row_b
        self._req_flag_off = self._req_hdr_off + 8 * NSLOT
        self._req_ack_off = self._req_flag_off + 4 * NSLOT
        size = self._req_ack_off + 64
        self._req_host, self._req_dev = self.n.host_alloc_mapped(size)
        buf = (ctypes.c_char * size).from_address(self._req_host)
        words = np.frombuffer(buf, dtype=np.int32)
        self.req_hdr = words[self._req_hdr_off // 4:self._req_flag_off // 4].reshape(NSLOT, 2)
        self.req_flag = words[self._req_flag_off // 4:self._req_ack_off // 4]
        self.req_ack = words[self._req_ack_off // 4:self._req_ack_off // 4 + 1]
        self.req_rows = torch.from_numpy(
            np.frombuffer(buf, dtype=np.int16, count=NSLOT * self.max_rows * self.in_w)
            .reshape(NSLOT, self.max_rows, self.in_w)).view(torch.bfloat16)
        self._res_acked = 0
        self._res_done: set = set()

    def _close_doorbell(self) -> None:
        if getattr(self, "_res_mm", None) is not None:
            if getattr(self, "_res_dev", None):
                self.n.host_unregister(self._res_host)
                self._res_dev = 0
            self.res_np = None
            self._res_anchor = None
            try:
                self._res_mm.close()
            except (BufferError, ValueError):
                pass
            self._res_mm = None
            if self.rank == 0:
                try:
                    os.unlink(self._res_path)
                except FileNotFoundError:
                    pass
        if getattr(self, "_req_host", None):
            self.req_rows = self.req_hdr = self.req_flag = self.req_ack = None
            self.n.host_free(self._req_host)
            self._req_host = 0

    def _agree(self, ok: bool) -> bool:
        from ..parallel.comm import _cpu_group

        t = torch.tensor([0 if ok else 1], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=_cpu_group())
        return int(t.item()) == 0

    # ---- addresses ----------------------------------------------------------------------------
    def _dst(self, slot: int) -> tuple[int, int, int, int]:
        """(rows address, leading dimension bytes, header address, flag address) of the
        consumer's slot ``slot``."""
        if self.rank == self.world - 1:  # rank 0's result slot: header, then fp32 rows
            base = self.dst + slot * self.res_bytes
            return base + HDR, self.out_w * 4, base, self.res_flags_ptr + 4 * slot
        row_b = self.out_w * 2
        return (self.dst + slot * self.max_rows * row_b, row_b,
                self.next_flags + 4 * (F_HDR + 2 * slot), self.next_flags + 4 * (F_IN + slot))

    def _send(self, s: torch.cuda.Stream, out: Optional[torch.Tensor], rows: int, seq: int,
              status: int, in_hdr: int) -> None:
        slot = seq % NSLOT
        dst, dld, dhdr, dflag = self._dst(slot)
        if out is None:
            src, sld, rb = 0, 0, 0
        else:
            src, sld = out.data_ptr(), out.stride(0) * out.element_size()
            rb = self.out_w * out.element_size()
        self.n.chain_send(s.cuda_stream, src, sld, dst, dld, rows if out is not None else 0, rb,
                          dhdr, in_hdr, _ptr(self.flags, F_ERR), self.rank, status,
                          self.ack_ptr, (seq - NSLOT) & 0xFFFFFFFF, dflag, seq, 0,
                          self.cr.hop_timeout)  # (ack compares wrap: seq < NSLOT passes)

    def _gemv_send(self, s: torch.cuda.Stream, x: torch.Tensor, rows: int, seq: int,
                   in_hdr: int, recv: bool = False) -> None:
        """The stage's layers up to the last, then the last one fused with the hop's send:
        its rows go straight into the consumer's slot (csrc/kernels/chain.hip). ``recv``
        (one-layer stages > 0): the receive is folded in too -- the kernel waits for this
        stage's input flag and reads the rows from the slot itself, one launch per hop."""
        st = self.cr.stage
        L = len(st.layers)
        if L > 1:
            x = st.forward(rows, x=x, upto=L - 1)
        w, b = st.w[-1], st.b[-1]
        slot = seq % NSLOT
        dst, dld, dhdr, dflag = self._dst(slot)
        f32 = self.rank == self.world - 1  # the last rank fills rank 0's fp32 result slots
        if recv:
            x_ptr, ldx = self.slots[slot].data_ptr(), self.in_w
            in_flag, prev_ack = _ptr(self.flags, F_IN + slot), self.prev_flags + 4 * F_ACK
        else:
            x_ptr, ldx, in_flag, prev_ack = x.data_ptr(), x.stride(0), 0, 0
        self.n.chain_gemv_send(s.cuda_stream, x_ptr, ldx, w.data_ptr(), w.stride(0),
                               b.data_ptr(), ops.kernels._act(st.acts[-1]), rows, w.shape[0],
                               self.in_w if recv else x.shape[1], int(f32), dst,
                               dld // (4 if f32 else 2), dhdr, in_hdr, _ptr(self.flags, F_ERR),
                               self.rank, 0, self.ack_ptr,
                               (seq - NSLOT) & 0xFFFFFFFF, dflag, seq, prev_ack,
                               self.counter.data_ptr(), self.cr.hop_timeout, in_flag=in_flag)

    # ---- rank 0 -------------------------------------------------------------------------------
    def predict(self, x: np.ndarray, timeout: Optional[float]) -> np.ndarray:
        """One request of <= max_rows rows through the device-side chain -> float64 outputs.
        Back-pressure: the stages read the announcement ring in order, so rank 0 never has
        more than half a ring of requests in flight (RESOURCE_EXHAUSTED beyond that)."""
        import grpc

        from .ingress import StageFailure

        with self.lock:
            if self.inflight >= ANN_SLOTS // 2:
                raise StageFailure(self.cr.names[0], grpc.StatusCode.RESOURCE_EXHAUSTED,
                                   f"{self.inflight} requests in flight on the device-side "
                                   f"chain")
            self.inflight += 1
        try:
            if self.doorbell:
                return self._predict_doorbell(x, timeout)
            return self._predict(x, timeout)
        finally:
            with self.lock:
                self.inflight -= 1

    def _predict(self, x: np.ndarray, timeout: Optional[float]) -> np.ndarray:
        import grpc

        from .ingress import StageFailure

        t_in = time.perf_counter()
        rows = x.shape[0]
        st = self.cr.stage
        n = self.n
        with self.lock:
            self.seq += 1
            seq = self.seq
            slot = seq % NSLOT
            hin = self.h_in[slot]
            hin[:rows, :x.shape[1]].copy_(torch.from_numpy(np.ascontiguousarray(x, np.float32)))
            self.ann.announce(seq, rows)
            if self.host is not None:
                self._native_request(seq, slot, rows)
        if self.host is not None:
            limit = self.cr.hop_timeout * self.world
            if timeout is not None:
                limit = min(limit, max(0.0, timeout))
            if self.host.wait(slot, limit):
                k = self.cr.blame(seq) if self.cr.store is not None else self.world - 1
                raise StageFailure(self.cr.names[k], grpc.StatusCode.DEADLINE_EXCEEDED,
                                   f"Deadline Exceeded (request {seq} not answered within "
                                   f"{limit:.1f} s)")
            return self._result(seq, slot, rows, t_in)
        with self.lock:
            if self.trace:
                self._trace(seq, f"announced rows={rows}")
            with torch.cuda.stream(self.stream):
                self.x0[:rows].copy_(hin[:rows], non_blocking=True)
                status, out, sent = 0, None, False
                try:
                    if self.fused:
                        self._gemv_send(self.stream, self.x0[:rows], rows, seq, 0)
                        sent = True
                    else:
                        out = st.forward(rows, x=self.x0[:rows])
                except ValueError:
                    out, status = None, ST_VALUE
                if not sent:
                    self._send(self.stream, out, rows, seq, status, 0)
            rs = self.res_stream
            base = self.res[slot]
            n.chain_wait(rs.cuda_stream, _ptr(self.flags, F_RES + slot), seq, _ptr(base, 2),
                         self.cr.hop_timeout * self.world)
            ho = self.h_out[slot]
            nbytes = HDR + rows * self.res_w * 4
            with torch.cuda.stream(rs):
                ho[:nbytes // 4].copy_(base[:nbytes // 4], non_blocking=True)
            # the result slot is free again (the last rank waits for this before reusing it)
            n.chain_signal(rs.cuda_stream, self.prev_flags_of_last() + 4 * F_ACK, seq)
            ev = self.events[slot]
            ev.record(rs)
        limit = self.cr.hop_timeout * self.world
        if timeout is not None:
            limit = min(limit, max(0.0, timeout))
        t_end = time.monotonic() + limit
        spins = 0
        while not ev.query():
            if time.monotonic() > t_end:
                k = self.cr.blame(seq) if self.cr.store is not None else self.world - 1
                raise StageFailure(self.cr.names[k], grpc.StatusCode.DEADLINE_EXCEEDED,
                                   f"Deadline Exceeded (request {seq} not answered within "
                                   f"{limit:.1f} s)")
            spins += 1
            if spins > 2000:
                time.sleep(20e-6)
        return self._result(seq, slot, rows, t_in)

    def _predict_doorbell(self, x: np.ndarray, timeout: Optional[float]) -> np.ndarray:
        """The request through host memory: rows (bf16), header, flag -> rank 0's persistent
        stage kernel; the logits come back in the shared result ring, polled here."""
        import grpc

        from .ingress import StageFailure

        t_in = time.perf_counter()
        rows, cols = x.shape
        xb = torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(torch.bfloat16)
        limit = self.cr.hop_timeout * self.world
        if timeout is not None:
            limit = min(limit, max(0.0, timeout))
        t_end = time.monotonic() + limit
        with self.lock:
            self.seq += 1
            seq = self.seq
            slot = seq % NSLOT
            # the slot's previous request was read by the stage kernel (practically always)
            while int(self.req_ack[0]) - (seq - NSLOT) < 0:
                if time.monotonic() > t_end:
                    raise StageFailure(self.cr.names[0], grpc.StatusCode.DEADLINE_EXCEEDED,
                                       f"Deadline Exceeded (request slot {slot} not free)")
                time.sleep(0)
            self.req_rows[slot, :rows, :cols].copy_(xb)
            self.req_hdr[slot, 0] = 0
            self.req_hdr[slot, 1] = rows
            self.req_flag[slot] = seq  # last: the kernel reads rows and header after it
            self.ann.announce(seq, rows)  # (stages on the host loop follow the ring)
        base = slot * self.res_bytes // 4
        flag_i = self._res_flag_off // 4 + slot
        res = self.res_np
        spins = 0
        try:
            while res[flag_i] != seq:
                spins += 1
                if spins > 2000:
                    if time.monotonic() > t_end:
                        k = self.cr.blame(seq) if self.cr.store is not None else self.world - 1
                        raise StageFailure(self.cr.names[k], grpc.StatusCode.DEADLINE_EXCEEDED,
                                           f"Deadline Exceeded (request {seq} not answered "
                                           f"within {limit:.1f} s)")
                    time.sleep(20e-6)
            hdr = res[base:base + 2].tolist()
            out = res[base + HDR // 4:base + HDR // 4 + rows * self.res_w].view(np.float32)
            out = out.reshape(rows, self.res_w)[:, :self.n_out].astype(np.float64)
        finally:
            self._consume(seq)
        code, who = hdr[0] & 0xFF, (hdr[0] >> 8) & 0xFF
        if code != ST_OK:
            bad = self.cr.names[who % self.world]
            if code == ST_DEADLINE:
                raise StageFailure(bad, grpc.StatusCode.DEADLINE_EXCEEDED,
                                   f"Deadline Exceeded (request {seq}: {bad} did not answer "
                                   f"within {self.cr.hop_timeout:.1f} s)")
            raise StageFailure(bad, grpc.StatusCode.INVALID_ARGUMENT if code == ST_VALUE
                               else grpc.StatusCode.INTERNAL, f"stage {bad} failed (status "
                               f"{code})")
        self.lat.append(time.perf_counter() - t_in)
        return out

    def _consume(self, seq: int) -> None:
        """Result slot of ``seq`` read (or abandoned): the shared ack word advances over the
        contiguous run of consumed requests (the last rank reuses a slot only behind it)."""
        with self.lock:
            self._res_done.add(seq)
            a = self._res_acked
            while a + 1 in self._res_done:
                a += 1
                self._res_done.discard(a)
            self._res_acked = a
            self.res_np[self._res_flag_off // 4 + NSLOT] = a

    def _native_request(self, seq: int, slot: int, rows: int) -> None:
        """Rank 0, one-layer stage, fused path: H2D + layer-and-send + result wait + D2H +
        ack + event as one native call (runtime/chain_host.cpp)."""
        st = self.cr.stage
        w, b = st.w[0], st.b[0]
        dst, dld, dhdr, dflag = self._dst(slot)
        base = self.res[slot]
        f32 = self.world == 1  # (rank 0 feeds rank 1's bf16 slot)
        self.host.request(
            slot, self.stream.cuda_stream, self.res_stream.cuda_stream, self.x0.data_ptr(),
            self.h_in[slot].data_ptr(), rows * self.in_w * 2, w.data_ptr(), w.stride(0),
            b.data_ptr(), ops.kernels._act(st.acts[0]), rows, w.shape[0], self.in_w, dst,
            dld // (4 if f32 else 2), dhdr, _ptr(self.flags, F_ERR), _ptr(self.flags, F_ACK),
            (seq - NSLOT) & 0xFFFFFFFF, dflag, seq, self.counter.data_ptr(),
            self.cr.hop_timeout, _ptr(self.flags, F_RES + slot), _ptr(base, 2),
            base.data_ptr(), self.h_out[slot].data_ptr(),
            HDR + rows * self.res_w * 4, self.prev_flags_of_last() + 4 * F_ACK,
            self.cr.hop_timeout * self.world)

    def _result(self, seq: int, slot: int, rows: int, t_in: float) -> np.ndarray:
        """Decode the result slot's host copy (header, then fp32 rows) of request ``seq``."""
        import grpc

        from .ingress import StageFailure

        ho = self.h_out[slot]
        hdr = ho[:4].tolist()
        if self.trace:
            self._trace(seq, f"result hdr {hdr}")
        code, who = hdr[0] & 0xFF, (hdr[0] >> 8) & 0xFF
        if hdr[2]:  # rank 0's own wait gave up: the last stage never answered
            code, who = ST_DEADLINE, self.world - 1
        if code != ST_OK:
            bad = self.cr.names[who % self.world]
            if code == ST_DEADLINE:
                raise StageFailure(bad, grpc.StatusCode.DEADLINE_EXCEEDED,
                                   f"Deadline Exceeded (request {seq}: {bad} did not answer "
                                   f"within {self.cr.hop_timeout:.1f} s)")
            raise StageFailure(bad, grpc.StatusCode.INVALID_ARGUMENT if code == ST_VALUE
                               else grpc.StatusCode.INTERNAL, f"stage {bad} failed (status "
                               f"{code})")
        vals = ho[HDR // 4:HDR // 4 + rows * self.res_w].view(torch.float32)
        out = vals.view(rows, self.res_w)[:, :self.n_out].double().numpy()
        self.lat.append(time.perf_counter() - t_in)
        return out

    def latency_summary(self) -> str:
        """Rank 0: percentiles of predict() itself -- request in to logits out, the whole
        device-side chain without the gRPC ingress around it."""
        t = np.asarray(self.lat, dtype=np.float64) * 1e3
        if t.size == 0:
            return "device-side chain: no requests"
        p = np.percentile(t, [50, 90, 99])
        return (f"device-side chain predict latency over {t.size} requests: p50 {p[0]:.4f} ms "
                f"p90 {p[1]:.4f} ms p99 {p[2]:.4f} ms")

    def _trace(self, seq: int, what: str) -> None:
        f = self.flags.tolist()
        log.warning(f"[chain-fast r{self.rank} {time.monotonic():.4f}] seq {seq}: {what}; "
                    f"in={f[F_IN:F_IN + NSLOT]} hdr={f[F_HDR:F_HDR + 2 * NSLOT]} "
                    f"ack={f[F_ACK]} err={f[F_ERR]} lhdr={f[F_LHDR:F_LHDR + 2]}"
                    + (f" res={f[F_RES:F_RES + NSLOT]}" if self.rank == 0 else ""))

    def prev_flags_of_last(self) -> int:
        """Rank 0: the last rank's flag block (its ack word is what rank 0 writes)."""
        return self._last_flags

    # ---- ranks > 0 ----------------------------------------------------------------------------
    def loop(self) -> None:
        """Serve announced requests in order until the ring stops. A failure of this thread is
        logged and ends the stage's device-side serving: its progress stops, so rank 0 blames
        this stage by name for every later request (chain.ChainRank.blame)."""
        try:
            if self.persist:
                self._persist_loop()
            else:
                self._host_loop()
        except Exception:  # noqa: BLE001
            self.failed = True
            log.exception(f"({self.cr.names[self.rank]}) device-side chain thread failed; this "
                          f"stage stops serving serving-size requests")

    def _host_loop(self) -> None:
        n = self.n
        seq = 0
        s = self.stream
        row_b = self.in_w * 2
        while True:
            seq += 1
            rows = self.ann.next(seq)
            if rows is None:
                break
            slot = seq % NSLOT
            one_launch = self.one_launch and len(self.cr.stage.layers) == 1 and \
                self.cr.fault_stage != str(self.rank)
            if one_launch:  # receive + layer + send in ONE kernel
                with torch.cuda.stream(s):
                    self._gemv_send(s, None, rows, seq, _ptr(self.flags, F_HDR + 2 * slot),
                                    recv=True)
                if self.trace:
                    self._trace(seq, f"enqueued (one launch) rows={rows}")
                    s.synchronize()
                    self._trace(seq, "done")
                self.processed = seq
                self.cr._processed = seq
                continue
            with torch.cuda.stream(s):
                n.chain_recv(s.cuda_stream, _ptr(self.flags, F_IN + slot),
                             self.slots[slot].data_ptr(), row_b,
                             _ptr(self.flags, F_HDR + 2 * slot), self.x_local.data_ptr(), row_b,
                             _ptr(self.flags, F_LHDR), rows, row_b, _ptr(self.flags, F_ERR), seq,
                             self.prev_flags + 4 * F_ACK, self.cr.hop_timeout)
                status, out, sent = 0, None, False
                try:
                    self.cr._maybe_fault(self.processed)
                    if self.fused:
                        self._gemv_send(s, self.x_local[:rows], rows, seq,
                                        _ptr(self.flags, F_LHDR))
                        sent = True
                    else:
                        out = self.cr.stage.forward(rows, x=self.x_local[:rows])
                except ValueError:
                    status = ST_VALUE | (self.rank << 8)
                except Exception:  # noqa: BLE001
                    log.exception(f"({self.cr.names[self.rank]}) stage failure")
                    status = ST_INTERNAL | (self.rank << 8)
                if not sent:
                    self._send(s, out, rows, seq, status, _ptr(self.flags, F_LHDR))
            if self.trace:
                self._trace(seq, f"enqueued rows={rows} status={status}")
                s.synchronize()
                self._trace(seq, "done")
            self.processed = seq
            self.cr._processed = seq
        torch.cuda.synchronize(self.dev)

    # ---- the persistent stage kernel (ranks > 0; rank 0 with the doorbell) --------------------
    def _set_persist_state(self) -> None:
        # the kernel never returns while requests flow: it gets a hardware queue of its own
        # (work of this process's other streams would otherwise wait behind it whenever the
        # runtime maps their stream onto the same queue)
        self._pstream_ptr = self.n.stream_create_dedicated()
        self.pstream = torch.cuda.ExternalStream(self._pstream_ptr, device=self.dev)
        # per-slot arrival counters, ack failures, go, exit (chain.hip ChainStage) and the
        # stop word / progress counter in coherent host memory
        self.sync = torch.zeros(2 * NSLOT + 4, dtype=torch.int32, device=self.dev)
        self._ctl_host, self._ctl_dev = self.n.host_alloc_mapped(64)
        self.ctl = np.ctypeslib.as_array((ctypes.c_uint32 * 16).from_address(self._ctl_host))
        self._want_pause = False
        self._pause_lock = threading.Lock()
        self._parked = threading.Event()
        self._resume = threading.Event()
        self._runner_done = threading.Event()
        self.workgroups = 0

    def _persist_ok(self, rank0: bool = False) -> bool:
        st = self.cr.stage
        if (self.rank == 0) != rank0 or switches.get("DNN_CHAIN_PERSIST") != "1" or \
                len(st.layers) != 1:
            return False
        if self.cr.fault_stage == str(self.rank) or self.trace:
            return False  # fault injection and tracing act per request on the host
        n = st.dims[-1] if st.acts[0] == "softmax" else st.w[0].shape[0]
        lds = self.max_rows * self.in_w * 2 + (self.max_rows * n * 4
                                                if st.acts[0] == "softmax" else 0)
        return lds <= 64 * 1024 and st.w[0].shape[1] == self.in_w

    def _persist_launch(self, start: int, epoch: int) -> None:
        st = self.cr.stage
        w, b, act = st.w[0], st.b[0], st.acts[0]
        last = self.rank == self.world - 1
        if last:  # rank 0's result slots: header, then fp32 rows
            dst, slot_b = self.dst + HDR, self.res_bytes
            hdr, hstride, nflags = self.dst, self.res_bytes // 4, self.res_flags_ptr
        else:
            dst, slot_b = self.dst, self.max_rows * self.out_w * 2
            hdr, hstride, nflags = self.next_flags + 4 * F_HDR, 2, self.next_flags + 4 * F_IN
        if self.rank == 0:  # the doorbell: requests from host memory
            in_flags = self._req_dev + self._req_flag_off
            in_hdrs = self._req_dev + self._req_hdr_off
            in_slots = self._req_dev + self._req_rows_off
            prev_ack = self._req_dev + self._req_ack_off
        else:
            in_flags, in_hdrs = _ptr(self.flags, F_IN), _ptr(self.flags, F_HDR)
            in_slots, prev_ack = self.slots.data_ptr(), self.prev_flags + 4 * F_ACK
        n_out = st.dims[-1] if act == "softmax" else w.shape[0]
        self.workgroups = self.n.chain_stage_run(
            self.pstream.cuda_stream, in_flags, in_hdrs, in_slots, self.in_w, prev_ack,
            w.data_ptr(), w.stride(0), b.data_ptr(), ops.kernels._act(act), n_out, self.in_w,
            int(last), dst, slot_b, self.out_w, hdr, hstride, nflags, self.ack_ptr, self._ctl_dev,
            self._ctl_dev + 4, self.sync.data_ptr(), start & 0xFFFFFFFF, epoch, self.rank, NSLOT,
            self.max_rows, PERSIST_IDLE_S, self.cr.hop_timeout, share=max(1, self.gpu_share))

    def _persist_loop(self) -> None:
        """Keep the stage kernel running until the ring stops: relaunch it after an idle exit,
        park it while ``paused`` holds the GPU, publish its progress for rank 0's blame."""
        s = self.pstream
        start, epoch = 0, 0
        try:
            while not self.ann.a[1]:
                if self._want_pause:
                    self._parked.set()
                    self._resume.wait()
                    self._resume.clear()
                    continue
                self.ctl[0] = 0
                epoch += 1
                with torch.cuda.stream(s):
                    self._persist_launch(start, epoch)
                ev = torch.cuda.Event()
                ev.record(s)
                asked = False
                while not ev.query():
                    d = int(self.ctl[1])
                    if d != self.processed:  # (the message chain's progress shares the key)
                        self.processed = self.cr._processed = d
                    if not asked and (self.ann.a[1] or self._want_pause):
                        self.ctl[0] = 1  # the kernel returns within ~20 us of waiting
                        asked = True
                    time.sleep(PERSIST_POLL_S)
                start = int(self.ctl[1])
                if start != self.processed:
                    self.processed = self.cr._processed = start
        finally:
            self._runner_done.set()
            self._parked.set()

    @contextlib.contextmanager
    def paused(self):
        """Ranks > 0: hold the GPU for other work (a message-chain request: its kernels, a
        device-wide sync) with the persistent stage kernel stopped; requests arriving meanwhile
        wait in their slots and are served on resume."""
        if not getattr(self, "persist", False):
            yield
            return
        with self._pause_lock:
            self._want_pause = True
            self._parked.wait(self.cr.hop_timeout)
            try:
                yield
            finally:
                self._want_pause = False
                self._parked.clear()
                self._resume.set()

    def stop(self) -> None:
        if self.rank == 0 and self.ok:
            self.ann.stop()
            log.info(self.latency_summary())

    def close(self) -> None:
        if self.ok:
            if self.doorbell and self.rank == 0:
                self._runner.join(5.0)
            self.ann.close()
            if self.persist and self._runner_done.is_set():
                # (a runner still alive may have a kernel that writes these words: leaked)
                self.pstream.synchronize()
                self.n.host_free(self._ctl_host)
                self.n.stream_destroy(self._pstream_ptr)
                self.persist = False
            if self.doorbell and (not self.persist or self.rank != 0):
                self._close_doorbell()
