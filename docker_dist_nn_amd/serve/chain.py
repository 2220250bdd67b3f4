"""Distributed inference chain: one rank (process / GPU) per non-empty stage.

Reference behaviour (/root/reference/src/grpc_node.py:99-158): stage i computes its layers and
forwards to stage i+1 over a fresh gRPC channel; the last stage's result unwinds back through
every hop. Here:

* rank 0 hosts the gRPC ingress (port 5101) and stage 0; a request becomes a small header
  tensor (request id, rows, cols, status) plus the padded bf16 activations, sent rank to rank
  with torch.distributed (RCCL over xGMI on GPUs, gloo on CPU);
* the LAST rank sends the fp32 result straight back to rank 0 -- one hop, not S;
* a stage that fails turns the header status into an error code carrying its stage index; the
  error travels on to rank 0, which raises ``StageFailure`` -> gRPC status + "Failed to forward
  request to <stage>: ..." like grpc_node.py:136-140;
* ``STOP`` headers shut the chain down in order.

Run by the launcher: ``python -m docker_dist_nn_amd.serve.chain --plan plan.json``.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import signal
import threading
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

log = logging.getLogger(__name__)

ST_OK, ST_STOP, ST_VALUE, ST_INTERNAL = 0, 1, 2, 3
_CODES = {ST_VALUE: grpc.StatusCode.INVALID_ARGUMENT, ST_INTERNAL: grpc.StatusCode.INTERNAL}


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
                 device: torch.device):
        self.stage, self.rank, self.world, self.names = stage, rank, world, names
        self.device = device
        self.comm_dev = device if dist.get_backend() == "nccl" else torch.device("cpu")
        self.lock = threading.Lock()
        self.req = 0
        self.out_pad = round_up(stage.out_dim, 64)

    # -- transport ----------------------------------------------------------------------------
    def _hdr(self, *vals) -> torch.Tensor:
        return torch.tensor(list(vals), dtype=torch.int64, device=self.comm_dev)

    def _send(self, t: torch.Tensor, dst: int) -> None:
        dist.send(t if t.device == self.comm_dev else t.to(self.comm_dev), dst)

    def _recv_into(self, t: torch.Tensor, src: int) -> torch.Tensor:
        if t.device == self.comm_dev:
            dist.recv(t, src)
            return t
        tmp = torch.empty(t.shape, dtype=t.dtype, device=self.comm_dev)
        dist.recv(tmp, src)
        t.copy_(tmp)
        return t

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()

    # -- rank 0 -------------------------------------------------------------------------------
    def predict(self, x: np.ndarray) -> np.ndarray:
        x = np.asarray(x)
        if x.ndim != 2:
            x = x.reshape(x.shape[0], -1)
        rows, cols = x.shape
        self.stage.check_input_dim(cols)  # ValueError -> INVALID_ARGUMENT
        R = bucket(rows)
        with self.lock:
            self.req += 1
            buf = self.stage.buffers(R)
            xb = buf["x"]
            xb.zero_()
            ops.pack_bf16(torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(self.device),
                          xb[:rows])
            out = self.stage.forward(R)
            if self.world == 1:
                res = out[:rows, :self.stage.out_dim].double().cpu().numpy()
                return res
            self._sync()
            self._send(self._hdr(self.req, R, out.shape[1], ST_OK, rows), 1)
            self._send(out, 1)
            hdr = self._recv_into(self._hdr(0, 0, 0, 0, 0), self.world - 1).tolist()
            status = hdr[3]
            if status != ST_OK:
                bad = self.names[hdr[4]] if 0 <= hdr[4] < len(self.names) else "stage"
                raise StageFailure(bad, _CODES.get(status, grpc.StatusCode.INTERNAL),
                                   f"stage {bad} failed (status {status})")
            n_out = hdr[2]
            res = torch.empty(R, n_out, dtype=torch.float32, device=self.device)
            self._recv_into(res, self.world - 1)
            return res[:rows].double().cpu().numpy()

    def stop_chain(self) -> None:
        if self.world > 1:
            with self.lock:
                self._send(self._hdr(0, 0, 0, ST_STOP, 0), 1)

    # -- ranks > 0 ------------------------------------------------------------------------------
    def loop(self) -> None:
        prev = self.rank - 1
        last = self.rank == self.world - 1
        nxt = 0 if last else self.rank + 1
        while True:
            hdr = self._recv_into(self._hdr(0, 0, 0, 0, 0), prev).tolist()
            req, R, width, status, extra = hdr
            if status == ST_STOP:
                if not last:
                    self._send(self._hdr(0, 0, 0, ST_STOP, 0), nxt)
                return
            if status != ST_OK:  # propagate an upstream failure
                self._send(self._hdr(req, R, 0, status, extra), nxt)
                continue
            buf = self.stage.buffers(R)
            self._recv_into(buf["x"], prev)
            try:
                if os.environ.get("DNN_FAULT_STAGE") == str(self.rank):
                    raise RuntimeError("injected fault")
                out = self.stage.forward(R)
                self._sync()
            except ValueError:
                self._send(self._hdr(req, R, 0, ST_VALUE, self.rank), nxt)
                continue
            except Exception:  # noqa: BLE001
                log.exception(f"({self.names[self.rank]}) stage failure")
                self._send(self._hdr(req, R, 0, ST_INTERNAL, self.rank), nxt)
                continue
            if last:
                self._send(self._hdr(req, R, self.stage.out_dim, ST_OK, 0), nxt)
                self._send(out[:, :self.stage.out_dim].contiguous(), nxt)
            else:
                self._send(self._hdr(req, R, out.shape[1], ST_OK, 0), nxt)
                self._send(out, nxt)


def main(argv: Optional[list[str]] = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--plan", required=True, help="JSON written by run_grpc_fcnn.py")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    plan = json.load(open(a.plan))
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    use_gpu = plan.get("device", "auto") != "cpu" and torch.cuda.is_available()
    if use_gpu:
        local = int(os.environ.get("LOCAL_RANK", rank))
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
    else:
        device = torch.device("cpu")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    st = plan["stages"][rank]
    layers = load_model_config(st["neurons_file"]).layers
    names = [s["name"] for s in plan["stages"]]
    stage = InferenceStage(layers, device, expected_input=st["expected_input"], name=st["name"],
                           is_last=rank == world - 1)
    cr = ChainRank(stage, rank, world, names, device)
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
    else:
        signal.signal(signal.SIGINT, signal.SIG_IGN)
        cr.loop()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
