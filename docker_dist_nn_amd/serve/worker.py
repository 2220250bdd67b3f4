"""Process-per-stage worker honouring the reference's stage env contract.

The reference runs one container per stage whose behaviour is fixed by environment variables
(/root/reference/src/grpc_node.py:17-58, set by run_grpc_fcnn.py:101-126):

  CONTAINER_NAME      stage name (default "layer")
  LISTEN_PORT         gRPC port (default 8000)
  EXPECTED_INPUT_DIM  width the first local layer must receive (default 0)
  NEXT_NODES          JSON list of {"host", "port"}; only the first entry is used
  NEURONS_CONFIG      the stage's {"layer_1": [neurons...], ...} JSON inline, or
  NEURONS_FILE_CONFIG a path to it (the launcher's choice for configs > 1000 characters)

This worker keeps that contract, the LayerService protocol and the error mapping of
grpc_node.py:99-158 (ValueError -> INVALID_ARGUMENT, a failed forward keeps the downstream
code and reports "Failed to forward request to <host:port>: <details>", anything else ->
INTERNAL "An internal error occurred: ..."), with the stage's layers on a GPU (gfx950 kernels:
serve/ingress + engine/inference) instead of NumPy fp64, a persistent channel to the next hop
instead of one per request (reference defect #7), a per-hop deadline of 10 s (grpc_node.py:133)
capped by the caller's remaining deadline (defect #8), and no 4 MiB receive cap (defect #1).

Launched by ``run_grpc_fcnn.py --mode workers`` (one process per stage, env written by
weights_io.write_stage_files), or by hand: ``CONTAINER_NAME=... python -m
docker_dist_nn_amd.serve.worker``.
"""
from __future__ import annotations

import json
import logging
import os
import signal
import sys
import threading
from typing import Optional

import grpc
import numpy as np
from .. import switches

log = logging.getLogger("worker")
HOP_TIMEOUT_S = float(switches.get("DNN_HOP_TIMEOUT"))


class StageWorker:
    def __init__(self, env: Optional[dict] = None):
        from ..weights_io import load_stage_env

        env = dict(os.environ if env is None else env)
        self.container_name = env.get("CONTAINER_NAME", "layer")
        self.listen_port = int(env.get("LISTEN_PORT", "8000"))
        self.expected_input_dim = int(env.get("EXPECTED_INPUT_DIM", "0"))
        self.layers = load_stage_env(env)
        self.next_nodes = json.loads(env.get("NEXT_NODES", "[]") or "[]")
        self._next = None
        self._next_lock = threading.Lock()
        self.engine = self._engine(env)
        log.info(f"({self.container_name}) {len(self.layers)} layer(s), expected input dim "
                 f"{self.expected_input_dim}, next nodes {self.next_nodes}")

    def _engine(self, env: dict):
        import torch

        from ..engine.inference import InferenceEngine

        from .. import switches

        want = switches.get("DNN_WORKER_DEVICE", env)
        if want == "cpu" or not torch.cuda.is_available():
            dev = torch.device("cpu")
        else:
            n = torch.cuda.device_count()
            dev = torch.device("cuda", int(env.get("LOCAL_RANK", "0")) % max(1, n))
            torch.cuda.set_device(dev)
        return InferenceEngine([self.layers], dev, expected_input=self.expected_input_dim,
                               names=[self.container_name])

    def _client(self):
        from .ingress import LayerClient

        with self._next_lock:
            if self._next is None:
                n = self.next_nodes[0]
                self._addr = f"{n['host']}:{n['port']}"
                self._next = LayerClient(self._addr, timeout=HOP_TIMEOUT_S)
            return self._next

    def predict(self, x: np.ndarray, timeout: Optional[float] = None) -> np.ndarray:
        from .ingress import StageFailure

        out = self.engine.predict(x)  # ValueError (dim check) -> INVALID_ARGUMENT
        if not self.next_nodes:
            return out
        c = self._client()
        hop = HOP_TIMEOUT_S if timeout is None else max(0.0, min(HOP_TIMEOUT_S, timeout))
        try:
            return c.process(out, timeout=hop)
        except grpc.RpcError as e:
            log.error(f"({self.container_name}) ERROR: gRPC call to {self._addr} failed: "
                      f"{e.code()} - {e.details()}")
            raise StageFailure(self._addr, e.code(), e.details() or "") from None

    def serve(self, block: bool = True):
        from .ingress import serve

        return serve(self.predict, port=self.listen_port, name=self.container_name,
                     max_workers=10, block=block)


def main() -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    try:
        w = StageWorker()
    except Exception as e:  # noqa: BLE001  (grpc_node.py:163-167)
        print(f"Failed to initialize Layer: {e}", flush=True)
        return 1
    server = w.serve(block=False)
    done = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: done.set())
    signal.signal(signal.SIGINT, lambda *_: done.set())
    done.wait()
    server.stop(grace=1.0)
    return 0


if __name__ == "__main__":
    sys.exit(main())
