"""gRPC ingress speaking the reference protocol on the first stage's port (default 5101).

Behaviour of the reference servicer (/root/reference/src/grpc_node.py:99-158) that is kept:
  * an empty request returns an empty Matrix;
  * a dimension problem (ValueError) -> status INVALID_ARGUMENT with the message as details;
  * any other failure -> INTERNAL "An internal error occurred: ..." ;
  * a failure while forwarding to a downstream stage keeps that stage's code and reports
    "Failed to forward request to <stage>: <details>" (grpc_node.py:136-140);
  * on error the response body is an empty Matrix.
Fixed reference defects: the receive limit is unbounded (the reference kept gRPC's 4 MiB
default, grpc_node.py:169, capping a 784-wide batch at 668 rows -- SURVEY §2.7 #1), and no
channel is opened per request: the chain behind this ingress is the GPU pipeline.
"""
from __future__ import annotations

import logging
from concurrent import futures
from typing import Callable, Optional

import grpc
import numpy as np

from . import codec
from .proto import SERVICE

log = logging.getLogger(__name__)

# No 4 MiB cap (reference defect) and bulk-friendly HTTP/2 transport: 16-MiB
# frames, a 64-MiB write buffer and large TCP read chunks. A 4096 x 784 fp64 request (25.7 MB)
# round-trips in 35 ms instead of 82 ms with gRPC's defaults (measured on 127.0.0.1).
UNLIMITED = [("grpc.max_send_message_length", -1), ("grpc.max_receive_message_length", -1),
             ("grpc.http2.max_frame_size", 16777215),
             ("grpc.http2.write_buffer_size", 64 << 20),
             ("grpc.experimental.tcp_read_chunk_size", 4 << 20),
             ("grpc.experimental.tcp_min_read_chunk_size", 1 << 20),
             ("grpc.experimental.tcp_max_read_chunk_size", 16 << 20)]


class StageFailure(Exception):
    """A downstream stage failed: carries the gRPC code and the stage's details."""

    def __init__(self, stage: str, code: grpc.StatusCode, detail: str):
        super().__init__(f"Failed to forward request to {stage}: {detail}")
        self.stage, self.code, self.detail = stage, code, detail


def make_handler(predict: Callable[[np.ndarray], np.ndarray], name: str = "layer_container_0"):
    import inspect

    try:  # a chain's predict honours the caller's deadline (serve/chain.py)
        takes_timeout = "timeout" in inspect.signature(predict).parameters
    except (TypeError, ValueError):
        takes_timeout = False

    def process(x: np.ndarray, context) -> np.ndarray:
        try:
            if x.size == 0:
                log.info(f"({name}) Received empty input matrix.")
                return np.zeros((0, 0))
            if takes_timeout:
                return predict(x, timeout=context.time_remaining())
            return predict(x)
        except StageFailure as e:
            context.set_code(e.code)
            context.set_details(str(e))
        except ValueError as e:
            context.set_code(grpc.StatusCode.INVALID_ARGUMENT)
            context.set_details(str(e))
        except Exception as e:  # noqa: BLE001
            log.exception(f"({name}) unexpected error")
            context.set_code(grpc.StatusCode.INTERNAL)
            context.set_details(f"An internal error occurred: {e}")
        return np.zeros((0, 0))

    def deser(b: bytes):
        try:
            return codec.decode(b)
        except ValueError:
            return None

    def process_raw(x, context):
        if x is None:
            context.set_code(grpc.StatusCode.INVALID_ARGUMENT)
            context.set_details("Matrix rows have different lengths")
            return np.zeros((0, 0))
        return process(x, context)

    return grpc.method_handlers_generic_handler(SERVICE, {
        "Process": grpc.unary_unary_rpc_method_handler(
            process_raw, request_deserializer=deser, response_serializer=codec.encode)})


def serve(predict: Callable[[np.ndarray], np.ndarray], port: int = 5101,
          host: str = "0.0.0.0", max_workers: int = 10, name: str = "layer_container_0",
          block: bool = False) -> grpc.Server:
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers), options=UNLIMITED)
    server.add_generic_rpc_handlers((make_handler(predict, name),))
    bound = server.add_insecure_port(f"{host}:{port}")
    if bound == 0:
        raise RuntimeError(f"could not bind {host}:{port}")
    server.start()
    log.info(f"({name}) gRPC LayerService started on {host}:{bound}")
    if block:
        server.wait_for_termination()
    return server


class LayerClient:
    """Persistent-channel client (the reference cached one stub per process,
    run_grpc_inference.py:122-131)."""

    def __init__(self, address: str, timeout: float = 10.0, wait_ready: Optional[float] = None):
        self.channel = grpc.insecure_channel(address, options=UNLIMITED)
        if wait_ready:
            grpc.channel_ready_future(self.channel).result(timeout=wait_ready)
        self._call = self.channel.unary_unary(f"/{SERVICE}/Process",
                                              request_serializer=codec.encode,
                                              response_deserializer=codec.decode)
        self.timeout = timeout

    def process(self, x, timeout: Optional[float] = None) -> np.ndarray:
        return self._call(np.asarray(x, dtype=np.float64), timeout=timeout or self.timeout)

    def close(self):
        self.channel.close()
