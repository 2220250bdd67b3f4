"""Forward-only (serving) engine: the MI355X counterpart of the reference's stage chain.

The reference ran inference as a chain of containers, each ``np.dot(x, W) + b`` + activation
in fp64 (/root/reference/src/grpc_node.py:75-97), forwarding protobuf rows hop by hop. Here a
stage is a slice of layers on one GPU:

* weights come straight from the reference JSON (any per-layer activation: relu, sigmoid,
  linear, or a row softmax -- grpc_node.py:62-73), stored padded bf16 + fp32 bias;
* inputs are validated against the expected width first, raising the reference's
  ``ValueError("(<stage>) Layer k: expected input dim d, got x")`` (grpc_node.py:83-84);
* each layer is one fused GEMM (bias + activation epilogue); a softmax layer writes fp32 and
  runs the row-softmax kernel; the last layer writes fp32 outputs;
* requests are padded to a row bucket (multiple of 64) and, per bucket, the whole forward is
  captured once in a HIP graph, so a batch-1 request is a single graph launch.
"""
from __future__ import annotations

import os
import threading
from typing import Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..config import LayerWeights
from ..models.mlp import normalize_activation, round_up
from ..utils.native import native
from .. import switches


class InferenceStage:
    def __init__(self, layers: Sequence[LayerWeights], device: torch.device, *,
                 expected_input: int, name: str = "layer", is_last: bool = True,
                 case_sensitive: bool = True):
        self.device = device
        self.name = name
        self.is_last = is_last
        self.expected_input = int(expected_input)
        self.layers = list(layers)
        self.acts = [normalize_activation(L.activation, case_sensitive) for L in self.layers]
        self.dims = [L.in_dim for L in self.layers] + [self.layers[-1].out_dim]
        self.pads = [round_up(d, 64) for d in self.dims]
        self.w, self.b = [], []
        for L, kp, np_ in zip(self.layers, self.pads, self.pads[1:]):
            w = torch.zeros(np_, kp, dtype=torch.float32)
            w[:L.out_dim, :L.in_dim] = torch.as_tensor(np.asarray(L.weight, np.float32))
            b = torch.zeros(np_, dtype=torch.float32)
            b[:L.out_dim] = torch.as_tensor(np.asarray(L.bias, np.float32))
            self.w.append(w.to(device=device, dtype=torch.bfloat16))
            self.b.append(b.to(device))
        self._bufs: dict[int, dict] = {}

    @property
    def in_pad(self) -> int:
        return self.pads[0]

    @property
    def out_dim(self) -> int:
        return self.dims[-1]

    def check_input_dim(self, cols: int) -> None:
        """Dimension walk of grpc_node.py:80-93 against the configured widths."""
        expected, cur = self.expected_input, cols
        for i, L in enumerate(self.layers):
            if cur != expected:
                raise ValueError(f"({self.name}) Layer {i + 1}: expected input dim {expected}, "
                                 f"got {cur}")
            if L.in_dim != cur:  # what np.dot raises for an inconsistent config
                raise ValueError(f"({self.name}) Layer {i + 1}: shapes (n,{cur}) and "
                                 f"({L.in_dim},{L.out_dim}) not aligned")
            cur = expected = L.out_dim

    def buffers(self, rows: int) -> dict:
        b = self._bufs.get(rows)
        if b is None:
            dev = self.device
            b = {"x": torch.zeros(rows, self.pads[0], dtype=torch.bfloat16, device=dev),
                 "h": [], "f32": []}
            for i, np_ in enumerate(self.pads[1:]):
                last = i == len(self.layers) - 1
                need_f32 = (last and self.is_last) or self.acts[i] == "softmax"
                b["h"].append(torch.zeros(rows, np_, dtype=torch.bfloat16, device=dev))
                b["f32"].append(torch.zeros(rows, np_, dtype=torch.float32, device=dev)
                                if need_f32 else None)
            self._bufs[rows] = b
        return b

    def forward(self, rows: int, x: Optional[torch.Tensor] = None,
                upto: Optional[int] = None) -> torch.Tensor:
        """Run on buffers(rows)['x'] (or on ``x``, e.g. the device-side chain's input rows);
        returns fp32 [rows][out_pad] (last stage) or bf16. ``upto``: only layers [0, upto)
        (the device-side chain runs the last one fused with its send)."""
        b = self.buffers(rows)
        if x is None:
            x = b["x"]
        n = len(self.layers)
        for i in range(n if upto is None else upto):
            act = self.acts[i]
            last = i == n - 1
            h, f = b["h"][i], b["f32"][i]
            if act == "softmax":
                ops.linear_fwd(x, self.w[i], self.b[i], f, act="linear")
                ops.softmax_rows(f, f, self.dims[i + 1])
                if last and self.is_last:
                    return f
                ops.pack_bf16(f[:, :self.dims[i + 1]], h)
                x = h
            elif last and self.is_last:
                ops.linear_fwd(x, self.w[i], self.b[i], f, act=act)
                return f
            else:
                ops.linear_fwd(x, self.w[i], self.b[i], h, act=act)
                x = h
        return x


class InferenceEngine:
    """Local (single-process) chain of inference stages; thread-safe ``predict``."""

    def __init__(self, stage_layers: Sequence[Sequence[LayerWeights]], device: torch.device,
                 expected_input: int, names: Optional[Sequence[str]] = None,
                 max_rows: int = 65536, use_graphs: bool = True):
        self.device = device
        self.stages: list[InferenceStage] = []
        exp = expected_input
        names = list(names or [f"layer_container_{i}" for i in range(len(stage_layers))])
        for i, ls in enumerate(stage_layers):
            st = InferenceStage(ls, device, expected_input=exp, name=names[i],
                                is_last=i == len(stage_layers) - 1)
            self.stages.append(st)
            exp = st.out_dim
        self.max_rows = max_rows
        self.use_graphs = use_graphs and device.type == "cuda"
        self._graphs: dict[int, object] = {}
        self._lock = threading.Lock()
        self._stream = torch.cuda.Stream(device) if device.type == "cuda" else None
        self.n_out = self.stages[-1].out_dim
        self._stage_bufs: dict = {}
        # per-bucket replay: "graph" (HIP graph) or "native" (recorded launch Program)
        self.replay = switches.get("DNN_SERVE_REPLAY")
        self._programs: dict[int, tuple] = {}

    @property
    def input_dim(self) -> int:
        return self.stages[0].expected_input

    def validate(self, cols: int) -> None:
        c = cols
        for st in self.stages:
            st.check_input_dim(c)
            c = st.out_dim

    def _bucket(self, rows: int) -> int:
        if self.device.type == "cuda" and rows <= ops.GEMV_MAX_ROWS:
            return rows  # serving sizes run the GEMV kernel on exact rows, no padding
        b = 64
        while b < rows:
            b *= 2
        return min(b, round_up(self.max_rows, 64)) if rows <= self.max_rows else round_up(rows, 64)

    def _run(self, rows: int) -> torch.Tensor:
        out = None
        for k, st in enumerate(self.stages):
            if k > 0:  # hop on one device: the next stage reads the previous output in place
                st.buffers(rows)["x"] = out
            out = st.forward(rows)
        return out

    def _forward_padded(self, rows: int) -> torch.Tensor:
        if not self.use_graphs:
            return self._run(rows)
        if self.replay == "native":  # recorded launches replayed from C++ (no graph launch)
            entry = self._programs.get(rows)
            if entry is None:
                with torch.cuda.stream(self._stream):
                    self._run(rows)  # allocate buffers
                    prog = native().Program()
                    native().record_begin(prog)
                    try:
                        prog.mark("fwd")
                        out = self._run(rows)
                    finally:
                        native().record_end()
                entry = self._programs[rows] = (prog, out)
            prog, out = entry
            prog.run(["fwd"], self._stream.cuda_stream)
            return out
        entry = self._graphs.get(rows)
        if entry is None:
            with torch.cuda.stream(self._stream):
                self._run(rows)  # allocate buffers + warm up
                self._stream.synchronize()
                g = native().GraphExec()
                g.begin_capture(self._stream.cuda_stream)
                try:
                    out = self._run(rows)
                finally:
                    g.end_capture()
            entry = self._graphs[rows] = (g, out)
        g, out = entry
        g.replay(self._stream.cuda_stream)
        return out

    def predict(self, x: np.ndarray) -> np.ndarray:
        """x: [rows][input_dim] (any float dtype) -> float64 [rows][n_out]."""
        x = np.asarray(x)
        if x.ndim == 1:
            x = x[None, :]
        if x.ndim != 2:
            x = x.reshape(x.shape[0], -1)
        rows, cols = x.shape
        if rows == 0:
            return np.zeros((0, 0))
        self.validate(cols)
        out = np.empty((rows, self.n_out), dtype=np.float64)
        with self._lock:
            for r0 in range(0, rows, self.max_rows):
                r1 = min(rows, r0 + self.max_rows)
                out[r0:r1] = self._predict_chunk(x[r0:r1])
        return out

    def _staging(self, rows: int, cols: int):
        """Pinned host input/output buffers + device fp32 input for a row bucket."""
        key = (rows, cols)
        st = self._stage_bufs.get(key)
        if st is None:
            st = (torch.empty(rows, cols, dtype=torch.float32, pin_memory=True),
                  torch.empty(rows, cols, dtype=torch.float32, device=self.device),
                  torch.empty(rows, self.n_out, dtype=torch.float32, pin_memory=True))
            self._stage_bufs[key] = st
        return st

    def _predict_chunk(self, x: np.ndarray) -> np.ndarray:
        rows = x.shape[0]
        R = self._bucket(rows)
        st0 = self.stages[0]
        xb = st0.buffers(R)["x"]
        if self.device.type == "cuda":
            stream = self._stream
            hin, din, hout = self._staging(R, x.shape[1])
            # pinned host staging, reused across calls; torch's CPU copy converts fp64 -> fp32
            # on all intra-op threads (a numpy assignment converts on one: ~7x slower for a
            # 60k x 784 fp64 batch)
            hin[:rows].copy_(torch.from_numpy(np.ascontiguousarray(x)))
            with torch.cuda.stream(stream):
                din[:rows].copy_(hin[:rows], non_blocking=True)
                if R != rows:
                    xb[rows:].zero_()
                ops.pack_bf16(din[:rows], xb[:rows])
                out = self._forward_padded(R)
                hout[:rows].copy_(out[:rows, :self.n_out], non_blocking=True)
            stream.synchronize()
            res = hout[:rows]
        else:
            if R != rows:
                xb[rows:].zero_()
            ops.pack_bf16(torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)), xb[:rows])
            out = self._run(R)
            res = out[:rows, :self.n_out].clone()
        return res.double().numpy()
