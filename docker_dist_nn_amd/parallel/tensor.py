"""Tensor parallelism for the MLP: Megatron-style column / row splits over a TP group.

SURVEY.md §2.5 lists TP as the optional P3 ("the 8192-wide layers could be column/row
split"); the reference itself has none. Consecutive layer pairs are split so that only ONE
collective per pair and direction is needed:

* layer 2k (column-parallel): rank r owns output neurons [r*n/t, (r+1)*n/t) -- W rows and bias
  shard. Its input is replicated, its output y is a column shard: no communication.
* layer 2k+1 (row-parallel): rank r owns the weight COLUMNS that read that shard. Each rank's
  GEMM gives an fp32 partial sum of the full output (rank 0 adds the bias); one all-reduce,
  then activation + bf16 cast (ops.bias_act_cast). Output replicated.
* a trailing unpaired layer (odd depth) is replicated.

Backward mirrors it: the row-parallel dgrad lands directly in the column shard (activation
derivative fused in the GEMM epilogue); the column-parallel dgrad is an fp32 partial sum that
is all-reduced before the previous layer's activation derivative is applied
(ops.dact_colsum). Weight gradients are local; replicated parameters get identical gradients
on every rank, so every update is local too. All GEMMs are the gfx950 kernels of ops.*; the
collectives go through torch.distributed (RCCL on GPUs, gloo on CPU).

Bytes per step per pair: rows x out(2k+1) fp32 forward and rows x in(2k) fp32 backward; the
pairing therefore suits models whose odd layers are narrow (e.g. 784-8192-8192-10 pairs the
8192x8192 product with the 784 input: 16384 x 8192 fp32 per step forward).
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from ..engine.stage import OptimConfig
from ..models.mlp import MLPSpec


def _pad(d: int, m: int = 64) -> int:
    return (d + m - 1) // m * m


def layer_modes(n: int) -> list[str]:
    """col / row for every full pair, rep for a trailing unpaired layer."""
    return ["col" if i % 2 == 0 and i + 1 < n else "row" if i % 2 == 1 else "rep"
            for i in range(n)]


class TensorParallelMLP:
    """One TP rank of an MLP trained on a replicated batch of ``rows`` rows (SGD with
    momentum / weight decay). ``group`` = the TP process group (None = WORLD)."""

    def __init__(self, spec: MLPSpec, *, rows: int, tp: int, rank: int, device: torch.device,
                 group=None, optim: Optional[OptimConfig] = None, seed: int = 0):
        if rows % 64:
            raise ValueError("rows must be a multiple of 64 (pad with label -1)")
        self.spec, self.rows, self.tp, self.rank = spec, rows, tp, rank
        self.device, self.group = device, group
        self.optim = optim or OptimConfig()
        if self.optim.name != "sgd":
            raise ValueError("tensor-parallel training implements SGD (momentum, weight decay)")
        L = spec.layers
        self.modes = layer_modes(len(L))
        self.layers = []
        for i, l in enumerate(L):
            mode = self.modes[i]
            if mode == "col":
                n_full = _pad(l.out_dim, 64 * tp)
                g = dict(n=n_full // tp, k=_pad(l.in_dim), n_full=n_full, k_full=_pad(l.in_dim),
                         rows=slice(rank * (n_full // tp), (rank + 1) * (n_full // tp)),
                         cols=slice(0, _pad(l.in_dim)))
            elif mode == "row":
                prev = self.layers[i - 1]
                g = dict(n=_pad(l.out_dim), k=prev["n"], n_full=_pad(l.out_dim),
                         k_full=prev["n_full"], rows=slice(0, _pad(l.out_dim)),
                         cols=slice(rank * prev["n"], (rank + 1) * prev["n"]))
            else:
                g = dict(n=_pad(l.out_dim), k=_pad(l.in_dim), n_full=_pad(l.out_dim),
                         k_full=_pad(l.in_dim), rows=slice(0, _pad(l.out_dim)),
                         cols=slice(0, _pad(l.in_dim)))
            g.update(mode=mode, act=l.activation, spec=l)
            self.layers.append(g)
        self._init_params(seed)
        self._alloc()
        self.steps_done = 0

    # ---- parameters ------------------------------------------------------------------------
    def _init_params(self, seed: int) -> None:
        """The single-process trainer's init (StageParams.init_default: nn.Linear uniform,
        seeded by global layer index), padded and sliced to this rank's shard."""
        dev, o = self.device, self.optim
        for i, g in enumerate(self.layers):
            l = g["spec"]
            gen = torch.Generator().manual_seed(seed * 7919 + i)
            bound = 1.0 / math.sqrt(l.in_dim)
            w = (torch.rand(l.out_dim, l.in_dim, generator=gen) * 2 - 1) * bound
            b = (torch.rand(l.out_dim, generator=gen) * 2 - 1) * bound
            wf = torch.zeros(g["n_full"], g["k_full"])
            wf[:l.out_dim, :l.in_dim] = w
            bf = torch.zeros(g["n_full"])
            bf[:l.out_dim] = b
            g["w"] = wf[g["rows"], g["cols"]].contiguous().to(dev)
            g["b"] = bf[g["rows"]].contiguous().to(dev)
            g["wbf"] = g["w"].to(torch.bfloat16)
            g["gw"] = torch.zeros_like(g["w"])
            g["gb"] = torch.zeros_like(g["b"])
            g["mw"] = torch.zeros_like(g["w"]) if o.momentum else None
            g["mb"] = torch.zeros_like(g["b"]) if o.momentum else None

    def _alloc(self) -> None:
        R, dev = self.rows, self.device
        bf, f32 = torch.bfloat16, torch.float32
        self.x = torch.zeros(R, self.layers[0]["k"], dtype=bf, device=dev)
        self.labels = torch.full((R,), -1, dtype=torch.int32, device=dev)
        last = len(self.layers) - 1
        for i, g in enumerate(self.layers):
            g["y"] = torch.zeros(R, g["n"], dtype=f32 if i == last else bf, device=dev)
            g["dz"] = torch.zeros(R, g["n"], dtype=bf, device=dev)
            if g["mode"] == "row":
                g["part"] = torch.zeros(R, g["n"], dtype=f32, device=dev)
            if g["mode"] == "col" and i > 0:
                g["dxp"] = torch.zeros(R, g["k"], dtype=f32, device=dev)
            g["splits"] = ops.pick_splits(g["n"], g["k"], R)
            g["slabs"] = torch.zeros(g["splits"], g["n"], g["k"], dtype=f32, device=dev)
            g["bpart"] = torch.zeros(max(1, R // 64), g["n"], dtype=f32, device=dev)
        self.loss_part = torch.zeros(ops.xent_blocks(R), dtype=f32, device=dev)
        self.correct = torch.zeros(ops.xent_blocks(R), dtype=torch.int32, device=dev)
        self.xent_part = torch.zeros(ops.xent_blocks(R), self.layers[-1]["n"], dtype=f32,
                                     device=dev)

    def _all_reduce(self, t: torch.Tensor) -> None:
        if self.tp > 1:
            dist.all_reduce(t, group=self.group)

    # ---- one step ----------------------------------------------------------------------------
    def set_batch(self, x: torch.Tensor, labels: torch.Tensor) -> None:
        """x: [rows][>= in_dim] (any float dtype, replicated on every TP rank); labels [rows]."""
        self.x.zero_()
        self.x[:, :x.shape[1]] = x.to(self.device, torch.bfloat16)
        self.labels.copy_(labels.to(self.device, torch.int32))

    def forward(self) -> None:
        inp = self.x
        last = len(self.layers) - 1
        for i, g in enumerate(self.layers):
            act = g["act"] if i < last else "linear"
            if g["mode"] == "row":  # fp32 partial sums (bias once), all-reduce, activation
                ops.gemm(inp, g["wbf"], g["part"], layout_a=ops.KMAJ, layout_b=ops.KMAJ,
                         M=self.rows, N=g["n"], K=g["k"],
                         bias=g["b"] if self.rank == 0 else None)
                self._all_reduce(g["part"])
                if i == last:
                    g["y"].copy_(g["part"])
                else:
                    ops.bias_act_cast(g["part"], None, g["y"], act=act)
            else:  # column shard or replicated: the fused bias + activation GEMM
                ops.linear_fwd(inp, g["wbf"], g["b"], g["y"], act=act)
            inp = g["y"]

    def backward(self) -> None:
        L = self.layers
        last = len(L) - 1
        n_cls = self.spec.out_dim
        ops.softmax_xent(L[last]["y"], self.labels, L[last]["dz"], n_cls, 1.0 / self.rows,
                         self.loss_part, self.correct)
        for i in range(last, -1, -1):
            g = L[i]
            x_i = self.x if i == 0 else L[i - 1]["y"]
            # weight / bias gradients (local: the shard's rows / columns)
            ops.linear_wgrad(g["dz"], x_i, g["slabs"], splits=g["splits"])
            ops.reduce_slabs(g["slabs"], g["splits"], g["n"] * g["k"], g["n"] * g["k"],
                             g["gw"].view(-1))
            nb = g["bpart"].shape[0]
            ops.colsum_partial(g["dz"], g["bpart"], nb)
            ops.reduce_slabs(g["bpart"], nb, g["n"], g["n"], g["gb"])
            if i == 0:
                continue
            p = L[i - 1]
            act_prev = p["act"]
            if g["mode"] == "col":  # partial dX over the output shard: all-reduce, then act'
                ops.gemm(g["dz"], g["wbf"], g["dxp"], layout_a=ops.KMAJ, layout_b=ops.MNMAJ,
                         M=self.rows, N=g["k"], K=g["n"])
                self._all_reduce(g["dxp"])
                ops.pack_bf16(g["dxp"], p["dz"])
                ops.dact_colsum(p["dz"], p["y"], act_prev)
            else:  # lands in the previous layer's (shard) layout; act' fused in the epilogue
                ops.linear_dgrad(g["dz"], g["wbf"], p["dz"], y_prev=p["y"], act_prev=act_prev)

    def update(self) -> None:
        o = self.optim
        for g in self.layers:
            ops.sgd_update(g["w"].view(-1), g["gw"].view(-1),
                           g["mw"].view(-1) if g["mw"] is not None else None,
                           g["wbf"].view(-1), lr=o.lr, momentum=o.momentum,
                           weight_decay=o.weight_decay)
            ops.sgd_update(g["b"], g["gb"], g["mb"], None, lr=o.lr, momentum=o.momentum,
                           weight_decay=o.weight_decay)

    def step(self) -> None:
        self.forward()
        self.backward()
        self.update()
        self.steps_done += 1

    # ---- results -------------------------------------------------------------------------------
    def loss(self) -> float:
        return float(self.loss_part.detach().cpu().double().sum()) / self.rows

    def full_weights(self) -> list[tuple[np.ndarray, np.ndarray]]:
        """Unpadded full [out][in] weights and [out] biases of every layer, gathered from
        the shards (a collective: every TP rank calls it)."""
        out = []
        for g in self.layers:
            l = g["spec"]
            w, b = g["w"], g["b"]
            if self.tp > 1 and g["mode"] != "rep":
                ws = [torch.zeros_like(w) for _ in range(self.tp)]
                dist.all_gather(ws, w.contiguous(), group=self.group)
                if g["mode"] == "col":
                    w = torch.cat(ws, 0)
                    bs = [torch.zeros_like(b) for _ in range(self.tp)]
                    dist.all_gather(bs, b.contiguous(), group=self.group)
                    b = torch.cat(bs, 0)
                else:
                    w = torch.cat(ws, 1)
            out.append((w[:l.out_dim, :l.in_dim].cpu().numpy().copy(),
                        b[:l.out_dim].cpu().numpy().copy()))
        return out
