"""One pipeline stage: a contiguous slice of Linear layers resident on one device.

This is the MI355X replacement of the reference's stage worker
(/root/reference/src/grpc_node.py:16-97), which held its layers' fp64 weights and ran
``np.dot(x, W) + b`` + activation per request. A Stage instead owns, for one training step of
``num_micro`` micro-batches of ``micro_batch`` rows:

* parameters in ONE flat fp32 master buffer (padded [Np][Kp] weight + [Np] bias per layer),
  a bf16 shadow of it that the GEMMs read, one flat fp32 gradient buffer (the unit of the DP
  all-reduce) and flat optimizer state -- so the optimizer is a single fused kernel;
* step buffers for every micro-batch (activations, dZ, logits, labels) laid out as
  [num_micro * micro_batch] rows, so micro-batch j is a row slice and the deferred weight
  gradient can run as ONE batch-contraction GEMM over all rows (or per micro-batch);
* split-K wgrad slabs and bias-gradient partials, reduced deterministically (no atomics).

Per layer the compute is three fused gfx950 kernels: forward GEMM with bias+activation
epilogue, dgrad GEMM whose epilogue applies the previous layer's activation derivative (read
from the stored activation -- no mask tensor), and the wgrad GEMM. The last layer of the last
stage writes fp32 logits and runs the fused softmax-cross-entropy kernel.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..models.mlp import LayerGeom, MLPSpec, round_up
from ..utils.native import native
from .. import switches

_ALIGN = 64  # elements; keeps every layer's region 256-B aligned
RELU_MASK_AUTO_WIDTH = 1024  # DNN_RELU_MASK=auto: masks for hidden layers at least this wide


@dataclass
class OptimConfig:
    name: str = "sgd"
    lr: float = 0.05
    momentum: float = 0.0
    weight_decay: float = 0.0
    betas: tuple[float, float] = (0.9, 0.999)
    eps: float = 1e-8
    decoupled: bool = False


class StageParams:
    """Flat parameter / gradient / optimizer buffers of a stage's layers."""

    def __init__(self, geoms: Sequence[LayerGeom], device: torch.device,
                 optim: Optional[OptimConfig] = None, shard: Optional[tuple[int, int]] = None):
        self.geoms = list(geoms)
        self.device = device
        self.optim = optim or OptimConfig()
        # sharded data parallelism (shard = (dp, dp_rank), see shard_piece): every layer's
        # region ends on a multiple of dp * _ALIGN, so any bucket of whole layers splits into
        # dp equal, aligned pieces
        self.sharded = shard is not None
        self.dp, self.dp_rank = shard or (1, 0)
        off = 0
        self.w_off, self.b_off = [], []
        if self.sharded:
            # weights first, each padded to dp pieces; then every bias (replicated update)
            for g in self.geoms:
                self.w_off.append(off)
                off = round_up(off + g.np_ * g.kp, _ALIGN * self.dp)
            self.bias_lo = off
            for g in self.geoms:
                self.b_off.append(off)
                off = round_up(off + g.np_, _ALIGN)
        else:
            for g in self.geoms:
                self.w_off.append(off)
                off = round_up(off + g.np_ * g.kp, _ALIGN)
                self.b_off.append(off)
                off = round_up(off + g.np_, _ALIGN)
        self.numel = off
        self.master = torch.zeros(off, dtype=torch.float32, device=device)
        self.shadow = torch.zeros(off, dtype=torch.bfloat16, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        if self.sharded:
            # bf16 gradient (reduce-scatter input) and the reduced pieces this rank owns: the
            # piece of bucket [e0, e1) lives at [e0 / dp, e1 / dp) of grad_piece
            self.grad16 = torch.zeros(off, dtype=torch.bfloat16, device=device)
            self.grad_piece = torch.zeros(off // self.dp, dtype=torch.bfloat16, device=device)
            self.shard_buckets: list[tuple[int, int]] = []
        self.state: list[torch.Tensor] = []
        self.step_count = 0
        # transposed bf16 weight shadows W^T[Kp][Np] of the layers whose dgrad reads them
        # (enable_wt); refreshed after every update of their layer (refresh_t)
        self.wt: dict[int, torch.Tensor] = {}
        # layers whose weight gradient GEMM applies the SGD step itself (Stage.enable_fused_
        # wgrad_update): the per-step update paths below skip their weights and W^T
        self.fused_layers: set[int] = set()
        self._init_state()

    def _init_state(self):
        o = self.optim
        if o.name == "sgd":
            self.state = [torch.zeros_like(self.master)] if o.momentum else []
        elif o.name in ("adam", "adamw"):
            self.state = [torch.zeros_like(self.master), torch.zeros_like(self.master)]
        else:
            raise ValueError(f"unknown optimizer {o.name!r} (sgd | adam | adamw)")

    # views ------------------------------------------------------------------------------
    def w32(self, i):
        g = self.geoms[i]
        return self.master[self.w_off[i]:self.w_off[i] + g.np_ * g.kp].view(g.np_, g.kp)

    def b32(self, i):
        return self.master[self.b_off[i]:self.b_off[i] + self.geoms[i].np_]

    def wbf(self, i):
        g = self.geoms[i]
        return self.shadow[self.w_off[i]:self.w_off[i] + g.np_ * g.kp].view(g.np_, g.kp)

    def gw(self, i):
        g = self.geoms[i]
        return self.grad[self.w_off[i]:self.w_off[i] + g.np_ * g.kp]

    def gb(self, i):
        return self.grad[self.b_off[i]:self.b_off[i] + self.geoms[i].np_]

    def layer_grad_range(self, i) -> tuple[int, int]:
        """Flat [start, end) of layer i's W and b gradients (a DP all-reduce bucket). Sharded
        layout: layer i's WEIGHTS only (the biases live together at [bias_lo, numel))."""
        if self.sharded:
            return self.w_off[i], (self.w_off[i + 1] if i + 1 < len(self.geoms)
                                   else self.bias_lo)
        end = self.w_off[i + 1] if i + 1 < len(self.geoms) else self.numel
        return self.w_off[i], end

    # weights in/out -----------------------------------------------------------------------
    def load(self, weights: Sequence[np.ndarray], biases: Sequence[np.ndarray]) -> None:
        """Set from unpadded [out][in] weights / [out] biases (any float dtype)."""
        self.master.zero_()
        for i, g in enumerate(self.geoms):
            w = torch.as_tensor(np.asarray(weights[i], dtype=np.float32))
            b = torch.as_tensor(np.asarray(biases[i], dtype=np.float32))
            if tuple(w.shape) != (g.spec.out_dim, g.spec.in_dim):
                raise ValueError(f"layer {g.index}: weight shape {tuple(w.shape)} != "
                                 f"{(g.spec.out_dim, g.spec.in_dim)}")
            self.w32(i)[:g.spec.out_dim, :g.spec.in_dim] = w.to(self.device)
            self.b32(i)[:g.spec.out_dim] = b.to(self.device)
        self.refresh_shadow()

    def init_default(self, seed: int) -> None:
        """nn.Linear default init, U(-1/sqrt(in), 1/sqrt(in)); seeded by GLOBAL layer index so
        any stage split of the same model starts from identical weights."""
        ws, bs = [], []
        for g in self.geoms:
            gen = torch.Generator().manual_seed(seed * 7919 + g.index)
            bound = 1.0 / math.sqrt(g.spec.in_dim)
            ws.append((torch.rand(g.spec.out_dim, g.spec.in_dim, generator=gen) * 2 - 1) * bound)
            bs.append((torch.rand(g.spec.out_dim, generator=gen) * 2 - 1) * bound)
        self.load([w.numpy() for w in ws], [b.numpy() for b in bs])

    def refresh_shadow(self) -> None:
        self.shadow.copy_(self.master.to(torch.bfloat16))
        self.refresh_t()

    def enable_wt(self, i: int) -> None:
        g = self.geoms[i]
        if i not in self.wt:
            self.wt[i] = torch.zeros(g.kp, g.np_, dtype=torch.bfloat16, device=self.device)
            ops.transpose_bf16(self.wbf(i), self.wt[i])

    def refresh_t(self, a: int = 0, b: Optional[int] = None, step: bool = False,
                  skip: frozenset = frozenset()) -> None:
        """Re-derive W^T of the local layers [a, b) that keep one (after their update).
        ``step``: a per-step update -- layers updated by their wgrad epilogue (which writes
        W^T itself) are skipped; so are the ``skip`` layers (W^T written by the update)."""
        b = len(self.geoms) if b is None else b
        ops.transpose_multi([(self.wbf(i), self.wt[i]) for i in range(a, b) if i in self.wt and
                             i not in skip and not (step and i in self.fused_layers)])

    def _layers_of(self, e0: int, e1: int) -> tuple[int, int]:
        """Local layers whose parameters lie in the flat element range [e0, e1)."""
        ls = [i for i in range(len(self.geoms)) if self.w_off[i] < e1 and
              self.b_off[i] + self.geoms[i].np_ > e0]
        return (ls[0], ls[-1] + 1) if ls else (0, 0)

    def _export_flat(self, buf: torch.Tensor) -> tuple[list[np.ndarray], list[np.ndarray]]:
        ws, bs = [], []
        for i, g in enumerate(self.geoms):
            w = buf[self.w_off[i]:self.w_off[i] + g.np_ * g.kp].view(g.np_, g.kp)
            ws.append(w[:g.spec.out_dim, :g.spec.in_dim].detach().cpu().numpy().copy())
            bs.append(buf[self.b_off[i]:self.b_off[i] + g.spec.out_dim]
                      .detach().cpu().numpy().copy())
        return ws, bs

    def export(self) -> tuple[list[np.ndarray], list[np.ndarray]]:
        return self._export_flat(self.master)

    def export_state(self, k: int) -> tuple[list[np.ndarray], list[np.ndarray]]:
        """Unpadded per-layer view of optimizer state buffer k (momentum / Adam m, v)."""
        return self._export_flat(self.state[k])

    def load_state(self, k: int, weights: Sequence[np.ndarray],
                   biases: Sequence[np.ndarray]) -> None:
        """Set optimizer state buffer k from unpadded per-layer arrays (padding stays 0)."""
        buf = self.state[k]
        buf.zero_()
        for i, g in enumerate(self.geoms):
            w = torch.as_tensor(np.asarray(weights[i], dtype=np.float32))
            b = torch.as_tensor(np.asarray(biases[i], dtype=np.float32))
            if tuple(w.shape) != (g.spec.out_dim, g.spec.in_dim):
                raise ValueError(f"layer {g.index}: state shape {tuple(w.shape)} != "
                                 f"{(g.spec.out_dim, g.spec.in_dim)}")
            view = buf[self.w_off[i]:self.w_off[i] + g.np_ * g.kp].view(g.np_, g.kp)
            view[:g.spec.out_dim, :g.spec.in_dim] = w.to(self.device)
            buf[self.b_off[i]:self.b_off[i] + g.spec.out_dim] = b.to(self.device)

    # optimizer ----------------------------------------------------------------------------
    def _device_scalars(self) -> None:
        if getattr(self, "lr_dev", None) is None:
            self.lr_dev = torch.full((1,), float(self.optim.lr), dtype=torch.float32,
                                     device=self.device)
            self.step_dev = torch.full((1,), int(self.step_count), dtype=torch.int32,
                                       device=self.device)
            self._lr_cur = float(self.optim.lr)

    def set_lr(self, lr: float) -> None:
        """Learning rate of the device-scalar (recorded) update path."""
        self._device_scalars()
        if float(lr) != self._lr_cur:
            self.lr_dev.fill_(float(lr))
            self._lr_cur = float(lr)

    def set_step(self, n: int) -> None:
        """Number of updates done (checkpoint resume): host counter and device counter."""
        self.step_count = int(n)
        if getattr(self, "step_dev", None) is not None:
            self.step_dev.fill_(int(n))

    def _unfused_ranges(self) -> list[tuple[int, int]]:
        """[0, numel) minus the weight regions of fused_layers (updated by their wgrad)."""
        cuts = sorted((self.w_off[i], self.w_off[i] + self.geoms[i].np_ * self.geoms[i].kp)
                      for i in self.fused_layers)
        out, lo = [], 0
        for a, b in cuts:
            if a > lo:
                out.append((lo, a))
            lo = b
        if lo < self.numel:
            out.append((lo, self.numel))
        return out

    def record_update(self) -> None:
        """The launches of one optimizer update reading lr / step from device memory (for
        recording into a native Program: no per-step host values)."""
        self._device_scalars()
        o = self.optim
        if self.fused_layers:  # SGD only (Stage.enable_fused_wgrad_update)
            for a, b in self._unfused_ranges():
                sl = slice(a, b)
                ops.sgd_update(self.master[sl], self.grad[sl],
                               self.state[0][sl] if self.state else None, self.shadow[sl],
                               lr=o.lr, momentum=o.momentum, weight_decay=o.weight_decay,
                               lr_dev=self.lr_dev)
            self.refresh_t(step=True)
            return
        if o.name == "sgd":
            ops.sgd_update(self.master, self.grad, self.state[0] if self.state else None,
                           self.shadow, lr=o.lr, momentum=o.momentum,
                           weight_decay=o.weight_decay, lr_dev=self.lr_dev)
        else:
            ops.adam_update(self.master, self.grad, self.state[0], self.state[1], self.shadow,
                            lr=o.lr, betas=o.betas, eps=o.eps, weight_decay=o.weight_decay,
                            decoupled=o.decoupled or o.name == "adamw", lr_dev=self.lr_dev,
                            step_dev=self.step_dev)
            ops.step_advance(self.step_dev)
        self.refresh_t(step=True)

    def record_update_range(self, a: int, b: int, advance: bool, refresh: bool = True) -> None:
        """record_update over the flat element range [a, b) only (a DP bucket of whole layers);
        the device step counter advances only when ``advance`` (once per step: the last range
        of a split update). ``refresh=False``: leave W^T alone (a shard piece, whose layers are
        complete only after the all-gather)."""
        self._device_scalars()
        o = self.optim
        sl = slice(a, b)
        if o.name == "sgd":
            ops.sgd_update(self.master[sl], self.grad[sl], self.state[0][sl] if self.state else None,
                           self.shadow[sl], lr=o.lr, momentum=o.momentum,
                           weight_decay=o.weight_decay, lr_dev=self.lr_dev)
        else:
            ops.adam_update(self.master[sl], self.grad[sl], self.state[0][sl], self.state[1][sl],
                            self.shadow[sl], lr=o.lr, betas=o.betas, eps=o.eps,
                            weight_decay=o.weight_decay,
                            decoupled=o.decoupled or o.name == "adamw", lr_dev=self.lr_dev,
                            step_dev=self.step_dev)
        if advance and o.name != "sgd":
            ops.step_advance(self.step_dev)
        if refresh:
            self.refresh_t(*self._layers_of(a, b))

    # sharded data parallelism --------------------------------------------------------------
    # Per bucket [e0, e1) of whole layers' WEIGHTS: the fp32 gradient is cast to bf16
    # (shard_pack), reduce-scattered over the DP group (rank r receives the sum of piece r),
    # cast back into grad[piece] (shard_unpack) and only that piece is updated (fp32 master +
    # optimizer state of the piece are authoritative on this rank); the bf16 shadow is then
    # all-gathered and W^T refreshed. The biases (fp32 in the GEMM epilogues, a few KB) are
    # all-reduced in fp32 and updated on every rank. Bytes on the wire: 2 x (dp-1)/dp x 2 B per
    # weight, half of an fp32 all-reduce, and the optimizer touches 1/dp of the weights.
    def shard_piece(self, e0: int, e1: int) -> tuple[int, int]:
        c = (e1 - e0) // self.dp
        if c * self.dp != e1 - e0:
            raise ValueError("bucket length is not a multiple of the DP degree")
        return e0 + self.dp_rank * c, e0 + (self.dp_rank + 1) * c

    def shard_pack(self, e0: int, e1: int) -> None:
        ops.pack_bf16(self.grad[e0:e1].view(1, -1), self.grad16[e0:e1].view(1, -1))

    def shard_unpack(self, e0: int, e1: int) -> None:
        p0, p1 = self.shard_piece(e0, e1)
        d = self.dp
        ops.unpack_bf16(self.grad_piece[e0 // d:e1 // d].view(1, -1),
                        self.grad[p0:p1].view(1, -1))

    def gather_full(self, group) -> None:
        """All-gather the fp32 master and optimizer state over the DP group: afterwards every
        rank holds the whole (checkpoint / export); a no-op without sharding."""
        if not self.sharded or not self.shard_buckets:
            return
        import torch.distributed as dist

        for buf in [self.master] + list(self.state):
            for e0, e1 in self.shard_buckets:
                p0, p1 = self.shard_piece(e0, e1)
                dist.all_gather_into_tensor(buf[e0:e1], buf[p0:p1].clone(), group=group)

    def update_range(self, a: int, b: int, lr: Optional[float], advance: bool,
                     refresh: bool = True) -> None:
        """Optimizer update of the flat range [a, b) (see record_update_range); the host step
        counter counts whole steps (advance=True)."""
        o = self.optim
        lr = o.lr if lr is None else lr
        if self.device.type == "cuda":
            self.set_lr(lr)
            self.record_update_range(a, b, advance, refresh)
        else:
            sl = slice(a, b)
            step = self.step_count + 1
            if o.name == "sgd":
                ops.sgd_update(self.master[sl], self.grad[sl],
                               self.state[0][sl] if self.state else None, self.shadow[sl],
                               lr=lr, momentum=o.momentum, weight_decay=o.weight_decay)
            else:
                ops.adam_update(self.master[sl], self.grad[sl], self.state[0][sl],
                                self.state[1][sl], self.shadow[sl], lr=lr, betas=o.betas,
                                eps=o.eps, weight_decay=o.weight_decay,
                                decoupled=o.decoupled or o.name == "adamw", step=step)
            if refresh:
                self.refresh_t(*self._layers_of(a, b))
        if advance:
            self.step_count += 1

    def layers_range(self, a: int, b: int) -> tuple[int, int]:
        """Flat [start, end) of layers a..b-1 (weights, biases and alignment padding)."""
        if self.sharded:
            raise ValueError("sharded layout: layer ranges are not contiguous")
        return self.w_off[a], (self.w_off[b] if b < len(self.geoms) else self.numel)

    def optimizer_step(self, lr: Optional[float] = None) -> None:
        o = self.optim
        lr = o.lr if lr is None else lr
        if self.device.type == "cuda":
            # GPU: lr and step always come from device memory, so the same launches are valid
            # eagerly, recorded into a native Program, or captured in a HIP graph (by-value
            # Adam bias corrections would be frozen by a capture)
            self.set_lr(lr)
            self.record_update()
            self.step_count += 1
            return
        self.step_count += 1
        if o.name == "sgd":
            ops.sgd_update(self.master, self.grad, self.state[0] if self.state else None,
                           self.shadow, lr=lr, momentum=o.momentum, weight_decay=o.weight_decay)
        else:
            ops.adam_update(self.master, self.grad, self.state[0], self.state[1], self.shadow,
                            lr=lr, betas=o.betas, eps=o.eps, weight_decay=o.weight_decay,
                            decoupled=o.decoupled or o.name == "adamw", step=self.step_count)
        self.refresh_t(step=True)


class Stage:
    """Compute of one pipeline stage for one step (see module doc)."""

    def __init__(self, spec: MLPSpec, layer_start: int, layer_end: int, *, micro_batch: int,
                 num_micro: int, device: torch.device, global_batch: Optional[int] = None,
                 optim: Optional[OptimConfig] = None, wgrad: str = "batched",
                 stage_index: int = 0, num_stages: int = 1, wgrad_algo: Optional[str] = None,
                 dp_shard: Optional[tuple[int, int]] = None):
        if not 0 <= layer_start < layer_end <= len(spec.layers):
            raise ValueError("bad layer range")
        if micro_batch <= 0 or micro_batch % 64:
            raise ValueError("micro_batch must be a positive multiple of 64 (MFMA row tiles); "
                             "pad the batch with label -1 rows")
        self.spec = spec
        self.l0, self.l1 = layer_start, layer_end
        self.first = layer_start == 0
        self.last = layer_end == len(spec.layers)
        self.stage_index, self.num_stages = stage_index, num_stages
        self.mb, self.nm = micro_batch, num_micro
        self.rows = micro_batch * num_micro
        self.device = device
        self.global_batch = global_batch or self.rows
        self.wgrad_mode = wgrad
        self.wgrad_algo = wgrad_algo or switches.get("DNN_WGRAD_ALGO")
        if self.wgrad_algo not in ("streamk", "splitk"):
            raise ValueError(f"wgrad_algo must be streamk | splitk, got {self.wgrad_algo!r}")
        self.geoms = [LayerGeom(i, spec.layers[i]) for i in range(layer_start, layer_end)]
        self.params = StageParams(self.geoms, device, optim, shard=dp_shard)
        self.prev_act = spec.layers[layer_start - 1].activation if not self.first else "linear"
        self.n_cls = spec.out_dim
        self._alloc()

    # -------------------------------------------------------------------------------------
    def _alloc(self):
        R, dev = self.rows, self.device
        bf, f32 = torch.bfloat16, torch.float32
        g0 = self.geoms[0]
        self.x_buf = torch.zeros(R, g0.kp, dtype=bf, device=dev)
        self.x_in = self.x_buf  # may be re-pointed at a resident dataset slice (zero-copy)
        # the last layer's softmax-CE is fused into its GEMM epilogue when the padded class
        # count is one 64/128-wide tile: logits then never exist in memory
        gl = self.geoms[-1]
        self.fused_xent = (self.last and gl.np_ in (64, 128) and
                           switches.get("DNN_FUSED_XENT") == "1")
        self.acts: list[torch.Tensor] = []  # output of local layer i
        for i, g in enumerate(self.geoms):
            is_logits = self.last and i == len(self.geoms) - 1
            if is_logits and self.fused_xent:
                self.acts.append(torch.empty(0, g.np_, dtype=f32, device=dev))
            else:
                self.acts.append(torch.zeros(R, g.np_, dtype=f32 if is_logits else bf,
                                             device=dev))
        # 1-bit ReLU masks of the hidden outputs consumed by this stage's own dgrads (GPU,
        # DNN_RELU_MASK=1; off by default: measured 0.380 vs 0.371 ms on the headline step,
        # the byte-granular mask stores/loads cost more than the activation bytes saved):
        # the dgrad epilogue then reads N/8 bytes per row instead of the bf16 activation (the
        # activation itself is still kept: it is the next layer's wgrad operand)
        # DNN_RELU_MASK=2: fragment-order masks (ops.FragMask: one 16-byte access per lane), only
        # where a GEMM dgrad of this stage consumes them and it runs the forward's tile shape
        self.tail = self._tail_ok()
        mask_mode = switches.get("DNN_RELU_MASK") if dev.type == "cuda" else "0"
        L = len(self.geoms)
        self.relu_mask = []
        for i, g in enumerate(self.geoms):
            m = None
            # auto: fragment-order masks for layers >= 1024 wide, where the dgrad's activation
            # read is the big term (wide 5.81 -> 5.44 ms, mlp8 2.73 -> 2.71; the headline's
            # 512-wide layer 0 loses: profiles/r5_tables/relu_mask_*)
            mode_i = ("2" if g.np_ >= RELU_MASK_AUTO_WIDTH else "0") if mask_mode == "auto" \
                else mask_mode
            if mode_i == "1" and i < L - 1 and g.spec.activation == "relu":
                m = torch.zeros(R, g.np_ // 8, dtype=torch.uint8, device=dev)
            elif mode_i == "2" and i < L - 1 and g.spec.activation == "relu" and \
                    not (self.tail and i + 1 >= L - 2):
                tiles = ops.frag_mask_tiles(self.mb, g.np_, g.kp, self.geoms[i + 1].np_)
                if tiles is not None:
                    m = ops.FragMask.alloc(R, g.np_, tiles, dev)
            self.relu_mask.append(m)
        self.dz = [torch.zeros(R, g.np_, dtype=bf, device=dev) for g in self.geoms]
        self.dx_send = None if self.first else torch.zeros(R, g0.kp, dtype=bf, device=dev)
        self.labels = torch.full((R,), -1, dtype=torch.int32, device=dev) if self.last else None
        self.labels_buf = self.labels  # owned buffer; ``labels`` may alias a dataset slice
        # Narrow classifier tail (csrc/kernels/mlp_tail.hip): the forward of the last two
        # layers, the softmax CE and both of their dgrads run as ONE kernel inside the last
        # layer's forward; the second-to-last layer's forward and both dgrads are then no-ops.
        # K-major weight gradients (ops.linear_wgrad dzt / xt): for big hidden layers whose dZ
        # and input activation come from this stage's own one-tile GEMMs, those GEMMs also write
        # the transposed copies in their epilogues (+1 write of each, -20 % wgrad time)
        self.dzT: dict[int, torch.Tensor] = {}
        self.actT: dict[int, torch.Tensor] = {}
        kk = switches.get("DNN_WGRAD_KK")
        if dev.type == "cuda" and self.wgrad_mode == "batched" and kk != "0":
            L = len(self.geoms)
            for i in range(1, L):
                g = self.geoms[i]
                big = kk == "1" or g.np_ * g.kp >= (1 << 24)
                dz_by_dgrad = i + 1 < L and not (self.tail and i + 1 >= L - 2) and \
                    self.relu_mask[i] is None
                x_by_fwd = not (self.tail and i - 1 >= L - 2) and self.relu_mask[i - 1] is None
                if big and dz_by_dgrad and x_by_fwd:
                    self.dzT[i] = torch.zeros(g.np_, R, dtype=bf, device=dev)
                    self.actT[i - 1] = torch.zeros(g.kp, R, dtype=bf, device=dev)
        # dgrad GEMMs read W^T (contraction-contiguous B operand, see ops.linear_dgrad)
        if dev.type == "cuda" and switches.get("DNN_DGRAD_WT") == "1":
            L = len(self.geoms)
            for i in range(L):
                if (i > 0 or not self.first) and not (self.tail and i >= L - 2):
                    self.params.enable_wt(i)
        if self.tail:
            self.xent_per_micro = ops.tail_blocks(self.mb)
        else:
            self.xent_per_micro = (self.mb // ops.xent_tiles(self.mb, gl.np_)[0]
                                   if self.fused_xent else ops.xent_blocks(self.mb))
        self.loss_part = torch.zeros(self.xent_per_micro * self.nm, dtype=f32, device=dev)
        # per-block correct counts, written (not accumulated) by the loss kernels
        self.correct = torch.zeros(self.xent_per_micro * self.nm, dtype=torch.int32, device=dev)
        # wgrad geometry: batched = one GEMM over all rows; per_micro = one per micro-batch
        wrows = R if self.wgrad_mode == "batched" else self.mb
        if self.wgrad_algo == "streamk":  # balanced stream-K, reduced straight into the grads
            self.w_splits = [1] * len(self.geoms)
            self.slabs = []
            n = max(ops.streamk_partial_elems(g.np_, g.kp) for g in self.geoms)
            self.sk_part = torch.zeros(n, dtype=f32, device=dev)
        else:  # classic split-K slabs + reduce
            self.w_splits = [ops.pick_splits(g.np_, g.kp, wrows) for g in self.geoms]
            self.slabs = [torch.zeros(s, g.np_, g.kp, dtype=f32, device=dev)
                          for s, g in zip(self.w_splits, self.geoms)]
        # Bias-gradient partials (column sums of dZ) come fused from whichever kernel produces
        # dZ: the dgrad epilogue of the next local layer (one partial per output row tile), the
        # softmax-CE kernel (one per 64-row block), or -- for a gradient received from the next
        # stage -- a colsum kernel. self.bp[i] = partials per micro-batch.
        self.bp = []
        L = len(self.geoms)
        for i in range(L):
            if i < L - 1:
                g1 = self.geoms[i + 1]
                self.bp.append(self.mb // ops.dgrad_tiles(self.mb, g1.kp, g1.np_)[0])
            elif self.last:
                self.bp.append(self.xent_per_micro)
            else:
                # one partial per 128 rows: enough workgroups to fill the chip (1024-row
                # partitions left a 4096-row boundary colsum at 32 workgroups, 12 us)
                self.bp.append(max(1, self.mb // 128))
        if self.tail:  # dz of the last three local layers come from the tail kernel
            for i in range(L - 3, L):
                self.bp[i] = self.xent_per_micro
        self.bpart = [torch.zeros(self.bp[i] * self.nm, g.np_, dtype=f32, device=dev)
                      for i, g in enumerate(self.geoms)]
        self._w_done = 0
        self._reduce_jobs: dict = {}
        self._colsum_by = None  # loopback: the next stage computes our boundary colsum
        self._colsum_for = None  # ... and this is the stage we compute it for
        self._prog = None  # native Program once compile_native() ran
        self._recording = False
        self._has_w = False
        self._o_native = False  # "O" recorded (device-side lr / step)
        self._rx = self._rl = None
        self.boundary = "bf16"
        self._fp8_next = self._fp8_prev = False

    def _tail_ok(self) -> bool:
        if not (self.fused_xent and self.device.type == "cuda" and len(self.geoms) >= 3 and
                switches.get("DNN_TAIL") == "1"):
            return False
        g2, g3, g4 = self.geoms[-3], self.geoms[-2], self.geoms[-1]
        acts = ("relu", "sigmoid", "linear")
        return (ops.tail_supported(g3.kp, g3.np_, g4.np_, self.n_cls) and
                g3.spec.activation in acts and g2.spec.activation in acts and
                self.mb % 16 == 0)

    # ---- fp8 pipeline boundary (opt-in: Trainer(boundary="fp8")) -------------------------
    def enable_fp8_boundary(self, has_prev: bool, has_next: bool) -> None:
        """Hops to/from neighbouring stages carry OCP e4m3 rows + one fp32 scale per row
        (ops.quant_rows_fp8): half the bytes of bf16 on the xGMI link, for activations forward
        and gradients backward. Buffers are step-sized like the bf16 ones."""
        R, dev, u8 = self.rows, self.device, torch.uint8
        self.boundary = "fp8"
        if has_next:
            w = self.output.shape[1]
            self.q_out, self.s_out = torch.zeros(R, w, dtype=u8, device=dev), \
                torch.zeros(R, device=dev)
            self.q_gin, self.s_gin = torch.zeros(R, w, dtype=u8, device=dev), \
                torch.zeros(R, device=dev)
        if has_prev:
            w = self.x_buf.shape[1]
            self.q_in, self.s_in = torch.zeros(R, w, dtype=u8, device=dev), \
                torch.zeros(R, device=dev)
            self.q_dx, self.s_dx = torch.zeros(R, w, dtype=u8, device=dev), \
                torch.zeros(R, device=dev)
        self._fp8_next, self._fp8_prev = has_next, has_prev

    def pack_fwd(self, j: int) -> None:
        if self._prog is not None and not self._recording:
            return self._replay(f"QF{j}")
        r = self.rows_of(j)
        ops.quant_rows_fp8(self.output[r], self.q_out[r], self.s_out[r])

    def unpack_fwd(self, j: int) -> None:
        if self._prog is not None and not self._recording:
            return self._replay(f"DQF{j}")
        r = self.rows_of(j)
        ops.dequant_rows_fp8(self.q_in[r], self.s_in[r], self.x_in[r])

    def pack_bwd(self, j: int) -> None:
        if self._prog is not None and not self._recording:
            return self._replay(f"QB{j}")
        r = self.rows_of(j)
        ops.quant_rows_fp8(self.dx_send[r], self.q_dx[r], self.s_dx[r])

    def unpack_bwd(self, j: int) -> None:
        if self._prog is not None and not self._recording:
            return self._replay(f"DQB{j}")
        r = self.rows_of(j)
        ops.dequant_rows_fp8(self.q_gin[r], self.s_gin[r], self.grad_out[r])

    def rows_of(self, j: int) -> slice:
        if not 0 <= j < self.nm:
            raise IndexError(f"micro-batch {j} out of range [0, {self.nm})")
        return slice(j * self.mb, (j + 1) * self.mb)

    def input_of(self, i: int) -> torch.Tensor:
        return self.x_in if i == 0 else self.acts[i - 1]

    @property
    def output(self) -> torch.Tensor:
        """Activation sent to the next stage (bf16 [rows][Np])."""
        return self.acts[-1]

    @property
    def grad_out(self) -> torch.Tensor:
        """dZ of this stage's last layer, written by the next stage (received gradient)."""
        return self.dz[-1]

    # -------------------------------------------------------------------------------------
    def begin_step(self) -> None:
        self._w_done = 0

    def forward(self, j: int) -> None:
        if self._prog is not None and not self._recording:
            return self._replay(f"F{j}")
        for i in range(len(self.geoms)):
            self._forward_layer(j, i)

    def forward_layers(self, j: int, i0: int, i1: int) -> None:
        """Forward of micro-batch j through local layers [i0, i1) only (a DP step whose
        update of later layers is deferred runs the earlier layers first)."""
        if self._prog is not None and not self._recording:
            self._prog.run([f"F{j}.L{i}" for i in range(i0, i1)],
                           torch.cuda.current_stream(self.device).cuda_stream)
            return
        for i in range(i0, i1):
            self._forward_layer(j, i)

    def _forward_layer(self, j: int, i: int) -> None:
        r = self.rows_of(j)
        p = self.params
        g = self.geoms[i]
        x = self.input_of(i)[r]
        y = self.acts[i][r]
        L = len(self.geoms)
        if self.tail and i == L - 2:
            return  # computed by the tail kernel at i == L - 1
        if self.tail and i == L - 1:
            k = j * self.xent_per_micro
            ops.mlp_tail(self.acts[L - 3][r], p.wbf(L - 2), p.b32(L - 2), p.wbf(L - 1),
                         p.b32(L - 1), self.labels[r], self.acts[L - 2][r], self.dz[L - 1][r],
                         self.dz[L - 2][r], self.dz[L - 3][r], self.n_cls,
                         1.0 / self.global_batch, act3=self.geoms[L - 2].spec.activation,
                         act2=self.geoms[L - 3].spec.activation,
                         loss_part=self.loss_part[k:k + self.xent_per_micro],
                         correct=self.correct[k:k + self.xent_per_micro],
                         cs4=self._bpart(L - 1, j), cs3=self._bpart(L - 2, j),
                         cs2=self._bpart(L - 3, j))
        elif self.last and i == len(self.geoms) - 1 and self.fused_xent:
            k = j * self.xent_per_micro
            ops.linear_fwd_xent(x, p.wbf(i), p.b32(i), self.dz[i][r], self.labels[r],
                                self.n_cls, 1.0 / self.global_batch,
                                self.loss_part[k:k + self.xent_per_micro],
                                self.correct[k:k + self.xent_per_micro],
                                colsum=self._bpart(i, j))
        elif self.last and i == len(self.geoms) - 1:
            ops.linear_fwd(x, p.wbf(i), p.b32(i), y, act="linear")  # fp32 logits
            k = j * self.xent_per_micro
            ops.softmax_xent(y, self.labels[r], self.dz[i][r], self.n_cls,
                             1.0 / self.global_batch,
                             self.loss_part[k:k + self.xent_per_micro],
                             self.correct[k:k + self.xent_per_micro],
                             colsum=self._bpart(i, j))
        else:
            m = self.relu_mask[i]
            ops.linear_fwd(x, p.wbf(i), p.b32(i), y, act=g.spec.activation,
                           mask=None if m is None else m[r],
                           yt=self.actT[i][:, r] if i in self.actT else None)

    def backward(self, j: int) -> None:
        """dgrad chain of micro-batch j; dZ of the last local layer must already be present."""
        if self._prog is not None and not self._recording:
            return self._replay(f"B{j}")
        self._backward_pre(j)
        for i in range(len(self.geoms) - 1, -1, -1):
            self._backward_layer(j, i)

    def _backward_pre(self, j: int) -> None:
        if not self.last and self._colsum_by is None:  # dZ of our last layer arrived from
            L = len(self.geoms) - 1                       # the next stage
            ops.colsum_partial(self.dz[L][self.rows_of(j)], self._bpart(L, j), self.bp[L])

    def _backward_layer(self, j: int, i: int) -> None:
        """dgrad of local layer i for micro-batch j: dZ of layer i -> dZ of layer i-1 (or the
        gradient sent to the previous stage when i == 0)."""
        if self.tail and i >= len(self.geoms) - 2:
            return  # both dgrads ran inside the tail kernel (forward of micro-batch j)
        r = self.rows_of(j)
        p = self.params
        if i > 0:
            prev = self.geoms[i - 1].spec.activation
            m = self.relu_mask[i - 1]
            ops.linear_dgrad(self.dz[i][r], p.wbf(i), self.dz[i - 1][r],
                             y_prev=self.acts[i - 1][r], act_prev=prev,
                             colsum=self._bpart(i - 1, j),
                             mask_prev=None if m is None else m[r], wt=p.wt.get(i),
                             dxt=self.dzT[i - 1][:, r] if (i - 1) in self.dzT else None)
        elif not self.first:
            # gradient for the previous stage, already multiplied by the derivative of its
            # last layer's activation (its output is our input x_in)
            up = self._colsum_for
            ops.linear_dgrad(self.dz[0][r], p.wbf(0), self.dx_send[r], y_prev=self.x_in[r],
                             act_prev=self.prev_act,
                             colsum=None if up is None else up._bpart(len(up.geoms) - 1, j),
                             wt=p.wt.get(0))

    def wgrad(self, j: int = -1) -> None:
        """Weight/bias gradients for micro-batch j (slab-accumulated) or all rows (j = -1)."""
        if j < 0 and self._prog is not None and not self._recording and self._has_w:
            self._replay("W")
            self._w_done += 1
            return
        self._wgrad_all(j)
        self._w_done += 1

    def _wgrad_all(self, j: int = -1) -> None:
        """Every local layer's weight gradient: one grouped launch per shared tile configuration
        (ops.linear_wgrad_group; DNN_WGRAD_GROUP=0 disables), one launch per remaining layer."""
        if (self.wgrad_algo == "splitk" and self.device.type == "cuda" and
                switches.get("DNN_WGRAD_GROUP") == "1" and len(self.geoms) > 1):
            if j < 0:
                r, acc = slice(0, self.rows), False
            else:
                r, acc = self.rows_of(j), self._w_done > 0
            if j < 0 or self.wgrad_mode != "batched":
                fused = self.params.fused_layers
                idx = [i for i in range(len(self.geoms)) if i not in fused]
                items = [(self.dz[i][r], self.input_of(i)[r], self.slabs[i], self.w_splits[i],
                          acc) for i in idx]
                for k in ops.linear_wgrad_group(items):
                    self.wgrad_layer(idx[k], j)
                for i in sorted(fused):
                    self.wgrad_layer(i, j)
                return
        for i in range(len(self.geoms)):
            self.wgrad_layer(i, j)

    def _bpart(self, i: int, j: int) -> torch.Tensor:
        return self.bpart[i][j * self.bp[i]:(j + 1) * self.bp[i]]

    def wgrad_layer(self, i: int, j: int = -1) -> None:
        """Weight gradient GEMM of local layer i (bias partials were produced with dZ)."""
        if j < 0 and self._prog is not None and not self._recording and self._has_w:
            return self._replay(f"W{i}")
        if j < 0:
            r, accumulate = slice(0, self.rows), False
        else:
            if self.wgrad_mode == "batched":
                raise RuntimeError("per-micro wgrad on a stage built with wgrad='batched'")
            r, accumulate = self.rows_of(j), self._w_done > 0
        if self.wgrad_algo == "streamk":
            g = self.geoms[i]
            ops.linear_wgrad_streamk(self.dz[i][r], self.input_of(i)[r],
                                     self.params.gw(i).view(g.np_, g.kp), self.sk_part,
                                     accumulate=accumulate)
        else:
            kk = j < 0 and i in self.dzT
            upd = wt = None
            p = self.params
            if i in p.fused_layers:  # the epilogue applies SGD to W_i and writes W_i^T
                if j >= 0:
                    raise RuntimeError("fused weight update runs on the batched wgrad only")
                p._device_scalars()
                g, o = self.geoms[i], p.optim
                w0, w1 = p.w_off[i], p.w_off[i] + g.np_ * g.kp
                upd = dict(master=p.w32(i), shadow=p.wbf(i), lr_dev=p.lr_dev,
                           mom=p.state[0][w0:w1].view(g.np_, g.kp) if p.state else None,
                           momentum=o.momentum, weight_decay=o.weight_decay)
                wt = p.wt.get(i)
            ops.linear_wgrad(self.dz[i][r], self.input_of(i)[r], self.slabs[i],
                             splits=self.w_splits[i], accumulate=accumulate,
                             dzt=self.dzT[i] if kk else None,
                             xt=self.actT[i - 1] if kk else None, upd=upd, wt=wt)

    def finalize_grads(self, layers: Optional[Sequence[int]] = None) -> None:
        """Reduce bias partials (and, for split-K, weight slabs) into the flat gradient."""
        if self._prog is not None and not self._recording:
            if layers is None:
                return self._replay("FIN")
            ls = list(layers)
            if len(ls) == 1:
                return self._replay(f"FIN{ls[0]}")
            if ls == list(range(ls[0], ls[-1] + 1)):
                return self._replay(f"FIN{ls[0]}-{ls[-1]}")
        key = tuple(range(len(self.geoms))) if layers is None else tuple(layers)
        ops.reduce_multi(self._jobs(key))  # one launch for every slab set and bias-partial set

    # W^T written by the fused update for layers up to this many weights: its transposed
    # stores are 2-byte scatters, cheaper than a transpose launch for the headline's 256x512
    # (step 0.3724 -> 0.3678 ms) but not measurably for mlp8's 1024x1024 layers (3.318 vs
    # 3.329 ms), which keep the coalesced LDS transpose (profiles/r2_sched/fin_wt_*)
    WT_BY_UPDATE_MAX = 1 << 19

    def _wt_by_update_layers(self) -> list:
        p = self.params
        if self.wgrad_algo == "streamk":
            return []
        return [i for i in p.wt if i not in p.fused_layers and
                self.geoms[i].np_ * self.geoms[i].kp <= self.WT_BY_UPDATE_MAX]

    def _jobs(self, key: tuple, with_wt: bool = False) -> list:
        """reduce_multi job table of the layers in ``key`` (buffers are fixed for the stage's
        lifetime: built once). ``with_wt`` (fused update only): the weight jobs of layers that
        keep a W^T shadow also write it (no transpose launch after the update)."""
        jobs = self._reduce_jobs.get((key, with_wt))
        if jobs is None:
            p = self.params
            jobs = []
            for i in key:
                g = self.geoms[i]
                n = g.np_ * g.kp
                if self.wgrad_algo != "streamk" and i not in p.fused_layers:
                    jobs.append((self.slabs[i], self.w_splits[i], n, n, p.gw(i), 1.0, False,
                                 p.wt[i] if with_wt and i in self._wt_by_update_layers()
                                 else None))
                jobs.append((self.bpart[i], self.bpart[i].shape[0], g.np_, g.np_, p.gb(i), 1.0,
                             False))
            self._reduce_jobs[(key, with_wt)] = jobs
        return jobs

    def fused_fin_sgd_ok(self) -> bool:
        """FIN + optimizer step as one launch: every gradient element must come out of a reduce
        job (not stream-K wgrad, which writes weight gradients directly); SGD, Adam or AdamW."""
        return (self.params.optim.name in ("sgd", "adam", "adamw") and
                self.wgrad_algo != "streamk" and self.device.type == "cuda" and
                switches.get("DNN_FUSE_FIN_SGD") == "1")

    def _record_fin_sgd(self, a: int = 0, b: Optional[int] = None) -> None:
        """Record the gradient reduction of local layers [a, b) (default: all) with the SGD
        update fused in (segment FINO, or FINO{a}-{b-1} for a layer range: SGD only, so the
        step counter needs no advance; lr from device memory like record_update)."""
        p = self.params
        p._device_scalars()
        o = p.optim
        L = len(self.geoms)
        b = L if b is None else b
        wt_fused = switches.get("DNN_FIN_WT") == "1" and p.shadow is not None
        jobs = self._jobs(tuple(range(a, b)), with_wt=wt_fused)
        # layers whose W^T comes out of the update launch itself (no transpose launch after it)
        skip = frozenset(i for i in self._wt_by_update_layers()) if wt_fused else frozenset()
        if o.name == "sgd":
            ops.reduce_multi(jobs, sgd=dict(grad=p.grad, master=p.master,
                                            mom=p.state[0] if p.state else None,
                                            shadow=p.shadow, lr=o.lr, momentum=o.momentum,
                                            weight_decay=o.weight_decay, lr_dev=p.lr_dev))
            p.refresh_t(a, b, step=True, skip=skip)
            return
        if (a, b) != (0, L):
            raise ValueError("layer-range fused updates are SGD only")
        ops.reduce_multi(jobs, sgd=dict(grad=p.grad, master=p.master, mom=p.state[0],
                                        v=p.state[1], shadow=p.shadow, lr=o.lr,
                                        weight_decay=o.weight_decay, lr_dev=p.lr_dev,
                                        adam=True, betas=o.betas, eps=o.eps,
                                        decoupled=o.decoupled or o.name == "adamw",
                                        step_dev=p.step_dev))
        ops.step_advance(p.step_dev)  # as record_update: the segment replaces FIN + O
        p.refresh_t(step=True, skip=skip)

    def update_then_forward(self, j: int, s: int, lr: Optional[float] = None) -> None:
        """Deferred DP update of layers [s, L) (completing the step: advance) followed by the
        forward of micro-batch j through [s, L) -- ONE native call when recorded."""
        L = len(self.geoms)
        if self._prog is not None and self._o_native and not self._recording:
            p = self.params
            p.set_lr(p.optim.lr if lr is None else lr)
            self._prog.run([f"O{s}-{L}", "OADV"] + [f"F{j}.L{i}" for i in range(s, L)],
                           torch.cuda.current_stream(self.device).cuda_stream)
            p.step_count += 1
            return
        self.update_layers(s, L, lr, advance=True)
        self.forward_layers(j, s, L)

    def wgrad_finalize(self, layers: Sequence[int]) -> None:
        """Batched wgrad of ``layers`` (in the given order) + their gradient reduction: one
        native call when recorded (a DP bucket)."""
        ls = list(layers)
        lo, hi = min(ls), max(ls)
        if (self._prog is not None and not self._recording and self._has_w and
                sorted(ls) == list(range(lo, hi + 1))):
            fin = f"FIN{lo}" if lo == hi else f"FIN{lo}-{hi}"
            self._prog.run([f"W{i}" for i in ls] + [fin],
                           torch.cuda.current_stream(self.device).cuda_stream)
            return
        for i in ls:
            self.wgrad_layer(i)
        self.finalize_grads(sorted(ls))

    def enable_fused_wgrad_update(self) -> list[int]:
        """Layers whose weight gradient is ONE split (big layers: the wide model's 8192x8192)
        apply the SGD step in their wgrad GEMM's epilogue (ops.linear_wgrad upd): no fp32
        gradient round trip through HBM, no separate update pass over those weights, and W^T
        written by the same epilogue instead of a transpose launch. Only without data
        parallelism (the gradient must be complete where it is produced) and for SGD; call
        before compile_native. Returns the layers."""
        p = self.params
        if (self.device.type != "cuda" or self.wgrad_mode != "batched" or
                self.wgrad_algo != "splitk" or p.optim.name != "sgd" or p.sharded or
                switches.get("DNN_WGRAD_FUSED_UPDATE") == "0" or self._prog is not None):
            return []
        p.fused_layers = {i for i in range(len(self.geoms)) if self.w_splits[i] == 1}
        self._reduce_jobs.clear()
        return sorted(p.fused_layers)

    def shard_update(self, e0: int, e1: int, lr: Optional[float] = None) -> None:
        """Sharded DP: unpack this rank's reduced piece of bucket [e0, e1) and update it (no
        step advance, no W^T refresh: both follow once per step)."""
        p = self.params
        p.shard_unpack(e0, e1)
        p0, p1 = p.shard_piece(e0, e1)
        p.update_range(p0, p1, lr, advance=False, refresh=False)

    def bias_update(self, lr: Optional[float] = None) -> None:
        """Sharded DP: every rank updates all biases (their fp32 gradients are all-reduced)."""
        p = self.params
        p.update_range(p.bias_lo, p.numel, lr, advance=False, refresh=False)

    def update_layers(self, a: int, b: int, lr: Optional[float] = None,
                      advance: bool = True) -> None:
        """Optimizer update of local layers [a, b) only (``advance``: this completes the
        step's update -- Adam's step counter moves once per step)."""
        if self._prog is not None and self._o_native and not self._recording:
            p = self.params
            p.set_lr(p.optim.lr if lr is None else lr)
            segs = [f"O{a}-{b}"] + (["OADV"] if advance else [])
            self._prog.run(segs, torch.cuda.current_stream(self.device).cuda_stream)
            if advance:
                p.step_count += 1
            return
        e0, e1 = self.params.layers_range(a, b)
        self.params.update_range(e0, e1, lr, advance)

    def optimizer_step(self, lr: Optional[float] = None) -> None:
        if self._prog is not None and self._o_native and not self._recording:
            self.params.set_lr(self.params.optim.lr if lr is None else lr)
            self.params.step_count += 1
            return self._replay("O")
        self.params.optimizer_step(lr)

    def fuse_boundary_colsum(self, consumer: "Stage") -> None:
        """Same-process pipeline: ``consumer`` (the next stage) writes our last layer's
        bias-gradient partials from its input-gradient dgrad epilogue (loopback only)."""
        if consumer.mb != self.mb or consumer.nm != self.nm:
            raise ValueError("loopback stages must share the micro-batch layout")
        L = len(self.geoms) - 1
        g0 = consumer.geoms[0]
        bm = ops.dgrad_tiles(consumer.mb, g0.kp, g0.np_)[0]
        self.bp[L] = self.mb // bm
        self.bpart[L] = torch.zeros(self.bp[L] * self.nm, self.geoms[L].np_,
                                    dtype=torch.float32, device=self.device)
        self._reduce_jobs.clear()
        self._colsum_by = consumer
        consumer._colsum_for = self

    # ---- native replay (csrc/runtime/program.{hpp,cpp}) ---------------------------------
    def compile_native(self) -> None:
        """Record every per-op kernel sequence of this stage ONCE into a native Program:
        F{j} / B{j} per micro-batch, W{i} / W (batched wgrad), FIN{i} / FIN (gradient
        reduction) and O (SGD update). Afterwards forward/backward/... replay their segment
        from C++ (one Python call per schedule op instead of one per kernel). The first
        stage's input and the last stage's labels are relocatable regions, so zero-copy
        batches (bind_input / bind_labels) work without re-recording. The Python bodies stay
        the reference path (CPU, per-micro wgrad, Adam)."""
        nat = native()
        prog = nat.Program()
        self.x_in = self.x_buf
        if self.labels is not None:
            self.labels = self.labels_buf
        self._rx = (prog.region(self.x_buf.data_ptr(), self.x_buf.numel() * 2)
                    if self.first else None)
        self._rl = (prog.region(self.labels_buf.data_ptr(), self.labels_buf.numel() * 4)
                    if self.labels is not None else None)
        # DNN_H0_DOUBLE: the layer-0 activation alternates between two buffers from step to
        # step (a relocatable region re-based by flip_h0), so the next step's layer-0 forward
        # never has to wait for this step's side-stream weight gradient that reads it
        # (pipeline._xstep_plan drops that wait)
        L = len(self.geoms)
        self.h0_double = (switches.get("DNN_H0_DOUBLE") == "1" and self.device.type == "cuda"
                          and self.first and self.last and self.nm == 1 and L >= 2 and
                          0 not in self.actT and
                          not (self.tail and L - 2 <= 0))
        self._rh0 = None
        if self.h0_double:
            a0 = self.acts[0]
            self._h0_alt = torch.zeros_like(a0)
            self._h0_ptrs = (a0.data_ptr(), self._h0_alt.data_ptr())
            self._h0_flip = 0
            self._rh0 = prog.region(a0.data_ptr(), a0.numel() * a0.element_size())
        self._recording = True
        nat.record_begin(prog)
        try:
            for j in range(self.nm):
                prog.mark(f"F{j}")
                self.forward(j)
            for j in range(self.nm):  # per-layer forward segments (deferred DP updates)
                for i in range(len(self.geoms)):
                    prog.mark(f"F{j}.L{i}")
                    self._forward_layer(j, i)
            for j in range(self.nm):
                prog.mark(f"B{j}")
                self.backward(j)
            for j in range(self.nm):  # per-layer dgrad segments (dgrad/wgrad overlap plans)
                prog.mark(f"B{j}.pre")
                self._backward_pre(j)
                for i in range(len(self.geoms) - 1, -1, -1):
                    prog.mark(f"B{j}.L{i}")
                    self._backward_layer(j, i)
            self._has_w = self.wgrad_mode == "batched"
            if self._has_w:
                for i in range(len(self.geoms)):
                    prog.mark(f"W{i}")
                    self.wgrad_layer(i)
                prog.mark("W")
                self._wgrad_all()
            L = len(self.geoms)
            for a in range(L):  # every contiguous layer range: one reduce launch per DP bucket
                for b in range(a, L):
                    prog.mark(f"FIN{a}" if a == b else f"FIN{a}-{b}")
                    self.finalize_grads(list(range(a, b + 1)))
            prog.mark("FIN")
            self.finalize_grads()
            if self.fused_fin_sgd_ok():
                prog.mark("FINO")
                self._record_fin_sgd()
                if self.params.optim.name == "sgd" and L > 1:
                    # per-layer-range forms: the overlap plan updates the small layers on the
                    # side stream while the big layer's wgrad still runs (DNN_SPLIT_FINO)
                    for a in range(L):
                        for b in range(a, L):
                            prog.mark(f"FINO{a}-{b}")
                            self._record_fin_sgd(a, b + 1)
            prog.mark("O")
            self.params.record_update()
            for a in range(L if not (self.params.sharded or self.params.fused_layers) else 0):
                # split updates: every contiguous layer range, no step advance
                for b in range(a + 1, L + 1):
                    prog.mark(f"O{a}-{b}")
                    e0, e1 = self.params.layers_range(a, b)
                    self.params.record_update_range(e0, e1, advance=False)
            prog.mark("OADV")
            if self.params.optim.name != "sgd":
                ops.step_advance(self.params.step_dev)
            if self.params.sharded:  # sharded DP: per bucket pack / unpack + piece update
                p = self.params
                for a in range(L):
                    for b in range(a, L):
                        e0, _ = p.layer_grad_range(a)
                        _, e1 = p.layer_grad_range(b)
                        prog.mark(f"SP{a}-{b}")
                        p.shard_pack(e0, e1)
                        prog.mark(f"SU{a}-{b}")
                        self.shard_update(e0, e1)
                prog.mark("SB")
                self.bias_update()
                prog.mark("T")
                p.refresh_t()
            for j in range(self.nm):  # fp8 boundary packs / unpacks per micro-batch
                if self._fp8_next:
                    prog.mark(f"QF{j}")
                    self.pack_fwd(j)
                    prog.mark(f"DQB{j}")
                    self.unpack_bwd(j)
                if self._fp8_prev:
                    prog.mark(f"DQF{j}")
                    self.unpack_fwd(j)
                    prog.mark(f"QB{j}")
                    self.pack_bwd(j)
            self._o_native = True
        finally:
            nat.record_end()
            self._recording = False
        self._prog = prog

    def _replay(self, seg: str) -> None:
        self._prog.run([seg], torch.cuda.current_stream(self.device).cuda_stream)

    def flip_h0(self) -> None:
        """Start a step on the other layer-0 activation buffer (DNN_H0_DOUBLE)."""
        if self._rh0 is not None:
            self._h0_flip ^= 1
            self._prog.rebase(self._rh0, self._h0_ptrs[self._h0_flip])

    def bind_input(self, x: torch.Tensor) -> None:
        """First stage reads ``x`` in place (zero-copy) from now on."""
        self.x_in = x
        if self._prog is not None and self._rx is not None:
            self._prog.rebase(self._rx, x.data_ptr())

    def bind_labels(self, y: torch.Tensor) -> None:
        self.labels = y
        if self._prog is not None and self._rl is not None:
            self._prog.rebase(self._rl, y.data_ptr())

    # convenience: a whole step when this stage holds the entire model ----------------------
    def set_batch(self, x: torch.Tensor, labels: torch.Tensor) -> None:
        self.bind_input(self.x_buf)  # never write through an alias of the caller's dataset
        self.x_in.copy_(x)
        if self.labels is not None:
            self.bind_labels(self.labels_buf)
            self.labels.copy_(labels)

    def loss_sum(self) -> float:
        """Sum of per-row CE losses of the last step (fixed-order fp64 host sum)."""
        return float(self.loss_part.detach().cpu().double().sum())

    def flops_per_step(self) -> float:
        f = 0.0
        for i, g in enumerate(self.geoms):
            mult = 3 if (i > 0 or not self.first) else 2
            f += 2.0 * mult * self.rows * g.np_ * g.kp
        return f
