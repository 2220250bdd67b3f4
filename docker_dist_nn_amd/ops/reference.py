"""PyTorch reference implementations with the kernels' numerics contract.

bf16 operands, fp32 accumulation, outputs rounded once to bf16 (or kept fp32). Used (a) as the
CPU execution path so the engine, pipeline schedules and DP logic run in CPU tests with gloo,
and (b) as the fp32 oracle for the GPU kernel tests.
"""
from __future__ import annotations

import torch

KMAJ, MNMAJ = 0, 1
_LINEAR, _RELU, _SIGMOID = 0, 1, 2


def act_fwd(v: torch.Tensor, act: int) -> torch.Tensor:
    if act == _RELU:
        return torch.clamp_min(v, 0.0)
    if act == _SIGMOID:
        return torch.sigmoid(v)
    return v


def act_bwd(g: torch.Tensor, y: torch.Tensor, act: int) -> torch.Tensor:
    if act == _RELU:
        return torch.where(y > 0, g, torch.zeros_like(g))
    if act == _SIGMOID:
        return g * y * (1.0 - y)
    return g


def _logical(a, b, layout_a, layout_b, M, N, Ktot):
    A = a[:M, :Ktot] if layout_a == KMAJ else a[:Ktot, :M].t()
    B = b[:N, :Ktot].t() if layout_b == KMAJ else b[:Ktot, :N]
    return A.float(), B.float()


def _colsum_blocks(vals, out, rows_per):
    nb = vals.shape[0] // rows_per
    out[:nb, :vals.shape[1]] = vals[:nb * rows_per].reshape(nb, rows_per, -1).sum(1)


def gemm(a, b, c, *, layout_a, layout_b, M, N, K, bias=None, aux=None, act=0, accumulate=False,
         splits=1, colsum=None, colsum_rows=0, k_total=0):
    ktot = k_total or K * splits
    A, B = _logical(a, b, layout_a, layout_b, M, N, ktot)
    out_f32 = c.dtype == torch.float32
    ks = ktot // 64
    for s in range(splits):
        if k_total:  # uneven split-K: same k-step ranges as the kernel
            k0, k1 = (s * ks // splits) * 64, ((s + 1) * ks // splits) * 64
        else:
            k0, k1 = s * K, (s + 1) * K
        acc = A[:, k0:k1] @ B[k0:k1, :]
        if bias is not None:
            acc = acc + bias[:N].float()
        if out_f32:
            dst = c[s] if c.dim() == 3 else c
            if accumulate:
                acc = acc + dst[:M, :N]
            else:
                acc = act_fwd(acc, act)
            dst[:M, :N] = acc
        else:
            if aux is not None:
                acc = act_bwd(acc, aux[:M, :N].float(), act)
            else:
                acc = act_fwd(acc, act)
            c[:M, :N] = acc.to(c.dtype)
            if colsum is not None:
                _colsum_blocks(c[:M, :N].float(), colsum, colsum_rows)
    return c


def softmax_xent(logits, labels, dz, n_cls, scale, loss_part=None, correct=None,
                 rows_per_block=64, colsum=None):
    rows, width = dz.shape
    lg = logits[:rows, :n_cls].float()
    lab = labels[:rows].long()
    valid = lab >= 0
    p = torch.softmax(lg, dim=1)
    g = p.clone()
    safe = lab.clamp_min(0)
    g[torch.arange(rows), safe] -= 1.0
    g = g * float(scale)
    g[~valid] = 0.0
    dz.zero_()
    dz[:, :n_cls] = g.to(dz.dtype)
    if loss_part is not None:
        logp = torch.log_softmax(lg, dim=1)
        nll = torch.where(valid, -logp[torch.arange(rows), safe], torch.zeros_like(lg[:, 0]))
        nb = -(-rows // rows_per_block)
        pad = torch.zeros(nb * rows_per_block)
        pad[:rows] = nll
        loss_part[:nb] = pad.view(nb, rows_per_block).sum(1).to(loss_part.dtype)
    if correct is not None:  # per-block partial counts (written, not accumulated)
        pred = torch.argmax(lg, dim=1)
        nb = -(-rows // rows_per_block)
        hit = torch.zeros(nb * rows_per_block, dtype=torch.int64)
        hit[:rows] = ((pred == lab) & valid).long()
        correct[:nb] = hit.view(nb, rows_per_block).sum(1).to(correct.dtype)
    if colsum is not None:
        nb = -(-rows // rows_per_block)
        pad = torch.zeros(nb * rows_per_block, width)
        pad[:rows] = dz.float()
        colsum[:nb, :width] = pad.view(nb, rows_per_block, width).sum(1)


def softmax_rows(logits, out, n_cls, labels=None, pred=None, correct=None):
    rows = logits.shape[0]
    lg = logits[:rows, :n_cls].float()
    if out is not None:
        out[:rows, :n_cls] = torch.softmax(lg, dim=1)
    am = torch.argmax(lg, dim=1)
    if pred is not None:
        pred[:rows] = am.to(pred.dtype)
    if correct is not None and labels is not None:
        correct += (am == labels[:rows].long()).sum().to(correct.dtype)


def colsum_partial(x, part, n_part):
    rows, cols = x.shape
    per = (rows + n_part - 1) // n_part
    xf = x.float()
    for i in range(n_part):
        part[i, :cols] = xf[i * per:min(rows, (i + 1) * per)].sum(0)


def reduce_slabs(src, n_src, stride, n, out, scale=1.0, accumulate=False):
    flat = src.reshape(-1)
    acc = flat[:n].clone()
    for s in range(1, n_src):
        acc += flat[s * stride:s * stride + n]
    acc *= scale
    o = out.reshape(-1)
    if accumulate:
        o[:n] += acc
    else:
        o[:n] = acc


def sgd_update(p, g, mom, shadow, lr, momentum, weight_decay):
    gv = g + weight_decay * p if weight_decay else g.clone()
    if momentum and mom is not None:
        mom.mul_(momentum).add_(gv)
        gv = mom
    p.sub_(lr * gv)
    if shadow is not None:
        shadow.copy_(p.to(shadow.dtype))


def adam_update(p, g, m, v, shadow, lr, b1, b2, eps, weight_decay, decoupled, bc1, bc2):
    gv = g.clone()
    if decoupled:
        p.mul_(1.0 - lr * weight_decay)
    elif weight_decay:
        gv += weight_decay * p
    m.mul_(b1).add_((1.0 - b1) * gv)
    v.mul_(b2).add_((1.0 - b2) * gv * gv)
    p.sub_(lr * (m * bc1) / (torch.sqrt(v * bc2) + eps))
    if shadow is not None:
        shadow.copy_(p.to(shadow.dtype))


def pack_bf16(src, out):
    rows, cols = src.shape
    out.zero_()
    out[:rows, :cols] = src.to(out.dtype)


TAIL_BLOCK_ROWS = 16  # rows per 16-row block; the mlp_tail grid is one workgroup per block,
# at most one per CU, blocks dealt round-robin


def tail_waves(act3: int, act2: int) -> int:
    """Waves per workgroup of csrc/kernels/mlp_tail.hip (16 rows each): 16 for ReLU/ReLU."""
    return 16 if act3 == _RELU and act2 == _RELU else 8


def mlp_tail(x, w3, b3, w4, b4, labels, h3, dz4, dz3, dz2, n_cls, scale, act3, act2,
             loss_part, correct, cs4, cs3, cs2, n_blocks):
    """Unfused reference of the fused classifier tail. Partials follow the kernel's row
    assignment: 16-row block rb belongs to workgroup rb % n_blocks."""
    rows, k3 = x.shape
    n3, n4 = w3.shape[0], w4.shape[0]
    gemm(x, w3, h3, layout_a=KMAJ, layout_b=KMAJ, M=rows, N=n3, K=k3, bias=b3, act=act3)
    logits = torch.zeros(rows, n4, dtype=torch.float32)
    gemm(h3, w4, logits, layout_a=KMAJ, layout_b=KMAJ, M=rows, N=n4, K=n3, bias=b4, act=0)
    lg = logits[:, :n_cls]
    lab = labels[:rows].long()
    valid = lab >= 0
    safe = lab.clamp_min(0)
    per_row_loss = torch.where(valid, -torch.log_softmax(lg, 1)[torch.arange(rows), safe],
                               torch.zeros(rows))
    hit = ((torch.argmax(lg, 1) == lab) & valid).long()
    softmax_xent(logits, labels, dz4, n_cls, scale)
    gemm(dz4, w4, dz3, layout_a=KMAJ, layout_b=MNMAJ, M=rows, N=n3, K=n4, aux=h3, act=act3)
    gemm(dz3, w3, dz2, layout_a=KMAJ, layout_b=MNMAJ, M=rows, N=k3, K=n3, aux=x, act=act2)
    owner = (torch.arange(rows) // 16) % n_blocks
    for t, src, cols in ((cs4, dz4, n4), (cs3, dz3, n3), (cs2, dz2, k3)):
        part = torch.zeros(n_blocks, cols)
        part.index_add_(0, owner, src[:rows, :cols].float())
        t[:n_blocks, :cols] = part
    loss_part[:n_blocks] = 0.0
    loss_part.index_add_(0, owner, per_row_loss.to(loss_part.dtype))
    correct[:n_blocks] = 0
    correct.index_add_(0, owner, hit.to(correct.dtype))
