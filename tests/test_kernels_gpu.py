"""Numerics of the gfx950 HIP kernels against plain PyTorch fp32 references of the same op.

GEMM checks use (1) small-integer operands, for which every product and partial sum is exact
in fp32, so the kernel must match bit-for-bit -- this is what catches a transposed fragment map
or a wrong LDS swizzle (guide §3: "always A=I-check with ASYMMETRIC B"); and (2) random data
with bf16-level tolerances.
"""
import pytest
import torch

from docker_dist_nn_amd import ops
from docker_dist_nn_amd.ops import KMAJ, MNMAJ
from docker_dist_nn_amd.utils import native

pytestmark = pytest.mark.gpu

LAYOUTS = [(KMAJ, KMAJ), (KMAJ, MNMAJ), (MNMAJ, MNMAJ), (MNMAJ, KMAJ)]
TILES = [(128, 128), (128, 64), (64, 128), (64, 64)]


def _storage(layout, mn, k, gen, dev, integer):
    shape = (mn, k) if layout == KMAJ else (k, mn)
    if integer:
        t = torch.randint(-3, 4, shape, generator=gen, dtype=torch.int32).float()
    else:
        t = torch.randn(shape, generator=gen)
    return t.to(torch.bfloat16).to(dev)


def _logical(t, layout, mn, k):
    return t.float()[:mn, :k] if layout == KMAJ else t.float()[:k, :mn].t()


def test_native_extension_is_loaded():
    mod = native()
    assert mod.__file__.endswith(".so")


@pytest.mark.parametrize("la,lb", LAYOUTS)
@pytest.mark.parametrize("bm,bn", TILES)
def test_gemm_exact_integer(dev, la, lb, bm, bn):
    gen = torch.Generator().manual_seed(1234 + 10 * la + lb + bm + 3 * bn)
    M, N, K = 256, 192 if bn == 64 else 256, 320
    a = _storage(la, M, K, gen, dev, True)
    b = _storage(lb, N, K, gen, dev, True)
    c = torch.empty(M, N, device=dev, dtype=torch.float32)
    ops.gemm(a, b, c, layout_a=la, layout_b=lb, M=M, N=N, K=K, tiles=(bm, bn))
    ref = _logical(a, la, M, K) @ _logical(b, lb, N, K).t()
    torch.cuda.synchronize()
    assert torch.equal(c, ref), (c - ref).abs().max()


BIG = [(256, 256), (256, 128), (128, 256), (256, 64)]


@pytest.mark.parametrize("la,lb", LAYOUTS)
@pytest.mark.parametrize("bm,bn", BIG)
def test_gemm_exact_integer_8wave(dev, la, lb, bm, bn):
    """8-wave tiles (row-chunked epilogue, 512 threads): exact on integer data, bf16 output
    with bias + colsum partials, and split-K slabs."""
    gen = torch.Generator().manual_seed(99 + bm + 7 * bn + 10 * la + lb)
    M, N, K = 2 * bm, 2 * bn, 448
    a = _storage(la, M, K, gen, dev, True)
    b = _storage(lb, N, K, gen, dev, True)
    ref = _logical(a, la, M, K) @ _logical(b, lb, N, K).t()
    c = torch.empty(M, N, device=dev, dtype=torch.float32)
    ops.gemm(a, b, c, layout_a=la, layout_b=lb, M=M, N=N, K=K, tiles=(bm, bn))
    assert torch.equal(c, ref), (c - ref).abs().max()
    bias = torch.randint(-4, 5, (N,), generator=gen).float().to(dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    cs = torch.full((M // bm, N), 7.0, device=dev)
    ops.gemm(a, b, y, layout_a=la, layout_b=lb, M=M, N=N, K=K, bias=bias, act="relu",
             tiles=(bm, bn), colsum=cs)
    yr = (ref + bias).clamp_min(0).to(torch.bfloat16)
    assert torch.equal(y, yr)
    torch.testing.assert_close(cs, yr.float().view(M // bm, bm, N).sum(1), rtol=1e-5, atol=1e-2)
    S = 3
    slabs = torch.empty(S, M, N, device=dev)
    ops.gemm(a, b, slabs, layout_a=la, layout_b=lb, M=M, N=N, K=K, k_total=K, splits=S,
             tiles=(bm, bn))
    assert torch.equal(slabs.sum(0), ref)


@pytest.mark.parametrize("la,lb", LAYOUTS)
@pytest.mark.parametrize("bm,bn", [(256, 256), (128, 128), (256, 128)])
def test_gemm_partial_edge_tiles(dev, la, lb, bm, bn):
    """N (and M) not a multiple of the tile: partial edge tiles in one launch (clamped loads,
    masked stores) -- exact on integer data for bf16 output (+bias, relu, colsum) and split-K
    slabs; storage past N/M is never written."""
    gen = torch.Generator().manual_seed(5 + bm + bn + 3 * la + lb)
    M, N, K = 2 * bm, 832, 320
    a = _storage(la, M, K, gen, dev, True)
    b = _storage(lb, N, K, gen, dev, True)
    ref = _logical(a, la, M, K) @ _logical(b, lb, N, K).t()
    bias = torch.randint(-4, 5, (N,), generator=gen).float().to(dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    cs = torch.full((M // bm, N), 3.0, device=dev)
    ops.gemm(a, b, y, layout_a=la, layout_b=lb, M=M, N=N, K=K, bias=bias, act="relu",
             tiles=(bm, bn), colsum=cs)
    yr = (ref + bias).clamp_min(0).to(torch.bfloat16)
    assert torch.equal(y, yr)
    torch.testing.assert_close(cs, yr.float().view(M // bm, bm, N).sum(1), rtol=1e-5, atol=1e-2)
    slabs = torch.empty(3, M, N, device=dev)
    ops.gemm(a, b, slabs, layout_a=la, layout_b=lb, M=M, N=N, K=K, k_total=K, splits=3,
             tiles=(bm, bn))
    assert torch.equal(slabs.sum(0), ref)
    # partial rows too (M = bm + 40), into a wider buffer whose extra rows/cols must stay
    Mp = bm + 40
    big = torch.full((Mp + 8, N + 8), -1.0, device=dev)
    ops.gemm(a, b, big, layout_a=la, layout_b=lb, M=Mp, N=N, K=K, tiles=(bm, bn))
    assert torch.equal(big[:Mp, :N], ref[:Mp])
    assert torch.all(big[Mp:] == -1.0) and torch.all(big[:, N:] == -1.0)


def test_gemm_identity_asymmetric(dev):
    M = N = K = 128
    eye = torch.eye(M, dtype=torch.bfloat16, device=dev)
    b = (torch.arange(N * K, dtype=torch.float32).reshape(N, K) % 97).to(torch.bfloat16).to(dev)
    c = torch.empty(M, N, device=dev)
    ops.gemm(eye, b, c, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K)
    assert torch.equal(c, b.float().t())


@pytest.mark.parametrize("la,lb", LAYOUTS)
def test_gemm_random_bf16_out(dev, la, lb):
    gen = torch.Generator().manual_seed(7)
    M, N, K = 512, 384, 832
    a = _storage(la, M, K, gen, dev, False)
    b = _storage(lb, N, K, gen, dev, False)
    bias = torch.randn(N, generator=gen).to(dev)
    for act in ("linear", "relu", "sigmoid"):
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ops.gemm(a, b, c, layout_a=la, layout_b=lb, M=M, N=N, K=K, bias=bias, act=act)
        ref = _logical(a, la, M, K) @ _logical(b, lb, N, K).t() + bias
        ref = {"linear": ref, "relu": ref.clamp_min(0), "sigmoid": torch.sigmoid(ref)}[act]
        torch.testing.assert_close(c.float(), ref, rtol=1.6e-2, atol=2e-2)


def test_gemm_split_k_accumulate(dev):
    gen = torch.Generator().manual_seed(3)
    R, N, K, S = 1024, 128, 256, 4
    dz = torch.randn(R, N, generator=gen).to(torch.bfloat16).to(dev)
    x = torch.randn(R, K, generator=gen).to(torch.bfloat16).to(dev)
    slabs = torch.empty(S, N, K, device=dev)
    ops.linear_wgrad(dz, x, slabs, splits=S)
    ops.linear_wgrad(dz, x, slabs, splits=S, accumulate=True)
    full = 2 * dz.float().t() @ x.float()
    torch.testing.assert_close(slabs.sum(0), full, rtol=1e-4, atol=1e-3)
    part = dz.float()[: R // S].t() @ x.float()[: R // S]
    torch.testing.assert_close(slabs[0], 2 * part, rtol=1e-4, atol=1e-3)


def test_linear_triplet_matches_autograd(dev):
    """fwd/dgrad(+relu mask)/wgrad of one hidden layer vs torch autograd in fp32."""
    gen = torch.Generator().manual_seed(11)
    M, K, N = 256, 832, 512
    x = torch.rand(M, K, generator=gen).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=gen) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, generator=gen) * 0.1
    g_out = torch.randn(M, N, generator=gen).to(torch.bfloat16)
    xd, wd, bd, gd = x.to(dev), w.to(dev), b.to(dev), g_out.to(dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.linear_fwd(xd, wd, bd, y, act="relu")
    xr = x.float().requires_grad_()
    wr = w.float().requires_grad_()
    yr = torch.relu(xr @ wr.t() + b)
    torch.testing.assert_close(y.float().cpu(), yr.detach(), rtol=1.6e-2, atol=1e-2)
    # dz of this layer given upstream grad: dz = g * relu'(y)
    dz = torch.where(y > 0, gd, torch.zeros_like(gd))
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    ops.linear_dgrad(dz, wd, dx)
    slabs = torch.empty(2, N, K, device=dev)
    ops.linear_wgrad(dz, xd, slabs, splits=2)
    yr.backward(g_out.float())
    torch.testing.assert_close(dx.float().cpu(), xr.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(slabs.sum(0).cpu(), wr.grad, rtol=2e-2, atol=5e-2)


def test_dgrad_fused_mask(dev):
    gen = torch.Generator().manual_seed(5)
    M, N, K = 128, 128, 256
    dz = torch.randn(M, N, generator=gen).to(torch.bfloat16).to(dev)
    w = torch.randn(N, K, generator=gen).to(torch.bfloat16).to(dev)
    y_prev = torch.randn(M, K, generator=gen).clamp_min(0).to(torch.bfloat16).to(dev)
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    ops.linear_dgrad(dz, w, dx, y_prev=y_prev, act_prev="relu")
    ref = (dz.float() @ w.float()) * (y_prev.float() > 0)
    torch.testing.assert_close(dx.float(), ref, rtol=1.6e-2, atol=2e-2)


def test_gemm_rejects_bad_shapes(dev):
    a = torch.zeros(100, 64, device=dev, dtype=torch.bfloat16)
    w = torch.zeros(64, 64, device=dev, dtype=torch.bfloat16)
    y = torch.zeros(100, 64, device=dev, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        ops.linear_fwd(a, w, None, y)


def test_softmax_xent(dev):
    gen = torch.Generator().manual_seed(9)
    rows, ncls, width = 300, 10, 64
    logits = torch.randn(rows, width, generator=gen) * 3
    labels = torch.randint(0, ncls, (rows,), generator=gen, dtype=torch.int32)
    labels[::7] = -1  # padding rows
    dz = torch.empty(rows, width, dtype=torch.bfloat16, device=dev)
    loss = torch.zeros(ops.xent_blocks(rows), device=dev)
    corr = torch.full((ops.xent_blocks(rows),), 7777, dtype=torch.int32, device=dev)  # no zeroing
    ops.softmax_xent(logits.to(dev), labels.to(dev), dz, ncls, 1.0 / rows, loss, corr)
    dz_r = torch.empty(rows, width, dtype=torch.bfloat16)
    loss_r = torch.zeros(ops.xent_blocks(rows))
    corr_r = torch.zeros(ops.xent_blocks(rows), dtype=torch.int32)
    from docker_dist_nn_amd.ops import reference as ref
    ref.softmax_xent(logits, labels, dz_r, ncls, 1.0 / rows, loss_r, corr_r)
    assert loss.shape == loss_r.shape
    torch.testing.assert_close(dz.float().cpu(), dz_r.float(), rtol=1e-2, atol=1e-4)
    torch.testing.assert_close(loss.cpu(), loss_r, rtol=1e-5, atol=1e-3)
    assert corr.cpu().tolist() == corr_r.tolist()


def test_softmax_rows_and_argmax(dev):
    gen = torch.Generator().manual_seed(10)
    rows, ncls = 257, 10
    logits = torch.randn(rows, 64, generator=gen).to(dev)
    out = torch.zeros(rows, 64, device=dev)
    labels = torch.randint(0, ncls, (rows,), generator=gen, dtype=torch.int32).to(dev)
    pred = torch.empty(rows, dtype=torch.int32, device=dev)
    corr = torch.zeros(1, dtype=torch.int32, device=dev)
    ops.softmax_rows(logits, out, ncls, labels, pred, corr)
    p = torch.softmax(logits[:, :ncls], 1)
    torch.testing.assert_close(out[:, :ncls], p, rtol=1e-5, atol=1e-6)
    am = torch.argmax(logits[:, :ncls], 1)
    assert torch.equal(pred.long(), am)
    assert int(corr.item()) == int((am == labels.long()).sum())


def test_colsum_and_reduce(dev):
    gen = torch.Generator().manual_seed(4)
    rows, cols, P = 1000, 192, 7
    x = torch.randn(rows, cols, generator=gen).to(torch.bfloat16).to(dev)
    part = torch.empty(P, cols, device=dev)
    ops.colsum_partial(x, part)
    out = torch.empty(cols, device=dev)
    ops.reduce_slabs(part, P, cols, cols, out, scale=0.5)
    torch.testing.assert_close(out, 0.5 * x.float().sum(0), rtol=1e-4, atol=1e-3)


def test_sgd_and_adam_match_torch(dev):
    gen = torch.Generator().manual_seed(2)
    n = 4096
    p0 = torch.randn(n, generator=gen)
    g = torch.randn(n, generator=gen)
    # SGD with momentum + weight decay vs torch.optim.SGD
    p = p0.clone().to(dev)
    mom = torch.zeros(n, device=dev)
    sh = torch.empty(n, device=dev, dtype=torch.bfloat16)
    tp = torch.nn.Parameter(p0.clone())
    opt = torch.optim.SGD([tp], lr=0.1, momentum=0.9, weight_decay=0.01)
    for _ in range(3):
        ops.sgd_update(p, g.to(dev), mom, sh, lr=0.1, momentum=0.9, weight_decay=0.01)
        tp.grad = g.clone()
        opt.step()
    torch.testing.assert_close(p.cpu(), tp.detach(), rtol=1e-5, atol=1e-6)
    assert torch.equal(sh, p.to(torch.bfloat16))
    # Adam vs torch.optim.Adam
    p = p0.clone().to(dev)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    tp = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([tp], lr=1e-3)
    for step in range(1, 4):
        ops.adam_update(p, g.to(dev), m, v, None, lr=1e-3, step=step)
        tp.grad = g.clone()
        opt.step()
    torch.testing.assert_close(p.cpu(), tp.detach(), rtol=1e-5, atol=1e-6)


def test_pack_unpack(dev):
    x = torch.rand(100, 784, device=dev)
    out = torch.full((128, 832), 7.0, device=dev, dtype=torch.bfloat16)
    ops.pack_bf16(x, out)
    assert torch.equal(out[:100, :784], x.to(torch.bfloat16))
    assert out[100:].abs().sum() == 0 and out[:, 784:].abs().sum() == 0
    back = torch.empty(100, 784, device=dev)
    ops.unpack_bf16(out, back)
    assert torch.equal(back, x.to(torch.bfloat16).float())


@pytest.mark.parametrize("n_src", [1, 3, 8, 17, 40, 64, 128, 300])  # every source-group class
def test_reduce_slabs_many_sources(dev, n_src):
    gen = torch.Generator().manual_seed(n_src)
    n = 4096 + 64
    src = torch.randn(n_src, n, generator=gen).to(dev)
    out = torch.ones(n, device=dev)
    ops.reduce_slabs(src, n_src, n, n, out, scale=0.25, accumulate=True)
    torch.testing.assert_close(out, 1 + 0.25 * src.sum(0), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("max_blocks", [0, 7, 128])
def test_reduce_multi_bitwise_equals_reduce_slabs(dev, max_blocks):
    """One launch over jobs with every source-group class (1..64 groups of sources) and > 16
    jobs (several launches) must reproduce per-job reduce_slabs bit for bit -- also with the
    grid capped (max_blocks: each workgroup loops over blocks)."""
    gen = torch.Generator().manual_seed(5)
    shapes = [(1, 64), (3, 4096), (7, 832 * 512), (16, 256), (512, 128), (40, 1024),
              (9, 2048), (18, 832 * 512), (64, 256 * 512), (128, 4096)] * 2
    jobs, expect = [], []
    for k, (ns, n) in enumerate(shapes):
        src = torch.randn(ns, n + 8, generator=gen).to(dev)
        out = torch.randn(n, generator=gen).to(dev)
        acc, scale = bool(k % 2), 0.5 + k
        ref_out = out.clone()
        ops.reduce_slabs(src, ns, n + 8, n, ref_out, scale=scale, accumulate=acc)
        jobs.append((src, ns, n + 8, n, out, scale, acc))
        expect.append(ref_out)
    ops.reduce_multi(jobs, max_blocks=max_blocks)
    for j, e in zip(jobs, expect):
        assert torch.equal(j[4], e)


def test_dgrad_colsum_partials(dev):
    gen = torch.Generator().manual_seed(21)
    M, N, K = 512, 128, 832
    dz = torch.randn(M, N, generator=gen).to(torch.bfloat16).to(dev)
    w = torch.randn(N, K, generator=gen).to(torch.bfloat16).to(dev)
    y_prev = torch.randn(M, K, generator=gen).clamp_min(0).to(torch.bfloat16).to(dev)
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    bm = ops.dgrad_tiles(M, K, N)[0]
    part = torch.full((M // bm, K), 99.0, device=dev)
    ops.linear_dgrad(dz, w, dx, y_prev=y_prev, act_prev="relu", colsum=part)
    ref = dx.float().view(M // bm, bm, K).sum(1)
    torch.testing.assert_close(part, ref, rtol=1e-5, atol=1e-4)


def test_xent_colsum_partials(dev):
    gen = torch.Generator().manual_seed(22)
    rows, width, ncls = 1000, 64, 10
    logits = (torch.randn(rows, width, generator=gen) * 2).to(dev)
    labels = torch.randint(0, ncls, (rows,), generator=gen, dtype=torch.int32).to(dev)
    dz = torch.empty(rows, width, dtype=torch.bfloat16, device=dev)
    nb = ops.xent_blocks(rows)
    part = torch.full((nb, width), 5.0, device=dev)
    ops.softmax_xent(logits, labels, dz, ncls, 1.0, None, None, colsum=part)
    pad = torch.zeros(nb * 64, width, device=dev)
    pad[:rows] = dz.float()
    torch.testing.assert_close(part, pad.view(nb, 64, width).sum(1), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("R,N,K,nwg", [(65536, 512, 832, 512), (4096, 64, 128, 512),
                                       (2048, 256, 512, 7), (8192, 1024, 1024, 512),
                                       (1024, 128, 192, 3)])
def test_wgrad_streamk(dev, R, N, K, nwg):
    gen = torch.Generator().manual_seed(R + N)
    dz = torch.randn(R, N, generator=gen).to(torch.bfloat16).to(dev)
    x = torch.randn(R, K, generator=gen).to(torch.bfloat16).to(dev)
    part = torch.empty(ops.streamk_partial_elems(N, K, nwg), device=dev)
    g = torch.full((N, K), 3.0, device=dev)
    ops.linear_wgrad_streamk(dz, x, g, part, accumulate=False, nwg=nwg)
    ref = dz.float().t() @ x.float()
    torch.testing.assert_close(g, ref, rtol=1e-4, atol=2e-3 * (R / 1024) ** 0.5)
    ops.linear_wgrad_streamk(dz, x, g, part, accumulate=True, nwg=nwg)
    torch.testing.assert_close(g, 2 * ref, rtol=1e-4, atol=4e-3 * (R / 1024) ** 0.5)
    g2 = torch.empty_like(g)
    ops.linear_wgrad_streamk(dz, x, g2, part, nwg=nwg)
    assert torch.equal(g2, g / 2) or torch.equal(g2 * 2, g)  # deterministic


@pytest.mark.parametrize("R,S", [(65536 // 8, 14), (640, 3), (4096, 48)])
def test_uneven_split_k_exact(dev, R, S):
    gen = torch.Generator().manual_seed(S)
    N, K = 128, 192
    dz = torch.randint(-2, 3, (R, N), generator=gen).float().to(torch.bfloat16).to(dev)
    x = torch.randint(-2, 3, (R, K), generator=gen).float().to(torch.bfloat16).to(dev)
    slabs = torch.empty(S, N, K, device=dev)
    ops.linear_wgrad(dz, x, slabs, splits=S)
    assert torch.equal(slabs.sum(0), dz.float().t() @ x.float())
    ks = R // 64
    for s in (0, S - 1):
        a, b = (s * ks // S) * 64, ((s + 1) * ks // S) * 64
        assert torch.equal(slabs[s], dz.float()[a:b].t() @ x.float()[a:b])


@pytest.mark.parametrize("M,Np", [(1024, 64), (256, 64), (512, 128)])
def test_fused_linear_xent_matches_unfused(dev, M, Np):
    gen = torch.Generator().manual_seed(M + Np)
    K, ncls = 128, 10
    x = torch.randn(M, K, generator=gen).to(torch.bfloat16).to(dev)
    w = torch.zeros(Np, K)
    w[:ncls] = torch.randn(ncls, K, generator=gen) * 0.2
    w = w.to(torch.bfloat16).to(dev)
    b = torch.zeros(Np)
    b[:ncls] = torch.randn(ncls, generator=gen)
    b = b.to(dev)
    labels = torch.randint(0, ncls, (M,), generator=gen, dtype=torch.int32)
    labels[::9] = -1
    labels = labels.to(dev)
    bm = ops.xent_tiles(M, Np)[0]
    dz = torch.empty(M, Np, dtype=torch.bfloat16, device=dev)
    lp = torch.zeros(M // bm, device=dev)
    cor = torch.full((M // bm,), -5, dtype=torch.int32, device=dev)
    cs = torch.zeros(M // bm, Np, device=dev)
    ops.linear_fwd_xent(x, w, b, dz, labels, ncls, 1.0 / M, lp, cor, colsum=cs)
    logits = torch.empty(M, Np, device=dev)
    ops.linear_fwd(x, w, b, logits, act="linear")
    dz2 = torch.empty(M, Np, dtype=torch.bfloat16, device=dev)
    lp2 = torch.zeros(ops.xent_blocks(M), device=dev)
    cor2 = torch.zeros(ops.xent_blocks(M), dtype=torch.int32, device=dev)
    ops.softmax_xent(logits, labels, dz2, ncls, 1.0 / M, lp2, cor2)
    torch.testing.assert_close(dz.float(), dz2.float(), rtol=2e-2, atol=1e-5)
    torch.testing.assert_close(lp.sum(), lp2.sum(), rtol=1e-4, atol=1e-3)
    assert int(cor.sum().item()) == int(cor2.sum().item())
    torch.testing.assert_close(cs, dz.float().view(M // bm, bm, Np).sum(1), rtol=1e-5, atol=1e-5)


def test_sync_debug_mode(dev, monkeypatch):
    """DNN_SYNC_DEBUG=1 routes every native call through a synchronising proxy; results are
    unchanged and host-side validation errors still surface with their message."""
    import importlib

    nat = importlib.import_module("docker_dist_nn_amd.utils.native")

    monkeypatch.setenv("DNN_SYNC_DEBUG", "1")
    monkeypatch.setattr(nat, "_debug", None)
    assert type(nat.native()).__name__ == "_SyncDebug"
    g = torch.Generator().manual_seed(3)
    x = torch.randn(128, 64, generator=g).to(torch.bfloat16).to(dev)
    w = torch.randn(64, 64, generator=g).to(torch.bfloat16).to(dev)
    b = torch.randn(64, generator=g).to(dev)
    y = torch.empty(128, 64, dtype=torch.bfloat16, device=dev)
    ops.linear_fwd(x, w, b, y, act="relu")
    ref = torch.relu(x.float() @ w.float().t() + b)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    with pytest.raises((RuntimeError, ValueError)):
        ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=128, N=64, K=63)


@pytest.mark.parametrize("la,lb", LAYOUTS)
@pytest.mark.parametrize("ns", [3, 4, 5, "big5"])
def test_pipeline_depth_bitwise(dev, la, lb, ns):
    """NS-stage LDS pipelines only change WHEN tiles are loaded, never the MFMA order: output
    must equal the 2-stage kernel bit for bit, including K shorter than the pipeline (nk < NS)
    and uneven split-K ranges. 5 = the asymmetric ring (A 3 deep, B 2 deep), also on the
    8-wave tiles ("big5")."""
    tiles = TILES
    if ns == "big5":
        ns, tiles = 5, BIG
    gen = torch.Generator().manual_seed(17 + ns + 4 * la + 2 * lb)
    for (bm, bn) in tiles:
        for K in (64, 128, 192, 320):
            M, N = 256, 256
            a = _storage(la, M, K, gen, dev, False)
            b = _storage(lb, N, K, gen, dev, False)
            bias = torch.randn(N, generator=gen).to(dev)
            c2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            cn = torch.empty_like(c2)
            for c, st in ((c2, 2), (cn, ns)):
                ops.gemm(a, b, c, layout_a=la, layout_b=lb, M=M, N=N, K=K, bias=bias,
                         act="relu", tiles=(bm, bn), stages=st)
            assert torch.equal(c2, cn), (bm, bn, K)
    # uneven split-K into fp32 slabs (batch contraction)
    R, S = 64 * 23, 5
    a = _storage(la, 128, R, gen, dev, False)
    b = _storage(lb, 128, R, gen, dev, False)
    s2 = torch.empty(S, 128, 128, device=dev)
    sn = torch.empty_like(s2)
    for c, st in ((s2, 2), (sn, ns)):
        ops.gemm(a, b, c, layout_a=la, layout_b=lb, M=128, N=128, K=R, k_total=R, splits=S,
                 tiles=(64, 64), stages=st)
    assert torch.equal(s2, sn)


RP = [((256, 256), 6), ((256, 128), 6), ((128, 128), 6), ((128, 64), 6), ((64, 64), 6),
      ((256, 256), 9), ((256, 128), 9), ((128, 128), 9), ((128, 64), 9), ((64, 64), 9),
      ((256, 256), 11), ((256, 128), 11), ((128, 128), 11)]


@pytest.mark.parametrize("la,lb", LAYOUTS)
def test_register_prefetch_bitwise(dev, la, lb):
    """Register-prefetched main loop (stage codes 6 / 9 / 11: the next half's fragments are read
    under the current half's MFMAs, strength-reduced LDS-DMA issued from asm, past-the-end
    restaging, accumulators in VGPRs) keeps the
    MFMA order of the 2-stage kernel: bit-identical for nk = 1, 2, 3, 5, 13, partial edge tiles
    and uneven split-K."""
    gen = torch.Generator().manual_seed(43 + 4 * la + 2 * lb)
    for (bm, bn), code in RP:
        for K in (64, 128, 192, 320, 832):
            M, N = 320, 264  # partial edge tiles in both dimensions
            a = _storage(la, M, K, gen, dev, False)
            b = _storage(lb, N, K, gen, dev, False)
            bias = torch.randn(N, generator=gen).to(dev)
            c2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            cn = torch.empty_like(c2)
            for c, st in ((c2, 2), (cn, code)):
                ops.gemm(a, b, c, layout_a=la, layout_b=lb, M=M, N=N, K=K, bias=bias,
                         act="relu", tiles=(bm, bn), stages=st)
            assert torch.equal(c2, cn), (bm, bn, code, K)
        R, S = 64 * 23, 5
        a = _storage(la, bm, R, gen, dev, False)
        b = _storage(lb, bn, R, gen, dev, False)
        s2 = torch.empty(S, bm, bn, device=dev)
        sn = torch.empty_like(s2)
        for c, st in ((s2, 2), (sn, code)):
            ops.gemm(a, b, c, layout_a=la, layout_b=lb, M=bm, N=bn, K=R, k_total=R, splits=S,
                     tiles=(bm, bn), stages=st)
        assert torch.equal(s2, sn), (bm, bn, code)
    # register-direct epilogue (codes 9 / 11): ReLU dgrad from the activation + colsum
    for (bm, bn), code in RP:
        if code < 9:
            continue
        M, N, K = 320, 264, 192
        a = _storage(la, M, K, gen, dev, False)
        b = _storage(lb, N, K, gen, dev, False)
        aux = torch.randn(M, N, generator=gen).to(torch.bfloat16).to(dev)
        outs, sums = [], []
        for st in (2, code):
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            cs = torch.empty(-(-M // bm), N, device=dev)
            ops.gemm(a, b, c, layout_a=la, layout_b=lb, M=M, N=N, K=K, aux=aux, act="relu",
                     tiles=(bm, bn), stages=st, colsum=cs)
            outs.append(c)
            sums.append(cs)
        assert torch.equal(outs[0], outs[1]), (bm, bn, code)
        # column sums: same values, summed in another order (per-wave butterflies + wave rows)
        torch.testing.assert_close(sums[0], sums[1], rtol=1e-5, atol=1e-3)
    # 1-bit ReLU masks through the register-direct epilogue: the forward writes the mask of
    # its stored output, a dgrad applies one instead of reading the activation
    for (bm, bn), code in RP:
        if code < 9:
            continue
        M, N, K = 320, 264, 192
        a = _storage(la, M, K, gen, dev, False)
        b = _storage(lb, N, K, gen, dev, False)
        bias = torch.randn(N, generator=gen).to(dev)
        res = []
        for st in (2, code):
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            m = torch.full((M, 40), 0xAA, device=dev, dtype=torch.uint8)
            ops.gemm(a, b, c, layout_a=la, layout_b=lb, M=M, N=N, K=K, bias=bias, act="relu",
                     tiles=(bm, bn), stages=st, mask_out=m)
            d = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ops.gemm(a, b, d, layout_a=la, layout_b=lb, M=M, N=N, K=K, act="relu",
                     tiles=(bm, bn), stages=st, mask_in=m)
            res.append((c, m, d))
        (c2, m2, d2), (cn, mn, dn) = res
        assert torch.equal(c2, cn) and torch.equal(m2, mn) and torch.equal(d2, dn), (bm, bn, code)
        blocked = mn.view(-1).view(M // 16, 40, 16)  # row-block-major mask bytes
        assert torch.all(blocked[:, 33:, :] == 0xAA)  # chunks past N/8 untouched
        assert torch.equal(ops.relu_mask_bits(mn, M, N), cn > 0)
        # fragment-order masks (ld_mask < 0): same outputs, one wide access per lane
        if (bm, bn) in ops.kernels.FRAG_WAVES:
            fm = ops.FragMask.alloc(M, N, (bm, bn), dev)
            cf = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ops.gemm(a, b, cf, layout_a=la, layout_b=lb, M=M, N=N, K=K, bias=bias, act="relu",
                     tiles=(bm, bn), stages=code, mask_out=fm)
            df = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ops.gemm(a, b, df, layout_a=la, layout_b=lb, M=M, N=N, K=K, act="relu",
                     tiles=(bm, bn), stages=code, mask_in=fm)
            assert torch.equal(cf, cn) and torch.equal(df, dn), ("frag", bm, bn, code)
            assert torch.equal(fm.bits(), cn > 0), ("frag bits", bm, bn, code)
            if la == KMAJ:  # rows from a tile boundary on: a byte range of the same buffer
                sub = fm[slice(bm, M)]
                ds = torch.empty(M - bm, N, device=dev, dtype=torch.bfloat16)
                ops.gemm(a[bm:], b, ds, layout_a=la, layout_b=lb, M=M - bm, N=N, K=K,
                         act="relu", tiles=(bm, bn), stages=code, mask_in=sub)
                assert torch.equal(ds, dn[bm:]), ("frag rows", bm, bn, code)
            with pytest.raises(ValueError, match="fragment mask"):
                ops.gemm(a, b, df, layout_a=la, layout_b=lb, M=M, N=N, K=K, act="relu",
                         tiles=(bm, bn), stages=2, mask_in=fm)
    # and against fp32 once (the 2-stage kernel itself is pinned by the tests above)
    M, N, K = 256, 256, 832
    a = _storage(la, M, K, gen, dev, False)
    b = _storage(lb, N, K, gen, dev, False)
    c = torch.empty(M, N, device=dev)
    ops.gemm(a, b, c, layout_a=la, layout_b=lb, M=M, N=N, K=K, tiles=(256, 256), stages=6)
    ref = _logical(a, la, M, K) @ _logical(b, lb, N, K).t()
    torch.testing.assert_close(c, ref, rtol=1e-3, atol=1e-3)


def test_pipeline_depth_rejects_bad_stages(dev):
    a = torch.zeros(128, 64, device=dev, dtype=torch.bfloat16)
    c = torch.zeros(128, 128, device=dev)
    with pytest.raises(ValueError, match="stages"):
        ops.gemm(a, a, c, layout_a=KMAJ, layout_b=KMAJ, M=128, N=128, K=64, stages=11)
    with pytest.raises(ValueError, match="stages"):  # no 3-deep 256x256 ring
        ops.gemm(a, a, c, layout_a=KMAJ, layout_b=KMAJ, M=128, N=128, K=64, stages=7,
                 tiles=(256, 256))



@pytest.mark.parametrize("M", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("N,K", [(10, 832), (1024, 1024), (64, 8192), (300, 4104)])
def test_gemv_matches_fp32(dev, M, N, K):
    """Serving-size layer kernel vs torch fp32: all row counts 1..8 (rows beyond M untouched),
    K tails past the 4x512 unroll, bias + activation, bf16 and fp32 outputs."""
    gen = torch.Generator().manual_seed(M * 1000 + N + K)
    x = torch.randn(M, K, generator=gen).to(torch.bfloat16).to(dev)
    w = (torch.randn(N, K, generator=gen) / K ** 0.5).to(torch.bfloat16).to(dev)
    b = torch.randn(N, generator=gen).to(dev)
    ref = x.float() @ w.float().t() + b
    for act, fn in (("relu", torch.relu), ("sigmoid", torch.sigmoid), ("linear", lambda t: t)):
        y = torch.full((M + 1, N), 7.0, device=dev)
        ops.gemv(x, w, b, y, act=act)
        torch.testing.assert_close(y[:M], fn(ref), rtol=1e-3, atol=1e-3)
        assert torch.all(y[M] == 7.0)  # row beyond M untouched
    yb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    ops.linear_fwd(x, w, b, yb, act="relu")  # dispatches to gemv for <= 8 rows
    torch.testing.assert_close(yb.float(), torch.relu(ref), rtol=1.6e-2, atol=1e-2)


@pytest.mark.parametrize("rows,cols", [(64, 64), (512, 832), (1024, 192)])
def test_transpose_bf16(dev, rows, cols):
    gen = torch.Generator().manual_seed(rows + cols)
    src = torch.randn(rows, cols, generator=gen).to(torch.bfloat16).to(dev)
    dst = torch.full((cols, rows), 7.0, dtype=torch.bfloat16, device=dev)
    ops.transpose_bf16(src, dst)
    assert torch.equal(dst, src.t())


@pytest.mark.parametrize("M,N,K,tiles", [(512, 128, 832, None), (1024, 1024, 1024, None),
                                         (4096, 1024, 1024, (256, 256))])
def test_dgrad_transposed_weight_bitwise(dev, M, N, K, tiles):
    """dgrad through the transposed weight shadow (both operands contraction-contiguous) equals
    the transposing-read dgrad bit for bit: same fragments, same MFMA k order; epilogue with the
    ReLU derivative and the bias-gradient partials included."""
    gen = torch.Generator().manual_seed(M + N + K)
    dz = torch.randn(M, N, generator=gen).to(torch.bfloat16).to(dev)
    w = torch.randn(N, K, generator=gen).to(torch.bfloat16).to(dev)
    wt = torch.empty(K, N, dtype=torch.bfloat16, device=dev)
    ops.transpose_bf16(w, wt)
    y_prev = torch.randn(M, K, generator=gen).clamp_min(0).to(torch.bfloat16).to(dev)
    bm = ops.dgrad_tiles(M, K, N)[0]
    outs = []
    for use_t in (False, True):
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        part = torch.zeros(M // bm, K, device=dev)
        ops.linear_dgrad(dz, w, dx, y_prev=y_prev, act_prev="relu", colsum=part,
                         wt=wt if use_t else None)
        outs.append((dx, part))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    ref = (dz.float() @ w.float()) * (y_prev.float() > 0)
    torch.testing.assert_close(outs[1][0].float(), ref, rtol=2e-2, atol=2e-2 * K ** 0.5)


@pytest.mark.parametrize("M,N,K,tiles", [(512, 256, 832, (256, 256)), (384, 192, 128, (128, 64)),
                                         (296, 136, 64, (64, 64))])
def test_gemm_transposed_second_output(dev, M, N, K, tiles):
    """ct (the transposed bf16 copy written by the staged epilogue) equals C^T bit for bit,
    including partial edge tiles and a column-slice destination (a micro-batch of a
    [N][rows] buffer)."""
    gen = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, K, generator=gen).to(torch.bfloat16).to(dev)
    w = torch.randn(N, K, generator=gen).to(torch.bfloat16).to(dev)
    b = torch.randn(N, generator=gen).to(dev)
    y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    big = torch.full((N, 2 * M + 8), 3.0, dtype=torch.bfloat16, device=dev)
    ct = big[:, M:2 * M]  # column slice: ld_ct = 2M + 8
    ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, bias=b, act="relu",
             tiles=tiles, ct=ct)
    assert torch.equal(ct, y.t())
    assert torch.all(big[:, :M] == 3.0) and torch.all(big[:, 2 * M:] == 3.0)


def test_wgrad_kmajor_bitwise_equals_transposing(dev):
    """K-major wgrad on transposed copies == the transposing-read wgrad, bit for bit."""
    gen = torch.Generator().manual_seed(5)
    R, N, K = 2048, 512, 768
    dz = torch.randn(R, N, generator=gen).to(torch.bfloat16).to(dev)
    x = torch.randn(R, K, generator=gen).to(torch.bfloat16).to(dev)
    for splits in (1, 3):
        a = torch.empty(splits, N, K, device=dev)
        b = torch.empty(splits, N, K, device=dev)
        ops.linear_wgrad(dz, x, a, splits=splits)
        ops.linear_wgrad(dz, x, b, splits=splits, dzt=dz.t().contiguous(), xt=x.t().contiguous())
        assert torch.equal(a, b)


def test_transpose_multi(dev):
    gen = torch.Generator().manual_seed(3)
    shapes = [(64, 64), (512, 832), (1024, 192), (128, 1024)] * 5  # > 16 jobs: two launches
    srcs = [torch.randn(r, c, generator=gen).to(torch.bfloat16).to(dev) for r, c in shapes]
    dsts = [torch.zeros(c, r, dtype=torch.bfloat16, device=dev) for r, c in shapes]
    ops.transpose_multi(list(zip(srcs, dsts)))
    for s_, d_ in zip(srcs, dsts):
        assert torch.equal(d_, s_.t())


@pytest.mark.parametrize("rows,cols", [(1, 64), (300, 512), (64, 1024), (33, 136)])
def test_fp8_boundary_kernels_match_reference(dev, rows, cols):
    """gfx950 e4m3 row quantisation (v_cvt_pk_fp8_f32, OCP encoding) vs torch float8_e4m3fn:
    identical scales; codes identical except rare one-step rounding ties (the hardware and
    torch's software conversion may break exact ties / subnormal rounding differently), so
    the dequantised values agree within one e4m3 step."""
    gen = torch.Generator().manual_seed(rows * cols)
    x = (torch.randn(rows, cols, generator=gen) * 3).to(torch.bfloat16)
    if rows > 2:
        x[1] = 0
    q_c, s_c = torch.empty(rows, cols, dtype=torch.uint8), torch.empty(rows)
    ops.quant_rows_fp8(x, q_c, s_c)
    xd = x.to(dev)
    q_g = torch.empty(rows, cols, dtype=torch.uint8, device=dev)
    s_g = torch.empty(rows, device=dev)
    ops.quant_rows_fp8(xd, q_g, s_g)
    assert torch.equal(s_g.cpu(), s_c)
    assert (q_g.cpu() != q_c).float().mean() < 2e-3
    y_c, y_g = torch.empty_like(x), torch.empty_like(xd)
    ops.dequant_rows_fp8(q_c, s_c, y_c)
    ops.dequant_rows_fp8(q_g, s_g, y_g)
    yc, yg = y_c.float(), y_g.cpu().float()
    amax = x.float().abs().amax(1, keepdim=True)
    assert torch.all((yg - yc).abs() <= 0.125 * yc.abs() + amax * 2.0 ** -9 / 448 * 2 + 1e-6)
    # and the GPU dequantiser itself is exact on the same codes
    y_g2 = torch.empty_like(xd)
    ops.dequant_rows_fp8(q_c.to(dev), s_c.to(dev), y_g2)
    assert torch.equal(y_g2.cpu(), y_c)
