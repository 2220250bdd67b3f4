"""Ping-pong 256x256 GEMM (csrc/kernels/gemm_pp.hip, stages=8) against fp32 references.

Integer operands make every partial sum exact in fp32, so outputs must match bit for bit:
that catches a wrong half-tile image swizzle, a ring slot reused too early (stale k-halves),
a wrong ping-pong wait count, or a fragment-map error. K values cover the prologue-only path
(K = 64: fewer half-tiles than the look-ahead), odd k-step counts and long streams."""
import pytest
import torch

from docker_dist_nn_amd import ops
from docker_dist_nn_amd.ops import KMAJ, MNMAJ

pytestmark = pytest.mark.gpu

LAYOUTS = [(KMAJ, KMAJ), (KMAJ, MNMAJ), (MNMAJ, MNMAJ), (MNMAJ, KMAJ)]


def _storage(layout, mn, k, gen, dev, integer=True):
    shape = (mn, k) if layout == KMAJ else (k, mn)
    t = (torch.randint(-3, 4, shape, generator=gen, dtype=torch.int32).float() if integer
         else torch.randn(shape, generator=gen))
    return t.to(torch.bfloat16).to(dev)


def _logical(t, layout, mn, k):
    return t.float()[:mn, :k] if layout == KMAJ else t.float()[:k, :mn].t()


@pytest.mark.parametrize("la,lb", LAYOUTS)
@pytest.mark.parametrize("K", [64, 192, 832, 2048])
def test_pp_exact(dev, la, lb, K):
    gen = torch.Generator().manual_seed(11 + K + 10 * la + lb)
    M, N = 3 * 256 + 40, 2 * 256 + 8  # partial edge tiles in both dims
    a = _storage(la, M, K, gen, dev)
    b = _storage(lb, N, K, gen, dev)
    ref = _logical(a, la, M, K) @ _logical(b, lb, N, K).t()
    big = torch.full((M + 8, N + 16), -1.0, device=dev)
    ops.gemm(a, b, big, layout_a=la, layout_b=lb, M=M, N=N, K=K, tiles=(256, 256), stages=8)
    assert torch.equal(big[:M, :N], ref), (big[:M, :N] - ref).abs().max()
    assert torch.all(big[M:] == -1.0) and torch.all(big[:, N:] == -1.0)
    bias = torch.randint(-4, 5, (N,), generator=gen).float().to(dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    tm = -(-M // 256)
    cs = torch.full((tm, N), 7.0, device=dev)
    ops.gemm(a, b, y, layout_a=la, layout_b=lb, M=M, N=N, K=K, bias=bias, act="relu",
             tiles=(256, 256), colsum=cs, stages=8)
    yr = (ref + bias).clamp_min(0).to(torch.bfloat16)
    assert torch.equal(y, yr)
    want = torch.cat([yr.float(), torch.zeros(tm * 256 - M, N, device=dev)]).view(tm, 256, N)
    torch.testing.assert_close(cs, want.sum(1), rtol=1e-5, atol=1e-2)
    if K >= 192:
        S = 3
        slabs = torch.empty(S, M, N, device=dev)
        ops.gemm(a, b, slabs, layout_a=la, layout_b=lb, M=M, N=N, K=K, k_total=K, splits=S,
                 tiles=(256, 256), stages=8)
        assert torch.equal(slabs.sum(0), ref)


def test_pp_dgrad_equals_classic(dev):
    """Random data, dgrad epilogue (relu derivative from the stored activation): the ping-pong
    loop accumulates in the same k order as the one-tile kernel -> identical bf16 output."""
    gen = torch.Generator().manual_seed(5)
    M, N, K = 2048, 1024, 1024
    dz = torch.randn(M, K, generator=gen).to(torch.bfloat16).to(dev)
    w = (torch.randn(K, N, generator=gen) * 0.05).to(torch.bfloat16).to(dev)
    y = (torch.rand(M, N, generator=gen) - 0.5).clamp_min(0).to(torch.bfloat16).to(dev)
    outs = []
    for stages in (2, 8):
        dx = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ops.gemm(dz, w, dx, layout_a=KMAJ, layout_b=MNMAJ, M=M, N=N, K=K, aux=y, act="relu",
                 tiles=(256, 256), stages=stages)
        outs.append(dx)
    ref = (dz.float() @ w.float()) * (y.float() > 0)
    torch.testing.assert_close(outs[1].float(), ref, rtol=1.6e-2, atol=2e-2)
    assert torch.equal(outs[0], outs[1])


def test_pp_rejects_other_tiles(dev):
    a = torch.zeros(256, 128, device=dev, dtype=torch.bfloat16)
    c = torch.zeros(256, 256, device=dev)
    with pytest.raises(ValueError):
        ops.gemm(a, a, c, layout_a=KMAJ, layout_b=KMAJ, M=256, N=256, K=128, tiles=(128, 128),
                 stages=8)

