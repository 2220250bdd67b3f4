"""Persistent-workgroup GEMM (csrc/kernels/gemm_persist.hip) against fp32 PyTorch references.

Integer operands make every product and partial sum exact in fp32, so the fp32 outputs must
match bit for bit: that catches a wrong fragment map, a wrong permlane16_swap pairing in the
16-byte bf16 stores, or a tile/k-range mix-up across the tiles one workgroup walks. Workgroup
counts below the tile count force multi-tile runs (the cross-tile LDS ring)."""
import pytest
import torch

from docker_dist_nn_amd import ops
from docker_dist_nn_amd.ops import KMAJ, MNMAJ

pytestmark = pytest.mark.gpu

LAYOUTS = [(KMAJ, KMAJ), (KMAJ, MNMAJ), (MNMAJ, MNMAJ), (MNMAJ, KMAJ)]
TILES = [(128, 128), (128, 64), (64, 128), (64, 64), (256, 256), (256, 128), (128, 256),
         (256, 64)]


def _storage(layout, mn, k, gen, dev, integer=True):
    shape = (mn, k) if layout == KMAJ else (k, mn)
    t = (torch.randint(-3, 4, shape, generator=gen, dtype=torch.int32).float() if integer
         else torch.randn(shape, generator=gen))
    return t.to(torch.bfloat16).to(dev)


def _logical(t, layout, mn, k):
    return t.float()[:mn, :k] if layout == KMAJ else t.float()[:k, :mn].t()


@pytest.mark.parametrize("la,lb", LAYOUTS)
@pytest.mark.parametrize("bm,bn", TILES)
@pytest.mark.parametrize("persist", [-1, 3])
def test_persist_exact(dev, la, lb, bm, bn, persist):
    gen = torch.Generator().manual_seed(17 + bm + 3 * bn + 10 * la + lb + persist)
    # partial edge tiles in both dims: M = 2 bm + 40, N = 2 bn + 8 (multiple of 8)
    M, N, K = 2 * bm + 40, 2 * bn + 8, 320
    a = _storage(la, M, K, gen, dev)
    b = _storage(lb, N, K, gen, dev)
    ref = _logical(a, la, M, K) @ _logical(b, lb, N, K).t()
    # fp32 out into a wider buffer: nothing outside [M][N] may be written
    big = torch.full((M + 8, N + 16), -1.0, device=dev)
    ops.gemm(a, b, big, layout_a=la, layout_b=lb, M=M, N=N, K=K, tiles=(bm, bn), persist=persist)
    assert torch.equal(big[:M, :N], ref), (big[:M, :N] - ref).abs().max()
    assert torch.all(big[M:] == -1.0) and torch.all(big[:, N:] == -1.0)
    # bf16 out + bias + relu + colsum partials
    bias = torch.randint(-4, 5, (N,), generator=gen).float().to(dev)
    y = torch.full((M, N + 8), 5.0, device=dev, dtype=torch.bfloat16)
    tm = -(-M // bm)
    cs = torch.full((tm, N), 7.0, device=dev)
    ops.gemm(a, b, y, layout_a=la, layout_b=lb, M=M, N=N, K=K, bias=bias, act="relu",
             tiles=(bm, bn), colsum=cs, persist=persist)
    yr = (ref + bias).clamp_min(0).to(torch.bfloat16)
    assert torch.equal(y[:, :N], yr)
    assert torch.all(y[:, N:] == 5.0)
    pad = torch.zeros(tm * bm - M, N, device=dev)
    want = torch.cat([yr.float(), pad]).view(tm, bm, N).sum(1)
    torch.testing.assert_close(cs, want, rtol=1e-5, atol=1e-2)
    # split-K fp32 slabs, then accumulate on top
    S = 3
    slabs = torch.empty(S, M, N, device=dev)
    ops.gemm(a, b, slabs, layout_a=la, layout_b=lb, M=M, N=N, K=K, k_total=K, splits=S,
             tiles=(bm, bn), persist=persist)
    assert torch.equal(slabs.sum(0), ref)
    ops.gemm(a, b, slabs, layout_a=la, layout_b=lb, M=M, N=N, K=K, k_total=K, splits=S,
             tiles=(bm, bn), persist=persist, accumulate=True)
    assert torch.equal(slabs.sum(0), 2 * ref)


@pytest.mark.parametrize("bm,bn", [(256, 256), (128, 128), (256, 64)])
@pytest.mark.parametrize("act", ["relu", "sigmoid"])
@pytest.mark.parametrize("wt", [False, True])
def test_persist_dgrad_mask_equals_classic(dev, bm, bn, act, wt):
    """dgrad epilogue (activation derivative from the stored output) on random data: the
    persistent form rounds the same fp32 values as the one-tile form (ReLU: the mask applied
    after the 16-lane swap, 16-byte activation reads). ``wt``: B is the transposed weight
    copy (K-major, the engine's default dgrad operand)."""
    gen = torch.Generator().manual_seed(3 + bm + bn)
    M, N, K = 1024, 512, 256  # dx[M][N] = dz[M][K] . w[K][N]
    dz = torch.randn(M, K, generator=gen).to(torch.bfloat16).to(dev)
    w = (torch.randn(K, N, generator=gen) * 0.1).to(torch.bfloat16).to(dev)
    y = torch.rand(M, N, generator=gen).to(torch.bfloat16).to(dev)
    if act == "relu":
        y = (y - 0.5).clamp_min(0).to(torch.bfloat16)
    outs = []
    for persist in (0, -1):
        dx = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        cs = torch.empty(M // bm, N, device=dev)
        b, lb = (w.t().contiguous(), KMAJ) if wt else (w, MNMAJ)
        ops.gemm(dz, b, dx, layout_a=KMAJ, layout_b=lb, M=M, N=N, K=K, aux=y, act=act,
                 tiles=(bm, bn), colsum=cs, persist=persist)
        outs.append((dx, cs))
    ref = dz.float() @ w.float()
    ref = ref * (y.float() > 0) if act == "relu" else ref * y.float() * (1 - y.float())
    torch.testing.assert_close(outs[1][0].float(), ref, rtol=1.6e-2, atol=2e-2)
    torch.testing.assert_close(outs[1][0], outs[0][0], rtol=0, atol=0)
    torch.testing.assert_close(outs[1][1], outs[0][1], rtol=1e-5, atol=1e-3)


def test_persist_step_ops_env(dev, monkeypatch):
    """The linear_* ops honour DNN_GEMM_PERSIST / the tuned table's "persist" field."""
    monkeypatch.setitem(ops.kernels.PERSIST, "fwd", 1)
    gen = torch.Generator().manual_seed(0)
    x = torch.randn(4096, 832, generator=gen).to(torch.bfloat16).to(dev)
    w = (torch.randn(512, 832, generator=gen) * 0.05).to(torch.bfloat16).to(dev)
    b = torch.randn(512, generator=gen).to(dev)
    y = torch.empty(4096, 512, device=dev, dtype=torch.bfloat16)
    ops.linear_fwd(x, w, b, y, act="relu")
    ref = (x.float() @ w.float().t() + b).clamp_min(0)
    torch.testing.assert_close(y.float(), ref, rtol=1.6e-2, atol=2e-2)
