"""1-bit ReLU masks (forward epilogue writes them, dgrad epilogue reads them instead of the bf16
activation): bitwise identical to the activation-derivative path, at kernel and engine level."""
import importlib

import pytest
import torch

from docker_dist_nn_amd import ops
from docker_dist_nn_amd.ops import KMAJ, MNMAJ

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tile,stages", [((256, 64), 2), ((128, 128), 2), ((64, 64), 3),
                                         ((256, 256), 2), ((256, 256), 8)])
def test_mask_roundtrip_bitwise(dev, tile, stages):
    gen = torch.Generator().manual_seed(1 + tile[0] + tile[1] + stages)
    M, K, N = 1024 + 64, 320, 520  # partial tiles; N % 8 == 0
    x = torch.randn(M, K, generator=gen).to(torch.bfloat16).to(dev)
    w = (torch.randn(N, K, generator=gen) * 0.1).to(torch.bfloat16).to(dev)
    b = torch.randn(N, generator=gen).to(dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    mask = torch.full((M, N // 8 + 3), 0xAA, device=dev, dtype=torch.uint8)
    ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, bias=b, act="relu",
             tiles=tile, stages=stages, mask_out=mask)
    assert torch.equal(ops.relu_mask_bits(mask, M, N), y > 0)
    ld = mask.shape[1]  # row-block-major: [M/16][ld][16]; chunks past N/8 never written
    blocked = mask.view(-1).view(M // 16, ld, 16)
    assert torch.all(blocked[:, N // 8:, :] == 0xAA)
    # dgrad: dz[M][R2] . w2[R2][N] with the relu derivative of y (aux) vs its mask
    R2 = 192
    dz = torch.randn(M, R2, generator=gen).to(torch.bfloat16).to(dev)
    w2 = (torch.randn(R2, N, generator=gen) * 0.1).to(torch.bfloat16).to(dev)
    tm = -(-M // tile[0])
    outs = []
    for use_mask in (False, True):
        dx = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        cs = torch.empty(tm, N, device=dev)
        ops.gemm(dz, w2, dx, layout_a=KMAJ, layout_b=MNMAJ, M=M, N=N, K=R2, act="relu",
                 aux=None if use_mask else y, mask_in=mask if use_mask else None, tiles=tile,
                 stages=stages, colsum=cs)
        outs.append((dx, cs))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


def test_mask_rejected_where_unsupported(dev):
    x = torch.zeros(256, 64, device=dev, dtype=torch.bfloat16)
    y = torch.zeros(256, 64, device=dev, dtype=torch.bfloat16)
    m = torch.zeros(256, 8, device=dev, dtype=torch.uint8)
    with pytest.raises(ValueError):  # sigmoid has no 1-bit derivative
        ops.gemm(x, x, y, layout_a=KMAJ, layout_b=KMAJ, M=256, N=64, K=64, act="sigmoid",
                 mask_out=m, tiles=(64, 64))
    with pytest.raises(ValueError):  # the persistent form's direct epilogue has no mask path
        ops.gemm(x, x, y, layout_a=KMAJ, layout_b=KMAJ, M=256, N=64, K=64, act="relu",
                 mask_out=m, tiles=(64, 64), persist=-1)


def test_engine_mask_path_bitwise_equals_activation_path(dev, monkeypatch):
    from docker_dist_nn_amd import NAMED_MODELS
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    x, y = synthetic_mnist(4096, seed=2)
    xb = torch.zeros(4096, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xb, yb = xb.to(dev), torch.from_numpy(y).to(dev)
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("DNN_RELU_MASK", flag)
        tr = Trainer(NAMED_MODELS["mnist-fcnn"], micro_batch=2048, num_micro=2,
                     optim=OptimConfig(lr=0.1), device=dev)
        assert (tr.stages[0].relu_mask[0] is not None) == (flag == "1")
        losses = []
        for _ in range(3):
            tr.set_batch(xb, yb)
            tr.step()
            losses.append(tr.loss())
        res.append((losses, tr.stages[0].params.master.clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])


def test_engine_fragment_mask_bitwise_equals_activation_path(dev, monkeypatch):
    """DNN_RELU_MASK=2 on the headline shape (65536 rows: the tuned table runs the 784->512
    forward and the 256->512 dgrad as the same 256x256 register-direct tile, so the
    fragment-order mask applies): the same losses and weights as reading the activation."""
    from docker_dist_nn_amd import NAMED_MODELS
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    R = 65536
    x, y = synthetic_mnist(R, seed=3)
    xb = torch.zeros(R, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xb, yb = xb.to(dev), torch.from_numpy(y).to(dev)
    res = []
    for flag in ("0", "2"):
        monkeypatch.setenv("DNN_RELU_MASK", flag)
        tr = Trainer(NAMED_MODELS["mnist-fcnn"], micro_batch=R, num_micro=1,
                     optim=OptimConfig(lr=0.1), device=dev)
        m = tr.stages[0].relu_mask
        if flag == "2":
            assert isinstance(m[0], ops.FragMask) and m[0].tiles == (256, 256)
            assert all(v is None for v in m[1:])  # the tail's own dgrads read activations
        else:
            assert all(v is None for v in m)
        losses = []
        for _ in range(3):
            tr.set_batch(xb, yb)
            tr.step()
            losses.append(tr.loss())
        res.append((losses, tr.stages[0].params.master.clone()))
        del tr
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])


def test_engine_auto_mask_only_for_wide_layers_bitwise(dev, monkeypatch):
    """DNN_RELU_MASK=auto (the default): fragment-order masks only for hidden layers at least
    RELU_MASK_AUTO_WIDTH wide (here layer 0, 1024 wide; layer 1, 512 wide, reads its
    activation), and the same losses and weights as reading every activation."""
    from docker_dist_nn_amd import MLPSpec
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer
    from docker_dist_nn_amd.engine.stage import RELU_MASK_AUTO_WIDTH

    R = 16384
    spec = MLPSpec.parse("784-1024-512-10")
    x, y = synthetic_mnist(R, seed=5)
    xb = torch.zeros(R, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xb, yb = xb.to(dev), torch.from_numpy(y).to(dev)
    res = []
    for flag in ("0", "auto"):
        monkeypatch.setenv("DNN_RELU_MASK", flag)
        tr = Trainer(spec, micro_batch=R, num_micro=1, optim=OptimConfig(lr=0.1), device=dev)
        st = tr.stages[0]
        for g, m in zip(st.geoms, st.relu_mask):
            if flag == "0" or g.np_ < RELU_MASK_AUTO_WIDTH:
                assert m is None
        losses = []
        for _ in range(3):
            tr.set_batch(xb, yb)
            tr.step()
            losses.append(tr.loss())
        tr.flush()
        res.append((losses, st.params.master.clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])
