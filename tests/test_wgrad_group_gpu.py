"""Grouped weight-gradient launch (gemm.hip gemm_group_kernel): several split-K wgrads sharing a
tile configuration in one launch, bitwise equal to one launch per layer, at kernel level and in
whole training steps (headline model at batch 65536 and the batch-64 recipe, SGD and Adam)."""
import pytest
import torch

from docker_dist_nn_amd import ops

pytestmark = pytest.mark.gpu


def test_group_kernel_bitwise_equals_separate(dev):
    g = torch.Generator(device=dev).manual_seed(4)
    R = 8192
    shapes = [(256, 512, 8), (128, 256, 16), (64, 128, 4)]  # (N, K, splits): kernel-level, any size
    dz = [torch.randn(R, n, device=dev, generator=g).to(torch.bfloat16) for n, _, _ in shapes]
    x = [torch.randn(R, k, device=dev, generator=g).to(torch.bfloat16) for _, k, _ in shapes]
    outs = []
    for grouped in (False, True):
        slabs = [torch.full((s, n, k), 5.0, device=dev) for n, k, s in shapes]
        if grouped:
            probs = [(ops.kernels._p(d), d.stride(0), ops.kernels._p(xx), xx.stride(0),
                      ops.kernels._p(sl), sl.stride(1), sl.stride(0), n, k, R, R, 0, s)
                     for d, xx, sl, (n, k, s) in zip(dz, x, slabs, shapes)]
            ops.kernels.native().gemm_bf16_group(probs, ops.MNMAJ, ops.MNMAJ, 1, 64, 64, 2,
                                                 torch.cuda.current_stream().cuda_stream)
        else:
            for d, xx, sl, (n, k, s) in zip(dz, x, slabs, shapes):
                ops.gemm(d, xx, sl, layout_a=ops.MNMAJ, layout_b=ops.MNMAJ, M=n, N=k, K=R,
                         k_total=R, splits=s, tiles=(64, 64), stages=2)
        outs.append(slabs)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("model,batch,opt", [("mnist-fcnn", 65536, "sgd"),
                                             ("784-128-64-10", 64, "adam"),
                                             ("784-1024-1024-10", 4096, "sgd")])
def test_engine_grouped_wgrad_bitwise(dev, monkeypatch, model, batch, opt):
    from docker_dist_nn_amd import NAMED_MODELS, MLPSpec
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    spec = NAMED_MODELS.get(model) or MLPSpec.parse(model)
    x, y = synthetic_mnist(min(batch, 60000), seed=12)
    xb = torch.zeros(batch, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16).repeat(-(-batch // len(x)), 1)[:batch]
    yb = torch.from_numpy(y).repeat(-(-batch // len(y)))[:batch]
    xb, yb = xb.to(dev), yb.to(dev)
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("DNN_WGRAD_GROUP", flag)
        tr = Trainer(spec, micro_batch=batch, num_micro=1, optim=OptimConfig(name=opt, lr=1e-3),
                     device=dev)
        losses = []
        for _ in range(3):
            tr.set_batch(xb, yb)
            tr.step()
            losses.append(tr.loss())
        res.append((losses, tr.stages[0].params.master.clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])
