"""Fused classifier tail (csrc/kernels/mlp_tail.hip): one launch = fwd of layer L-2, fwd + softmax
CE of layer L-1, dgrads of both. Its outputs must equal the four unfused kernels bit for bit
(h3, dz4, dz3, dz2); the bias-gradient partials are grouped per workgroup, so their totals are
compared with a tolerance, and against the fp32 CPU reference."""
import pytest
import torch

from docker_dist_nn_amd import ops

pytestmark = pytest.mark.gpu


def _case(rows, k3, n3, n4, n_cls, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.relu(torch.randn(rows, k3, generator=g)).to(torch.bfloat16)
    w3 = (torch.randn(n3, k3, generator=g) / k3 ** 0.5).to(torch.bfloat16)
    w4 = torch.zeros(n4, n3)
    w4[:n_cls] = torch.randn(n_cls, n3, generator=g) / n3 ** 0.5
    w4 = w4.to(torch.bfloat16)
    b3 = torch.randn(n3, generator=g) * 0.1
    b4 = torch.zeros(n4)
    b4[:n_cls] = torch.randn(n_cls, generator=g) * 0.1
    labels = torch.randint(0, n_cls, (rows,), generator=g, dtype=torch.int32)
    labels[::7] = -1  # padding rows
    return x, w3, b3, w4, b4, labels


def _run_tail(dev, x, w3, b3, w4, b4, labels, n_cls, scale, act="relu"):
    rows, k3 = x.shape
    n3, n4 = w3.shape[0], w4.shape[0]
    nb = ops.tail_blocks(rows)
    bf, f32 = torch.bfloat16, torch.float32
    out = dict(h3=torch.full((rows, n3), 7.0, dtype=bf, device=dev),
               dz4=torch.zeros(rows, n4, dtype=bf, device=dev),  # padding stays the caller's
               dz3=torch.full((rows, n3), 7.0, dtype=bf, device=dev),
               dz2=torch.full((rows, k3), 7.0, dtype=bf, device=dev),
               loss=torch.zeros(nb, dtype=f32, device=dev),
               corr=torch.zeros(nb, dtype=torch.int32, device=dev),
               cs4=torch.full((nb, n4), 7.0, dtype=f32, device=dev),
               cs3=torch.full((nb, n3), 7.0, dtype=f32, device=dev),
               cs2=torch.full((nb, k3), 7.0, dtype=f32, device=dev))
    t = [a.to(dev) for a in (x, w3, b3, w4, b4, labels)]
    ops.mlp_tail(*t, out["h3"], out["dz4"], out["dz3"], out["dz2"], n_cls, scale,
                 act3=act, act2=act, loss_part=out["loss"], correct=out["corr"],
                 cs4=out["cs4"], cs3=out["cs3"], cs2=out["cs2"])
    return out


def _unfused(dev, x, w3, b3, w4, b4, labels, n_cls, scale, act="relu"):
    rows, k3 = x.shape
    n3, n4 = w3.shape[0], w4.shape[0]
    x, w3, b3, w4, b4, labels = (a.to(dev) for a in (x, w3, b3, w4, b4, labels))
    bf, f32 = torch.bfloat16, torch.float32
    h3 = torch.empty(rows, n3, dtype=bf, device=dev)
    ops.linear_fwd(x, w3, b3, h3, act=act)
    nx = rows // ops.xent_tiles(rows, n4)[0]
    dz4 = torch.empty(rows, n4, dtype=bf, device=dev)
    loss = torch.zeros(nx, dtype=f32, device=dev)
    corr = torch.zeros(nx, dtype=torch.int32, device=dev)
    cs4 = torch.zeros(nx, n4, dtype=f32, device=dev)
    ops.linear_fwd_xent(h3, w4, b4, dz4, labels, n_cls, scale, loss, corr, colsum=cs4)
    dz3 = torch.empty(rows, n3, dtype=bf, device=dev)
    cs3 = torch.zeros(rows // ops.dgrad_tiles(rows, n3, n4)[0], n3, dtype=f32, device=dev)
    ops.linear_dgrad(dz4, w4, dz3, y_prev=h3, act_prev=act, colsum=cs3)
    dz2 = torch.empty(rows, k3, dtype=bf, device=dev)
    cs2 = torch.zeros(rows // ops.dgrad_tiles(rows, k3, n3)[0], k3, dtype=f32, device=dev)
    ops.linear_dgrad(dz3, w3, dz2, y_prev=x, act_prev=act, colsum=cs2)
    return dict(h3=h3, dz4=dz4, dz3=dz3, dz2=dz2, loss=loss, corr=corr, cs4=cs4, cs3=cs3,
                cs2=cs2)


@pytest.mark.parametrize("rows,k3,n3,n4,n_cls,act", [(4096, 256, 128, 64, 10, "relu"),
                                                     (65536, 256, 128, 64, 10, "relu"),
                                                     (1024, 64, 64, 64, 10, "relu"),
                                                     (2048, 128, 64, 128, 16, "relu"),
                                                     (512, 256, 64, 64, 3, "relu"),
                                                     (8192, 128, 128, 64, 1, "relu"),
                                                     (4096, 256, 128, 64, 10, "sigmoid"),
                                                     (1024, 64, 64, 128, 7, "linear")])
def test_tail_equals_unfused_kernels(dev, monkeypatch, rows, k3, n3, n4, n_cls, act):
    monkeypatch.setenv("DNN_BLAS", "0")  # the reference is the hand-written kernels
    case = _case(rows, k3, n3, n4, n_cls, seed=rows + k3 + n3 + n_cls)
    scale = 1.0 / rows
    got = _run_tail(dev, *case, n_cls, scale, act)
    want = _unfused(dev, *case, n_cls, scale, act)
    for k in ("h3", "dz4", "dz3", "dz2"):
        assert torch.equal(got[k], want[k]), (k, (got[k].float() - want[k].float()).abs().max())
    assert int(got["corr"].sum()) == int(want["corr"].sum())
    torch.testing.assert_close(got["loss"].sum(), want["loss"].sum(), rtol=1e-5, atol=1e-3)
    for k in ("cs4", "cs3", "cs2"):
        torch.testing.assert_close(got[k].sum(0), want[k].sum(0), rtol=1e-4, atol=1e-5)
    assert torch.all(got["cs4"][:, 16:] == 0)


def test_tail_matches_cpu_reference(dev):
    case = _case(2048, 256, 128, 64, 10, seed=5)
    got = _run_tail(dev, *case, 10, 1.0 / 2048)
    ref = _run_tail(torch.device("cpu"), *case, 10, 1.0 / 2048)
    for k in ("h3", "dz4", "dz3", "dz2"):
        torch.testing.assert_close(got[k].cpu().float(), ref[k].float(), rtol=2e-2, atol=2e-3)
    for k in ("cs4", "cs3", "cs2", "loss"):  # same per-workgroup row grouping as the kernel
        torch.testing.assert_close(got[k].cpu(), ref[k], rtol=2e-2, atol=2e-3)
    assert torch.equal(got["corr"].cpu(), ref["corr"])


def test_tail_rejects_bad_geometry(dev):
    x, w3, b3, w4, b4, labels = _case(1024, 512, 128, 64, 10, seed=3)
    with pytest.raises(ValueError):
        _run_tail(dev, x, w3, b3, w4, b4, labels, 10, 1e-3)


@pytest.mark.parametrize("num_micro", [1, 2])
def test_engine_tail_matches_unfused_training(dev, monkeypatch, num_micro):
    """Whole training steps with the fused tail vs the four unfused kernels. The bias gradients
    are summed in a different order, so the weights agree to rounding, not bit for bit."""
    from docker_dist_nn_amd import NAMED_MODELS
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    x, y = synthetic_mnist(4096, seed=4)
    xb = torch.zeros(4096, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xb, yb = xb.to(dev), torch.from_numpy(y).to(dev)
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("DNN_TAIL", flag)
        tr = Trainer(NAMED_MODELS["mnist-fcnn"], micro_batch=4096 // num_micro,
                     num_micro=num_micro, optim=OptimConfig(lr=0.1), device=dev)
        assert tr.stages[0].tail == (flag == "1")
        losses = []
        for _ in range(3):
            tr.set_batch(xb, yb)
            tr.step()
            losses.append(tr.loss())
        res.append((losses, tr.stages[0].params.master.clone()))
    for a, b in zip(res[0][0], res[1][0]):
        assert abs(a - b) <= 1e-4 * abs(a) + 1e-5
    torch.testing.assert_close(res[1][1], res[0][1], rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("schedule", ["1f1b", "gpipe"])
def test_loopback_pipeline_last_stage_uses_tail(dev, monkeypatch, schedule):
    """Two stages on one GPU, distribution [1, 3]: the last stage holds three layers, so its
    tail kernel produces the dZ that its own first layer's dgrad sends upstream."""
    from docker_dist_nn_amd import NAMED_MODELS
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    x, y = synthetic_mnist(4096, seed=9)
    xb = torch.zeros(4096, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xb, yb = xb.to(dev), torch.from_numpy(y).to(dev)
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("DNN_TAIL", flag)
        tr = Trainer(NAMED_MODELS["mnist-fcnn"], micro_batch=1024, num_micro=4, pp=2,
                     distribution=[1, 3], schedule=schedule, optim=OptimConfig(lr=0.1),
                     device=dev)
        assert tr.stages[-1].tail == (flag == "1") and not tr.stages[0].tail
        losses = []
        for _ in range(3):
            tr.set_batch(xb, yb)
            tr.step()
            losses.append(tr.loss())
        res.append((losses, torch.cat([s.params.master for s in tr.stages]).clone()))
    for a, b in zip(res[0][0], res[1][0]):
        assert abs(a - b) <= 1e-4 * abs(a) + 1e-5
    torch.testing.assert_close(res[1][1], res[0][1], rtol=1e-3, atol=1e-5)
