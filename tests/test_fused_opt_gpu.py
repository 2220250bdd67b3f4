"""The whole-step gradient reduction with the optimizer step fused into the same launch (native
plan segment FINO): bitwise equal to reduction + separate update, for SGD (momentum, weight
decay), Adam and AdamW (device-side step counter and learning rate)."""
import pytest
import torch

from docker_dist_nn_amd import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("opt", [dict(name="sgd", momentum=0.9, weight_decay=1e-4),
                                 dict(name="adam", weight_decay=1e-4),
                                 dict(name="adamw", weight_decay=1e-2)])
def test_engine_fused_reduce_update_bitwise(dev, monkeypatch, opt):
    from docker_dist_nn_amd import NAMED_MODELS
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    x, y = synthetic_mnist(4096, seed=8)
    xb = torch.zeros(4096, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xb, yb = xb.to(dev), torch.from_numpy(y).to(dev)
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("DNN_FUSE_FIN_SGD", flag)
        tr = Trainer(NAMED_MODELS["mnist-fcnn"], micro_batch=4096, num_micro=1,
                     optim=OptimConfig(lr=1e-3, **opt), device=dev)
        st = tr.stages[0]
        assert ("FINO" in st._prog.segments()) == (flag == "1")
        losses = []
        for _ in range(4):
            tr.set_batch(xb, yb)
            tr.step()
            losses.append(tr.loss())
        p = st.params
        res.append((losses, p.master.clone(), [s.clone() for s in p.state],
                    int(p.step_dev[0]) if p.step_dev is not None else None, p.step_count))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])
    for a, b in zip(res[0][2], res[1][2]):
        assert torch.equal(a, b)
    assert res[0][3] == res[1][3] and res[0][4] == res[1][4]


def test_reduce_multi_fused_adam_matches_separate_update(dev):
    g = torch.Generator(device=dev).manual_seed(2)
    n = 4096
    slabs = torch.randn(5, n, device=dev, generator=g)
    outs = []
    for fused in (False, True):
        grad = torch.zeros(n, device=dev)
        master = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
        m, v = torch.full((n,), 0.01, device=dev), torch.full((n,), 0.02, device=dev)
        shadow = torch.empty(n, device=dev, dtype=torch.bfloat16)
        step_dev = torch.full((1,), 6, device=dev, dtype=torch.int32)
        job = [(slabs, 5, n, n, grad, 0.5, False)]
        kw = dict(lr=3e-3, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-3, decoupled=True,
                  step_dev=step_dev)
        if fused:
            ops.reduce_multi(job, sgd=dict(grad=grad, master=master, mom=m, v=v, shadow=shadow,
                                           adam=True, **kw))
        else:
            ops.reduce_multi(job)
            ops.adam_update(master, grad, m, v, shadow, **kw)
        outs.append((grad, master, m, v, shadow))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("n_src,adam", [(5, False), (64, False), (18, True)])
def test_reduce_multi_writes_wt(dev, n_src, adam):
    """A job's W^T output (fused update only) is bitwise the transpose of the refreshed bf16
    shadow of that job's [rows][cols] weights; other jobs of the launch are unaffected."""
    rows, cols = 96, 832
    n = rows * cols
    gen = torch.Generator(device=dev).manual_seed(5)
    slabs = torch.randn(n_src, n, device=dev, generator=gen)
    bias_src = torch.randn(n_src, rows, device=dev, generator=gen)
    grad = torch.zeros(n + rows, device=dev)
    master = torch.randn(n + rows, device=dev, generator=gen)
    mom = torch.zeros(n + rows, device=dev)
    v = torch.full((n + rows,), 0.01, device=dev)
    shadow = torch.zeros(n + rows, device=dev, dtype=torch.bfloat16)
    wt = torch.zeros(cols, rows, device=dev, dtype=torch.bfloat16)
    jobs = [(slabs, n_src, n, n, grad[:n], 1.0, False, wt),
            (bias_src, n_src, rows, rows, grad[n:], 1.0, False)]
    sgd = dict(grad=grad, master=master, mom=mom, shadow=shadow, lr=0.05, momentum=0.9)
    if adam:
        sgd.update(adam=True, v=v, betas=(0.9, 0.99), eps=1e-8, step=3)
    ops.reduce_multi(jobs, sgd=sgd)
    torch.cuda.synchronize(dev)
    assert torch.equal(wt, shadow[:n].view(rows, cols).t().contiguous())
    ref = slabs.sum(0)
    assert torch.allclose(grad[:n], ref, rtol=1e-5, atol=1e-5)


def test_engine_update_writes_wt_bitwise(dev, monkeypatch):
    """DNN_FIN_WT=1 (W^T written by the fused reduce + update launch) trains bit for bit like
    the separate transpose launch, and W^T equals the transpose of the shadow afterwards."""
    from docker_dist_nn_amd import NAMED_MODELS
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    x, y = synthetic_mnist(4096, seed=9)
    xb = torch.zeros(4096, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xb, yb = xb.to(dev), torch.from_numpy(y).to(dev)
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("DNN_FIN_WT", flag)
        tr = Trainer(NAMED_MODELS["mnist-fcnn"], micro_batch=4096, num_micro=1,
                     optim=OptimConfig(lr=0.05, momentum=0.9), device=dev)
        p = tr.stages[0].params
        assert p.wt, "the headline model keeps W^T shadows for its dgrads"
        losses = []
        for _ in range(4):
            tr.set_batch(xb, yb)
            tr.step()
            losses.append(tr.loss())
        torch.cuda.synchronize(dev)
        for i, t in p.wt.items():
            assert torch.equal(t, p.wbf(i).t().contiguous())
        res.append((losses, p.master.clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])
