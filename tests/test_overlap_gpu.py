"""dgrad/wgrad overlap plans (DNN_BW_OVERLAP=1: wgrad_i on a side stream concurrent with the
next dgrad; =5: the small wgrads on the side, W1 and W0 on the main stream): must be bitwise
identical to the sequential native plan."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model,rows", [("mnist-fcnn", 8192), ("784-8192-8192-10", 2048)])
def test_overlap_plan_bitwise(dev, monkeypatch, model, rows):
    """784-8192-8192-10 at 2048 rows: layer 1's one-split wgrad updates W_1 / W_1^T in its
    epilogue (fused update), so the plan must start it only after dgrad_1 has read W_1^T."""
    from docker_dist_nn_amd import NAMED_MODELS, MLPSpec
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    spec = NAMED_MODELS.get(model) or MLPSpec.parse(model)
    monkeypatch.setenv("DNN_BW_OVERLAP_MIN_ROWS", "0")
    x, y = synthetic_mnist(rows, seed=4)
    xb = torch.zeros(rows, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xb, yb = xb.to(dev), torch.from_numpy(y).to(dev)
    res = []
    # 1s: plan 1 with DNN_SPLIT_FINO (layers 1.. reduced and updated on the side stream
    # during W0); 5 / 5s: small wgrads on the side, W1 then W0 on the main stream (unsplit /
    # split FINO)
    for flag in ("0", "1", "1s", "5", "5s"):
        monkeypatch.setenv("DNN_BW_OVERLAP", flag[0])
        monkeypatch.setenv("DNN_SPLIT_FINO", "1" if flag[-1] == "s" else "0")
        tr = Trainer(spec, micro_batch=rows, num_micro=1,
                     optim=OptimConfig(lr=0.1, momentum=0.9), device=dev)
        losses = []
        for _ in range(4):
            tr.set_batch(xb, yb)
            tr.step()
            losses.append(tr.loss())
        plan = tr.executor._native_plan()
        assert any(seg == "@fork" for _, seg, _ in plan) == (flag != "0")
        res.append((losses, tr.stages[0].params.master.clone()))
    for r in res[1:]:
        assert res[0][0] == r[0]
        assert torch.equal(res[0][1], r[1])


def test_mode5_without_tail_bitwise(dev, monkeypatch):
    """Overlap mode 5 with the classifier tail off: W2 on the side stream reads dZ_2, which the
    main stream's dgrad of layer 3 writes, so the plan must fork after that dgrad.
    Bitwise equal to the sequential plan."""
    from docker_dist_nn_amd import NAMED_MODELS
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    rows = 8192
    monkeypatch.setenv("DNN_BW_OVERLAP_MIN_ROWS", "0")
    monkeypatch.setenv("DNN_TAIL", "0")
    x, y = synthetic_mnist(rows, seed=6)
    xb = torch.zeros(rows, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xb, yb = xb.to(dev), torch.from_numpy(y).to(dev)
    res = []
    for flag in ("0", "5"):
        monkeypatch.setenv("DNN_BW_OVERLAP", flag)
        tr = Trainer(NAMED_MODELS["mnist-fcnn"], micro_batch=rows, num_micro=1,
                     optim=OptimConfig(lr=0.1, momentum=0.9), device=dev)
        losses = []
        for _ in range(4):
            tr.set_batch(xb, yb)
            tr.step()
            losses.append(tr.loss())
        segs = [seg for _, seg, _ in tr.executor._native_plan()]
        if flag == "5":
            assert segs.index("B0.L3") < segs.index("W2") and \
                "@fork" in segs[segs.index("B0.L3"):segs.index("W2")], segs
        res.append((losses, tr.stages[0].params.master.clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("model,rows,split", [("mnist-fcnn", 8192, True),
                                              ("784-8192-8192-10", 2048, False)])
def test_split_fino_auto_plan(dev, monkeypatch, model, rows, split):
    """DNN_SPLIT_FINO=auto (the default): layers 1.. are reduced and updated on the side stream
    during W0 unless a layer updates in its wgrad epilogue (the wide model's layer 1)."""
    from docker_dist_nn_amd import NAMED_MODELS, MLPSpec
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    monkeypatch.delenv("DNN_SPLIT_FINO", raising=False)
    monkeypatch.delenv("DNN_BW_OVERLAP", raising=False)
    monkeypatch.setenv("DNN_BW_OVERLAP_MIN_ROWS", "0")
    from docker_dist_nn_amd.data import synthetic_mnist

    spec = NAMED_MODELS.get(model) or MLPSpec.parse(model)
    x, y = synthetic_mnist(rows, seed=4)
    xb = torch.zeros(rows, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    tr = Trainer(spec, micro_batch=rows, num_micro=1, optim=OptimConfig(lr=0.1), device=dev)
    tr.set_batch(xb.to(dev), torch.from_numpy(y).to(dev))
    tr.step()
    segs = [(seg, side) for _, seg, side in tr.executor._native_plan()]
    L = len(spec.layers)
    assert ((f"FINO1-{L - 1}", 1) in segs and ("FINO0-0", 0) in segs) == split, segs
    assert (("FINO", 0) in segs) == (not split), segs


def test_cross_step_overlap_bitwise(dev, monkeypatch):
    """DNN_XSTEP=1 moves the side stream's join from the end of a step to in front of the
    next step's layer-1 forward (the layer-0 forward runs beside the reduce + update of layers
    1..L-1). Bitwise the same training as the joined plan, for the losses of every step and
    the weights after flush."""
    from docker_dist_nn_amd import NAMED_MODELS
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    rows = 8192
    monkeypatch.setenv("DNN_BW_OVERLAP_MIN_ROWS", "0")
    monkeypatch.setenv("DNN_SPLIT_FINO", "1")
    x, y = synthetic_mnist(2 * rows, seed=7)
    xb = torch.zeros(2 * rows, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xb, yb = xb.to(dev), torch.from_numpy(y).to(dev)
    res = []
    for xs, dbl in (("0", "0"), ("1", "0"), ("1", "1")):
        monkeypatch.setenv("DNN_XSTEP", xs)
        monkeypatch.setenv("DNN_H0_DOUBLE", dbl)
        tr = Trainer(NAMED_MODELS["mnist-fcnn"], micro_batch=rows, num_micro=1,
                     optim=OptimConfig(lr=0.1, momentum=0.9), device=dev)
        losses = []
        for k in range(6):  # alternating batches, zero-copy views as in the bench
            r = slice((k % 2) * rows, (k % 2 + 1) * rows)
            tr.set_batch(xb[r], yb[r], zero_copy=True)
            tr.step()
            losses.append(tr.loss())
        tr.flush()
        if xs == "1":
            segs = [seg for _, seg, _ in tr.executor._xstep_plan(tr.executor._native_plan())]
            assert ("@xwait:w" in segs) == (dbl == "0") and segs[-1] == "@xmark:end", segs
            assert tr.stages[0].h0_double == (dbl == "1")
        res.append((losses, tr.stages[0].params.master.clone()))
    for r in res[1:]:  # DNN_XSTEP and DNN_H0_DOUBLE: bitwise the same training
        assert r[0] == res[0][0]
        assert torch.equal(r[1], res[0][1])


def _xstep_trainer(dev, seed, lr):
    from docker_dist_nn_amd import NAMED_MODELS
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    return Trainer(NAMED_MODELS["mnist-fcnn"], micro_batch=8192, num_micro=1, seed=seed,
                   optim=OptimConfig(lr=lr, momentum=0.9), device=dev)


def _xstep_batches(dev):
    from docker_dist_nn_amd.data import synthetic_mnist

    rows = 8192
    x, y = synthetic_mnist(2 * rows, seed=11)
    xb = torch.zeros(2 * rows, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xb, yb = xb.to(dev), torch.from_numpy(y).to(dev)
    return [(xb[k * rows:(k + 1) * rows], yb[k * rows:(k + 1) * rows]) for k in range(2)]


def test_interleaved_cross_step_trainers_bitwise(dev, monkeypatch):
    """the cross-step events belong to each executor. Two DNN_XSTEP trainers
    stepping in turn on one thread must each wait on THEIR OWN side stream's marks -- bitwise
    the same training as each trainer stepping alone."""
    monkeypatch.setenv("DNN_BW_OVERLAP_MIN_ROWS", "0")
    monkeypatch.setenv("DNN_SPLIT_FINO", "1")
    monkeypatch.setenv("DNN_XSTEP", "1")
    bat = _xstep_batches(dev)
    alone = []
    for seed, lr in ((0, 0.1), (1, 0.05)):
        tr = _xstep_trainer(dev, seed, lr)
        for k in range(6):
            tr.set_batch(*bat[k % 2], zero_copy=True)
            tr.step()
        tr.flush()
        alone.append(tr.stages[0].params.master.clone())
    a, b = _xstep_trainer(dev, 0, 0.1), _xstep_trainer(dev, 1, 0.05)
    for k in range(6):
        for tr in (a, b):
            tr.set_batch(*bat[k % 2], zero_copy=True)
            tr.step()
    a.flush()
    b.flush()
    assert torch.equal(a.stages[0].params.master, alone[0])
    assert torch.equal(b.stages[0].params.master, alone[1])


def test_capture_after_eager_cross_step_bitwise(dev, monkeypatch):
    """capture() after eager DNN_XSTEP steps joins the pending side-stream update
    first -- 2 eager steps, a capture (1 executed step) and 2 replays train bit for bit like 5
    eager steps."""
    monkeypatch.setenv("DNN_BW_OVERLAP_MIN_ROWS", "0")
    monkeypatch.setenv("DNN_SPLIT_FINO", "1")
    monkeypatch.setenv("DNN_XSTEP", "1")
    x, y = _xstep_batches(dev)[0]
    ref = _xstep_trainer(dev, 0, 0.1)
    for _ in range(5):
        ref.set_batch(x, y)
        ref.step()
    ref.flush()
    tr = _xstep_trainer(dev, 0, 0.1)
    for _ in range(2):
        tr.set_batch(x, y)
        tr.step()
    tr.set_batch(x, y)
    tr.capture(warmup=0, copies=1)  # executes one real step
    for _ in range(2):
        tr.step()
    torch.cuda.synchronize()
    assert torch.equal(tr.stages[0].params.master, ref.stages[0].params.master)


def test_cross_step_with_layer0_mask_bitwise(dev, monkeypatch):
    """The layer-0 fragment-order ReLU mask (DNN_RELU_MASK=2) together with the cross-step plan
    and the double-buffered layer-0 activation -- overlap modes 1 and 5 -- trains bit for bit
    like the joined plan with the same mask (the mask is written by the forward and read by
    the dgrad of the same step, both on the main stream)."""
    monkeypatch.setenv("DNN_BW_OVERLAP_MIN_ROWS", "0")
    monkeypatch.setenv("DNN_SPLIT_FINO", "1")
    monkeypatch.setenv("DNN_RELU_MASK", "2")
    from docker_dist_nn_amd import NAMED_MODELS
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    rows = 65536  # the tuned table gives both GEMMs one register-direct tile at this size
    x, y = synthetic_mnist(2 * rows, seed=11)
    xb = torch.zeros(2 * rows, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xb, yb = xb.to(dev), torch.from_numpy(y).to(dev)
    bat = [(xb[k * rows:(k + 1) * rows], yb[k * rows:(k + 1) * rows]) for k in range(2)]
    res = []
    for xs, dbl, mode in (("0", "0", "1"), ("1", "1", "1"), ("1", "1", "5")):
        monkeypatch.setenv("DNN_XSTEP", xs)
        monkeypatch.setenv("DNN_H0_DOUBLE", dbl)
        monkeypatch.setenv("DNN_BW_OVERLAP", mode)
        tr = Trainer(NAMED_MODELS["mnist-fcnn"], micro_batch=rows, num_micro=1, seed=0,
                     optim=OptimConfig(lr=0.1, momentum=0.9), device=dev)
        assert tr.stages[0].relu_mask[0] is not None
        assert tr.stages[0].h0_double == (dbl == "1")
        losses = []
        for k in range(6):
            tr.set_batch(*bat[k % 2], zero_copy=True)
            tr.step()
            losses.append(tr.loss())
        tr.flush()
        res.append((losses, tr.stages[0].params.master.clone()))
    for r in res[1:]:
        assert r[0] == res[0][0]
        assert torch.equal(r[1], res[0][1])

