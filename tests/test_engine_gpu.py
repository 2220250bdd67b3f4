"""End-to-end training on the GPU through the native kernels: parity with the CPU reference
path, S-stage loopback pipelines == 1 stage, HIP-graph replay == eager execution."""
import numpy as np
import pytest
import torch

from docker_dist_nn_amd import MLPSpec
from docker_dist_nn_amd.data import synthetic_mnist
from docker_dist_nn_amd.engine import OptimConfig, Trainer

pytestmark = pytest.mark.gpu


def _batch(n, dev, seed=1):
    x, y = synthetic_mnist(n, seed=seed)
    xt = torch.zeros(n, 832, dtype=torch.bfloat16)
    xt[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    return xt.to(dev), torch.from_numpy(y).to(dev)


def _run(spec, dev, steps, **kw):
    tr = Trainer(spec, device=dev, optim=OptimConfig(lr=0.1), **kw)
    x, y = _batch(kw["micro_batch"] * kw.get("num_micro", 1), dev)
    losses = []
    for _ in range(steps):
        tr.set_batch(x, y)
        tr.step()
        losses.append(tr.loss())
    return tr, losses


def test_gpu_training_matches_cpu_reference(dev):
    spec = MLPSpec.parse("784-128-64-10")
    _, lg = _run(spec, dev, 8, micro_batch=512, num_micro=2)
    _, lc = _run(spec, torch.device("cpu"), 8, micro_batch=512, num_micro=2)
    assert lg[-1] < lg[0]
    np.testing.assert_allclose(lg, lc, rtol=2e-2, atol=2e-3)


@pytest.mark.parametrize("pp,sched", [(2, "1f1b"), (4, "gpipe"), (4, "zb"), (3, "1f1b_w")])
def test_gpu_pipeline_equals_single_stage(dev, pp, sched):
    spec = MLPSpec.parse("784-512-256-128-10")
    t1, l1 = _run(spec, dev, 4, micro_batch=256, num_micro=4)
    tp, lp = _run(spec, dev, 4, micro_batch=256, num_micro=4, pp=pp, schedule=sched)
    np.testing.assert_allclose(lp, l1, rtol=1e-3, atol=1e-4)
    w1, wp = t1.local_weights(), tp.local_weights()
    for k in w1:
        np.testing.assert_allclose(wp[k][0], w1[k][0], rtol=1e-3, atol=1e-5)


def test_gpu_graph_replay_equals_eager(dev):
    spec = MLPSpec.parse("784-512-256-128-10")
    x, y = _batch(1024, dev)
    ta = Trainer(spec, device=dev, micro_batch=1024, optim=OptimConfig(lr=0.1))
    tb = Trainer(spec, device=dev, micro_batch=1024, optim=OptimConfig(lr=0.1))
    ta.set_batch(x, y)
    tb.set_batch(x, y)
    tb.capture(warmup=0)  # capture executes one real step
    ta.step()
    la, lb = [ta.loss()], [tb.loss()]
    for _ in range(5):
        ta.set_batch(x, y)
        ta.step()
        tb.set_batch(x, y)
        tb.step()
        la.append(ta.loss())
        lb.append(tb.loss())
    assert la == lb
    wa, wb = ta.local_weights(), tb.local_weights()
    for k in wa:
        assert np.array_equal(wa[k][0], wb[k][0])


def test_gpu_bitwise_deterministic(dev):
    spec = MLPSpec.parse("784-512-256-128-10")
    _, la = _run(spec, dev, 3, micro_batch=2048)
    _, lb = _run(spec, dev, 3, micro_batch=2048)
    assert la == lb


@pytest.mark.parametrize("pp,sched", [(1, "1f1b"), (2, "1f1b"), (4, "gpipe")])
def test_native_executor_equals_python(dev, pp, sched):
    """Recorded-launch replay from C++ == the Python op-by-op path, bit for bit (same
    kernels, same order), including zero-copy inputs relocated into the program."""
    spec = MLPSpec.parse("784-512-256-128-10")
    x, y = _batch(2048, dev)
    out = []
    for native_exec in (False, True):
        tr = Trainer(spec, device=dev, micro_batch=512, num_micro=4, pp=pp, schedule=sched,
                     optim=OptimConfig(lr=0.1, momentum=0.9), native_exec=native_exec)
        assert tr.native_exec == native_exec
        losses = []
        for k in range(4):
            xs = x.roll(k * 64, 0).contiguous()  # a different buffer each step
            ys = y.roll(k * 64, 0).contiguous()
            tr.set_batch(xs, ys, zero_copy=True)
            tr.step()
            losses.append(tr.loss())
        # all-native loopback steps run as ONE C++ call over a precomputed segment plan
        assert (tr.executor._native_plan() is not None) == native_exec
        out.append((losses, tr.local_weights(), tr.correct()))
    (l0, w0, c0), (l1, w1, c1) = out
    assert l0 == l1 and c0 == c1
    for k in w0:
        assert np.array_equal(w0[k][0], w1[k][0]) and np.array_equal(w0[k][1], w1[k][1])


def test_native_program_record_relocate(dev):
    from docker_dist_nn_amd import ops
    from docker_dist_nn_amd.utils import native

    nat = native()
    g = torch.Generator().manual_seed(0)
    a = torch.randn(256, 128, generator=g).to(torch.bfloat16).to(dev)
    a2 = torch.randn(256, 128, generator=g).to(torch.bfloat16).to(dev)
    w = torch.randn(64, 128, generator=g).to(torch.bfloat16).to(dev)
    b = torch.randn(64, generator=g).to(dev)
    y = torch.zeros(256, 64, dtype=torch.bfloat16, device=dev)
    prog = nat.Program()
    rid = prog.region(a.data_ptr(), a.numel() * 2)
    nat.record_begin(prog)
    try:
        prog.mark("fwd")
        ops.linear_fwd(a, w, b, y, act="relu")
    finally:
        nat.record_end()
    assert prog.segments() == ["fwd"] and prog.segment_size("fwd") == 1
    assert not y.any()  # recording launched nothing
    stream = torch.cuda.current_stream(dev).cuda_stream
    prog.run(["fwd"], stream)
    ref = torch.relu(a.float() @ w.float().t() + b)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    prog.rebase(rid, a2.data_ptr())
    prog.run(["fwd"], stream)
    torch.testing.assert_close(y.float(), torch.relu(a2.float() @ w.float().t() + b),
                               rtol=2e-2, atol=2e-2)
    with pytest.raises(IndexError):
        prog.run(["nope"], stream)


@pytest.mark.parametrize("optim", [OptimConfig(name="adam", lr=1e-3),
                                   OptimConfig(name="adamw", lr=2e-3, weight_decay=0.01),
                                   OptimConfig(lr=0.1, momentum=0.9)])
def test_native_and_graph_optimizers_with_lr_schedule(dev, optim):
    """Adam/AdamW/SGD with a changing learning rate: native replay, HIP-graph replay and the
    Python path agree bit for bit (lr and the Adam step live in device memory, so recorded and
    captured updates stay correct across steps). SGD includes layers whose wgrad epilogue
    applies the update (fused_layers): they must see this step's rate on every path."""
    import dataclasses

    # SGD: a 1024-wide first layer, whose 1024-row weight gradient is ONE split (fused update)
    spec = MLPSpec.parse("784-1024-128-10" if optim.name == "sgd" else "784-256-128-10")
    x, y = _batch(1024, dev)
    lrs = [optim.lr * f for f in (1.0, 0.5, 0.25, 0.5, 1.0)]
    results = []
    for mode in ("python", "native", "graph"):
        tr = Trainer(spec, device=dev, micro_batch=512, num_micro=2,
                     optim=dataclasses.replace(optim), native_exec=mode != "python")
        if optim.name == "sgd":  # one-split wgrads apply SGD in their epilogue (read lr_dev
            assert tr.stages[0].params.fused_layers  # during W, before O: ADVICE r2)
        tr.set_batch(x, y)
        if mode == "graph":
            tr.capture(warmup=0)  # executes step 1 at lrs[0]
        losses = []
        for k, lr in enumerate(lrs):
            for st in tr.stages:
                st.params.optim.lr = lr
            if not (mode == "graph" and k == 0):
                tr.step()
            losses.append(tr.loss())
        results.append((losses, tr.local_weights(), tr.stages[0].params.step_count))
    (l0, w0, s0) = results[0]
    for (l1, w1, s1) in results[1:]:
        assert s1 == s0 == len(lrs)
        assert l1 == l0
        for k in w0:
            assert np.array_equal(w0[k][0], w1[k][0])


@pytest.mark.parametrize("model", ["784-256-256-256-10", "784-512-512-512-256-10"])
def test_kmajor_wgrad_training_bitwise(dev, monkeypatch, model):
    """Training with K-major weight gradients (forward / dgrad epilogues also write X^T and
    dZ^T, wgrad reads both K-major; DNN_WGRAD_KK=1 forces it on these small layers) gives the
    same weights, bit for bit, as the transposing-read path (DNN_WGRAD_KK=0)."""
    spec = MLPSpec.parse(model)
    x, y = _batch(1024, dev)
    out = []
    for kk in ("0", "1"):
        monkeypatch.setenv("DNN_WGRAD_KK", kk)
        tr = Trainer(spec, device=dev, micro_batch=512, num_micro=2, pp=1,
                     optim=OptimConfig(lr=0.1, momentum=0.9))
        assert bool(tr.stages[0].dzT) == (kk == "1")
        for _ in range(3):
            tr.set_batch(x, y)
            tr.step()
        out.append(tr.local_weights())
    for k in out[0]:
        assert np.array_equal(out[0][k][0], out[1][k][0]), k


def test_fused_wgrad_update_bitwise(dev, monkeypatch):
    """One-split weight gradients that apply SGD (momentum + weight decay) and write W^T in
    their GEMM epilogue (Stage.enable_fused_wgrad_update) train bit-identically to the
    separate reduction + update + transpose."""
    import numpy as np

    from docker_dist_nn_amd import MLPSpec
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    rows = 2048
    x, y = synthetic_mnist(rows, seed=3)
    xb = torch.zeros(rows, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xd, yd = xb.to(dev), torch.from_numpy(y).to(dev)
    out = {}
    for fused in ("0", "1"):
        monkeypatch.setenv("DNN_WGRAD_FUSED_UPDATE", fused)
        tr = Trainer(MLPSpec.parse("784-8192-8192-10"), micro_batch=rows, num_micro=1,
                     device=dev, optim=OptimConfig(lr=0.02, momentum=0.9, weight_decay=1e-4))
        p = tr.stages[0].params
        assert bool(p.fused_layers) == (fused == "1")
        if fused == "1":
            assert 1 in p.fused_layers and 1 in p.wt
        for _ in range(3):
            tr.set_batch(xd, yd)
            tr.step()
        torch.cuda.synchronize(dev)
        out[fused] = (tr.local_weights(), tr.loss(), p.wt[1].cpu().clone(),
                      p.state[0].cpu().clone())
    for k, (w, b) in out["0"][0].items():
        assert np.array_equal(w, out["1"][0][k][0]), k
        assert np.array_equal(b, out["1"][0][k][1]), k
    assert out["0"][1] == out["1"][1]
    assert torch.equal(out["0"][2], out["1"][2])  # W^T written by the epilogue
    assert torch.equal(out["0"][3], out["1"][3])  # momentum
