"""CPU paths: fp64 oracles (config 1), schedules, and the engine's training numerics."""
import numpy as np
import pytest
import torch

from docker_dist_nn_amd import MLPSpec
from docker_dist_nn_amd.config import LayerWeights, model_config_from_dict
from docker_dist_nn_amd.cpu_ref import manual_forward, stage_forward, train_step
from docker_dist_nn_amd.data import synthetic_mnist
from docker_dist_nn_amd.engine import OptimConfig, Trainer
from docker_dist_nn_amd.metrics import classification_report
from docker_dist_nn_amd.parallel.pipeline import schedule_ops
from docker_dist_nn_amd.utils.native import native


def _cfg(rng, widths, acts):
    layers = []
    for i in range(len(widths) - 1):
        w = rng.standard_normal((widths[i + 1], widths[i]))
        b = rng.standard_normal(widths[i + 1])
        layers.append({"type": "hidden", "nodes": widths[i + 1],
                       "neurons": [{"weights": w[j].tolist(), "bias": float(b[j]),
                                    "activation": acts[i]} for j in range(widths[i + 1])]})
    return {"layers": layers}


def test_manual_and_stage_forward_agree():
    rng = np.random.default_rng(0)
    cfg = _cfg(rng, [784, 128, 10], ["relu", "softmax"])
    mc = model_config_from_dict(cfg)
    x = rng.random(784)
    a = manual_forward(cfg, x)
    b = stage_forward(mc.layers, x, 784)[0]
    np.testing.assert_allclose(a, b, rtol=1e-12)
    assert abs(a.sum() - 1) < 1e-12


def test_stage_forward_dim_error_text():
    L = [LayerWeights(np.ones((3, 2)), np.zeros(3), "relu")]
    with pytest.raises(ValueError, match=r"\(layer_container_0\) Layer 1: expected input dim 2, got 5"):
        stage_forward(L, np.ones((1, 5)), 2, name="layer_container_0")


def test_manual_forward_semantics_sigmoid_is_linear():
    cfg = {"layers": [{"neurons": [{"weights": [2.0], "bias": -5.0, "activation": "SIGMOID"}]}]}
    assert manual_forward(cfg, [1.0])[0] == -3.0  # sigmoid not in manual_nn's map -> linear


@pytest.mark.parametrize("kind", ["gpipe", "1f1b", "1f1b_w", "zb"])
@pytest.mark.parametrize("S,M", [(1, 1), (2, 3), (4, 4), (4, 9), (8, 8)])
def test_schedules_cover_every_micro_batch(kind, S, M):
    for s in range(S):
        ops = schedule_ops(kind, S, M, s)
        f = [j for o, j in ops if o == "F"]
        b = [j for o, j in ops if o == "B"]
        w = [j for o, j in ops if o == "W"]
        assert f == list(range(M)) and b == list(range(M))
        assert w == [-1] or sorted(w) == list(range(M))
        assert ops[-1] == ("O", -1)
        for j in range(M):  # backward after its forward
            assert ops.index(("F", j)) < ops.index(("B", j))


def test_simulator_gpipe_bubble_formula():
    S, M = 4, 12
    mk, busy, bubble = native().simulate_schedule("gpipe", S, M, [1.0], [1.0], [0.0], 0.0)
    assert abs(mk - (M + S - 1) * 2) < 1e-9
    assert abs(bubble - (S - 1) / (M + S - 1)) < 1e-9


def _xy(n, seed=3):
    x, y = synthetic_mnist(n, seed=seed)
    xt = torch.zeros(n, 832, dtype=torch.bfloat16)
    xt[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    return x, y, xt, torch.from_numpy(y)


def test_engine_matches_fp64_training_oracle():
    spec = MLPSpec.parse("784-64-10")
    x, y, xt, yt = _xy(256)
    tr = Trainer(spec, micro_batch=256, optim=OptimConfig(lr=0.2), device=torch.device("cpu"))
    ws = {k: (w.astype(np.float64), b.astype(np.float64)) for k, (w, b) in tr.local_weights().items()}
    W = [ws[0][0], ws[1][0]]
    B = [ws[0][1], ws[1][1]]
    xb = xt[:, :784].float().numpy().astype(np.float64)  # the bf16-rounded inputs
    ref_losses, eng_losses = [], []
    for _ in range(5):
        ref_losses.append(train_step(W, B, ["relu", "softmax"], xb, y, 0.2))
        tr.set_batch(xt, yt)
        tr.step()
        eng_losses.append(tr.loss())
    np.testing.assert_allclose(eng_losses, ref_losses, rtol=1e-2)
    w_eng = tr.local_weights()[0][0]
    assert np.abs(w_eng - W[0]).max() < 5e-3


def test_engine_multi_stage_cpu_matches_single_stage():
    spec = MLPSpec.parse("784-256-128-64-10")
    _, _, xt, yt = _xy(1024)
    out = {}
    for pp, sched in [(1, "1f1b"), (4, "1f1b"), (2, "gpipe"), (3, "zb")]:
        tr = Trainer(spec, micro_batch=256, num_micro=4, pp=pp, schedule=sched,
                     optim=OptimConfig(lr=0.1, momentum=0.9), device=torch.device("cpu"))
        ls = []
        for _ in range(3):
            tr.set_batch(xt, yt)
            tr.step()
            ls.append(tr.loss())
        out[(pp, sched)] = (ls, tr.local_weights()[0][0])
    base_l, base_w = out[(1, "1f1b")]
    for k, (ls, w) in out.items():
        np.testing.assert_allclose(ls, base_l, rtol=1e-5)
        np.testing.assert_allclose(w, base_w, rtol=1e-5, atol=1e-6)


def test_adam_training_decreases_loss():
    spec = MLPSpec.parse("784-64-10")
    _, _, xt, yt = _xy(512)
    tr = Trainer(spec, micro_batch=512, optim=OptimConfig(name="adam", lr=1e-2),
                 device=torch.device("cpu"))
    ls = []
    for _ in range(10):
        tr.set_batch(xt, yt)
        tr.step()
        ls.append(tr.loss())
    assert ls[-1] < 0.7 * ls[0]


def test_classification_report_matches_weighted_definition():
    y = np.array([0, 0, 1, 1, 2, 2, 2])
    p = np.array([0, 1, 1, 1, 2, 0, 2])
    r = classification_report(y, p)
    assert abs(r["accuracy"] - 5 / 7) < 1e-12
    # class precisions 0.5, 2/3, 1 ; recalls 0.5, 1, 2/3 ; weights 2/7, 2/7, 3/7
    prec = (2 * 0.5 + 2 * 2 / 3 + 3 * 1.0) / 7
    assert abs(r["precision"] - prec) < 1e-12


def test_dp_buckets_partition_flat_gradient():
    from docker_dist_nn_amd.engine.stage import StageParams
    from docker_dist_nn_amd.models.mlp import LayerGeom
    spec = MLPSpec.parse("784-512-256-10")
    geoms = [LayerGeom(i, l) for i, l in enumerate(spec.layers)]
    p = StageParams(geoms, torch.device("cpu"))
    covered = np.zeros(p.numel, np.int32)
    for i in range(len(geoms)):
        a, b = p.layer_grad_range(i)
        covered[a:b] += 1
        assert a <= p.w_off[i] and p.b_off[i] + geoms[i].np_ <= b
    assert (covered == 1).all()
