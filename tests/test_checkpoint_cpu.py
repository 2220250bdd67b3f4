"""Checkpoint / resume (docker_dist_nn_amd/checkpoint.py) on the CPU engine: same-layout and
re-partitioned resume (weights AND optimizer state), the stale-shard regression of round 1
(train pp2 -> resume pp3 -> resume pp1 in one directory), crash safety of the commit protocol,
and the export to the reference's neuron-JSON model format (…ipynb:464-506)."""
import json
import os

import numpy as np
import pytest
import torch

from docker_dist_nn_amd import MLPSpec
from docker_dist_nn_amd import checkpoint as ckpt
from docker_dist_nn_amd.config import load_model_config
from docker_dist_nn_amd.data import synthetic_mnist
from docker_dist_nn_amd.engine import OptimConfig, Trainer

SPEC = MLPSpec.parse("784-96-48-10")
CPU = torch.device("cpu")


def _trainer(pp, dist_, optim):
    return Trainer(SPEC, micro_batch=64, num_micro=2, pp=pp, distribution=dist_,
                   optim=optim, device=CPU, seed=3)


def _batches(n_steps, seed=11):
    x, y = synthetic_mnist(128 * n_steps, seed=seed)
    out = []
    for s in range(n_steps):
        xb = torch.zeros(128, 832, dtype=torch.bfloat16)
        xb[:, :784] = torch.from_numpy(x[s * 128:(s + 1) * 128]).to(torch.bfloat16)
        out.append((xb, torch.from_numpy(y[s * 128:(s + 1) * 128].astype(np.int32))))
    return out


def _run(tr, batches):
    for xb, yb in batches:
        tr.set_batch(xb, yb)
        tr.step()


def _weights(tr):
    ww = tr.local_weights()
    return [ww[i] for i in range(len(SPEC.layers))]


OPTIMS = [OptimConfig(name="sgd", lr=0.05, momentum=0.9),
          OptimConfig(name="adam", lr=1e-3)]


@pytest.mark.parametrize("optim", OPTIMS, ids=["sgd_momentum", "adam"])
@pytest.mark.parametrize("layouts", [([1, 2], [1, 2]), ([1, 2], [2, 1]), ([1, 2], [3]),
                                     ([3], [1, 1, 1])])
def test_resume_matches_uninterrupted(tmp_path, optim, layouts):
    """k steps, checkpoint, resume onto (possibly) another layout, n-k more steps ==
    n uninterrupted steps: the optimizer state (momentum / Adam moments, update count) must
    survive the re-partition, not only the weights."""
    before, after = layouts
    bs = _batches(6)
    ref = _trainer(len(before), before, optim)
    _run(ref, bs)

    a = _trainer(len(before), before, optim)
    _run(a, bs[:3])
    ckpt.save_trainer(str(tmp_path), a, 3)
    b = _trainer(len(after), after, optim)
    assert ckpt.restore_trainer(str(tmp_path), b) == 3
    _run(b, bs[3:])
    for (w0, b0), (w1, b1) in zip(_weights(ref), _weights(b)):
        np.testing.assert_allclose(w1, w0, rtol=0, atol=1e-6)
        np.testing.assert_allclose(b1, b0, rtol=0, atol=1e-6)


def test_stale_shards_never_mix(tmp_path):
    """Round-1 bug: pp2 -> pp3 -> pp1 in one directory; every load must see the newest
    weights (the old layouts' stage1/stage2 shards are deleted at commit and never read)."""
    d = str(tmp_path)
    optim = OptimConfig(name="sgd", lr=0.05)
    bs = _batches(3)
    t2 = _trainer(2, [1, 2], optim)
    _run(t2, bs[:1])
    ckpt.save_trainer(d, t2, 1)
    t3 = _trainer(3, [1, 1, 1], optim)
    ckpt.restore_trainer(d, t3)
    _run(t3, bs[1:2])
    ckpt.save_trainer(d, t3, 2)
    assert sorted(f for f in os.listdir(d) if f.endswith(".safetensors")) == [
        "stage0.step2.safetensors", "stage1.step2.safetensors", "stage2.step2.safetensors"]
    t1 = _trainer(1, [3], optim)
    ckpt.restore_trainer(d, t1)
    _run(t1, bs[2:3])
    ckpt.save_trainer(d, t1, 3)
    assert sorted(f for f in os.listdir(d) if f.endswith(".safetensors")) == [
        "stage0.step3.safetensors"]
    ws, bs_, meta = ckpt.load_full_weights(d)
    fresh = _weights(t1)
    assert meta["step"] == 3 and meta["layer_distribution"] == [3]
    for (w, b), w1, b1 in zip(fresh, ws, bs_):
        np.testing.assert_array_equal(w1, w)
        np.testing.assert_array_equal(b1, b)


def test_crash_before_commit_keeps_previous_checkpoint(tmp_path):
    """Shards of a new step written but meta.json not replaced (crash mid-save): loading still
    returns the committed step, bit for bit."""
    d = str(tmp_path)
    optim = OptimConfig(name="sgd", lr=0.05)
    tr = _trainer(2, [1, 2], optim)
    bs = _batches(2)
    _run(tr, bs[:1])
    ckpt.save_trainer(d, tr, 1)
    committed = _weights(tr)
    _run(tr, bs[1:])
    ckpt.save_stage(d, tr.stages[0], 2, SPEC, [1, 2])  # stage 1's shard + commit never happen
    ws, bs_, meta = ckpt.load_full_weights(d)
    assert meta["step"] == 1
    for (w, b), w1, b1 in zip(committed, ws, bs_):
        np.testing.assert_array_equal(w1, w)
        np.testing.assert_array_equal(b1, b)
    with pytest.raises(RuntimeError, match="shards not written"):
        ckpt.commit(d, 2, SPEC, [1, 2], "sgd")


def test_shard_validation(tmp_path):
    d = str(tmp_path)
    tr = _trainer(2, [1, 2], OptimConfig())
    ckpt.save_trainer(d, tr, 5)
    meta = json.load(open(os.path.join(d, "meta.json")))
    meta["step"] = 6  # a meta that names a step its shards do not carry
    json.dump(meta, open(os.path.join(d, "meta.json"), "w"))
    with pytest.raises(ValueError, match="shard step 5 != committed step 6"):
        ckpt.load_full_weights(d)


def test_export_json_round_trip(tmp_path):
    """The exported model loads through the reference-schema loader with identical weights
    (neuron j = output unit j, weights over the inputs: src/grpc_node.py:43-55)."""
    d = str(tmp_path / "ck")
    tr = _trainer(2, [1, 2], OptimConfig())
    _run(tr, _batches(1))
    ckpt.save_trainer(d, tr, 1)
    out = str(tmp_path / "model.json")
    ckpt.export_json(d, out)
    mc = load_model_config(out)
    assert mc.layer_distribution == [1, 2]
    for L, (w, b) in zip(mc.layers, _weights(tr)):
        np.testing.assert_allclose(L.weight, w, rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(L.bias, b, rtol=1e-6, atol=1e-7)
    acts = [L.activation for L in mc.layers]
    assert acts == [l.activation for l in SPEC.layers]


def test_train_cli_resume_skips_consumed_batches(tmp_path):
    """cli/train: 4 steps in one go == 2 steps + resume for 2 more (same data order)."""
    from docker_dist_nn_amd.cli.train import main

    common = ["--model", "784-64-10", "--device", "cpu", "--synthetic", "512",
              "--micro-batch", "64", "--num-micro-batches", "2", "--optimizer", "adam",
              "--lr", "0.001", "--epochs", "2"]
    d1, d2 = str(tmp_path / "a"), str(tmp_path / "b")
    assert main(common + ["--steps", "6", "--checkpoint-dir", d1]) == 0
    assert main(common + ["--steps", "3", "--checkpoint-dir", d2]) == 0
    assert main(common + ["--steps", "6", "--checkpoint-dir", d2, "--resume",
                          "--pp", "2"]) == 0
    w1, b1, m1 = ckpt.load_full_weights(d1)
    w2, b2, m2 = ckpt.load_full_weights(d2)
    assert m1["step"] == m2["step"] == 6
    for a, b in zip(w1 + b1, w2 + b2):
        np.testing.assert_allclose(b, a, rtol=0, atol=1e-6)
