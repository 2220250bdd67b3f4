"""Metrics stream, per-op step profiler / Chrome trace and latency statistics (CPU).

The reference only logs wall-clock lines (/root/reference/src/run_grpc_fcnn.py:321-322,
/root/reference/src/run_grpc_inference.py:139-142, 195-216); these are the structured
equivalents: docker_dist_nn_amd/metrics.py and docker_dist_nn_amd/profiler.py."""
import json

import numpy as np
import torch

from docker_dist_nn_amd import MLPSpec
from docker_dist_nn_amd.data import synthetic_mnist
from docker_dist_nn_amd.engine import OptimConfig, Trainer
from docker_dist_nn_amd.metrics import LatencyStats, MetricsWriter
from docker_dist_nn_amd.profiler import StepProfiler


def test_metrics_writer_jsonl(tmp_path):
    p = tmp_path / "sub" / "m.jsonl"
    w = MetricsWriter(str(p), rank=3)
    w.write("train", step=1, loss=2.5, samples_per_s=1e6)
    w.write("done", step=2)
    w.close()
    w2 = MetricsWriter(str(p), rank=0)  # append mode
    w2.write("resume", step=2)
    w2.close()
    recs = [json.loads(l) for l in open(p)]
    assert [r["kind"] for r in recs] == ["train", "done", "resume"]
    assert recs[0]["rank"] == 3 and recs[0]["loss"] == 2.5 and "ts" in recs[0]
    MetricsWriter(None).write("x", a=1)  # disabled writer is a no-op


def test_latency_stats():
    s = LatencyStats()
    for v in range(1, 101):
        s.add(v / 1000)
    d = s.summary()
    assert d["n"] == 100 and abs(d["p50_s"] - 0.0505) < 1e-9 and d["max_s"] == 0.1
    assert LatencyStats().summary() == {}


def test_step_profiler_chrome_trace(tmp_path):
    spec = MLPSpec.parse("784-64-32-10")
    tr = Trainer(spec, micro_batch=64, num_micro=3, pp=3, distribution=[1, 1, 1],
                 schedule="1f1b", optim=OptimConfig(lr=0.05), device=torch.device("cpu"))
    prof = StepProfiler(tr.executor, rank=0)
    x, y = synthetic_mnist(192, seed=0)
    xb = torch.zeros(192, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    tr.set_batch(xb, torch.from_numpy(y))
    tr.step()
    ops = prof.collect()
    # every schedule op of every stage is timed: 3 F + 3 B + W + O per stage
    assert len(ops) == 3 * 8
    assert {o["stage"] for o in ops} == {0, 1, 2}
    assert sorted(o["micro"] for o in ops if o["op"] == "F" and o["stage"] == 1) == [0, 1, 2]
    s = StepProfiler.summarize(ops)
    assert 0.0 <= s["bubble"] < 1.0 and s["makespan_ms"] > 0
    out = tmp_path / "trace.json"
    prof.chrome_trace(str(out))
    doc = json.load(open(out))
    ev = doc["traceEvents"]
    assert len(ev) == len(ops) and all(e["ph"] == "X" for e in ev)
    assert {e["tid"] for e in ev} == {0, 1, 2}
    assert any(e["name"] == "forward mb0" for e in ev)


def test_train_cli_writes_metrics_and_trace(tmp_path):
    from docker_dist_nn_amd.cli.train import main

    m, t = tmp_path / "m_{rank}.jsonl", tmp_path / "t_{rank}.json"
    assert main(["--model", "784-64-10", "--device", "cpu", "--synthetic", "512",
                 "--micro-batch", "64", "--num-micro-batches", "2", "--steps", "4",
                 "--check-every", "2", "--pp", "2", "--metrics", str(m), "--trace", str(t)]) == 0
    recs = [json.loads(l) for l in open(tmp_path / "m_0.jsonl")]
    assert [r["kind"] for r in recs] == ["train", "train", "done"]
    assert all(np.isfinite(r["loss"]) for r in recs)
    ev = json.load(open(tmp_path / "t_0.json"))["traceEvents"]
    assert {e["tid"] for e in ev} == {0, 1}
