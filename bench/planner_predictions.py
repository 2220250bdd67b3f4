"""Planner predictions for every BASELINE config at N = 1, 2, 4, 8 GPUs (weak scaling):
the uniform pipeline (bf16 and fp8 hops, relays), the best replicated-stage ("fan") pipeline
bench.py runs (parallel/fan.py; bf16 hops, direct links), and the data-parallel-only layout,
each with its efficiency against N x the one-GPU rate.

    python bench/planner_predictions.py > profiles/r6_planner/predictions.jsonl

Round 6: every planner here is calibrated on one MI355X (Planner.calibrated: the measured
single-stage step and the measured replica steps of every layer range at every micro-batch
size and count, docker_dist_nn_amd/parallel/stage_times_gfx950.json), and the fan search
includes the light last stage co-located on a heavy replica's GPU.
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from docker_dist_nn_amd.models.mlp import NAMED_MODELS  # noqa: E402
from docker_dist_nn_amd.parallel.planner import Planner  # noqa: E402

FP8_BYTES = 1.0 + 4.0 / 64  # e4m3 element + one fp32 scale per row (>= 64 elements)


def main():
    for model, rows in (("mnist-fcnn", 65536), ("mlp8", 65536), ("wide", 16384)):
        spec = NAMED_MODELS[model]
        pl = Planner.calibrated(spec)
        p8 = Planner.calibrated(spec, boundary_bytes=FP8_BYTES)
        pr = Planner.calibrated(spec, relays=2)  # DNN_PIPE=ipc DNN_IPC_RELAYS=2
        pa = Planner.calibrated(spec, relays="plan")  # DNN_IPC_RELAYS=auto: per-hop plan
        for n in (1, 2, 4, 8):
            a = pl.pipeline_layout(spec, n, rows)
            b = p8.evaluate(spec, a.pp, a.dp, rows * a.pp, distribution=a.distribution)
            c = pr.evaluate(spec, a.pp, a.dp, rows * a.pp, distribution=a.distribution)
            e = pa.pipeline_layout(spec, n, rows)
            d = pl.evaluate(spec, 1, n, rows)
            one = pl.evaluate(spec, 1, 1, rows).samples_per_s
            f = pl.best_fan(spec, n, rows) if n > 1 else a
            fs = pl.best_fan(spec, n, rows, colocate=False) if n > 1 else a
            f8 = p8.best_fan(spec, n, rows) if n > 1 else a
            print(json.dumps({"model": model, "n": n, "layout": a.parallelism,
                              "dist": a.distribution, "nm": a.num_micro,
                              "pipe_bf16_Msps": round(a.samples_per_s / 1e6, 1),
                              "pipe_fp8_Msps": round(b.samples_per_s / 1e6, 1),
                              "pipe_ipc_relay2_Msps": round(c.samples_per_s / 1e6, 1),
                              "pipe_ipc_planned_Msps": round(e.samples_per_s / 1e6, 1),
                              "planned_dist": e.distribution,
                              "fan_layout": f.parallelism, "fan_dist": f.distribution,
                              "fan_reps": f.reps, "fan_nm": f.num_micro,
                              "fan_bf16_Msps": round(f.samples_per_s / 1e6, 1),
                              "fan_eff": round(f.samples_per_s / (n * one), 3),
                              "fan_no_colocation": fs.parallelism,
                              "fan_no_colocation_Msps": round(fs.samples_per_s / 1e6, 1),
                              "fan_detail": f.detail if n > 1 else None,
                              "fan_fp8_layout": f8.parallelism,
                              "fan_fp8_Msps": round(f8.samples_per_s / 1e6, 1),
                              "fan_fp8_eff": round(f8.samples_per_s / (n * one), 3),
                              "uniform_eff": round(a.samples_per_s / (n * one), 3),
                              "dp_only_Msps": round(d.samples_per_s / 1e6, 1),
                              "dp_eff": round(d.samples_per_s / (n * one), 3),
                              "dp_allreduce_ms": d.detail["allreduce_ms"]}))


if __name__ == "__main__":
    main()
