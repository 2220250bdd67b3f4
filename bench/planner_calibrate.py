"""One-GPU calibration of the parallel-layout planner: the compute of ONE
pipeline-stage replica per training step, measured on an MI355X at its real micro-batch size
and count -- layers [a, b) of a BASELINE model, n micro-batches of mb rows through the stage's
recorded forward / backward segments, then its batched weight gradient and the fused update
(a replica with a stage of its own: one-split wgrads update in their epilogue, as the fan
trainer runs it). Receives and sends are not part of it (the planner's link model prices
them), so this is exactly the term the planner used to extrapolate from the 65536-row
whole-model rate.

One JSON line per (model, a, b, mb, n): {"ms": median of 10 timed replays}.

    python bench/planner_calibrate.py [--models mnist-fcnn,mlp8,wide] > stage_times.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from docker_dist_nn_amd import NAMED_MODELS  # noqa: E402
from docker_dist_nn_amd.engine.stage import OptimConfig, Stage  # noqa: E402

def _mlp8_ranges(L=8):
    """Every prefix, every suffix and every single layer (the planner composes the rest)."""
    out = {(0, b) for b in range(1, L + 1)} | {(a, L) for a in range(L)}
    out |= {(a, a + 1) for a in range(L)}
    return sorted(out)


GRID = {  # model -> (micro-batch rows, micro-batch counts, layer ranges or None = all)
    "mnist-fcnn": ((4096, 8192, 16384, 32768), (1, 2, 4, 8, 16), None),
    "mlp8": ((8192, 16384), (2, 4, 8, 16), _mlp8_ranges()),
    "wide": ((1024, 2048, 4096, 8192), (1, 2, 4, 8), None),
}


def measure(spec, a, b, mb, n, dev, reps=10):
    S = len(spec.layers)
    st = Stage(spec, a, b, micro_batch=mb, num_micro=n, device=dev, global_batch=mb * n,
               optim=OptimConfig(lr=0.01), wgrad="batched", stage_index=0 if a == 0 else 1,
               num_stages=1 if (a, b) == (0, S) else 2)
    st.params.init_default(0)
    st.enable_fused_wgrad_update()
    st.compile_native()
    st.params.set_lr(0.01)
    segs = st._prog.segments()
    names = [f"F{j}" for j in range(n)] + [f"B{j}" for j in range(n)] + ["W"]
    names += ["FINO"] if "FINO" in segs else ["FIN", "O"]
    s = torch.cuda.current_stream(dev)
    for _ in range(3):
        st._prog.run(names, s.cuda_stream)
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        st._prog.run(names, s.cuda_stream)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    del st
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="mnist-fcnn,mlp8,wide")
    a_ = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for model in a_.models.split(","):
        spec = NAMED_MODELS[model]
        mbs, ns, ranges = GRID[model]
        L = len(spec.layers)
        ranges = ranges or [(a, b) for a in range(L) for b in range(a + 1, L + 1)]
        for a, b in ranges:
            for mb in mbs:
                for n in ns:
                    try:
                        ms = measure(spec, a, b, mb, n, dev)
                    except Exception as e:  # noqa: BLE001
                        print(json.dumps({"model": model, "a": a, "b": b, "mb": mb, "n": n,
                                          "err": str(e)[:120]}), flush=True)
                        continue
                    print(json.dumps({"model": model, "widths": spec.widths, "a": a, "b": b,
                                      "mb": mb, "n": n, "ms": round(ms, 4)}), flush=True)
                    torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
