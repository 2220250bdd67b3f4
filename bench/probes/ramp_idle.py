"""Per-process or per-idle? One process runs the headline step 60 times, idles 3 s, runs 60
more, idles 0.2 s, runs 60 more; every step timed with HIP events. A ramp that restarts after
the 3 s idle but not after 0.2 s is the chip's power management; a ramp only at process start
is the process. Prints one JSON line per block of 10 steps.
Usage: python bench/probes/ramp_idle.py"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from docker_dist_nn_amd import NAMED_MODELS  # noqa: E402
from docker_dist_nn_amd.data import synthetic_mnist  # noqa: E402
from docker_dist_nn_amd.engine import OptimConfig, Trainer  # noqa: E402


def main():
    dev = torch.device("cuda")
    R = 65536
    spec = NAMED_MODELS["mnist-fcnn"]
    xs, ys = synthetic_mnist(R, seed=3)
    x = torch.zeros(R, 832, dtype=torch.bfloat16)
    x[:, :xs.shape[1]] = torch.from_numpy(xs).to(torch.bfloat16)
    y = torch.from_numpy(ys).to(torch.int32)
    tr = Trainer(spec, micro_batch=R, num_micro=1, optim=OptimConfig(lr=0.01), device=dev)
    tr.set_batch(x.to(dev), y.to(dev), zero_copy=True)
    for phase, idle in (("start", 0.0), ("after_3s_idle", 3.0), ("after_0.2s_idle", 0.2)):
        torch.cuda.synchronize()
        time.sleep(idle)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(61)]
        for i in range(60):
            ev[i].record()
            tr.step()
        ev[60].record()
        ev[60].synchronize()
        ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(60)]
        blocks = [round(sum(ms[k:k + 10]) / 10, 4) for k in range(0, 60, 10)]
        print(json.dumps({"phase": phase, "block_ms": blocks, "first": round(ms[0], 4)}),
              flush=True)


if __name__ == "__main__":
    main()
