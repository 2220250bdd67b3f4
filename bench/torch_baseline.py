"""PyTorch-ROCm baseline of the headline training step on the same MI355X ("each
result will be compared ... with a torch-ROCm single-GPU baseline on the same MI355X").

Same model (nn.Linear stack, ReLU, softmax cross-entropy), same synthetic data shape, same
batch, one step = forward + backward + SGD update. Variants:
  eager-bf16   : bf16 parameters and activations, torch.optim.SGD (hipBLASLt GEMMs)
  amp          : fp32 master parameters + torch.autocast(bf16) -- the usual mixed precision
                 recipe, the closest to our numerics (fp32 master, bf16 operands)
  graph        : the amp step captured in a HIP graph (torch.cuda.graphs), static inputs
Prints one JSON line per variant (samples/s, ms/step)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from docker_dist_nn_amd import NAMED_MODELS, MLPSpec  # noqa: E402


def build(spec, dtype, dev):
    layers = []
    for i, l in enumerate(spec.layers):
        layers.append(nn.Linear(l.in_dim, l.out_dim))
        if i < len(spec.layers) - 1:
            layers.append(nn.ReLU())
    return nn.Sequential(*layers).to(dev, dtype)


def run(variant, spec, batch, steps, warmup, dev, optimizer="sgd"):
    torch.manual_seed(0)
    pdtype = torch.bfloat16 if variant == "eager-bf16" else torch.float32
    model = build(spec, pdtype, dev)
    opt = (torch.optim.Adam(model.parameters(), lr=1e-3, capturable=variant == "graph")
           if optimizer == "adam" else torch.optim.SGD(model.parameters(), lr=0.05))
    x = torch.randn(batch, spec.layers[0].in_dim, device=dev).to(pdtype)
    y = torch.randint(0, spec.layers[-1].out_dim, (batch,), device=dev)
    lossf = nn.CrossEntropyLoss()

    def step():
        opt.zero_grad(set_to_none=False)  # (graph capture needs persistent .grad tensors)
        if variant == "eager-bf16":
            loss = lossf(model(x).float(), y)
        else:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = lossf(model(x).float(), y)
        loss.backward()
        opt.step()
        return loss

    if variant == "graph":
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        fn = g.replay
    else:
        fn = step
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return {"variant": variant, "model": spec.describe(), "batch": batch,
            "ms_per_step": round(dt * 1e3, 4), "samples_per_s": round(batch / dt, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mnist-fcnn")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--variants", default="eager-bf16,amp,graph")
    ap.add_argument("--optimizer", default="sgd", choices=["sgd", "adam"])
    a = ap.parse_args()
    spec = NAMED_MODELS.get(a.model) or MLPSpec.parse(a.model)
    dev = torch.device("cuda")
    for v in a.variants.split(","):
        r = run(v, spec, a.batch, a.steps, a.warmup, dev, a.optimizer)
        r["optimizer"] = a.optimizer
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
