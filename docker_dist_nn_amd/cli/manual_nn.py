"""Single-process CPU forward (BASELINE config 1; /root/reference/scripts/manual_nn.py:73-99).

Same per-neuron fp64 semantics and output lines ("Inference time: X seconds",
"Total inference time", "Average inference time"); the hard-coded paths became flags with the
reference's values as defaults, and both example forms (raw lists and {"input","label"}
objects, which the reference crashed on -- SURVEY §2.7 #11) are accepted.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from typing import Optional

from ..cpu_ref import manual_forward
from ..config import load_model_config


def main(argv: Optional[list[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--config", default="config/config_mnist.json")
    ap.add_argument("--inputs", default="config/example_inputs/example_inputs_mnist.json")
    ap.add_argument("--print-outputs", action="store_true")
    a = ap.parse_args(argv)
    with open(a.config) as f:
        cfg = json.load(f)
    if "layers" not in cfg and "model" in cfg:
        cfg = cfg["model"]
    with open(a.inputs) as f:
        examples = json.load(f)["examples"]
    total = 0.0
    for ex in examples:
        vec = ex["input"] if isinstance(ex, dict) else ex
        t0 = time.time()
        out = manual_forward(cfg, vec)
        dt = time.time() - t0
        total += dt
        print(f"Inference time: {dt:.4f} seconds")
        if a.print_outputs:
            print(f"Network output: {out}")
    print(f"Total inference time: {total:.4f} seconds")
    print(f"Average inference time: {total / max(1, len(examples)):.4f} seconds")
    return 0


if __name__ == "__main__":
    sys.exit(main())
