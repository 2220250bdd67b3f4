"""Convenience copy of src/run_grpc_inference.py at the repository root; defaults resolve
relative to src/."""
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
from docker_dist_nn_amd.cli.inference import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(script_dir=os.path.join(ROOT, "src")))
