"""Convenience copy of src/run_grpc_fcnn.py at the repository root (README of the reference
names `python3 run_fcnn.py`); defaults resolve relative to src/."""
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
from docker_dist_nn_amd.cli.fcnn import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(script_dir=os.path.join(ROOT, "src")))
